// PatchGAN head: the last layer of NLayerDiscriminator, Conv2d(ndf * 8, 1, 4, stride 1, pad 1) ->
// raw logits (DSGAN/models/networks.py:567-568), 256 channels at 31x31 -> 30x30 for 256^2 inputs.
//
// One output channel: the GEMM views have M = 1 and the generic kernels ran this layer at 0.4-0.8
// TB/s on 16 MB (small_out 28 us forward, wgrad_small 36 us, the implicit-GEMM data-grad 20-25 us,
// three forwards and three backwards per step).  Here every direction splits the input channels
// into chunks of KC planes staged zero-padded in LDS, one workgroup per (chunk, image):
//   * pgl_fwd   : thread = 4 adjacent outputs of a row, KC x 16 taps from LDS, weights uniform;
//                 per-chunk partials summed in chunk order by pgl_fin (+ bias);
//   * pgl_wgrad : thread = (channel, kh, row group): 4 kw sums over a sliding window of the padded
//                 x rows against the dy plane; chunk 0 also sums the bias grad; per-image partials
//                 [K*16 + 1] that launch_split_reduce_kk adds in a fixed order into dw and db;
//   * pgl_dgrad : thread = input pixels of the chunk's planes, 16 taps of the zero-padded dy plane.
// Exact fp32 throughout (the layer's operands are fp32 in HBM), fixed summation orders
// (deterministic, no atomics).
#include "common.h"

namespace dsg {

struct PlArgs {
  const float* x; long x_bs;     // [nb][K][H][W]
  const float* dy; long dy_bs;   // [nb][1][Ho][Wo]
  const float* w;                // [1][K][4][4]
  float* out; long out_bs;       // dgrad: dx [nb][K][H][W]
  float* ws;
  int nb, K, H, W, Ho, Wo, KC, accumulate;
};

// zero-padded planes of this workgroup's KC channels: xs[c][(H+2)(W+2)] (+ 8 zero floats of slack:
// the last row's 7-wide window may run 2 past a plane)
__device__ __forceinline__ void pgl_stage_x(const PlArgs& a, float* xs, int k0, int b) {
  const int H = a.H, W = a.W, WP = W + 2, PS = (H + 2) * WP, n = a.KC * PS + 8;
  for (int i = threadIdx.x; i < n; i += 256) xs[i] = 0.f;
  __syncthreads();
  const float* xb = a.x + (long)b * a.x_bs + (long)k0 * H * W;
  // thread = (column tx of a CW-wide block, row phase ty); (channel, row) items in batches of 8 loads
  // in flight (a load per loop trip waits for its data before the LDS write: latency x trips)
  const int CW = W <= 32 ? 32 : 64, tx = threadIdx.x % CW, ty = threadIdx.x / CW, RS = 256 / CW;
  const int RPT = (H + RS - 1) / RS, NIT = a.KC * RPT;   // rows per thread per channel, items per thread
  for (int ix = tx; ix < W; ix += CW)
    for (int i0 = 0; i0 < NIT; i0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int it = i0 + u, c = it / RPT, iy = ty + (it - c * RPT) * RS;
        v[u] = it < NIT && iy < H ? xb[((long)c * H + iy) * W + ix] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int it = i0 + u, c = it / RPT, iy = ty + (it - c * RPT) * RS;
        if (it < NIT && iy < H) xs[c * PS + (iy + 1) * WP + ix + 1] = v[u];
      }
    }
}

__global__ __launch_bounds__(256) void pgl_fwd_kernel(PlArgs a) {
  extern __shared__ float xs[];
  const int ch = blockIdx.x, b = blockIdx.y, nch = gridDim.x, k0 = ch * a.KC;
  pgl_stage_x(a, xs, k0, b);
  __syncthreads();
  const int WP = a.W + 2, PS = (a.H + 2) * WP, Ho = a.Ho, Wo = a.Wo, n4 = (Wo + 3) >> 2;
  for (int it = threadIdx.x; it < Ho * n4; it += 256) {
    const int oy = it / n4, ox0 = (it - oy * n4) * 4;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < a.KC; ++c) {
      const float* wr = a.w + (k0 + c) * 16;
      const float* xr = xs + c * PS + oy * WP + ox0;   // padded row oy + kh, column ox0 + kw
#pragma unroll
      for (int kh = 0; kh < 4; ++kh) {
        float v[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) v[j] = xr[kh * WP + j];
#pragma unroll
        for (int kw = 0; kw < 4; ++kw)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = fmaf(wr[kh * 4 + kw], v[j + kw], acc[j]);
      }
    }
    float* o = a.ws + ((long)b * nch + ch) * Ho * Wo + oy * Wo + ox0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (ox0 + j < Wo) o[j] = acc[j];
  }
}

// y[b][p] (+)= bias + sum over chunks c = 0.. in order of ws[b][c][p]
__global__ __launch_bounds__(256) void pgl_fin_kernel(const float* __restrict__ ws, int nch, int HoWo,
                                                      const float* __restrict__ bias, float* __restrict__ y,
                                                      long y_bs, int nb, int accumulate) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= nb * HoWo) return;
  const int b = idx / HoWo, p = idx - b * HoWo;
  const float* s = ws + (long)b * nch * HoWo + p;
  float t = 0.f;
#pragma unroll 8
  for (int c = 0; c < nch; ++c) t += s[(long)c * HoWo];   // (the loads of 8 chunks in flight; same order)
  const float v = t + (bias ? bias[0] : 0.f);
  float* o = y + (long)b * y_bs + p;
  *o = accumulate ? *o + v : v;
}

__global__ __launch_bounds__(256) void pgl_wgrad_kernel(PlArgs a) {
  extern __shared__ float sm[];
  const int ch = blockIdx.x, b = blockIdx.y, k0 = ch * a.KC;
  const int WP = a.W + 2, PS = (a.H + 2) * WP, Ho = a.Ho, Wo = a.Wo, HoWo = Ho * Wo;
  float* xs = sm;
  float* dys = sm + a.KC * PS + 8;
  pgl_stage_x(a, xs, k0, b);
  const float* dyb = a.dy + (long)b * a.dy_bs;
  for (int i = threadIdx.x; i < HoWo; i += 256) dys[i] = dyb[i];
  __syncthreads();
  const int E = a.K * 16 + 1;
  float* out = a.ws + (long)b * E;
  // thread = (channel c, kernel row kh, row group rg of 8): the 4 kw sums over its output rows with a
  // sliding 4-column window (2 LDS reads per position for 4 FMAs); the 8 row groups (adjacent lanes)
  // meet in a butterfly -- commutative pairs, so every lane of a group holds the same bits
  const int RG = (Ho + 7) >> 3;
  for (int it = threadIdx.x; it < a.KC * 32; it += 256) {
    const int rg = it & 7, kh = (it >> 3) & 3, c = it >> 5;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    const int oy1 = min(Ho, (rg + 1) * RG);
    for (int oy = rg * RG; oy < oy1; ++oy) {
      const float* d = dys + oy * Wo;
      const float* xo = xs + c * PS + (oy + kh) * WP;   // padded row oy + kh, column ox + kw
      float w0 = xo[0], w1 = xo[1], w2 = xo[2];
#pragma unroll 6
      for (int ox = 0; ox < Wo; ++ox) {
        const float w3 = xo[ox + 3], dv = d[ox];
        s0 = fmaf(dv, w0, s0); s1 = fmaf(dv, w1, s1); s2 = fmaf(dv, w2, s2); s3 = fmaf(dv, w3, s3);
        w0 = w1; w1 = w2; w2 = w3;
      }
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      s0 += __shfl_xor(s0, m, 64); s1 += __shfl_xor(s1, m, 64);
      s2 += __shfl_xor(s2, m, 64); s3 += __shfl_xor(s3, m, 64);
    }
    if (rg == 0) {
      float* o = out + (k0 + c) * 16 + kh * 4;
      o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3;
    }
  }
  if (ch == 0) {   // bias grad of this image: sum of dy
    __shared__ float red[4];
    float s = 0.f;
    for (int i = threadIdx.x; i < HoWo; i += 256) s += dys[i];
    s = block_sum<256>(s, red);
    if (threadIdx.x == 0) out[E - 1] = s;
  }
}

__global__ __launch_bounds__(256) void pgl_dgrad_kernel(PlArgs a) {
  extern __shared__ float sm[];
  const int ch = blockIdx.x, b = blockIdx.y, k0 = ch * a.KC;
  const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo, DW = Wo + 6, DS = (Ho + 6) * DW;
  float* dyp = sm;          // dy zero-padded by 3: dyp[(oy + 3) * DW + ox + 3]
  float* wl = sm + DS;      // this chunk's weights [KC][16]
  for (int i = threadIdx.x; i < DS; i += 256) dyp[i] = 0.f;
  for (int i = threadIdx.x; i < a.KC * 16; i += 256) wl[i] = a.w[k0 * 16 + i];
  __syncthreads();
  const float* dyb = a.dy + (long)b * a.dy_bs;
  for (int i = threadIdx.x; i < Ho * Wo; i += 256) {
    const int oy = i / Wo, ox = i - oy * Wo;
    dyp[(oy + 3) * DW + ox + 3] = dyb[i];
  }
  __syncthreads();
  const int HW = H * W;
  float* dxb = a.out + (long)b * a.out_bs + (long)k0 * HW;
  // thread = (column tx of a CW-wide block, row phase ty): no per-element divisions
  const int CW = W <= 32 ? 32 : 64, tx = threadIdx.x % CW, ty = threadIdx.x / CW, RS = 256 / CW;
#pragma unroll 1
  for (int c = 0; c < a.KC; ++c) {
    float wv[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) wv[t] = wl[c * 16 + t];
    for (int iy = ty; iy < H; iy += RS)
      for (int ix = tx; ix < W; ix += CW) {
        const float* d = dyp + (iy + 4) * DW + ix + 4;   // oy = iy + 1 - kh -> padded row iy + 4 - kh
        float s = 0.f;
#pragma unroll
        for (int kh = 0; kh < 4; ++kh)
#pragma unroll
          for (int kw = 0; kw < 4; ++kw) s = fmaf(wv[kh * 4 + kw], d[-kh * DW - kw], s);
        float* o = dxb + (long)c * HW + iy * W + ix;
        *o = a.accumulate ? *o + s : s;
      }
  }
}

constexpr int PGL_LDS = 40 * 1024;
static int pgl_kc(int K, int H, int W) {   // channels per chunk: the largest of 8, 4, 2, 1 that fits
  const long ps = (long)(H + 2) * (W + 2);
  for (int kc = 8; kc >= 1; kc >>= 1)
    if (K % kc == 0 && ((long)kc * ps + 8 + (long)(H - 1) * (W - 1)) * 4 <= PGL_LDS) return kc;
  return 0;
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Shapes the head kernels take: Cout = 1, 4x4, stride 1, pad 1 (output (H-1) x (W-1)), a plane
// small enough that one channel chunk stages in 40 KB of LDS (H, W <= ~100).
int dsgan_pglast_supported(int K, int H, int W) {
  if (K <= 0 || H < 2 || W < 2) return 0;
  const long DS = (long)(H - 1 + 6) * (W - 1 + 6);
  return pgl_kc(K, H, W) > 0 && (DS + 8 * 16) * 4 <= PGL_LDS ? 1 : 0;
}

long dsgan_pglast_workspace(int N, int K, int H, int W) {
  const int kc = pgl_kc(K, H, W);
  if (kc <= 0) return 0;
  const long fwd = (long)N * (K / kc) * (H - 1) * (W - 1), wg = (long)N * (K * 16 + 1);
  return fwd > wg ? fwd : wg;
}

static PlArgs pgl_args(int N, int K, int H, int W) {
  PlArgs a{};
  a.nb = N; a.K = K; a.H = H; a.W = W; a.Ho = H - 1; a.Wo = W - 1; a.KC = pgl_kc(K, H, W);
  return a;
}

// y (+)= bias + conv4x4s1p1(x, w), y [N][1][H-1][W-1]; w [1][K][4][4]; bias nullable.
int dsgan_pglast_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int N, int K,
                     int H, int W, int accumulate, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(x && w && y && N > 0, "dsgan_pglast_fwd: bad args");
  DSG_REQUIRE(dsgan_pglast_supported(K, H, W), "dsgan_pglast_fwd: unsupported shape (see dsgan_pglast_supported)");
  PlArgs a = pgl_args(N, K, H, W);
  const int nch = K / a.KC;
  DSG_WS((long)N * nch * a.Ho * a.Wo, ws, ws_elems, "dsgan_pglast_fwd (dsgan_pglast_workspace)");
  a.x = x; a.x_bs = x_bs; a.w = w; a.ws = ws;
  const size_t lds = ((size_t)a.KC * (H + 2) * (W + 2) + 8) * 4;
  hipLaunchKernelGGL(pgl_fwd_kernel, dim3(nch, N), dim3(256), lds, st, a);
  const int HoWo = a.Ho * a.Wo;
  hipLaunchKernelGGL(pgl_fin_kernel, dim3(cdiv((long)N * HoWo, 256)), dim3(256), 0, st, ws, nch, HoWo, bias, y, y_bs, N,
                     accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dw += dW, db += dB (db nullable) from dy [N][1][H-1][W-1] and x.
int dsgan_pglast_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* db, int N, int K,
                       int H, int W, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && N > 0, "dsgan_pglast_wgrad: bad args");
  DSG_REQUIRE(dsgan_pglast_supported(K, H, W), "dsgan_pglast_wgrad: unsupported shape (see dsgan_pglast_supported)");
  PlArgs a = pgl_args(N, K, H, W);
  DSG_WS((long)N * (K * 16 + 1), ws, ws_elems, "dsgan_pglast_wgrad (dsgan_pglast_workspace)");
  a.x = x; a.x_bs = x_bs; a.dy = dy; a.dy_bs = dy_bs; a.ws = ws;
  const size_t lds = ((size_t)a.KC * (H + 2) * (W + 2) + 8 + (size_t)a.Ho * a.Wo) * 4;
  hipLaunchKernelGGL(pgl_wgrad_kernel, dim3(K / a.KC, N), dim3(256), lds, st, a);
  launch_split_reduce_kk(ws, N, (long)K * 16 + 1, dw, db, K * 16 + 1, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dx (+)= the input gradient [N][K][H][W] from dy [N][1][H-1][W-1].
int dsgan_pglast_dgrad(const float* dy, long dy_bs, const float* w, float* dx, long dx_bs, int N, int K, int H, int W,
                       int accumulate, hipStream_t st) {
  DSG_REQUIRE(dy && w && dx && N > 0, "dsgan_pglast_dgrad: bad args");
  DSG_REQUIRE(dsgan_pglast_supported(K, H, W), "dsgan_pglast_dgrad: unsupported shape (see dsgan_pglast_supported)");
  PlArgs a = pgl_args(N, K, H, W);
  a.dy = dy; a.dy_bs = dy_bs; a.w = w; a.out = dx; a.out_bs = dx_bs; a.accumulate = accumulate;
  const size_t lds = ((size_t)(a.Ho + 6) * (a.Wo + 6) + (size_t)a.KC * 16) * 4;
  hipLaunchKernelGGL(pgl_dgrad_kernel, dim3(K / a.KC, N), dim3(256), lds, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
