// 3x3 / stride 1 / pad 1 convolutions with <= 4 channels on one side, at full resolution (gfx950):
// the generator head `res = nn.Conv2d(64, 3, 3, padding=1)` (DSGAN/models/model/MixConvNeXtML.py:459,
// applied at :492 to O4 + Loc at 256^2) -- its forward, weight-grad and data-grad.
//
// These are HBM streams with a small exact-fp32 VALU contraction per pixel (27 MACs per input
// channel and output pixel), so the kernels are built around the loads:
//   * a wave owns a 4-row x 256-column strip: lane l holds columns 4l..4l+3 of each row as ONE
//     16-byte buffer load; the two halo columns come from the neighbour lanes (ds_bpermute), and
//     only the strip's outer lanes load a halo column of their own (segment edges of W > 256);
//     rows outside the image read 0 through the buffer range check (= the zero padding);
//   * the 4+2 rows loaded for a strip serve all 4 x 4 x 9 tap products of the lane's 16 pixels
//     (1.5 loads per pixel per channel instead of 9 scalar tap loads);
//   * weights are wave-uniform (the channel loop is per wave) and come through scalar loads.
// fwd  : y[b][m][h][w] (+)= bias[m] + sum_{k,kh,kw} w[m][k][kh][kw] x[b][k][h+kh-1][w+kw-1], M <= 4;
//        the four waves split the input channels, partials combined through LDS in a fixed order.
// wgrad: dw[m][k][kh][kw] += sum_{b,h,w} dy[b][m][h][w] x[b][k][h+kh-1][w+kw-1]; workgroup =
//        (8 channels, a run of strips), wave = 2 channels; per-split partials reduced in a fixed
//        order by launch_split_reduce (deterministic).
// dgrad: dx[b][k][h][w] (+)= sum_{m,kh,kw} w[m][k][kh][kw] dy[b][m][h+1-kh][w+1-kw], M <= 4; the
//        dy window of a strip stays in registers while the waves walk the K output channels.
#include "common.h"

namespace dsg {

constexpr unsigned T3_OOB = 0xFFFFFFF0u;

struct T3Args {
  const float* x; long x_bs;   // fwd / wgrad: input [nb][K][H][W];  dgrad: dy [nb][M][H][W]
  const float* g; long g_bs;   // wgrad: dy [nb][M][H][W]
  const float* w;              // [M][K][3][3]
  const float* bias;
  float* y; long y_bs;         // fwd: [nb][M][H][W];  dgrad: dx [nb][K][H][W]
  float* ws;                   // wgrad partials [splits][M][K][9]
  int nb, K, M, H, W, accumulate, strips_per_wg;
  unsigned x_range, g_range;
};

__device__ __forceinline__ float4 t3_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ float t3_ld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// Row h of plane `plane` (element offset), columns c0-1 .. c0+4 of this lane (c0 = seg*256 + 4*lane):
// the loads (t3_row_ld: the lane's 16 bytes + the outer lanes' halo columns) and the assembly from
// the neighbour lanes (t3_row_asm) are separate, so a loop can issue the next channel's loads first.
struct T3Row { float4 q; float el, er; };
__device__ __forceinline__ T3Row t3_row_ld(__amdgpu_buffer_rsrc_t r, unsigned plane, int h, int H, int W, int c0,
                                           int lane) {
  const bool ok = (unsigned)h < (unsigned)H;
  const unsigned rowoff = plane + (unsigned)(h * W);
  T3Row o;
  o.q = t3_ld4(r, ok ? (rowoff + (unsigned)c0) * 4u : T3_OOB);
  // halo columns of the segment's outer lanes (a neighbouring segment, or the zero padding)
  o.el = t3_ld1(r, (ok && lane == 0 && c0 > 0) ? (rowoff + (unsigned)c0 - 1u) * 4u : T3_OOB);
  o.er = t3_ld1(r, (ok && lane == 63 && c0 + 4 < W) ? (rowoff + (unsigned)c0 + 4u) * 4u : T3_OOB);
  return o;
}
__device__ __forceinline__ void t3_row_asm(const T3Row& o, int lane, float (&v)[6]) {
  const float l = __shfl_up(o.q.w, 1, 64), rr = __shfl_down(o.q.x, 1, 64);
  v[0] = lane == 0 ? o.el : l;
  v[1] = o.q.x; v[2] = o.q.y; v[3] = o.q.z; v[4] = o.q.w;
  v[5] = lane == 63 ? o.er : rr;
}
__device__ __forceinline__ void t3_row6(__amdgpu_buffer_rsrc_t r, unsigned plane, int h, int H, int W, int c0,
                                        int lane, float (&v)[6]) {
  t3_row_asm(t3_row_ld(r, plane, h, H, W, c0, lane), lane, v);
}

__device__ __forceinline__ void t3_strip(int id, int H, int W, int& b, int& h0, int& c0, int lane) {
  const int S = W >> 8, RB = H >> 2;
  const int seg = id % S;
  id /= S;
  h0 = (id % RB) * 4;
  b = id / RB;
  c0 = seg * 256 + 4 * lane;
}

template <int MS>
__global__ __launch_bounds__(256) void thin3_fwd_kernel(T3Args a) {
  __shared__ float red[3][MS * 16][64];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int b, h0, c0;
  t3_strip(blockIdx.x, a.H, a.W, b, h0, c0, lane);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const unsigned HW = (unsigned)(a.H * a.W);
  float acc[4][4][MS];
  // the next channel's 6 rows are loaded before this channel's FMAs (one channel in flight)
  T3Row nx[6];
  if (wave < a.K) {
    const unsigned plane = (unsigned)((long)b * a.x_bs) + (unsigned)wave * HW;
#pragma unroll
    for (int i = 0; i < 6; ++i) nx[i] = t3_row_ld(rx, plane, h0 - 1 + i, a.H, a.W, c0, lane);
  }
  // output rows (r, r + 1) as the two halves of packed FMAs (v_pk_fma_f32, the weight broadcast):
  // half the FMA instructions, each half the same fmaf chain as the scalar form (same bits)
  f32x2 acc2[2][4][MS];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int m = 0; m < MS; ++m) acc2[q][p][m] = f32x2{0.f, 0.f};
  for (int k = wave; k < a.K; k += 4) {
    float in[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i) t3_row_asm(nx[i], lane, in[i]);
    if (k + 4 < a.K) {
      const unsigned plane = (unsigned)((long)b * a.x_bs) + (unsigned)(k + 4) * HW;
#pragma unroll
      for (int i = 0; i < 6; ++i) nx[i] = t3_row_ld(rx, plane, h0 - 1 + i, a.H, a.W, c0, lane);
    }
    f32x2 in2[5][6];   // rows (i, i + 1) of each column
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) in2[i][j] = f32x2{in[i][j], in[i + 1][j]};
    float wv[MS][9];
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t) wv[m][t] = a.w[((long)m * a.K + k) * 9 + t];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int m = 0; m < MS; ++m)
            acc2[q][p][m] = pk_fma(f32x2{wv[m][t], wv[m][t]}, in2[2 * q + t / 3][p + t % 3], acc2[q][p][m]);
  }
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int m = 0; m < MS; ++m) {
        acc[2 * q][p][m] = acc2[q][p][m].x;
        acc[2 * q + 1][p][m] = acc2[q][p][m].y;
      }
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int m = 0; m < MS; ++m) red[wave - 1][(r * 4 + p) * MS + m][lane] = acc[r][p][m];
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int m = 0; m < MS; ++m) {
    const float bv = a.bias ? a.bias[m] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int i = (r * 4 + p) * MS + m;
        v[p] = (((acc[r][p][m] + red[0][i][lane]) + red[1][i][lane]) + red[2][i][lane]) + bv;
      }
      float4* dst = reinterpret_cast<float4*>(a.y + (long)b * a.y_bs + ((long)m * a.H + h0 + r) * a.W + c0);
      float4 o = make_float4(v[0], v[1], v[2], v[3]);
      if (a.accumulate) { const float4 q = *dst; o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w; }
      *dst = o;
    }
  }
}

// wave = CW channels; workgroup = 4 waves = 4*CW channels over strips [s0, s1)
template <int MS, int CW>
__global__ __launch_bounds__(256) void thin3_wgrad_kernel(T3Args a) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kb = (blockIdx.x * 4 + wave) * CW;
  const int nstrips = a.nb * (a.H >> 2) * (a.W >> 8);
  const int s0 = blockIdx.y * a.strips_per_wg, s1 = min(nstrips, s0 + a.strips_per_wg);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.g, (short)0, a.g_range, 0x00020000);
  const unsigned HW = (unsigned)(a.H * a.W);
  float acc[CW][MS][9];
#pragma unroll
  for (int c = 0; c < CW; ++c)
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[c][m][t] = 0.f;
#pragma unroll 1
  for (int s = s0; s < s1; ++s) {
    int b, h0, c0;
    t3_strip(s, a.H, a.W, b, h0, c0, lane);
    float4 gv[MS][4];
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        gv[m][r] = t3_ld4(rg, ((unsigned)((long)b * a.g_bs) + (unsigned)m * HW + (unsigned)((h0 + r) * a.W + c0)) * 4u);
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      const int k = kb + c;
      if (k >= a.K) break;
      const unsigned plane = (unsigned)((long)b * a.x_bs) + (unsigned)k * HW;
      float in[6][6];
#pragma unroll
      for (int i = 0; i < 6; ++i) t3_row6(rx, plane, h0 - 1 + i, a.H, a.W, c0, lane, in[i]);
#pragma unroll
      for (int m = 0; m < MS; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gr[4] = {gv[m][r].x, gv[m][r].y, gv[m][r].z, gv[m][r].w};
#pragma unroll
          for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[c][m][t] = fmaf(gr[p], in[r + t / 3][p + t % 3], acc[c][m][t]);
        }
    }
  }
  float* dst = a.ws + (long)blockIdx.y * a.M * a.K * 9;
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const int k = kb + c;
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float v = warp_sum(acc[c][m][t]);
        if (lane == 0 && k < a.K) dst[((long)m * a.K + k) * 9 + t] = v;
      }
  }
}

// workgroup = one strip; wave w computes output channels k = w, w+4, ... from the strip's dy window
template <int MS>
__global__ __launch_bounds__(256) void thin3_dgrad_kernel(T3Args a) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int b, h0, c0;
  t3_strip(blockIdx.x, a.H, a.W, b, h0, c0, lane);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const unsigned HW = (unsigned)(a.H * a.W);
  float in[MS][6][6];
#pragma unroll
  for (int m = 0; m < MS; ++m) {
    const unsigned plane = (unsigned)((long)b * a.x_bs) + (unsigned)m * HW;
#pragma unroll
    for (int i = 0; i < 6; ++i) t3_row6(rx, plane, h0 - 1 + i, a.H, a.W, c0, lane, in[m][i]);
  }
#pragma unroll 1
  for (int k = wave; k < a.K; k += 4) {
    // flipped taps: dx[h][w] += w[m][k][2-i][2-j] dy[h-1+i][w-1+j]
    float wv[MS][9];
#pragma unroll
    for (int m = 0; m < MS; ++m)
#pragma unroll
      for (int t = 0; t < 9; ++t) wv[m][t] = a.w[((long)m * a.K + k) * 9 + (8 - t)];
    float* yk = a.y + (long)b * a.y_bs + ((long)k * a.H + h0) * a.W + c0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float s = 0.f;
#pragma unroll
        for (int m = 0; m < MS; ++m)
#pragma unroll
          for (int t = 0; t < 9; ++t) s = fmaf(wv[m][t], in[m][r + t / 3][p + t % 3], s);
        v[p] = s;
      }
      float4* dst = reinterpret_cast<float4*>(yk + (long)r * a.W);
      float4 o = make_float4(v[0], v[1], v[2], v[3]);
      if (a.accumulate) { const float4 q = *dst; o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w; }
      *dst = o;
    }
  }
}

constexpr int T3_CW = 2;   // wgrad channels per wave

static long t3_wgrad_plan(int nb, int K, int H, int W, int* spw) {
  const long nstrips = (long)nb * (H / 4) * (W / 256);
  const long groups = (K + 4 * T3_CW - 1) / (4 * T3_CW);
  // ~512 workgroups: the closing lane reductions (54 sums per wave) amortised over more strips
  // (measured at the G head, B=16: 2048 / 1024 / 512 workgroups 149 / 124 / 115 us)
  long splits = (512 + groups - 1) / groups;
  if (splits > nstrips) splits = nstrips;
  long per = (nstrips + splits - 1) / splits;
  *spw = (int)per;
  return (nstrips + per - 1) / per;
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Shapes the thin 3x3 kernels take: H % 4 == 0, W % 256 == 0, 1 <= M <= 4 (the small side),
// 16-byte aligned planes.
int dsgan_thin3_supported(int M, int H, int W, long bs_small, long bs_big) {
  return M >= 1 && M <= 4 && H % 4 == 0 && H > 0 && W % 256 == 0 && W > 0 && (bs_small % 4) == 0 &&
         (bs_big % 4) == 0;
}

static bool t3_args(T3Args& a, const float* x, long x_bs, int xc, int nb, int H, int W) {
  const long xr = ((long)(nb - 1) * x_bs + (long)xc * H * W) * 4;
  a.x = x; a.x_bs = x_bs; a.x_range = (unsigned)xr;
  return xr < (long)T3_OOB && ((uintptr_t)x & 15) == 0;
}

// y[nb][M][H][W] (+)= bias + conv3x3(x[nb][K][H][W], w[M][K][3][3]), pad 1
int dsgan_thin3_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int nb, int K,
                    int M, int H, int W, int accumulate, hipStream_t st) {
  DSG_REQUIRE(x && w && y && nb > 0 && K > 0 && dsgan_thin3_supported(M, H, W, y_bs, x_bs) && ((uintptr_t)y & 15) == 0,
              "dsgan_thin3_fwd: unsupported shape/alignment");
  T3Args a{};
  DSG_REQUIRE(t3_args(a, x, x_bs, K, nb, H, W), "dsgan_thin3_fwd: input exceeds 4 GiB / unaligned");
  a.w = w; a.bias = bias; a.y = y; a.y_bs = y_bs; a.nb = nb; a.K = K; a.M = M; a.H = H; a.W = W;
  a.accumulate = accumulate;
  const dim3 grid((unsigned)((long)nb * (H / 4) * (W / 256)));
  if (M == 1) hipLaunchKernelGGL(thin3_fwd_kernel<1>, grid, dim3(256), 0, st, a);
  else if (M == 2) hipLaunchKernelGGL(thin3_fwd_kernel<2>, grid, dim3(256), 0, st, a);
  else if (M == 3) hipLaunchKernelGGL(thin3_fwd_kernel<3>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(thin3_fwd_kernel<4>, grid, dim3(256), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

long dsgan_thin3_wgrad_workspace(int nb, int K, int M, int H, int W) {
  int spw;
  return t3_wgrad_plan(nb, K, H, W, &spw) * (long)M * K * 9;
}

// dw[M][K][3][3] += weight-grad (dy [nb][M][H][W], x [nb][K][H][W]); ws: dsgan_thin3_wgrad_workspace floats
int dsgan_thin3_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* ws, long ws_elems,
                      int nb, int K, int M, int H, int W, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && nb > 0 && K > 0 && dsgan_thin3_supported(M, H, W, dy_bs, x_bs) &&
                  ((uintptr_t)dy & 15) == 0,
              "dsgan_thin3_wgrad: unsupported shape/alignment");
  T3Args a{};
  DSG_REQUIRE(t3_args(a, x, x_bs, K, nb, H, W), "dsgan_thin3_wgrad: input exceeds 4 GiB / unaligned");
  const long gr = ((long)(nb - 1) * dy_bs + (long)M * H * W) * 4;
  DSG_REQUIRE(gr < (long)T3_OOB, "dsgan_thin3_wgrad: dy exceeds 4 GiB");
  a.g = dy; a.g_bs = dy_bs; a.g_range = (unsigned)gr;
  a.w = nullptr; a.ws = ws; a.nb = nb; a.K = K; a.M = M; a.H = H; a.W = W;
  int spw;
  const long splits = t3_wgrad_plan(nb, K, H, W, &spw);
  a.strips_per_wg = spw;
  DSG_WS(splits * (long)M * K * 9, ws, ws_elems, "dsgan_thin3_wgrad (dsgan_thin3_wgrad_workspace)");
  const dim3 grid((unsigned)((K + 4 * T3_CW - 1) / (4 * T3_CW)), (unsigned)splits);
  if (M == 1) hipLaunchKernelGGL((thin3_wgrad_kernel<1, T3_CW>), grid, dim3(256), 0, st, a);
  else if (M == 2) hipLaunchKernelGGL((thin3_wgrad_kernel<2, T3_CW>), grid, dim3(256), 0, st, a);
  else if (M == 3) hipLaunchKernelGGL((thin3_wgrad_kernel<3, T3_CW>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((thin3_wgrad_kernel<4, T3_CW>), grid, dim3(256), 0, st, a);
  DSG_CHECK_LAUNCH();
  launch_split_reduce(ws, (int)splits, (long)M * K * 9, dw, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dx[nb][K][H][W] (+)= data-grad of the conv above (dy [nb][M][H][W], w[M][K][3][3])
int dsgan_thin3_dgrad(const float* dy, long dy_bs, const float* w, float* dx, long dx_bs, int nb, int K, int M, int H,
                      int W, int accumulate, hipStream_t st) {
  DSG_REQUIRE(dy && w && dx && nb > 0 && K > 0 && dsgan_thin3_supported(M, H, W, dy_bs, dx_bs) &&
                  ((uintptr_t)dx & 15) == 0,
              "dsgan_thin3_dgrad: unsupported shape/alignment");
  T3Args a{};
  DSG_REQUIRE(t3_args(a, dy, dy_bs, M, nb, H, W), "dsgan_thin3_dgrad: dy exceeds 4 GiB / unaligned");
  a.w = w; a.y = dx; a.y_bs = dx_bs; a.nb = nb; a.K = K; a.M = M; a.H = H; a.W = W; a.accumulate = accumulate;
  const dim3 grid((unsigned)((long)nb * (H / 4) * (W / 256)));
  if (M == 1) hipLaunchKernelGGL(thin3_dgrad_kernel<1>, grid, dim3(256), 0, st, a);
  else if (M == 2) hipLaunchKernelGGL(thin3_dgrad_kernel<2>, grid, dim3(256), 0, st, a);
  else if (M == 3) hipLaunchKernelGGL(thin3_dgrad_kernel<3>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(thin3_dgrad_kernel<4>, grid, dim3(256), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
