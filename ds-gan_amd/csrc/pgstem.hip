// PatchGAN stem: the first layer of NLayerDiscriminator, Conv2d(input_nc, ndf, 4, stride 2, pad 1)
// + bias + LeakyReLU(0.2) (DSGAN/models/networks.py:543-545), at the full image resolution.
//
// Its input has 6 channels (cat(A, B)) and its output 32 (ndf), so the layer is a streaming
// problem, not a GEMM tile: 96 taps per output, ~1.6 GFLOP per B=16 pass at 256^2 against ~60 MB
// of HBM traffic.  The generic implicit GEMM gathered each tap with a scalar load (34 / 68 us for
// the forward / weight-grad, 0.7-1.7 TB/s), and the backward ran three more launches (LeakyReLU
// backward, bias channel sum, the transposed data-grad).  Here each direction is one kernel:
//   * pgs_fwd   : thread = 2 adjacent output pixels x all CO channels, fp32 packed FMA, the weights
//                 as scalar-cache operands; y = lrelu(bias + conv) (NCHW fp32).
//   * pgs_wgrad : dy' = dy * lrelu'(y) staged with x into LDS per two output rows; dW on exact fp32
//                 MFMA (32x32x2: M = CO, N = CI*16 taps, K = positions), db from the same dy'
//                 operands; per-workgroup partials [CO][CI*16 + 1] that launch_split_reduce_kk adds
//                 in a fixed order into dw (OIHW) and db (deterministic, no atomics).
//   * pgs_dgrad : thread = one 2x2 input block x all CI channels (the four stride-2 parities share
//                 a 3x3 dy' neighbourhood), dy' staged in LDS, fp32 packed FMA.
// Every product is exact fp32 (both precision modes): the layer's operands are fp32 in HBM and
// its ~0.3 GFLOP per pass does not need bf16.  lrelu'(y): y > 0 ? 1 : slope -- the reference's
// in-place LeakyReLU differentiates through its output (networks.py:545).
#include "common.h"

namespace dsg {

typedef __attribute__((ext_vector_type(2))) float pg_f2;
constexpr unsigned PG_OOB = 0xFFFFFFF0u;

__device__ __forceinline__ float pg_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ float4 pg_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}
__device__ __forceinline__ float pg_lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }

// ---- forward ----------------------------------------------------------------------------------
// Exact fp32 MFMA (32x32x2): M = CO output channels, N = 32 consecutive output positions of a row,
// K = CI * 16 taps, walked exactly as the generic implicit GEMM walks them (igemm.hip: per input
// channel the K steps (k, 8 + k), k = 0..7, k = 4 kh + kw), then + bias, then the LeakyReLU: the
// same fp32 fma chain per output, so y is bit-identical to that path in fp32 mode and the step's
// LeakyReLU / InstanceNorm decisions downstream are the ones the validated path makes (a near-zero
// pre-activation is a kink that a different rounding order can flip).
// A (weights) stays in registers for the whole launch: lane l holds w[co = l % 32][ci][8 (l / 32) + k].
// B (im2col of x) is read from an LDS stage of two output rows = six input rows, stored with the
// column parities apart (column ix at (ix & 1) * HS + (ix >> 1) + 2): a B read of 32 consecutive
// positions is 32 consecutive floats, and the half-wave 8 taps later (two rows down, row stride
// = 16 mod 32) the other 32 banks.  Stage = two output rows; wave w computes the 32-position
// tiles w, w + 4, ... of it.
constexpr int pgf_hs(int W) { return W / 2 + 4; }                       // one parity half of a row
constexpr int pgf_xc(int W) { return ((2 * pgf_hs(W) - 16 + 31) / 32) * 32 + 16; }   // = 16 mod 32
template <int CI, int CO, int WMAX>
__global__ __launch_bounds__(256, 2) void pgs_fwd_kernel(const float* __restrict__ x, long x_bs,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      float* __restrict__ y, long y_bs, int nb, int H, int W,
                                                      float slope) {
  constexpr int MB = CO / 32;
  __shared__ __attribute__((aligned(16))) float xt[CI * 6 * pgf_xc(WMAX)];
  const int Ho = H >> 1, Wo = W >> 1, HS = pgf_hs(W), XC = pgf_xc(W), XS = 6 * XC;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  for (int i = tid; i < CI * 6 * 8; i += 256) {   // the 4 pad slots of each parity half stay 0
    const int rowi = i >> 3, k = i & 7, half = k >> 2, slot = k & 3;
    xt[rowi * XC + half * HS + (slot < 2 ? slot : W / 2 + slot)] = 0.f;
  }
  float wa[MB][CI][8];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int k = 0; k < 8; ++k) wa[mb][ci][k] = w[((32 * mb + lr) * CI + ci) * 16 + 8 * lh + k];

  const int spi = Ho >> 1, stages = nb * spi, ntile = Wo >> 4;   // 32-position tiles per stage
  const __amdgpu_buffer_rsrc_t rxa = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, 0xFFFFFFF0u, 0x00020000);
  // persistent over stages: the next stage's input rows are loaded into registers before this
  // stage's MFMAs (a one-stage-per-workgroup grid runs every workgroup's load, MFMA and store
  // phases in lockstep: HBM idles while the MFMAs run)
  constexpr int NXI = (CI * 6 * WMAX / 4 + 255) / 256;   // 16-byte items per lane per stage
  const int W4 = W >> 2, nx = CI * 6 * W4;
  float4 v[NXI];
  auto load_stage = [&](int st_) __attribute__((always_inline)) {
    const int b_ = st_ / spi, oy_ = (st_ - b_ * spi) * 2;
    const long xb = (long)b_ * x_bs;
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int i = tid + 256 * u, ix4 = i % W4, q = i / W4, rr = q % 6, ci = q / 6;
      const int iy = 2 * oy_ - 1 + rr;
      const bool ok = i < nx && (unsigned)iy < (unsigned)H;
      v[u] = pg_ld4(rxa, ok ? (unsigned)((xb + (long)ci * H * W + (long)iy * W + 4 * ix4) * 4) : PG_OOB);
    }
  };
  if (blockIdx.x < stages) load_stage(blockIdx.x);
  for (int st = blockIdx.x; st < stages; st += gridDim.x) {
    const int b = st / spi, oy0 = (st - b * spi) * 2;
    __syncthreads();   // the previous stage's B reads are done
#pragma unroll
    for (int u = 0; u < NXI; ++u) {
      const int i = tid + 256 * u, ix4 = i % W4, q = i / W4;
      if (i < nx) {
        float* row = xt + q * XC + 2 * ix4 + 2;   // q = ci * 6 + rr
        *reinterpret_cast<float2*>(row) = make_float2(v[u].x, v[u].z);        // even columns
        *reinterpret_cast<float2*>(row + HS) = make_float2(v[u].y, v[u].w);   // odd columns
      }
    }
    __syncthreads();
    if (st + (int)gridDim.x < stages) load_stage(st + gridDim.x);
    // tiles t0 and t0 + 4 (Cout 32): two independent accumulator chains per wave
    constexpr int TT = MB == 1 ? 2 : 1;
    for (int t0 = wave; t0 < ntile; t0 += 4 * TT) {
      const bool two = TT == 2 && t0 + 4 < ntile;
      int cbs[TT][4];
      const float* xr[TT];
      long yoff[TT];
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        const int t = j && two ? t0 + 4 : t0;
        const int n = 32 * t + lr, oyl = n >= Wo ? 1 : 0, ox = n - oyl * Wo;
        // B column of this lane's position for kw = 0..3 (parity halves: ix = 2 ox + kw - 1)
        cbs[j][0] = HS + ox + 1; cbs[j][1] = ox + 2; cbs[j][2] = HS + ox + 2; cbs[j][3] = ox + 3;
        xr[j] = xt + (2 * oyl + 2 * lh) * XC;   // rows kh = k / 4 + 2 (l / 32)
        yoff[j] = (long)b * y_bs + (long)(oy0 + oyl) * Wo + ox;
      }
      f32x16_t acc[TT][MB];
#pragma unroll
      for (int j = 0; j < TT; ++j)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[j][mb][r] = 0.f;
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) {
        float bvv[TT][8];
#pragma unroll
        for (int j = 0; j < TT; ++j)
#pragma unroll
          for (int k = 0; k < 8; ++k) bvv[j][k] = xr[j][ci * XS + (k >> 2) * XC + cbs[j][k & 3]];
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int j = 0; j < TT; ++j)
#pragma unroll
            for (int mb = 0; mb < MB; ++mb)
              acc[j][mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[mb][ci][k], bvv[j][k], acc[j][mb], 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < TT; ++j) {
        if (j == 1 && !two) break;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int co = 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * lh;
            y[yoff[j] + (long)co * Ho * Wo] = pg_lrelu(acc[j][mb][r] + (bias ? bias[co] : 0.f), slope);
          }
      }
    }
  }
}
static int pg_fwd_grid(int N, int H) {   // two workgroups per CU, each walking several stages
  const int stages = N * (H / 4);
  return stages < 512 ? stages : 512;
}

// ---- weight-grad --------------------------------------------------------------------------------
// Stage = two output rows (oy0, oy0 + 1) of one image: dy' as [position][CO + 2] (lanes of one
// MFMA A read: 32 channels x a position pair 16 apart -> 64 distinct banks), x as
// [ci][6 rows][W + 8] (input column ix at ix + 4, 16-byte aligned rows; columns 3 and W + 4 are
// the zero padding) with the row stride = 8 and the channel stride = 4 mod 64 banks, so a B read of
// 32 taps (two ci x 4 kh x 4 kw) x the same position pair covers 64 distinct banks.  K step s of a
// stage pairs positions p and p + 16, p = 32 (s / 16) + s % 16; wave w takes steps
// [w Wo/4, (w+1) Wo/4).  Both tiles are filled from 16-byte loads, all of a batch in flight before
// the LDS writes (8 per lane and operand).
struct PgWArgs {
  const float* dy; long dy_bs;
  const float* y; long y_bs;
  const float* x; long x_bs;
  float* ws;                 // [gridDim.x][CO][CI*16 + 1]
  int nb, H, W, XS;
  float slope;
};

constexpr int pg_xs(int W) {   // x-tile channel stride: >= 6 (W + 8) floats, = 4 mod 64 (banks)
  return ((6 * (W + 8) - 4 + 63) / 64) * 64 + 4;
}
constexpr int pg_wgrad_lds(int CI, int CO, int W) {   // floats: the stage tiles, or the wave reduction
  return W * (CO + 2) + CI * pg_xs(W) > 4 * CO * (CI * 16 + 1) ? W * (CO + 2) + CI * pg_xs(W) : 4 * CO * (CI * 16 + 1);
}

// WMAX: the widest image the static LDS stage holds (256: two workgroups per CU at Cout 32)
template <int CI, int CO, int WMAX>
__global__ __launch_bounds__(256, 2) void pgs_wgrad_kernel(PgWArgs a) {
  constexpr int MB = CO / 32, NTAP = CI * 16, NB = (NTAP + 31) / 32, SC = CO + 2, E = CO * (NTAP + 1);
  __shared__ __attribute__((aligned(16))) float lds[pg_wgrad_lds(CI, CO, WMAX)];
  const int H = a.H, W = a.W, Ho = H >> 1, Wo = W >> 1, XC = W + 8, XS = a.XS;
  float* dyt = lds;
  float* xt = lds + 2 * Wo * SC;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;

  for (int i = tid; i < CI * 6 * 2; i += 256) {
    const int ci = i / 12, rr = (i >> 1) % 6;
    xt[ci * XS + rr * XC + ((i & 1) ? W + 4 : 3)] = 0.f;
  }
  int tb[NB];
  bool tv[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int tap = nb * 32 + lr;
    tv[nb] = tap < NTAP;
    tb[nb] = tv[nb] ? (tap >> 4) * XS + ((tap >> 2) & 3) * XC + (tap & 3) + 3 : 0;
  }
  f32x16_t acc[MB][NB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mb][nb][r] = 0.f;
  float bs[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) bs[mb] = 0.f;

  const int spi = Ho >> 1, stages = a.nb * spi, P2 = 2 * Wo, kpw = Wo >> 2;
  for (int s = blockIdx.x; s < stages; s += gridDim.x) {
    const int b = s / spi, oy0 = (s - b * spi) * 2;
    __syncthreads();   // the previous stage's fragment reads are done
    {
      // dy', 16-byte chunks: lane = (8 channels) x (8 position quads) -> conflict-free transposing
      // LDS writes; chunk c = (channel octet c / PH, quad octet c % PH); wave w takes c = w, w+4, ...
      const float* dyb = a.dy + (long)b * a.dy_bs + (long)oy0 * Wo;   // rows oy0, oy0+1: P2 contiguous
      const float* yb = a.y + (long)b * a.y_bs + (long)oy0 * Wo;
      const int PH = P2 >> 5, nch = (CO >> 3) * PH, co_lo = lane & 7, q_lo = lane >> 3;
      for (int c0 = wave; c0 < nch; c0 += 32) {
        float4 gv[8], yv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + 4 * u;
          if (c < nch) {
            const long o = (long)((c / PH) * 8 + co_lo) * Ho * Wo + 4 * ((c % PH) * 8 + q_lo);
            gv[u] = *reinterpret_cast<const float4*>(dyb + o);
            yv[u] = *reinterpret_cast<const float4*>(yb + o);
          }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int c = c0 + 4 * u;
          if (c < nch) {
            float* d = dyt + 4 * ((c % PH) * 8 + q_lo) * SC + (c / PH) * 8 + co_lo;
            d[0] = yv[u].x > 0.f ? gv[u].x : gv[u].x * a.slope;
            d[SC] = yv[u].y > 0.f ? gv[u].y : gv[u].y * a.slope;
            d[2 * SC] = yv[u].z > 0.f ? gv[u].z : gv[u].z * a.slope;
            d[3 * SC] = yv[u].w > 0.f ? gv[u].w : gv[u].w * a.slope;
          }
        }
      }
      // (branch-free: a guarded load would be branched around and drain vmcnt per element)
      const __amdgpu_buffer_rsrc_t rxb = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(a.x + (long)b * a.x_bs), (short)0, (unsigned)(CI * H * W * 4), 0x00020000);
      const int W4 = W >> 2, nx = CI * 6 * W4;
      for (int i0 = tid; i0 < nx; i0 += 256 * 8) {
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + 256 * u, ix4 = i % W4, q = i / W4, rr = q % 6, ci = q / 6;
          const int iy = 2 * oy0 - 1 + rr;
          const bool ok = i < nx && (unsigned)iy < (unsigned)H;
          v[u] = pg_ld4(rxb, ok ? (unsigned)((ci * H * W + iy * W + 4 * ix4) * 4) : PG_OOB);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + 256 * u, ix4 = i % W4, q = i / W4, rr = q % 6, ci = q / 6;
          if (i < nx) *reinterpret_cast<float4*>(xt + ci * XS + rr * XC + 4 + 4 * ix4) = v[u];
        }
      }
    }
    __syncthreads();
    for (int kk = 0; kk < kpw; ++kk) {
      const int st = wave * kpw + kk;
      const int p = (st >> 4) * 32 + (st & 15) + 16 * lh;
      const int oyl = p >= Wo ? 1 : 0, ox = p - oyl * Wo;
      const int xo = 2 * oyl * XC + 2 * ox;
      float av[MB], bv[NB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        av[mb] = dyt[p * SC + 32 * mb + lr];
        bs[mb] += av[mb];
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const float v = xt[tb[nb] + xo];
        bv[nb] = tv[nb] ? v : 0.f;
      }
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mb], bv[nb], acc[mb][nb], 0, 0, 0);
    }
  }

  // the four waves' partial sums meet in LDS and leave as one workgroup partial (fixed order)
  __syncthreads();
  float* red = lds;   // [4][CO][NTAP + 1]
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = nb * 32 + lr;
      if (n < NTAP) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * lh;
          red[(wave * CO + m) * (NTAP + 1) + n] = acc[mb][nb][r];
        }
      }
    }
    const float t = bs[mb] + __shfl_xor(bs[mb], 32, 64);
    if (lh == 0) red[(wave * CO + 32 * mb + lr) * (NTAP + 1) + NTAP] = t;
  }
  __syncthreads();
  float* out = a.ws + (long)blockIdx.x * E;
  for (int i = tid; i < E; i += 256) out[i] = ((red[i] + red[E + i]) + red[2 * E + i]) + red[3 * E + i];
}

// ---- data-grad ----------------------------------------------------------------------------------
// Input pixel (2i + py, 2j + px) receives the taps kh = 1 - py (+2), kw = 1 - px (+2):
//   py = 0: (kh 1, oy i), (kh 3, oy i-1)    py = 1: (kh 0, oy i+1), (kh 2, oy i)
//   px = 0: (kw 1, ox j), (kw 3, ox j-1)    px = 1: (kw 0, ox j+1), (kw 2, ox j)
// so the 2x2 block (i, j) reads the 3x3 dy' neighbourhood rows i-1..i+1, cols j-1..j+1.  The two
// column parities run as one packed FMA pair per dy' operand they share (ox j: kw 1 / kw 2; the
// other pair ox j-1 / ox j+1 with kw 3 / kw 0).  Workgroup = RB x CB blocks (256 threads), dy' of
// 32 channels at a time staged with its halo (zero outside the output), lrelu' applied on load.
template <int CI, int CO, int CB>
__global__ __launch_bounds__(256) void pgs_dgrad_kernel(const float* __restrict__ dy, long dy_bs,
                                                        const float* __restrict__ y, long y_bs,
                                                        const float* __restrict__ w, float* __restrict__ dx,
                                                        long dx_bs, int nb, int H, int W, float slope,
                                                        int accumulate) {
  constexpr int RB = 256 / CB, TR = RB + 2, TCP = CB + 8, CS = TR * TCP, C4 = CB / 4;
  // dt[co][row][col]: output row i0 - 1 + row, column j0 + col - 4 (interior 16-byte aligned at
  // col 4; halo columns 3 and CB + 4; zero outside the output)
  __shared__ __attribute__((aligned(16))) float dt[32 * CS];
  const int Ho = H >> 1, Wo = W >> 1;
  const int tr = Ho / RB, tcn = Wo / CB;
  const int tile = blockIdx.x, b = tile / (tr * tcn), q = tile - b * tr * tcn;
  const int i0 = (q / tcn) * RB, j0 = (q % tcn) * CB;
  const int tid = threadIdx.x, rb = tid / CB, cb = tid % CB;
  pg_f2 acc[CI][2];   // [ci][py] = (px 0, px 1)
#pragma unroll
  for (int ci = 0; ci < CI; ++ci) acc[ci][0] = acc[ci][1] = pg_f2{0.f, 0.f};
  const long HWo = (long)Ho * Wo;
#pragma unroll 1
  for (int c0 = 0; c0 < CO; c0 += 32) {
    __syncthreads();
    // branch-free loads (a guarded load would be branched around and drain vmcnt per element)
    const unsigned rng = (unsigned)(32 * HWo * 4);
    const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc((void*)(dy + (long)b * dy_bs + c0 * HWo),
                                                                         (short)0, rng, 0x00020000);
    const __amdgpu_buffer_rsrc_t ryy = __builtin_amdgcn_make_buffer_rsrc((void*)(y + (long)b * y_bs + c0 * HWo),
                                                                         (short)0, rng, 0x00020000);
    constexpr int NI = 32 * TR * C4;       // interior 16-byte items, 8 in flight per lane
    for (int k0 = tid; k0 < NI; k0 += 256 * 8) {
      float4 gv[8], yv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 256 * u, co = k / (TR * C4), rem = k - co * (TR * C4), rr = rem / C4, c4 = rem - rr * C4;
        const int oy = i0 - 1 + rr;
        const unsigned o = k < NI && (unsigned)oy < (unsigned)Ho ? (unsigned)((co * HWo + oy * Wo + j0 + 4 * c4) * 4)
                                                                 : PG_OOB;
        gv[u] = pg_ld4(rdy, o);
        yv[u] = pg_ld4(ryy, o);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + 256 * u, co = k / (TR * C4), rem = k - co * (TR * C4), rr = rem / C4, c4 = rem - rr * C4;
        if (k < NI) {
          float4 v;
          v.x = yv[u].x > 0.f ? gv[u].x : gv[u].x * slope;
          v.y = yv[u].y > 0.f ? gv[u].y : gv[u].y * slope;
          v.z = yv[u].z > 0.f ? gv[u].z : gv[u].z * slope;
          v.w = yv[u].w > 0.f ? gv[u].w : gv[u].w * slope;
          *reinterpret_cast<float4*>(dt + co * CS + rr * TCP + 4 + 4 * c4) = v;
        }
      }
    }
    for (int k = tid; k < 32 * TR * 2; k += 256) {   // halo columns j0 - 1, j0 + CB
      const int co = k / (TR * 2), rem = k - co * (TR * 2), rr = rem >> 1, side = rem & 1;
      const int oy = i0 - 1 + rr, ox = side ? j0 + CB : j0 - 1;
      const unsigned o = (unsigned)oy < (unsigned)Ho && (unsigned)ox < (unsigned)Wo
                             ? (unsigned)((co * HWo + oy * Wo + ox) * 4) : PG_OOB;
      const float g = pg_ld(rdy, o), yy = pg_ld(ryy, o);
      dt[co * CS + rr * TCP + (side ? CB + 4 : 3)] = yy > 0.f ? g : g * slope;
    }
    __syncthreads();
    // channel groups of 3 input channels outside, output channels inside (a runtime loop): 48
    // weights per iteration as scalar-cache operands (unrolled, the compiler hoists all 96 x 32 of
    // them and spills SGPRs; as LDS broadcast reads they bound the kernel on LDS bandwidth)
#pragma unroll
    for (int cg = 0; cg < CI; cg += 3) {
#pragma unroll 1
      for (int co = 0; co < 32; ++co) {
        const float* d = dt + co * CS + rb * TCP + cb + 3;
        float dd[3][3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) dd[r][c] = d[r * TCP + c];
#pragma unroll
        for (int ci = cg; ci < cg + 3 && ci < CI; ++ci) {
          const float* wr = w + ((c0 + co) * CI + ci) * 16;   // [kh][kw]
#pragma unroll
          for (int py = 0; py < 2; ++py) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {   // the two kh taps of this row parity
              const int kh = py == 0 ? (t == 0 ? 1 : 3) : (t == 0 ? 0 : 2);
              const int r = py == 0 ? (t == 0 ? 1 : 0) : (t == 0 ? 2 : 1);
              acc[ci][py] = __builtin_elementwise_fma(pg_f2{wr[kh * 4 + 1], wr[kh * 4 + 2]},
                                                      pg_f2{dd[r][1], dd[r][1]}, acc[ci][py]);
              acc[ci][py] = __builtin_elementwise_fma(pg_f2{wr[kh * 4 + 3], wr[kh * 4 + 0]},
                                                      pg_f2{dd[r][0], dd[r][2]}, acc[ci][py]);
            }
          }
        }
      }
    }
  }
  const int i = i0 + rb, j = j0 + cb;
#pragma unroll
  for (int ci = 0; ci < CI; ++ci)
#pragma unroll
    for (int py = 0; py < 2; ++py) {
      float2* o = reinterpret_cast<float2*>(dx + (long)b * dx_bs + (long)ci * H * W + (long)(2 * i + py) * W + 2 * j);
      float2 v = make_float2(acc[ci][py].x, acc[ci][py].y);
      if (accumulate) { const float2 u = *o; v.x += u.x; v.y += u.y; }
      *o = v;
    }
}

static int pg_wgrad_grid(int N, int H) {
  const int stages = N * (H / 4);
  return stages < 512 ? stages : 512;
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Shapes the stem kernels take: Cin in {3, 6}, Cout in {32, 64}, H % 8 == 0, W % 64 == 0, and
// the weight-grad's LDS stage fitting one workgroup (W <= 512 at Cout 32, <= 256 at Cout 64).
int dsgan_pgstem_supported(int Cin, int Cout, int H, int W) {
  if (!(Cin == 3 || Cin == 6) || !(Cout == 32 || Cout == 64)) return 0;
  if (H <= 0 || W <= 0 || H % 8 || W % 64 || W > 512) return 0;
  if ((W / 2) % 64 && H % 16) return 0;                      // the data-grad's 8-row block tiles
  return pg_wgrad_lds(Cin, Cout, W <= 256 ? 256 : 512) * 4 <= 160 * 1024 ? 1 : 0;
}

#define PG_DISPATCH(CI_, CO_, ...)                                   \
  if (Cin == 3 && Cout == 32) { constexpr int CI_ = 3, CO_ = 32; __VA_ARGS__; }      \
  else if (Cin == 3) { constexpr int CI_ = 3, CO_ = 64; __VA_ARGS__; }               \
  else if (Cout == 32) { constexpr int CI_ = 6, CO_ = 32; __VA_ARGS__; }             \
  else { constexpr int CI_ = 6, CO_ = 64; __VA_ARGS__; }

// y = lrelu(bias + conv4x4s2p1(x, w)), NCHW fp32; w OIHW [Cout][Cin][4][4]; bias nullable.
// (reference: networks.py:543-545, Conv2d(input_nc, ndf, 4, 2, 1) + LeakyReLU(0.2, True))
int dsgan_pgstem_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int N,
                     int Cin, int Cout, int H, int W, float slope, hipStream_t st) {
  DSG_REQUIRE(x && w && y && N > 0, "dsgan_pgstem_fwd: bad args");
  DSG_REQUIRE(dsgan_pgstem_supported(Cin, Cout, H, W), "dsgan_pgstem_fwd: unsupported shape (see dsgan_pgstem_supported)");
  DSG_REQUIRE((x_bs & 3) == 0 && ((uintptr_t)x & 15) == 0, "dsgan_pgstem_fwd: x needs 16-byte aligned planes");
  const long xr = ((long)(N - 1) * x_bs + (long)Cin * H * W) * 4;
  DSG_REQUIRE(xr < (long)PG_OOB - 64, "dsgan_pgstem_fwd: input exceeds 4 GiB");
  const dim3 grid((unsigned)pg_fwd_grid(N, H));
  if (W <= 256) {
    PG_DISPATCH(CI, CO, hipLaunchKernelGGL((pgs_fwd_kernel<CI, CO, 256>), grid, dim3(256), 0, st, x, x_bs, w, bias, y,
                                           y_bs, N, H, W, slope))
  } else {
    PG_DISPATCH(CI, CO, hipLaunchKernelGGL((pgs_fwd_kernel<CI, CO, 512>), grid, dim3(256), 0, st, x, x_bs, w, bias, y,
                                           y_bs, N, H, W, slope))
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

long dsgan_pgstem_wgrad_workspace(int N, int Cin, int Cout, int H, int W) {
  (void)W;
  return (long)pg_wgrad_grid(N, H) * Cout * (Cin * 16 + 1);
}

// dw += dW, db += dB (db nullable) of the stem, from dy (grad of the LeakyReLU output y) and x.
int dsgan_pgstem_wgrad(const float* dy, long dy_bs, const float* y, long y_bs, const float* x, long x_bs, float* dw,
                       float* db, int N, int Cin, int Cout, int H, int W, float slope, float* ws, long ws_elems,
                       hipStream_t st) {
  DSG_REQUIRE(dy && y && x && dw && N > 0, "dsgan_pgstem_wgrad: bad args");
  DSG_REQUIRE(((dy_bs | y_bs | x_bs) & 3) == 0 && (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)x) & 15) == 0,
              "dsgan_pgstem_wgrad: dy, y, x need 16-byte aligned planes");
  DSG_REQUIRE(dsgan_pgstem_supported(Cin, Cout, H, W), "dsgan_pgstem_wgrad: unsupported shape (see dsgan_pgstem_supported)");
  const int grid = pg_wgrad_grid(N, H);
  DSG_WS((long)grid * Cout * (Cin * 16 + 1), ws, ws_elems, "dsgan_pgstem_wgrad (dsgan_pgstem_wgrad_workspace)");
  PgWArgs a{};
  a.dy = dy; a.dy_bs = dy_bs; a.y = y; a.y_bs = y_bs; a.x = x; a.x_bs = x_bs; a.ws = ws;
  a.nb = N; a.H = H; a.W = W; a.XS = pg_xs(W); a.slope = slope;
  if (W <= 256) {
    PG_DISPATCH(CI, CO, hipLaunchKernelGGL((pgs_wgrad_kernel<CI, CO, 256>), dim3(grid), dim3(256), 0, st, a))
  } else {
    PG_DISPATCH(CI, CO, if constexpr (pg_wgrad_lds(CI, CO, 512) * 4 <= 160 * 1024)
                            hipLaunchKernelGGL((pgs_wgrad_kernel<CI, CO, 512>), dim3(grid), dim3(256), 0, st, a))
  }
  launch_split_reduce_kk(ws, grid, (long)Cout * (Cin * 16 + 1), dw, db, Cin * 16 + 1, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dx (+)= the stem's input gradient from dy (grad of the LeakyReLU output y).
int dsgan_pgstem_dgrad(const float* dy, long dy_bs, const float* y, long y_bs, const float* w, float* dx, long dx_bs,
                       int N, int Cin, int Cout, int H, int W, float slope, int accumulate, hipStream_t st) {
  DSG_REQUIRE(dy && y && w && dx && N > 0, "dsgan_pgstem_dgrad: bad args");
  DSG_REQUIRE(dsgan_pgstem_supported(Cin, Cout, H, W), "dsgan_pgstem_dgrad: unsupported shape (see dsgan_pgstem_supported)");
  DSG_REQUIRE((dx_bs & 1) == 0 && ((uintptr_t)dx & 7) == 0, "dsgan_pgstem_dgrad: dx needs 8-byte rows");
  DSG_REQUIRE(((dy_bs | y_bs) & 3) == 0 && (((uintptr_t)dy | (uintptr_t)y) & 15) == 0,
              "dsgan_pgstem_dgrad: dy, y need 16-byte aligned planes");
  const int Wo = W / 2, Ho = H / 2;
  const bool wide = Wo % 64 == 0;
  const int CB = wide ? 64 : 32, RB = 256 / CB;
  DSG_REQUIRE(Ho % RB == 0, "dsgan_pgstem_dgrad: H must be a multiple of %d", 2 * RB);
  const dim3 grid((unsigned)((long)N * (Ho / RB) * (Wo / CB)));
  if (wide) {
    PG_DISPATCH(CI, CO, hipLaunchKernelGGL((pgs_dgrad_kernel<CI, CO, 64>), grid, dim3(256), 0, st, dy, dy_bs, y, y_bs,
                                           w, dx, dx_bs, N, H, W, slope, accumulate))
  } else {
    PG_DISPATCH(CI, CO, hipLaunchKernelGGL((pgs_dgrad_kernel<CI, CO, 32>), grid, dim3(256), 0, st, dy, dy_bs, y, y_bs,
                                           w, dx, dx_bs, N, H, W, slope, accumulate))
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

#undef PG_DISPATCH

}  // extern "C"
