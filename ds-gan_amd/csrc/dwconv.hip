// Depthwise KxK conv (stride 1, pad K/2, groups = C) -- forward, data-grad, weight/bias-grad.
//
// Reference sites: Block.dwconv 7x7 (DSGAN/models/model/MixConvNeXtML.py:220) and
// MidMLKA.X3/X5/X7/X9 on channel quarters (:94-97, :110-111).  HBM/LDS-bound: one workgroup
// stages a 32x32 output tile plus its (K-1) halo in LDS and every thread produces 4 outputs.
// The data-grad is the forward with the kernel flipped (K odd, pad = K/2).  Inputs/outputs take
// a batch stride so channel slices of a concat buffer are read/written in place.
#include "common.h"

namespace dsg {

constexpr int DW_T = 32;          // output tile edge
constexpr int DW_MAXK = 9;
constexpr int DW_HALO = DW_T + DW_MAXK - 1;

template <int K>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x, long x_bs,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, long y_bs, int C,
                                                         int H, int W, int flip, int tiles_w) {
  __shared__ float tile[DW_HALO][DW_HALO + 1];
  __shared__ float wk[DW_MAXK * DW_MAXK];
  const int plane = blockIdx.y;                 // n * C + c
  const int n = plane / C, c = plane - n * C;
  const int th0 = (blockIdx.x / tiles_w) * DW_T, tw0 = (blockIdx.x % tiles_w) * DW_T;
  constexpr int p = K / 2, E = DW_T + K - 1;
  const float* xp = x + (long)n * x_bs + (long)c * H * W;
  for (int i = threadIdx.x; i < K * K; i += 256) wk[i] = flip ? w[c * K * K + (K * K - 1 - i)] : w[c * K * K + i];
  for (int i = threadIdx.x; i < E * E; i += 256) {
    const int r = i / E, q = i - r * E;
    const int ih = th0 - p + r, iw = tw0 - p + q;
    tile[r][q] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xp[(long)ih * W + iw] : 0.f;
  }
  __syncthreads();
  // thread = one column, 4 consecutive rows: the K+3 input rows of its window are loaded once
  // per kw and reused by all 4 outputs (4K^2 FMAs from (K+3)K LDS reads)
  const int tx = threadIdx.x & 31, r0 = (threadIdx.x >> 5) * 4;
  const float b = bias ? bias[c] : 0.f;
  float acc[4] = {b, b, b, b};
#pragma unroll
  for (int kw = 0; kw < K; ++kw) {
    float v[K + 3];
#pragma unroll
    for (int i = 0; i < K + 3; ++i) v[i] = tile[r0 + i][tx + kw];
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const float wv = wk[kh * K + kw];
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[s] += wv * v[s + kh];
    }
  }
  float* yp = y + (long)n * y_bs + (long)c * H * W;
  const int ow = tw0 + tx;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int oh = th0 + r0 + s;
    if (oh < H && ow < W) yp[(long)oh * W + ow] = acc[s];
  }
}

// dw[c,kh,kw] += sum_{n,h,w} dy[n,c,h,w] * x[n,c,h+kh-p,w+kw-p];  db[c] += sum dy.
// Workgroup = (plane, group of tiles).  Thread item = (kh, tile row r, column half): it walks
// the row keeping a sliding window of K input values in registers, so each step costs two LDS
// reads for K FMAs (all kw taps of its kh); partials are reduced through LDS once at the end.
template <int K>
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy, long dy_bs,
                                                           const float* __restrict__ x, long x_bs,
                                                           float* __restrict__ dw,
                                                           float* __restrict__ db, int C, int H,
                                                           int W, int tiles_per_block) {
  __shared__ float xt[DW_HALO][DW_HALO + 1];
  __shared__ float gt[DW_T][DW_T + 1];
  __shared__ float red[DW_MAXK * DW_MAXK];
  __shared__ float sh[4];
  const int plane = blockIdx.x;
  const int n = plane / C, c = plane - n * C;
  constexpr int p = K / 2, E = DW_T + K - 1;
  constexpr int QS = K * DW_T * 2 <= 256 ? 2 : 1;    // column splits
  constexpr int items = K * DW_T * QS;
  constexpr int qlen = DW_T / QS;
  const float* xp = x + (long)n * x_bs + (long)c * H * W;
  const float* gp = dy + (long)n * dy_bs + (long)c * H * W;
  float acc[2][K];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int kw = 0; kw < K; ++kw) acc[a][kw] = 0.f;
  float bacc = 0.f;
  const int tw_n = (W + DW_T - 1) / DW_T, th_n = (H + DW_T - 1) / DW_T;
  const int ntiles = tw_n * th_n;
  const int t_beg = blockIdx.y * tiles_per_block, t_end = min(ntiles, t_beg + tiles_per_block);
  for (int ti = t_beg; ti < t_end; ++ti) {
    const int th0 = (ti / tw_n) * DW_T, tw0 = (ti % tw_n) * DW_T;
    __syncthreads();
    for (int i = threadIdx.x; i < E * E; i += 256) {
      const int r = i / E, q = i - r * E;
      const int ih = th0 - p + r, iw = tw0 - p + q;
      xt[r][q] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xp[(long)ih * W + iw] : 0.f;
    }
    for (int i = threadIdx.x; i < DW_T * DW_T; i += 256) {
      const int r = i >> 5, q = i & 31;
      const int oh = th0 + r, ow = tw0 + q;
      const float v = (oh < H && ow < W) ? gp[(long)oh * W + ow] : 0.f;
      gt[r][q] = v;
      bacc += v;
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int it = threadIdx.x + a * 256;
      if (it >= items) break;
      const int kh = it / (DW_T * QS), rem = it - kh * DW_T * QS;
      const int r = rem / QS, qs = rem - r * QS;
      const int q0 = qs * qlen;
      const float* xr = &xt[r + kh][q0];
      const float* gr = &gt[r][q0];
      float win[K];                       // win[i] = x[q + i] at step q
#pragma unroll
      for (int j = 0; j < K - 1; ++j) win[j] = xr[j];
#pragma unroll 8
      for (int q = 0; q < qlen; ++q) {
        win[K - 1] = xr[q + K - 1];
        const float gv = gr[q];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) acc[a][kw] += gv * win[kw];
#pragma unroll
        for (int j = 0; j < K - 1; ++j) win[j] = win[j + 1];
      }
    }
  }
  // reduce: for each (kh, kw) sum over rows / column halves
  __syncthreads();
  for (int i = threadIdx.x; i < K * K; i += 256) red[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int it = threadIdx.x + a * 256;
    if (it < items) {
      const int kh = it / (DW_T * QS);
#pragma unroll
      for (int kw = 0; kw < K; ++kw) atomicAdd(&red[kh * K + kw], acc[a][kw]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * K; i += 256) atomicAdd(dw + c * K * K + i, red[i]);
  if (db) {
    const float bs = block_sum<256>(bacc, sh);
    if (threadIdx.x == 0) atomicAdd(db + c, bs);
  }
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// y = dwconv(x, w) + bias   (flip=1, bias=NULL gives the data-grad of dy)
int dsgan_dwconv_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y,
                     long y_bs, int N, int C, int H, int W, int K, int flip, hipStream_t st) {
  DSG_REQUIRE(x && w && y && N > 0 && C > 0 && H > 0 && W > 0, "dsgan_dwconv_fwd: bad args");
  DSG_REQUIRE(K == 3 || K == 5 || K == 7 || K == 9, "dsgan_dwconv_fwd: K must be odd and <= 9");
  const int tw = cdiv(W, DW_T), th = cdiv(H, DW_T);
  DSG_REQUIRE((long)N * C <= 65535, "dsgan_dwconv_fwd: N*C > 65535");
  const dim3 grid(tw * th, N * C);
  switch (K) {
    case 3: hipLaunchKernelGGL(dwconv_fwd_kernel<3>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw); break;
    case 5: hipLaunchKernelGGL(dwconv_fwd_kernel<5>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw); break;
    case 7: hipLaunchKernelGGL(dwconv_fwd_kernel<7>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw); break;
    case 9: hipLaunchKernelGGL(dwconv_fwd_kernel<9>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw); break;
    default: DSG_REQUIRE(false, "dsgan_dwconv_fwd: K must be 3, 5, 7 or 9");
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_dwconv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* db,
                       int N, int C, int H, int W, int K, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && K >= 1 && K <= DW_MAXK && (K & 1), "dsgan_dwconv_wgrad: bad args");
  const int ntiles = cdiv(W, DW_T) * cdiv(H, DW_T);
  // spread a plane's tiles over several workgroups when there are few planes
  int groups = (int)((2048 + (long)N * C - 1) / ((long)N * C));
  if (groups > ntiles) groups = ntiles;
  if (groups < 1) groups = 1;
  const int tpb = (ntiles + groups - 1) / groups;
  groups = (ntiles + tpb - 1) / tpb;
  DSG_REQUIRE((long)N * C < (1L << 31) && groups <= 65535, "dsgan_dwconv_wgrad: grid too large");
  const dim3 grid(N * C, groups);
  switch (K) {
    case 3: hipLaunchKernelGGL(dwconv_wgrad_kernel<3>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, dw, db, C, H, W, tpb); break;
    case 5: hipLaunchKernelGGL(dwconv_wgrad_kernel<5>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, dw, db, C, H, W, tpb); break;
    case 7: hipLaunchKernelGGL(dwconv_wgrad_kernel<7>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, dw, db, C, H, W, tpb); break;
    case 9: hipLaunchKernelGGL(dwconv_wgrad_kernel<9>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, dw, db, C, H, W, tpb); break;
    default: DSG_REQUIRE(false, "dsgan_dwconv_wgrad: K must be 3, 5, 7 or 9");
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
