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

__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x, long x_bs,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, long y_bs, int C,
                                                         int H, int W, int K, int flip,
                                                         int tiles_w) {
  __shared__ float tile[DW_HALO][DW_HALO + 1];
  __shared__ float wk[DW_MAXK * DW_MAXK];
  const int plane = blockIdx.y;                 // n * C + c
  const int n = plane / C, c = plane - n * C;
  const int th0 = (blockIdx.x / tiles_w) * DW_T, tw0 = (blockIdx.x % tiles_w) * DW_T;
  const int p = K / 2, E = DW_T + K - 1;
  const float* xp = x + (long)n * x_bs + (long)c * H * W;
  for (int i = threadIdx.x; i < K * K; i += 256) wk[i] = flip ? w[c * K * K + (K * K - 1 - i)] : w[c * K * K + i];
  for (int i = threadIdx.x; i < E * E; i += 256) {
    const int r = i / E, q = i - r * E;
    const int ih = th0 - p + r, iw = tw0 - p + q;
    tile[r][q] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? xp[(long)ih * W + iw] : 0.f;
  }
  __syncthreads();
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows x 32 cols, 4 row-steps
  const float b = bias ? bias[c] : 0.f;
  float acc[4] = {b, b, b, b};
  for (int kh = 0; kh < K; ++kh)
    for (int kw = 0; kw < K; ++kw) {
      const float wv = wk[kh * K + kw];
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[s] += wv * tile[ty + 8 * s + kh][tx + kw];
    }
  float* yp = y + (long)n * y_bs + (long)c * H * W;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int oh = th0 + ty + 8 * s, ow = tw0 + tx;
    if (oh < H && ow < W) yp[(long)oh * W + ow] = acc[s];
  }
}

// dw[c,kh,kw] += sum_{n,h,w} dy[n,c,h,w] * x[n,c,h+kh-p,w+kw-p];  db[c] += sum dy.
// One workgroup per (n,c) plane walks all tiles; thread t owns tap t % K^2 and the rows
// part, part + nparts, ... of each tile; partial sums are combined through LDS once.
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy, long dy_bs,
                                                           const float* __restrict__ x, long x_bs,
                                                           float* __restrict__ dw,
                                                           float* __restrict__ db, int C, int H,
                                                           int W, int K) {
  __shared__ float xt[DW_HALO][DW_HALO + 1];
  __shared__ float gt[DW_T][DW_T + 1];
  __shared__ float red[256];
  const int plane = blockIdx.x;
  const int n = plane / C, c = plane - n * C;
  const int p = K / 2, E = DW_T + K - 1, KK = K * K;
  const int nparts = 256 / KK;
  const int tap = threadIdx.x % KK, part = threadIdx.x / KK;
  const bool active = part < nparts;
  const int kh = tap / K, kw = tap - kh * K;
  const float* xp = x + (long)n * x_bs + (long)c * H * W;
  const float* gp = dy + (long)n * dy_bs + (long)c * H * W;
  float acc = 0.f, bacc = 0.f;
  for (int th0 = 0; th0 < H; th0 += DW_T)
    for (int tw0 = 0; tw0 < W; tw0 += DW_T) {
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
      if (active) {
        const int rmax = min(DW_T, H - th0), cmax = min(DW_T, W - tw0);
        for (int r = part; r < rmax; r += nparts)
          for (int q = 0; q < cmax; ++q) acc += gt[r][q] * xt[r + kh][q + kw];
      }
    }
  // combine parts of each tap
  red[threadIdx.x] = active ? acc : 0.f;
  __syncthreads();
  if (threadIdx.x < KK) {
    float s = 0.f;
    for (int q = 0; q < nparts; ++q) s += red[q * KK + threadIdx.x];
    atomicAdd(dw + c * KK + threadIdx.x, s);
  }
  if (db) {
    __shared__ float sh[4];
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
  DSG_REQUIRE(K >= 1 && K <= DW_MAXK && (K & 1), "dsgan_dwconv_fwd: K must be odd and <= 9");
  const int tw = cdiv(W, DW_T), th = cdiv(H, DW_T);
  DSG_REQUIRE((long)N * C <= 65535, "dsgan_dwconv_fwd: N*C > 65535");
  hipLaunchKernelGGL(dwconv_fwd_kernel, dim3(tw * th, N * C), dim3(256), 0, st, x, x_bs, w, bias, y,
                     y_bs, C, H, W, K, flip, tw);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_dwconv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* db,
                       int N, int C, int H, int W, int K, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && K >= 1 && K <= DW_MAXK && (K & 1), "dsgan_dwconv_wgrad: bad args");
  hipLaunchKernelGGL(dwconv_wgrad_kernel, dim3(N * C), dim3(256), 0, st, dy, dy_bs, x, x_bs, dw, db,
                     C, H, W, K);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
