// Depthwise KxK conv (stride 1, pad K/2, groups = C) -- forward, data-grad, weight/bias-grad.
//
// Reference sites: Block.dwconv 7x7 (DSGAN/models/model/MixConvNeXtML.py:220) and
// MidMLKA.X3/X5/X7/X9 on channel quarters (:94-97, :110-111).  HBM/LDS-bound: one workgroup
// stages a 32x32 output tile plus its (K-1) halo in LDS and every thread produces 4 outputs.
// The data-grad is the forward with the kernel flipped (K odd, pad = K/2).  Inputs/outputs take
// a batch stride so channel slices of a concat buffer are read/written in place.
#include "common.h"
#include <stdlib.h>

namespace dsg {

constexpr int DW_T = 32;          // output tile edge
constexpr int DW_MAXK = 9;
constexpr int DW_HALO = DW_T + DW_MAXK - 1;

template <int K>
__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const float* __restrict__ x, long x_bs,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ y, long y_bs, int C,
                                                         int H, int W, int flip, int tiles_w, int accumulate) {
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
    if (oh < H && ow < W) yp[(long)oh * W + ow] = accumulate ? yp[(long)oh * W + ow] + acc[s] : acc[s];
  }
}

// dw[c,kh,kw] += sum_{n,h,w} dy[n,c,h,w] * x[n,c,h+kh-p,w+kw-p];  db[c] += sum dy.
// Workgroup = (plane, group of tiles).  Thread item = (kh, tile row r, column half): it walks
// the row keeping a sliding window of K input values in registers, so each step costs two LDS
// reads for K FMAs (all kw taps of its kh); partials are reduced through LDS once at the end.
template <int K>
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const float* __restrict__ dy, long dy_bs,
                                                           const float* __restrict__ x, long x_bs,
                                                           float* __restrict__ ws, int C, int H,
                                                           int W, int tiles_per_block) {
  __shared__ float xt[DW_HALO][DW_HALO + 1];
  __shared__ float gt[DW_T][DW_T + 1];
  __shared__ float part[(K * DW_T * 2 <= 256 ? 2 : 1) * K * DW_T][K];
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
  // reduce: for each (kh, kw) the sum over rows / column halves in a fixed order; this
  // workgroup's K*K + 1 partials go to its slot of ws (dsgan_dwconv_wgrad sums the slots)
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int it = threadIdx.x + a * 256;
    if (it < items) {
#pragma unroll
      for (int kw = 0; kw < K; ++kw) part[it][kw] = acc[a][kw];
    }
  }
  const float bs = block_sum<256>(bacc, sh);   // (its barrier also publishes part[])
  const long g = (long)n * gridDim.y + blockIdx.y;              // slot of this workgroup ([g][c][i])
  float* slot = ws + (g * C + c) * (K * K + 1);
  for (int i = threadIdx.x; i < K * K; i += 256) {
    const int kh = i / K, kw = i - kh * K;
    float v = 0.f;
    for (int j = 0; j < DW_T * QS; ++j) v += part[kh * DW_T * QS + j][kw];
    slot[i] = v;
  }
  if (threadIdx.x == 0) slot[K * K] = bs;
}


// ------------------------------------------------------------------------------------------
// Register-blocked variants for W % 4 == 0 planes of width >= 32 (every DS-GAN plane but the
// 16x16 bottleneck).  Thread (tx, ty) owns a 4-column x R-row output block; the workgroup tile
// (4*TWT) x (R*THT) plus halo is staged as float4 rows with the LDS column origin 4 to the left
// of the tile, so each input row of a thread's window is three ds_read_b128 and serves
// up to R*4*K FMAs.  The per-plane weights are wave-uniform (scalar loads).
// ------------------------------------------------------------------------------------------
// LDS row pitch (floats) of a tile whose loaded rows are lw floats: the window reads are
// ds_read_b128 whose 16-lane groups span two thread rows (TWT = 16: rows ty, ty+1) or four (TWT = 8),
// R tile rows apart; a pitch with R*LP = 0 (TWT 16) / 32 (TWT 8) mod 64 dwords puts them in disjoint
// bank ranges (tools/lds_banks.py: 2-3-way -> conflict-free; the staging writes become 1.3-1.6-way)
constexpr int dw_pitch(int twt, int r, int lw) {
  if (twt != 16 && twt != 8) return lw;
  const int tgt = twt == 16 ? 0 : 32;
  int lp = lw;
  while ((r * lp) % 64 != tgt) lp += 4;
  return lp;
}

template <int K, int TWT, int THT, int R>
struct DwTile {
  static constexpr int TW = 4 * TWT, TH = R * THT, P = K / 2;
  static constexpr int LW = TW + 8, LH = TH + K - 1, F4 = LW / 4;
  static constexpr int LP = dw_pitch(TWT, R, LW);   // LDS pitch (LW loaded, LP apart)
  static constexpr int OFF = 4 - P;      // LDS column of input (out col - P) for i = kw = 0
  static_assert(TWT * THT == 256, "256 threads");
};

// 1-D grid, XCD-aware: workgroup id -> logical index so that each XCD walks one contiguous range
// (dispatch round-robins ids over the 8 XCDs): the tiles of a plane, which share halo rows and
// columns, run on one XCD and re-read those halos from its L2 instead of HBM.
__device__ __forceinline__ int dw_xcd_index() {
  const int nwg = gridDim.x, id = blockIdx.x;
  const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
}

template <int K, int TWT, int THT, int R, bool BATCH = false>
__device__ __forceinline__ void dw_stage(float* tile, const float* __restrict__ xp, int H, int W, int th0, int tw0) {
  using T = DwTile<K, TWT, THT, R>;
  if constexpr (BATCH) {
    // every 16-byte load of the halo tile is issued before the first LDS write (one memory
    // latency per tile instead of one per item; ITEMS x 4 VGPRs, which the forward can afford)
    constexpr int ITEMS = (T::LH * T::F4 + 255) / 256;
    float4 v[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = threadIdx.x + j * 256;
      const int r = i / T::F4, q = i - r * T::F4;
      const int ih = th0 - T::P + r, iw = tw0 - 4 + 4 * q;
      v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < T::LH * T::F4 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        v[j] = *reinterpret_cast<const float4*>(xp + (long)ih * W + iw);
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = threadIdx.x + j * 256;
      const int r = i / T::F4, q = i - r * T::F4;
      if (i < T::LH * T::F4) *reinterpret_cast<float4*>(tile + r * T::LP + 4 * q) = v[j];
    }
    return;
  }
  for (int i = threadIdx.x; i < T::LH * T::F4; i += 256) {
    const int r = i / T::F4, q = i - r * T::F4;
    const int ih = th0 - T::P + r, iw = tw0 - 4 + 4 * q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = *reinterpret_cast<const float4*>(xp + (long)ih * W + iw);
    *reinterpret_cast<float4*>(tile + r * T::LP + 4 * q) = v;
  }
}

// One window row as three ds_read_b128.  The empty asm pins every component: without it the
// compiler drops the window elements a K < 9 kernel never touches and splits the rest into
// ds_read2_b32 pairs, whose 32-bank lane groups see the 16-B lane stride as a 4-way conflict
// (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.70 measured); b128 lane groups are conflict-free here.
typedef __attribute__((ext_vector_type(4))) float dwf4;
template <int K>   // (K = 9 uses the whole window: already b128, and the pin would spill it)
__device__ __forceinline__ void dw_row(float (&v)[12], const float* row) {
  dwf4 a = *reinterpret_cast<const dwf4*>(row);
  dwf4 b = *reinterpret_cast<const dwf4*>(row + 4);
  dwf4 c = *reinterpret_cast<const dwf4*>(row + 8);
  if constexpr (K < 9) asm volatile("" ::"v"(a), "v"(b), "v"(c));
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[i] = a[i]; v[4 + i] = b[i]; v[8 + i] = c[i]; }
}

// One workgroup's output tile (bx) of plane `plane`; `tile` = LDS of DwTile<K,...>::LH * LP floats.
template <int K, int TWT, int THT, int R>
__device__ __forceinline__ void dw_fwd_body(const float* __restrict__ x, long x_bs, const float* __restrict__ w,
                                            const float* __restrict__ bias, float* __restrict__ y, long y_bs, int C,
                                            int H, int W, int flip, int accumulate, int tiles_w, int bx, int plane,
                                            float* tile) {
  using T = DwTile<K, TWT, THT, R>;
  const int n = plane / C, c = plane - n * C;
  const int th0 = (bx / tiles_w) * T::TH, tw0 = (bx % tiles_w) * T::TW;
  dw_stage<K, TWT, THT, R, true>(tile, x + (long)n * x_bs + (long)c * H * W, H, W, th0, tw0);
  float wv[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wv[i] = w[c * K * K + (flip ? K * K - 1 - i : i)];
  const float b = bias ? bias[c] : 0.f;
  const int tx = threadIdx.x % TWT, ty = threadIdx.x / TWT;
  float acc[R][4];
#pragma unroll
  for (int s = 0; s < R; ++s)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[s][i] = b;
  __syncthreads();
  // one input row in flight ahead of the FMAs; the scheduling barrier keeps the compiler from
  // hoisting every row load of the unrolled loop (which costs occupancy or spills)
  float cur[12], nxt[12];
  dw_row<K>(cur, tile + (R * ty) * T::LP + 4 * tx);
#pragma unroll
  for (int r = 0; r < R + K - 1; ++r) {
    if (r + 1 < R + K - 1) dw_row<K>(nxt, tile + (R * ty + r + 1) * T::LP + 4 * tx);
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const int kh = r - s;
      if (kh < 0 || kh >= K) continue;
#pragma unroll
      for (int kw = 0; kw < K; ++kw)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[s][i] = fmaf(wv[kh * K + kw], cur[i + kw + T::OFF], acc[s][i]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // pin this row's FMAs here: otherwise the compiler sinks every FMA below the last row read and
    // computes one output row at a time, which keeps all R + K - 1 window rows live (127 VGPRs,
    // 4 waves per SIMD; pinned: 44 VGPRs, the LDS-bound 7 workgroups per CU).  Same FMA order per
    // accumulator, same bits.
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(acc[s][i])::"memory");
#pragma unroll
    for (int i = 0; i < 12; ++i) cur[i] = nxt[i];
  }
  // (loading the accumulated values before the FMAs instead measured 2.5 % slower: dw_micro A/B)
  float* yp = y + (long)n * y_bs + (long)c * H * W + tw0 + 4 * tx;
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const int oh = th0 + R * ty + s;
    if (oh >= H) continue;
    float4* o = reinterpret_cast<float4*>(yp + (long)oh * W);
    float4 v = make_float4(acc[s][0], acc[s][1], acc[s][2], acc[s][3]);
    if (accumulate) {
      const float4 u = *o;
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    *o = v;
  }
}

template <int K, int TWT, int THT, int R>
__global__ __launch_bounds__(256, 4) void dwconv_fwd_v2(const float* __restrict__ x, long x_bs,
                                                     const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     float* __restrict__ y, long y_bs, int C, int H,
                                                     int W, int flip, int accumulate, int tiles_w, int tiles) {
  using T = DwTile<K, TWT, THT, R>;
  __shared__ __attribute__((aligned(16))) float tile[T::LH * T::LP];
  const int t = dw_xcd_index(), plane = t / tiles;
  dw_fwd_body<K, TWT, THT, R>(x, x_bs, w, bias, y, y_bs, C, H, W, flip, accumulate, tiles_w, t - plane * tiles, plane,
                              tile);
}

// MidMLKA's four channel quarters (X3/X5/X7/X9 depthwise, MixConvNeXtML.py:94-97,110-111) in one
// launch: blockIdx.z = quarter (K = 3 + 2z), one tile configuration for all four (the 9x9-safe
// rows per thread).  The quarters' launches are each too small to fill the chip on their own.
struct DwQuad { const float* w[4]; const float* b[4]; float* ws[4]; float* dw[4]; float* db[4]; };

template <int TWT, int THT, int R>
__global__ __launch_bounds__(256, 3) void dwconv_multi_fwd(const float* __restrict__ x, long x_bs, DwQuad q4,
                                                           float* __restrict__ y, long y_bs, int q, int H, int W,
                                                           int flip, int accumulate, int tiles_w) {
  using T = DwTile<9, TWT, THT, R>;
  __shared__ __attribute__((aligned(16))) float tile[T::LH * T::LP];
  const int qi = blockIdx.z;
  const float* xq = x + (long)qi * q * H * W;
  float* yq = y + (long)qi * q * H * W;
  switch (qi) {
    case 0: dw_fwd_body<3, TWT, THT, R>(xq, x_bs, q4.w[0], q4.b[0], yq, y_bs, q, H, W, flip, accumulate, tiles_w, blockIdx.x, blockIdx.y, tile); break;
    case 1: dw_fwd_body<5, TWT, THT, R>(xq, x_bs, q4.w[1], q4.b[1], yq, y_bs, q, H, W, flip, accumulate, tiles_w, blockIdx.x, blockIdx.y, tile); break;
    case 2: dw_fwd_body<7, TWT, THT, R>(xq, x_bs, q4.w[2], q4.b[2], yq, y_bs, q, H, W, flip, accumulate, tiles_w, blockIdx.x, blockIdx.y, tile); break;
    default: dw_fwd_body<9, TWT, THT, R>(xq, x_bs, q4.w[3], q4.b[3], yq, y_bs, q, H, W, flip, accumulate, tiles_w, blockIdx.x, blockIdx.y, tile); break;
  }
}

// dw[c] += sum over (images [n0, n0+nper), tile) of the 7x7 (KxK) correlation of dy with x;
// db[c] += sum dy.  The dy block of a thread stays in registers; partial sums are reduced over
// the workgroup once, after all of its images.
// Weight-grad partials of channel c, tile bx, image split `split` (slot split * ntiles + bx).
// `tile` = LH * LP floats of LDS, `red` = 4 * (K*K + 1) floats.
template <int K, int TWT, int THT, int R, bool PF = false>
__device__ __forceinline__ void dw_wgrad_body(const float* __restrict__ dy, long dy_bs, const float* __restrict__ x,
                                              long x_bs, float* __restrict__ ws, int N, int C, int H, int W,
                                              int tiles_w, int nper, int bx, int c, int split, int ntiles, float* tile,
                                              float* red_) {
  using T = DwTile<K, TWT, THT, R>;
  float (*red)[K * K + 1] = reinterpret_cast<float (*)[K * K + 1]>(red_);
  const int th0 = (bx / tiles_w) * T::TH, tw0 = (bx % tiles_w) * T::TW;
  const int n0 = split * nper, n1 = min(N, n0 + nper);
  const int tx = threadIdx.x % TWT, ty = threadIdx.x / TWT;
  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  float bacc = 0.f;
  // PF: the next image's halo tile and dy block are loaded into registers while this image's FMAs
  // run (the loop otherwise waits one memory latency per image); same values, same bits
  constexpr int ITEMS = (T::LH * T::F4 + 255) / 256;
  float4 pv[PF ? ITEMS : 1], pg[PF ? R : 1];
  auto issue = [&](int n) {
    const float* xp = x + (long)n * x_bs + (long)c * H * W;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const int i = threadIdx.x + j * 256;
      const int r = i / T::F4, q = i - r * T::F4;
      const int ih = th0 - T::P + r, iw = tw0 - 4 + 4 * q;
      pv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < T::LH * T::F4 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        pv[j] = *reinterpret_cast<const float4*>(xp + (long)ih * W + iw);
    }
    const float* gp = dy + (long)n * dy_bs + (long)c * H * W + tw0 + 4 * tx;
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const int oh = th0 + R * ty + s;
      pg[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (oh < H) pg[s] = *reinterpret_cast<const float4*>(gp + (long)oh * W);
    }
  };
  if constexpr (PF) {
    if (n0 < n1) issue(n0);
  }
  for (int n = n0; n < n1; ++n) {
    __syncthreads();
    float g[R][4];
    if constexpr (PF) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const int i = threadIdx.x + j * 256;
        const int r = i / T::F4, q = i - r * T::F4;
        if (i < T::LH * T::F4) *reinterpret_cast<float4*>(tile + r * T::LP + 4 * q) = pv[j];
      }
#pragma unroll
      for (int s = 0; s < R; ++s) {
        const float4 v = pg[s];
        g[s][0] = v.x; g[s][1] = v.y; g[s][2] = v.z; g[s][3] = v.w;
        bacc += (v.x + v.y) + (v.z + v.w);
      }
    } else {
      dw_stage<K, TWT, THT, R>(tile, x + (long)n * x_bs + (long)c * H * W, H, W, th0, tw0);
      const float* gp = dy + (long)n * dy_bs + (long)c * H * W + tw0 + 4 * tx;
#pragma unroll
      for (int s = 0; s < R; ++s) {
        const int oh = th0 + R * ty + s;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (oh < H) v = *reinterpret_cast<const float4*>(gp + (long)oh * W);
        g[s][0] = v.x; g[s][1] = v.y; g[s][2] = v.z; g[s][3] = v.w;
        bacc += (v.x + v.y) + (v.z + v.w);
      }
    }
    __syncthreads();
    if constexpr (PF) {
      if (n + 1 < n1) issue(n + 1);
    }
    float cur[12], nxt[12];
    dw_row<K>(cur, tile + (R * ty) * T::LP + 4 * tx);
#pragma unroll
    for (int r = 0; r < R + K - 1; ++r) {
      if (r + 1 < R + K - 1) dw_row<K>(nxt, tile + (R * ty + r + 1) * T::LP + 4 * tx);
#pragma unroll
      for (int s = 0; s < R; ++s) {
        const int kh = r - s;
        if (kh < 0 || kh >= K) continue;
#pragma unroll
        for (int kw = 0; kw < K; ++kw)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[kh * K + kw] = fmaf(g[s][i], cur[i + kw + T::OFF], acc[kh * K + kw]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 12; ++i) cur[i] = nxt[i];
    }
  }
  // workgroup reduction of the K*K + 1 partials
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < K * K; ++i) {
    const float v = warp_sum(acc[i]);
    if (lane == 0) red[wv][i] = v;
  }
  {
    const float v = warp_sum(bacc);
    if (lane == 0) red[wv][K * K] = v;
  }
  __syncthreads();
  if (threadIdx.x < K * K + 1) {   // this workgroup's slot of ws (summed in order by dw_partial_reduce)
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    const long g = (long)split * ntiles + bx;   // slot layout [g][c][i]
    ws[(g * C + c) * (K * K + 1) + threadIdx.x] = v;
  }
}

template <int K, int TWT, int THT, int R, bool PF = false>
__global__ __launch_bounds__(256, PF ? 3 : 4) void dwconv_wgrad_v2(const float* __restrict__ dy, long dy_bs,
                                                       const float* __restrict__ x, long x_bs,
                                                       float* __restrict__ ws,
                                                       int N, int C, int H, int W, int tiles_w, int nper, int tiles) {
  using T = DwTile<K, TWT, THT, R>;
  __shared__ __attribute__((aligned(16))) float tile[T::LH * T::LP];
  __shared__ float red[4 * (K * K + 1)];
  const int t = dw_xcd_index(), cs = t / tiles, split = cs / C;   // t = (split * C + c) * tiles + tile
  dw_wgrad_body<K, TWT, THT, R, PF>(dy, dy_bs, x, x_bs, ws, N, C, H, W, tiles_w, nper, t - cs * tiles, cs - split * C,
                                    split, tiles, tile, red);
}

// The four MidMLKA quarters' weight-grads in one launch: blockIdx.z = quarter * nsplit + split.
template <int TWT, int THT, int R, bool PF = false>
__global__ __launch_bounds__(256, PF ? 3 : 4) void dwconv_multi_wgrad(const float* __restrict__ dy, long dy_bs,
                                                             const float* __restrict__ x, long x_bs, DwQuad q4,
                                                             int N, int q, int H, int W, int tiles_w, int nper,
                                                             int nsplit) {
  using T = DwTile<9, TWT, THT, R>;
  __shared__ __attribute__((aligned(16))) float tile[T::LH * T::LP];
  __shared__ float red[4 * 82];
  const int qi = blockIdx.z / nsplit, split = blockIdx.z - qi * nsplit;
  const long co = (long)qi * q * H * W;
  switch (qi) {
    case 0: dw_wgrad_body<3, TWT, THT, R, PF>(dy + co, dy_bs, x + co, x_bs, q4.ws[0], N, q, H, W, tiles_w, nper, blockIdx.x, blockIdx.y, split, gridDim.x, tile, red); break;
    case 1: dw_wgrad_body<5, TWT, THT, R, PF>(dy + co, dy_bs, x + co, x_bs, q4.ws[1], N, q, H, W, tiles_w, nper, blockIdx.x, blockIdx.y, split, gridDim.x, tile, red); break;
    case 2: dw_wgrad_body<7, TWT, THT, R, PF>(dy + co, dy_bs, x + co, x_bs, q4.ws[2], N, q, H, W, tiles_w, nper, blockIdx.x, blockIdx.y, split, gridDim.x, tile, red); break;
    default: dw_wgrad_body<9, TWT, THT, R, PF>(dy + co, dy_bs, x + co, x_bs, q4.ws[3], N, q, H, W, tiles_w, nper, blockIdx.x, blockIdx.y, split, gridDim.x, tile, red); break;
  }
}

// tile configuration by plane width: 0 = generic kernel
static int dw_cfg(int H, int W) {
  if ((W & 3) || H < 8) return 0;
  // (built with -fno-slp-vectorize: packed-f32 FMAs would need even-aligned register pairs of
  // the shifted input window and spill)
  if (W % 128 == 0) return 1;   // 128 x 64 tile, 4x8 per thread
  if (W == 64) return 2;        // 64 x 64, 4x4
  if (W == 32) return 3;        // 32 x 32, 4x1
  return 0;
}

template <int K, int TWT, int THT, int R>
static void dw_fwd_v2(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs,
                      int N, int C, int H, int W, int flip, int accumulate, hipStream_t st) {
  using T = DwTile<K, TWT, THT, R>;
  const int tw = W / T::TW, th = (H + T::TH - 1) / T::TH;
  hipLaunchKernelGGL((dwconv_fwd_v2<K, TWT, THT, R>), dim3(tw * th * N * C), dim3(256), 0, st, x, x_bs, w, bias, y,
                     y_bs, C, H, W, flip, accumulate, tw, tw * th);
}

// images per workgroup of the tiled weight-grad: about `target` workgroups, as many images each as
// that allows -- every workgroup ends in a block reduction of its K*K+1 sums, so a workgroup per
// image tile over-fills the chip with reductions (tools/dw_wgrad_micro.py, B=16: the 7x7 launches
// are fastest at ~1024 workgroups, the four-quarter MidMLKA launch at ~256 per quarter set:
// 1024 ch @ 32^2 67 -> 55 us, C=128 @ 128^2 quarters 162 -> 99 us).  Returns the workgroups per
// channel (= partial slots).
template <int K, int TWT, int THT, int R>
static long dw_wgrad_v2_plan(int N, int C, int H, int W, int* nsplit_out, int* nper_out, long target = 1024) {
  using T = DwTile<K, TWT, THT, R>;
  const int tw = W / T::TW, th = (H + T::TH - 1) / T::TH;
  const long base = (long)tw * th * C;
  int nsplit = (int)((target + base - 1) / base);
  if (nsplit > N) nsplit = N;
  const int nper = (N + nsplit - 1) / nsplit;
  nsplit = (N + nper - 1) / nper;
  *nsplit_out = nsplit;
  *nper_out = nper;
  return (long)tw * th * nsplit;
}

template <int K, int TWT, int THT, int R, bool PF = false>
static long dw_wgrad_v2(const float* dy, long dy_bs, const float* x, long x_bs, float* ws, int N, int C, int H, int W,
                        hipStream_t st) {
  using T = DwTile<K, TWT, THT, R>;
  const int tw = W / T::TW, th = (H + T::TH - 1) / T::TH;
  int nsplit, nper;
  const long G = dw_wgrad_v2_plan<K, TWT, THT, R>(N, C, H, W, &nsplit, &nper);
  if (ws)
    hipLaunchKernelGGL((dwconv_wgrad_v2<K, TWT, THT, R, PF>), dim3(tw * th * C * nsplit), dim3(256), 0, st, dy, dy_bs, x,
                       x_bs, ws, N, C, H, W, tw, nper, tw * th);
  return G;
}

// rows per thread: as many as the registers allow without spilling (K = 7, 9 windows are big)
template <int K>
static void dw_fwd_dispatch(int cfg, const float* x, long x_bs, const float* w, const float* bias, float* y,
                            long y_bs, int N, int C, int H, int W, int flip, int accumulate, hipStream_t st) {
  constexpr int R1 = K >= 9 ? 2 : K >= 7 ? 4 : 8, R2 = K >= 9 ? 2 : 4;
  if (cfg == 1) dw_fwd_v2<K, 32, 8, R1>(x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st);
  else if (cfg == 2) dw_fwd_v2<K, 16, 16, R2>(x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st);
  else dw_fwd_v2<K, 8, 32, 1>(x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st);
}

// ws == NULL: only the partial-slot count per channel is returned (workspace query)
// Workgroups that walk >= 8 images prefetch the next image's tile and dy block under the FMAs
// (dw_wgrad_body PF; the 7x7 128-wide tiles then take 4 rows per thread so the prefetch registers
// fit).  Build A/B at the step's shapes (profiles/r04/dw_micro_wgpf.txt): 289 -> 252 us at
// C=128 @ 256^2, 165 -> 144 at 256 @ 128^2, 54 -> 46 at 1024 @ 32^2; with 2-4 images per workgroup
// the lower occupancy lost 8-12 %, so those keep the plain loop.
constexpr int DW_PF_MIN_IMAGES = 8;
template <int K, int TWT, int THT, int R, int RPF>
static long dw_wgrad_pick(const float* dy, long dy_bs, const float* x, long x_bs, float* ws, int N, int C, int H,
                          int W, hipStream_t st) {
  int nsplit, nper;
  dw_wgrad_v2_plan<K, TWT, THT, RPF>(N, C, H, W, &nsplit, &nper);
  if (nper >= DW_PF_MIN_IMAGES) return dw_wgrad_v2<K, TWT, THT, RPF, true>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  return dw_wgrad_v2<K, TWT, THT, R>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
}
template <int K>
static long dw_wgrad_dispatch(int cfg, const float* dy, long dy_bs, const float* x, long x_bs, float* ws,
                              int N, int C, int H, int W, hipStream_t st) {
  constexpr int R1 = K >= 9 ? 2 : 8, R2 = K >= 9 ? 2 : 4;
  if constexpr (K == 7) {
    if (cfg == 1) return dw_wgrad_pick<7, 32, 8, R1, 4>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
    if (cfg == 2) return dw_wgrad_pick<7, 16, 16, R2, R2>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
    return dw_wgrad_pick<7, 8, 32, 1, 1>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  }
  if (cfg == 1) return dw_wgrad_v2<K, 32, 8, R1>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  if (cfg == 2) return dw_wgrad_v2<K, 16, 16, R2>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  return dw_wgrad_v2<K, 8, 32, 1>(dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
}

static long dw_wgrad_any(int K, int cfg, const float* dy, long dy_bs, const float* x, long x_bs, float* ws, int N,
                         int C, int H, int W, hipStream_t st) {
  switch (K) {
    case 3: return dw_wgrad_dispatch<3>(cfg, dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
    case 5: return dw_wgrad_dispatch<5>(cfg, dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
    case 7: return dw_wgrad_dispatch<7>(cfg, dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
    default: return dw_wgrad_dispatch<9>(cfg, dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  }
}

// generic kernel: (tiles per workgroup, workgroups per plane)
static int dw_generic_groups(int N, int C, int H, int W, int* tpb_out) {
  const int ntiles = cdiv(W, DW_T) * cdiv(H, DW_T);
  int groups = (int)((2048 + (long)N * C - 1) / ((long)N * C));   // spread a plane's tiles when planes are few
  if (groups > ntiles) groups = ntiles;
  if (groups < 1) groups = 1;
  const int tpb = (ntiles + groups - 1) / groups;
  *tpb_out = tpb;
  return (ntiles + tpb - 1) / tpb;
}

static bool dw_tiled_ok(int K, int cfg, const void* x, const void* dy, long x_bs, long dy_bs) {
  return cfg && K >= 3 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 && (x_bs & 3) == 0 && (dy_bs & 3) == 0;
}

// MidMLKA quarters: one tile configuration for all four kernel sizes (rows per thread safe for
// 9x9: cfg 1 -> 32 x 8 threads x 2 rows, cfg 2 -> 16 x 16 x 2, cfg 3 -> 8 x 32 x 1)
template <int TWT, int THT, int R>
static void dw_multi_fwd_launch(const float* x, long x_bs, const DwQuad& q4, float* y, long y_bs, int N, int q, int H,
                                int W, int flip, int accumulate, hipStream_t st) {
  using T = DwTile<9, TWT, THT, R>;
  const int tw = W / T::TW, th = (H + T::TH - 1) / T::TH;
  hipLaunchKernelGGL((dwconv_multi_fwd<TWT, THT, R>), dim3(tw * th, N * q, 4), dim3(256), 0, st, x, x_bs, q4, y, y_bs,
                     q, H, W, flip, accumulate, tw);
}

template <int TWT, int THT, int R>
static long dw_multi_wgrad_run(const float* dy, long dy_bs, const float* x, long x_bs, const DwQuad* q4, int N, int q,
                               int H, int W, hipStream_t st) {
  using T = DwTile<9, TWT, THT, R>;
  const int tw = W / T::TW, th = (H + T::TH - 1) / T::TH;
  int nsplit, nper;
  const long G = dw_wgrad_v2_plan<9, TWT, THT, R>(N, q, H, W, &nsplit, &nper, 256);
  if (q4) {
    // (the next-image prefetch where a workgroup walks >= 8 images: 101 -> 98 us at C = 128 @ 128^2,
    // profiles/r04/dw_micro_multi_pf.txt; shorter loops lose 2-6 % to the lower occupancy)
    if (nper >= DW_PF_MIN_IMAGES)
      hipLaunchKernelGGL((dwconv_multi_wgrad<TWT, THT, R, true>), dim3(tw * th, q, 4 * nsplit), dim3(256), 0, st, dy,
                         dy_bs, x, x_bs, *q4, N, q, H, W, tw, nper, nsplit);
    else
      hipLaunchKernelGGL((dwconv_multi_wgrad<TWT, THT, R, false>), dim3(tw * th, q, 4 * nsplit), dim3(256), 0, st, dy,
                         dy_bs, x, x_bs, *q4, N, q, H, W, tw, nper, nsplit);
  }
  return G;
}

static long dw_multi_wgrad_any(int cfg, const float* dy, long dy_bs, const float* x, long x_bs, const DwQuad* q4,
                               int N, int q, int H, int W, hipStream_t st) {
  if (cfg == 1) return dw_multi_wgrad_run<32, 8, 2>(dy, dy_bs, x, x_bs, q4, N, q, H, W, st);
  if (cfg == 2) return dw_multi_wgrad_run<16, 16, 2>(dy, dy_bs, x, x_bs, q4, N, q, H, W, st);
  return dw_multi_wgrad_run<8, 32, 1>(dy, dy_bs, x, x_bs, q4, N, q, H, W, st);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// MidMLKA chunk(4) -> X3/X5/X7/X9 depthwise (MixConvNeXtML.py:94-97,110-111) as one launch per
// pass.  Supported when every quarter takes a tiled configuration: W % 4 == 0, W in {32, 64,
// multiples of 128}, 16-byte aligned x / y (dy) with batch strides % 4 == 0.
int dsgan_dwconv_multi_supported(int H, int W, const void* x, long x_bs, const void* y, long y_bs) {
  return dw_cfg(H, W) != 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && (x_bs & 3) == 0 &&
         (y_bs & 3) == 0;
}

// y[:, 4 quarters] (+)= dwconv_{3,5,7,9}(x quarter) + bias (flip = 1, biases NULL: the data-grad)
int dsgan_dwconv_multi_fwd(const float* x, long x_bs, const float* w3, const float* b3, const float* w5,
                           const float* b5, const float* w7, const float* b7, const float* w9, const float* b9,
                           float* y, long y_bs, int N, int q, int H, int W, int flip, int accumulate, hipStream_t st) {
  DSG_REQUIRE(x && y && w3 && w5 && w7 && w9 && N > 0 && q > 0, "dsgan_dwconv_multi_fwd: bad args");
  DSG_REQUIRE(dsgan_dwconv_multi_supported(H, W, x, x_bs, y, y_bs) && (long)N * q <= 65535,
              "dsgan_dwconv_multi_fwd: unsupported H=%d W=%d / alignment", H, W);
  DwQuad q4{};
  q4.w[0] = w3; q4.w[1] = w5; q4.w[2] = w7; q4.w[3] = w9;
  q4.b[0] = b3; q4.b[1] = b5; q4.b[2] = b7; q4.b[3] = b9;
  const int cfg = dw_cfg(H, W);
  if (cfg == 1) dw_multi_fwd_launch<32, 8, 2>(x, x_bs, q4, y, y_bs, N, q, H, W, flip, accumulate, st);
  else if (cfg == 2) dw_multi_fwd_launch<16, 16, 2>(x, x_bs, q4, y, y_bs, N, q, H, W, flip, accumulate, st);
  else dw_multi_fwd_launch<8, 32, 1>(x, x_bs, q4, y, y_bs, N, q, H, W, flip, accumulate, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// floats of scratch: the four quarters' slot partials, back to back (quarter K uses G*q*(K*K+1))
long dsgan_dwconv_multi_wgrad_workspace(int N, int q, int H, int W) {
  const int cfg = dw_cfg(H, W);
  if (!cfg) return 0;
  const long G = dw_multi_wgrad_any(cfg, nullptr, 0, nullptr, 0, nullptr, N, q, H, W, 0);
  return G * q * (10 + 26 + 50 + 82);
}

// dw_K += sum dy * x, db_K += sum dy for the four quarters (fixed-order slot reduction)
int dsgan_dwconv_multi_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw3, float* db3,
                             float* dw5, float* db5, float* dw7, float* db7, float* dw9, float* db9, int N, int q,
                             int H, int W, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw3 && dw5 && dw7 && dw9 && N > 0 && q > 0 && q <= 65535,
              "dsgan_dwconv_multi_wgrad: bad args");
  DSG_REQUIRE(dsgan_dwconv_multi_supported(H, W, x, x_bs, dy, dy_bs), "dsgan_dwconv_multi_wgrad: unsupported H=%d W=%d",
              H, W);
  const int cfg = dw_cfg(H, W);
  const long G = dw_multi_wgrad_any(cfg, nullptr, 0, nullptr, 0, nullptr, N, q, H, W, 0);
  DSG_WS(G * q * (10 + 26 + 50 + 82), ws, ws_elems, "dsgan_dwconv_multi_wgrad (dsgan_dwconv_multi_wgrad_workspace)");
  DwQuad q4{};
  float* dws[4] = {dw3, dw5, dw7, dw9};
  float* dbs[4] = {db3, db5, db7, db9};
  long off = 0;
  for (int i = 0; i < 4; ++i) {
    const int K = 3 + 2 * i;
    q4.ws[i] = ws + off;
    off += G * q * (K * K + 1);
  }
  dw_multi_wgrad_any(cfg, dy, dy_bs, x, x_bs, &q4, N, q, H, W, st);
  DSG_CHECK_LAUNCH();
  for (int i = 0; i < 4; ++i) {
    const int K = 3 + 2 * i;
    launch_split_reduce_kk(q4.ws[i], (int)G, (long)q * (K * K + 1), dws[i], dbs[i], K * K + 1, st);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

// y (+)= dwconv(x, w) + bias   (flip=1, bias=NULL gives the data-grad of dy; accumulate adds
// into y -- the data-grad of a tensor that has another consumer)
int dsgan_dwconv_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y,
                     long y_bs, int N, int C, int H, int W, int K, int flip, int accumulate, hipStream_t st) {
  DSG_REQUIRE(x && w && y && N > 0 && C > 0 && H > 0 && W > 0, "dsgan_dwconv_fwd: bad args");
  DSG_REQUIRE(K == 3 || K == 5 || K == 7 || K == 9, "dsgan_dwconv_fwd: K must be odd and <= 9");
  DSG_REQUIRE((long)N * C <= 65535, "dsgan_dwconv_fwd: N*C > 65535");
  const int cfg = dw_cfg(H, W);
  if (cfg && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && (x_bs & 3) == 0 && (y_bs & 3) == 0) {
    switch (K) {
      case 3: dw_fwd_dispatch<3>(cfg, x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st); break;
      case 5: dw_fwd_dispatch<5>(cfg, x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st); break;
      case 7: dw_fwd_dispatch<7>(cfg, x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st); break;
      default: dw_fwd_dispatch<9>(cfg, x, x_bs, w, bias, y, y_bs, N, C, H, W, flip, accumulate, st); break;
    }
    DSG_CHECK_LAUNCH();
    return 0;
  }
  const int tw = cdiv(W, DW_T), th = cdiv(H, DW_T);
  const dim3 grid(tw * th, N * C);
  switch (K) {
    case 3: hipLaunchKernelGGL(dwconv_fwd_kernel<3>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw, accumulate); break;
    case 5: hipLaunchKernelGGL(dwconv_fwd_kernel<5>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw, accumulate); break;
    case 7: hipLaunchKernelGGL(dwconv_fwd_kernel<7>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw, accumulate); break;
    case 9: hipLaunchKernelGGL(dwconv_fwd_kernel<9>, grid, dim3(256), 0, st, x, x_bs, w, bias, y, y_bs, C, H, W, flip, tw, accumulate); break;
    default: DSG_REQUIRE(false, "dsgan_dwconv_fwd: K must be 3, 5, 7 or 9");
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

// floats of partial-sum scratch dsgan_dwconv_wgrad needs (alignment as the call will see it)
long dsgan_dwconv_wgrad_workspace(int N, int C, int H, int W, int K, int aligned16) {
  const int cfg = dw_cfg(H, W);
  long G;
  if (cfg && K >= 3 && aligned16) {
    G = dw_wgrad_any(K, cfg, nullptr, 0, nullptr, 0, nullptr, N, C, H, W, 0);
  } else {
    int tpb;
    G = (long)N * dw_generic_groups(N, C, H, W, &tpb);
  }
  return G * C * (K * K + 1);
}

// dw[c] += sum dy * x (KxK correlation), db[c] += sum dy: every workgroup writes its partial
// sums to ws, dw_partial_reduce_kernel adds them in a fixed order (deterministic).
int dsgan_dwconv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, float* db,
                       int N, int C, int H, int W, int K, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && K >= 1 && K <= DW_MAXK && (K & 1), "dsgan_dwconv_wgrad: bad args");
  const int cfg = dw_cfg(H, W);
  long G;
  const bool tiled = dw_tiled_ok(K, cfg, x, dy, x_bs, dy_bs);
  int tpb = 0, groups = 0;
  if (tiled) {
    G = dw_wgrad_any(K, cfg, nullptr, 0, nullptr, 0, nullptr, N, C, H, W, st);   // (plan only)
  } else {
    groups = dw_generic_groups(N, C, H, W, &tpb);
    DSG_REQUIRE((long)N * C < (1L << 31) && groups <= 65535, "dsgan_dwconv_wgrad: grid too large");
    G = (long)N * groups;
  }
  DSG_WS(G * C * (K * K + 1), ws, ws_elems, "dsgan_dwconv_wgrad (dsgan_dwconv_wgrad_workspace)");
  if (tiled) {
    dw_wgrad_any(K, cfg, dy, dy_bs, x, x_bs, ws, N, C, H, W, st);
  } else {
    const dim3 grid(N * C, groups);
    switch (K) {
      case 3: hipLaunchKernelGGL(dwconv_wgrad_kernel<3>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, ws, C, H, W, tpb); break;
      case 5: hipLaunchKernelGGL(dwconv_wgrad_kernel<5>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, ws, C, H, W, tpb); break;
      case 7: hipLaunchKernelGGL(dwconv_wgrad_kernel<7>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, ws, C, H, W, tpb); break;
      case 9: hipLaunchKernelGGL(dwconv_wgrad_kernel<9>, grid, dim3(256), 0, st, dy, dy_bs, x, x_bs, ws, C, H, W, tpb); break;
      default: DSG_REQUIRE(false, "dsgan_dwconv_wgrad: K must be 3, 5, 7 or 9");
    }
  }
  // dw[c][i] += sum_g ws[g][c][i] (i < K*K), db[c] += sum_g ws[g][c][K*K]; g in a fixed order
  launch_split_reduce_kk(ws, (int)G, (long)C * (K * K + 1), dw, db, K * K + 1, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
