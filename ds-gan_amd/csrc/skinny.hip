// Direct convolutions for contractions with a handful of channels on one side (gfx950).
//
// A 128x128 MFMA tile wastes >95% of its work when one GEMM dimension is 1..8, and these
// layers sit at the full 256x256 resolution, so they are HBM/L2-bound streaming kernels here:
//   * small_out: outputs with M <= 8 channels -- the G head conv 64->3 (MixConvNeXtML.py:459),
//     the PatchGAN last conv 256->1 (networks.py:567), and the data-grads INTO a 3/6-channel
//     tensor (VGG16 conv1_1, vgg.py:17; PatchGAN conv 0, networks.py:543) as transposed convs.
//     Thread = output pixel, all M accumulators in registers, weights via scalar loads, the
//     input through branch-free buffer loads (zero padding = out-of-range offset).
//   * wgrad_small: weight-grads with <= 8 channels on one side -- the G head (Cout 3), the
//     first 1x1 convs from the 3-channel input (to32 / shortcut, MixConvNeXtML.py:124,145) and
//     the PatchGAN ends.  Workgroup = (big-side channel, pixel chunk); the small side x taps are
//     register accumulators, reduced once per workgroup into per-chunk partials that
//     launch_split_reduce sums in a fixed order (deterministic, no atomics).
#include "common.h"

namespace dsg {

constexpr unsigned SK_OOB = 0xFFFFFFF0u;

struct SkArgs {
  const float* x; long x_bs;        // input [nb][K][Hin][Win]
  const float* w;                   // element (m, k, kh, kw) at w[m*wm + k*wk + kh*wh + kw*ww]
  long wm, wk, wh, ww;
  const float* bias;
  float* y; long y_bs;              // output [nb][M][Ho][Wo]
  int nb, K, M, Hin, Win, Ho, Wo, KH, KW, stride, pad, transposed;
  int accumulate;
  unsigned x_range;
  int act; float slope;   // small_in only
};

__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}

// out[b][m][oh][ow] (+)= bias[m] + sum_{k,kh,kw} w(m,k,kh,kw) * in(b, k, tap)
//   conv:        in = x[b][k][oh*s - pad + kh][ow*s - pad + kw]
//   transposed:  in = x[b][k][(oh + pad - kh)/s][(ow + pad - kw)/s]  (when divisible)
// Workgroup = 64 output pixels x 4 waves; wave w sums channels k = w, w+4, ...; the four partial
// sums are combined through LDS in a fixed order (deterministic, no atomics).  The weights are
// staged once per workgroup into LDS as [k][tap][MS] (broadcast reads in the loop); KH/KW are
// template constants for the common 1x1/3x3/4x4 cases so every tap load of a channel is issued
// back to back (KH_ = 0: runtime taps).
// PAR (transposed, stride 2, KH_ x KW_ = 4x4): only the 2x2 taps whose parity matches the output
// pixel can land on an input pixel, so each lane walks its own four taps (kh = (oh+pad)&1 + 2i,
// kw = (ow+pad)&1 + 2j) instead of issuing 16 loads of which 12 are out of range.
// NWV = 16 (1024 threads, K > 64): the sixteen waves split the channels of one 64-pixel block --
// for the under-filled launches (the PatchGAN last layer: 225 blocks of 64 pixels, K = 256), 16
// channels per wave instead of 64 channel round trips in series.
template <int MS, int KH_, int KW_, bool PAR = false, int NWV = 4>
__global__ __launch_bounds__(64 * NWV) void small_out_kernel(SkArgs a) {
  extern __shared__ float wsm[];                 // [K][KH*KW][MS]
  __shared__ float part[NWV - 1][MS][64];
  const int KH = KH_ ? KH_ : a.KH, KW = KW_ ? KW_ : a.KW, T = KH * KW;
  for (int i = threadIdx.x; i < a.K * T * MS; i += 64 * NWV) {
    const int m = i % MS, kt = i / MS, k = kt / T, t = kt - k * T;
    wsm[i] = m < a.M ? a.w[m * a.wm + k * a.wk + (t / KW) * a.wh + (t % KW) * a.ww] : 0.f;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int HWo = a.Ho * a.Wo;
  const long total = (long)a.nb * HWo;
  // the staged weights serve a grid-stride run of 64-pixel blocks (staging them per block cost
  // more L2 traffic than the activations when K*T*MS is large: 16 KB per 64 pixels for the
  // PatchGAN conv-0 data-grad)
  // K <= 64: each wave owns its own 64 pixels over all K (no cross-wave combine or barrier per
  // block); larger K: the four waves split the channels of one 64-pixel block.
  const bool own = NWV == 4 && a.K <= 64;
  const int PB = own ? 256 : 64;
  for (long blk = blockIdx.x; blk * PB < total; blk += gridDim.x) {
    long q = blk * PB + (own ? wave * 64 : 0) + lane;
    const bool qv = q < total;
    if (!qv) q = 0;
    const int b = (int)(q / HWo), r = (int)(q - (long)b * HWo);
    const int oh = r / a.Wo, ow = r - (r / a.Wo) * a.Wo;
    const int HWi = a.Hin * a.Win;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
    const unsigned xb = (unsigned)((long)b * a.x_bs);

    // per-tap in-plane offsets (or OOB), independent of k
    constexpr int TMAX = PAR ? 4 : (KH_ ? KH_ * KW_ : 1);
    unsigned toff[TMAX];
    int tsel[TMAX];                               // weight tap of each slot (PAR: per lane)
    auto tap_off = [&](int kh, int kw) -> unsigned {
      int ih, iw; bool ok;
      if (!a.transposed) {
        ih = oh * a.stride - a.pad + kh; iw = ow * a.stride - a.pad + kw;
        ok = ((unsigned)ih < (unsigned)a.Hin) & ((unsigned)iw < (unsigned)a.Win);
      } else {
        const int th = oh + a.pad - kh, tw = ow + a.pad - kw;
        ih = a.stride == 1 ? th : (th >> 1); iw = a.stride == 1 ? tw : (tw >> 1);
        ok = (th >= 0) & (tw >= 0) & ((a.stride == 1) | !((th | tw) & 1)) & (ih < a.Hin) & (iw < a.Win);
      }
      return ok ? (unsigned)(ih * a.Win + iw) : 0x3FFFFFF0u;
    };
    if (PAR) {
      const int kh0 = (oh + a.pad) & 1, kw0 = (ow + a.pad) & 1;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int kh = kh0 + 2 * (t >> 1), kw = kw0 + 2 * (t & 1);
        toff[t] = tap_off(kh, kw);
        tsel[t] = kh * KW_ + kw;
      }
    } else if (KH_) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) { toff[t] = tap_off(t / KW_, t % KW_); tsel[t] = t; }
    }

    float acc[MS];
#pragma unroll
    for (int m = 0; m < MS; ++m) acc[m] = 0.f;
    for (int k = own ? 0 : wave; k < a.K; k += own ? 1 : NWV) {
      const unsigned xk = xb + (unsigned)k * HWi;
      const float* wk = wsm + k * T * MS;
      if (KH_) {
        float xv[TMAX];
#pragma unroll
        for (int t = 0; t < TMAX; ++t) xv[t] = bld(rx, toff[t] >= 0x3FFFFFF0u ? SK_OOB : (xk + toff[t]) * 4u);
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
#pragma unroll
          for (int m = 0; m < MS; ++m) acc[m] = fmaf(wk[tsel[t] * MS + m], xv[t], acc[m]);
      } else {
        for (int t = 0; t < T; ++t) {
          const unsigned o = tap_off(t / KW, t % KW);
          const float xv = bld(rx, o >= 0x3FFFFFF0u ? SK_OOB : (xk + o) * 4u);
#pragma unroll
          for (int m = 0; m < MS; ++m) acc[m] = fmaf(wk[t * MS + m], xv, acc[m]);
        }
      }
    }
    if (own) {
      if (qv) {
        float* yp = a.y + (long)b * a.y_bs + r;
#pragma unroll
        for (int m = 0; m < MS; ++m) {
          if (m >= a.M) break;
          float v = acc[m];
          if (a.bias) v += a.bias[m];
          if (a.accumulate) v += yp[(long)m * HWo];
          yp[(long)m * HWo] = v;
        }
      }
      continue;   // (uniform over the workgroup)
    }
    if (wave > 0) {
#pragma unroll
      for (int m = 0; m < MS; ++m) part[wave - 1][m][lane] = acc[m];
    }
    __syncthreads();
    if (wave == 0 && qv) {
      float* yp = a.y + (long)b * a.y_bs + r;
#pragma unroll
      for (int m = 0; m < MS; ++m) {
        if (m >= a.M) break;
        float v = acc[m];
#pragma unroll
        for (int w = 0; w < NWV - 1; ++w) v += part[w][m][lane];   // fixed order
        if (a.bias) v += a.bias[m];
        if (a.accumulate) v += yp[(long)m * HWo];
        yp[(long)m * HWo] = v;
      }
    }
    __syncthreads();   // part[] is rewritten by the next block
  }
}

// small_in: few INPUT taps (K*KH*KW <= 36) into many output channels -- VGG16 conv1_1 (3 -> 64,
// vgg.py:17) and the data-grad of the G head (3 -> 64 transposed, MixConvNeXtML.py:459).  The
// GEMM view (M = 64, K = 27) starves an MFMA tile on its im2col gather; here a thread owns PX
// consecutive output pixels of a row: their K*T inputs are loaded once into registers, then
// every output channel is an exact fp32 dot product with weights broadcast from LDS (one
// float4 read serves 4 channels x PX pixels -- the LDS return path, not the FMAs, bounds this
// kernel), written as one 16-byte store per channel (PX = 4).  blockIdx.y = 64-channel chunk.
template <int KT, int PX>
__global__ __launch_bounds__(256) void small_in_kernel(SkArgs a) {
  __shared__ __attribute__((aligned(16))) float wsm[KT][64];   // [k*T + t][m - m0]
  __shared__ __attribute__((aligned(16))) float bsm[64];
  const int T = a.KH * a.KW, KTr = a.K * T;
  const int m0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < KT * 64; i += 256) {
    const int j = i / 64, mm = i - j * 64, m = m0 + mm;
    float v = 0.f;
    if (j < KTr && m < a.M) {
      const int k = j / T, t = j - k * T;
      v = a.w[m * a.wm + k * a.wk + (t / a.KW) * a.wh + (t % a.KW) * a.ww];
    }
    wsm[j][mm] = v;
  }
  if (threadIdx.x < 64) bsm[threadIdx.x] = a.bias && m0 + (int)threadIdx.x < a.M ? a.bias[m0 + threadIdx.x] : 0.f;
  __syncthreads();
  const int HWo = a.Ho * a.Wo;
  const int total = a.nb * HWo / PX;            // PX | Wo (host check)
  int q = blockIdx.x * 256 + threadIdx.x;
  const bool qv = q < total;
  if (!qv) q = 0;
  q *= PX;
  const int b = q / HWo, r = q - b * HWo;
  const int oh = r / a.Wo, ow0 = r - oh * a.Wo;
  const int HWi = a.Hin * a.Win;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const unsigned xb = (unsigned)((long)b * a.x_bs);
  float xv[KT][PX];
#pragma unroll
  for (int j = 0; j < KT; ++j) {
#pragma unroll
    for (int p = 0; p < PX; ++p) {
      if (j < KTr) {
        const int k = j / T, t = j - k * T, kh = t / a.KW, kw = t - kh * a.KW, ow = ow0 + p;
        int ih, iw;
        if (!a.transposed) { ih = oh * a.stride - a.pad + kh; iw = ow * a.stride - a.pad + kw; }
        else { ih = oh + a.pad - kh; iw = ow + a.pad - kw; }
        const bool ok = ((unsigned)ih < (unsigned)a.Hin) & ((unsigned)iw < (unsigned)a.Win);
        xv[j][p] = bld(rx, ok ? (xb + (unsigned)k * HWi + (unsigned)(ih * a.Win + iw)) * 4u : SK_OOB);
      } else {
        xv[j][p] = 0.f;
      }
    }
  }
  if (!qv) return;
  float* yp = a.y + (long)b * a.y_bs + (long)m0 * HWo + r;
  const int mn = min(64, a.M - m0);
  for (int mm = 0; mm < mn; mm += 4) {
    float acc[4][PX];
    const float4 bv = *reinterpret_cast<const float4*>(&bsm[mm]);
#pragma unroll
    for (int p = 0; p < PX; ++p) { acc[0][p] = bv.x; acc[1][p] = bv.y; acc[2][p] = bv.z; acc[3][p] = bv.w; }
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const float4 wv = *reinterpret_cast<const float4*>(&wsm[j][mm]);
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        acc[0][p] = fmaf(wv.x, xv[j][p], acc[0][p]); acc[1][p] = fmaf(wv.y, xv[j][p], acc[1][p]);
        acc[2][p] = fmaf(wv.z, xv[j][p], acc[2][p]); acc[3][p] = fmaf(wv.w, xv[j][p], acc[3][p]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (mm + u < mn) {
        float* dst = yp + (long)(mm + u) * HWo;
        if constexpr (PX == 4) {
          float4 v = make_float4(act_f(a.act, acc[u][0], a.slope), act_f(a.act, acc[u][1], a.slope),
                                 act_f(a.act, acc[u][2], a.slope), act_f(a.act, acc[u][3], a.slope));
          if (a.accumulate) { const float4 o = *reinterpret_cast<const float4*>(dst); v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
          *reinterpret_cast<float4*>(dst) = v;
        } else {
#pragma unroll
          for (int p = 0; p < PX; ++p) {
            float v = act_f(a.act, acc[u][p], a.slope);
            if (a.accumulate) v += dst[p];
            dst[p] = v;
          }
        }
      }
    }
  }
}

// dw[co][ci][kh][kw] += sum_{b,oh,ow} dy[b][co][oh][ow] * x[b][ci][oh*s-pad+kh][ow*s-pad+kw]
// SMALL_OUT: Cout <= S (block = ci); else Cin <= S (block = co).  T = KH*KW taps.
struct WsArgs {
  const float* dy; long dy_bs;
  const float* x; long x_bs;
  float* dw;
  int nb, Cin, Hin, Win, Cout, Ho, Wo, KW, stride, pad, nsmall;
  long pix_per_block;
  unsigned x_range, dy_range;
  float* ws;   // chunk partials [gridDim.y][Cout*Cin*T] (NULL: one chunk, += into dw)
};

template <int S, int T, bool SMALL_OUT>
__global__ __launch_bounds__(256) void wgrad_small_kernel(WsArgs a) {
  __shared__ float red[4][S * T];
  const int c = blockIdx.x;                      // ci (SMALL_OUT) or co
  const int HWo = a.Ho * a.Wo, HWi = a.Hin * a.Win;
  const long total = (long)a.nb * HWo;
  const long p0 = (long)blockIdx.y * a.pix_per_block;
  const long p1 = min(total, p0 + a.pix_per_block);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_range, 0x00020000);

  float acc[S][T];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int t = 0; t < T; ++t) acc[s][t] = 0.f;

  // pixel walk without a 64-bit division per pixel (it used to cost more than the loads):
  // (b, oh, ow) of p = p0 + tid once, then advanced by 256 pixels per iteration
  int b, oh, ow;
  {
    const int q = (int)(p0 + threadIdx.x);   // nb*Ho*Wo < 2^31 (host check)
    b = q / HWo;
    const int r = q - b * HWo;
    oh = r / a.Wo;
    ow = r - oh * a.Wo;
  }
  const int dq = 256 / a.Wo, dw = 256 - dq * a.Wo;
  for (int p = (int)p0 + threadIdx.x; p < (int)p1; p += 256) {
    const int r = oh * a.Wo + ow;
    const int ih0 = oh * a.stride - a.pad, iw0 = ow * a.stride - a.pad;
    unsigned toff[T];                            // tap offsets inside one input plane (or OOB)
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int ih = ih0 + t / a.KW, iw = iw0 + t % a.KW;
      const bool ok = ((unsigned)ih < (unsigned)a.Hin) & ((unsigned)iw < (unsigned)a.Win);
      toff[t] = ok ? (unsigned)(ih * a.Win + iw) : 0x3FFFFFF0u;
    }
    const unsigned xb = (unsigned)((long)b * a.x_bs), gb = (unsigned)((long)b * a.dy_bs) + r;
    if (SMALL_OUT) {
      float g[S];
#pragma unroll
      for (int s = 0; s < S; ++s)
        g[s] = s < a.nsmall ? bld(rg, (gb + (unsigned)s * HWo) * 4u) : 0.f;
      const unsigned xc = xb + (unsigned)c * HWi;
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const float xv = bld(rx, toff[t] >= 0x3FFFFFF0u ? SK_OOB : (xc + toff[t]) * 4u);
#pragma unroll
        for (int s = 0; s < S; ++s) acc[s][t] = fmaf(g[s], xv, acc[s][t]);
      }
    } else {
      const float g = bld(rg, (gb + (unsigned)c * HWo) * 4u);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s >= a.nsmall) break;
        const unsigned xc = xb + (unsigned)s * HWi;
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const float xv = bld(rx, toff[t] >= 0x3FFFFFF0u ? SK_OOB : (xc + toff[t]) * 4u);
          acc[s][t] = fmaf(g, xv, acc[s][t]);
        }
      }
    }
    ow += dw; oh += dq;
    if (ow >= a.Wo) { ow -= a.Wo; ++oh; }
    while (oh >= a.Ho) { oh -= a.Ho; ++b; }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s >= a.nsmall) break;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const float v = warp_sum(acc[s][t]);
      if (ln == 0) red[wv][s * T + t] = v;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < a.nsmall * T; i += 256) {
    const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    const int s = i / T, t = i - s * T;
    const long o = SMALL_OUT ? ((long)s * a.Cin + c) * T + t : ((long)c * a.Cin + s) * T + t;
    if (a.ws) a.ws[(long)blockIdx.y * a.Cout * a.Cin * T + o] = v;   // this chunk's partial
    else a.dw[o] += v;                                               // one chunk: the only writer
  }
}

// 1x1 / stride 1 form of the above (the 3-channel-input 1x1 convs at 256^2: the c1 shortcut and
// pwconv1, the local branch's to32; MixConvNeXtML.py:124,145,221): a thread walks pixel QUADS with
// 16-byte loads (dy of the workgroup's channel once, the small side's <= S planes), four products
// per FMA chain step -- a quarter of the load instructions of the pixel-per-thread walk.
template <int S, bool SMALL_OUT>
__global__ __launch_bounds__(256) void wgrad_small_pw4_kernel(WsArgs a) {
  __shared__ float red[4][S];
  const int c = blockIdx.x;
  const int HW = a.Ho * a.Wo;
  const long total = (long)a.nb * HW;
  const long p0 = (long)blockIdx.y * a.pix_per_block;
  const long p1 = min(total, p0 + a.pix_per_block);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, a.x_range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.dy, (short)0, a.dy_range, 0x00020000);
  auto ld4 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  };
  float acc[S];
#pragma unroll
  for (int s = 0; s < S; ++s) acc[s] = 0.f;
  // (b, r) of this thread's first quad, then advanced by 1024 pixels per quad (HW % 4 == 0).  U quads
  // per step: all of their loads are issued before the FMAs (one memory latency per U quads instead
  // of per quad); each accumulator still takes the quads in pixel order (same sums, same bits).
  constexpr int U = S <= 4 ? 4 : 2;
  long p = p0 + 4 * threadIdx.x;
  int b = (int)(p / HW), r = (int)(p - (long)b * HW);
  for (; p < p1; p += 1024 * U) {
    float4 one[U], many[U][S];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = p + 1024 * u < p1;
      const unsigned xb = (unsigned)((long)b * a.x_bs) + r, gb = (unsigned)((long)b * a.dy_bs) + r;
      // (an out-of-range quad reads zeros through the buffer range check: offset SK_OOB)
      if (SMALL_OUT) {
        one[u] = ld4(rx, ok ? (xb + (unsigned)c * HW) * 4u : SK_OOB);
#pragma unroll
        for (int s = 0; s < S; ++s)
          many[u][s] = s < a.nsmall ? ld4(rg, ok ? (gb + (unsigned)s * HW) * 4u : SK_OOB) : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        one[u] = ld4(rg, ok ? (gb + (unsigned)c * HW) * 4u : SK_OOB);
#pragma unroll
        for (int s = 0; s < S; ++s)
          many[u][s] = s < a.nsmall ? ld4(rx, ok ? (xb + (unsigned)s * HW) * 4u : SK_OOB) : float4{0.f, 0.f, 0.f, 0.f};
      }
      r += 1024;
      while (r >= HW) { r -= HW; ++b; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (p + 1024 * u >= p1) break;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s >= a.nsmall) break;
        const float4 g = SMALL_OUT ? many[u][s] : one[u], xv = SMALL_OUT ? one[u] : many[u][s];
        acc[s] = fmaf(g.x, xv.x, fmaf(g.y, xv.y, fmaf(g.z, xv.z, fmaf(g.w, xv.w, acc[s]))));
      }
    }
  }
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (s >= a.nsmall) break;
    const float v = warp_sum(acc[s]);
    if (ln == 0) red[wv][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < a.nsmall) {
    const int s = threadIdx.x;
    const float v = red[0][s] + red[1][s] + red[2][s] + red[3][s];
    const long o = SMALL_OUT ? (long)s * a.Cin + c : (long)c * a.Cin + s;
    if (a.ws) a.ws[(long)blockIdx.y * a.Cout * a.Cin + o] = v;
    else a.dw[o] += v;
  }
}

// pixel chunks of a small weight-grad (gridDim.y): ~2048 workgroups, >= 16 pixels per thread
static long ws_chunks(int big, long total, long* ppb_out) {
  long chunks = (2048 + big - 1) / big;
  const long max_chunks = (total + 4095) / 4096;
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks < 1) chunks = 1;
  long ppb = (total + chunks - 1) / chunks;
  ppb = (ppb + 255) / 256 * 256;
  *ppb_out = ppb;
  return (total + ppb - 1) / ppb;
}

template <int S, int T, bool SO>
static void ws_launch(const WsArgs& a, int big, int chunks, hipStream_t st) {
  hipLaunchKernelGGL((wgrad_small_kernel<S, T, SO>), dim3(big, chunks), dim3(256), 0, st, a);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Small-output direct conv / transposed conv (see small_out_kernel).  Weight strides are in
// elements and may be negative (flipped kernels).  accumulate=0 overwrites y.
int dsgan_conv_small_out(const float* x, long x_bs, const float* w, long wm, long wk, long wh, long ww,
                         const float* bias, float* y, long y_bs, int nb, int K, int M, int Hin, int Win,
                         int Ho, int Wo, int KH, int KW, int stride, int pad, int transposed,
                         int accumulate, hipStream_t st) {
  DSG_REQUIRE(x && w && y && nb > 0 && K > 0 && M >= 1 && M <= 8 && Ho > 0 && Wo > 0 && KH > 0 && KW > 0,
              "dsgan_conv_small_out: bad args");
  DSG_REQUIRE(!transposed || stride == 1 || stride == 2, "dsgan_conv_small_out: transposed stride must be 1 or 2");
  const long xr = ((long)(nb - 1) * x_bs + (long)K * Hin * Win) * 4;
  DSG_REQUIRE(xr < (long)SK_OOB && (long)nb * x_bs * 4 < (long)SK_OOB, "dsgan_conv_small_out: input exceeds 4 GiB");
  SkArgs a{};
  a.x = x; a.x_bs = x_bs; a.w = w; a.wm = wm; a.wk = wk; a.wh = wh; a.ww = ww; a.bias = bias;
  a.y = y; a.y_bs = y_bs; a.nb = nb; a.K = K; a.M = M; a.Hin = Hin; a.Win = Win; a.Ho = Ho; a.Wo = Wo;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.transposed = transposed;
  a.x_range = (unsigned)xr;
  a.accumulate = accumulate;
  const long pblocks = ((long)nb * Ho * Wo + 63) / 64;
  DSG_REQUIRE(pblocks < (1L << 31), "dsgan_conv_small_out: too many pixels");
  const long wblocks = K <= 64 ? (pblocks + 3) / 4 : pblocks;       // 256-pixel blocks when K <= 64
  const dim3 grid((unsigned)(wblocks < 2048 ? wblocks : 2048));    // grid-stride over pixel blocks
  // few pixel blocks over many channels (PatchGAN last layer, 4x4 K = 256 -> 1 at 31^2): 16 waves
  const bool wide = K >= 128 && pblocks < 1024 && KH == 4 && KW == 4 && M == 1 && !transposed;
  const int MSr = M == 1 ? 1 : (M <= 4 ? 4 : 8);
  const size_t lds = (size_t)K * KH * KW * MSr * 4;
  DSG_REQUIRE(lds <= 64 * 1024, "dsgan_conv_small_out: K*KH*KW*M too large for the LDS weight stage");
#define SO_LAUNCH(MS_, KH__, KW__) hipLaunchKernelGGL((small_out_kernel<MS_, KH__, KW__>), grid, dim3(256), lds, st, a)
#define SO_SHAPES(MS_)                                                      \
  if (KH == 1 && KW == 1) SO_LAUNCH(MS_, 1, 1);                             \
  else if (KH == 3 && KW == 3) SO_LAUNCH(MS_, 3, 3);                        \
  else if (KH == 4 && KW == 4 && transposed && stride == 2)                 \
    hipLaunchKernelGGL((small_out_kernel<MS_, 4, 4, true>), grid, dim3(256), lds, st, a); \
  else if (KH == 4 && KW == 4) SO_LAUNCH(MS_, 4, 4);                        \
  else SO_LAUNCH(MS_, 0, 0);
  if (wide) hipLaunchKernelGGL((small_out_kernel<1, 4, 4, false, 16>), grid, dim3(1024), lds, st, a);
  else if (MSr == 1) { SO_SHAPES(1) } else if (MSr == 4) { SO_SHAPES(4) } else { SO_SHAPES(8) }
#undef SO_SHAPES
#undef SO_LAUNCH
  DSG_CHECK_LAUNCH();
  return 0;
}

// Few-input-tap direct conv / stride-1 transposed conv (see small_in_kernel): K*KH*KW <= 36,
// y (+)= act(bias + conv).  Weight strides in elements, as dsgan_conv_small_out.
int dsgan_conv_small_in(const float* x, long x_bs, const float* w, long wm, long wk, long wh, long ww,
                        const float* bias, float* y, long y_bs, int nb, int K, int M, int Hin, int Win,
                        int Ho, int Wo, int KH, int KW, int stride, int pad, int transposed, int act,
                        float slope, int accumulate, hipStream_t st) {
  DSG_REQUIRE(x && w && y && nb > 0 && K > 0 && M > 0 && Ho > 0 && Wo > 0 && KH > 0 && KW > 0,
              "dsgan_conv_small_in: bad args");
  DSG_REQUIRE(K * KH * KW <= 36 && (!transposed || stride == 1), "dsgan_conv_small_in: K*KH*KW <= 36, transposed stride 1");
  const long xr = ((long)(nb - 1) * x_bs + (long)K * Hin * Win) * 4;
  DSG_REQUIRE(xr < (long)SK_OOB && (long)nb * Ho * Wo < (1L << 31), "dsgan_conv_small_in: operand too large");
  SkArgs a{};
  a.x = x; a.x_bs = x_bs; a.w = w; a.wm = wm; a.wk = wk; a.wh = wh; a.ww = ww; a.bias = bias;
  a.y = y; a.y_bs = y_bs; a.nb = nb; a.K = K; a.M = M; a.Hin = Hin; a.Win = Win; a.Ho = Ho; a.Wo = Wo;
  a.KH = KH; a.KW = KW; a.stride = stride; a.pad = pad; a.transposed = transposed;
  a.x_range = (unsigned)xr; a.accumulate = accumulate; a.act = act; a.slope = slope;
  const int kt = K * KH * KW;
  const bool v4 = Wo % 4 == 0 && (y_bs & 3) == 0 && (((uintptr_t)y) & 15) == 0;
  const int px = v4 ? 4 : 1;
  const dim3 grid((unsigned)(((long)nb * Ho * Wo / px + 255) / 256), (unsigned)((M + 63) / 64));
#define SI_LAUNCH(KT_)                                                                        \
  if (v4) hipLaunchKernelGGL((small_in_kernel<KT_, 4>), grid, dim3(256), 0, st, a);          \
  else hipLaunchKernelGGL((small_in_kernel<KT_, 1>), grid, dim3(256), 0, st, a);
  if (kt <= 12) { SI_LAUNCH(12) } else if (kt <= 27) { SI_LAUNCH(27) } else { SI_LAUNCH(36) }
#undef SI_LAUNCH
  DSG_CHECK_LAUNCH();
  return 0;
}

// Weight-grad with Cout <= 8 or Cin <= 8 and KH*KW in {1, 9, 16}; dw += (OIHW).
long dsgan_conv_wgrad_small_workspace(int N, int Cin, int Cout, int KH, int KW, int Ho, int Wo) {
  long ppb;
  const long chunks = ws_chunks(Cout <= 8 ? Cin : Cout, (long)N * Ho * Wo, &ppb);
  return chunks > 1 ? chunks * Cout * Cin * KH * KW : 0;
}

int dsgan_conv_wgrad_small(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, int N,
                           int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad, int Ho,
                           int Wo, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(dy && x && dw && N > 0 && Cin > 0 && Cout > 0 && Ho > 0 && Wo > 0, "dsgan_conv_wgrad_small: bad args");
  const int T = KH * KW;
  DSG_REQUIRE(T == 1 || T == 9 || T == 16, "dsgan_conv_wgrad_small: KH*KW must be 1, 9 or 16");
  const bool so = Cout <= 8;
  DSG_REQUIRE(so || Cin <= 8, "dsgan_conv_wgrad_small: needs Cout <= 8 or Cin <= 8");
  const long xr = ((long)(N - 1) * x_bs + (long)Cin * H * W) * 4;
  const long gr = ((long)(N - 1) * dy_bs + (long)Cout * Ho * Wo) * 4;
  DSG_REQUIRE(xr < 0x3FFFFFF0L && gr < (long)SK_OOB, "dsgan_conv_wgrad_small: operand exceeds buffer range");
  DSG_REQUIRE((long)H * W < 0x3FFFFFF0L && (long)N * Ho * Wo + 256 < (1L << 31), "dsgan_conv_wgrad_small: plane too large");
  WsArgs a{};
  a.dy = dy; a.dy_bs = dy_bs; a.x = x; a.x_bs = x_bs; a.dw = dw; a.nb = N; a.Cin = Cin; a.Hin = H;
  a.Win = W; a.Cout = Cout; a.Ho = Ho; a.Wo = Wo; a.KW = KW; a.stride = stride; a.pad = pad;
  a.nsmall = so ? Cout : Cin;
  a.x_range = (unsigned)xr; a.dy_range = (unsigned)gr;
  const int big = so ? Cin : Cout;
  long ppb;
  const long chunks = ws_chunks(big, (long)N * Ho * Wo, &ppb);
  a.pix_per_block = ppb;
  DSG_REQUIRE(chunks <= 65535, "dsgan_conv_wgrad_small: grid too large");
  a.ws = chunks > 1 ? ws : nullptr;
  const bool s4 = a.nsmall <= 4;
  const bool quad = T == 1 && stride == 1 && pad == 0 && Ho == H && Wo == W && (Ho * Wo) % 4 == 0 && (x_bs & 3) == 0 &&
                    (dy_bs & 3) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0;
  // pixel-quad walk: chunks of whole 1024-pixel steps (never more chunks than the general plan)
  const long ppb4 = (ppb + 1023) / 1024 * 1024;
  const long chunks4 = ((long)N * Ho * Wo + ppb4 - 1) / ppb4;
  const long used = quad ? chunks4 : chunks;
  DSG_WS(used > 1 ? used * Cout * Cin * T : 0, ws, ws_elems, "dsgan_conv_wgrad_small (dsgan_conv_wgrad_small_workspace)");
  if (quad) {
    a.pix_per_block = ppb4;
    a.ws = chunks4 > 1 ? ws : nullptr;
    const dim3 grid((unsigned)big, (unsigned)chunks4);
    if (so) { if (s4) hipLaunchKernelGGL((wgrad_small_pw4_kernel<4, true>), grid, dim3(256), 0, st, a);
              else hipLaunchKernelGGL((wgrad_small_pw4_kernel<8, true>), grid, dim3(256), 0, st, a); }
    else { if (s4) hipLaunchKernelGGL((wgrad_small_pw4_kernel<4, false>), grid, dim3(256), 0, st, a);
           else hipLaunchKernelGGL((wgrad_small_pw4_kernel<8, false>), grid, dim3(256), 0, st, a); }
    if (chunks4 > 1) launch_split_reduce(ws, (int)chunks4, (long)Cout * Cin, dw, st);
    DSG_CHECK_LAUNCH();
    return 0;
  }
#define WS_CASE(TT)                                                                    \
  if (T == TT) {                                                                       \
    if (so) { if (s4) ws_launch<4, TT, true>(a, big, (int)chunks, st); else ws_launch<8, TT, true>(a, big, (int)chunks, st); } \
    else { if (s4) ws_launch<4, TT, false>(a, big, (int)chunks, st); else ws_launch<8, TT, false>(a, big, (int)chunks, st); } \
  }
  WS_CASE(1) else WS_CASE(9) else WS_CASE(16)
#undef WS_CASE
  if (chunks > 1) launch_split_reduce(ws, (int)chunks, (long)Cout * Cin * T, dw, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
