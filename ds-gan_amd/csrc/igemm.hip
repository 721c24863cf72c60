// Implicit-GEMM convolution on MFMA (gfx950): forward, data-grad and weight-grad.
//
// One kernel template covers every dense contraction of the DS-GAN step:
//   * the ConvNeXt pointwise MLP (nn.Linear on NHWC == 1x1 conv on NCHW,
//     DSGAN/models/model/MixConvNeXtML.py:222-224,236-238) and all 1x1 convs,
//   * 3x3 convs (VGG16 features, DSGAN/models/vgg.py:15-24; G head :459),
//   * 4x4 s2/s1 PatchGAN convs (DSGAN/models/networks.py:543-569),
//   * ConvTranspose2d 3x3 s2 (DSGAN/models/model/MixConvNeXtML.py:53,150): its forward is the
//     data-grad of a conv whose weight is the ConvT weight, its data-grad a conv forward.
//
// GEMM views (NCHW activations, OIHW weights, P = Ho*Wo, Q = H*W, KK = KH*KW):
//   FWD  : y[b,co,p]        M=Cout  N=B*P      K=Cin*KK   A=w (dense)      B=x  (im2col gather)
//   DGRAD: dx[b,ci,q]       M=Cin   N=B*Q      K=Cout*KK  A=w^T (gather)   B=dy (col2im gather)
//   WGRAD: dw[co,(ci,kk)]   M=Cout  N=Cin*KK   K=B*P      A=dy             B=x  (gather), split-K into
//          per-split partials reduced in a fixed order (pwgemm.hip launch_split_reduce): deterministic
//   DGRAD2: stride-2 data-grad split into the 4 output parity classes (ph,pw).  Pixel
//           ih = 2*ih'+ph only receives taps kh = kh0 + 2*th with kh0 = (ph+pad)&1, so each class
//           is a dense stride-1 GEMM with K = Cout*ceil((KH-kh0)/2)*ceil((KW-kw0)/2): no MFMA
//           work on the structural zeros of the strided transpose (ConvTranspose2d forward,
//           PatchGAN s2 data-grad).  One launch per class.
//
// The M dimension runs over channels and N over pixels, so an MFMA 32x32 accumulator column
// (lane & 31) walks 32 consecutive pixels of one channel plane: epilogue stores of NCHW
// outputs are 128-byte coalesced with no transpose.
//
// Precision: PREC_F32 runs exact f32 MFMA (v_mfma_f32_32x32x2_f32, fp32 parity mode);
// PREC_BF16 converts both operands to bf16 while staging to LDS and runs
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation.  HBM tensors stay fp32 in both modes.
#include "common.h"
#include <stdlib.h>

namespace dsg {

enum Mode : int { FWD = 0, DGRAD = 1, WGRAD = 2, DGRAD2 = 3 };
enum Prec : int { PREC_F32 = 0, PREC_BF16 = 1, PREC_F16 = 2 };   // PREC_F16: internal (PREC_BF16 + HALF_F16)

typedef __attribute__((ext_vector_type(16))) float f32x16;

struct GemmArgs {
  int N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo;
  const float* x;  long x_bs;   // activations (FWD, WGRAD)
  const float* dy; long dy_bs;  // output gradient (DGRAD, WGRAD)
  const float* w;               // OIHW weights (FWD, DGRAD)
  int M, NN, K;
  int k_split;                  // WGRAD: K elements per split (multiple of BK)
  float* ws;                    // WGRAD with splits > 1: partials [split][M][NN]
  // epilogue
  const float* bias;
  float* y;    long y_bs;
  float* ypre; long ypre_bs;
  const float* gpre; long gpre_bs; int gact;
  int act; float slope; int accumulate;
  int bact;                     // FWD/WGRAD: apply act code to the B operand on load (gelu(z))
  // DGRAD2 parity class
  int ph, pw, kh0, kw0, nth, ntw, Hc, Wc;
};

template <int PREC> struct PT;
template <> struct PT<PREC_F32>  { using T = float;  static constexpr int BK = 16; };
template <> struct PT<PREC_BF16> { using T = __bf16; static constexpr int BK = 32; };
template <> struct PT<PREC_F16>  { using T = _Float16; static constexpr int BK = 32; };

// ---------------------------------------------------------------------------------------
// Per-thread row state.  Each thread owns fixed (row, k-chunk) items of the A and B tiles for
// the whole K loop, so the pixel decode of a row happens once.
// ---------------------------------------------------------------------------------------
struct RowB {         // B-tile row (an output pixel for FWD/DGRAD, a (ci,kh,kw) tap for WGRAD)
  const float* base;  // per-row base pointer
  int a0, a1;         // FWD: ih0, iw0 ; DGRAD: ih+pad, iw+pad ; WGRAD: kh-pad, kw-pad
  int valid;
};

template <int MODE, bool PW>
__device__ __forceinline__ RowB make_rowB(const GemmArgs& g, int n) {
  RowB r;
  r.valid = n < g.NN;
  if (!r.valid) n = 0;
  if (MODE == FWD) {
    const int P = g.Ho * g.Wo;
    const int b = n / P, p = n - b * P;
    if (PW) { r.base = g.x + (long)b * g.x_bs + p; r.a0 = r.a1 = 0; }
    else {
      const int oh = p / g.Wo, ow = p - oh * g.Wo;
      r.base = g.x + (long)b * g.x_bs;
      r.a0 = oh * g.stride - g.pad; r.a1 = ow * g.stride - g.pad;
    }
  } else if (MODE == DGRAD) {
    const int Q = g.H * g.W;
    const int b = n / Q, q = n - b * Q;
    if (PW) { r.base = g.dy + (long)b * g.dy_bs + q; r.a0 = r.a1 = 0; }
    else {
      const int ih = q / g.W, iw = q - ih * g.W;
      r.base = g.dy + (long)b * g.dy_bs;
      r.a0 = ih + g.pad; r.a1 = iw + g.pad;
    }
  } else if (MODE == DGRAD2) {  // n = (b, ih', iw') of parity class (ph, pw)
    const int Q = g.Hc * g.Wc;
    const int b = n / Q, q = n - b * Q;
    const int ihc = q / g.Wc, iwc = q - ihc * g.Wc;
    r.base = g.dy + (long)b * g.dy_bs;
    r.a0 = ihc + ((g.ph + g.pad - g.kh0) >> 1);
    r.a1 = iwc + ((g.pw + g.pad - g.kw0) >> 1);
  } else {  // WGRAD: n = (ci, kh, kw)
    const int KK = g.KH * g.KW;
    const int ci = n / KK, kk = n - ci * KK;
    const int kh = kk / g.KW, kw = kk - kh * g.KW;
    r.base = g.x + (long)ci * g.H * g.W;
    r.a0 = kh - g.pad; r.a1 = kw - g.pad;
  }
  return r;
}

// Branch-free guarded load: always dereference an in-bounds address (offset 0 of a live row when
// the element is outside the tensor), then select.  A `ok ? p[i] : 0` expression makes hipcc
// branch around every load and drain vmcnt(0) per element, serialising the whole tile.
__device__ __forceinline__ float ldsel(const float* base, long off, bool ok) {
  const float t = base[ok ? off : 0];
  return ok ? t : 0.f;
}

// Load CH consecutive-k elements of B row `r` starting at kbeg.
template <int MODE, bool PW, int CH>
__device__ __forceinline__ void load_B(const GemmArgs& g, const RowB& r, int kbeg, float* v) {
  if (MODE == FWD) {
    const int HW = g.H * g.W;
    if (PW) {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int k = kbeg + j;
        v[j] = ldsel(r.base, (long)k * HW, r.valid && k < g.K);
      }
    } else {
      const int KK = g.KH * g.KW;
      int ci = kbeg / KK, kk = kbeg - ci * KK;
      int kh = kk / g.KW, kw = kk - kh * g.KW;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int ih = r.a0 + kh, iw = r.a1 + kw;
        const bool ok = r.valid && (kbeg + j) < g.K && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W;
        v[j] = ldsel(r.base, (long)ci * HW + ih * g.W + iw, ok);
        if (++kw == g.KW) { kw = 0; if (++kh == g.KH) { kh = 0; ++ci; } }
      }
    }
  } else if (MODE == DGRAD) {
    const int P = g.Ho * g.Wo;
    if (PW) {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int k = kbeg + j;
        v[j] = ldsel(r.base, (long)k * P, r.valid && k < g.K);
      }
    } else {
      const int KK = g.KH * g.KW;
      int co = kbeg / KK, kk = kbeg - co * KK;
      int kh = kk / g.KW, kw = kk - kh * g.KW;
      const int s = g.stride;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int th = r.a0 - kh, tw = r.a1 - kw;
        int oh = th, ow = tw;
        bool ok = r.valid && (kbeg + j) < g.K && th >= 0 && tw >= 0;
        if (s != 1) { ok = ok && (th % s == 0) && (tw % s == 0); oh = th / s; ow = tw / s; }
        ok = ok && oh < g.Ho && ow < g.Wo;
        v[j] = ldsel(r.base, (long)co * P + oh * g.Wo + ow, ok);
        if (++kw == g.KW) { kw = 0; if (++kh == g.KH) { kh = 0; ++co; } }
      }
    }
  } else if (MODE == DGRAD2) {  // k = (co, th, tw): oh = a0 - th, ow = a1 - tw
    const int P = g.Ho * g.Wo, T = g.nth * g.ntw;
    int co = kbeg / T, tt = kbeg - co * T;
    int th = tt / g.ntw, tw = tt - th * g.ntw;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int oh = r.a0 - th, ow = r.a1 - tw;
      const bool ok = r.valid && (kbeg + j) < g.K && (unsigned)oh < (unsigned)g.Ho &&
                      (unsigned)ow < (unsigned)g.Wo;
      v[j] = ldsel(r.base, (long)co * P + oh * g.Wo + ow, ok);
      if (++tw == g.ntw) { tw = 0; if (++th == g.nth) { th = 0; ++co; } }
    }
  } else {  // WGRAD, k = (b, oh, ow)
    const int P = g.Ho * g.Wo;
    int b = kbeg / P, p = kbeg - b * P;
    if (PW) {
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const bool ok = r.valid && (kbeg + j) < g.K;
        v[j] = ldsel(r.base, (long)b * g.x_bs + p, ok);
        if (++p == P) { p = 0; ++b; }
      }
    } else {
      int oh = p / g.Wo, ow = p - oh * g.Wo;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int ih = oh * g.stride + r.a0, iw = ow * g.stride + r.a1;
        const bool ok = r.valid && (kbeg + j) < g.K && (unsigned)ih < (unsigned)g.H &&
                        (unsigned)iw < (unsigned)g.W;
        v[j] = ldsel(r.base, (long)b * g.x_bs + ih * g.W + iw, ok);
        if (++ow == g.Wo) { ow = 0; if (++oh == g.Ho) { oh = 0; ++b; } }
      }
    }
  }
}

// A rows: output channel (FWD/WGRAD) or input channel (DGRAD).
template <int MODE, int CH>
__device__ __forceinline__ void load_A(const GemmArgs& g, int m, int kbeg, float* v) {
  const bool mv = m < g.M;
  if (MODE == FWD) {
    const float* base = g.w + (long)(mv ? m : 0) * g.K;
    if (mv && (g.K & 3) == 0 && kbeg + CH <= g.K && ((uintptr_t)(base + kbeg) & 15) == 0) {
#pragma unroll
      for (int j = 0; j < CH; j += 4) {
        const float4 t = *reinterpret_cast<const float4*>(base + kbeg + j);
        v[j] = t.x; v[j + 1] = t.y; v[j + 2] = t.z; v[j + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < CH; ++j) v[j] = ldsel(base, kbeg + j, mv && kbeg + j < g.K);
    }
  } else if (MODE == DGRAD) {  // A[ci][(co,kk)] = w[co][ci][kk]
    const int KK = g.KH * g.KW;
    int co = kbeg / KK, kk = kbeg - co * KK;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const bool ok = mv && (kbeg + j) < g.K;
      v[j] = ldsel(g.w, ((long)co * g.Cin + m) * KK + kk, ok);
      if (++kk == KK) { kk = 0; ++co; }
    }
  } else if (MODE == DGRAD2) {  // A[ci][(co,th,tw)] = w[co][ci][kh0+2th][kw0+2tw]
    const int T = g.nth * g.ntw;
    int co = kbeg / T, tt = kbeg - co * T;
    int th = tt / g.ntw, tw = tt - th * g.ntw;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const bool ok = mv && (kbeg + j) < g.K;
      v[j] = ldsel(g.w, (((long)co * g.Cin + m) * g.KH + g.kh0 + 2 * th) * g.KW + g.kw0 + 2 * tw, ok);
      if (++tw == g.ntw) { tw = 0; if (++th == g.nth) { th = 0; ++co; } }
    }
  } else {  // WGRAD: A[co][(b,p)] = dy[b][co][p]
    const int P = g.Ho * g.Wo;
    int b = kbeg / P, p = kbeg - b * P;
    const float* base = g.dy + (long)(mv ? m : 0) * P;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const bool ok = mv && (kbeg + j) < g.K;
      v[j] = ldsel(base, (long)b * g.dy_bs + p, ok);
      if (++p == P) { p = 0; ++b; }
    }
  }
}

template <typename T, int CH>
__device__ __forceinline__ void store_chunk(T* dst, const float* v) {
  if constexpr (sizeof(T) == 2) {
    // CH == 16 bf16 = 32 bytes -> two 16-byte LDS writes
    hx8<T> lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) { lo[j] = (T)v[j]; hi[j] = (T)v[8 + j]; }
    reinterpret_cast<hx8<T>*>(dst)[0] = lo;
    reinterpret_cast<hx8<T>*>(dst)[1] = hi;
  } else {
#pragma unroll
    for (int j = 0; j < CH; j += 4)
      *reinterpret_cast<float4*>(dst + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  }
}

// ---------------------------------------------------------------------------------------
// Kernel.  256 threads = 4 waves laid out WM x WN; each wave owns TM x TN 32x32 MFMA tiles.
// LDS double buffer, one barrier per K-step; next tile's global loads are issued before the
// MFMAs of the current one.
// ---------------------------------------------------------------------------------------
template <int MODE, int PREC, int BM, int BN, int WM, int WN, bool PW>
__global__ __launch_bounds__(256) void igemm_kernel(GemmArgs g) {
  using T = typename PT<PREC>::T;
  constexpr int BK = PT<PREC>::BK;
  constexpr int CH = BK / 2;             // elements per (row, chunk) item
  constexpr int PADK = BK + 16 / (int)sizeof(T);  // +16 bytes per row
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_ITEMS = (2 * BM + 255) / 256, B_ITEMS = (2 * BN + 255) / 256;

  __shared__ __attribute__((aligned(16))) T smem[2 * (BM + BN) * PADK];
  T* As = smem;                      // [2][BM][PADK]
  T* Bs = smem + 2 * BM * PADK;      // [2][BN][PADK]

  // wave index through readfirstlane: the compiler then knows it is uniform (SGPR), so
  // per-wave row offsets can be scalar soffsets instead of readfirstlane waterfall loops
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // 1-D grid, XCD-aware: blocks b, b+8, b+16, ... share an XCD (round-robin dispatch), so the
  // bijective remap below gives each XCD a contiguous run of tile ids; tiles are numbered with
  // the M (channel) tile fastest, so the M-tiles that read the same activation (B) columns run
  // together on one XCD and the activation streams from HBM once instead of M/BM times.
  const int mt = (g.M + BM - 1) / BM, nt = (g.NN + BN - 1) / BN;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile % mt, rest = tile / mt;
  const int n_t = rest % nt, split = rest / nt;
  const int n0 = n_t * BN, m0 = m_t * BM;

  int kbeg = 0, kend = g.K;
  if (MODE == WGRAD) { kbeg = split * g.k_split; kend = min(g.K, kbeg + g.k_split); }
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;

  // ---- item -> (row, chunk) maps (fixed over the K loop) ----
  int a_row[A_ITEMS], a_ch[A_ITEMS];
  bool a_on[A_ITEMS];
#pragma unroll
  for (int i = 0; i < A_ITEMS; ++i) {
    const int it = tid + i * 256;
    a_on[i] = it < 2 * BM;
    a_row[i] = (it >> 1) % BM; a_ch[i] = it & 1;
  }
  int b_row[B_ITEMS], b_ch[B_ITEMS];
  bool b_on[B_ITEMS];
  RowB rb[B_ITEMS];
#pragma unroll
  for (int i = 0; i < B_ITEMS; ++i) {
    const int it = tid + i * 256;
    b_on[i] = it < 2 * BN;
    if (MODE == WGRAD) { b_row[i] = (it >> 1) % BN; b_ch[i] = it & 1; }     // k-fast
    else { b_row[i] = it % BN; b_ch[i] = (it / BN) & 1; }                   // n-fast
    rb[i] = make_rowB<MODE, PW>(g, n0 + b_row[i]);
  }

  float ra[A_ITEMS][CH], rbv[B_ITEMS][CH];
  auto gload = [&](int kt) {
    const int kb = kbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i)
      if (a_on[i]) {
        const int k0 = kb + a_ch[i] * CH;
        if (k0 < kend) load_A<MODE, CH>(g, m0 + a_row[i], k0, ra[i]);
        else {
#pragma unroll
          for (int j = 0; j < CH; ++j) ra[i][j] = 0.f;
        }
        if (MODE == WGRAD) {  // zero the part of the chunk beyond this split
#pragma unroll
          for (int j = 0; j < CH; ++j) if (k0 + j >= kend) ra[i][j] = 0.f;
        }
      }
#pragma unroll
    for (int i = 0; i < B_ITEMS; ++i)
      if (b_on[i]) {
        const int k0 = kb + b_ch[i] * CH;
        if (k0 < kend) {
          load_B<MODE, PW, CH>(g, rb[i], k0, rbv[i]);
          if ((MODE == FWD || MODE == WGRAD) && g.bact) {
#pragma unroll
            for (int j = 0; j < CH; ++j) rbv[i][j] = act_f(g.bact, rbv[i][j], g.slope);
          }
        } else {
#pragma unroll
          for (int j = 0; j < CH; ++j) rbv[i][j] = 0.f;
        }
        if (MODE == WGRAD) {
#pragma unroll
          for (int j = 0; j < CH; ++j) if (k0 + j >= kend) rbv[i][j] = 0.f;
        }
      }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i)
      if (a_on[i]) store_chunk<T, CH>(As + (buf * BM + a_row[i]) * PADK + a_ch[i] * CH, ra[i]);
#pragma unroll
    for (int i = 0; i < B_ITEMS; ++i)
      if (b_on[i]) store_chunk<T, CH>(Bs + (buf * BN + b_row[i]) * PADK + b_ch[i] * CH, rbv[i]);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  sstore(0);
  __syncthreads();

  const int lr = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const T* Ab = As + buf * BM * PADK;
    const T* Bb = Bs + buf * BN * PADK;
    if constexpr (PREC != PREC_F32) {
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        hx8<T> af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const hx8<T>*>(Ab + (wm * TM * 32 + i * 32 + lr) * PADK + ks * 16 + lh * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const hx8<T>*>(Bb + (wn * TN * 32 + j * 32 + lr) * PADK + ks * 16 + lh * 8);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
    } else {
      // k permuted inside the tile: lane-half h owns k = h*8 + s (s = MFMA sub-step)
      float af[TM][8], bfr[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float4* p = reinterpret_cast<const float4*>(Ab + (wm * TM * 32 + i * 32 + lr) * PADK + lh * 8);
        const float4 u = p[0], v = p[1];
        af[i][0] = u.x; af[i][1] = u.y; af[i][2] = u.z; af[i][3] = u.w;
        af[i][4] = v.x; af[i][5] = v.y; af[i][6] = v.z; af[i][7] = v.w;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float4* p = reinterpret_cast<const float4*>(Bb + (wn * TN * 32 + j * 32 + lr) * PADK + lh * 8);
        const float4 u = p[0], v = p[1];
        bfr[j][0] = u.x; bfr[j][1] = u.y; bfr[j][2] = u.z; bfr[j][3] = u.w;
        bfr[j][4] = v.x; bfr[j][5] = v.y; bfr[j][6] = v.z; bfr[j][7] = v.w;
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  // C/D layout (32x32): col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
  if (MODE == WGRAD) {
    float* dst = g.ws ? g.ws + (long)split * g.M * g.NN : g.y;   // one split: the only writer, +=
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + lr;
      if (n >= g.NN) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < g.M) {
            float* o = dst + (long)m * g.NN + n;
            *o = g.ws ? acc[i][j][r] : *o + acc[i][j][r];
          }
        }
    }
    return;
  }
  const int Pout = (MODE == FWD) ? g.Ho * g.Wo : g.H * g.W;
  const bool has_bias = g.bias != nullptr, has_pre = g.ypre != nullptr, has_g = g.gpre != nullptr;
  const int act = g.act, gact = g.gact;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int n = n0 + wn * TN * 32 + j * 32 + lr;
    const bool nv = n < g.NN;
    if (!nv) n = 0;
    int b, p;
    if (MODE == DGRAD2) {
      const int Q = g.Hc * g.Wc;
      b = n / Q;
      const int q = n - b * Q, ihc = q / g.Wc, iwc = q - ihc * g.Wc;
      p = (2 * ihc + g.ph) * g.W + 2 * iwc + g.pw;
    } else {
      b = n / Pout; p = n - b * Pout;
    }
    float* yb = g.y + (long)b * g.y_bs + p;
    float* ypb = has_pre ? g.ypre + (long)b * g.ypre_bs + p : nullptr;
    const float* gpb = has_g ? g.gpre + (long)b * g.gpre_bs + p : nullptr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v[16];
      long off[16];
      bool ok[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        ok[r] = nv && m < g.M;
        off[r] = ok[r] ? (long)m * Pout : 0;
        v[r] = acc[i][j][r];
      }
      if (has_bias) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          v[r] += g.bias[m < g.M ? m : 0];
        }
      }
      if (has_g) {
        float gv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) gv[r] = gpb[off[r]];
        act_g_mul_arr(gact, v, gv, g.slope);
      }
      if (has_pre) {
#pragma unroll
        for (int r = 0; r < 16; ++r) if (ok[r]) ypb[off[r]] = v[r];
      }
      act_f_arr(act, v, g.slope);
      if (g.accumulate) {
        float o[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] = yb[off[r]];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] += o[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) if (ok[r]) yb[off[r]] = v[r];
    }
  }
}

// ---------------------------------------------------------------------------------------
template <int MODE, int PREC, bool PW>
static void launch_cfg(const GemmArgs& g, int splits, hipStream_t st) {
  const int M = g.M;
  if (M > 64) {
    dim3 grid(cdiv(g.NN, 128) * cdiv(M, 128) * splits);
    hipLaunchKernelGGL((igemm_kernel<MODE, PREC, 128, 128, 2, 2, PW>), grid, dim3(256), 0, st, g);
  } else if (M > 32) {
    dim3 grid(cdiv(g.NN, 128) * cdiv(M, 64) * splits);
    hipLaunchKernelGGL((igemm_kernel<MODE, PREC, 64, 128, 2, 2, PW>), grid, dim3(256), 0, st, g);
  } else {
    dim3 grid(cdiv(g.NN, 128) * cdiv(M, 32) * splits);
    hipLaunchKernelGGL((igemm_kernel<MODE, PREC, 32, 128, 1, 4, PW>), grid, dim3(256), 0, st, g);
  }
}

template <int MODE>
static void launch_mode(const GemmArgs& g, int prec, int splits, hipStream_t st) {
  const bool pw = MODE != DGRAD2 && g.KH == 1 && g.KW == 1 && g.stride == 1 && g.pad == 0;
  if (prec == PREC_BF16 && half_type() == HALF_F16) {
    if (pw) launch_cfg<MODE, PREC_F16, true>(g, splits, st);
    else launch_cfg<MODE, PREC_F16, false>(g, splits, st);
  } else if (prec == PREC_BF16) {
    if (pw) launch_cfg<MODE, PREC_BF16, true>(g, splits, st);
    else launch_cfg<MODE, PREC_BF16, false>(g, splits, st);
  } else {
    if (pw) launch_cfg<MODE, PREC_F32, true>(g, splits, st);
    else launch_cfg<MODE, PREC_F32, false>(g, splits, st);
  }
}

// K split of a weight-grad: about 640 workgroups, >= 8 K steps each, partials of at most a
// quarter of the operand bytes (see pwgemm.hip wgrad_plan).
static int igemm_wgrad_plan(int M, int NN, long K, int BK, int* k_split) {
  const int BM = M > 64 ? 128 : (M > 32 ? 64 : 32);
  const long tiles = (long)cdiv(NN, 128) * cdiv(M, BM);
  long splits = (640 + tiles - 1) / tiles;
  const long max_splits = (K + 8L * BK - 1) / (8L * BK);
  const long byte_cap = ((long)(M + NN) * K) / (4L * M * NN);
  if (splits > max_splits) splits = max_splits;
  if (splits > byte_cap) splits = byte_cap;
  if (splits < 1) splits = 1;
  if (splits > 65535) splits = 65535;
  long ks = (K + splits - 1) / splits;
  ks = (ks + BK - 1) / BK * BK;
  splits = (K + ks - 1) / ks;
  *k_split = (int)ks;
  return (int)splits;
}

}  // namespace dsg

using namespace dsg;

static GemmArgs base_args(int N, int Cin, int H, int W, int Cout, int KH, int KW, int stride,
                          int pad, int Ho, int Wo) {
  GemmArgs g{};
  g.N = N; g.Cin = Cin; g.H = H; g.W = W; g.Cout = Cout; g.KH = KH; g.KW = KW;
  g.stride = stride; g.pad = pad; g.Ho = Ho; g.Wo = Wo;
  g.slope = 0.2f;
  return g;
}

static int check_geom(int N, int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad,
                      int Ho, int Wo, int prec) {
  DSG_REQUIRE(N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 &&
                  pad >= 0 && Ho > 0 && Wo > 0,
              "igemm: bad geometry N=%d Cin=%d H=%d W=%d Cout=%d K=%dx%d s=%d p=%d Ho=%d Wo=%d", N,
              Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo);
  DSG_REQUIRE(prec == PREC_F32 || prec == PREC_BF16, "igemm: bad precision %d", prec);
  DSG_REQUIRE((long)N * Ho * Wo < (1L << 31) && (long)N * H * W < (1L << 31) &&
                  (long)Cin * KH * KW < (1L << 31),
              "igemm: problem too large for 32-bit GEMM indices");
  return 0;
}

extern "C" {

int dsgan_conv_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y,
                   long y_bs, float* ypre, long ypre_bs, int N, int Cin, int H, int W, int Cout,
                   int KH, int KW, int stride, int pad, int Ho, int Wo, int act, float slope,
                   int accumulate, int xact, int prec, hipStream_t st) {
  if (int e = check_geom(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo, prec)) return e;
  DSG_REQUIRE(x && w && y, "dsgan_conv_fwd: null pointer");
  GemmArgs g = base_args(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo);
  g.x = x; g.x_bs = x_bs; g.w = w; g.bias = bias; g.y = y; g.y_bs = y_bs;
  g.ypre = ypre; g.ypre_bs = ypre_bs; g.act = act; g.slope = slope; g.accumulate = accumulate;
  g.bact = xact;
  g.M = Cout; g.NN = N * Ho * Wo; g.K = Cin * KH * KW;
  launch_mode<FWD>(g, prec, 1, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_conv_dgrad(const float* dy, long dy_bs, const float* w, const float* bias, float* dx,
                     long dx_bs, float* ypre, long ypre_bs, const float* gpre, long gpre_bs,
                     int gact, int N, int Cin, int H, int W, int Cout, int KH, int KW, int stride,
                     int pad, int Ho, int Wo, int act, float slope, int accumulate, int prec,
                     hipStream_t st) {
  if (int e = check_geom(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo, prec)) return e;
  DSG_REQUIRE(dy && w && dx, "dsgan_conv_dgrad: null pointer");
  GemmArgs g = base_args(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo);
  g.dy = dy; g.dy_bs = dy_bs; g.w = w; g.bias = bias; g.y = dx; g.y_bs = dx_bs;
  g.ypre = ypre; g.ypre_bs = ypre_bs; g.gpre = gpre; g.gpre_bs = gpre_bs; g.gact = gact;
  g.act = act; g.slope = slope; g.accumulate = accumulate;
  g.M = Cin;
  if (stride == 2) {
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        GemmArgs c = g;
        c.ph = ph; c.pw = pw;
        c.kh0 = (ph + pad) & 1; c.kw0 = (pw + pad) & 1;
        c.nth = (KH - c.kh0 + 1) / 2; c.ntw = (KW - c.kw0 + 1) / 2;
        c.Hc = (H - ph + 1) / 2; c.Wc = (W - pw + 1) / 2;
        if (c.Hc <= 0 || c.Wc <= 0) continue;
        c.NN = N * c.Hc * c.Wc;
        c.K = Cout * c.nth * c.ntw;
        if (c.K == 0) {  // no tap reaches this class: bias/act only -- not needed on the DS-GAN path
          dsgan_set_error("dsgan_conv_dgrad: empty parity class (K=%d, stride 2)", KH);
          return -1;
        }
        launch_mode<DGRAD2>(c, prec, 1, st);
      }
  } else {
    g.NN = N * H * W; g.K = Cout * KH * KW;
    launch_mode<DGRAD>(g, prec, 1, st);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

// floats of split-K scratch dsgan_conv_wgrad needs for this shape (0: no split)
long dsgan_conv_wgrad_workspace(int N, int Cin, int Cout, int KH, int KW, int Ho, int Wo, int prec) {
  int ks;
  const int BK = prec == PREC_BF16 ? PT<PREC_BF16>::BK : PT<PREC_F32>::BK;
  const int splits = igemm_wgrad_plan(Cout, Cin * KH * KW, (long)N * Ho * Wo, BK, &ks);
  return splits > 1 ? (long)splits * Cout * Cin * KH * KW : 0;
}

// dw[Cout][Cin][KH][KW] += sum_b,p dy[b,co,p] * x[b,ci,p*stride-pad+k]   (caller zeroes dw once
// per step; concurrent uses of one weight accumulate, as autograd would).
int dsgan_conv_wgrad(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, int N,
                     int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad, int Ho,
                     int Wo, int xact, int prec, float* ws, long ws_elems, hipStream_t st) {
  if (int e = check_geom(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo, prec)) return e;
  DSG_REQUIRE(dy && x && dw, "dsgan_conv_wgrad: null pointer");
  GemmArgs g = base_args(N, Cin, H, W, Cout, KH, KW, stride, pad, Ho, Wo);
  g.dy = dy; g.dy_bs = dy_bs; g.x = x; g.x_bs = x_bs; g.y = dw;
  g.bact = xact;
  g.M = Cout; g.NN = Cin * KH * KW; g.K = N * Ho * Wo;
  const int BK = prec == PREC_BF16 ? PT<PREC_BF16>::BK : PT<PREC_F32>::BK;
  const int splits = igemm_wgrad_plan(g.M, g.NN, g.K, BK, &g.k_split);
  g.ws = splits > 1 ? ws : nullptr;
  DSG_WS(splits > 1 ? (long)splits * g.M * g.NN : 0, ws, ws_elems, "dsgan_conv_wgrad (dsgan_conv_wgrad_workspace)");
  launch_mode<WGRAD>(g, prec, splits, st);
  if (splits > 1) launch_split_reduce(ws, splits, (long)g.M * g.NN, dw, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
