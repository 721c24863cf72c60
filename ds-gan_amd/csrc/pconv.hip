// Patch-staged implicit-GEMM convolution (gfx950, bf16 MFMA): KxK, stride 1 or 2, Cin % 32 == 0.
//
// Covers the dense contractions of VGG16 (3x3 s1, forward and data-grad; DSGAN/models/vgg.py:15-24)
// and the PatchGAN 4x4 convs (s2 and s1; DSGAN/models/networks.py:543-569).
//
//   out[b][m][oh][ow] = act( bias[m] + sum_{c, kh, kw} W[tap][m][c] * in[b][c][oh*S - pad + kh][ow*S - pad + kw] )
//
// A workgroup owns BM output channels x one TH x TW block of output pixels (128 pixels) of one
// image.  The K loop walks 32-channel blocks; per block the input patch that ALL taps of the
// block need ((TH-1)*S + KH) x ((TW-1)*S + KW) pixels) is staged once into LDS as bf16,
// pixel-major with the 32 channels contiguous, so the B fragment of any tap is one 16-byte LDS
// read at a shifted pixel -- the input is read from L2 ~1.4x instead of KH*KW times (tconv.hip).
// Per tap the bf16 weight slice [BM][32] is register-prefetched one tap ahead into a double
// buffer.  Weights are a bf16 tap-major copy (dsgan_conv_wtrans_bf16).
#include "common.h"
#include "lds_pitch.h"
#include <type_traits>
#include <stdlib.h>

namespace dsg {

typedef f32x16_t cf32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int cu32x4;

struct PcArgs {
  const float* X; long x_bs;          // [nb][K][H][W]
  const unsigned short* Wb;           // [taps][M][K] 16-bit (the half type; moved as raw bits)
  float* Y; long y_bs;                // [nb][M][Hdst][Wdst]
  const float* bias;
  const float* gpre; long gpre_bs;    // dst-shaped act' multiplier (data-grad of the producer's act)
  int nb, K, M, H, W, Ho, Wo, pad;
  int tiles_w, tiles_h;
  int act, gact; float slope;
  int accumulate;
  float* ws; int kchunk;              // split-K (ws != NULL): raw partials [split][nb][M][Ho*Wo], kchunk 32-channel blocks each
};

constexpr int PC_STR = 40;   // bf16 per staged pixel / weight row (32 + 8: conflict-free b128 reads)

template <typename T16, int BM, int TH, int TW, int S, int KH, int KW>
__global__ __launch_bounds__(256, 2) void pconv_kernel(PcArgs g) {
  typedef hx8<T16> cbf16x8;
  constexpr int BN = TH * TW;
  static_assert(BN == 128, "128 output pixels per tile");
  constexpr int WM = 2, WN = 2, TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int PH = (TH - 1) * S + KH, PW = (TW - 1) * S + KW, PPIX = PH * PW;
  // LDS pitch of a patch row, in pixels: 32 for stride 1 puts the two grid rows a B read spans
  // 32 pixels (= 0 mod 16 slots of 80 B) apart -> conflict-free ds_read_b128 (it was 2-way with
  // the patch rows packed at PW; tools/lds_banks.py).  Stride 2 keeps PW (2-way either way).
  constexpr int PWP = S == 1 ? 32 : PW;
  static_assert(PWP >= PW, "patch pitch");
  constexpr int TAPS = KH * KW;
  constexpr int A_SZ = BM * PC_STR, P_SZ = PH * PWP * PC_STR;
  constexpr int A_ITEMS = BM * 4 / 256;           // 16-byte items of a [BM][32] bf16 slice
  constexpr int P_ITEMS = (PPIX * 4 + 255) / 256; // (pixel, 8-channel group) items of the patch per thread
  __shared__ __attribute__((aligned(16))) T16 smem[2 * A_SZ + P_SZ];
  T16* Ps = smem + 2 * A_SZ;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // tile decode: M tile fastest (the tiles of one pixel block share its patch in L2)
  const int mt = (g.M + BM - 1) / BM;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile % mt, rest0 = tile / mt;
  const int tpi = g.tiles_w * g.tiles_h;
  const int split = rest0 / (g.nb * tpi), rest = rest0 - split * (g.nb * tpi);
  const int bimg = rest / tpi, t_i = rest - bimg * tpi;
  const int m0 = m_t * BM;
  const int oh0 = (t_i / g.tiles_w) * TH, ow0 = (t_i % g.tiles_w) * TW;
  const int ih0 = oh0 * S - g.pad, iw0 = ow0 * S - g.pad;   // patch origin in the input
  const int HW = g.H * g.W;
  const float* xb = g.X + (long)bimg * g.x_bs;

  // B fragment base (patch pixel of this lane's output column, tap (0,0)) per n-tile
  int pbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = wn * (BN / WN) + j * 32 + lr;
    pbase[j] = ((n / TW) * S * PWP + (n % TW) * S) * PC_STR + lh * 8;
  }

  cu32x4 ra[A_ITEMS];
  auto aload = [&](int tap, int k0) {
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256, row = p80_row16(it), c8 = p80_slot16(it);
      const int m = m0 + row;
      ra[i] = m < g.M ? *reinterpret_cast<const cu32x4*>(g.Wb + ((long)tap * g.M + m) * g.K + k0 + c8 * 8)
                      : cu32x4{0u, 0u, 0u, 0u};
    }
  };
  auto astore = [&](int buf) {
    T16* As = smem + buf * A_SZ;
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256;
      *reinterpret_cast<cu32x4*>(As + p80_row16(it) * PC_STR + p80_slot16(it) * 8) = ra[i];
    }
  };
  // patch of channel block k0: item = (pixel, 8-channel group); lanes run along the pixels of
  // a patch row, so each of the 8 channel loads is coalesced across the wave.  The loads of
  // block k0+32 are issued before the taps of block k0 run (registers), written to LDS after.
  float rp[P_ITEMS][8];
  auto pload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < P_ITEMS; ++i) {
      const int it = tid + i * 256;
      const int cg = it / PPIX, pix = it - cg * PPIX;
      const int pr = pix / PW, pc = pix - pr * PW;
      const int ih = ih0 + pr, iw = iw0 + pc;
      const bool in = it < PPIX * 4 && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      const float* src = xb + (long)(k0 + (in ? cg : 0) * 8) * HW + (in ? ih * g.W + iw : 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) rp[i][e] = in ? src[(long)e * HW] : 0.f;
    }
  };
  auto pwrite = [&]() {
#pragma unroll
    for (int i = 0; i < P_ITEMS; ++i) {
      const int it = tid + i * 256;
      if (it < PPIX * 4) {
        const int cg = it / PPIX, pix = it - cg * PPIX;
        const int pr = pix / PW, pc = pix - pr * PW;
        cbf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (T16)rp[i][e];
        *reinterpret_cast<cbf16x8*>(Ps + (pr * PWP + pc) * PC_STR + cg * 8) = v;
      }
    }
  };

  cf32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      bv[r] = (g.bias && !g.ws && m < g.M) ? g.bias[m] : 0.f;   // split-K: the finishing pass adds it
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = bv[r];
  }

  const int kb0 = g.ws ? split * g.kchunk : 0;
  const int nkb = g.ws ? min(g.K / 32, kb0 + g.kchunk) : g.K / 32;   // this split's channel blocks [kb0, nkb)
  int buf = 0;
  aload(0, kb0 * 32);
  pload(kb0 * 32);
  for (int kb = kb0; kb < nkb; ++kb) {
    const int k0 = kb * 32;
    __syncthreads();                 // previous block's patch and A buffers are free
    pwrite();
    astore(buf);
    __syncthreads();
    if (kb + 1 < nkb) pload(k0 + 32);
#pragma unroll 1
    for (int tap = 0; tap < TAPS; ++tap) {
      if (tap + 1 < TAPS) aload(tap + 1, k0);
      else if (kb + 1 < nkb) aload(0, k0 + 32);
      const T16* As = smem + buf * A_SZ;
      const int kh = tap / KW, kw = tap - (tap / KW) * KW;
      const int toff = (kh * PWP + kw) * PC_STR;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        cbf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const cbf16x8*>(As + (wm * TM * 32 + i * 32 + lr) * PC_STR + ks * 16 + lh * 8);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const cbf16x8*>(Ps + pbase[j] + toff + ks * 16);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
      if (tap + 1 < TAPS) {
        astore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
  }

  // ---- epilogue ----
  const int HWo = g.Ho * g.Wo;
  if (g.ws) {   // split-K partial: raw sums, lanes along the pixels
    float* wp = g.ws + ((long)split * g.nb + bimg) * g.M * HWo;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wn * (BN / WN) + j * 32 + lr;
      const int oh = oh0 + n / TW, ow = ow0 + n % TW;
      if (oh >= g.Ho || ow >= g.Wo) continue;
      const long pofs = (long)oh * g.Wo + ow;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < g.M) wp[(long)m * HWo + pofs] = acc[i][j][r];
        }
    }
    return;
  }
  float* yb = g.Y + (long)bimg * g.y_bs;
  const float* gb = g.gpre ? g.gpre + (long)bimg * g.gpre_bs : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = wn * (BN / WN) + j * 32 + lr;
    const int oh = oh0 + n / TW, ow = ow0 + n % TW;
    const bool nv = oh < g.Ho && ow < g.Wo;
    const long pofs = (long)oh * g.Wo + ow;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r];
      if (gb) {
        float gv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          gv[r] = (nv && m < g.M) ? gb[(long)m * HWo + pofs] : 0.f;
        }
        act_g_mul_arr(g.gact, v, gv, g.slope);
      }
      act_f_arr(g.act, v, g.slope);
      if (nv) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < g.M) {
            float* o = yb + (long)m * HWo + pofs;
            *o = g.accumulate ? *o + v[r] : v[r];
          }
        }
      }
    }
  }
}

// Split-K finish: y (+)= act( sum_s ws[s] + bias ) (* gact'(gpre)), splits in a fixed order.
__global__ __launch_bounds__(256) void pconv_reduce_kernel(PcArgs g, int S) {
  const int HWo = g.Ho * g.Wo;
  const long per = (long)g.nb * g.M * HWo;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < per; e += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += g.ws[(long)s * per + e];
    const int p = (int)(e % HWo);
    const long bm = e / HWo;
    const int m = (int)(bm % g.M), b = (int)(bm / g.M);
    if (g.bias) v += g.bias[m];
    if (g.gpre) v *= act_g(g.gact, g.gpre[(long)b * g.gpre_bs + (long)m * HWo + p], g.slope);
    v = act_f(g.act, v, g.slope);
    float* o = g.Y + (long)b * g.y_bs + (long)m * HWo + p;
    *o = g.accumulate ? *o + v : v;
  }
}

// K split of a launch whose tiles under-fill the chip (the PatchGAN stride-1 data-grad at 31^2:
// 128 tiles of 8 channel blocks): about 1024 workgroups, >= 2 channel blocks each, only for
// K >= 256 (tools/pconv_micro.py, B=16: K=256 70 -> 44 us; K=128 split in two measured 44 -> 49 us).
static int pc_splits(long tiles, int nkb, int* kchunk) {
  long S = (1024 + tiles - 1) / tiles;
  if (S > nkb / 2) S = nkb / 2;
  if (tiles >= 512 || nkb < 8 || S < 2) { *kchunk = nkb; return 1; }
  const int kc = (int)((nkb + S - 1) / S);
  *kchunk = kc;
  return (nkb + kc - 1) / kc;
}

// bf16 tap-major weights (same modes as dsgan_conv_wtrans):
//   mode 0 (forward):      Wb[tap][co][ci], tap = (kh, kw)
//   mode 1 (data-grad s1): Wb[tap][ci][co], tap = (kh', kw') with kh = KH-1-kh', kw = KW-1-kw'
//   mode 2 (stride-2 data-grad / ConvTranspose, pconvt.hip): Wb[tap][ci][co], tap = (kh, kw)
template <typename T16>
__global__ void wtrans_bf16_kernel(const float* __restrict__ W, T16* __restrict__ Wb, int Co, int Ci, int KH,
                                   int KW, int mode) {
  const int M = mode == 0 ? Co : Ci, K = mode == 0 ? Ci : Co;
  const long total = (long)KH * KW * M * K;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int k = e % K;
    const long t = e / K;
    const int m = t % M, tap = t / M;
    int kh = tap / KW, kw = tap % KW, co = m, ci = k;
    if (mode == 1) { kh = KH - 1 - kh; kw = KW - 1 - kw; co = k; ci = m; }
    if (mode == 2) { co = k; ci = m; }
    Wb[e] = (T16)W[(((long)co * Ci + ci) * KH + kh) * KW + kw];
  }
}

// Batched refresh of the 16-bit weight copies after an optimizer step (dsgan_wtrans_multi): entry
// blockIdx.y, grid-stride over its elements; mode -1 is a plain fp32 -> 16-bit cast of the
// parameter (bf16_weight), modes 0-2 the tap-major transforms of wtrans_bf16_kernel.
struct WtEnt { const float* W; void* Wb; long total; int Co, Ci, KH, KW, mode; };
constexpr int WT_MAXE = 48;
struct WtList { WtEnt e[WT_MAXE]; };

template <typename T16>
__global__ __launch_bounds__(256) void wtrans_multi_kernel(WtList L) {
  const WtEnt en = L.e[blockIdx.y];
  T16* __restrict__ Wb = (T16*)en.Wb;
  const float* __restrict__ W = en.W;
  const long stride = (long)gridDim.x * 256;
  if (en.mode < 0) {
    for (long e = blockIdx.x * 256L + threadIdx.x; e < en.total; e += stride) Wb[e] = (T16)W[e];
    return;
  }
  // thread = one (m, k) pair, all taps: it reads the KH*KW contiguous source floats of (co, ci) and
  // writes one element per tap plane -- adjacent lanes take adjacent k, so every tap's writes are
  // coalesced and each lane's reads share one or two cache lines (per-element threads read one
  // float per line)
  const int Co = en.Co, Ci = en.Ci, KH = en.KH, KW = en.KW, mode = en.mode;
  const int M = mode == 0 ? Co : Ci, K = mode == 0 ? Ci : Co, T = KH * KW;
  const long pairs = (long)M * K, plane = pairs;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < pairs; e += stride) {
    const int k = (int)(e % K), m = (int)(e / K);
    const int co = mode == 0 ? m : k, ci = mode == 0 ? k : m;
    const float* src = W + ((long)co * Ci + ci) * T;
    for (int tap = 0; tap < T; ++tap) {
      int kh = tap / KW, kw = tap - (tap / KW) * KW;
      if (mode == 1) { kh = KH - 1 - kh; kw = KW - 1 - kw; }
      Wb[(long)tap * plane + e] = (T16)src[kh * KW + kw];
    }
  }
}

// pixel tile of every pconv form
constexpr int PC_TH = 8, PC_TW = 16;
static long pc_tiles(int nb, int M, int Ho, int Wo, int BM) {
  return (long)nb * ((Wo + PC_TW - 1) / PC_TW) * ((Ho + PC_TH - 1) / PC_TH) * ((M + BM - 1) / BM);
}

// (the split plan -- g.ws / g.kchunk, `splits` -- comes from the entry point, which checked its scratch)
template <typename T16, int BM, int TH, int TW, int S, int KH, int KW>
static void pc_launch(PcArgs& g, int splits, hipStream_t st) {
  static_assert(TH == PC_TH && TW == PC_TW, "pc_tiles");
  g.tiles_w = (g.Wo + TW - 1) / TW;
  g.tiles_h = (g.Ho + TH - 1) / TH;
  const long tiles = pc_tiles(g.nb, g.M, g.Ho, g.Wo, BM);
  hipLaunchKernelGGL((pconv_kernel<T16, BM, TH, TW, S, KH, KW>), dim3((unsigned)(tiles * splits)), dim3(256), 0, st, g);
  if (splits > 1) {
    const long per = (long)g.nb * g.M * g.Ho * g.Wo;
    long blocks = (per + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(pconv_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g, splits);
  }
}

template <typename T16, int BM>
static int pc_dispatch(PcArgs& g, int KH, int S, int splits, hipStream_t st) {
  if constexpr (BM <= 128) {   // BM = 256 only for stride 2 (its stride-1 forms spill registers)
    if (KH == 3 && S == 1) { pc_launch<T16, BM, PC_TH, PC_TW, 1, 3, 3>(g, splits, st); return 0; }
    if (KH == 4 && S == 1) { pc_launch<T16, BM, PC_TH, PC_TW, 1, 4, 4>(g, splits, st); return 0; }
  }
  if (KH == 4 && S == 2) { pc_launch<T16, BM, PC_TH, PC_TW, 2, 4, 4>(g, splits, st); return 0; }
  return -1;
}

}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_pconv_supported(int K, int KH, int KW, int stride) {
  if (K % 32 != 0 || K <= 0 || KH != KW) return 0;
  return (KH == 3 && stride == 1) || (KH == 4 && (stride == 1 || stride == 2));
}

int dsgan_conv_wtrans_bf16(const float* W, void* Wb, int Co, int Ci, int KH, int KW, int mode, hipStream_t st) {
  DSG_REQUIRE(W && Wb && mode >= 0 && mode <= 2, "dsgan_conv_wtrans_bf16: bad args");
  const long total = (long)KH * KW * Co * Ci;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((wtrans_bf16_kernel<T16>), dim3((unsigned)blocks), dim3(256), 0, st, W, (T16*)Wb, Co, Ci, KH, KW,
                       mode);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// n weight copies in as few launches as possible: W[i] (fp32 [Co][Ci][KH][KW]) -> Wb[i] (16-bit), desc[5i..5i+4]
// = (Co, Ci, KH, KW, mode), mode 0-2 as dsgan_conv_wtrans_bf16, -1 a plain cast of the Co*Ci*KH*KW elements.
int dsgan_wtrans_multi(const void* const* W, void* const* Wb, const int* desc, int n, hipStream_t st) {
  DSG_REQUIRE(W && Wb && desc && n >= 0, "dsgan_wtrans_multi: bad args");
  for (int i0 = 0; i0 < n; i0 += WT_MAXE) {
    WtList L{};
    const int ne = n - i0 < WT_MAXE ? n - i0 : WT_MAXE;
    long most = 1;
    for (int i = 0; i < ne; ++i) {
      const int* d = desc + 5 * (i0 + i);
      DSG_REQUIRE(W[i0 + i] && Wb[i0 + i] && d[0] > 0 && d[1] > 0 && d[2] > 0 && d[3] > 0 && d[4] >= -1 && d[4] <= 2,
                  "dsgan_wtrans_multi: bad entry %d", i0 + i);
      WtEnt& e = L.e[i];
      e.W = (const float*)W[i0 + i]; e.Wb = Wb[i0 + i];
      e.Co = d[0]; e.Ci = d[1]; e.KH = d[2]; e.KW = d[3]; e.mode = d[4];
      e.total = (long)d[0] * d[1] * d[2] * d[3];
      if (e.total > most) most = e.total;
    }
    long bx = (most + 256L * 8 - 1) / (256L * 8);   // ~8 elements (casts) / tap rows per thread at most
    if (bx > 1024) bx = 1024;
    with_half([&](auto* t_) {
      using T16 = std::remove_pointer_t<decltype(t_)>;
      hipLaunchKernelGGL((wtrans_multi_kernel<T16>), dim3((unsigned)bx, (unsigned)ne), dim3(256), 0, st, L);
    });
    DSG_CHECK_LAUNCH();
  }
  return 0;
}

// BM = 256 for the wide layers (VGG conv3/conv4, 256/512 output channels): per tap twice the
// MFMAs between barriers and half the patch traffic per MAC, only while the launch still has >= 2
// workgroups per CU (at 32x32 it would have one); stride-1 launches take 128 instead (same
// tile count >= 512, so neither form is K-split and dsgan_pconv_workspace needs no stride)
static int pc_bm(int nb, int M, int Ho, int Wo) {
  const long ptiles = (long)nb * ((Ho + 7) / 8) * ((Wo + 15) / 16);
  return M >= 256 && ptiles * ((M + 255) / 256) >= 512 ? 256 : M > 64 ? 128 : 64;
}

// fp32 scratch dsgan_pconv_ws needs (0: the launch is not split)
// (an upper bound over the strides: a stride-1 launch runs the 256-row choice on 128-row tiles)
long dsgan_pconv_workspace(int nb, int K, int M, int Ho, int Wo) {
  if (K % 32 != 0 || K <= 0) return 0;
  const int bm = pc_bm(nb, M, Ho, Wo);
  int kc;
  const int S = max(pc_splits(pc_tiles(nb, M, Ho, Wo, bm), K / 32, &kc),
                    pc_splits(pc_tiles(nb, M, Ho, Wo, bm == 256 ? 128 : bm), K / 32, &kc));
  return S > 1 ? (long)S * nb * M * Ho * Wo : 0;
}

int dsgan_pconv_ws(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int act, int gact, float slope, int accumulate,
                   float* ws, long ws_elems, hipStream_t st);

// y[b][m][oh][ow] (+)= act(bias[m] + sum W * x) (* gact'(gpre)); Wb from dsgan_conv_wtrans_bf16.
int dsgan_pconv(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                const float* gpre, long gpre_bs, int nb, int K, int M, int H, int W, int Ho, int Wo,
                int KH, int KW, int stride, int pad, int act, int gact, float slope, int accumulate,
                hipStream_t st) {
  return dsgan_pconv_ws(X, x_bs, Wb, bias, Y, y_bs, gpre, gpre_bs, nb, K, M, H, W, Ho, Wo, KH, KW, stride, pad, act,
                        gact, slope, accumulate, nullptr, 0, st);
}

// Same, with the split-K scratch of dsgan_pconv_workspace (NULL: never split).
int dsgan_pconv_ws(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int H, int W, int Ho, int Wo,
                   int KH, int KW, int stride, int pad, int act, int gact, float slope, int accumulate,
                   float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(X && Wb && Y && nb > 0 && M > 0 && Ho > 0 && Wo > 0, "dsgan_pconv: bad args");
  DSG_REQUIRE(dsgan_pconv_supported(K, KH, KW, stride), "dsgan_pconv: unsupported K=%d KH=%d KW=%d stride=%d", K, KH, KW, stride);
  DSG_REQUIRE(((uintptr_t)Wb & 15) == 0, "dsgan_pconv: Wb must be 16-byte aligned");
  DSG_REQUIRE((Ho - 1) * stride - pad + KH <= H + pad && (Wo - 1) * stride - pad + KW <= W + pad,
              "dsgan_pconv: output size inconsistent with input/pad");
  PcArgs g{};
  g.X = X; g.x_bs = x_bs; g.Wb = (const unsigned short*)Wb; g.Y = Y; g.y_bs = y_bs; g.bias = bias;
  g.gpre = gpre; g.gpre_bs = gpre_bs; g.nb = nb; g.K = K; g.M = M; g.H = H; g.W = W; g.Ho = Ho;
  g.Wo = Wo; g.pad = pad; g.act = act; g.gact = gact; g.slope = slope; g.accumulate = accumulate;
  // tile rows: 256 only at stride 2 (the stride-1 forms spill), where the planner asks for 256
  const int bm0 = pc_bm(nb, M, Ho, Wo);
  const int bm = bm0 == 256 ? (stride == 2 ? 256 : 128) : bm0;
  int kc = 0;
  const int splits = ws ? pc_splits(pc_tiles(nb, M, Ho, Wo, bm), K / 32, &kc) : 1;
  g.ws = splits > 1 ? ws : nullptr;
  g.kchunk = kc;
  DSG_WS(splits > 1 ? (long)splits * nb * M * Ho * Wo : 0, ws, ws_elems, "dsgan_pconv (dsgan_pconv_workspace)");
  const int rc = with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    return bm == 256 ? pc_dispatch<T16, 256>(g, KH, stride, splits, st)
           : bm == 128 ? pc_dispatch<T16, 128>(g, KH, stride, splits, st)
                       : pc_dispatch<T16, 64>(g, KH, stride, splits, st);
  });
  DSG_REQUIRE(rc == 0, "dsgan_pconv: no kernel for KH=%d stride=%d", KH, stride);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
