// Patch-staged stride-2 transposed convolution, all four output parities in one workgroup
// (gfx950, bf16 MFMA, fp32 accumulate).
//
//   y[b][m][2i+ph][2j+pw] = bias[m] + sum_{c} sum_{kh = ph+pad (mod 2), kw = pw+pad (mod 2)}
//                           Wb[kh][kw][m][c] * x[b][c][i + (ph+pad-kh)/2][j + (pw+pad-kw)/2]
//
// This is ConvTranspose2d(k3, s2, p1, op1) forward (MixConvNeXtML.py:53,149-152) and the
// data-grad of a Conv2d(k4, s2, p1) (PatchGAN, DSGAN/models/networks.py:545-563).  The tap-major
// implicit GEMM (tconv.hip) runs the four parities as four launches that each re-read the input;
// here a workgroup stages the input patch of its TH x TW grid tile ONCE per 32-channel block
// (bf16, pixel-major, 32 channels contiguous as in pconv.hip) together with the bf16 weights of
// every tap, and accumulates the four parity outputs side by side:
//   * B fragments are the patch read at the few distinct (dh, dw) shifts, shared by the taps of
//     all parities that use that shift;
//   * the epilogue writes the two column parities of an output row as one float2 per lane
//     (adjacent lanes = adjacent grid columns: fully coalesced).
#include "common.h"
#include "lds_pitch.h"
#include <type_traits>
#include <stdlib.h>

namespace dsg {

typedef f32x16_t tf32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int tu32x4;

struct PtArgs {
  const float* X; long x_bs;          // [nb][K][Hi][Wi]   (grid = input)
  const unsigned short* Wb;                   // [KS*KS][M][K] bf16, tap = kh*KS + kw (unflipped)
  float* Y; long y_bs;                // [nb][M][Ho][Wo], Ho <= 2*Hi, Wo <= 2*Wi
  const float* bias;
  const float* gpre; long gpre_bs;    // Y-shaped act' multiplier
  int nb, K, M, Hi, Wi, Ho, Wo, pad;
  int tiles_w, tiles_h;
  int gact; float slope;
  int accumulate;
};

constexpr int PT_STR = 40;            // bf16 per staged pixel / weight row (32 + 8)
constexpr long PT_WGS = 512;          // resident workgroups: 2 per CU x 256 CUs

template <int KS, int PAD>
struct PtGeo {
  // row shift of tap kh for output parity ph (valid when kh = ph + PAD mod 2): (ph + PAD - kh) / 2
  static constexpr int ext(bool want_max) {
    int r = want_max ? -99 : 99;
    for (int ph = 0; ph < 2; ++ph)
      for (int kh = 0; kh < KS; ++kh)
        if (((kh + ph + PAD) & 1) == 0) {
          const int d = (ph + PAD - kh) / 2;
          r = want_max ? (d > r ? d : r) : (d < r ? d : r);
        }
    return r;
  }
  static constexpr int dmin = ext(false), dmax = ext(true);
  static constexpr int NSH = dmax - dmin + 1;
};
static_assert(PtGeo<3, 1>::dmin == 0 && PtGeo<3, 1>::dmax == 1, "ConvT 3x3 shifts");
static_assert(PtGeo<4, 1>::dmin == -1 && PtGeo<4, 1>::dmax == 1, "4x4 s2 data-grad shifts");

template <typename T16, int BM, int KS, bool PERSIST>
__global__ __launch_bounds__(256, BM == 32 ? 4 : 2) void pconvt_kernel(PtArgs g) {
  typedef hx8<T16> tbf16x8;
  constexpr int PAD = 1;
  constexpr int TH = 8, TW = 16, BN = TH * TW;
  constexpr int T = KS * KS;
  using G = PtGeo<KS, PAD>;
  constexpr int DMIN = G::dmin, NSH = G::NSH;
  constexpr int PH = TH + NSH - 1, PW = TW + NSH - 1, PPIX = PH * PW;
  // LDS pitch of a patch row in pixels: 32 puts the two grid rows of a B read 32 pixels (0 mod 16
  // slots of 80 B) apart -> conflict-free ds_read_b128 (2-way at the packed pitch PW)
  constexpr int PWP = 32;
  static_assert(PWP >= PW, "patch pitch");
  constexpr int WMW = BM / 32, WNW = 4 / WMW, NT = (BN / 32) / WNW;
  constexpr int A_SZ = BM * PT_STR;
  constexpr int A_ITEMS = T * BM * 4;             // 16-byte items of all taps' [BM][32] slices
  static_assert(BM % 8 == 0, "lds_pitch.h maps pair rows r, r + 4 within 8-row blocks");
  constexpr int A_IT = (A_ITEMS + 255) / 256;
  constexpr int P_ITEMS = PPIX * 4;                // (pixel, 8-channel group)
  constexpr int P_IT = (P_ITEMS + 255) / 256;
  __shared__ __attribute__((aligned(16))) T16 smem[T * A_SZ + PH * PWP * PT_STR];
  T16* Ps = smem + T * A_SZ;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WMW, wn = wave / WMW;
  const int lr = lane & 31, lh = lane >> 5;

  const int mt = (g.M + BM - 1) / BM;
  const int tpi = g.tiles_w * g.tiles_h;
  const int ntiles = g.nb * tpi * mt;
  const int HWi = g.Hi * g.Wi;
  // persistent: this workgroup runs tiles rank, rank + nwg, ... (rank XCD-aware: consecutive
  // ranks share an XCD, so the M tiles of one pixel tile share its patch in L2).  The first K
  // block of the next tile is fetched while the current tile's epilogue stores drain.
  const int nwg = gridDim.x;
  int rank;
  {
    const int id = blockIdx.x, xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    rank = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  struct Tc { int m0, i0, j0, b; };
  auto coords = [&](int tile) __attribute__((always_inline)) {
    const int m_t = tile % mt, rest = tile / mt;
    const int b = rest / tpi, t_i = rest - b * tpi;
    return Tc{m_t * BM, (t_i / g.tiles_w) * TH, (t_i % g.tiles_w) * TW, b};
  };

  // B fragment base per n-tile (patch pixel of this lane's grid pixel at shift (DMIN, DMIN))
  int pbase[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = (wn * NT + j) * 32 + lr;
    pbase[j] = ((n / TW) * PWP + (n % TW)) * PT_STR + lh * 8;
  }

  // global -> registers for K block kb of tile t (issued one block ahead of its use), -> LDS
  tu32x4 ra[A_IT];
  float rp[P_IT][8];
  auto load = [&](const Tc& t, int kb) __attribute__((always_inline)) {
    const int k0 = kb * 32;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256;
      const int r = p80_row16(it), c8 = p80_slot16(it), row = r % BM, tap = r / BM;
      const int m = t.m0 + row;
      ra[i] = (it < A_ITEMS && m < g.M)
                  ? *reinterpret_cast<const tu32x4*>(g.Wb + ((long)tap * g.M + m) * g.K + k0 + c8 * 8)
                  : tu32x4{0u, 0u, 0u, 0u};
    }
    const float* xb = g.X + (long)t.b * g.x_bs;
#pragma unroll
    for (int i = 0; i < P_IT; ++i) {
      const int it = tid + i * 256;
      const int cg = it / PPIX, pix = it - cg * PPIX;
      const int pr = pix / PW, pc = pix - pr * PW;
      const int ih = t.i0 + DMIN + pr, iw = t.j0 + DMIN + pc;
      const bool in = it < P_ITEMS && (unsigned)ih < (unsigned)g.Hi && (unsigned)iw < (unsigned)g.Wi;
      const float* src = xb + (long)(k0 + (in ? cg : 0) * 8) * HWi + (in ? ih * g.Wi + iw : 0);
#pragma unroll
      for (int e = 0; e < 8; ++e) rp[i][e] = in ? src[(long)e * HWi] : 0.f;
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256;
      if (it < A_ITEMS) {
        const int r = p80_row16(it), c8 = p80_slot16(it), row = r % BM, tap = r / BM;
        *reinterpret_cast<tu32x4*>(smem + tap * A_SZ + row * PT_STR + c8 * 8) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < P_IT; ++i) {
      const int it = tid + i * 256;
      if (it < P_ITEMS) {
        const int cg = it / PPIX, pix = it - cg * PPIX;
        const int pr = pix / PW, pc = pix - pr * PW;
        tbf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (T16)rp[i][e];
        *reinterpret_cast<tbf16x8*>(Ps + (pr * PWP + pc) * PT_STR + cg * 8) = v;
      }
    }
  };

  const int nkb = g.K / 32;
  const long HWo = (long)g.Ho * g.Wo;
  int tile = rank;
  Tc cur = coords(tile < ntiles ? tile : 0);
  if (tile < ntiles) load(cur, 0);
  for (; tile < ntiles; tile += nwg) {
    tf32x16 acc[4][NT];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][j][r] = 0.f;
    const int next = tile + nwg;
    const Tc nxt = coords(next < ntiles ? next : tile);
    for (int kb = 0; kb < nkb; ++kb) {
      __syncthreads();
      store();
      __syncthreads();
      if (kb + 1 < nkb) load(cur, kb + 1);
      else if (PERSIST && next < ntiles) load(nxt, 0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        tbf16x8 bfr[NSH][NSH][NT];
#pragma unroll
        for (int sh = 0; sh < NSH; ++sh)
#pragma unroll
          for (int sw = 0; sw < NSH; ++sw)
#pragma unroll
            for (int j = 0; j < NT; ++j)
              bfr[sh][sw][j] = *reinterpret_cast<const tbf16x8*>(Ps + pbase[j] + (sh * PWP + sw) * PT_STR + ks * 16);
#pragma unroll
        for (int kh = 0; kh < KS; ++kh) {
          const int ph = (kh + PAD) & 1;             // parity served by this tap row
          const int dh = (ph + PAD - kh) / 2;
#pragma unroll
          for (int kw = 0; kw < KS; ++kw) {
            const int pw = (kw + PAD) & 1;
            const int dw = (pw + PAD - kw) / 2;
            const tbf16x8 af = *reinterpret_cast<const tbf16x8*>(smem + (kh * KS + kw) * A_SZ + (wm * 32 + lr) * PT_STR +
                                                                 ks * 16 + lh * 8);
#pragma unroll
            for (int j = 0; j < NT; ++j)
              acc[ph * 2 + pw][j] = mfma16(af, bfr[dh - DMIN][dw - DMIN][j],
                                                                            acc[ph * 2 + pw][j]);
          }
        }
      }
    }

    // ---- epilogue: (+bias) (*act'(gpre)) (+= y), column parities paired into float2 ----
    float* yb = g.Y + (long)cur.b * g.y_bs;
    const float* gb = g.gpre ? g.gpre + (long)cur.b * g.gpre_bs : nullptr;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = (wn * NT + j) * 32 + lr;
      const int gi = cur.i0 + n / TW, gj = cur.j0 + n % TW;
      const int ow = 2 * gj;
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        const int oh = 2 * gi + ph;
        const bool rowok = gi < g.Hi && oh < g.Ho && gj < g.Wi;
        const bool pair = ow + 1 < g.Wo;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = cur.m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (!rowok || m >= g.M || ow >= g.Wo) continue;
          const float bv = g.bias ? g.bias[m] : 0.f;
          float v0 = acc[ph * 2][j][r] + bv, v1 = acc[ph * 2 + 1][j][r] + bv;
          const long o = (long)m * HWo + (long)oh * g.Wo + ow;
          if (pair) {
            if (gb) {
              const float2 gv = *reinterpret_cast<const float2*>(gb + o);
              v0 *= act_g(g.gact, gv.x, g.slope);
              v1 *= act_g(g.gact, gv.y, g.slope);
            }
            float2* dst = reinterpret_cast<float2*>(yb + o);
            if (g.accumulate) { const float2 old = *dst; v0 += old.x; v1 += old.y; }
            *dst = make_float2(v0, v1);
          } else {
            if (gb) v0 *= act_g(g.gact, gb[o], g.slope);
            yb[o] = g.accumulate ? yb[o] + v0 : v0;
          }
        }
      }
    }
    if (!PERSIST) break;
    cur = nxt;
  }
}

template <typename T16, int BM, int KS, bool PERSIST>
static void pt_launch(PtArgs& g, hipStream_t st) {
  g.tiles_w = (g.Wi + 15) / 16;
  g.tiles_h = (g.Hi + 7) / 8;
  const long tiles = (long)g.nb * g.tiles_w * g.tiles_h * ((g.M + BM - 1) / BM);
  const long grid = PERSIST && tiles > PT_WGS ? PT_WGS : tiles;
  hipLaunchKernelGGL((pconvt_kernel<T16, BM, KS, PERSIST>), dim3((unsigned)grid), dim3(256), 0, st, g);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_pconvt_supported(int K, int KS, int stride, int pad) {
  return K > 0 && K % 32 == 0 && stride == 2 && pad == 1 && (KS == 3 || KS == 4);
}

// y[b][m][oh][ow] (+)= (bias[m] + sum_taps Wb[tap][m][c] x[b][c][..]) (* gact'(gpre)): the stride-2,
// pad-1 transposed conv of x [nb][K][Hi][Wi] into y [nb][M][Ho][Wo] (Ho <= 2*Hi, Wo <= 2*Wi, both
// even or the last row/column dropped); Wb from dsgan_conv_wtrans_bf16 mode 2.
int dsgan_pconvt(const float* X, long x_bs, const void* Wb, const float* bias, float* Y, long y_bs,
                 const float* gpre, long gpre_bs, int nb, int K, int M, int Hi, int Wi, int Ho, int Wo,
                 int KS, int stride, int pad, int gact, float slope, int accumulate, hipStream_t st) {
  DSG_REQUIRE(X && Wb && Y && nb > 0 && M > 0 && Hi > 0 && Wi > 0, "dsgan_pconvt: bad args");
  DSG_REQUIRE(dsgan_pconvt_supported(K, KS, stride, pad), "dsgan_pconvt: unsupported K=%d KS=%d stride=%d pad=%d", K,
              KS, stride, pad);
  DSG_REQUIRE(Ho <= 2 * Hi && Wo <= 2 * Wi && Ho > 2 * Hi - 2 && Wo > 2 * Wi - 2, "dsgan_pconvt: bad output size");
  DSG_REQUIRE(((uintptr_t)Wb & 15) == 0 && ((uintptr_t)Y & 7) == 0 && (y_bs & 1) == 0 && (Wo & 1) == 0 &&
                  (!gpre || (((uintptr_t)gpre & 7) == 0 && (gpre_bs & 1) == 0)),
              "dsgan_pconvt: alignment (Wb 16 B, Y/gpre rows 8 B, even Wo)");
  PtArgs g{};
  g.X = X; g.x_bs = x_bs; g.Wb = (const unsigned short*)Wb; g.Y = Y; g.y_bs = y_bs; g.bias = bias;
  g.gpre = gpre; g.gpre_bs = gpre_bs; g.nb = nb; g.K = K; g.M = M; g.Hi = Hi; g.Wi = Wi; g.Ho = Ho; g.Wo = Wo;
  g.pad = pad; g.gact = gact; g.slope = slope; g.accumulate = accumulate;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    if (KS == 3) pt_launch<T16, 64, 3, false>(g, st);
    else pt_launch<T16, 32, 4, false>(g, st);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
