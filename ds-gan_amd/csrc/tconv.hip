// Tap-major implicit-GEMM convolution for KxK convs with K-channel count % 32 == 0 (gfx950, bf16 MFMA).
//
// Covers the dense 3x3 / 4x4 contractions of the step: VGG16 3x3 convs forward and data-grad
// (DSGAN/models/vgg.py:15-24), the PatchGAN 4x4 s2/s1 convs (DSGAN/models/networks.py:543-569),
// the G head (MixConvNeXtML.py:459) and the ConvTranspose2d 3x3 s2 forward (its stride-2
// parity classes, :53,150).
//
//   out[b][m][dst(o)] = act( sum_{tap, k} Wt[tap][m][k] * in[b][k][o*s + d(tap)] + bias[m] )
//
// * K is ordered tap-major (tap outer, channel inner): one 32-deep K step is 32 channels of ONE
//   tap, so every B row of the step has the same spatial shift.  Each thread owns one output
//   pixel (column) of the 128-pixel tile and 16 consecutive channels; the pixel's input offset
//   for the tap is computed once per tap, and channels advance by a scalar plane stride.
// * Loads are buffer loads; a tap that falls in the zero padding gets an offset past the
//   buffer range, so the hardware returns 0 -- no per-element mask VALU.
// * Weights are pre-transformed once per call into Wt[tap][m][k] (dsgan_conv_wtrans), so the A
//   tile is a row-major float4 stream.  Data-grads are the same kernel: stride 1 with the
//   flipped/transposed kernel, stride 2 as four parity classes each a stride-1 conv whose
//   outputs land on a stride-2 lattice of the destination.
#include "common.h"
#include "lds_pitch.h"
#include <type_traits>

namespace dsg {

typedef f32x16_t tf32x16;

constexpr int TBK = 32;
constexpr int T_STR = TBK + 8;  // [rows][k] bf16 tile stride, 80 B (conflict-free ds_read_b128)
constexpr int T_MAXTAPS = 16;

struct TcArgs {
  const float* X; long x_bs;     // input  [nb][K][Hin][Win]
  const float* Wt;               // [taps][M][K]
  float* Y; long y_bs;           // output [nb][M][Hdst][Wdst]
  const float* bias;
  const float* gpre; long gpre_bs;  // dst-shaped, act' multiplier (data-grad of the producer's act)
  int nb, K, M, Hin, Win, Hout, Wout, stride;
  int ntaps;
  int dh[T_MAXTAPS], dw[T_MAXTAPS];   // input offset of each tap: ih = oh*stride + dh
  int Hdst, Wdst, os, ph, pw;          // dst pixel = (oh*os + ph, ow*os + pw)
  int act, gact; float slope;
  float* ws; int kchunk;               // split-K (ws != NULL): raw partials [split][nb][M][Hout*Wout]
};

// ABF: Wt is bf16 (dsgan_conv_wtrans_bf16, cached per weight version): half the A bytes, copied to
// LDS unconverted.  XH: X is 16-bit (the half type; the ConvTranspose backward's output grad from
// dsgan_instnorm_bwd_h): half the B bytes, no conversion.
template <typename T16, int BM, bool ABF, bool XH = false>
__global__ __launch_bounds__(256, 2) void tconv_kernel(TcArgs g) {
  typedef hx8<T16> tbf16x8;
  constexpr int BN = 128;
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int A_SZ = BM * T_STR, B_SZ = BN * T_STR;
  constexpr int A_ITEMS = ABF ? BM * 4 / 256 : BM * 8 / 256;  // 16-byte items of the [BM][32] A tile
  __shared__ __attribute__((aligned(16))) T16 smem[2 * (A_SZ + B_SZ)];

  // wave index through readfirstlane: the compiler then knows it is uniform (SGPR), so
  // per-wave row offsets can be scalar soffsets instead of readfirstlane waterfall loops
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  const int Pout = g.Hout * g.Wout;
  const int ntpi = (Pout + BN - 1) / BN;       // N tiles per image
  const int mt = (g.M + BM - 1) / BM;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile % mt, rest0 = tile / mt;
  const int nn = g.nb * ntpi, split = rest0 / nn, rest = rest0 - split * nn;
  const int bimg = rest / ntpi, nt_i = rest - bimg * ntpi;
  const int m0 = m_t * BM, q0 = nt_i * BN;

  const int HWin = g.Hin * g.Win;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.Wt, (short)0, (unsigned)((long)g.ntaps * g.M * g.K * (ABF ? 2 : 4)), 0x00020000);
  constexpr int XB = XH ? 2 : 4;   // bytes per X element
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)g.X + (long)bimg * g.x_bs * XB), (short)0, (unsigned)((long)g.K * HWin * XB), 0x00020000);

  // B staging: thread -> column c = tid % 128, channels 16*(tid/128) .. +15 of the step
  const int col = tid & 127, kc = wave >> 1;   // kc uniform per wave: channel rows are soffsets
  const int q = q0 + col;
  const bool qv = q < Pout;
  const int oh = qv ? q / g.Wout : 0, ow = qv ? q - (q / g.Wout) * g.Wout : 0;
  const int ih0 = oh * g.stride, iw0 = ow * g.stride;

  const int ksteps_per_tap = g.K / TBK;
  const int nk_all = g.ntaps * ksteps_per_tap;
  const int kb0 = g.ws ? split * g.kchunk : 0;
  const int nk = g.ws ? min(g.kchunk, nk_all - kb0) : nk_all;   // K steps of this split

  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  float4 ra[ABF ? 1 : A_ITEMS];
  u32x4 rha[ABF ? A_ITEMS : 1];
  float rb[XH ? 1 : 16];
  unsigned short rh[XH ? 16 : 1];
  auto gload = [&](int kt0) {
    const int kt = kb0 + kt0;
    const int tap = kt / ksteps_per_tap;
    const int k0 = (kt - tap * ksteps_per_tap) * TBK;
    // A rows past M get an offset past the resource range (reads 0, no branch)
    const unsigned wtap = (unsigned)tap * g.M * g.K * (ABF ? 2u : 4u);
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256;
      if constexpr (ABF) {   // 8 bf16 per item, 4 items per 32-deep row
        const int m = m0 + p80_row16(it), kk = k0 + p80_slot16(it) * 8;
        const unsigned off = m < g.M ? ((unsigned)m * g.K + kk) * 2u : 0xFFFFFFF0u;
        rha[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, (int)off, wtap, 0));
      } else {
        const int m = m0 + p80_row8(it), kk = k0 + p80_piece8(it) * 4;
        const unsigned off = m < g.M ? ((unsigned)m * g.K + kk) * 4u : 0xFFFFFFF0u;
        ra[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw, (int)off, wtap, 0));
      }
    }
    const int ih = ih0 + g.dh[tap], iw = iw0 + g.dw[tap];
    const bool in = qv && (unsigned)ih < (unsigned)g.Hin && (unsigned)iw < (unsigned)g.Win;
    const int voff = in ? (ih * g.Win + iw) * XB : 0x7fffffff;
    const int kb = k0 + 16 * kc;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (XH) rh[j] = __builtin_amdgcn_raw_buffer_load_b16(rx, voff, (kb + j) * HWin * 2, 0);
      else rb[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rx, voff, (kb + j) * HWin * 4, 0));
    }
  };
  auto sstore = [&](int buf) {
    T16* As = smem + buf * (A_SZ + B_SZ);
    T16* Bs = As + A_SZ;
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256;
      if constexpr (ABF) {
        *reinterpret_cast<u32x4*>(As + p80_row16(it) * T_STR + p80_slot16(it) * 8) = rha[i];
        continue;
      }
      typedef __attribute__((ext_vector_type(4))) T16 b4;
      b4 v;
      v[0] = (T16)ra[i].x; v[1] = (T16)ra[i].y; v[2] = (T16)ra[i].z; v[3] = (T16)ra[i].w;
      *reinterpret_cast<b4*>(As + p80_row8(it) * T_STR + p80_piece8(it) * 4) = v;
    }
    tbf16x8 lo, hi;
    if constexpr (XH) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { lo[j] = __builtin_bit_cast(T16, rh[j]); hi[j] = __builtin_bit_cast(T16, rh[8 + j]); }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) { lo[j] = (T16)rb[j]; hi[j] = (T16)rb[8 + j]; }
    }
    tbf16x8* dst = reinterpret_cast<tbf16x8*>(Bs + col * T_STR + 16 * kc);
    dst[0] = lo;
    dst[1] = hi;
  };

  tf32x16 acc[TM][TN];
  const bool has_bias = g.bias != nullptr && !g.ws;   // split-K: the bias is added by the reduce
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = 0.f;
    if (has_bias) {   // one uniform branch; guarded loads are clamp + select (see igemm.hip ldsel)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float t = g.bias[m < g.M ? m : 0];
        bv[r] = m < g.M ? t : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = bv[r];
  }

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const T16* As = smem + buf * (A_SZ + B_SZ);
    const T16* Bs = As + A_SZ;
#pragma unroll
    for (int ks = 0; ks < TBK / 16; ++ks) {
      tbf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = *reinterpret_cast<const tbf16x8*>(As + (wm * TM * 32 + i * 32 + lr) * T_STR + ks * 16 + lh * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = *reinterpret_cast<const tbf16x8*>(Bs + (wn * TN * 32 + j * 32 + lr) * T_STR + ks * 16 + lh * 8);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  if (g.ws) {   // split-K partial: rows m, pixel-contiguous along the lanes (coalesced)
    float* wp = g.ws + ((long)split * g.nb + bimg) * g.M * Pout;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int qq = q0 + wn * TN * 32 + j * 32 + lr;
      if (qq >= Pout) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < g.M) wp[(long)m * Pout + qq] = acc[i][j][r];
        }
    }
    return;
  }
  // ---- epilogue: dst pixel of this lane's column, channel rows via scalar offsets ----
  const int HWd = g.Hdst * g.Wdst;
  const unsigned range = (unsigned)((long)g.M * HWd * 4);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.Y + (long)bimg * g.y_bs), (short)0, range, 0x00020000);
  __amdgpu_buffer_rsrc_t rg = ry;
  if (g.gpre) rg = __builtin_amdgcn_make_buffer_rsrc((void*)(g.gpre + (long)bimg * g.gpre_bs), (short)0, range, 0x00020000);
  const bool full = m0 + BM <= g.M;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c = wn * TN * 32 + j * 32 + lr;
    const int qq = q0 + c;
    int vbase = 0x7fffffff;
    if (qq < Pout) {
      const int ohh = qq / g.Wout, oww = qq - ohh * g.Wout;
      vbase = (((ohh * g.os + g.ph) * g.Wdst + oww * g.os + g.pw) + 4 * lh * HWd) * 4;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mrow = m0 + wm * TM * 32 + i * 32;
      const int mlim = full ? BM : g.M - mrow - 4 * lh;   // rows (r&3)+8(r>>2) < mlim are valid
      int vrow[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) vrow[r] = ((r & 3) + 8 * (r >> 2) < mlim) ? vbase : 0x7fffffff;
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r];
      if (g.gpre) {
        float gv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          gv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
              rg, vrow[r], (mrow + (r & 3) + 8 * (r >> 2)) * HWd * 4, 0));
        act_g_mul_arr(g.gact, v, gv, g.slope);
      }
      act_f_arr(g.act, v, g.slope);
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[r]), ry, vrow[r],
                                              (mrow + (r & 3) + 8 * (r >> 2)) * HWd * 4, 0);
    }
  }
}

// Split-K finish: y[b][m][dst(q)] = act( sum_s ws[s][b][m][q] + bias[m] ) (* gact'(gpre)),
// splits added in a fixed order (deterministic).
__global__ __launch_bounds__(256) void tconv_reduce_kernel(TcArgs g, int S) {
  const int Pout = g.Hout * g.Wout, HWd = g.Hdst * g.Wdst;
  const long per = (long)g.nb * g.M * Pout;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < per; e += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += g.ws[(long)s * per + e];
    const int q = (int)(e % Pout);
    const long bm = e / Pout;
    const int m = (int)(bm % g.M), b = (int)(bm / g.M);
    if (g.bias) v += g.bias[m];
    const int oh = q / g.Wout, ow = q - oh * g.Wout;
    const long d = (long)m * HWd + (long)(oh * g.os + g.ph) * g.Wdst + ow * g.os + g.pw;
    if (g.gpre) v *= act_g(g.gact, g.gpre[(long)b * g.gpre_bs + d], g.slope);
    g.Y[(long)b * g.y_bs + d] = act_f(g.act, v, g.slope);
  }
}

// K split of a launch whose tiles leave the chip under-filled (the deep ConvT data-grads: 256
// tiles of 144 K steps at 16^2): about 1024 workgroups, >= 16 K steps each.
static int tc_splits(long tiles, int nk, int* kchunk) {
  long S = (1024 + tiles - 1) / tiles;
  if (S > nk / 16) S = nk / 16;
  if (tiles >= 512 || S < 2) { *kchunk = nk; return 1; }
  const int kc = (int)((nk + S - 1) / S);
  *kchunk = kc;
  return (nk + kc - 1) / kc;
}

// Wt[tap][m][k] from an OIHW weight W[Co][Ci][KH][KW].
//   mode 0 (forward):      m = co, k = ci, tap = (kh, kw)
//   mode 1 (data-grad s1): m = ci, k = co, tap = (kh', kw') with kh = KH-1-kh'
//   mode 2 (data-grad s2 parity class): m = ci, k = co, tap = (th', tw'),
//                          kh = kh0 + 2*(nth-1-th'), kw = kw0 + 2*(ntw-1-tw')
__global__ void wtrans_kernel(const float* __restrict__ W, float* __restrict__ Wt, int Co, int Ci,
                              int KH, int KW, int mode, int kh0, int kw0, int nth, int ntw) {
  const int M = mode == 0 ? Co : Ci, K = mode == 0 ? Ci : Co;
  const int taps = mode == 2 ? nth * ntw : KH * KW;
  const long total = (long)taps * M * K;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int k = e % K; const long t = e / K;
    const int m = t % M; const int tap = t / M;
    int kh, kw, co, ci;
    if (mode == 0) { kh = tap / KW; kw = tap % KW; co = m; ci = k; }
    else if (mode == 1) { kh = KH - 1 - tap / KW; kw = KW - 1 - tap % KW; co = k; ci = m; }
    else { const int th = tap / ntw, tw = tap % ntw; kh = kh0 + 2 * (nth - 1 - th); kw = kw0 + 2 * (ntw - 1 - tw); co = k; ci = m; }
    Wt[e] = W[(((long)co * Ci + ci) * KH + kh) * KW + kw];
  }
}

}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_conv_wtrans(const float* W, float* Wt, int Co, int Ci, int KH, int KW, int mode, int kh0,
                      int kw0, int nth, int ntw, hipStream_t st) {
  DSG_REQUIRE(W && Wt && mode >= 0 && mode <= 2, "dsgan_conv_wtrans: bad args");
  const long taps = mode == 2 ? (long)nth * ntw : (long)KH * KW;
  const long total = taps * Co * Ci;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(wtrans_kernel, dim3((unsigned)blocks), dim3(256), 0, st, W, Wt, Co, Ci, KH, KW,
                     mode, kh0, kw0, nth, ntw);
  DSG_CHECK_LAUNCH();
  return 0;
}

static long tc_tiles(int nb, int M, int Hout, int Wout) {
  return (long)nb * ((Hout * Wout + 127) / 128) * (M > 64 ? (M + 127) / 128 : (M + 63) / 64);
}

// fp32 scratch dsgan_tconv_ws needs (0: the launch is not split)
long dsgan_tconv_workspace(int nb, int K, int M, int Hout, int Wout, int ntaps) {
  if (K % TBK != 0 || K <= 0) return 0;
  int kc;
  const int S = tc_splits(tc_tiles(nb, M, Hout, Wout), ntaps * (K / TBK), &kc);
  return S > 1 ? (long)S * nb * M * Hout * Wout : 0;
}

int dsgan_tconv_ws(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                   int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                   int os, int ph, int pw, int act, int gact, float slope, int wt_bf16, float* ws, long ws_elems,
                   hipStream_t st);

// Generic launcher.  taps: ntaps pairs (dh, dw).  dst lattice: (oh*os+ph, ow*os+pw) in Hdst x Wdst.
int dsgan_tconv(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                int os, int ph, int pw, int act, int gact, float slope, hipStream_t st) {
  return dsgan_tconv_ws(X, x_bs, Wt, bias, Y, y_bs, gpre, gpre_bs, nb, K, M, Hin, Win, Hout, Wout, stride, ntaps,
                        dh, dw, Hdst, Wdst, os, ph, pw, act, gact, slope, 0, nullptr, 0, st);
}

}  // extern "C"

static int tconv_impl(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                      const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                      int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                      int os, int ph, int pw, int act, int gact, float slope, int wt_bf16, int x_half, float* ws,
                      long ws_elems, hipStream_t st) {
  DSG_REQUIRE(X && Wt && Y && nb > 0 && M > 0 && Hout > 0 && Wout > 0, "dsgan_tconv: bad args");
  DSG_REQUIRE(K % TBK == 0 && K > 0, "dsgan_tconv: K (input channels) must be a multiple of 32");
  DSG_REQUIRE(ntaps >= 1 && ntaps <= T_MAXTAPS, "dsgan_tconv: 1..16 taps");
  DSG_REQUIRE((long)K * Hin * Win * 4 < 0x7fffffffL && (long)M * Hdst * Wdst * 4 < 0x7fffffffL,
              "dsgan_tconv: tensor exceeds a 2 GiB buffer resource");
  DSG_REQUIRE(((uintptr_t)Wt & 15) == 0, "dsgan_tconv: Wt must be 16-byte aligned");
  DSG_REQUIRE((long)ntaps * M * K * 4 < 0xFFFFFFF0L, "dsgan_tconv: Wt exceeds a 4 GiB buffer resource");
  DSG_REQUIRE(!wt_bf16 || K % 8 == 0, "dsgan_tconv: bf16 Wt needs K %% 8 == 0");
  TcArgs g{};
  g.X = X; g.x_bs = x_bs; g.Wt = Wt; g.Y = Y; g.y_bs = y_bs; g.bias = bias; g.gpre = gpre;
  g.gpre_bs = gpre_bs; g.nb = nb; g.K = K; g.M = M; g.Hin = Hin; g.Win = Win; g.Hout = Hout;
  g.Wout = Wout; g.stride = stride; g.ntaps = ntaps;
  for (int t = 0; t < ntaps; ++t) { g.dh[t] = dh[t]; g.dw[t] = dw[t]; }
  g.Hdst = Hdst; g.Wdst = Wdst; g.os = os; g.ph = ph; g.pw = pw;
  g.act = act; g.gact = gact; g.slope = slope;
  const long tiles = tc_tiles(nb, M, Hout, Wout);
  int kc;
  const int S = ws ? tc_splits(tiles, ntaps * (K / TBK), &kc) : 1;
  g.ws = S > 1 ? ws : nullptr;
  g.kchunk = S > 1 ? kc : 0;
  DSG_REQUIRE(S == 1 || (long)S * nb * M * Hout * Wout < (1L << 31), "dsgan_tconv: split partials too large");
  DSG_WS(S > 1 ? (long)S * nb * M * Hout * Wout : 0, ws, ws_elems, "dsgan_tconv (dsgan_tconv_workspace)");
  const dim3 grid((unsigned)(tiles * S));
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    if (x_half) {   // (the ConvTranspose data-grads: bf16 weights)
      if (M > 64) hipLaunchKernelGGL((tconv_kernel<T16, 128, true, true>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((tconv_kernel<T16, 64, true, true>), grid, dim3(256), 0, st, g);
    } else if (M > 64) {
      if (wt_bf16) hipLaunchKernelGGL((tconv_kernel<T16, 128, true>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((tconv_kernel<T16, 128, false>), grid, dim3(256), 0, st, g);
    } else {
      if (wt_bf16) hipLaunchKernelGGL((tconv_kernel<T16, 64, true>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((tconv_kernel<T16, 64, false>), grid, dim3(256), 0, st, g);
    }
  });
  DSG_CHECK_LAUNCH();
  if (S > 1) {
    const long per = (long)nb * M * Hout * Wout;
    long blocks = (per + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(tconv_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g, S);
    DSG_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" {

// Same, with the split-K scratch of dsgan_tconv_workspace (NULL: never split).
int dsgan_tconv_ws(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                   const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                   int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                   int os, int ph, int pw, int act, int gact, float slope, int wt_bf16, float* ws, long ws_elems,
                   hipStream_t st) {
  return tconv_impl(X, x_bs, Wt, bias, Y, y_bs, gpre, gpre_bs, nb, K, M, Hin, Win, Hout, Wout, stride, ntaps, dh, dw,
                    Hdst, Wdst, os, ph, pw, act, gact, slope, wt_bf16, 0, ws, ws_elems, st);
}

// Same with X in the library's 16-bit half type (x_bs in elements) and 16-bit Wt
// (dsgan_conv_wtrans_bf16): the ConvTranspose backward on dsgan_instnorm_bwd_h's output.
int dsgan_tconv_ws_xh(const void* Xh, long x_bs, const void* Wt, const float* bias, float* Y, long y_bs,
                      const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                      int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                      int os, int ph, int pw, int act, int gact, float slope, float* ws, long ws_elems,
                      hipStream_t st) {
  DSG_REQUIRE(K % 8 == 0, "dsgan_tconv_ws_xh: K %% 8 != 0");
  return tconv_impl((const float*)Xh, x_bs, (const float*)Wt, bias, Y, y_bs, gpre, gpre_bs, nb, K, M, Hin, Win, Hout,
                    Wout, stride, ntaps, dh, dw, Hdst, Wdst, os, ph, pw, act, gact, slope, 1, 1, ws, ws_elems, st);
}

}  // extern "C"
