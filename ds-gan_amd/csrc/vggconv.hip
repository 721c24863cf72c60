// The frozen VGG16 perceptual pass (DSGAN/models/vgg.py:15-42, used by backward_G at
// DSGAN/models/pix2pix_model.py:180-186) in channel-blocked bf16 for gfx950.
//
// Layout "CB16": [n][c / 16][h][w][c % 16].  One pixel of one 16-channel block is 32 contiguous
// bytes (bf16) or 64 (fp32), a row of a block is W * 32 contiguous bytes, so the implicit-GEMM
// operand of a 16-channel K chunk is a dense 2-D region: 16-byte vector loads, whole cache lines.
//
// Storage precision is exact with respect to the bf16-operand arithmetic: every activation the
// next conv reads is the bf16 rounding the MFMA would apply anyway, max commutes with that
// (monotone) rounding, and a ReLU mask only needs the sign.  Only the four tapped features
// (relu1_2, relu2_2, relu3_3, relu4_3) the L1 loss reads stay fp32.  The data-grads in the
// backward walk are likewise stored as the bf16 they are consumed as.
//
// Kernels:
//   vconv3x3_kernel   3x3 / pad 1 / stride 1 conv as implicit GEMM on v_mfma_f32_32x32x16_bf16:
//                     M = output channels, N = 32-wide pixel rows, K = 9 taps x input channels.
//                     A workgroup owns BM channels x (TH x 32) pixels of one image; per 16-channel
//                     chunk it stages the weights of all 9 taps (pre-swizzled in HBM into the LDS
//                     image, one contiguous block) and the (TH+2) x 34 input patch once, then runs
//                     9 taps x (TM x TN) MFMAs per wave from LDS.  Epilogue: bias + ReLU (forward)
//                     or x ReLU'(mask) (data-grad), bf16 or fp32 CB16 out.
//   vgg_conv1_fwd     conv1_1 (3 -> 64, K = 27): NCHW fp32 image -> CB16 bf16, exact fp32 FMAs.
//   vgg_conv1_dgrad   its data-grad (64 -> 3): CB16 bf16 -> NCHW fp32.
//   cb16_maxpool      MaxPool2d(2) of a tapped fp32 feature -> bf16 + 2-bit window argmax.
//   cb16_tap_bwd      (maxpool backward + L1 backward) x ReLU' at a tapped layer -> bf16.
#include "common.h"
#include "lds_dma.h"
#include <type_traits>

namespace dsg {

typedef f32x16_t vgf16;
typedef __attribute__((ext_vector_type(4))) unsigned int vgu4;
typedef __attribute__((ext_vector_type(4))) unsigned char vgc4;

__device__ __forceinline__ long cb16(int n, int c, int h, int w, int C, int H, int W) {
  return ((((long)n * (C >> 4) + (c >> 4)) * H + h) * W + w) * 16 + (c & 15);
}

template <typename T16>
struct VcArgs {
  const T16* X;      // CB16 [N][K][H][W]
  const T16* Wt;     // [M/BM][K/16][9][2][BM][8] (dsgan_vconv_wtrans)
  const float* bias;    // [M] or null
  const T16* mask;   // CB16 [N][M][H][W] or null: out *= (mask > 0)
  void* Y;              // CB16 [N][M][H][W], bf16 or fp32 (y_f32)
  int N, K, M, H, W;
  int tiles_w, tiles_h;
  int relu, y_f32;
  const void* zero;     // 16 zero bytes in global memory (the LDS-DMA kernel's out-of-image source)
};

template <typename T16, int BM, int TH>
__global__ __launch_bounds__(256, 2) void vconv3x3_kernel(VcArgs<T16> g) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  constexpr int TW = 32, BN = TH * TW;
  constexpr int WM = BM / 64, WN = 4 / WM;           // waves along M (64 rows each) and N
  constexpr int TM = 2, TN = BN / WN / 32;           // 32x32 MFMA tiles per wave
  constexpr int PH = TH + 2, PW = TW + 2;            // input patch of one pixel tile
  constexpr int A_PIECES = 9 * 2 * BM;               // 16-byte pieces per K chunk (all taps)
  constexpr int B_PIECES = 2 * PH * PW;
  constexpr int A_IT = (A_PIECES + 255) / 256, B_IT = (B_PIECES + 255) / 256;
  static_assert(TN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) vgu4 smem[A_PIECES + B_PIECES];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // Tile decode: pixel tile fastest; each XCD gets a contiguous run of tile ids (blocks
  // b, b+8, ... share an XCD under round-robin dispatch), so an XCD mostly streams ONE M tile's
  // weights from its L2 while the patches (read once per M tile) come from the Infinity Cache.
  const int npt = g.N * g.tiles_w * g.tiles_h;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile / npt, pt = tile - m_t * npt;
  const int tpi = g.tiles_w * g.tiles_h;
  const int img = pt / tpi, ti = pt - img * tpi;
  const int oh0 = (ti / g.tiles_w) * TH, ow0 = (ti % g.tiles_w) * TW;
  const int nkc = g.K >> 4;

  const vgu4* wsrc = reinterpret_cast<const vgu4*>(g.Wt) + (long)m_t * nkc * A_PIECES;
  vgu4 ra[A_IT], rb[B_IT];
  auto gload = [&](int kc) {
    const vgu4* a = wsrc + (long)kc * A_PIECES;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256;
      if (A_PIECES % 256 == 0 || it < A_PIECES) ra[i] = a[it];
    }
    const T16* xb = g.X + (((long)img * nkc + kc) * g.H) * (long)g.W * 16;
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + i * 256;
      const int pix = it >> 1, half = it & 1;
      const int ph = pix / PW, pw = pix - ph * PW;
      const int ih = oh0 - 1 + ph, iw = ow0 - 1 + pw;
      const bool ok = it < B_PIECES && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
      vgu4 v = {0u, 0u, 0u, 0u};
      if (ok) v = *reinterpret_cast<const vgu4*>(xb + ((long)ih * g.W + iw) * 16 + half * 8);
      rb[i] = v;
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256;
      if (A_PIECES % 256 == 0 || it < A_PIECES) smem[it] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + i * 256;
      if (it < B_PIECES) {
        const int pix = it >> 1, half = it & 1;
        smem[A_PIECES + half * PH * PW + pix] = rb[i];   // [half][ph][pw]
      }
    }
  };

  vgf16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const T16* Ab = reinterpret_cast<const T16*>(smem);
  const T16* Bb = reinterpret_cast<const T16*>(smem + A_PIECES);
  gload(0);
  for (int kc = 0; kc < nkc; ++kc) {
    __syncthreads();   // the previous chunk's fragments have been read
    sstore();
    __syncthreads();
    if (kc + 1 < nkc) gload(kc + 1);   // next chunk in flight under this chunk's MFMAs
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap - (tap / 3) * 3;
      vgb8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * 64 + i * 32 + lr;
        af[i] = *reinterpret_cast<const vgb8*>(Ab + ((tap * 2 + lh) * BM + row) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int prow = (wn * (BN / WN) + j * 32) / TW;   // output row of this 32-pixel tile
        bfr[j] = *reinterpret_cast<const vgb8*>(Bb + ((lh * PH + prow + kh) * PW + lr + kw) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  // ---- epilogue: lane holds pixel lr of each 32-pixel tile, channels (r&3)+8(r>>2)+4lh: four
  // consecutive channels per register quad -> one 8-byte (bf16) or 16-byte (fp32) store ----
  // bias quads of this lane's channels loaded once (re-read after every store otherwise: the compiler
  // cannot prove Y and bias apart) and each j's mask quads before their first use -- the epilogue
  // waited one memory latency per quad
  float4 bias4[TM][4];
  if (g.bias) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) bias4[i][q] = *reinterpret_cast<const float4*>(g.bias + m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = wn * (BN / WN) + j * 32 + lr;
    const int oh = oh0 + n / TW, ow = ow0 + n % TW;
    vgb4 mks[TM][4];   // this j's mask quads, all loaded before the first use
    if (g.mask) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          mks[i][q] = *reinterpret_cast<const vgb4*>(
              g.mask + cb16(img, m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh, oh, ow, g.M, g.H, g.W));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        if (g.bias) {
          const float4 bv = bias4[i][q];
          v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
        }
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        const long o = cb16(img, m, oh, ow, g.M, g.H, g.W);
        if (g.mask) {
          const vgb4 mk = mks[i][q];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (float)mk[e] > 0.f ? v[e] : 0.f;
        }
        if (g.y_f32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.Y) + o) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          vgb4 b;
#pragma unroll
          for (int e = 0; e < 4; ++e) b[e] = (T16)v[e];
          *reinterpret_cast<vgb4*>(reinterpret_cast<T16*>(g.Y) + o) = b;
        }
      }
  }
}

// The same 3x3 implicit GEMM as vconv3x3_kernel, restructured around an LDS-DMA ring: 8 waves
// (2 per SIMD, one workgroup per CU) own BM channels x (TH x 32) pixels; the K chunk (16 input
// channels: all 9 taps of the pre-swizzled weight image + the (TH+2) x 34 input patch) is copied
// global -> LDS by global_load_lds_dwordx4 straight into one of two stage buffers -- no VGPR
// staging, no ds_write pass -- while the MFMAs run on the other: ONE barrier per chunk.  The patch
// is a gather (per-lane source address; lanes outside the image read a 16-byte zero block), its LDS
// image lane-linear in [half][ph][pw] order as in vconv3x3_kernel.  Per tap the next tap's A / B
// fragments are read while this tap's MFMAs issue.  Arithmetic (operand values, accumulation order
// per output: chunks in order, taps in order within a chunk) is vconv3x3_kernel's: same bits.
// KWM: taps in kw-major order so that one kw's B fragments serve all three kh: per kw the TN + 2
// patch rows are read once (TN + 2 row fragments instead of 3 TN), 18 B reads per chunk instead of
// 36.  The taps of an output are then summed (kw, kh) in kw-major order: the same products, another
// order of the fp32 sums (not the register-staged kernel's bits).
template <typename T16, int BM, int TH, bool KWM = false>
__global__ __launch_bounds__(512, 1) void vconv3x3_dma_kernel(VcArgs<T16> g) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  constexpr int TW = 32, BN = TH * TW;
  constexpr int WM = BM / 64, WN = 8 / WM;           // waves along M (64 rows each) and N
  constexpr int TM = 2, TN = BN / WN / 32;           // 32x32 MFMA tiles per wave
  constexpr int PH = TH + 2, PW = TW + 2;
  constexpr int A_BYTES = 9 * 2 * BM * 16;           // weight image of one K chunk (1 KB multiple)
  constexpr int B_SLOTS = 2 * PH * PW;               // 16-byte patch slots [half][ph][pw]
  constexpr int B_PIECES = (B_SLOTS + 63) / 64;      // 1 KB LDS-DMA pieces (the tail slots read zeros)
  constexpr int STAGE = A_BYTES + B_PIECES * 1024;
  constexpr int A_PIECES = A_BYTES / 1024;
  constexpr int NBW = (B_PIECES + 7) / 8;            // patch pieces per wave (at most)
  static_assert(TN >= 1 && A_BYTES % 1024 == 0 && 2 * STAGE <= 160 * 1024, "tile");
  __shared__ __attribute__((aligned(16))) vgu4 smem[2 * STAGE / 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  const int npt = g.N * g.tiles_w * g.tiles_h;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile / npt, pt = tile - m_t * npt;
  const int tpi = g.tiles_w * g.tiles_h;
  const int img = pt / tpi, ti = pt - img * tpi;
  const int oh0 = (ti / g.tiles_w) * TH, ow0 = (ti % g.tiles_w) * TW;
  const int nkc = g.K >> 4;
  const long plane = (long)g.H * g.W * 16;           // elements of one 16-channel block of one image

  // per-lane patch gather offsets (elements within a chunk plane; -1 = outside the image)
  int boff[NBW];
#pragma unroll
  for (int q = 0; q < NBW; ++q) {
    const int s = (wave + 8 * q) * 64 + lane;
    int off = -1;
    if (s < B_SLOTS) {
      const int half = s / (PH * PW), rem = s - half * (PH * PW);
      const int ph = rem / PW, pw = rem - ph * PW;
      const int ih = oh0 - 1 + ph, iw = ow0 - 1 + pw;
      if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W) off = (ih * g.W + iw) * 16 + half * 8;
    }
    boff[q] = off;
  }
  const char* wsrc = reinterpret_cast<const char*>(g.Wt) + (long)m_t * nkc * A_BYTES;
  const unsigned lbase = lds_off(smem);
  auto issue = [&](int kc, int stage) __attribute__((always_inline)) {
    const unsigned ls = lbase + stage * STAGE;
    const char* a = wsrc + (long)kc * A_BYTES + lane * 16;
#pragma unroll
    for (int p0 = 0; p0 < A_PIECES; p0 += 8)
      if (p0 + wave < A_PIECES) dma16(a + (p0 + wave) * 1024, ls + (p0 + wave) * 1024);
    const T16* xb = g.X + ((long)img * nkc + kc) * plane;
#pragma unroll
    for (int q = 0; q < NBW; ++q) {
      const int p = wave + 8 * q;
      if (p < B_PIECES)
        dma16(boff[q] >= 0 ? (const void*)(xb + boff[q]) : g.zero, ls + A_BYTES + p * 1024);
    }
  };

  vgf16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  issue(0, 0);
  for (int kc = 0; kc < nkc; ++kc) {
    dma_wait_all();                 // this wave's pieces of chunk kc have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();   // every wave's pieces landed; every wave is done with chunk kc-1
    if (kc + 1 < nkc) issue(kc + 1, (kc + 1) & 1);
    const T16* Ab = reinterpret_cast<const T16*>(reinterpret_cast<const char*>(smem) + (kc & 1) * STAGE);
    const T16* Bb = Ab + A_BYTES / 2;
    if constexpr (KWM) {
      vgb8 af[2][TM], bq[2][TN + 2];
      auto afr = [&](int tap, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[b][i] = *reinterpret_cast<const vgb8*>(Ab + ((tap * 2 + lh) * BM + wm * 64 + i * 32 + lr) * 8);
      };
      auto bro = [&](int kw, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < TN + 2; ++r)
          bq[b][r] = *reinterpret_cast<const vgb8*>(Bb + ((lh * PH + wn * TN + r) * PW + lr + kw) * 8);
      };
      bro(0, 0);
      afr(0, 0);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        if (kw + 1 < 3) bro(kw + 1, (kw + 1) & 1);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int s = kw * 3 + kh;   // step in kw-major order; tap = kh * 3 + kw
          if (s + 1 < 9) afr(((s + 1) % 3) * 3 + (s + 1) / 3, (s + 1) & 1);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = mfma16(af[s & 1][i], bq[kw & 1][j + kh], acc[i][j]);
        }
      }
    } else {
    vgb8 af[2][TM], bfr[2][TN];
    auto frags = [&](int tap, int b) __attribute__((always_inline)) {
      const int kh = tap / 3, kw = tap - (tap / 3) * 3;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[b][i] = *reinterpret_cast<const vgb8*>(Ab + ((tap * 2 + lh) * BM + wm * 64 + i * 32 + lr) * 8);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[b][j] = *reinterpret_cast<const vgb8*>(Bb + ((lh * PH + wn * TN + j + kh) * PW + lr + kw) * 8);
    };
    frags(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) frags(tap + 1, (tap + 1) & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16(af[tap & 1][i], bfr[tap & 1][j], acc[i][j]);
    }
    }
  }

  // ---- epilogue (vconv3x3_kernel's) ----
  // bias quads of this lane's channels loaded once (re-read after every store otherwise: the compiler
  // cannot prove Y and bias apart) and each j's mask quads before their first use -- the epilogue
  // waited one memory latency per quad
  float4 bias4[TM][4];
  if (g.bias) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) bias4[i][q] = *reinterpret_cast<const float4*>(g.bias + m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = (wn * TN + j) * 32 + lr;
    const int oh = oh0 + n / TW, ow = ow0 + n % TW;
    vgb4 mks[TM][4];   // this j's mask quads, all loaded before the first use
    if (g.mask) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          mks[i][q] = *reinterpret_cast<const vgb4*>(
              g.mask + cb16(img, m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh, oh, ow, g.M, g.H, g.W));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m_t * BM + wm * 64 + i * 32 + q * 8 + 4 * lh;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        if (g.bias) {
          const float4 bv = bias4[i][q];
          v[0] += bv.x; v[1] += bv.y; v[2] += bv.z; v[3] += bv.w;
        }
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        const long o = cb16(img, m, oh, ow, g.M, g.H, g.W);
        if (g.mask) {
          const vgb4 mk = mks[i][q];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = (float)mk[e] > 0.f ? v[e] : 0.f;
        }
        if (g.y_f32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(g.Y) + o) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          vgb4 b;
#pragma unroll
          for (int e = 0; e < 4; ++e) b[e] = (T16)v[e];
          *reinterpret_cast<vgb4*>(reinterpret_cast<T16*>(g.Y) + o) = b;
        }
      }
  }
}

// Wt[mt][kc][tap][half][BM][8]: the LDS image of weight chunk kc of M tile mt.  Forward: row m =
// output channel, k = input channel, tap (kh, kw).  Data-grad (dgrad=1): row m = input channel,
// k = output channel, W flipped: value W[k][m][2-kh][2-kw].
template <typename T16>
__global__ void vconv_wtrans_kernel(const float* __restrict__ W, T16* __restrict__ Wt, int Co, int Ci, int BM,
                                    int dgrad) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  const int M = dgrad ? Ci : Co, K = dgrad ? Co : Ci;
  const long total = 9L * M * K;
  const int nkc = K >> 4;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    long t = e;
    const int j = (int)(t & 7); t >>= 3;
    const int row = (int)(t % BM); t /= BM;
    const int half = (int)(t & 1); t >>= 1;
    const int tap = (int)(t % 9); t /= 9;
    const int kc = (int)(t % nkc);
    const int mt = (int)(t / nkc);
    const int m = mt * BM + row, k = kc * 16 + half * 8 + j;
    const int kh = tap / 3, kw = tap % 3;
    const int co = dgrad ? k : m, ci = dgrad ? m : k;
    const int fh = dgrad ? 2 - kh : kh, fw = dgrad ? 2 - kw : kw;
    Wt[e] = (T16)W[(((long)co * Ci + ci) * 3 + fh) * 3 + fw];
  }
}

// conv1_1 (DSGAN/models/vgg.py:17): y[n][c][h][w] = relu(b[c] + sum_{ci,kh,kw} w[c][ci][kh][kw] *
// x[n][ci][h-1+kh][w-1+kw]), exact fp32 FMAs in (ci, kh, kw) order, stored CB16 bf16.  Thread =
// (pixel, 16-channel block).
template <typename T16, bool UNI>
__global__ __launch_bounds__(256) void vgg_conv1_fwd_kernel(const float* __restrict__ x, long x_bs,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            T16* __restrict__ y, int N, int H, int W) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  // UNI (HW % 64 == 0): a wave's 64 pixels share (n, cb), so the channel block is wave-uniform and
  // its 16 x 27 weights + biases come through the scalar cache (s_load), not one LDS read per FMA
  const long HW = (long)H * W;
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= (long)N * 4 * HW) return;
  const long pix = t % HW;
  const int cb = UNI ? __builtin_amdgcn_readfirstlane((int)((t / HW) & 3)) : (int)((t / HW) & 3);
  const int n = (int)(t / (HW * 4));
  const int h = (int)(pix / W), wc = (int)(pix - (long)h * W);
  float in[27];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ih = h - 1 + kh, iw = wc - 1 + kw;
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        in[(ci * 3 + kh) * 3 + kw] = ok ? x[(long)n * x_bs + ci * HW + (long)ih * W + iw] : 0.f;
      }
  vgb8 o[2];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const int co = cb * 16 + c;
    float a = b[co];
#pragma unroll
    for (int i = 0; i < 27; ++i) a = fmaf(w[co * 27 + i], in[i], a);
    o[c >> 3][c & 7] = (T16)fmaxf(a, 0.f);
  }
  vgb8* dst = reinterpret_cast<vgb8*>(y + cb16(n, cb * 16, h, wc, 64, H, W));
  dst[0] = o[0];
  dst[1] = o[1];
}

// conv1_1 data-grad: dx[n][ci][h][w] = sum_{co,kh,kw} w[co][ci][kh][kw] * d[n][co][h+1-kh][w+1-kw],
// d = CB16 bf16 [N][64][H][W] (the grad at conv1_1's pre-activation), dx NCHW fp32.  Thread = pixel.
template <typename T16>
__global__ __launch_bounds__(256) void vgg_conv1_dgrad_kernel(const T16* __restrict__ d, const float* __restrict__ w,
                                                              float* __restrict__ dx, long dx_bs, int N, int H, int W) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  __shared__ float ws[9 * 64 * 3];   // [tap][co][ci]
  for (int i = threadIdx.x; i < 9 * 64 * 3; i += 256) {
    const int ci = i % 3, co = (i / 3) % 64, tap = i / 192;
    ws[i] = w[(co * 3 + ci) * 9 + tap];
  }
  __syncthreads();
  // XCD-aware row order: consecutive workgroups (neighbouring pixel rows, whose 3x3 windows read the
  // same rows of d) run on one XCD and share its L2 -- dispatch round-robins workgroups over the 8
  // XCDs, which made every row of d come from HBM ~9 times (FETCH_SIZE 1.22 GB for a 134 MB d)
  const long HW = (long)H * W;
  int blk;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    blk = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const long t = blk * 256L + threadIdx.x;
  if (t >= (long)N * HW) return;
  const int n = (int)(t / HW);
  const long pix = t - (long)n * HW;
  const int h = (int)(pix / W), wc = (int)(pix - (long)h * W);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int oh = h + 1 - kh, ow = wc + 1 - kw;
    if ((unsigned)oh >= (unsigned)H || (unsigned)ow >= (unsigned)W) continue;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const vgb8* p = reinterpret_cast<const vgb8*>(d + cb16(n, cb * 16, oh, ow, 64, H, W));
      const vgb8 u0 = p[0], u1 = p[1];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const float g = (float)(c < 8 ? u0[c] : u1[c - 8]);
        const float* wr = ws + (tap * 64 + cb * 16 + c) * 3;
        a0 = fmaf(wr[0], g, a0);
        a1 = fmaf(wr[1], g, a1);
        a2 = fmaf(wr[2], g, a2);
      }
    }
  }
  float* o = dx + (long)n * dx_bs + pix;
  o[0] = a0;
  o[HW] = a1;
  o[2 * HW] = a2;
}

// conv1_1 data-grad, row-sliding form: a thread owns one column and R consecutive output rows and walks
// the R + 2 input rows of d that feed them once each, keeping the three output rows an input row
// touches (kh = 0, 1, 2) in registers.  The 27 weights of one output channel co (w[co][ci][kh][kw], 27
// contiguous floats) are wave-uniform: they come through the scalar cache as SGPR operands of the
// FMAs (the per-pixel kernel spent one LDS read per FMA: 1728 per pixel).
template <typename T16, int R>
__global__ __launch_bounds__(256) void vgg_conv1_dgrad_rows_kernel(const T16* __restrict__ d, const float* __restrict__ w,
                                                                   float* __restrict__ dx, long dx_bs, int N, int H, int W) {
  typedef hx8<T16> vgb8;
  const int wt = (W + 255) / 256, ht = (H + R - 1) / R;
  int b = blockIdx.x;
  const int wb = b % wt;
  b /= wt;
  const int hb = b % ht, n = b / ht;
  const int wc = wb * 256 + threadIdx.x, h0 = hb * R;
  if (wc >= W) return;
  const long HW = (long)H * W;
  float a0[3] = {0.f, 0.f, 0.f}, a1[3] = {0.f, 0.f, 0.f}, a2[3] = {0.f, 0.f, 0.f};   // rows ih-1, ih, ih+1
  float* o = dx + (long)n * dx_bs + wc;
  const bool lv = wc >= 1, rv = wc + 1 < W;   // iw = wc + 1 - kw in range for kw = 2 / kw = 0
  for (int ih = h0 - 1; ih <= h0 + R; ++ih) {
    if (ih >= 0 && ih < H) {
#pragma unroll 1
      for (int cb = 0; cb < 4; ++cb) {
        vgb8 u[3][2];
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int iw = wc + 1 - kw;
          const bool ok = kw == 1 || (kw == 0 ? rv : lv);
          const vgb8* p = reinterpret_cast<const vgb8*>(d + cb16(n, cb * 16, ih, ok ? iw : wc, 64, H, W));
          u[kw][0] = p[0];
          u[kw][1] = p[1];
          if (!ok) { u[kw][0] = vgb8{}; u[kw][1] = vgb8{}; }
        }
        const float* wcb = w + cb * 16 * 27;   // w[co][ci][kh][kw], co = cb * 16 + c
#pragma unroll
        for (int c = 0; c < 16; ++c) {
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const float g = (float)(c < 8 ? u[kw][0][c] : u[kw][1][c - 8]);
#pragma unroll
            for (int ci = 0; ci < 3; ++ci) {
              a0[ci] = fmaf(wcb[c * 27 + ci * 9 + 0 * 3 + kw], g, a0[ci]);   // kh = 0 -> output row ih - 1
              a1[ci] = fmaf(wcb[c * 27 + ci * 9 + 1 * 3 + kw], g, a1[ci]);   // kh = 1 -> row ih
              a2[ci] = fmaf(wcb[c * 27 + ci * 9 + 2 * 3 + kw], g, a2[ci]);   // kh = 2 -> row ih + 1
            }
          }
        }
      }
    }
    const int h = ih - 1;   // complete after input row ih
    if (h >= h0 && h < H) {
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) o[ci * HW + (long)h * W] = a0[ci];
    }
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) { a0[ci] = a1[ci]; a1[ci] = a2[ci]; a2[ci] = 0.f; }
  }
}

// MaxPool2d(2) of an fp32 CB16 feature -> bf16 CB16 + window argmax (dh*2 + dw, first max wins as
// in torch).  Thread = (output pixel, 4 channels).
// L1: also the perceptual L1 of the pooled feature against the real image's feature rf (same CB16
// fp32 layout) from the same read of x: per workgroup sum of |x - rf| over its threads' 2 x 2 x 4
// values (in window order) -> part[blockIdx.x], summed in order by final_sum_kernel.
// codes (L1 form, nullable): per element of x one byte, bit 0 = (x > 0), bit 1 = (x > rf),
// bit 2 = (x < rf) -- all the tap's backward needs of x and rf (cb16_tap_bwd_code_kernel).
template <typename T16, bool L1 = false>
__global__ __launch_bounds__(256) void cb16_maxpool_kernel(const float* __restrict__ x, T16* __restrict__ y,
                                                           unsigned char* __restrict__ idx, int N, int C, int H, int W,
                                                           const float* __restrict__ rf = nullptr,
                                                           float* __restrict__ part = nullptr,
                                                           unsigned char* __restrict__ codes = nullptr) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  const int Ho = H >> 1, Wo = W >> 1;
  const long total = (long)N * (C >> 2) * Ho * Wo;
  long t = blockIdx.x * 256L + threadIdx.x;
  float l1 = 0.f;
  if constexpr (L1) {
    if (t >= total) t = -1;   // (every thread reaches the block sum)
  } else if (t >= total) {
    return;
  }
  if (t >= 0) {
  // t -> (n, cblock, c4 (0..3), oh, ow) with ow fastest after c4 groups of one block
  const int q = (int)(t & 3);                 // 4-channel group inside the 16-channel block
  long r = t >> 2;
  const int ow = (int)(r % Wo); r /= Wo;
  const int oh = (int)(r % Ho); r /= Ho;
  const int cbk = (int)(r % (C >> 4));
  const int n = (int)(r / (C >> 4));
  const int c = cbk * 16 + q * 4;
  float best[4];
  int bi[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int dh = k >> 1, dw = k & 1;
    const long xo = cb16(n, c, 2 * oh + dh, 2 * ow + dw, C, H, W);
    const float4 v = *reinterpret_cast<const float4*>(x + xo);
    const float a[4] = {v.x, v.y, v.z, v.w};
    if constexpr (L1) {
      const float4 u = *reinterpret_cast<const float4*>(rf + xo);
      l1 += ((fabsf(v.x - u.x) + fabsf(v.y - u.y)) + (fabsf(v.z - u.z) + fabsf(v.w - u.w)));
      if (codes) {
        const float ua[4] = {u.x, u.y, u.z, u.w};
        vgc4 cd;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          cd[e] = (unsigned char)((a[e] > 0.f ? 1 : 0) | (a[e] > ua[e] ? 2 : 0) | (a[e] < ua[e] ? 4 : 0));
        *reinterpret_cast<vgc4*>(codes + xo) = cd;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (k == 0 || a[e] > best[e]) { best[e] = a[e]; bi[e] = k; }
    }
  }
  const long o = cb16(n, c, oh, ow, C, Ho, Wo);
  vgb4 b;
  vgc4 ix;
#pragma unroll
  for (int e = 0; e < 4; ++e) { b[e] = (T16)best[e]; ix[e] = (unsigned char)bi[e]; }
  *reinterpret_cast<vgb4*>(y + o) = b;
  *reinterpret_cast<vgc4*>(idx + o) = ix;
  }
  if constexpr (L1) {
    __shared__ float sh[4];
    const float s = block_sum<256>(l1, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// Gradient at the pre-ReLU output of a tapped conv (f = its fp32 output, r = the real image's):
//   d = (maxpool_bwd(dpool, idx) [dpool != NULL] + gout * coef * sign(f - r)) * (f > 0),  bf16 out.
// Thread = (pooled pixel, 4 channels), covering the 2x2 window.
template <typename T16>
__global__ __launch_bounds__(256) void cb16_tap_bwd_kernel(const T16* __restrict__ dpool,
                                                           const unsigned char* __restrict__ idx,
                                                           const float* __restrict__ f, const float* __restrict__ rr,
                                                           T16* __restrict__ d, int N, int C, int H, int W,
                                                           const float* __restrict__ gout, float coef) {
  typedef hx8<T16> vgb8;
  typedef hx4<T16> vgb4;
  const int Ho = H >> 1, Wo = W >> 1;
  const long total = (long)N * (C >> 2) * Ho * Wo;
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= total) return;
  const int q = (int)(t & 3);
  long r = t >> 2;
  const int ow = (int)(r % Wo); r /= Wo;
  const int oh = (int)(r % Ho); r /= Ho;
  const int cbk = (int)(r % (C >> 4));
  const int n = (int)(r / (C >> 4));
  const int c = cbk * 16 + q * 4;
  const float g = gout[0] * coef;
  float up[4] = {0.f, 0.f, 0.f, 0.f};
  vgc4 ix = {0, 0, 0, 0};
  if (dpool) {
    const long o = cb16(n, c, oh, ow, C, Ho, Wo);
    const vgb4 u = *reinterpret_cast<const vgb4*>(dpool + o);
    ix = *reinterpret_cast<const vgc4*>(idx + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) up[e] = (float)u[e];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int h = 2 * oh + (k >> 1), w = 2 * ow + (k & 1);
    const long o = cb16(n, c, h, w, C, H, W);
    const float4 fv = *reinterpret_cast<const float4*>(f + o);
    const float4 rv = *reinterpret_cast<const float4*>(rr + o);
    const float fa[4] = {fv.x, fv.y, fv.z, fv.w}, ra[4] = {rv.x, rv.y, rv.z, rv.w};
    vgb4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float df = fa[e] - ra[e];
      float v = df > 0.f ? g : (df < 0.f ? -g : 0.f);
      if (dpool && (int)ix[e] == k) v += up[e];
      out[e] = (T16)(fa[e] > 0.f ? v : 0.f);
    }
    *reinterpret_cast<vgb4*>(d + o) = out;
  }
}

// The same gradient from the forward's per-element codes (cb16_maxpool_kernel L1 form) instead of
// f and r: 1 byte per element read instead of 8.  Same values: the codes hold exactly the sign of
// f - r and the ReLU mask f > 0.
template <typename T16>
__global__ __launch_bounds__(256) void cb16_tap_bwd_code_kernel(const T16* __restrict__ dpool,
                                                                const unsigned char* __restrict__ idx,
                                                                const unsigned char* __restrict__ codes,
                                                                T16* __restrict__ d, int N, int C, int H, int W,
                                                                const float* __restrict__ gout, float coef) {
  typedef hx4<T16> vgb4;
  const int Ho = H >> 1, Wo = W >> 1;
  const long total = (long)N * (C >> 2) * Ho * Wo;
  const long t = blockIdx.x * 256L + threadIdx.x;
  if (t >= total) return;
  const int q = (int)(t & 3);
  long r = t >> 2;
  const int ow = (int)(r % Wo); r /= Wo;
  const int oh = (int)(r % Ho); r /= Ho;
  const int cbk = (int)(r % (C >> 4));
  const int n = (int)(r / (C >> 4));
  const int c = cbk * 16 + q * 4;
  const float g = gout[0] * coef;
  const long o = cb16(n, c, oh, ow, C, Ho, Wo);
  const vgb4 u = *reinterpret_cast<const vgb4*>(dpool + o);
  const vgc4 ix = *reinterpret_cast<const vgc4*>(idx + o);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int h = 2 * oh + (k >> 1), w = 2 * ow + (k & 1);
    const long p = cb16(n, c, h, w, C, H, W);
    const vgc4 cd = *reinterpret_cast<const vgc4*>(codes + p);
    vgb4 out;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = (cd[e] & 2) ? g : ((cd[e] & 4) ? -g : 0.f);
      if ((int)ix[e] == k) v += (float)u[e];
      out[e] = (T16)((cd[e] & 1) ? v : 0.f);
    }
    *reinterpret_cast<vgb4*>(d + p) = out;
  }
}

// Planner knob (measurement tools): 0 = the LDS-DMA ring kernel where a launch fills the chip
// (the step's 14 VGG launches 1014 -> 936 us at B = 16, same bits; profiles/r04/vconv_micro.txt),
// 1 = always the register-staged kernel, 3 = the ring with kw-major taps and B row reuse (default:
// 940 -> 924 us, relative difference 2-4e-5 from the tap-order change; profiles/r04/vconv_micro_kwm.txt).  (A 4-wave form, one wave
// per SIMD owning 4 x 4 MFMA tiles -- half the fragment reads per MFMA -- measured 1103 us against
// the 8-wave ring's 957 over the same launches: profiles/r04/vconv_micro_4wave.txt.)
static int g_vc_mode = 3;

template <typename T16, int BM, int TH>
static void vc_launch(VcArgs<T16>& g, hipStream_t st) {
  g.tiles_w = g.W / 32;
  g.tiles_h = g.H / TH;
  const long tiles = (long)g.N * g.tiles_w * g.tiles_h * (g.M / BM);
  hipLaunchKernelGGL((vconv3x3_kernel<T16, BM, TH>), dim3((unsigned)tiles), dim3(256), 0, st, g);
}

// device address of the 16-byte zero block (nullptr if it cannot be resolved: the register-staged
// kernel runs instead)
static const void* vc_zero() {
  static const void* zero = nullptr;
  if (!zero) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_dma_zero16)) == hipSuccess) zero = p;
  }
  return zero;
}

template <typename T16, int BM, int TH>
static void vc_launch_dma(VcArgs<T16>& g, hipStream_t st) {
  g.tiles_w = g.W / 32;
  g.tiles_h = g.H / TH;
  const long tiles = (long)g.N * g.tiles_w * g.tiles_h * (g.M / BM);
  if (g_vc_mode == 3)
    hipLaunchKernelGGL((vconv3x3_dma_kernel<T16, BM, TH, true>), dim3((unsigned)tiles), dim3(512), 0, st, g);
  else
    hipLaunchKernelGGL((vconv3x3_dma_kernel<T16, BM, TH>), dim3((unsigned)tiles), dim3(512), 0, st, g);
}

static int vc_bm(int M) { return (M % 128 == 0) ? 128 : 64; }



}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_vconv_supported(int K, int M, int H, int W) {
  return K > 0 && M > 0 && K % 16 == 0 && M % 64 == 0 && W % 32 == 0 && H % 4 == 0;
}

// planner knob `key` <- val (val < 0: read only), returns the previous value (measurement tools):
// key 0 = kernel form (0 LDS-DMA ring where it fills the chip, 1 register-staged, 3 the ring with
// kw-major taps and B row reuse)
int dsgan_vconv_tune(int key, int val) {
  if (key != 0) return -1;
  const int old = g_vc_mode;
  if (val >= 0) g_vc_mode = val;
  return old;
}

// bf16 elements of the swizzled weights of a Co x Ci 3x3 conv (either mode)
long dsgan_vconv_wtrans_size(int Co, int Ci) { return 9L * Co * Ci; }

int dsgan_vconv_wtrans(const float* W, void* Wt, int Co, int Ci, int dgrad, hipStream_t st) {
  DSG_REQUIRE(W && Wt && Co > 0 && Ci > 0 && Co % 16 == 0 && Ci % 16 == 0, "dsgan_vconv_wtrans: bad args");
  const int M = dgrad ? Ci : Co;
  DSG_REQUIRE(M % 64 == 0, "dsgan_vconv_wtrans: output channels of the GEMM must be a multiple of 64");
  const long total = 9L * Co * Ci;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((vconv_wtrans_kernel<T16>), dim3((unsigned)blocks), dim3(256), 0, st, W, (T16*)Wt, Co, Ci,
                       vc_bm(M), dgrad);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// Y (CB16, bf16 or fp32) = [relu](conv3x3(X, W) + bias) [* (mask > 0)]; Wt from dsgan_vconv_wtrans
// (dgrad = 1 turns the same kernel into the data-grad of a conv whose weights were transformed so).
int dsgan_vconv3x3(const void* X, const void* Wt, const float* bias, const void* mask, void* Y, int y_f32, int relu,
                   int N, int K, int M, int H, int W, hipStream_t st) {
  DSG_REQUIRE(X && Wt && Y && N > 0, "dsgan_vconv3x3: bad args");
  DSG_REQUIRE(dsgan_vconv_supported(K, M, H, W), "dsgan_vconv3x3: unsupported K=%d M=%d H=%d W=%d", K, M, H, W);
  DSG_REQUIRE((((uintptr_t)X | (uintptr_t)Wt | (uintptr_t)Y | (uintptr_t)bias | (uintptr_t)mask) & 15) == 0,
              "dsgan_vconv3x3: 16-byte aligned operands required");
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    VcArgs<T16> g{};
    g.X = (const T16*)X; g.Wt = (const T16*)Wt; g.bias = bias; g.mask = (const T16*)mask; g.Y = Y;
    g.N = N; g.K = K; g.M = M; g.H = H; g.W = W; g.relu = relu; g.y_f32 = y_f32;
    const int BM = vc_bm(M);
    // LDS-DMA ring kernel (one 8-wave workgroup per CU): 16-row pixel tiles where they still give a
    // workgroup per CU, else 8-row ones
    const long pt16 = H % 16 == 0 ? (long)N * (W / 32) * (H / 16) * (M / BM) : 0;
    const long pt8 = H % 8 == 0 ? (long)N * (W / 32) * (H / 8) * (M / BM) : 0;
    g.zero = g_vc_mode != 1 && (pt16 >= 256 || pt8 >= 256) ? vc_zero() : nullptr;
    if (g.zero) {
      if (BM == 128) {
        if (pt16 >= 256) vc_launch_dma<T16, 128, 16>(g, st); else vc_launch_dma<T16, 128, 8>(g, st);
      } else {
        if (pt16 >= 256) vc_launch_dma<T16, 64, 16>(g, st); else vc_launch_dma<T16, 64, 8>(g, st);
      }
      return;
    }
    // 8-row pixel tiles unless that leaves fewer than two workgroups per CU
    const bool th8 = H % 8 == 0 && (long)N * (W / 32) * (H / 8) * (M / BM) >= 512;
    if (BM == 128) {
      if (th8) vc_launch<T16, 128, 8>(g, st); else vc_launch<T16, 128, 4>(g, st);
    } else {
      if (th8) vc_launch<T16, 64, 8>(g, st); else vc_launch<T16, 64, 4>(g, st);
    }
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// conv1_1: x NCHW fp32 [N][3][H][W] (batch stride x_bs) -> y CB16 bf16 [N][64][H][W], relu
int dsgan_vgg_conv1_fwd(const float* x, long x_bs, const float* w, const float* b, void* y, int N, int H, int W,
                        hipStream_t st) {
  DSG_REQUIRE(x && w && b && y && N > 0 && H > 0 && W > 0 && (((uintptr_t)y) & 15) == 0, "dsgan_vgg_conv1_fwd: bad args");
  const long total = (long)N * 4 * H * W;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    if ((H * W) % 64 == 0)
      hipLaunchKernelGGL((vgg_conv1_fwd_kernel<T16, true>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x,
                         x_bs, w, b, (T16*)y, N, H, W);
    else
      hipLaunchKernelGGL((vgg_conv1_fwd_kernel<T16, false>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x,
                         x_bs, w, b, (T16*)y, N, H, W);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// conv1_1 data-grad: d CB16 bf16 [N][64][H][W] -> dx NCHW fp32 [N][3][H][W] (batch stride dx_bs)
int dsgan_vgg_conv1_dgrad(const void* d, const float* w, float* dx, long dx_bs, int N, int H, int W, hipStream_t st) {
  DSG_REQUIRE(d && w && dx && N > 0 && (((uintptr_t)d) & 15) == 0, "dsgan_vgg_conv1_dgrad: bad args");
  const long total = (long)N * H * W;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    constexpr int R = 4;
    const long blocks = (long)N * ((H + R - 1) / R) * ((W + 255) / 256);
    hipLaunchKernelGGL((vgg_conv1_dgrad_rows_kernel<T16, R>), dim3((unsigned)blocks), dim3(256), 0, st, (const T16*)d, w,
                       dx, dx_bs, N, H, W);
    (void)total;
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// MaxPool2d(2): x fp32 CB16 [N][C][H][W] -> y bf16 CB16 [N][C][H/2][W/2], idx u8 (same indexing)
int dsgan_cb16_maxpool(const float* x, void* y, void* idx, int N, int C, int H, int W, hipStream_t st) {
  DSG_REQUIRE(x && y && idx && C % 16 == 0 && H % 2 == 0 && W % 2 == 0, "dsgan_cb16_maxpool: bad args");
  const long total = (long)N * (C / 4) * (H / 2) * (W / 2);
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((cb16_maxpool_kernel<T16>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x,
                       (T16*)y, (unsigned char*)idx, N, C, H, W);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// workgroup partials of dsgan_cb16_maxpool_l1 (floats of its `part` scratch)
long dsgan_cb16_maxpool_l1_parts(int N, int C, int H, int W) {
  return ((long)N * (C / 4) * (H / 2) * (W / 2) + 255) / 256;
}

// dsgan_cb16_maxpool, plus out[0] = mean |x - r| over the whole feature (the perceptual L1 of that
// tap, DSGAN/models/pix2pix_model.py:182-186 over vgg.py's relu features) from the same read of x;
// r = the real image's feature, same CB16 fp32 layout.  Deterministic: workgroup partials summed in
// a fixed order.  codes (nullable, 1 byte per element of x, CB16): what dsgan_cb16_tap_bwd_codes
// needs of x and r.
int dsgan_cb16_maxpool_l1(const float* x, const float* r, void* y, void* idx, void* codes, float* out, float* part,
                          long part_elems, int N, int C, int H, int W, hipStream_t st) {
  DSG_REQUIRE(x && r && y && idx && out && C % 16 == 0 && H % 2 == 0 && W % 2 == 0, "dsgan_cb16_maxpool_l1: bad args");
  const long blocks = dsgan_cb16_maxpool_l1_parts(N, C, H, W);
  DSG_WS(blocks, part, part_elems, "dsgan_cb16_maxpool_l1 (dsgan_cb16_maxpool_l1_parts)");
  DSG_REQUIRE(blocks < (1L << 31), "dsgan_cb16_maxpool_l1: feature too large");
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((cb16_maxpool_kernel<T16, true>), dim3((unsigned)blocks), dim3(256), 0, st, x, (T16*)y,
                       (unsigned char*)idx, N, C, H, W, r, part, (unsigned char*)codes);
  });
  DSG_CHECK_LAUNCH();
  launch_final_sum(part, (int)blocks, 1.f / ((float)N * C * H * W), out, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dsgan_cb16_tap_bwd of a pooled tap from dsgan_cb16_maxpool_l1's codes instead of f and r
int dsgan_cb16_tap_bwd_codes(const void* dpool, const void* idx, const void* codes, void* d, int N, int C, int H, int W,
                             const float* gout, hipStream_t st) {
  DSG_REQUIRE(dpool && idx && codes && d && gout && C % 16 == 0 && H % 2 == 0 && W % 2 == 0,
              "dsgan_cb16_tap_bwd_codes: bad args");
  const long total = (long)N * (C / 4) * (H / 2) * (W / 2);
  const float coef = 1.f / ((float)N * C * H * W);
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((cb16_tap_bwd_code_kernel<T16>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       (const T16*)dpool, (const unsigned char*)idx, (const unsigned char*)codes, (T16*)d, N, C, H, W,
                       gout, coef);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// d (bf16 CB16 [N][C][H][W]) = (maxpool_bwd(dpool, idx) + gout*sign(f - r)/(N*C*H*W)) * (f > 0);
// dpool/idx [N][C][H/2][W/2] nullable (the top tapped layer)
int dsgan_cb16_tap_bwd(const void* dpool, const void* idx, const float* f, const float* r, void* d, int N, int C,
                       int H, int W, const float* gout, hipStream_t st) {
  DSG_REQUIRE(f && r && d && gout && C % 16 == 0 && H % 2 == 0 && W % 2 == 0 && (!dpool || idx),
              "dsgan_cb16_tap_bwd: bad args");
  const long total = (long)N * (C / 4) * (H / 2) * (W / 2);
  const float coef = 1.f / ((float)N * C * H * W);
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    hipLaunchKernelGGL((cb16_tap_bwd_kernel<T16>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       (const T16*)dpool, (const unsigned char*)idx, f, r, (T16*)d, N, C, H, W, gout, coef);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
