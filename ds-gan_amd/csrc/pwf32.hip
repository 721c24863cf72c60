// Exact-fp32 pointwise (1x1, stride 1) convolution GEMMs on v_mfma_f32_32x32x2_f32 (gfx950).
//
// Serves the contractions the build runs with fp32 operands: the 1x1 conv inside every MidMLKA
// (DSGAN/models/model/MixConvNeXtML.py:85,112 -- pinned to fp32 because it feeds an
// InstanceNorm whose input variance is far below eps at the reference init) and,
// in --precision fp32 (the parity mode), every 1x1 conv / nn.Linear.  The f32 MFMA runs at the
// f32 vector rate (1/16 of bf16), so these GEMMs are about balanced between MFMA and HBM; the
// kernel streams fp32 operand tiles through LDS (no conversion) with register prefetch of the
// next K step, one barrier per step, and the same modes / epilogues as pwgemm.hip:
//   FWD  : Y[b][m][p]  = act( sum_k W[m][k] X[b][k][p] + bias[m] ) (+Y)
//   DGRAD: DX[b][m][p] = ( sum_k W[k][m] DY[b][k][p] ) * gact'(G[b][m][p])        (+DX)
//   WGRAD: DW[m][n]   += sum_{b,p} DY[b][m][p] X[b][n][p]   (pixel splits -> partials in ws,
//          reduced in a fixed order by launch_split_reduce: deterministic)
#include "common.h"

namespace dsg {

typedef __attribute__((ext_vector_type(16))) float pff32x16;

enum PfMode : int { PF_FWD = 0, PF_DGRAD = 1, PF_WGRAD = 2 };

struct PfArgs {
  const float* A; long a_bs;   // FWD: W[M][K]  DGRAD: W[K][M]  WGRAD: DY[b][M][P]
  const float* B; long b_bs;   // FWD/DGRAD: X/DY [b][K][P]     WGRAD: X[b][N][P]
  float* Y; long y_bs;
  const float* bias;
  const float* gpre; long gpre_bs;
  int M, N, K, P;
  int act, gact, accumulate; float slope;
  int k_split;
  float* ws;
  unsigned a_range, b_range;   // buffer-resource byte ranges (B: per image for FWD/DGRAD)
  float* asum;                 // WGRAD (nullable): the bias grad asum[m] += sum_k DY[m][k], from the staged
                               // A tiles (split partials after the S*M*N weight partials)
};

constexpr int FBK = 16;           // K per main-loop step (8 MFMA k-pairs)
constexpr int FRM = FBK + 1;      // row-major LDS row stride: conflict-free column reads

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256, 2) void pwf32_kernel(PfArgs g) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr bool A_KMAJ = MODE == PF_DGRAD, B_KMAJ = MODE != PF_WGRAD;
  constexpr int A_STR = A_KMAJ ? BM + 4 : FRM;
  constexpr int B_STR = B_KMAJ ? BN + 4 : FRM;
  constexpr int A_SZ = A_KMAJ ? FBK * A_STR : BM * A_STR;
  constexpr int B_SZ = B_KMAJ ? FBK * B_STR : BN * B_STR;
  constexpr int A_ITEMS = BM * FBK / 4 / 256, B_ITEMS = BN * FBK / 4 / 256;   // float4 items per thread
  __shared__ float smem[2 * (A_SZ + B_SZ)];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  const int mt = (g.M + BM - 1) / BM;
  const int nt = (MODE == PF_WGRAD) ? (g.N + BN - 1) / BN : g.N / BN;
  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int m_t = tile % mt, rest = tile / mt;
  const int n_t = rest % nt, split = rest / nt;
  const int m0 = m_t * BM, n0 = n_t * BN;
  int kbeg = 0, kend = g.K;
  if (MODE == PF_WGRAD) { kbeg = split * g.k_split; kend = min(g.K, kbeg + g.k_split); }
  const int nk = (kend - kbeg + FBK - 1) / FBK;
  const int bimg = (MODE == PF_WGRAD) ? 0 : n0 / g.P;
  const int p0 = (MODE == PF_WGRAD) ? 0 : n0 - bimg * g.P;

  // Operand loads are 16-byte buffer loads; an element outside its tensor gets an offset past
  // the resource range and reads 0 in hardware (no branch, no select -- see pwgemm.hip).
  constexpr unsigned OOB = 0xFFFFFFF0u;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, g.a_range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(g.B + (MODE == PF_WGRAD ? 0L : (long)bimg * g.b_bs)), (short)0, g.b_range, 0x00020000);
  auto bld = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  };
  float4 ra[A_ITEMS], rb[B_ITEMS];
  float asr[A_ITEMS];   // WGRAD asum: this thread's running row sums of its A items (fixed order)
#pragma unroll
  for (int i = 0; i < A_ITEMS; ++i) asr[i] = 0.f;
  auto gload = [&](int kt) {
    const int kb = kbeg + kt * FBK;
    // WGRAD: a 16-pixel K step lies inside one image (P % 16 == 0)
    const unsigned bw = (MODE == PF_WGRAD) ? (unsigned)(kb / g.P) : 0u;
    const unsigned pw = (MODE == PF_WGRAD) ? (unsigned)(kb - (int)bw * g.P) : 0u;
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256;
      unsigned off;
      if (MODE == PF_FWD) {               // W[M][K]: row m, k = kb + 4q
        const int m = m0 + (it >> 2), k = kb + (it & 3) * 4;
        off = (m < g.M && k < kend) ? ((unsigned)m * g.K + k) * 4u : OOB;
      } else if (MODE == PF_DGRAD) {      // W[K][M]: row k, m = m0 + 4q
        const int k = kb + it / (BM / 4), m = m0 + (it % (BM / 4)) * 4;
        off = (k < kend && m < g.M) ? ((unsigned)k * g.M + m) * 4u : OOB;
      } else {                            // DY[b][M][P]: row m, pixels pw + 4q
        const int m = m0 + (it >> 2);
        off = (m < g.M && kb + (it & 3) * 4 < kend)
                  ? (bw * (unsigned)g.a_bs + (unsigned)m * g.P + pw + (it & 3) * 4) * 4u : OOB;
      }
      ra[i] = bld(rA, off);
    }
#pragma unroll
    for (int i = 0; i < B_ITEMS; ++i) {
      const int it = tid + i * 256;
      unsigned off;
      if (MODE != PF_WGRAD) {             // [K][P] of image bimg: row k, pixels p0 + 4q
        const int k = kb + it / (BN / 4), c = (it % (BN / 4)) * 4;
        off = k < kend ? ((unsigned)k * g.P + p0 + c) * 4u : OOB;
      } else {                            // X[b][N][P]: row n, pixels pw + 4q
        const int n = n0 + (it >> 2);
        off = (n < g.N && kb + (it & 3) * 4 < kend)
                  ? (bw * (unsigned)g.b_bs + (unsigned)n * g.P + pw + (it & 3) * 4) * 4u : OOB;
      }
      rb[i] = bld(rB, off);
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * (A_SZ + B_SZ);
    float* Bs = As + A_SZ;
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * 256;
      if (A_KMAJ) {
        *reinterpret_cast<float4*>(As + (it / (BM / 4)) * A_STR + (it % (BM / 4)) * 4) = ra[i];
      } else {
        float* d = As + (it >> 2) * A_STR + (it & 3) * 4;
        d[0] = ra[i].x; d[1] = ra[i].y; d[2] = ra[i].z; d[3] = ra[i].w;
        if (MODE == PF_WGRAD && g.asum) asr[i] += (ra[i].x + ra[i].y) + (ra[i].z + ra[i].w);
      }
    }
#pragma unroll
    for (int i = 0; i < B_ITEMS; ++i) {
      const int it = tid + i * 256;
      if (B_KMAJ) {
        *reinterpret_cast<float4*>(Bs + (it / (BN / 4)) * B_STR + (it % (BN / 4)) * 4) = rb[i];
      } else {
        float* d = Bs + (it >> 2) * B_STR + (it & 3) * 4;
        d[0] = rb[i].x; d[1] = rb[i].y; d[2] = rb[i].z; d[3] = rb[i].w;
      }
    }
  };

  pff32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const float* As = smem + buf * (A_SZ + B_SZ);
    const float* Bs = As + A_SZ;
#pragma unroll
    for (int kk = 0; kk < FBK / 2; ++kk) {
      const int k = 2 * kk + lh;
      float af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = wm * TM * 32 + i * 32 + lr;
        af[i] = A_KMAJ ? As[k * A_STR + m] : As[m * A_STR + k];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wn * TN * 32 + j * 32 + lr;
        bfr[j] = B_KMAJ ? Bs[k * B_STR + n] : Bs[n * B_STR + k];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C layout col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) ----
  if (MODE == PF_WGRAD) {
    if (g.asum) {
      // a row's 4 items (16 pixels) are adjacent lanes: butterfly over them; the n-tile-0 workgroup
      // writes (its split's partial, or asum += when unsplit)
#pragma unroll
      for (int i = 0; i < A_ITEMS; ++i) {
        float t = asr[i];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        const int it = tid + i * 256, m = m0 + (it >> 2);
        if (n_t == 0 && (it & 3) == 0 && m < g.M) {
          if (g.ws) g.ws[(long)gridDim.x / mt / nt * g.M * g.N + (long)split * g.M + m] = t;
          else g.asum[m] += t;
        }
      }
    }
    float* dst = g.ws ? g.ws + (long)split * g.M * g.N : g.Y;   // one split: the only writer, +=
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * TN * 32 + j * 32 + lr;
      if (n >= g.N) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (m < g.M) {
            float* o = dst + (long)m * g.N + n;
            *o = g.ws ? acc[i][j][r] : *o + acc[i][j][r];
          }
        }
    }
    return;
  }
  float* yb = g.Y + (long)bimg * g.y_bs + p0;
  const float* gb = g.gpre ? g.gpre + (long)bimg * g.gpre_bs + p0 : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * TN * 32 + j * 32 + lr;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float v[16];
      int mrow[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        mrow[r] = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        v[r] = acc[i][j][r];
      }
      if (MODE == PF_FWD && g.bias) {
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] += mrow[r] < g.M ? g.bias[mrow[r]] : 0.f;
      }
      if (gb) {
        float gv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) gv[r] = mrow[r] < g.M ? gb[(long)mrow[r] * g.P + col] : 0.f;
        act_g_mul_arr(g.gact, v, gv, g.slope);
      }
      act_f_arr(g.act, v, g.slope);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (mrow[r] < g.M) {
          float* o = yb + (long)mrow[r] * g.P + col;
          *o = g.accumulate ? *o + v[r] : v[r];
        }
      }
    }
  }
}

template <int MODE, int BM, int BN = 128>
static void pf_launch(const PfArgs& g, int splits, hipStream_t st) {
  const int mt = (g.M + BM - 1) / BM;
  const int nt = (MODE == PF_WGRAD) ? (g.N + BN - 1) / BN : g.N / BN;
  hipLaunchKernelGGL((pwf32_kernel<MODE, BM, BN>), dim3((unsigned)((long)mt * nt * splits)), dim3(256), 0, st, g);
}

// FWD / DGRAD tile: 128 x 128 while that gives >= 1024 workgroups, else smaller tiles (the f32
// MFMA is 16x slower than bf16, so a small GEMM needs the parallelism more than the reuse)
template <int MODE>
static void pf_launch_fd(const PfArgs& g, hipStream_t st) {
  const long n128 = g.N / 128;
  if (g.M > 64 && (long)((g.M + 127) / 128) * n128 >= 1024) pf_launch<MODE, 128, 128>(g, 1, st);
  else if ((long)((g.M + 63) / 64) * n128 >= 512 || g.P % 64) pf_launch<MODE, 64, 128>(g, 1, st);
  else pf_launch<MODE, 64, 64>(g, 1, st);
}

// Weight-grad tile and pixel split: 64 x 64 tiles when both sides have <= 64 channels (the MidMLKA(32)
// / (64) 1x1s: a 64 x 128 tile over a 32 x 32 weight was 7/8 idle MFMA work), else 128 (64) x 128;
// ~640 workgroups of >= 4 K steps each.  The f32 MFMA runs at 1/16 of the bf16 rate, so these
// launches are MFMA-bound and the fp32 partials are cheap next to them: the partial bytes may exceed
// a quarter of the operand bytes up to a floor of ~512 workgroups (the 256 x 256 weight at 16^2:
// 8 -> 64 splits, 50 -> ~10 us; 128 x 128 at 32^2: 64 -> 256 splits).
static int pf_wgrad_bn(int M, int N) { return M <= 64 && N <= 64 ? 64 : 128; }
static int pf_wgrad_plan(int M, int N, long K, int* k_split) {
  const int BM = M > 64 ? 128 : 64, BN = pf_wgrad_bn(M, N);
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  long splits = (640 + tiles - 1) / tiles;
  const long max_splits = (K + 4L * FBK - 1) / (4L * FBK);
  long byte_cap = ((long)(M + N) * K) / (4L * M * N);
  const long floor_splits = (512 + tiles - 1) / tiles;
  if (byte_cap < floor_splits) byte_cap = floor_splits;
  if (splits > max_splits) splits = max_splits;
  if (splits > byte_cap) splits = byte_cap;
  if (splits < 1) splits = 1;
  long ks = (K + splits - 1) / splits;
  ks = (ks + FBK - 1) / FBK * FBK;
  splits = (K + ks - 1) / ks;
  *k_split = (int)ks;
  return (int)splits;
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Fast-path eligibility: FWD/DGRAD need P % 128 == 0, WGRAD P % 16 == 0; K, M % 4 == 0 for the
// float4 rows; 16-byte aligned operands and batch strides % 4 == 0.
int dsgan_pw_f32_supported(int mode, int M, int K, int P, long a_bs, long b_bs, const void* a, const void* b) {
  if ((((uintptr_t)a | (uintptr_t)b) & 15) || (a_bs & 3) || (b_bs & 3) || M < 16) return 0;
  if (mode == PF_WGRAD) return (P % 16) == 0;
  return (P % 128) == 0 && (K & 3) == 0 && (M & 3) == 0;
}

long dsgan_pw_f32_wgrad_workspace(int M, int N, int P, int nb) {
  int ks;
  const int splits = pf_wgrad_plan(M, N, (long)nb * P, &ks);
  return splits > 1 ? (long)splits * ((long)M * N + M) : 0;   // weight partials, then bias-sum partials
}

// Same argument meaning as dsgan_pw_gemm (mode 0 FWD / 1 DGRAD / 2 WGRAD), fp32 operands.
int dsgan_pw_gemm_f32(int mode, const float* A, long a_bs, const float* B, long b_bs, float* Y, long y_bs,
                      const float* bias, const float* gpre, long gpre_bs, int M, int N, int K, int P, int nb, int act,
                      int gact, int accumulate, float slope, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(A && B && Y && M > 0 && N > 0 && K > 0 && P > 0 && nb > 0, "dsgan_pw_gemm_f32: bad args");
  PfArgs g{};
  g.A = A; g.a_bs = a_bs; g.B = B; g.b_bs = b_bs; g.Y = Y; g.y_bs = y_bs; g.bias = bias;
  g.gpre = gpre; g.gpre_bs = gpre_bs; g.act = act; g.gact = gact; g.accumulate = accumulate; g.slope = slope;
  g.P = P;
  const long lim = 0xFFFFFFF0L;
  if (mode == PF_WGRAD) {
    const long ar = ((long)(nb - 1) * a_bs + (long)M * P) * 4, br = ((long)(nb - 1) * b_bs + (long)N * P) * 4;
    DSG_REQUIRE(ar < lim && br < lim, "dsgan_pw_gemm_f32: WGRAD operands exceed the 4 GiB buffer range");
    g.a_range = (unsigned)ar; g.b_range = (unsigned)br;
  } else {
    DSG_REQUIRE((long)M * K * 4 < lim && (long)K * P * 4 < lim, "dsgan_pw_gemm_f32: operand exceeds 4 GiB");
    g.a_range = (unsigned)((long)M * K * 4);
    g.b_range = (unsigned)((long)K * P * 4);
  }
  if (mode == PF_WGRAD) {
    DSG_REQUIRE(dsgan_pw_f32_supported(mode, M, K, P, a_bs, b_bs, A, B), "dsgan_pw_gemm_f32: unsupported WGRAD shape");
    g.M = M; g.N = N; g.K = nb * P;
    const int splits = pf_wgrad_plan(M, N, g.K, &g.k_split);
    g.ws = splits > 1 ? ws : nullptr;
    g.asum = const_cast<float*>(bias);   // WGRAD: bias (nullable) receives the bias grad += sum_k DY
    g.bias = nullptr;
    DSG_WS(splits > 1 ? (long)splits * ((long)M * N + (g.asum ? M : 0)) : 0, ws, ws_elems,
           "dsgan_pw_gemm_f32 (WGRAD; dsgan_pw_f32_wgrad_workspace)");
    if (M > 64) pf_launch<PF_WGRAD, 128>(g, splits, st);
    else if (pf_wgrad_bn(M, N) == 64) pf_launch<PF_WGRAD, 64, 64>(g, splits, st);
    else pf_launch<PF_WGRAD, 64>(g, splits, st);
    if (splits > 1) {
      const float* wsv[2] = {ws, ws + (long)splits * M * N};
      const int sv[2] = {splits, splits};
      const long mv[2] = {(long)M * N, (long)M};
      float* dv[2] = {Y, g.asum};
      launch_split_reduce_multi(g.asum ? 2 : 1, wsv, sv, mv, dv, st);
    }
  } else {
    DSG_REQUIRE(dsgan_pw_f32_supported(mode, M, K, P, a_bs, b_bs, A, B), "dsgan_pw_gemm_f32: unsupported shape");
    g.M = M; g.N = nb * P; g.K = K;
    DSG_WS(0, ws, ws_elems, "dsgan_pw_gemm_f32");
    if (mode == PF_FWD) pf_launch_fd<PF_FWD>(g, st);
    else pf_launch_fd<PF_DGRAD>(g, st);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
