// Pointwise (1x1, stride 1) convolution / nn.Linear-on-NCHW GEMMs on MFMA bf16 (gfx950).
//
// The 1x1 contractions are ~70% of the DS-GAN generator's FLOPs (Block.pwconv1/pwconv2 +
// shortcut, DSGAN/models/model/MixConvNeXtML.py:218-242; downSkip* / OriginMLKA 1x1 convs
// :122-157,334-419).  In NCHW they are plain GEMMs over contiguous pixel rows, so this kernel
// drops the im2col machinery of igemm.hip and is built to keep VALU work per MFMA low:
//   * operands are staged global->LDS as 16-byte float4 loads, converted to bf16 in registers,
//     written as 8-byte LDS stores in the SAME layout they have in HBM (no register transpose);
//   * operands whose contiguous axis is not the MFMA k-axis (pixel-major activations, the W^T
//     of the data-grad) are read with the gfx950 hardware transpose ds_read_b64_tr_b16;
//   * the epilogue uses buffer stores whose row offset is a per-(tile,register) scalar, so an
//     output element costs a conversion-free store and no address VALU; rows past M are
//     dropped by the buffer range check; the bias is folded into the accumulator init.
//
// Modes (P = H*W pixels per image, all tensors NCHW / [out,in] weights, fp32 in HBM):
//   FWD  : Y[b][m][p]  = act( sum_k W[m][k] * xact(X[b][k][p]) + bias[m] ) (+Y)   (ypre = pre-act)
//   DGRAD: DX[b][m][p] = ( sum_k W[k][m] * DY[b][k][p] ) * gact'(G[b][m][p])
//   WGRAD: DW[m][n]   += sum_{b,p} DY[b][m][p] * xact(X[b][n][p])     (split over pixels: each split
//          writes its partial tile to a workspace, pw_wgrad_reduce_kernel adds the splits in a fixed
//          order -- deterministic, and plain stores stream faster than float atomics)
#include "pw_impl.h"

namespace dsg {

// the kernel instantiations live in pw_{fwd,dgrad,wgrad}_{bf16,f16}.hip
PW_EXTERN_LAUNCHERS(__bf16)
PW_EXTERN_LAUNCHERS(_Float16)
template <typename T16>
static void pw_fd_launch(int mode, const PwArgs& g, int bm, int abf, int bbf, int splits, hipStream_t st) {
  if (mode == PW_FWD) pw_fd_launch_m<T16, PW_FWD>(g, bm, abf, bbf, splits, st);
  else pw_fd_launch_m<T16, PW_DGRAD>(g, bm, abf, bbf, splits, st);
}

// Planner knobs, read by the host launchers only (tools/pw_bench.py flips them for in-process A/B):
//   [0] FWD/DGRAD split-K on/off, [1] its target workgroup count, [2] split only launches of fewer
//   tiles than this, [3] minimum K steps per split, [4] / [5] retired (64-deep K steps for the 128 /
//   64-row tiles: +1 % / neutral over the step's shapes, profiles/r04/pw_bench_knobs.txt; the variants
//   are gone, the keys are ignored), [6] gelu-pair forward tile (0 built-in,
//   1 256 x 128, 2 128 x 128, 3 wide 256 x 256), [7] gp-multiplied data-grad tile (same codes),
//   [8] gp loaded before the K loop (16-bit gp data-grads on 128 / 64-row tiles), [9] the LDS-DMA
//   ring form of the wide 16-bit-operand launches (pw_impl.h NS > 0): 1 = 256 x 256 tiles, 4 stages,
//   FWD / DGRAD only (default: the gelu-pair forwards 271 -> 262 and 203 -> 186 us, the data-grads
//   155 -> 149 and 138 -> 131 us, same bits; profiles/r04/pw_bench_dma.txt); 3 = the same plus the
//   weight-grads (3-5 % slower there); 2 = 256 x 128 tiles, 3 stages, two workgroups per CU (slower:
//   392 us for the 512-channel gelu-pair forward); 0 = register-staged everywhere.
//   [10] measurement builds only (build_lib.py --measure, DSG_MEASURE; ignored otherwise): bit 0 =
//   FWD / DGRAD epilogues drop their output stores (prices the writes), bit 1 = the gelu-pair
//   epilogue skips its GELU arithmetic (prices the VALU).  [11] retired: the persistent forms of the
//   gelu-pair forward (round 5, one wave per SIMD: 1.8x slower) and of the whole 8-wave LDS-DMA ring
//   (round 6: bitwise equal, 259.6 vs 267.9 us on the 512 -> 2048 gelu-pair forward, +3 % on the
//   1024 -> 4096 one, the step's pointwise launches 2958 vs 2960 us) and the ring's two wave groups
//   staggered by half a K step (bitwise equal, the wide launches within +-1 %) were measured and
//   removed.
static int g_tune[12] = {1, 512, 256, 4, 0, 0, 0, 0, 1, 1, 0, 0};

// the LDS-DMA ring form's conditions (full 256 x 256 tiles, 32-deep K steps, 16-byte pieces)
static int dma_ok(const PwArgs& g, int bm, int abf, int bbf, int mode) {
  if (!g_tune[9] || bm != PW_WIDE || !abf || !bbf) return 0;
  if (!al16(g.A) || !al16(g.B) || (g.a_bs & 7) || (g.b_bs & 7) || g.M % 256) return 0;
  // (the weight-grads stay register-staged unless asked for: 3-5 % slower on the ring)
  const bool ok = mode == PW_WGRAD ? g_tune[9] >= 3 && g.N % 256 == 0 && g.P % 32 == 0 && (g.k_split % 32) == 0
                                   : g.K % 32 == 0 && g.P % 256 == 0 && g.k_split == 0;
  if (!ok) return 0;
  return g_tune[9] == 2 ? 2 : 1;
}

// tile choice with the knob overrides of the two epilogue-heavy forms
static int fd_tile_k(const PwArgs& g, bool any_bf16) {
  const int bm = fd_tile(g, any_bf16);
  const bool gelu_pair = g.ypre && g.gbf, gp_dgrad = g.gpre && g.gbf;
  const int k = gelu_pair ? g_tune[6] : gp_dgrad ? g_tune[7] : 0;
  if (k == 0 || !any_bf16) return bm;
  if (k == 3 && use_wide(g)) return PW_WIDE;
  if (k == 1 && g.M % 256 == 0) return 256;
  return g.M > 64 ? 128 : 64;
}

// K split of an under-filled FWD / DGRAD launch (the 16^2 bottleneck layers: e.g. the downSkip 1x1
// data-grads, 32-128 tiles of 32-64 K steps each, ~40 us at 0.5 TB/s): about g_tune[1] workgroups,
// >= g_tune[3] K steps per split; partials [split][b][M][P] in ws, pw_split_finish_kernel adds them
// in split order and applies the epilogue (deterministic).  128 / 64-row tiles only (the wide and
// 256-row forms are chosen only for launches that fill the chip).
static int fd_splits(const PwArgs& g, int bm, int bk, int* k_split) {
  *k_split = 0;
  if (!g_tune[0] || bm == PW_WIDE || bm == 256) return 1;
  const long tiles = (long)((g.M + bm - 1) / bm) * (g.N / 128);
  if (tiles >= g_tune[2]) return 1;
  const int nkb = (g.K + bk - 1) / bk;
  long S = (g_tune[1] + tiles - 1) / tiles;
  if (S > nkb / g_tune[3]) S = nkb / g_tune[3];
  if (S < 2) return 1;
  const int kc = (int)((nkb + S - 1) / S);
  *k_split = kc * bk;
  return (nkb + kc - 1) / kc;
}
// the finishing pass moves 16-byte fp32 / 8-byte 16-bit groups of 4 pixels
static bool fd_split_ok(const PwArgs& g) {
  auto a16 = [](const void* p, long bs) { return !p || ((((uintptr_t)p) & 15) == 0 && (bs & 3) == 0); };
  return a16(g.Y, g.y_bs) && a16(g.ypre, g.ypre_bs) && a16(g.gpre, g.gpre_bs);
}

// The split plan of a FWD / DGRAD launch on tile bm (ws: the caller's scratch, NULL = never split):
// sets g.k_split / g.ws / the K-step variant and returns the split count.
static int fd_plan(PwArgs& g, int bm, float* ws) {
  int splits = 1;
  g.k_split = 0;
  g.ws = nullptr;
  g.gp_pref = g_tune[8];
#ifdef DSG_MEASURE
  g.dbg = g_tune[10];
#endif
  if (ws && fd_split_ok(g)) {
    splits = fd_splits(g, bm, PBK, &g.k_split);
    if (splits > 1) g.ws = ws;
    else g.k_split = 0;
  }
  return splits;
}
// scratch that plan writes: partials [split][b][M][P]
static long fd_need(const PwArgs& g, int splits) { return splits > 1 ? (long)splits * g.M * g.N : 0; }
static void fd_launch(int mode, const PwArgs& g0, int bm, int abf, int bbf, int splits, hipStream_t st) {
  PwArgs g = g0;
  g.dma = dma_ok(g, bm, abf, bbf, mode);
  if (half_type() == HALF_F16) pw_fd_launch<_Float16>(mode, g, bm, abf, bbf, splits, st);
  else pw_fd_launch<__bf16>(mode, g, bm, abf, bbf, splits, st);
}
static void wg_dispatch(const PwArgs& g0, int bm, int abf, int bbf, int splits, hipStream_t st) {
  PwArgs g = g0;
  g.dma = dma_ok(g, bm, abf, bbf, PW_WGRAD);
  if (half_type() == HALF_F16) pw_wgrad_launch<_Float16>(g, bm, abf, bbf, splits, st);
  else pw_wgrad_launch<__bf16>(g, bm, abf, bbf, splits, st);
}

// (the split reductions: split_reduce.hip)

static int wgrad_cfg_k(PwArgs& g, bool any_bf16, int* bm) { return wgrad_cfg(g, any_bf16, bm); }

// scratch a weight-grad plan writes: weight partials [split][M][N], then bias-sum partials [split][M]
static long wgrad_need(const PwArgs& g, int splits) {
  return splits > 1 ? (long)splits * ((long)g.M * g.N + (g.asum ? g.M : 0)) : 0;
}

static void wgrad_finish(const PwArgs& g, int splits, hipStream_t st) {
  if (splits > 1) {
    // the weight and bias-sum partials in one launch
    const float* wsv[2] = {g.ws, g.ws + (long)splits * g.M * g.N};
    const int sv[2] = {splits, splits};
    const long mv[2] = {(long)g.M * g.N, (long)g.M};
    float* dv[2] = {g.Y, g.asum};
    launch_split_reduce_multi(g.asum ? 2 : 1, wsv, sv, mv, dv, st);
  }
}

}  // namespace dsg

using namespace dsg;

// Fast-path eligibility (else the caller uses the generic implicit-GEMM kernel):
//   FWD/DGRAD: P % 128 == 0, K % 4 == 0 (and M % 4 == 0 for DGRAD), 16-byte aligned operands.
//   WGRAD:     P % 32 == 0, 16-byte aligned operands.
extern "C" int dsgan_pw_supported(int mode, int M, int K, int P, long a_bs, long b_bs, const void* a,
                                  const void* b) {
  if (!al16(a) || !al16(b) || (a_bs & 3) || (b_bs & 3) || M < 16) return 0;
  if (mode == PW_WGRAD) return (P % 32) == 0;
  if (P % 128 != 0 || (K & 3)) return 0;
  if (mode == PW_DGRAD && (M & 3)) return 0;
  return 1;
}

// mode FWD:   A=W[M][K], B=X[b][K][P] (b_bs), Y[b][M][P]
// mode DGRAD: A=W[K][M], B=DY[b][K][P], Y=DX[b][M][P], gpre/gact epilogue
// mode WGRAD: A=DY[b][M][P] (a_bs), B=X[b][N][P] (b_bs), Y=DW[M][N] (+=), nb images
extern "C" int dsgan_pw_gemm(int mode, const float* A, long a_bs, const float* B, long b_bs,
                             float* Y, long y_bs, const float* bias, float* ypre, long ypre_bs,
                             const float* gpre, long gpre_bs, int M, int N, int K, int P, int nb,
                             int act, int gact, int bact, int accumulate, float slope, float* ws,
                             long ws_elems, hipStream_t st) {
  DSG_REQUIRE(A && B && Y && M > 0 && N > 0 && K > 0 && P > 0 && nb > 0, "dsgan_pw_gemm: bad args");
  PwArgs g{};
  g.A = A; g.a_bs = a_bs; g.B = B; g.b_bs = b_bs; g.Y = Y; g.y_bs = y_bs; g.bias = bias;
  g.ypre = ypre; g.ypre_bs = ypre_bs; g.gpre = gpre; g.gpre_bs = gpre_bs;
  g.act = act; g.gact = gact; g.bact = bact; g.accumulate = accumulate; g.slope = slope;
  g.P = P;
  const long lim = (long)PW_OOB;
  if (mode == PW_WGRAD) {
    const long ar = ((long)(nb - 1) * a_bs + (long)M * P) * 4, br = ((long)(nb - 1) * b_bs + (long)N * P) * 4;
    DSG_REQUIRE(ar < lim && br < lim, "dsgan_pw_gemm: WGRAD operands exceed 4 GiB buffer range");
    g.a_range = (unsigned)ar; g.b_range = (unsigned)br;
    DSG_REQUIRE(dsgan_pw_supported(mode, M, K, P, a_bs, b_bs, A, B), "dsgan_pw_gemm: unsupported WGRAD shape");
    g.M = M; g.N = N; g.K = nb * P;
    int bm;
    const int splits = wgrad_cfg_k(g, false, &bm);
    g.ws = splits > 1 ? ws : nullptr;
    g.asum = const_cast<float*>(bias);   // WGRAD: bias (nullable) receives the bias grad += sum_k A
    g.bias = nullptr;
    DSG_WS(wgrad_need(g, splits), ws, ws_elems, "dsgan_pw_gemm (WGRAD; dsgan_pw_wgrad_workspace)");
    wg_dispatch(g, bm, 0, 0, splits, st);
    wgrad_finish(g, splits, st);
  } else {
    DSG_REQUIRE(dsgan_pw_supported(mode, M, K, P, a_bs, b_bs, A, B), "dsgan_pw_gemm: unsupported shape");
    DSG_REQUIRE((long)M * P * 4 < (1L << 32), "dsgan_pw_gemm: M*P too large for a buffer resource");
    g.M = M; g.N = nb * P; g.K = K;
    DSG_REQUIRE((long)K * P * 4 < lim && (long)M * K * 4 < lim, "dsgan_pw_gemm: operand exceeds 4 GiB buffer range");
    g.a_range = (unsigned)((long)M * K * 4);
    g.b_range = (unsigned)((long)K * P * 4);
    const int bm = fd_tile(g, false);
    const int splits = fd_plan(g, bm, ws);   // ws: dsgan_pw_fd_workspace (NULL: never split)
    DSG_WS(fd_need(g, splits), ws, ws_elems, "dsgan_pw_gemm (dsgan_pw_fd_workspace)");
    fd_launch(mode, g, bm, 0, 0, splits, st);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

// Forward with bf16 activations in and/or out (the unfused MLP blocks): Y[b][M][P] (+)=
// act(W X + bias), X fp32 or bf16 (x_bf16), Y fp32 or bf16 (y_bf16; accumulate needs fp32 Y);
// ypre (nullable): fp32 pre-activation, or (ypre_grad_bf16) bf16 act'(pre) for the backward.
// P % 128 == 0, K % 8 == 0, 16-byte aligned.
extern "C" int dsgan_pw_fwd_io_ws(const void* W, int w_bf16, const void* X, long x_bs, int x_bf16, void* Y, long y_bs,
                                  int y_bf16, const void* ypre, long ypre_bs, int ypre_grad_bf16, const float* bias, int M,
                                  int K, int P, int nb, int act, int accumulate, float slope, float* ws, long ws_elems,
                                  hipStream_t st) {
  DSG_REQUIRE(W && X && Y && M >= 16 && K > 0 && P > 0 && nb > 0, "dsgan_pw_fwd_io: bad args");
  DSG_REQUIRE(P % 128 == 0 && K % 8 == 0 && al16(W) && al16(X) && al16(Y) && (x_bs & 7) == 0 && (y_bs & 7) == 0 &&
                  !(y_bf16 && accumulate),
              "dsgan_pw_fwd_io: unsupported shape/alignment");
  DSG_REQUIRE((long)M * P * 4 < (1L << 32) && (long)K * P * 4 < (long)PW_OOB && (long)M * K * 4 < (long)PW_OOB,
              "dsgan_pw_fwd_io: operand exceeds the 4 GiB buffer range");
  PwArgs g{};
  g.A = (const float*)W; g.a_bs = 0; g.B = (const float*)X; g.b_bs = x_bs; g.Y = (float*)Y; g.y_bs = y_bs; g.bias = bias;
  g.ypre = (float*)ypre; g.ypre_bs = ypre_bs; g.gbf = ypre_grad_bf16; g.act = act; g.accumulate = accumulate;
  g.slope = slope; g.y_bf16 = y_bf16;
  g.P = P; g.M = M; g.N = nb * P; g.K = K;
  g.a_range = (unsigned)((long)M * K * (w_bf16 ? 2 : 4));
  g.b_range = (unsigned)((long)K * P * (x_bf16 ? 2 : 4));
  const int bm = fd_tile_k(g, w_bf16 || x_bf16);
  const int splits = fd_plan(g, bm, ws);
  DSG_WS(fd_need(g, splits), ws, ws_elems, "dsgan_pw_fwd_io (dsgan_pw_fd_workspace)");
  fd_launch(PW_FWD, g, bm, w_bf16, x_bf16, splits, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

extern "C" int dsgan_pw_fwd_io(const void* W, int w_bf16, const void* X, long x_bs, int x_bf16, void* Y, long y_bs,
                               int y_bf16, const void* ypre, long ypre_bs, int ypre_grad_bf16, const float* bias, int M,
                               int K, int P, int nb, int act, int accumulate, float slope, hipStream_t st) {
  return dsgan_pw_fwd_io_ws(W, w_bf16, X, x_bs, x_bf16, Y, y_bs, y_bf16, ypre, ypre_bs, ypre_grad_bf16, bias, M, K, P, nb,
                            act, accumulate, slope, nullptr, 0, st);
}

// Data-grad with bf16 operands/outputs (the unfused MLP blocks' backward):
//   DX[b][M][p] (+)= (sum_k W[k][M] DY[b][k][p]) (* GP[b][M][p])
// DY fp32 or bf16 (dy_bf16), DX fp32 or bf16 (dx_bf16; accumulate needs fp32), GP (nullable) the bf16
// act'(pre) written by dsgan_pw_fwd_io (ypre_grad_bf16).  P % 128 == 0, 16-byte aligned.
extern "C" int dsgan_pw_dgrad_io_ws(const void* W, int w_bf16, const void* DY, long dy_bs, int dy_bf16, void* DX,
                                    long dx_bs, int dx_bf16, const void* GP, long gp_bs, int M, int K, int P, int nb,
                                    int accumulate, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(W && DY && DX && M > 0 && K > 0 && nb > 0, "dsgan_pw_dgrad_io: bad args");
  DSG_REQUIRE(dsgan_pw_supported(PW_DGRAD, M, K, P, 0, dy_bs, W, DY) && al16(DX) && (dy_bs & 7) == 0 &&
                  (dx_bs & 7) == 0 && (!GP || (al16(GP) && (gp_bs & 7) == 0)) && !(dx_bf16 && accumulate),
              "dsgan_pw_dgrad_io: unsupported shape/alignment");
  DSG_REQUIRE((long)M * P * 4 < (1L << 32) && (long)K * P * 4 < (long)PW_OOB, "dsgan_pw_dgrad_io: operand too large");
  DSG_REQUIRE(!w_bf16 || (M % 8) == 0, "dsgan_pw_dgrad_io: bf16 W needs M %% 8 == 0");
  PwArgs g{};
  g.A = (const float*)W; g.B = (const float*)DY; g.b_bs = dy_bs; g.Y = (float*)DX; g.y_bs = dx_bs; g.y_bf16 = dx_bf16;
  g.gpre = (const float*)GP; g.gpre_bs = gp_bs; g.gbf = GP ? 1 : 0;
  g.accumulate = accumulate; g.P = P; g.M = M; g.N = nb * P; g.K = K;
  g.a_range = (unsigned)((long)M * K * (w_bf16 ? 2 : 4));
  g.b_range = (unsigned)((long)K * P * (dy_bf16 ? 2 : 4));
  const int bm = fd_tile_k(g, w_bf16 || dy_bf16);
  const int splits = fd_plan(g, bm, ws);
  DSG_WS(fd_need(g, splits), ws, ws_elems, "dsgan_pw_dgrad_io (dsgan_pw_fd_workspace)");
  fd_launch(PW_DGRAD, g, bm, w_bf16, dy_bf16, splits, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

extern "C" int dsgan_pw_dgrad_io(const void* W, int w_bf16, const void* DY, long dy_bs, int dy_bf16, void* DX, long dx_bs,
                                 int dx_bf16, const void* GP, long gp_bs, int M, int K, int P, int nb,
                                 int accumulate, hipStream_t st) {
  return dsgan_pw_dgrad_io_ws(W, w_bf16, DY, dy_bs, dy_bf16, DX, dx_bs, dx_bf16, GP, gp_bs, M, K, P, nb, accumulate,
                              nullptr, 0, st);
}

// Scratch (floats) of a split-K FWD (mode 0) / DGRAD (1) launch of M output channels over K at nb
// images of P pixels (0: never split).  An upper bound for either operand dtype and epilogue: the
// wide / 256-row tile forms, which some of those pick, are never split.
extern "C" long dsgan_pw_fd_workspace(int mode, int M, int K, int P, int nb) {
  if ((mode != PW_FWD && mode != PW_DGRAD) || M <= 0 || K <= 0 || P <= 0 || nb <= 0 || P % 128) return 0;
  PwArgs g{};
  g.M = M; g.N = nb * P; g.K = K; g.P = P;
  // the 128 / 64-row tile is the only one that splits (a knob may pick it where 256 rows would run)
  const int bm = M > 64 ? 128 : 64;
  int ks;
  const int splits = max(fd_splits(g, bm, PBK, &ks), fd_splits(g, bm, 64, &ks));
  return splits > 1 ? (long)splits * M * nb * P : 0;
}

// Planner knob key <- val (val < 0: read only); returns the previous value.  Measurement tools only.
extern "C" int dsgan_pw_tune(int key, int val) {
  if (key < 0 || key >= 12) return -1;
  const int old = g_tune[key];
  if (val >= 0) g_tune[key] = val;
  return old;
}

// Weight-grad with bf16 operand(s): DW[M][N] += sum_{b,p} A[b][M][P] * B[b][N][P], A/B fp32 or
// bf16 (a_bf16 / b_bf16); db (nullable) += sum_{b,p} A[b][M][P] -- the bias grad, summed from the
// staged A tiles (the bf16 values when A is bf16).  P % 32 == 0, 16-byte aligned operands.
// Scratch (floats) a weight-grad of M x N over nb*P pixels needs (0: no split).
extern "C" long dsgan_pw_wgrad_workspace(int M, int N, int P, int nb) {
  PwArgs g{};
  g.M = M; g.N = N; g.P = P; g.K = nb * P;
  int bm;   // enough for either tile plan (the caller's operand dtypes pick one)
  const int splits = max(wgrad_cfg_k(g, false, &bm), wgrad_cfg_k(g, true, &bm));
  return splits > 1 ? (long)splits * ((long)M * N + M) : 0;   // weight partials, then bias-sum partials
}

extern "C" int dsgan_pw_wgrad_mixed(const void* A, long a_bs, int a_bf16, const void* B, long b_bs,
                                    int b_bf16, float* DW, float* db, int M, int N, int P, int nb, float* ws,
                                    long ws_elems, hipStream_t st) {
  DSG_REQUIRE(A && B && DW && M >= 16 && N > 0 && P > 0 && nb > 0, "dsgan_pw_wgrad_mixed: bad args");
  DSG_REQUIRE(P % 32 == 0 && al16(A) && al16(B) && (a_bs & 7) == 0 && (b_bs & 7) == 0,
              "dsgan_pw_wgrad_mixed: P %% 32 and 16-byte alignment required");
  PwArgs g{};
  g.A = (const float*)A; g.a_bs = a_bs; g.B = (const float*)B; g.b_bs = b_bs; g.Y = DW; g.asum = db; g.P = P;
  const long ar = ((long)(nb - 1) * a_bs + (long)M * P) * (a_bf16 ? 2 : 4);
  const long br = ((long)(nb - 1) * b_bs + (long)N * P) * (b_bf16 ? 2 : 4);
  DSG_REQUIRE(ar < (long)PW_OOB && br < (long)PW_OOB, "dsgan_pw_wgrad_mixed: operands exceed 4 GiB buffer range");
  g.a_range = (unsigned)ar; g.b_range = (unsigned)br;
  g.M = M; g.N = N; g.K = nb * P;
  int bm;
  const int splits = wgrad_cfg_k(g, a_bf16 || b_bf16, &bm);
  g.ws = splits > 1 ? ws : nullptr;
  DSG_WS(wgrad_need(g, splits), ws, ws_elems, "dsgan_pw_wgrad_mixed (dsgan_pw_wgrad_workspace)");
  wg_dispatch(g, bm, a_bf16, b_bf16, splits, st);
  wgrad_finish(g, splits, st);
  DSG_CHECK_LAUNCH();
  return 0;
}
