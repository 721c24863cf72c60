// Persistent "epilogue beside the next tile's MFMAs" form of the gelu-pair pointwise forward: the
// unfused blocks' pwconv1 + GELU (MixConvNeXtML.py:218-242 at C = 512 / 1024), which writes
// y = gelu(z) and gp = gelu'(z) as 16-bit tensors for the GEMM that follows and for the backward.
//
// Why: in the one-tile-per-workgroup kernel (pw_impl.h, 256 x 256 tiles, 8 waves) every wave runs its
// K loop, then its epilogue -- ~20 VALU per output element (the erf-GELU pair, 16-bit packing) and
// the output stores -- and both waves of a SIMD reach the epilogue together: MFMA busy 0.21, VALU
// busy 0.33, co-issue 0.007 (profiles/r04/pw_pmc.json).
//
// Here one workgroup per CU (4 waves, one per SIMD, up to 512 registers each) walks a sequence of
// 256 x 128 tiles (wave tile 128 x 64, swapped operands: a lane ends with 4-pixel runs of one
// channel).  Each wave holds two accumulator sets (tile t's MFMA accumulators, and tile t-1's,
// copied out when its K loop ended): while the MFMAs of tile t run, the GELU pair of tile t-1 is
// evaluated, half a 32 x 32 block per K step, into packed 16-bit registers
// -- VALU work with no dependence on the MFMAs in flight, so the SIMD co-issues it -- and stored
// right away (four 16-byte stores per block), so the output writes spread over the K loop.
//
// Operand tiles arrive by LDS-DMA into a 4-stage ring that runs continuously across tiles (the first
// stages of tile t+1 land under tile t's last steps and the store burst).  The tile's bias slice
// (256 floats) rides with the tile's first stage into one of two bias slots.  Every VMEM
// instruction of the loop is counted on the host side of the wave (`issued`): the wait before a
// stage's barrier retires exactly that stage's pieces, whatever stores were issued after them
// (gfx950 retires loads and stores on one in-order counter).
//
// Arithmetic per output: z = bias + sum over 16-deep K chunks in order (the 256 x 256 kernel's
// order), y / gp from gelu_pair_fast1x2 (the packed form's operations, same bits).
//
// Measured (round 5, profiles/r05/pw_bench_persistent.txt): bitwise equal to the one-tile kernel in
// bf16, but 1.75-1.95x SLOWER (the 512 -> 2048 forward at 64^2: 269 -> 476 us).  With one wave per
// SIMD nothing hides the per-step latencies -- the barrier, the fragment reads before the MFMAs, the
// stage wait and the scalar address arithmetic of the DMA issue -- which the 8-wave kernel's second
// wave per SIMD covers; the VALU / MFMA overlap does not pay for them.  Kept behind planner knob 11
// (off by default) as the measured form; see DESIGN.md section 9.
#include "pw_impl.h"

namespace dsg {

constexpr int PP_BM = 256, PP_BN = 128, PP_BK = 32, PP_NS = 4;
constexpr int PP_DA = PP_BM * PP_BK, PP_DB = PP_BK * PP_BN;   // stage images (16-bit elements)
constexpr int PP_STAGE = PP_DA + PP_DB;

// s_waitcnt vmcnt(n) for a wave-uniform n (the immediate is compile-time: binary search, 6 levels)
template <int LO, int HI>
__device__ __forceinline__ void pp_vmwait(int n) {
  if constexpr (LO == HI) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(LO) : "memory");
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) pp_vmwait<LO, MID>(n);
    else pp_vmwait<MID + 1, HI>(n);
  }
}

struct PpTile { int m0, bimg, p0; };

// Per-wave constants of the kernel (all wave-uniform except the lane fields).
struct PpCtx {
  const void* A; const void* B; const float* bias; void* Y; void* YP;
  long b_bs, y_bs, yp_bs;
  int M, K, P, mt, G, rank, nk, total;
  int wave, wm, wn, lane, lr, lh;
};

__device__ __forceinline__ PpTile pp_tile(const PpCtx& c, int k) {
  const int t = c.rank + k * c.G, m_t = t % c.mt, n0 = (t / c.mt) * PP_BN;
  const int b = n0 / c.P;
  return PpTile{__builtin_amdgcn_readfirstlane(m_t * PP_BM), __builtin_amdgcn_readfirstlane(b),
                __builtin_amdgcn_readfirstlane(n0 - b * c.P)};
}

// LDS-DMA of global stage s (tile s / nk, K step s % nk) into ring slot s % NS; returns the number
// of VMEM instructions this wave issued (6, or 7 with the tile's bias slice on its first step).
template <typename T16>
__device__ __forceinline__ int pp_issue(const PpCtx& c, T16* smem, float* bias_lds, const unsigned* arow,
                                        const unsigned* bcol, int s) {
  const int k = s / c.nk, kt = s - k * c.nk;
  const PpTile t = pp_tile(c, k);
  T16* As = smem + (s % PP_NS) * PP_STAGE;
  T16* Bs = As + PP_DA;
  const T16* a = (const T16*)c.A + (long)t.m0 * c.K + kt * PP_BK;
  const T16* b = (const T16*)c.B + (long)t.bimg * c.b_bs + t.p0 + (long)kt * PP_BK * c.P;
#pragma unroll
  for (int i = 0; i < 4; ++i) dma16(a + arow[i], lds_off(As + (i * 4 + c.wave) * 512));
#pragma unroll
  for (int i = 0; i < 2; ++i) dma16(b + bcol[i], lds_off(Bs + (i * 4 + c.wave) * 512));
  if (kt != 0) return 6;
  // the tile's bias slice (every wave issues the same 1 KB, so that the counts stay uniform)
  const void* src = c.bias ? (const void*)(c.bias + t.m0 + 4 * c.lane) : (const void*)g_dma_zero16;
  dma16(src, lds_off(bias_lds + (k & 1) * PP_BM));
  return 7;
}

// The GELU pair of half of one finished 32 x 32 block (i, j) of tile t (accumulator registers
// 8h .. 8h + 7: pixels 16h + 4lh.. of the lane's channel), packed to 16 bits and stored right away:
// two 16-byte stores (lane lr = channel mrow + lr; two 4-pixel groups paired by permlane32 swaps as
// pw_impl.h's store16 pairs them).
template <typename T16>
__device__ __forceinline__ void pp_finish_half(const PpCtx& c, const f32x16_t& a, const PpTile& t, int i, int j, int h) {
  unsigned dy[4], dg[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 y, gp;
    gelu_pair_fast1x2(f32x2{a[8 * h + 2 * q], a[8 * h + 2 * q + 1]}, y, gp);
    dy[q] = (unsigned)f2h<T16>(y.x) | ((unsigned)f2h<T16>(y.y) << 16);
    dg[q] = (unsigned)f2h<T16>(gp.x) | ((unsigned)f2h<T16>(gp.y) << 16);
  }
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    auto x = __builtin_amdgcn_permlane32_swap(dy[w], dy[2 + w], false, false);
    dy[w] = x[0]; dy[2 + w] = x[1];
    x = __builtin_amdgcn_permlane32_swap(dg[w], dg[2 + w], false, false);
    dg[w] = x[0]; dg[2 + w] = x[1];
  }
  const unsigned range = (unsigned)(((long)c.M * c.P - t.p0) * 2);
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((T16*)c.Y + (long)t.bimg * c.y_bs + t.p0), (short)0, range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((T16*)c.YP + (long)t.bimg * c.yp_bs + t.p0), (short)0, range, 0x00020000);
  const int col0 = c.wn * 64 + j * 32;
  const int s2 = __builtin_amdgcn_readfirstlane((t.m0 + c.wm * 128 + i * 32) * c.P * 2) + 32 * h;
  const int vh = (c.lr * c.P + col0) * 2 + 16 * c.lh;
  const pu32x4 o = {dy[0], dy[1], dy[2], dy[3]};
  __builtin_amdgcn_raw_buffer_store_b128(o, ry, vh, s2, 0);
  const pu32x4 o2 = {dg[0], dg[1], dg[2], dg[3]};
  __builtin_amdgcn_raw_buffer_store_b128(o2, rp, vh, s2, 0);
}

template <typename T16>
__global__ __launch_bounds__(256, 1) void pwpp_gelu_kernel(PwArgs g, int ntiles) {
  typedef hx8<T16> pbf16x8;
  constexpr int TM = 4, TN = 2;   // 32 x 32 blocks per wave (wave tile 128 ch x 64 px)
  __shared__ __attribute__((aligned(1024))) T16 smem[PP_NS * PP_STAGE + 2 * PP_BM * 2];   // + 2 fp32 bias slots
  float* const bias_lds = reinterpret_cast<float*>(smem + PP_NS * PP_STAGE);

  PpCtx c;
  c.A = g.A; c.B = g.B; c.bias = g.bias; c.Y = g.Y; c.YP = g.ypre;
  c.b_bs = g.b_bs; c.y_bs = g.y_bs; c.yp_bs = g.ypre_bs;
  c.M = g.M; c.K = g.K; c.P = g.P; c.mt = g.M / PP_BM; c.G = gridDim.x;
  c.lane = threadIdx.x & 63;
  c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  c.wm = c.wave >> 1; c.wn = c.wave & 1; c.lr = c.lane & 31; c.lh = c.lane >> 5;
  {
    const int id = blockIdx.x, xcd = id & 7, q = c.G >> 3, r = c.G & 7;
    c.rank = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int nmine = c.rank < ntiles ? (ntiles - c.rank + c.G - 1) / c.G : 0;
  c.nk = g.K / PP_BK;
  c.total = nmine * c.nk;

  // per-lane DMA source offsets (elements), tile- and stage-invariant parts (pw_impl.h images)
  unsigned arow[4], bcol[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // A = W[M][K]: row image [256][32], 16-byte slot swizzle pw_rswz
    const int pc = (i * 4 + c.wave) * 64 + c.lane, r = pc >> 2, ls = (pc & 3) ^ pw_rswz(r);
    arow[i] = (unsigned)(r * c.K + 8 * ls);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // B = X[b][K][P]: k-major image [32][128], swizzle pw_kswz
    const int pc = (i * 4 + c.wave) * 64 + c.lane, k = pc / (PP_BN / 8), ls = (pc % (PP_BN / 8)) ^ pw_kswz(k);
    bcol[i] = (unsigned)(k * c.P + 8 * ls);
  }
  // fragment read offsets (bytes, K-step invariant), as pw_impl.h's ring
  unsigned ar[TM];
  uint2 bt[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = c.wm * TM * 32 + i * 32;
    ar[i] = (unsigned)((mb + c.lr) * 64 + ((c.lh ^ pw_rswz(mb + c.lr)) << 4));
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) bt[j] = pw_tr_addr<PP_BN / 8>(c.wn * TN * 32 + j * 32, c.lane);

  // VMEM instructions this wave has issued (DMA pieces and stores) and, per ring slot, the count right
  // after its stage's pieces: the wait before stage s retires exactly `issued - mark[s % NS]` later ops
  int issued = 0, mark0 = 0, mark1 = 0, mark2 = 0, mark3 = 0;
#define PP_ISSUE(S_)                                                                              \
  do {                                                                                            \
    const int s__ = (S_);                                                                         \
    issued += pp_issue<T16>(c, smem, bias_lds, arow, bcol, s__);                                  \
    const int sl__ = s__ % PP_NS;                                                                 \
    mark0 = sl__ == 0 ? issued : mark0; mark1 = sl__ == 1 ? issued : mark1;                       \
    mark2 = sl__ == 2 ? issued : mark2; mark3 = sl__ == 3 ? issued : mark3;                       \
  } while (0)

  // one K step of tile K_ (global stage s): wait, barrier, issue stage s + NS - 1, the step's MFMAs;
  // FIN_ (the previous tile's block of this step, or nothing) between the two MFMA groups
#define PP_KSTEP(K_, KT_, ACC_, FIN_)                                                                   \
  do {                                                                                                  \
    const int s = (K_) * c.nk + (KT_);                                                                  \
    const int sl = s % PP_NS;                                                                           \
    const int mk = sl == 0 ? mark0 : sl == 1 ? mark1 : sl == 2 ? mark2 : mark3;                         \
    const int later = issued - mk;                                                                      \
    pp_vmwait<0, 63>(later < 63 ? later : 63);                                                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                  \
    raw_barrier();                                                                                      \
    if (s + PP_NS - 1 < c.total) PP_ISSUE(s + PP_NS - 1);                                               \
    if ((KT_) == 0) {                                                                                   \
      const float* bl = bias_lds + ((K_) & 1) * PP_BM + c.wm * TM * 32 + c.lr;                          \
      _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                                  \
        const float bv = bl[i * 32];                                                                    \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                  \
          _Pragma("unroll") for (int r = 0; r < 16; ++r) ACC_[i][j][r] = bv;                            \
      }                                                                                                 \
    }                                                                                                   \
    const T16* As = smem + sl * PP_STAGE;                                                               \
    const T16* Bs = As + PP_DA;                                                                         \
    _Pragma("unroll") for (int ks = 0; ks < PP_BK / 16; ++ks) {                                         \
      pbf16x8 af[TM], bfr[TN];                                                                          \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                    \
        af[i] = *reinterpret_cast<const pbf16x8*>((const char*)As + (ar[i] ^ (unsigned)(32 * ks)));     \
      _Pragma("unroll") for (int j = 0; j < TN; ++j) bfr[j] = pw_tr_at(Bs, bt[j], ks * 16 * PP_BN * 2); \
      __builtin_amdgcn_s_setprio(1);                                                                    \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                    \
        _Pragma("unroll") for (int j = 0; j < TN; ++j) ACC_[i][j] = mfma16(bfr[j], af[i], ACC_[i][j]);  \
      __builtin_amdgcn_s_setprio(0);                                                                    \
      if (ks == 0) { FIN_; }                                                                            \
    }                                                                                                   \
  } while (0)

  // tile K_ into ACC_; the previous tile's 8 blocks (PREV_) finished beside its first 16 K steps, half
  // a block per step (its VALU about matches the step's 16 MFMAs).  The 16 steps are written out
  // (PP_HB) so that every PREV_ index is a compile-time constant.
#define PP_HB(HB_)                                                                                          \
  do {                                                                                                      \
    constexpr int b_ = (HB_) >> 1;                                                                          \
    if ((HB_) < c.nk) {                                                                                     \
      PP_KSTEP(k_, (HB_), acc, if (has_prev) {                                                              \
        pp_finish_half<T16>(c, prev[b_ % TM][b_ / TM], pt, b_ % TM, b_ / TM, (HB_) & 1); issued += 2; });   \
    } else if (has_prev) {                                                                                  \
      pp_finish_half<T16>(c, prev[b_ % TM][b_ / TM], pt, b_ % TM, b_ / TM, (HB_) & 1);                      \
      issued += 2;                                                                                          \
    }                                                                                                       \
  } while (0)

  // acc: the tile being computed (MFMA accumulators); prev: the previous tile's, copied out when
  // its K loop ends (one static register set each: no role swapping, one copy of the loop body)
  f32x16_t acc[TM][TN], prev[TM][TN];
#pragma unroll
  for (int s = 0; s < PP_NS - 1; ++s)
    if (s < c.total) PP_ISSUE(s);
  for (int k = 0; k < nmine; ++k) {
    const bool has_prev = k > 0;
    const int k_ = k;
    const PpTile pt = pp_tile(c, k > 0 ? k - 1 : 0);
    PP_HB(0); PP_HB(1); PP_HB(2); PP_HB(3); PP_HB(4); PP_HB(5); PP_HB(6); PP_HB(7);
    PP_HB(8); PP_HB(9); PP_HB(10); PP_HB(11); PP_HB(12); PP_HB(13); PP_HB(14); PP_HB(15);
    for (int kt = 2 * TM * TN; kt < c.nk; ++kt) PP_KSTEP(k_, kt, acc, (void)0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) prev[i][j] = acc[i][j];
  }
  if (nmine > 0) {   // the last tile: GELU pair and stores with nothing beside them
    const PpTile t = pp_tile(c, nmine - 1);
#pragma unroll
    for (int hb = 0; hb < 2 * TM * TN; ++hb) pp_finish_half<T16>(c, prev[(hb >> 1) % TM][(hb >> 1) / TM], t, (hb >> 1) % TM, (hb >> 1) / TM, hb & 1);
  }
#undef PP_HB
#undef PP_KSTEP
#undef PP_ISSUE
}

// host side: the plan conditions are checked by the caller (pwgemm.hip pp_ok)
template <typename T16>
static void pwpp_launch_t(const PwArgs& g, hipStream_t st) {
  const int ntiles = (g.M / PP_BM) * (g.N / PP_BN);
  int grid = 256;   // one workgroup per CU
  if (grid > ntiles) grid = ntiles;
  hipLaunchKernelGGL((pwpp_gelu_kernel<T16>), dim3((unsigned)grid), dim3(256), 0, st, g, ntiles);
}

void pwpp_gelu_launch(const PwArgs& g, hipStream_t st) {
  if (half_type() == HALF_F16) pwpp_launch_t<_Float16>(g, st);
  else pwpp_launch_t<__bf16>(g, st);
}

}  // namespace dsg
