// Persistent LDS-DMA ring form of the wide 16-bit-operand pointwise FWD / DGRAD (pwgemm.hip planner
// knob 11).  Its own header and translation units (pw_ring_{bf16,f16}.hip): the epilogue is
// pw_impl.h's pw_fd_epi, shared with the one-tile kernel.
#pragma once
#include "pw_impl.h"

namespace dsg {

// s_waitcnt vmcnt(N) with the immediate capped at the counter's 6-bit maximum
template <int N>
__device__ __forceinline__ void vm_wait_c() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N < 63 ? N : 63) : "memory");
}

// ---- persistent LDS-DMA ring form of the wide 16-bit-operand FWD / DGRAD ----
// The one-tile ring kernel (pwgemm_kernel, NS = 4) runs one 256 x 256 tile per workgroup and one
// workgroup per CU (128 KB of ring): every tile pays the workgroup launch, the ring's fill (NS - 1
// stages of HBM latency before the first MFMA) and, at the end, the drain of its output stores --
// a workgroup retires only when its stores have completed, so the next tile's loads queue behind
// them (the 512 -> 2048 gelu-pair forward: ~30 us of skeleton and ~120 us of exposed stores out of
// ~265).  Here one workgroup per CU walks its tiles and the ring runs on
// across tile boundaries: the next tile's first NS - 1 stages are issued during the current tile's
// last K steps, before its epilogue, and the stage waits are counted (vm_wait_n) so that the
// epilogue's stores stay in flight under the next tile's K loop -- the wait for a stage retires
// that stage's pieces and everything older, never the stores issued after it (gfx950 retires a
// wave's vector-memory operations in issue order on the one vmcnt counter).  The count of a wait
// uses a LOWER bound of the operations issued after the stage (the epilogue's output stores only:
// its loads are left out), so it can only wait longer than needed, never too little.
// The tile's bias slice (256 floats, FWD) rides ahead of the tile's first stage (wave 0's LDS-DMA,
// issued before that stage's pieces, so the stage wait covers it) into one of two slots and is
// assigned to the accumulators after that stage's barrier: z = bias + the 16-deep K chunks in order,
// the one-tile kernel's sequence of MFMAs, so the outputs are bitwise equal to it.
// Tiles: XCD x (blockIdx & 7) takes a contiguous chunk of the M-fastest tile order, which its
// workgroups walk in lockstep (the M tiles of one pixel block share the XCD's L2).
template <typename T16, int MODE, int SWP, int EPI>
__global__ __launch_bounds__(512, 1) void pwgemm_ring_kernel(PwArgs g) {
  constexpr bool SW = MODE != PW_WGRAD && SWP;
  static_assert(EPI == PW_EPI_GELU_PAIR || EPI == PW_EPI_PLAIN, "the ring serves the gelu-pair and plain epilogues");
  typedef hx8<T16> pbf16x8;
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NT = 512, BK = 32, NS = 4, NW = NT / 64;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr bool A_KMAJ = (MODE == PW_DGRAD);
  constexpr int DA_SZ = BM * BK, DB_SZ = BK * BN, STG = DA_SZ + DB_SZ;
  constexpr int AP = DA_SZ / 8 / NT, BP = DB_SZ / 8 / NT, PI = AP + BP;
  static_assert(MODE != PW_WGRAD, "FWD / DGRAD only");
  __shared__ __attribute__((aligned(1024))) T16 smem[NS * STG];
  __shared__ __attribute__((aligned(16))) float bias_lds[2][BM];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- this workgroup's tiles ----
  const int mt = g.M / BM, ntiles = mt * (g.N / BN);
  const int G = gridDim.x, xcd = blockIdx.x & 7, lw = blockIdx.x >> 3;
  const int gx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);               // workgroups of this XCD
  const int q8 = ntiles >> 3, r8 = ntiles & 7;
  const int cnt = q8 + (xcd < r8 ? 1 : 0);                          // tiles of this XCD
  const int start = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int my = lw < cnt ? (cnt - lw + gx - 1) / gx : 0;
  if (my == 0) return;
  const int nk = g.K / BK, total = my * nk;
  const bool has_bias = MODE == PW_FWD && g.bias != nullptr;
  // tile j's first M row, image and first pixel (one division chain per tile, not per stage)
  auto tile_at = [&](int j, int& m0, int& bimg, int& p0) __attribute__((always_inline)) {
    const int t = start + lw + j * gx;
    const int n_t = t / mt;
    m0 = (t - n_t * mt) * BM;
    const int n0 = n_t * BN;
    bimg = n0 / g.P;
    p0 = n0 - bimg * g.P;
  };

  // per-lane parts of the DMA source offsets (elements; the stage's uniform base is added per issue)
  unsigned aoff[AP], boff[BP];
#pragma unroll
  for (int i = 0; i < AP; ++i) {
    const int pc = (i * NW + wave) * 64 + lane;
    if constexpr (A_KMAJ) {          // DGRAD W[K][M]: k-major [32][BM]
      const int k = pc / (BM / 8), ls = (pc % (BM / 8)) ^ pw_kswz(k);
      aoff[i] = (unsigned)(k * g.M + 8 * ls);
    } else {                         // FWD W[M][K]: rows [BM][32]
      const int r = pc >> 2, ls = (pc & 3) ^ pw_rswz(r);
      aoff[i] = (unsigned)(r * g.K + 8 * ls);
    }
  }
#pragma unroll
  for (int i = 0; i < BP; ++i) {     // X / DY [b][K][P]: k-major [32][BN]
    const int pc = (i * NW + wave) * 64 + lane;
    const int k = pc / (BN / 8), ls = (pc % (BN / 8)) ^ pw_kswz(k);
    boff[i] = (unsigned)(k * g.P + 8 * ls);
  }
  // the issue cursor: the next stage to issue (tile ij, K step ikt) and its operand bases, advanced
  // one K step per issue; the tile decode runs when the cursor enters a tile
  const long a_step = A_KMAJ ? (long)BK * g.M : BK, b_step = (long)BK * g.P;
  int ij = 0, ikt = 0, islot = 0;
  const T16* ia = nullptr;
  const T16* ib = nullptr;
  const float* ibias = nullptr;
  auto enter = [&](int j) __attribute__((always_inline)) {
    int m0, bimg, p0;
    tile_at(j, m0, bimg, p0);
    ia = (const T16*)g.A + (A_KMAJ ? (long)m0 : (long)m0 * g.K);
    ib = (const T16*)g.B + (long)bimg * g.b_bs + p0;
    ibias = g.bias + m0;
  };
  auto issue = [&]() __attribute__((always_inline)) {
    T16* As = smem + islot * STG;
    T16* Bs = As + DA_SZ;
    if (ikt == 0 && has_bias && wave == 0)   // the tile's bias slice first: the stage wait covers it
      dma16(ibias + 4 * lane, lds_off(&bias_lds[ij & 1][0]));
#pragma unroll
    for (int i = 0; i < AP; ++i) dma16(ia + aoff[i], lds_off(As + (i * NW + wave) * 512));
#pragma unroll
    for (int i = 0; i < BP; ++i) dma16(ib + boff[i], lds_off(Bs + (i * NW + wave) * 512));
    islot = islot == NS - 1 ? 0 : islot + 1;
    if (++ikt == nk) {
      ikt = 0;
      if (++ij < my) enter(ij);
    } else {
      ia += a_step;
      ib += b_step;
    }
  };
  // fragment read offsets (bytes, K-step invariant)
  unsigned ar[TM];
  uint2 at[TM], bt[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wm * TM * 32 + i * 32;
    if constexpr (A_KMAJ) at[i] = pw_tr_addr<BM / 8>(mb, lane);
    else ar[i] = (unsigned)((mb + lr) * 64 + ((lh ^ pw_rswz(mb + lr)) << 4));
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) bt[j] = pw_tr_addr<BN / 8>(wn * TN * 32 + j * 32, lane);

  // VMEM instructions of one tile's epilogue, a lower bound (its output stores only; pw_fd_epi):
  // SW 16-bit tiles store 2 x 16 bytes per 32 x 32 block and tensor, the channel x pixel fp32 tiles
  // 16 dwords per block (the count then exceeds the counter's range: waits cap at 63)
  constexpr int EQ = !SW ? TM * TN * 16 : EPI == PW_EPI_GELU_PAIR ? TM * TN * 4 : TM * TN * 2;

  enter(0);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) issue();

  pf32x16 acc[TM][TN];
  int s = 0;
  for (int j = 0; j < my; ++j) {
    int m0, bimg, p0;
    tile_at(j, m0, bimg, p0);
    for (int kt = 0; kt < nk; ++kt, ++s) {
      // stage s landed: the stages issued after it (at most NS - 2) and, for the tile's first
      // NS - 1 stages (issued before the previous tile's epilogue), its stores may stay in flight
      static_assert(NS == 4, "the wait ladder covers two later stages");
      const int later = total - 1 - s;
      if (j > 0 && kt < NS - 1) {
        if (later >= 2) vm_wait_c<2 * PI + EQ>();
        else if (later == 1) vm_wait_c<PI + EQ>();
        else vm_wait_c<EQ>();
      } else {
        if (later >= 2) vm_wait_c<2 * PI>();
        else if (later == 1) vm_wait_c<PI>();
        else vm_wait_c<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();   // every wave's pieces of stage s landed; slot (s - 1) % NS is free
      if (s + NS - 1 < total) issue();
      if (kt == 0) {   // z = bias + sum: the accumulators start at the bias (one-tile kernel's order)
        if (has_bias) {
          const float* bl = &bias_lds[j & 1][0];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            float bv[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) bv[r] = bl[wm * TM * 32 + i * 32 + (SW ? lr : (r & 3) + 8 * (r >> 2) + 4 * lh)];
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[i][jj][r] = bv[r];
          }
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
#pragma unroll
              for (int r = 0; r < 16; ++r) acc[i][jj][r] = 0.f;
        }
      }
      const T16* As = smem + (s & (NS - 1)) * STG;
      const T16* Bs = As + DA_SZ;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        pbf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (A_KMAJ) af[i] = pw_tr_at(As, at[i], ks * 16 * BM * 2);
          else af[i] = *reinterpret_cast<const pbf16x8*>((const char*)As + (ar[i] ^ (unsigned)(32 * ks)));
        }
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) bfr[jj] = pw_tr_at(Bs, bt[jj], ks * 16 * BN * 2);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int jj = 0; jj < TN; ++jj)
            acc[i][jj] = SW ? mfma16(bfr[jj], af[i], acc[i][jj]) : mfma16(af[i], bfr[jj], acc[i][jj]);
      }
    }
    pw_fd_epi<T16, BM, TM, TN, SW, false, EPI>(g, acc, m0, bimg, p0, 0, wm, wn, lr, lh, false, nullptr);
  }
}

// persistent grid: one workgroup per CU (the ring's 128 KB of LDS), never more than the tiles.
// Returns false (nothing launched) for an epilogue the ring does not serve: the caller runs the
// one-tile ring kernel.
int pw_cu_count();   // pwgemm.hip (cached device attribute)
template <typename T16, int MODE, int SWP>
bool pw_ring_launch(const PwArgs& g, hipStream_t st) {
  const bool gelu_pair = MODE == PW_FWD && SWP && g.ypre && g.gbf && g.act == ACT_GELU && !g.gpre && !g.accumulate &&
                         g.y_bf16;
  const bool plain = !g.ypre && !g.gpre && g.act == ACT_NONE;
  if (g.ws || !(gelu_pair || plain)) return false;
  const long tiles = (long)(g.M / 256) * (g.N / 256);
  const long grid = tiles < pw_cu_count() ? tiles : pw_cu_count();
  ktimer_mark(st, 0);
  if constexpr (MODE == PW_FWD && SWP) {
    if (gelu_pair)
      hipLaunchKernelGGL((pwgemm_ring_kernel<T16, MODE, SWP, PW_EPI_GELU_PAIR>), dim3((unsigned)grid), dim3(512), 0, st, g);
    else
      hipLaunchKernelGGL((pwgemm_ring_kernel<T16, MODE, SWP, PW_EPI_PLAIN>), dim3((unsigned)grid), dim3(512), 0, st, g);
  } else {
    hipLaunchKernelGGL((pwgemm_ring_kernel<T16, MODE, SWP, PW_EPI_PLAIN>), dim3((unsigned)grid), dim3(512), 0, st, g);
  }
  ktimer_mark(st, 1);
  return true;
}

}  // namespace dsg
