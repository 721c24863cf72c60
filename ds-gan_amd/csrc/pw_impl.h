// Pointwise GEMM kernel templates (pwgemm.hip), shared by the translation units that instantiate
// them: pw_{fwd,dgrad,wgrad}_{bf16,f16}.hip (one mode x operand type each, compiled in parallel) and
// pwgemm.hip (the planner + the C ABI).  See pwgemm.hip for the design notes.
#pragma once
#include "common.h"
#include "lds_dma.h"
#include <stdlib.h>

namespace dsg {


typedef f32x16_t pf32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int pu32x4;   // 16 raw bytes (8 bf16)

enum PwMode : int { PW_FWD = 0, PW_DGRAD = 1, PW_WGRAD = 2 };

struct PwArgs {
  const float* A; long a_bs;   // FWD: W[M][K]  DGRAD: W[K][M]  WGRAD: DY[b][M][P]
  const float* B; long b_bs;   // FWD/DGRAD: X/DY [b][K][P]     WGRAD: X[b][N][P]
  float* Y; long y_bs;         // FWD/DGRAD output [b][M][P];   WGRAD: DW[M][N] (+=)
  const float* bias;
  float* ypre; long ypre_bs;
  const float* gpre; long gpre_bs;
  int M, N, K, P;
  int act, gact, bact, accumulate; float slope;
  int k_split;                 // K per split (WGRAD: always; FWD/DGRAD: 0 = unsplit)
  float* ws;                   // splits > 1: fp32 partials -- WGRAD [split][M][N]; FWD/DGRAD
                               // [split][b][M][P] (raw accumulators, pw_split_finish_kernel applies
                               // the epilogue)
  unsigned a_range, b_range;   // buffer-resource byte ranges of A and B (B: per image for FWD/DGRAD)
  int y_bf16;  // FWD: Y is bf16 [b][M][P] (y_bs in elements)
  int gbf;     // FWD: ypre is bf16 and receives act'(pre);  DGRAD: gpre is a bf16 multiplier (no act')
  int gp_pref; // DGRAD with a 16-bit gp multiplier (SWP tiles): load gp before the K loop
#ifdef DSG_MEASURE
  int dbg;     // measurement builds only (build_lib.py --measure; planner knob 10): bit 0 = drop the
               // epilogue's output stores, bit 1 = the gelu pair without its GELU arithmetic
#endif
  int dma;     // host planner: the wide 16-bit-operand launch runs an LDS-DMA ring form: 1 = 256 x 256
               // tiles (8 waves, 4 stages, one workgroup per CU), 2 = 256 x 128 tiles (4 waves, 3 stages,
               // two workgroups per CU: one's epilogue runs beside the other's MFMAs)
  float* asum; // WGRAD (nullable): db[m] += sum_k A[m][k] -- the bias grad of the layer whose output
               // grad is A, from the staged A tiles (split partials after the S*M*N weight partials)
};

constexpr int PBK = 32;                 // K per main-loop step
constexpr int RM_STR = PBK + 8;         // row-major [rows][k] tile stride (80 B: conflict-free b128)

template <typename T16>
__device__ __forceinline__ hx8<T16> tr_frag(const T16* p0, int stride) {
  // two ds_read_b64_tr_b16: rows k..k+3 then k+4..k+7 of a k-major tile
#if defined(__HIP_DEVICE_COMPILE__)
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * stride));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}

// ---- LDS-DMA stage images (NS > 0 kernels): unpadded tiles with XOR-swizzled 16-byte slots ----
// A DMA piece is lane-linear in LDS, so the swizzle goes on the global source address.
//   row image [rows][32] (4 slots per 64-byte row; row reads, ds_read_b128): slot ^ ((row >> 2) & 3)
//     -- 16 consecutive rows reading one logical slot touch 16 distinct 16-byte bank groups;
//   k-major image [32][cols] (cols / 8 >= 16 slots; transposed reads, 2 x ds_read_b64_tr_b16):
//     slot ^ (4 (k & 3) + ((k >> 2) & 3)) -- conflict-free for the 4-slot x 4-row transposed reads.
__device__ __forceinline__ int pw_rswz(int r) { return (r >> 2) & 3; }
__device__ __forceinline__ int pw_kswz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
typedef __attribute__((address_space(3))) s16x4 pw_lds_s16x4;
// transposed fragment of a k-major image [32][S*8] at rows k0 + (8h + tq, +4), cols col0 + 16 tG + 4 tp
// (the tr_frag lane map); byte offsets of the two reads for k0 = 0 (k0 % 16 == 0 adds k0 * S * 16 bytes)
template <int S>
__device__ __forceinline__ uint2 pw_tr_addr(int col0, int lane) {
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1, h = lane >> 5;
  const int col = col0 + 16 * tG + 4 * tp;
  const int rlo = 8 * h + tq, rhi = rlo + 4;
  return make_uint2((unsigned)(rlo * S * 8 + (((col >> 3) ^ pw_kswz(rlo)) << 3) + (col & 7)) * 2u,
                    (unsigned)(rhi * S * 8 + (((col >> 3) ^ pw_kswz(rhi)) << 3) + (col & 7)) * 2u);
}
template <typename T16>
__device__ __forceinline__ hx8<T16> pw_tr_at(const T16* T, uint2 a, unsigned kbytes) {
#if defined(__HIP_DEVICE_COMPILE__)
  const char* b = (const char*)T + kbytes;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_s16x4*)(b + a.x));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((pw_lds_s16x4*)(b + a.y));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}

constexpr unsigned PW_OOB = 0xFFFFFFF0u;   // voffset past every resource range (ranges < PW_OOB)

template <typename T16>
__device__ __forceinline__ hx4<T16> cvt4(float4 v, int bact, float slope) {
  if (bact) { v.x = act_f(bact, v.x, slope); v.y = act_f(bact, v.y, slope); v.z = act_f(bact, v.z, slope); v.w = act_f(bact, v.w, slope); }
  hx4<T16> r;
  r[0] = (T16)v.x; r[1] = (T16)v.y; r[2] = (T16)v.z; r[3] = (T16)v.w;
  return r;
}

// 16-byte buffer store followed by its wait states.  A VALU write to a VGPR that still holds the
// data of a preceding store of more than 8 bytes needs a wait state (the store reads its data after
// issue).  hipcc models that hazard only for buffer stores whose soffset is not a register, and ours
// always have one: in round 6's persistent ring kernel (measured, removed) it scheduled
// "buffer_store_dwordx4 v[138:141], ..., s1; v_or_b32 v138, ..." and some lanes stored the new v138
// (1.4e-4 of one output's elements, bitwise test vs the one-tile kernel).  The store stays the builtin (hipcc
// counts it in its vmcnt waits: an inline-asm store it cannot see made every later load wait for all
// earlier stores -- the gp-multiplied data-grad ran 8x slower), and an s_nop that reads the data
// registers follows it: they stay allocated until two wait states after the store.
__device__ __forceinline__ void pw_st128(pu32x4 v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
  asm volatile("s_nop 1" ::"v"(v));
}

// FWD / DGRAD epilogue of one output tile: bias already in the accumulators; side tensors,
// activation, accumulation and the stores.
template <typename T16, int BM, int TM, int TN, bool SW, bool GPF>
__device__ __forceinline__ void pw_fd_epi(const PwArgs& g, pf32x16 (&acc)[TM][TN], int m0, int bimg, int p0, int split,
                                          int wm, int wn, int lr, int lh, bool gpf_on, const uint2* gpf) {
  // FWD / DGRAD: element (m, n0+col) of image bimg lives at base + m*P + col; buffer resources
  // are based at pixel p0 of row 0, their range ends at row M (a lane whose channel is >= M gets an
  // offset past the range: its loads read 0, its stores are dropped).  Tile (i, j) is pixel x
  // channel: lane lr holds channel mrow + lr, register 4q + e pixel col0 + 8q + 4lh + e -- fp32
  // side tensors move as one 16-byte access per group q, 16-bit ones as 8-byte loads and, paired
  // by v_permlane32_swap, two 16-byte stores per tile (cdna_hip_programming.md T21).
  // A split-K partial (g.ws) stores the raw fp32 accumulator into its split's [b][M][P] slab; the
  // bias, activation, side tensors and accumulation are pw_split_finish_kernel's.
  const bool part = g.ws != nullptr;
  float* const ybase = part ? g.ws + (long)split * g.M * g.N : g.Y;
  const long ybs = part ? (long)g.M * g.P : g.y_bs;
  const float* const gpre = part ? nullptr : g.gpre;
  float* const ypre = part ? nullptr : g.ypre;
  const int act = part ? 0 : g.act, accumulate = part ? 0 : g.accumulate, y_bf16 = part ? 0 : g.y_bf16;
  const int gbf = g.gbf;
  const unsigned grange = (unsigned)(((long)g.M * g.P - p0) * 4);
#ifdef DSG_MEASURE
  // (g.dbg & 1: measurement builds only -- zero-range output descriptors drop every output store, so
  // an A/B prices the epilogue's HBM writes; cdna_hip_programming.md T8)
  const unsigned range = (g.dbg & 1) ? 0u : grange;
#else
  const unsigned range = grange;
#endif
  const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ybase + (long)bimg * ybs + p0), (short)0, range, 0x00020000);
  const __amdgpu_buffer_rsrc_t ryh = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((T16*)g.Y + (long)bimg * g.y_bs + p0), (short)0, range / 2, 0x00020000);
  __amdgpu_buffer_rsrc_t rp = ry, rg = ry;
  // bf16 side tensors (gbf): same element offsets, byte offsets halved
  const int esz = gbf ? 2 : 4;
  if (ypre) rp = __builtin_amdgcn_make_buffer_rsrc((void*)((char*)ypre + ((long)bimg * g.ypre_bs + p0) * esz), (short)0,
                                                   gbf ? range / 2 : range, 0x00020000);
  if (gpre) rg = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)gpre + ((long)bimg * g.gpre_bs + p0) * esz),
                                                   (short)0, gbf ? grange / 2 : grange, 0x00020000);
  // 16-bit store of this lane's 16 values: groups (q, q+1) swap halves so lanes 0-31 hold pixels
  // 8q..8q+7 and lanes 32-63 pixels 8q+8..8q+15 of their channel (byte offset +16)
  auto store16 = [&](__amdgpu_buffer_rsrc_t r, const float* v, int vh, int srow) __attribute__((always_inline)) {
    unsigned d[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) d[t] = (unsigned)f2h<T16>(v[2 * t]) | ((unsigned)f2h<T16>(v[2 * t + 1]) << 16);
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const auto x = __builtin_amdgcn_permlane32_swap(d[2 * q + w], d[2 * q + 2 + w], false, false);
        d[2 * q + w] = x[0];
        d[2 * q + 2 + w] = x[1];
      }
      const pu32x4 o = {d[2 * q], d[2 * q + 1], d[2 * q + 2], d[2 * q + 3]};
      pw_st128(o, r, vh, srow + 16 * q);
    }
  };
  if constexpr (SW) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col0 = wn * TN * 32 + j * 32;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mrow = m0 + wm * TM * 32 + i * 32;   // uniform
        const bool ok = mrow + lr < g.M;
        const int e0 = lr * g.P + col0 + 4 * lh;       // lane part (elements)
        const int v4 = ok ? e0 * 4 : (int)PW_OOB;      // fp32 byte offsets; + 32 q in soffset
        const int v2 = ok ? e0 * 2 : (int)PW_OOB;      // 16-bit loads; + 16 q
        const int vh = ok ? (e0 - 4 * lh) * 2 + 16 * lh : (int)PW_OOB;   // paired 16-bit stores
        const int s4 = mrow * g.P * 4, s2 = mrow * g.P * 2;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r];
        if (gpre && gbf) {          // DGRAD: v *= gp, gp = act'(pre) stored 16-bit by the forward
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint2 u;
            if (gpf_on) u = gpf[(GPF ? (j * TM + i) * 4 : 0) + (GPF ? q : 0)];
            else {
              const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(rg, v2, s2 + 16 * q, 0);
              u = make_uint2(w2[0], w2[1]);
            }
            v[4 * q] *= h2f<T16>((unsigned short)(u.x & 0xffffu));
            v[4 * q + 1] *= h2f<T16>((unsigned short)(u.x >> 16));
            v[4 * q + 2] *= h2f<T16>((unsigned short)(u.y & 0xffffu));
            v[4 * q + 3] *= h2f<T16>((unsigned short)(u.y >> 16));
          }
        } else if (gpre) {
          float gv[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 u = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg, v4, s4 + 32 * q, 0));
            gv[4 * q] = u.x; gv[4 * q + 1] = u.y; gv[4 * q + 2] = u.z; gv[4 * q + 3] = u.w;
          }
          act_g_mul_arr(g.gact, v, gv, g.slope);
        }
        bool acted = false;
        if (ypre && gbf) {          // FWD: ypre <- 16-bit act'(pre), v <- act(pre) (one GELU evaluation)
          float apv[16];
#ifdef DSG_MEASURE
          if (g.dbg & 2) {              // (measurement builds only: the pair without its GELU arithmetic)
#pragma unroll
            for (int r = 0; r < 16; ++r) apv[r] = v[r];
          } else
#endif
          if (act == ACT_GELU) {
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              f32x2 a, ap;
              gelu_pair_fast2(f32x2{v[r], v[r + 1]}, a, ap);
              v[r] = a.x; v[r + 1] = a.y;
              apv[r] = ap.x; apv[r + 1] = ap.y;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              apv[r] = act_g(act, v[r], g.slope);
              v[r] = act_f(act, v[r], g.slope);
            }
          }
          store16(rp, apv, vh, s2);
          acted = true;
        } else if (ypre) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const pu32x4 o = {__builtin_bit_cast(unsigned, v[4 * q]), __builtin_bit_cast(unsigned, v[4 * q + 1]),
                              __builtin_bit_cast(unsigned, v[4 * q + 2]), __builtin_bit_cast(unsigned, v[4 * q + 3])};
            pw_st128(o, rp, v4, s4 + 32 * q);
          }
        }
        if (!acted) act_f_arr(act, v, g.slope);
        if (accumulate) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 u = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ry, v4, s4 + 32 * q, 0));
            v[4 * q] += u.x; v[4 * q + 1] += u.y; v[4 * q + 2] += u.z; v[4 * q + 3] += u.w;
          }
        }
        if (y_bf16) {   // 16-bit output: same rows, half the byte offsets
          store16(ryh, v, vh, s2);
          continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const pu32x4 o = {__builtin_bit_cast(unsigned, v[4 * q]), __builtin_bit_cast(unsigned, v[4 * q + 1]),
                            __builtin_bit_cast(unsigned, v[4 * q + 2]), __builtin_bit_cast(unsigned, v[4 * q + 3])};
          pw_st128(o, ry, v4, s4 + 32 * q);
        }
      }
    }
  } else {
    const int P4 = g.P * 4;
    const bool full = m0 + BM <= g.M;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * TN * 32 + j * 32 + lr;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mrow = m0 + wm * TM * 32 + i * 32;   // uniform
        // lane part of the offset: rows 4h, column col.  In a partial M tile, rows >= M get an
        // offset past the resource range so the hardware drops the store / returns 0.
        const int vofs = (4 * lh * g.P + col) * 4;
        const int mlim = full ? BM : g.M - mrow - 4 * lh;   // rows (r&3)+8(r>>2) < mlim are valid
        int vrow[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) vrow[r] = ((r & 3) + 8 * (r >> 2) < mlim) ? vofs : (int)PW_OOB;
        // the row of register r as a scalar offset
        auto so = [&](int r, int div) __attribute__((always_inline)) { return (mrow + (r & 3) + 8 * (r >> 2)) * (P4 / div); };
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[i][j][r];
        if (gpre && gbf) {          // DGRAD: v *= gp, gp = act'(pre) stored bf16 by the forward
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned short hb = __builtin_amdgcn_raw_buffer_load_b16(
                rg, vrow[r] == (int)PW_OOB ? (int)PW_OOB : vrow[r] / 2, so(r, 2), 0);
            v[r] *= h2f<T16>(hb);
          }
        } else if (gpre) {
          float gv[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            gv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        rg, vrow[r], so(r, 1), 0));
          act_g_mul_arr(g.gact, v, gv, g.slope);
        }
        bool acted = false;
        if (ypre && gbf) {          // FWD: ypre <- bf16 act'(pre), v <- act(pre) (one GELU evaluation)
          float apv[16];
          if (act == ACT_GELU) {
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              f32x2 a, ap;
              gelu_pair_fast2(f32x2{v[r], v[r + 1]}, a, ap);
              v[r] = a.x; v[r + 1] = a.y;
              apv[r] = ap.x; apv[r + 1] = ap.y;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              apv[r] = act_g(act, v[r], g.slope);
              v[r] = act_f(act, v[r], g.slope);
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b16(f2h<T16>(apv[r]), rp,
                                                  vrow[r] == (int)PW_OOB ? (int)PW_OOB : vrow[r] / 2,
                                                  so(r, 2), 0);
          acted = true;
        } else if (ypre) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[r]), rp, vrow[r],
                                                  so(r, 1), 0);
        }
        if (!acted) act_f_arr(act, v, g.slope);
        if (accumulate) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            v[r] += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        ry, vrow[r], so(r, 1), 0));
        }
        if (y_bf16) {   // bf16 output: same rows, half the byte offsets
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned short hb = f2h<T16>(v[r]);
            __builtin_amdgcn_raw_buffer_store_b16(hb, ryh, vrow[r] == (int)PW_OOB ? (int)PW_OOB : vrow[r] / 2,
                                                  so(r, 2), 0);
          }
          continue;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[r]), ry, vrow[r],
                                                so(r, 1), 0);
      }
    }
  }
}

// ABF (WGRAD only) / BBF: the A (dy) / B (x, dy) operand is bf16 in HBM -- the block activation h
// (InstanceNorm bf16 output), gelu(z) and dz of the MLPs (mlp.hip and the unfused blocks) -- and
// is copied to LDS unconverted.
// BN x WN waves / BK: 128 x 2 / 32 (4 waves, two workgroups per CU), or the wide form 256 x 4 / 64
// (8 waves, 256 x 256 tiles, 64-deep K steps: twice the MFMAs per staged byte and per barrier)
// for the deep, wide GEMMs of the unfused blocks.
// SWP (FWD / DGRAD with a 16-bit output): the MFMA operands go in swapped, a pixel x channel tile,
// so each lane ends with runs of 4 consecutive pixels of one channel and the epilogue writes
// 16-byte stores (2 per 32x32 tile instead of 16 two-byte ones).  fp32 outputs keep the channel x
// pixel tile, whose 4-byte stores fill two whole 128-byte rows per instruction (measured: the
// swapped form's 16-byte row-strided fp32 stores are 10-15 % slower there).
// NS > 0 (16-bit A and B, full tiles, K per split % 32 == 0): the operand tiles arrive by LDS-DMA
// into an NS-stage ring of unpadded swizzled images, NS - 1 K steps ahead of the MFMAs, one raw
// barrier per K step and no register staging; the MFMAs, their order and the epilogue are the
// register-staged kernel's (same bits for the products; WGRAD's row sums of A are read back from
// the landed stage).
template <typename T16, int MODE, int BM, int ABF = 0, int BBF = 0, int BN = 128, int WN = 2, int BK = PBK, int SWP = 0,
          int NS = 0>
__global__ __launch_bounds__(128 * WN, WN == 2 ? 2 : 1) void pwgemm_kernel(PwArgs g) {
  constexpr bool SW = MODE != PW_WGRAD && SWP;
  typedef hx8<T16> pbf16x8;
  typedef hx4<T16> pbf16x4;
  constexpr int WM = 2, NT = 64 * WM * WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  constexpr int RM_STR = BK + 8;        // row-major [rows][k] stride (odd 16-byte slot count)
  constexpr int RF = BK / 4, RH = BK / 8;   // fp32 / bf16 16-byte items per row-major row
  // A tile: row-major [BM][RM_STR] (FWD, WGRAD) or k-major [PBK][BM+32] (DGRAD)
  // B tile: k-major [PBK][BN+32] (FWD, DGRAD) or row-major [BN][RM_STR] (WGRAD)
  constexpr bool A_KMAJ = (MODE == PW_DGRAD);
  constexpr bool B_KMAJ = (MODE != PW_WGRAD);
  constexpr int A_STR = A_KMAJ ? BM + 32 : RM_STR;
  constexpr int B_STR = B_KMAJ ? BN + 32 : RM_STR;
  constexpr int A_SZ = A_KMAJ ? BK * A_STR : BM * A_STR;
  constexpr int B_SZ = B_KMAJ ? BK * B_STR : BN * B_STR;
  constexpr bool DM = NS > 0;
  static_assert(!DM || (ABF && BBF && BK == 32 && NS >= 2), "LDS-DMA ring: 16-bit operands, 32-deep K steps");
  constexpr int DA_SZ = BM * BK, DB_SZ = BK * BN;   // DMA stage images (elements)
  __shared__ __attribute__((aligned(1024))) T16 smem[DM ? NS * (DA_SZ + DB_SZ) : 2 * (A_SZ + B_SZ)];

  // wave index through readfirstlane: the compiler then knows it is uniform (SGPR), so
  // per-wave row offsets can be scalar soffsets instead of readfirstlane waterfall loops
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- tile decode (1-D grid, XCD-aware, M-tile fastest; see igemm.hip) ----
  const int mt = (g.M + BM - 1) / BM;
  const int nt = (MODE == PW_WGRAD) ? (g.N + BN - 1) / BN : g.N / BN;
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
  if (g.k_split > 0) { kbeg = split * g.k_split; kend = min(g.K, kbeg + g.k_split); }
  if (kbeg >= kend) return;
  const int nk = (kend - kbeg + BK - 1) / BK;

  // FWD/DGRAD: the N tile lies inside one image (P % BN == 0)
  const int bimg = (MODE == PW_WGRAD) ? 0 : n0 / g.P;
  const int p0 = (MODE == PW_WGRAD) ? 0 : n0 - bimg * g.P;

  // ---- staging maps ----
  // row-major tiles: item = (row, c4) with c4 in [0,8): 8 float4 per 32-k row
  // k-major tiles  : item = (k, c4) with c4 in [0, C/4)
  constexpr int A_ITEMS = BK * BM / (ABF ? 8 : 4) / NT;
  constexpr int B_ITEMS = BK * BN / (BBF ? 8 : 4) / NT;
  static_assert(A_ITEMS * NT * (ABF ? 8 : 4) == BK * BM && B_ITEMS * NT * (BBF ? 8 : 4) == BK * BN, "staging split");
  float4 ra[ABF ? 1 : A_ITEMS], rb[BBF ? 1 : B_ITEMS];
  pu32x4 rha[ABF ? A_ITEMS : 1], rhb[BBF ? B_ITEMS : 1];
  float asr[A_ITEMS];   // WGRAD asum: this thread's running row sums of its A items (fixed order)
#pragma unroll
  for (int i = 0; i < A_ITEMS; ++i) asr[i] = 0.f;

  // Operand loads are 16-byte buffer loads: an element outside its tensor gets the offset
  // PW_OOB, past every resource range, and reads 0 in hardware -- no branch, no mask VALU.
  // (A select of the address followed by a select of the value is turned back into a branch
  // around the load by the compiler; see igemm.hip ldsel.)
  const int b_fix = (MODE == PW_WGRAD) ? 0 : bimg;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, (short)0, g.a_range, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const char*)g.B + (long)b_fix * g.b_bs * (BBF ? 2 : 4)), (short)0, g.b_range, 0x00020000);
  auto bld4 = [](__amdgpu_buffer_rsrc_t r, unsigned voff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0));
  };
  auto bldh = [](__amdgpu_buffer_rsrc_t r, unsigned voff) {
    return __builtin_bit_cast(pu32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0));
  };

  auto gload = [&](int kt) {
    const int kb = kbeg + kt * BK;
    // WGRAD: a BK-pixel K step lies inside one image (P % BK == 0): image index is uniform
    const unsigned bw = (MODE == PW_WGRAD) ? (unsigned)(kb / g.P) : 0u;
    const unsigned pw = (MODE == PW_WGRAD) ? (unsigned)(kb - (int)bw * g.P) : 0u;
    if constexpr (ABF) {   // bf16 A, 8 elements per item
#pragma unroll
      for (int i = 0; i < A_ITEMS; ++i) {
        const int it = tid + i * NT;
        unsigned off;
        if (MODE == PW_FWD) {                    // W[M][K] bf16, row m, k = kb + c8*8
          const int m = m0 + it / RH, k = kb + (it % RH) * 8;
          off = ((m < g.M) & (k < kend)) ? ((unsigned)m * g.K + k) * 2u : PW_OOB;
        } else if (MODE == PW_DGRAD) {           // W[K][M] bf16, row k (k >= K is past the range)
          const int k = kb + it / (BM / 8), m = m0 + (it % (BM / 8)) * 8;
          off = (m < g.M) ? ((unsigned)k * g.M + m) * 2u : PW_OOB;
        } else {                                 // DY[b][M][P] bf16, row m, 8 pixels per item
          const int m = m0 + it / RH;
          off = (m < g.M) ? (bw * (unsigned)g.a_bs + (unsigned)m * g.P + pw + (it % RH) * 8) * 2u : PW_OOB;
        }
        rha[i] = bldh(rA, off);
      }
    } else
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * NT;
      unsigned off;
      if (MODE == PW_FWD) {                      // W[M][K], row m, k = kb + c4*4
        const int m = m0 + it / RF, k = kb + (it % RF) * 4;
        off = ((m < g.M) & (k < kend)) ? ((unsigned)m * g.K + k) * 4u : PW_OOB;
      } else if (MODE == PW_DGRAD) {             // W[K][M], row k (k >= K is past the range)
        const int k = kb + it / (BM / 4), m = m0 + (it % (BM / 4)) * 4;
        off = (m < g.M) ? ((unsigned)k * g.M + m) * 4u : PW_OOB;
      } else {                                   // DY[b][M][P], row m
        const int m = m0 + it / RF;
        off = (m < g.M) ? (bw * (unsigned)g.a_bs + (unsigned)m * g.P + pw + (it % RF) * 4) * 4u : PW_OOB;
      }
      ra[i] = bld4(rA, off);
    }
    if constexpr (BBF && MODE != PW_WGRAD) {     // X/DY[b][K][P] bf16, k-major: row k, 8 pixels per item
#pragma unroll
      for (int i = 0; i < B_ITEMS; ++i) {
        const int it = tid + i * NT;
        const int k = kb + it / (BN / 8);
        rhb[i] = bldh(rB, ((unsigned)k * g.P + p0 + (it % (BN / 8)) * 8) * 2u);
      }
    } else if constexpr (BBF) {                  // X[b][N][P] bf16, row n
#pragma unroll
      for (int i = 0; i < B_ITEMS; ++i) {
        const int it = tid + i * NT;
        const int n = n0 + it / RH;
        const unsigned off = (n < g.N) ? (bw * (unsigned)g.b_bs + (unsigned)n * g.P + pw + (it % RH) * 8) * 2u : PW_OOB;
        rhb[i] = bldh(rB, off);
      }
    } else
#pragma unroll
    for (int i = 0; i < B_ITEMS; ++i) {
      const int it = tid + i * NT;
      unsigned off;
      if (MODE != PW_WGRAD) {                    // [K][P] k-major (k >= K is past the range)
        const int k = kb + it / (BN / 4);
        off = ((unsigned)k * g.P + p0 + (it % (BN / 4)) * 4) * 4u;
      } else {                                   // X[b][N][P], row n
        const int n = n0 + it / RF;
        off = (n < g.N) ? (bw * (unsigned)g.b_bs + (unsigned)n * g.P + pw + (it % RF) * 4) * 4u : PW_OOB;
      }
      rb[i] = bld4(rB, off);
    }
  };
  auto sstore = [&](int buf) {
    T16* As = smem + buf * (A_SZ + B_SZ);
    T16* Bs = As + A_SZ;
    if constexpr (ABF) {
#pragma unroll
      for (int i = 0; i < A_ITEMS; ++i) {
        const int it = tid + i * NT;
        const int off = A_KMAJ ? (it / (BM / 8)) * A_STR + (it % (BM / 8)) * 8 : (it / RH) * A_STR + (it % RH) * 8;
        *reinterpret_cast<pu32x4*>(As + off) = rha[i];
        if (MODE == PW_WGRAD && g.asum) {
          const pbf16x8 hv = __builtin_bit_cast(pbf16x8, rha[i]);
          asr[i] += (((float)hv[0] + (float)hv[1]) + ((float)hv[2] + (float)hv[3])) +
                    (((float)hv[4] + (float)hv[5]) + ((float)hv[6] + (float)hv[7]));
        }
      }
    } else
#pragma unroll
    for (int i = 0; i < A_ITEMS; ++i) {
      const int it = tid + i * NT;
      int off;
      if (A_KMAJ) off = (it / (BM / 4)) * A_STR + (it % (BM / 4)) * 4;
      else off = (it / RF) * A_STR + (it % RF) * 4;
      *reinterpret_cast<pbf16x4*>(As + off) = cvt4<T16>(ra[i], 0, 0.f);
      if (MODE == PW_WGRAD && g.asum) asr[i] += (ra[i].x + ra[i].y) + (ra[i].z + ra[i].w);
    }
    auto bstore = [&](auto cv) {
#pragma unroll
      for (int i = 0; i < B_ITEMS; ++i) {
        const int it = tid + i * NT;
        int off;
        if (B_KMAJ) off = (it / (BN / 4)) * B_STR + (it % (BN / 4)) * 4;
        else off = (it / RF) * B_STR + (it % RF) * 4;
        // WGRAD rows past N (a thin operand, e.g. a 12-channel hidden) read 0: skip their
        // conversion / activation-on-load (whole waves branch around it)
        if (MODE == PW_WGRAD && n0 + it / RF >= g.N) *reinterpret_cast<pbf16x4*>(Bs + off) = pbf16x4{};
        else *reinterpret_cast<pbf16x4*>(Bs + off) = cv(rb[i]);
      }
    };
    if constexpr (BBF && MODE != PW_WGRAD) {
#pragma unroll
      for (int i = 0; i < B_ITEMS; ++i) {
        const int it = tid + i * NT;
        *reinterpret_cast<pu32x4*>(Bs + (it / (BN / 8)) * B_STR + (it % (BN / 8)) * 8) = rhb[i];
      }
      return;
    } else if constexpr (BBF) {
#pragma unroll
      for (int i = 0; i < B_ITEMS; ++i) {
        const int it = tid + i * NT;
        *reinterpret_cast<pu32x4*>(Bs + (it / RH) * B_STR + (it % RH) * 8) = rhb[i];
      }
      return;
    }
    // activation-on-load switch hoisted out of the element loop (uniform)
    if (g.bact == ACT_NONE) bstore([](float4 v) { return cvt4<T16>(v, 0, 0.f); });
    else if (g.bact == ACT_GELU)
      bstore([](float4 v) {
        return cvt4<T16>(make_float4(gelu_f(v.x), gelu_f(v.y), gelu_f(v.z), gelu_f(v.w)), 0, 0.f);
      });
    else bstore([&](float4 v) { return cvt4<T16>(v, g.bact, g.slope); });
  };

  // ---- accumulators (bias folded into the init for FWD) ----
  pf32x16 acc[TM][TN];
  const bool has_bias = MODE == PW_FWD && g.bias != nullptr && g.ws == nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = 0.f;
    if (has_bias) {   // one uniform branch; guarded loads are clamp + select (see igemm.hip ldsel)
#pragma unroll
      for (int r = 0; r < 16; ++r) {   // SW: lane lr's channel; else row (r&3) + 8(r>>2) + 4lh
        const int m = m0 + wm * TM * 32 + i * 32 + (SW ? lr : (r & 3) + 8 * (r >> 2) + 4 * lh);
        const float t = g.bias[m < g.M ? m : 0];
        bv[r] = m < g.M ? t : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = bv[r];
  }

  if constexpr (!DM) {
    gload(0);
    sstore(0);
    __syncthreads();
  }

  // per-lane fragment address parts for the transposed reads:
  // lane = 32h + 16G + 4q + p supplies row (8h + q) and column 16G + 4p of its 16-column block
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;

  // DGRAD * 16-bit gp (the unfused blocks' dz = (W2^T dy) gelu'(z)): this tile's gp values are
  // loaded here, before the K loop, into TM*TN*4 8-byte registers -- their HBM latency then hides
  // behind the whole loop instead of opening the epilogue (the short-K data-grads run 8-16 K steps).
  // Same lanes / offsets as the SW epilogue below.  (TM*TN*8 VGPRs: 128 / 64-row 4-wave tiles only.)
  constexpr bool GPF = SW && MODE == PW_DGRAD && WN == 2 && BM <= 128;   // (register room: 4-wave tiles)
  const bool gpf_on = GPF && g.gp_pref && g.gpre && g.gbf && !g.ws;
  uint2 gpf[GPF ? TM * TN * 4 : 1];
  if constexpr (GPF) {
    if (gpf_on) {
      const unsigned grange = (unsigned)(((long)g.M * g.P - p0) * 2);
      const __amdgpu_buffer_rsrc_t rgp = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)g.gpre + ((long)bimg * g.gpre_bs + p0) * 2), (short)0, grange, 0x00020000);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int col0 = wn * TN * 32 + j * 32;
          const int mrow = m0 + wm * TM * 32 + i * 32;
          const bool ok = mrow + lr < g.M;
          const int v2 = ok ? (lr * g.P + col0 + 4 * lh) * 2 : (int)PW_OOB;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const auto u = __builtin_amdgcn_raw_buffer_load_b64(rgp, v2, mrow * g.P * 2 + 16 * q, 0);
            gpf[(j * TM + i) * 4 + q] = make_uint2(u[0], u[1]);
          }
        }
    }
  }

  if constexpr (DM) {
    // ---- LDS-DMA ring ----
    constexpr int NW = NT / 64;
    constexpr int AP = DA_SZ / 8 / NT, BP = DB_SZ / 8 / NT;   // 16-byte pieces per lane per stage
    constexpr int PI = AP + BP;                               // DMA instructions per wave per stage
    static_assert(AP * 8 * NT == DA_SZ && BP * 8 * NT == DB_SZ, "DMA pieces");
    // per-lane source offsets (elements, stage-invariant part) of this lane's pieces
    unsigned aoff[AP], boff[BP];
#pragma unroll
    for (int i = 0; i < AP; ++i) {
      const int pc = (i * NW + wave) * 64 + lane;
      if constexpr (A_KMAJ) {          // DGRAD W[K][M]: k-major [32][BM]
        const int k = pc / (BM / 8), ls = (pc % (BM / 8)) ^ pw_kswz(k);
        aoff[i] = (unsigned)(k * g.M + m0 + 8 * ls);
      } else {                         // FWD W[M][K] / WGRAD DY[b][M][P]: rows [BM][32]
        const int r = pc >> 2, ls = (pc & 3) ^ pw_rswz(r);
        aoff[i] = (unsigned)((m0 + r) * (MODE == PW_WGRAD ? g.P : g.K) + 8 * ls);
      }
    }
#pragma unroll
    for (int i = 0; i < BP; ++i) {
      const int pc = (i * NW + wave) * 64 + lane;
      if constexpr (B_KMAJ) {          // X / DY [b][K][P]: k-major [32][BN]
        const int k = pc / (BN / 8), ls = (pc % (BN / 8)) ^ pw_kswz(k);
        boff[i] = (unsigned)(k * g.P + p0 + 8 * ls);
      } else {                         // WGRAD X[b][N][P]: rows [BN][32]
        const int r = pc >> 2, ls = (pc & 3) ^ pw_rswz(r);
        boff[i] = (unsigned)((n0 + r) * g.P + 8 * ls);
      }
    }
    const T16* Ag = (const T16*)g.A;
    const T16* Bg = (const T16*)g.B + (long)b_fix * g.b_bs;
    auto issue = [&](int kt) __attribute__((always_inline)) {
      const int kb = kbeg + kt * BK;
      T16* As = smem + (kt % NS) * (DA_SZ + DB_SZ);
      T16* Bs = As + DA_SZ;
      unsigned ua, ub;                 // stage-dependent uniform element offsets
      if constexpr (MODE == PW_WGRAD) {
        const int bw = kb / g.P, pw = kb - bw * g.P;
        ua = (unsigned)(bw * g.a_bs + pw);
        ub = (unsigned)(bw * g.b_bs + pw);
      } else {
        ua = A_KMAJ ? (unsigned)kb * g.M : (unsigned)kb;
        ub = (unsigned)kb * g.P;
      }
#pragma unroll
      for (int i = 0; i < AP; ++i) dma16(Ag + (ua + aoff[i]), lds_off(As + (i * NW + wave) * 512));
#pragma unroll
      for (int i = 0; i < BP; ++i) dma16(Bg + (ub + boff[i]), lds_off(Bs + (i * NW + wave) * 512));
    };
    // fragment read offsets (bytes, K-step invariant)
    unsigned ar[TM];
    uint2 at[TM], bt[TN];
    unsigned br[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = wm * TM * 32 + i * 32;
      if constexpr (A_KMAJ) at[i] = pw_tr_addr<BM / 8>(mb, lane);
      else ar[i] = (unsigned)((mb + lr) * 64 + ((lh ^ pw_rswz(mb + lr)) << 4));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nbb = wn * TN * 32 + j * 32;
      if constexpr (B_KMAJ) bt[j] = pw_tr_addr<BN / 8>(nbb, lane);
      else br[j] = (unsigned)((nbb + lr) * 64 + ((lh ^ pw_rswz(nbb + lr)) << 4));
    }
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nk) issue(s);
    auto mma = [&](const pbf16x8 (&af)[TM], const pbf16x8 (&bfr)[TN]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = SW ? mfma16(bfr[j], af[i], acc[i][j]) : mfma16(af[i], bfr[j], acc[i][j]);
    };
    for (int kt = 0; kt < nk; ++kt) {
      // stage kt landed: this wave's later stages (at most NS - 2) may stay in flight
      const int later = min(NS - 2, nk - 1 - kt);
      if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PI) : "memory");
      else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      static_assert(NS <= 4, "vmcnt ladder covers <= 2 later stages");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();   // every wave's pieces of stage kt landed; slot (kt-1) % NS is free
      if (kt + NS - 1 < nk) issue(kt + NS - 1);
      const T16* As = smem + (kt % NS) * (DA_SZ + DB_SZ);
      const T16* Bs = As + DA_SZ;
      if constexpr (MODE == PW_WGRAD) {
        if (g.asum) {   // the register path's row sums: this thread's A items, read from the landed stage
#pragma unroll
          for (int i = 0; i < A_ITEMS; ++i) {
            const int it = tid + i * NT, r = it / RH, c8 = it % RH;
            const pbf16x8 hv = *reinterpret_cast<const pbf16x8*>(As + r * BK + ((c8 ^ pw_rswz(r)) << 3));
            asr[i] += (((float)hv[0] + (float)hv[1]) + ((float)hv[2] + (float)hv[3])) +
                      (((float)hv[4] + (float)hv[5]) + ((float)hv[6] + (float)hv[7]));
          }
        }
      }
      auto frags = [&](int ks, pbf16x8 (&af)[TM], pbf16x8 (&bfr)[TN]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (A_KMAJ) af[i] = pw_tr_at(As, at[i], ks * 16 * BM * 2);
          else af[i] = *reinterpret_cast<const pbf16x8*>((const char*)As + (ar[i] ^ (unsigned)(32 * ks)));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (B_KMAJ) bfr[j] = pw_tr_at(Bs, bt[j], ks * 16 * BN * 2);
          else bfr[j] = *reinterpret_cast<const pbf16x8*>((const char*)Bs + (br[j] ^ (unsigned)(32 * ks)));
        }
      };
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        pbf16x8 af[TM], bfr[TN];
        frags(ks, af, bfr);
        mma(af, bfr);
      }
    }
  } else
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const T16* As = smem + buf * (A_SZ + B_SZ);
    const T16* Bs = As + A_SZ;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      pbf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mb = wm * TM * 32 + i * 32;
        if (A_KMAJ)
          af[i] = tr_frag(As + (ks * 16 + 8 * lh + tq) * A_STR + mb + 16 * tG + 4 * tp, A_STR);
        else
          af[i] = *reinterpret_cast<const pbf16x8*>(As + (mb + lr) * A_STR + ks * 16 + lh * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nbb = wn * TN * 32 + j * 32;
        if (B_KMAJ)
          bfr[j] = tr_frag(Bs + (ks * 16 + 8 * lh + tq) * B_STR + nbb + 16 * tG + 4 * tp, B_STR);
        else
          bfr[j] = *reinterpret_cast<const pbf16x8*>(Bs + (nbb + lr) * B_STR + ks * 16 + lh * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = SW ? mfma16(bfr[j], af[i], acc[i][j]) : mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  if (MODE == PW_WGRAD) {
    if (g.asum) {
      // the threads of one A row (4 bf16 / 8 fp32 items per 32-pixel row) are adjacent lanes:
      // butterfly over them; the n-tile-0 workgroup writes (its split's partial, or db += when unsplit)
      constexpr int RT = ABF ? RH : RF;
#pragma unroll
      for (int i = 0; i < A_ITEMS; ++i) {
        float t = asr[i];
        t += __shfl_xor(t, 1, 64); t += __shfl_xor(t, 2, 64);
        if (RT >= 8) t += __shfl_xor(t, 4, 64);
        if (RT >= 16) t += __shfl_xor(t, 8, 64);
        const int it = tid + i * NT, m = m0 + it / RT;
        if (n_t == 0 && it % RT == 0 && m < g.M) {
          if (g.ws) g.ws[(long)gridDim.x / mt / nt * g.M * g.N + (long)split * g.M + m] = t;
          else g.asum[m] += t;
        }
      }
    }
    // splits > 1: this split's partial tile (plain stores); one split: the only writer, +=
    float* dst = g.ws ? g.ws + (long)split * g.M * g.N : g.Y;
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
  pw_fd_epi<T16, BM, TM, TN, SW, GPF>(g, acc, m0, bimg, p0, split, wm, wn, lr, lh, gpf_on, gpf);
}

template <typename T16, int MODE, int BM, int ABF = 0, int BBF = 0, int BN = 128, int WN = 2, int BK = PBK, int SWP = 0,
          int NS = 0>
static void pw_launch(const PwArgs& g, int splits, hipStream_t st) {
  const int mt = (g.M + BM - 1) / BM;
  const int nt = (MODE == PW_WGRAD) ? (g.N + BN - 1) / BN : g.N / BN;
  ktimer_mark(st, 0);
  hipLaunchKernelGGL((pwgemm_kernel<T16, MODE, BM, ABF, BBF, BN, WN, BK, SWP, NS>),
                     dim3((unsigned)((long)mt * nt * splits)), dim3(128 * WN), 0, st, g);
  ktimer_mark(st, 1);
}

constexpr int PW_WIDE = -1;   // tile selector: 256 x 256 tiles, 8 waves, 64-deep K steps

// FWD / DGRAD launch over (tile rows, bf16 weight, bf16 activation, 16-bit output)
template <typename T16, int MODE, int SWP>
static void pw_launch_abs(const PwArgs& g, int bm, int abf, int bbf, int splits, hipStream_t st) {
  const int sel = (abf ? 2 : 0) + (bbf ? 1 : 0);
#define PW_AB_K(BM, BK)                                                \
  switch (sel) {                                                       \
    case 0: pw_launch<T16, MODE, BM, 0, 0, 128, 2, BK, SWP>(g, splits, st); break;                \
    case 1: pw_launch<T16, MODE, BM, 0, 1, 128, 2, BK, SWP>(g, splits, st); break;                \
    case 2: pw_launch<T16, MODE, BM, 1, 0, 128, 2, BK, SWP>(g, splits, st); break;                \
    default: pw_launch<T16, MODE, BM, 1, 1, 128, 2, BK, SWP>(g, splits, st); break;               \
  }
#define PW_AB(BM) PW_AB_K(BM, PBK)
#define PW_ABW                                                                    \
  switch (sel) {                                                                  \
    case 0: pw_launch<T16, MODE, 128, 0, 0, 128, 2, PBK, SWP>(g, 1, st); break;  /* (not selected) */  \
    case 1: pw_launch<T16, MODE, 256, 0, 1, 256, 4, 64, SWP>(g, 1, st); break;              \
    case 2: pw_launch<T16, MODE, 256, 1, 0, 256, 4, 64, SWP>(g, 1, st); break;              \
    default:                                                                      \
      if (g.dma == 2) pw_launch<T16, MODE, 256, 1, 1, 128, 2, 32, SWP, 3>(g, 1, st);   \
      else if (g.dma) pw_launch<T16, MODE, 256, 1, 1, 256, 4, 32, SWP, 4>(g, 1, st);   \
      else pw_launch<T16, MODE, 256, 1, 1, 256, 4, 64, SWP>(g, 1, st);                 \
      break;                                                                      \
  }
  if (bm == PW_WIDE) { PW_ABW } else if (bm == 256) { PW_AB(256) } else if (bm == 128) { PW_AB(128) } else { PW_AB(64) }
#undef PW_AB
#undef PW_AB_K
#undef PW_ABW
}

// Finishing pass of a split-K FWD / DGRAD launch: y = epilogue(sum_s ws[s], s = 0..S-1 in order),
// the kernel epilogue's operations in the same order (bias; DGRAD: * act'(gpre) or * 16-bit gp;
// FWD: 16-bit act'(pre) / fp32 pre-activation to ypre, then act; accumulate; fp32 or 16-bit store),
// four consecutive pixels of one (image, channel) row per thread (P % 4 == 0).
template <typename T16>
__global__ __launch_bounds__(256) void pw_split_finish_kernel(PwArgs g, int S, int mode) {
  const long MN = (long)g.M * g.N, n4 = MN >> 2;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < n4; q += (long)gridDim.x * 256) {
    const long e = q << 2;
    float4 a = *reinterpret_cast<const float4*>(g.ws + e);
    for (int s = 1; s < S; ++s) {
      const float4 u = *reinterpret_cast<const float4*>(g.ws + (long)s * MN + e);
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
    const long bm = e / g.P;
    const int p = (int)(e - bm * g.P), m = (int)(bm % g.M), b = (int)(bm / g.M);
    const long off = (long)m * g.P + p;
    if (mode == PW_FWD && g.bias) {
      const float bv = g.bias[m];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bv;
    }
    if (mode == PW_DGRAD && g.gpre) {
      if (g.gbf) {
        const uint2 u = *reinterpret_cast<const uint2*>((const T16*)g.gpre + (long)b * g.gpre_bs + off);
        v[0] *= h2f<T16>((unsigned short)(u.x & 0xffffu)); v[1] *= h2f<T16>((unsigned short)(u.x >> 16));
        v[2] *= h2f<T16>((unsigned short)(u.y & 0xffffu)); v[3] *= h2f<T16>((unsigned short)(u.y >> 16));
      } else {
        const float4 u = *reinterpret_cast<const float4*>(g.gpre + (long)b * g.gpre_bs + off);
        const float gv[4] = {u.x, u.y, u.z, u.w};
        act_g_mul_arr(g.gact, v, gv, g.slope);
      }
    }
    if (mode == PW_FWD) {
      if (g.ypre && g.gbf) {
        float apv[4];
        if (g.act == ACT_GELU) {
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            f32x2 ga, gpa;
            gelu_pair_fast2(f32x2{v[r], v[r + 1]}, ga, gpa);
            v[r] = ga.x; v[r + 1] = ga.y; apv[r] = gpa.x; apv[r + 1] = gpa.y;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) { apv[r] = act_g(g.act, v[r], g.slope); v[r] = act_f(g.act, v[r], g.slope); }
        }
        *reinterpret_cast<uint2*>((T16*)g.ypre + (long)b * g.ypre_bs + off) =
            make_uint2((unsigned)f2h<T16>(apv[0]) | ((unsigned)f2h<T16>(apv[1]) << 16),
                       (unsigned)f2h<T16>(apv[2]) | ((unsigned)f2h<T16>(apv[3]) << 16));
      } else {
        if (g.ypre) *reinterpret_cast<float4*>(g.ypre + (long)b * g.ypre_bs + off) = make_float4(v[0], v[1], v[2], v[3]);
        act_f_arr(g.act, v, g.slope);
      }
    }
    if (g.y_bf16) {
      *reinterpret_cast<uint2*>((T16*)g.Y + (long)b * g.y_bs + off) =
          make_uint2((unsigned)f2h<T16>(v[0]) | ((unsigned)f2h<T16>(v[1]) << 16),
                     (unsigned)f2h<T16>(v[2]) | ((unsigned)f2h<T16>(v[3]) << 16));
    } else {
      float4* o = reinterpret_cast<float4*>(g.Y + (long)b * g.y_bs + off);
      if (g.accumulate) { const float4 y = *o; v[0] += y.x; v[1] += y.y; v[2] += y.z; v[3] += y.w; }
      *o = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

template <typename T16, int MODE>
static void pw_launch_ab(const PwArgs& g, int bm, int abf, int bbf, int splits, hipStream_t st) {
  if (splits > 1) {   // raw fp32 partials (the channel x pixel tile), then the finishing pass
    pw_launch_abs<T16, MODE, 0>(g, bm, abf, bbf, splits, st);
    const long n4 = (long)g.M * g.N / 4;
    long blocks = (n4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL((pw_split_finish_kernel<T16>), dim3((unsigned)blocks), dim3(256), 0, st, g, splits, MODE);
    return;
  }
  if (g.y_bf16 || (g.ypre && g.gbf)) pw_launch_abs<T16, MODE, 1>(g, bm, abf, bbf, 1, st);
  else pw_launch_abs<T16, MODE, 0>(g, bm, abf, bbf, 1, st);
}

// K (pixel) split of a weight-grad launch: about `target` workgroups (640 = 2.5 per CU for the
// 4-wave tiles: enough bytes in flight to stream HBM; 256 = one per CU for the 8-wave wide
// tiles), >= 8 K steps each, and partials of at most a quarter of the operand bytes (each split
// writes, and the reduce reads, an M x N fp32 tile) -- that cap yielding to a one-workgroup-per-CU
// floor: a deep weight-grad over few tiles (1024 x 2048 at 16^2, 128 tiles) is worth the traffic.
static int wgrad_plan(int M, int N, long K, int BM, int BN, int BK, long target, int* k_split) {
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  long splits = (target + tiles - 1) / tiles;
  const long max_splits = (K + 8L * BK - 1) / (8L * BK);
  long byte_cap = ((long)(M + N) * K) / (4L * M * N);
  const long floor_splits = (256 + tiles - 1) / tiles;
  if (byte_cap < floor_splits) byte_cap = floor_splits;
  if (splits > max_splits) splits = max_splits;
  if (splits > byte_cap) splits = byte_cap;
  if (splits < 1) splits = 1;
  long ks = (K + splits - 1) / splits;
  ks = (ks + BK - 1) / BK * BK;
  splits = (K + ks - 1) / ks;
  *k_split = (int)ks;
  return (int)splits;
}

// Weight-grad tile choice: 256 x 256 x 64 (8 waves) for the wide, deep ones (both sides >= 256
// channels), else 128 (64) x 128 x 32.
static bool wgrad_wide(int M, int N, int P) {
  return M >= 256 && N >= 256 && P % 64 == 0 && (M % 256 == 0 || M >= 1024) && (N % 256 == 0 || N >= 1024);
}
// (fp32-only operands stay on the 4-wave tiles: the wide tile's fp32 staging spills)
static int wgrad_cfg(PwArgs& g, bool any_bf16, int* bm) {
  if (any_bf16 && wgrad_wide(g.M, g.N, g.P)) { *bm = PW_WIDE; return wgrad_plan(g.M, g.N, g.K, 256, 256, 64, 256, &g.k_split); }
  *bm = g.M > 64 ? 128 : 64;
  return wgrad_plan(g.M, g.N, g.K, *bm, 128, PBK, 640, &g.k_split);
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// 256-row M tiles for the wide, deep FWD / DGRAD GEMMs: each staged pixel tile feeds twice the
// MFMAs, as long as the grid still keeps >= 2 workgroups per CU.  Isolated A/B at the step's
// shapes (tools/gpu_pw256_micro.sh, B=16): K=4096 dgrad into 1024 ch 0.356 -> 0.264 ms, K=1024
// fwd to 4096 ch 0.380 -> 0.342 ms; with K <= 512 the halved occupancy loses (K=256: +10 %),
// hence K >= 1024.  (WGRAD keeps 128-row tiles: 256 rows measured 4-7 % slower on the step's
// wide weight-grads, tools/gpu_pw256wg_micro.sh -- they already stream at ~5 TB/s.)
static bool use_bm256(const PwArgs& g) {
  return g.M >= 1024 && g.M % 256 == 0 && g.K >= 1024 && (long)(g.M / 256) * (g.N / 128) >= 512;
}
// 256 x 256 x 64 tiles (8 waves, one workgroup per CU) for the wide FWD / DGRAD GEMMs of the
// unfused blocks: 256-pixel tiles inside one image, M a multiple of 256, a grid of >= 256 tiles.
static bool use_wide(const PwArgs& g) {
  return g.M % 256 == 0 && g.P % 256 == 0 && g.K >= 128 && (long)(g.M / 256) * (g.N / 256) >= 256;
}
// (Not for the gp-multiplied data-grad: there one 8-wave workgroup per CU leaves the epilogue's
// 2-byte gp loads exposed.)
// The gelu-pair forward (bf16 act(z) and act'(z) out, packed-fp32 GELU) now measures faster on the
// wide tiles too (tools/pwio_micro.py, B=16: M=2048 K=512 at 64^2 0.455 -> 0.383 ms, M=4096 K=1024 at
// 32^2 0.256 -> 0.227 ms); the gp-multiplied data-grad stays on 128-row tiles (wide: +5-20 %,
// tools/pwdgrad_micro.py).
static int fd_tile(const PwArgs& g, bool any_bf16) {
  const bool plain = !g.ypre && !g.gpre;
  const bool gelu_pair = g.ypre && g.gbf;
  return any_bf16 && (plain || gelu_pair) && use_wide(g) ? PW_WIDE : use_bm256(g) ? 256 : g.M > 64 ? 128 : 64;
}


// Launch entry points per (16-bit operand type, mode), each explicitly instantiated in a
// translation unit of its own (pw_{fwd,dgrad,wgrad}_{bf16,f16}.hip) so the six kernel families
// compile in parallel.
template <typename T16, int MODE>
void pw_fd_launch_m(const PwArgs& g, int bm, int abf, int bbf, int splits, hipStream_t st) {
  pw_launch_ab<T16, MODE>(g, bm, abf, bbf, splits, st);
}
template <typename T16>
void pw_wgrad_launch(const PwArgs& g, int bm, int abf, int bbf, int splits, hipStream_t st) {
  const int sel = (abf ? 2 : 0) + (bbf ? 1 : 0) + (bm == 128 ? 4 : bm == PW_WIDE ? 8 : 0);
  switch (sel) {
    case 9: pw_launch<T16, PW_WGRAD, 256, 0, 1, 256, 4, 64>(g, splits, st); break;
    case 10: pw_launch<T16, PW_WGRAD, 256, 1, 0, 256, 4, 64>(g, splits, st); break;
    case 11:
      if (g.dma == 2) pw_launch<T16, PW_WGRAD, 256, 1, 1, 128, 2, 32, 0, 3>(g, splits, st);
      else if (g.dma) pw_launch<T16, PW_WGRAD, 256, 1, 1, 256, 4, 32, 0, 4>(g, splits, st);
      else pw_launch<T16, PW_WGRAD, 256, 1, 1, 256, 4, 64>(g, splits, st);
      break;
    case 0: pw_launch<T16, PW_WGRAD, 64, 0, 0>(g, splits, st); break;
    case 1: pw_launch<T16, PW_WGRAD, 64, 0, 1>(g, splits, st); break;
    case 2: pw_launch<T16, PW_WGRAD, 64, 1, 0>(g, splits, st); break;
    case 3: pw_launch<T16, PW_WGRAD, 64, 1, 1>(g, splits, st); break;
    case 4: pw_launch<T16, PW_WGRAD, 128, 0, 0>(g, splits, st); break;
    case 5: pw_launch<T16, PW_WGRAD, 128, 0, 1>(g, splits, st); break;
    case 6: pw_launch<T16, PW_WGRAD, 128, 1, 0>(g, splits, st); break;
    default: pw_launch<T16, PW_WGRAD, 128, 1, 1>(g, splits, st); break;
  }
}
#define PW_EXTERN_LAUNCHERS(T16)                                                                            \
  extern template void pw_fd_launch_m<T16, PW_FWD>(const PwArgs&, int, int, int, int, hipStream_t);         \
  extern template void pw_fd_launch_m<T16, PW_DGRAD>(const PwArgs&, int, int, int, int, hipStream_t);       \
  extern template void pw_wgrad_launch<T16>(const PwArgs&, int, int, int, int, hipStream_t);

}  // namespace dsg
