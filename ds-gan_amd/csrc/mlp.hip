// Fused ConvNeXt pointwise MLP (Block.pwconv1 -> GELU -> pwconv2, DSGAN/models/model/MixConvNeXtML.py:
// 221-223,236-240) on bf16 MFMA (gfx950).  The 4C-channel hidden activation never touches HBM.
//
//   forward : out[b][p][n] (+)= b2[p] + sum_m W2[p][m] * gelu( b1[m] + sum_c W1[m][c] h[b][c][n] )
//   backward: z = W1 h + b1 (recomputed), t = W2^T dy, dz = t * gelu'(z), g = gelu(z)
//             dh = W1^T dz                           (fp32, to the InstanceNorm backward)
//             g, dz -> HBM as bf16                   (operands of the two weight-grads)
//             bsum[tile][m] = sum_n dz[m][n]         (per-tile partials of the b1 grad)
//
// One workgroup owns BN pixels of one image.  Its activation tile(s) are staged once into LDS
// (bf16, k-major, read with ds_read_b64_tr_b16); the hidden dimension is walked in chunks of HC:
// per chunk the W1 rows and W2 columns are staged into LDS (register-prefetched one chunk
// ahead), GEMM1 produces the chunk of z in accumulators, the GELU epilogue writes it to LDS,
// and GEMM2 (forward) / GEMM-dh (backward) consumes it from there.  Per-pixel HBM traffic is
// C + P fp32 values forward (vs 2*(4C) + C + 2P unfused) -- the kernel is HBM/LDS bound, not
// MFMA bound, for every DS-GAN shape.
//
// Weights are bf16 copies (w1 [4C][C] as nn.Linear stores it, w2 [P][4C]); the same two LDS
// chunk layouts serve the transposed products of the backward through the transposing LDS read.
#include "common.h"
#include <type_traits>

namespace dsg {

typedef f32x16_t mf32x16;
typedef __attribute__((ext_vector_type(4))) short ms16x4;
typedef __attribute__((address_space(3))) ms16x4 lds_ms16x4;
typedef __attribute__((ext_vector_type(4))) unsigned int mu32x4;   // raw 16 bytes

// Fragment of a k-major LDS tile T[k][col] (row stride STR elements) for a 32x32x16 MFMA
// operand: lane (h = lane>>5, c = lane&31) receives T[8h + i][c], i = 0..7, via two
// ds_read_b64_tr_b16 (see pwgemm.hip).  `p` = T + (ks*16 + 8h + q)*STR + colbase + 16G + 4p.
template <typename T16>
__device__ __forceinline__ hx8<T16> mtr_frag(const T16* p0, int stride) {
#if defined(__HIP_DEVICE_COMPILE__)
  ms16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(p0));
  ms16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(p0 + 4 * stride));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}

template <typename T16>
__device__ __forceinline__ hx4<T16> mcvt4(float4 v) {
  hx4<T16> r;
  r[0] = (T16)v.x; r[1] = (T16)v.y; r[2] = (T16)v.z; r[3] = (T16)v.w;
  return r;
}

// GELU of the bf16 path: gelu_fast2 / gelu_pair_fast2 (common.h, A&S 7.1.26 erfc on packed fp32,
// two elements per instruction; the exact branch-free erf of gelu_f costs ~40 VALU per element).
// Packed (gelu_fast2 / gelu_pair_fast2) or unpacked (gelu_fast1x2 / gelu_pair_fast1x2) fp32 GELU:
// the same operations and bits; which issues faster depends on the MFMAs around it.  In-process
// build A/B (tools/mlp_micro.py --libs, profiles/r04/mlp_micro_pk.txt): the unpacked form is 8 % /
// 4 % faster in the weight-grad kernel at (C, P) = (256, 128) / (128, 256), where each hidden
// element's GELU sits between more MFMAs; every other kernel and shape is 1-3 % faster packed.
template <bool PK>
__device__ __forceinline__ f32x2 mlp_gelu2(f32x2 z) { return PK ? gelu_fast2(z) : gelu_fast1x2(z); }
template <bool PK>
__device__ __forceinline__ void mlp_gelu_pair2(f32x2 z, f32x2& g, f32x2& gp) {
  if (PK) gelu_pair_fast2(z, g, gp);
  else gelu_pair_fast1x2(z, g, gp);
}
template <bool PK>
__device__ __forceinline__ f32x2 mlp_mul2(f32x2 a, f32x2 b) { return PK ? a * b : f32x2{a.x * b.x, a.y * b.y}; }

struct MlpArgs {
  const void* h; long h_bs;         // [nb][C][HW]   block activation after InstanceNorm (fp32, or bf16 if h_bf16)
  const float* dy; long dy_bs;      // [nb][P][HW]   (backward) upstream grad of the block output
  const void* w1;                   // [4C][C]   (16-bit: the library's half type)
  const float* b1;                  // [4C]
  const void* w2;                   // [P][4C]
  const float* b2;                  // [P]           (forward; may be null)
  float* out; long out_bs;          // forward: out [nb][P][HW] (+= when accumulate); backward: dh [nb][C][HW]
  void* g_out;                      // (backward) gelu(z)  [nb][4C][HW]
  void* dz_out;                     // (backward) dz       [nb][4C][HW]
  float* bsum;                      // (backward) [ntiles][4C] per-tile sums of dz
  int HW, nb, accumulate;
  int h_bf16;
  float* ws;                        // (weight-grad kernel) per-split partials, see mlp_wgrad_kernel
  int splits;
};

__device__ __forceinline__ int xcd_tile(int id, int nwg) {
  // consecutive tiles on one XCD (dispatch round-robins workgroups over the 8 XCDs)
  const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
}

// Stage a [K][BN] fp32 tile (rows strided by HW) into a k-major bf16 LDS tile [K][STR].
template <int K, int BN, int STR, int NT, typename T16>
__device__ __forceinline__ void stage_rows(T16* dst, const float* __restrict__ src, int HW, int tid) {
  constexpr int ITEMS = K * BN / 4;
  static_assert(ITEMS % NT == 0, "tile must split evenly over the workgroup");
  constexpr int PER = ITEMS / NT;
  constexpr int BATCH = PER < 8 ? PER : 8;
#pragma unroll
  for (int i0 = 0; i0 < PER; i0 += BATCH) {
    float4 v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int it = tid + (i0 + i) * NT;
      const int k = it / (BN / 4), c4 = it % (BN / 4);
      v[i] = *reinterpret_cast<const float4*>(src + (long)k * HW + c4 * 4);
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int it = tid + (i0 + i) * NT;
      const int k = it / (BN / 4), c4 = it % (BN / 4);
      *reinterpret_cast<hx4<T16>*>(dst + k * STR + c4 * 4) = mcvt4<T16>(v[i]);
    }
  }
}

// Same, from a bf16 source (the InstanceNorm's bf16 output): 16-byte items copied unconverted.
template <int K, int BN, int STR, int NT, typename T16>
__device__ __forceinline__ void stage_rows_h16(T16* dst, const T16* __restrict__ src, int HW, int tid) {
  constexpr int ITEMS = K * BN / 8;
  static_assert(ITEMS % NT == 0, "tile must split evenly over the workgroup");
  constexpr int PER = ITEMS / NT;
  constexpr int BATCH = PER < 8 ? PER : 8;
#pragma unroll
  for (int i0 = 0; i0 < PER; i0 += BATCH) {
    mu32x4 v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int it = tid + (i0 + i) * NT;
      const int k = it / (BN / 8), c8 = it % (BN / 8);
      v[i] = *reinterpret_cast<const mu32x4*>(src + (long)k * HW + c8 * 8);
    }
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      const int it = tid + (i0 + i) * NT;
      const int k = it / (BN / 8), c8 = it % (BN / 8);
      *reinterpret_cast<mu32x4*>(dst + k * STR + c8 * 8) = v[i];
    }
  }
}

template <int K, int BN, int STR, int NT, typename T16>
__device__ __forceinline__ void stage_h(T16* dst, const MlpArgs& g, int img, int p0, int tid) {
  if (g.h_bf16) stage_rows_h16<K, BN, STR, NT>(dst, (const T16*)g.h + (long)img * g.h_bs + p0, g.HW, tid);
  else stage_rows<K, BN, STR, NT>(dst, (const float*)g.h + (long)img * g.h_bs + p0, g.HW, tid);
}

// Register-staged weight chunk j: W1 rows [j*HC, +HC) (all C columns) and W2 columns
// [j*HC, +HC) (all P rows), 16-byte items.  (Plain native-vector register arrays: a struct of
// HIP uint4 arrays is demoted to scratch/LDS by the compiler.)
template <int C, int P, int HC, int NT>
struct WCh {
  static constexpr int N1 = HC * C / 8 / NT, N2 = P * HC / 8 / NT;
  static_assert((HC * C / 8) % NT == 0 && (P * HC / 8) % NT == 0, "weight chunk split");
};

template <int C, int P, int HC, int NT, int N1, int N2>
__device__ __forceinline__ void wch_load(mu32x4 (&r1)[N1], mu32x4 (&r2)[N2], const void* w1v, const void* w2v, int j,
                                         int tid) {
  // raw 16-bit elements: the loads move bits, the half type does not matter here
  const unsigned short* __restrict__ w1 = (const unsigned short*)w1v;
  const unsigned short* __restrict__ w2 = (const unsigned short*)w2v;
  const mu32x4* s1 = reinterpret_cast<const mu32x4*>(w1 + (long)j * HC * C);
#pragma unroll
  for (int i = 0; i < N1; ++i) r1[i] = s1[tid + i * NT];
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    const int it = tid + i * NT, row = it / (HC / 8), c8 = it % (HC / 8);
    r2[i] = *reinterpret_cast<const mu32x4*>(w2 + (long)row * (4 * C) + j * HC + c8 * 8);
  }
}

template <int C, int P, int HC, int NT, int W1STR, int W2STR, int N1, int N2, typename T16>
__device__ __forceinline__ void wch_store(const mu32x4 (&r1)[N1], const mu32x4 (&r2)[N2], T16* W1s, T16* W2s,
                                          int tid) {
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int it = tid + i * NT, row = it / (C / 8), c8 = it % (C / 8);
    *reinterpret_cast<mu32x4*>(W1s + row * W1STR + c8 * 8) = r1[i];
  }
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    const int it = tid + i * NT, row = it / (HC / 8), c8 = it % (HC / 8);
    *reinterpret_cast<mu32x4*>(W2s + row * W2STR + c8 * 8) = r2[i];
  }
}

// wch_load through buffer loads: one lane VGPR offset per matrix, the item and chunk steps in the
// scalar offset (the flat form keeps a 64-bit address per item live across the chunk loop)
template <int C, int P, int HC, int NT, int N1, int N2>
__device__ __forceinline__ void wch_load_buf(mu32x4 (&r1)[N1], mu32x4 (&r2)[N2], __amdgpu_buffer_rsrc_t rw1,
                                             __amdgpu_buffer_rsrc_t rw2, int j, int tid) {
  static_assert(NT % (HC / 8) == 0, "W2 rows per item step");
  const int v1 = tid * 16, v2 = (tid / (HC / 8)) * (4 * C) * 2 + (tid % (HC / 8)) * 16;
#pragma unroll
  for (int i = 0; i < N1; ++i)
    r1[i] = __builtin_bit_cast(mu32x4, __builtin_amdgcn_raw_buffer_load_b128(rw1, v1, j * HC * C * 2 + i * NT * 16, 0));
#pragma unroll
  for (int i = 0; i < N2; ++i)
    r2[i] = __builtin_bit_cast(mu32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rw2, v2, j * HC * 2 + i * (NT / (HC / 8)) * (4 * C) * 2, 0));
}

// Wave grid of a [M x N] product over NW waves: 2 waves along M, NW/2 along N, each wave
// TM x TN tiles of 32x32.
template <int M, int N, int NW>
struct WGrid {
  static constexpr int WN = NW / 2, TM = M / 64, TN = N / 32 / WN;
  static_assert(M % 64 == 0 && N % (32 * WN) == 0 && TM >= 1 && TN >= 1, "wave grid");
};

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// Hidden-row order of the forward's W1 chunk: rows 16a + 4b + e with quads b = 1 and 2 swapped.
// Lane half h of a 32x32 accumulator holds rows 8q + 4h + e; with this order the rows it holds for
// q = 2kk, 2kk+1 are the LOGICAL hidden units 16kk + 8h + (0..7) -- exactly the k slice of a B
// fragment -- so gelu(z) feeds the second GEMM straight from registers against W2 in its natural
// layout.  (An involution: the same map takes logical rows back to physical ones.)
__device__ __forceinline__ int qswap(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

// XOR swizzle of the 16-byte slots of an unpadded LDS row of S slots, conflict-free for both
// readers of these tiles: ds_read_b128 of one logical slot by 16 consecutive rows (16 distinct bank
// groups), and ds_read_b64_tr_b16 of 4 consecutive slots (4-aligned) by 4 consecutive rows
// (4-aligned; the 32 lanes then cover the 64 banks once).  256-byte+ rows (S >= 16): rows 4i..4i+3
// take XOR masks 4(r & 3) + ((r >> 2) & 3).  128-byte rows (S = 8; two rows per bank window): the
// two rows of equal parity among 4 consecutive ones differ by mask bit 2.
template <int S>
__device__ __forceinline__ int slot_swz(int r) {
  return S >= 16 ? (((r & 3) << 2) | ((r >> 2) & 3)) : ((((r >> 1) & 1) << 2) | ((r >> 2) & 3));
}
// element offset of (row r, column c) in an unpadded [rows][S*8] tile with slot_swz'd 16-byte slots
template <int S>
__device__ __forceinline__ int swz_off(int r, int c) {
  return r * (S * 8) + ((((c >> 3) ^ slot_swz<S>(r))) << 3) + (c & 7);
}
// wch_store into unpadded, swizzled chunk images: W1s [HC][C] (slots slot_swz<C/8>), W2s [P][HC]
// (slot_swz<HC/8>): conflict-free for the row reads (ds_read_b128) AND the transposed reads
// (ds_read_b64_tr_b16) both backward kernels make of them (tools/lds_banks.py; the padded images
// were 2-4-way on the transposed reads)
template <int C, int P, int HC, int NT, int N1, int N2, typename T16>
__device__ __forceinline__ void wch_store_swz(const mu32x4 (&r1)[N1], const mu32x4 (&r2)[N2], T16* W1s, T16* W2s,
                                              int tid) {
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int it = tid + i * NT, row = it / (C / 8), c8 = it % (C / 8);
    *reinterpret_cast<mu32x4*>(W1s + row * C + ((c8 ^ slot_swz<C / 8>(row)) << 3)) = r1[i];
  }
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    const int it = tid + i * NT, row = it / (HC / 8), c8 = it % (HC / 8);
    *reinterpret_cast<mu32x4*>(W2s + row * HC + ((c8 ^ slot_swz<HC / 8>(row)) << 3)) = r2[i];
  }
}

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at LDS byte
// address lds + 16 l.  Issued from asm so that hipcc neither counts it nor drains it with a
// vmcnt(0) in front of every LDS read of the other buffer: completion is waited for by hand
// (s_waitcnt vmcnt + barrier before the buffer is read).  M0 is written and restored in the same
// statement (it is compiler-reserved).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {   // LDS byte offset of a __shared__ pointer
  return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)p);
}

// Weight chunk j -> LDS by LDS-DMA (no register staging): W1 rows [j*64, +64) as [64][C] (in qswap
// row order when QS), W2 columns [j*64, +64) as [P][64].  Every wave issues C/64 + P/64 wave-instructions
// of 1 KB each; the LDS image of one instruction is lane-linear, the swizzle is applied on the
// per-lane global source address.
template <int C, int P, int NW, bool QS = true>
__device__ __forceinline__ void glds_chunk(void* W1d, void* W2d, const void* w1v, const void* w2v, int j, int wave,
                                           int lane) {
  const unsigned short* __restrict__ w1 = (const unsigned short*)w1v;   // raw 16-bit elements
  const unsigned short* __restrict__ w2 = (const unsigned short*)w2v;
  unsigned short* const W1h = (unsigned short*)W1d;
  unsigned short* const W2h = (unsigned short*)W2d;
  constexpr int S1 = C / 8, R1 = 64 / S1, N1 = C / 8 / NW;
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int inst = wave * N1 + i, r = inst * R1 + lane / S1, ps = lane % S1;
    const unsigned short* src = w1 + ((long)j * 64 + (QS ? qswap(r) : r)) * C + (ps ^ slot_swz<S1>(r)) * 8;
    glds16(src, lds_addr(W1h + inst * 512));
  }
  constexpr int N2 = P / 8 / NW;
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    const int inst = wave * N2 + i, r = inst * 8 + lane / 8, ps = lane % 8;
    const unsigned short* src = w2 + (long)r * (4 * C) + j * 64 + (ps ^ slot_swz<8>(r)) * 8;
    glds16(src, lds_addr(W2h + inst * 512));
  }
}

// 8 waves = 2 (hidden half wm of the 64-row chunk) x 4 (32-pixel column wn of the 128-pixel tile).
// Each wave keeps the B fragments of its h columns (all C channels) in registers for the whole
// tile, so per chunk LDS serves only the weight A fragments: z (32 x 32 per wave) = W1[chunk]
// h + b1 on MFMA, gelu in registers (packed fp32), out[:, wn cols] += W2[:, wave's 32 hidden]
// gelu(z) (see qswap).  The two hidden halves' partial outputs meet once, through LDS, in a fixed
// order (acc[wm 0] + acc[wm 1]: deterministic).  Weight chunks are double-buffered and filled by
// LDS-DMA one chunk ahead: one barrier per chunk.
template <typename T16, int C, int P, int MINB>
__global__ __launch_bounds__(512, MINB) void mlp_fwd_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int NW = 8, NT = NW * 64, BN = 128, HC = 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC, KS = C / 16, PT = P / 32;
  constexpr int HSTR = BN + 32;
  constexpr int H_SZ = C * HSTR, W_SZ = HC * C + P * HC, R_SZ = 2 * 4 * PT * 16 * 64;   // bf16 elements
  constexpr int SM = H_SZ > 2 * W_SZ ? (H_SZ > R_SZ ? H_SZ : R_SZ) : (2 * W_SZ > R_SZ ? 2 * W_SZ : R_SZ);
  __shared__ __attribute__((aligned(16))) T16 smem[SM + 2 * (C4 + P)];
  float* b1s = reinterpret_cast<float*>(smem + SM);   // b1 [C4], then b2 [P]: no global load is in
  float* b2s = b1s + C4;                              // flight in the loop besides the LDS-DMA
  static_assert(C % 64 == 0 && P % 64 == 0 && NCH >= 2, "tile shape");

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave >> 2, wn = wave & 3;

  const int tpi = g.HW / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int img = tile / tpi, p0 = (tile - img * tpi) * BN;

  stage_h<C, BN, HSTR, NT>(smem, g, img, p0, tid);
  for (int i = tid; i < C4; i += NT) b1s[i] = g.b1[i];
  for (int i = tid; i < P; i += NT) b2s[i] = g.b2 ? g.b2[i] : 0.f;
  __syncthreads();
  mbf16x8 hb[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    hb[ks] = mtr_frag(smem + (ks * 16 + 8 * lh + tq) * HSTR + wn * 32 + 16 * tG + 4 * tp, HSTR);
  mf32x16 oacc[PT];
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      oacc[pt][r] = wm == 0 ? b2s[pt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] : 0.f;
  __syncthreads();   // the h staging area becomes the weight double buffer
  glds_chunk<C, P, NW>(smem, smem + HC * C, g.w1, g.w2, 0, wave, lane);
  glds_chunk<C, P, NW>(smem + W_SZ, smem + W_SZ + HC * C, g.w1, g.w2, 1, wave, lane);
  constexpr int NI = C / 8 / NW + P / 8 / NW;   // LDS-DMA instructions per wave per chunk
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NI) : "memory");   // chunk 0 landed (chunk 1 may still fly)
  raw_barrier();

  for (int j = 0; j < NCH; ++j) {
    const T16* W1c = smem + (j & 1) * W_SZ;
    const T16* W2c = W1c + HC * C;
    mf32x16 zacc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // bias of physical rows wm*32 + 8q + 4lh + e (qswap order)
      const float4 bv = *reinterpret_cast<const float4*>(b1s + j * HC + qswap(wm * 32 + 8 * q + 4 * lh));
      zacc[4 * q] = bv.x; zacc[4 * q + 1] = bv.y; zacc[4 * q + 2] = bv.z; zacc[4 * q + 3] = bv.w;
    }
    const int r1 = wm * 32 + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const mbf16x8 a =
          *reinterpret_cast<const mbf16x8*>(W1c + r1 * C + ((ks * 2 + lh) ^ slot_swz<C / 8>(r1)) * 8);
      zacc = mfma16(a, hb[ks], zacc);
    }
    // gelu of k slice kk -> its GEMM2 MFMAs (the second slice's VALU overlaps the first's MFMAs)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      mbf16x8 gb;
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        const f32x2 v = mlp_gelu2<true>(f32x2{zacc[8 * kk + i], zacc[8 * kk + i + 1]});
        gb[i] = (T16)v.x;
        gb[i + 1] = (T16)v.y;
      }
#pragma unroll
      for (int pt = 0; pt < PT; ++pt) {
        const int r2 = pt * 32 + lr;
        const mbf16x8 a = *reinterpret_cast<const mbf16x8*>(
            W2c + r2 * HC + ((wm * 4 + kk * 2 + lh) ^ slot_swz<8>(r2)) * 8);
        oacc[pt] = mfma16(a, gb, oacc[pt]);
      }
    }
    // chunk j+1 landed (each wave waits for its own DMA; the barrier makes all of it visible) and
    // every wave is done reading buffer j&1 -> refill it with chunk j+2
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (j + 2 < NCH) {
      T16* W1n = smem + (j & 1) * W_SZ;
      glds_chunk<C, P, NW>(W1n, W1n + HC * C, g.w1, g.w2, j + 2, wave, lane);
    }
  }

  // ---- epilogue: wave (wm, wn) finishes the tiles pt with pt % 2 == wm and parks the others ----
  float* red = reinterpret_cast<float*>(smem);   // [wn][pt][16][64]
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
    if ((pt & 1) != wm)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wn * PT + pt) * 16 + r) * 64 + lane] = oacc[pt][r];
  __syncthreads();
  float* ob = g.out + (long)img * g.out_bs + p0 + wn * 32 + lr;
#pragma unroll
  for (int pt = 0; pt < PT; ++pt)
    if ((pt & 1) == wm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float o = red[((wn * PT + pt) * 16 + r) * 64 + lane];
        const float v = wm == 0 ? oacc[pt][r] + o : o + oacc[pt][r];   // acc[wm 0] + acc[wm 1]
        float* d = ob + (long)(pt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * g.HW;
        *d = g.accumulate ? *d + v : v;
      }
}

// Forward for small C (C = 64: only 4 hidden chunks per tile, where the register-resident h of
// mlp_fwd_kernel costs the second workgroup per CU): h staged once into LDS and read by every
// chunk's GEMM1; gelu(z) goes through an LDS chunk buffer (aliasing the W1 chunk) to GEMM2; weight
// chunks register-prefetched one chunk ahead.
template <typename T16, int C, int P, int BN, int HC, int NW, int MINB>
__global__ __launch_bounds__(NW * 64, MINB) void mlp_fwd_lds_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int NT = NW * 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC;
  constexpr int HSTR = BN + 32, GSTR = HC + 8, W1STR = C + 8, W2STR = HC + 8;
  constexpr int H_SZ = C * HSTR, G_SZ = BN * GSTR, W1_SZ = HC * W1STR, W2_SZ = P * W2STR;
  // the g chunk overwrites the W1 chunk once GEMM1 is done with it
  constexpr int GW_SZ = G_SZ > W1_SZ ? G_SZ : W1_SZ;
  __shared__ __attribute__((aligned(16))) T16 smem[H_SZ + GW_SZ + W2_SZ];
  T16* Hs = smem;
  T16* Gs = Hs + H_SZ;
  T16* W1s = Gs;
  T16* W2s = Gs + GW_SZ;

  using ZG = WGrid<HC, BN, NW>;   // z chunk [HC x BN]
  using OG = WGrid<P, BN, NW>;    // out tile [P x BN]
  static_assert(C % 32 == 0, "C");

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave / ZG::WN, wn = wave % ZG::WN;   // same split for both grids (2 x NW/2)

  const int tpi = g.HW / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int img = tile / tpi, p0 = (tile - img * tpi) * BN;

  using WC = WCh<C, P, HC, NT>;
  mu32x4 wr1[WC::N1], wr2[WC::N2];
  wch_load<C, P, HC, NT>(wr1, wr2, g.w1, g.w2, 0, tid);
  stage_h<C, BN, HSTR, NT>(Hs, g, img, p0, tid);
  wch_store<C, P, HC, NT, W1STR, W2STR>(wr1, wr2, W1s, W2s, tid);

  mf32x16 oacc[OG::TM][OG::TN];
#pragma unroll
  for (int i = 0; i < OG::TM; ++i) {
    float bv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
      bv[r] = g.b2 ? g.b2[wm * (P / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] : 0.f;
#pragma unroll
    for (int t = 0; t < OG::TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[i][t][r] = bv[r];
  }
  __syncthreads();

  for (int j = 0; j < NCH; ++j) {
    if (j + 1 < NCH) wch_load<C, P, HC, NT>(wr1, wr2, g.w1, g.w2, j + 1, tid);
    // ---- GEMM1: z = W1[chunk] h + b1 ----
    mf32x16 zacc[ZG::TM][ZG::TN];
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i) {
      float bv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) bv[r] = g.b1[j * HC + wm * (HC / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh];
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) zacc[i][t][r] = bv[r];
    }
#pragma unroll 4
    for (int ks = 0; ks < C / 16; ++ks) {
      mbf16x8 af[ZG::TM], bf[ZG::TN];
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
        af[i] = *reinterpret_cast<const mbf16x8*>(W1s + (wm * (HC / 2) + i * 32 + lr) * W1STR + ks * 16 + lh * 8);
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
        bf[t] = mtr_frag(Hs + (ks * 16 + 8 * lh + tq) * HSTR + wn * (BN / ZG::WN) + t * 32 + 16 * tG + 4 * tp, HSTR);
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
        for (int t = 0; t < ZG::TN; ++t)
          zacc[i][t] = mfma16(af[i], bf[t], zacc[i][t]);
    }
    __syncthreads();   // every wave is done reading W1s (Gs aliases it)
    // ---- GELU -> Gs (pixel-major [BN][GSTR]) ----
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t) {
        const int n = wn * (BN / ZG::WN) + t * 32 + lr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          mbf16x4 v;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 gv = mlp_gelu2<true>(f32x2{zacc[i][t][4 * q + e], zacc[i][t][4 * q + e + 1]});
            v[e] = (T16)gv.x;
            v[e + 1] = (T16)gv.y;
          }
          *reinterpret_cast<mbf16x4*>(Gs + n * GSTR + wm * (HC / 2) + i * 32 + 8 * q + 4 * lh) = v;
        }
      }
    __syncthreads();
    // ---- GEMM2: out += W2[:, chunk] g ----
#pragma unroll
    for (int ks = 0; ks < HC / 16; ++ks) {
      mbf16x8 af[OG::TM], bf[OG::TN];
#pragma unroll
      for (int i = 0; i < OG::TM; ++i)
        af[i] = *reinterpret_cast<const mbf16x8*>(W2s + (wm * (P / 2) + i * 32 + lr) * W2STR + ks * 16 + lh * 8);
#pragma unroll
      for (int t = 0; t < OG::TN; ++t)
        bf[t] = *reinterpret_cast<const mbf16x8*>(Gs + (wn * (BN / OG::WN) + t * 32 + lr) * GSTR + ks * 16 + lh * 8);
#pragma unroll
      for (int i = 0; i < OG::TM; ++i)
#pragma unroll
        for (int t = 0; t < OG::TN; ++t)
          oacc[i][t] = mfma16(af[i], bf[t], oacc[i][t]);
    }
    __syncthreads();
    if (j + 1 < NCH) {
      wch_store<C, P, HC, NT, W1STR, W2STR>(wr1, wr2, W1s, W2s, tid);
      __syncthreads();
    }
  }

  // ---- epilogue ----
  float* ob = g.out + (long)img * g.out_bs + p0;
#pragma unroll
  for (int i = 0; i < OG::TM; ++i)
#pragma unroll
    for (int t = 0; t < OG::TN; ++t) {
      const int n = wn * (BN / OG::WN) + t * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wm * (P / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        float* o = ob + (long)m * g.HW + n;
        *o = g.accumulate ? *o + oacc[i][t][r] : oacc[i][t][r];
      }
    }
}


// Transposed 32x32x16 operand fragment of a swizzled [rows][S*8] LDS tile (k = row): lane (c, h)
// receives T[k0 + 4h + i][col0 + c] (i < 4) and T[k0 + 8 + 4h + i - 4][col0 + c] (i >= 4) -- the k
// order in which a 32x32 accumulator lane half holds rows 16kk + {4h + e, 8 + 4h + e}, so that
// accumulator, converted, is the matching B fragment (see mlp_dh_kernel).
template <int S, typename T16>
__device__ __forceinline__ hx8<T16> mtr_frag_q(const T16* T, int k0, int col0, int lane) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1, h = lane >> 5;
  const int col = col0 + 16 * tG + 4 * tp;
  const int rlo = k0 + 4 * h + tq, rhi = rlo + 8;
  const T16* plo = T + rlo * (S * 8) + (((col >> 3) ^ slot_swz<S>(rlo)) << 3) + (col & 7);
  const T16* phi = T + rhi * (S * 8) + (((col >> 3) ^ slot_swz<S>(rhi)) << 3) + (col & 7);
  ms16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(plo));
  ms16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(phi));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}
// Same, plain k order: lane (c, h) receives T[k0 + 8h + i][col0 + c], i = 0..7.
template <int S, typename T16>
__device__ __forceinline__ hx8<T16> mtr_frag_s(const T16* T, int k0, int col0, int lane) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1, h = lane >> 5;
  const int col = col0 + 16 * tG + 4 * tp;
  const int rlo = k0 + 8 * h + tq, rhi = rlo + 4;
  const T16* plo = T + rlo * (S * 8) + (((col >> 3) ^ slot_swz<S>(rlo)) << 3) + (col & 7);
  const T16* phi = T + rhi * (S * 8) + (((col >> 3) ^ slot_swz<S>(rhi)) << 3) + (col & 7);
  ms16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(plo));
  ms16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(phi));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}

// ------------------------------------------------------------------------------------------
// backward, data path only: dh = W1^T (W2^T dy * gelu'(W1 h + b1))
// ------------------------------------------------------------------------------------------
// Same decomposition as mlp_fwd_kernel: 8 waves = 2 hidden halves (wm) x 4 pixel columns (wn) of a
// 128-pixel tile.  Each wave holds the B fragments of its h AND dy columns in registers; per
// 64-row hidden chunk (weights double-buffered in LDS by LDS-DMA, natural order):
//   z = W1 h + b1, t = W2^T dy (A fragments by row / transposed LDS reads), dz = t gelu'(z) in
//   registers (packed fp32), dh[:, wn cols] += W1^T dz with dz as the B operand straight from the
//   accumulators (mtr_frag_q reads W1 in the accumulator's k order).
// The two hidden halves' partial dh meet once, through LDS, in a fixed order (deterministic).
template <typename T16, int C, int P, int MINB>
__global__ __launch_bounds__(512, MINB) void mlp_dh_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int NW = 8, NT = NW * 64, BN = 128, HC = 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC, KS = C / 16, PS = P / 16, CT = C / 32;
  constexpr int HSTR = BN + 32;
  constexpr int ST_SZ = (C + P) * HSTR, W_SZ = HC * C + P * HC, R_SZ = 2 * 4 * CT * 16 * 64;   // bf16 elements
  constexpr int SM = ST_SZ > 2 * W_SZ ? (ST_SZ > R_SZ ? ST_SZ : R_SZ) : (2 * W_SZ > R_SZ ? 2 * W_SZ : R_SZ);
  __shared__ __attribute__((aligned(16))) T16 smem[SM + 2 * C4];
  float* b1s = reinterpret_cast<float*>(smem + SM);
  static_assert(C % 64 == 0 && P % 64 == 0 && NCH >= 2, "tile shape");

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave >> 2, wn = wave & 3;

  const int tpi = g.HW / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int img = tile / tpi, p0 = (tile - img * tpi) * BN;

  T16* Hs = smem;
  T16* Ds = smem + C * HSTR;
  stage_h<C, BN, HSTR, NT>(Hs, g, img, p0, tid);
  stage_rows<P, BN, HSTR, NT>(Ds, g.dy + (long)img * g.dy_bs + p0, g.HW, tid);
  for (int i = tid; i < C4; i += NT) b1s[i] = g.b1[i];
  __syncthreads();
  mbf16x8 hb[KS], db[PS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    hb[ks] = mtr_frag(Hs + (ks * 16 + 8 * lh + tq) * HSTR + wn * 32 + 16 * tG + 4 * tp, HSTR);
#pragma unroll
  for (int ks = 0; ks < PS; ++ks)
    db[ks] = mtr_frag(Ds + (ks * 16 + 8 * lh + tq) * HSTR + wn * 32 + 16 * tG + 4 * tp, HSTR);
  mf32x16 hacc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[ct][r] = 0.f;
  __syncthreads();   // the staging area becomes the weight double buffer
  glds_chunk<C, P, NW, false>(smem, smem + HC * C, g.w1, g.w2, 0, wave, lane);
  glds_chunk<C, P, NW, false>(smem + W_SZ, smem + W_SZ + HC * C, g.w1, g.w2, 1, wave, lane);
  constexpr int NI = C / 8 / NW + P / 8 / NW;
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NI) : "memory");
  raw_barrier();

  for (int j = 0; j < NCH; ++j) {
    const T16* W1c = smem + (j & 1) * W_SZ;
    const T16* W2c = W1c + HC * C;
    mf32x16 zacc, tacc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 bv = *reinterpret_cast<const float4*>(b1s + j * HC + wm * 32 + 8 * q + 4 * lh);
      zacc[4 * q] = bv.x; zacc[4 * q + 1] = bv.y; zacc[4 * q + 2] = bv.z; zacc[4 * q + 3] = bv.w;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) tacc[r] = 0.f;
    const int r1 = wm * 32 + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const mbf16x8 a =
          *reinterpret_cast<const mbf16x8*>(W1c + r1 * C + ((ks * 2 + lh) ^ slot_swz<C / 8>(r1)) * 8);
      zacc = mfma16(a, hb[ks], zacc);
    }
#pragma unroll
    for (int ks = 0; ks < PS; ++ks) {   // A[m = hidden][k = p] = W2[p][hidden]: transposed read of W2c
      const mbf16x8 a = mtr_frag_s<8>(W2c, ks * 16, wm * 32, lane);
      tacc = mfma16(a, db[ks], tacc);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      mbf16x8 dzb;
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        f32x2 gv, gp;
        mlp_gelu_pair2<true>(f32x2{zacc[8 * kk + i], zacc[8 * kk + i + 1]}, gv, gp);
        const f32x2 dz = mlp_mul2<true>(f32x2{tacc[8 * kk + i], tacc[8 * kk + i + 1]}, gp);
        dzb[i] = (T16)dz.x;
        dzb[i + 1] = (T16)dz.y;
      }
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {   // A[m = c][k = hidden] = W1[hidden][c], in dz's k order
        const mbf16x8 a = mtr_frag_q<C / 8>(W1c, wm * 32 + 16 * kk, ct * 32, lane);
        hacc[ct] = mfma16(a, dzb, hacc[ct]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (j + 2 < NCH) {
      T16* W1n = smem + (j & 1) * W_SZ;
      glds_chunk<C, P, NW, false>(W1n, W1n + HC * C, g.w1, g.w2, j + 2, wave, lane);
    }
  }

  float* red = reinterpret_cast<float*>(smem);   // [wn][ct][16][64]
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
    if ((ct & 1) != wm)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wn * CT + ct) * 16 + r) * 64 + lane] = hacc[ct][r];
  __syncthreads();
  float* ob = g.out + (long)img * g.out_bs + p0 + wn * 32 + lr;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
    if ((ct & 1) == wm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float o = red[((wn * CT + ct) * 16 + r) * 64 + lane];
        ob[(long)(ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * g.HW] = wm == 0 ? hacc[ct][r] + o : o + hacc[ct][r];
      }
}

// ------------------------------------------------------------------------------------------
// backward (data path): dh, g, dz, per-(tile, quarter) sums of dz
// ------------------------------------------------------------------------------------------
// GD: also write g and dz (bf16) and the b1 partial sums for the weight-grad GEMMs; without it the
// kernel writes dh only (mlp_wgrad_kernel recomputes what the weight path needs), drops the g
// chunk buffer and fits two workgroups per CU (MINB) where the tiles allow.
// DMA: the weight chunks arrive by LDS-DMA into a two-chunk ring (chunk j+1 lands while chunk j
// computes; the h / dy staging area becomes the second ring slot once their fragments are in
// registers), the b1 slice comes from LDS: one barrier fewer per chunk and no register staging of
// the weights.  Same operands, same order of every sum: same bits as the register-staged form.
template <typename T16, int C, int P, int BN, int HC, int NW, bool GD, int MINB, bool DMA = false>
__global__ __launch_bounds__(NW * 64, MINB) void mlp_bwd_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int NT = NW * 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC;
  // Hs / Ds padded (transposed reads only); Zn / Gn and the weight chunks unpadded + slot-swizzled
  constexpr int HSTR = BN + 32, NSTR = HC, W1STR = C, W2STR = HC;
  constexpr int H_SZ = C * HSTR, D_SZ = P * HSTR, N_SZ = BN * NSTR, W1_SZ = HC * W1STR, W2_SZ = P * W2STR;
  constexpr int W_SZ = W1_SZ + W2_SZ;
  static_assert(!DMA || (H_SZ + D_SZ >= W_SZ && HC == 64 && (C / 8) % NW == 0 && (P / 8) % NW == 0), "DMA ring");
  constexpr int SM_SZ = DMA ? H_SZ + D_SZ + W_SZ + (GD ? 2 : 1) * N_SZ + 2 * C4
                            : H_SZ + D_SZ + (GD ? 2 : 1) * N_SZ + W1_SZ + W2_SZ;
  __shared__ __attribute__((aligned(16))) T16 smem[SM_SZ];
  T16* Hs = smem;
  T16* Ds = Hs + H_SZ;
  // DMA: ring slot 0 after the staging area, then Zn / Gn, then b1 (fp32); slot 1 = the staging area
  T16* Zn = Ds + D_SZ + (DMA ? W_SZ : 0);   // dz chunk, pixel-major [BN][NSTR]
  T16* Gn = Zn + (GD ? N_SZ : 0);           // g chunk,  pixel-major [BN][NSTR] (GD only)
  T16* W1s = DMA ? Ds + D_SZ : Zn + (GD ? 2 : 1) * N_SZ;
  T16* W2s = W1s + W1_SZ;
  float* b1s = reinterpret_cast<float*>(Zn + (GD ? 2 : 1) * N_SZ);   // (DMA only)

  using ZG = WGrid<HC, BN, NW>;   // z / t chunk [HC x BN]
  using HG = WGrid<C, BN, NW>;    // dh tile [C x BN]
  static_assert(P % 16 == 0 && HC == 64 && BN % 16 == 0, "tile shape");
  // copy-out: blocks of 16 pixels x 32 hidden (one transposing read per lane)
  constexpr int CB = (BN / 16) * (HC / 32);
  static_assert(CB % NW == 0, "copy-out split");
  constexpr int CPW = CB / NW;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave / ZG::WN, wn = wave % ZG::WN;

  const int tpi = g.HW / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int img = tile / tpi, p0 = (tile - img * tpi) * BN;

  using WC = WCh<C, P, HC, NT>;
  mu32x4 wr1[DMA ? 1 : WC::N1], wr2[DMA ? 1 : WC::N2];
  if constexpr (DMA) {
    glds_chunk<C, P, NW, false>(W1s, W2s, g.w1, g.w2, 0, wave, lane);   // chunk 0 -> ring slot 0
    for (int i = tid; i < C4; i += NT) b1s[i] = g.b1[i];
  } else {
    wch_load<C, P, HC, NT>(wr1, wr2, g.w1, g.w2, 0, tid);
  }
  stage_h<C, BN, HSTR, NT>(Hs, g, img, p0, tid);
  stage_rows<P, BN, HSTR, NT>(Ds, g.dy + (long)img * g.dy_bs + p0, g.HW, tid);
  if constexpr (!DMA) wch_store_swz<C, P, HC, NT>(wr1, wr2, W1s, W2s, tid);

  mf32x16 hacc[HG::TM][HG::TN];
#pragma unroll
  for (int i = 0; i < HG::TM; ++i)
#pragma unroll
    for (int t = 0; t < HG::TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) hacc[i][t][r] = 0.f;
  __syncthreads();
  // The B fragments of this wave's pixel column of h (all C channels) and dy (all P) are the same for
  // every hidden chunk: read them from LDS once, keep them in registers (the z / t GEMMs then read only
  // their weight A fragments per MFMA; same operands, same order -- same bits)
  static_assert(ZG::TN == 1 && ZG::TM == 1, "one 32 x 32 z / t tile per wave");
  mbf16x8 hbr[C / 16], dbr[P / 16];
#pragma unroll
  for (int ks = 0; ks < C / 16; ++ks)
    hbr[ks] = mtr_frag(Hs + (ks * 16 + 8 * lh + tq) * HSTR + wn * (BN / ZG::WN) + 16 * tG + 4 * tp, HSTR);
#pragma unroll
  for (int ks = 0; ks < P / 16; ++ks)
    dbr[ks] = mtr_frag(Ds + (ks * 16 + 8 * lh + tq) * HSTR + wn * (BN / ZG::WN) + 16 * tG + 4 * tp, HSTR);

  // copy-out block of this wave: hidden half (wave & 1), pixel blocks (wave >> 1) * CPW + c
  const int chh = (wave & 1) * 32;
  const long gbase = (long)img * C4 * g.HW + p0;
  for (int j = 0; j < NCH; ++j) {
    if constexpr (DMA) {
      // chunk j has landed (this wave's pieces: the only LDS-DMA in flight) and every wave is done
      // with chunk j-1 (its ring slot, Zn / Gn, and at j = 0 the h / dy staging area = slot 1)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      raw_barrier();
      if (j + 1 < NCH) {
        T16* W1n = (j & 1) ? Ds + D_SZ : Hs;
        glds_chunk<C, P, NW, false>(W1n, W1n + W1_SZ, g.w1, g.w2, j + 1, wave, lane);
      }
      W1s = (j & 1) ? Hs : Ds + D_SZ;
      W2s = W1s + W1_SZ;
    } else {
      if (j + 1 < NCH) wch_load<C, P, HC, NT>(wr1, wr2, g.w1, g.w2, j + 1, tid);
    }
    // ---- z = W1[chunk] h + b1 ;  t = W2[:, chunk]^T dy ----
    mf32x16 zacc[ZG::TM][ZG::TN], tacc[ZG::TM][ZG::TN];
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i) {
      float bv[16];
      if constexpr (DMA) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 b4 = *reinterpret_cast<const float4*>(b1s + j * HC + wm * (HC / 2) + i * 32 + 8 * q + 4 * lh);
          bv[4 * q] = b4.x; bv[4 * q + 1] = b4.y; bv[4 * q + 2] = b4.z; bv[4 * q + 3] = b4.w;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = g.b1[j * HC + wm * (HC / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh];
      }
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) { zacc[i][t][r] = bv[r]; tacc[i][t][r] = 0.f; }
    }
#pragma unroll
    for (int ks = 0; ks < C / 16; ++ks) {
      const mbf16x8 af = *reinterpret_cast<const mbf16x8*>(W1s + swz_off<C / 8>(wm * (HC / 2) + lr, ks * 16 + lh * 8));
      zacc[0][0] = mfma16(af, hbr[ks], zacc[0][0]);
    }
#pragma unroll
    for (int ks = 0; ks < P / 16; ++ks) {   // A[m][p] = W2[p][m]: W2s [P][W2STR] is k-major for this product
      const mbf16x8 af = mtr_frag_s<HC / 8>(W2s, ks * 16, wm * (HC / 2), lane);
      tacc[0][0] = mfma16(af, dbr[ks], tacc[0][0]);
    }
    // ---- epilogue: g = gelu(z), dz = t * gelu'(z) -> LDS, pixel-major, 4 hidden per write ----
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t) {
        const int n = wn * (BN / ZG::WN) + t * 32 + lr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          mbf16x4 gv4, dv4;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            f32x2 gv, gp;
            mlp_gelu_pair2<true>(f32x2{zacc[i][t][4 * q + e], zacc[i][t][4 * q + e + 1]}, gv, gp);
            const f32x2 dz = mlp_mul2<true>(f32x2{tacc[i][t][4 * q + e], tacc[i][t][4 * q + e + 1]}, gp);
            gv4[e] = (T16)gv.x; gv4[e + 1] = (T16)gv.y;
            dv4[e] = (T16)dz.x; dv4[e + 1] = (T16)dz.y;
          }
          const int m = wm * (HC / 2) + i * 32 + 8 * q + 4 * lh;
          if constexpr (GD) *reinterpret_cast<mbf16x4*>(Gn + swz_off<HC / 8>(n, m)) = gv4;
          *reinterpret_cast<mbf16x4*>(Zn + swz_off<HC / 8>(n, m)) = dv4;
        }
      }
    if constexpr (DMA) {   // raw barrier: the next chunk's LDS-DMA stays in flight across it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    } else {
      __syncthreads();
    }
    // ---- copy-out: 8 pixels of one hidden row per lane (transposing read) -> 16-byte stores;
    //      per-(tile, wave>>1) sums of dz for the b1 grad.  Skipped (g_out == NULL) when the
    //      weight-grads come from mlp_wgrad_kernel instead. ----
    if constexpr (GD) {
      float bacc = 0.f;
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        const int pb = ((wave >> 1) * CPW + c) * 16;
        const mbf16x8 gv = mtr_frag_s<HC / 8>(Gn, pb, chh, lane);
        const mbf16x8 dv = mtr_frag_s<HC / 8>(Zn, pb, chh, lane);
        const long o = gbase + (long)(j * HC + chh + lr) * g.HW + pb + 8 * lh;
        *reinterpret_cast<mbf16x8*>((T16*)g.g_out + o) = gv;
        *reinterpret_cast<mbf16x8*>((T16*)g.dz_out + o) = dv;
#pragma unroll
        for (int e = 0; e < 8; ++e) bacc += (float)dv[e];
      }
      bacc += __shfl_xor(bacc, 32, 64);
      if (lh == 0 && g.bsum) g.bsum[((long)tile * (NW / 2) + (wave >> 1)) * C4 + j * HC + chh + lr] = bacc;
    }
    // ---- dh += W1[chunk]^T dz ----
#pragma unroll
    for (int ks = 0; ks < HC / 16; ++ks) {
      mbf16x8 af[HG::TM], bf[HG::TN];
#pragma unroll
      for (int i = 0; i < HG::TM; ++i)   // A[c][m] = W1[m][c]: W1s [HC][W1STR] is k-major here
        af[i] = mtr_frag_s<C / 8>(W1s, ks * 16, wm * (C / 2) + i * 32, lane);
#pragma unroll
      for (int t = 0; t < HG::TN; ++t)
        bf[t] = *reinterpret_cast<const mbf16x8*>(Zn + swz_off<HC / 8>(wn * (BN / HG::WN) + t * 32 + lr, ks * 16 + lh * 8));
#pragma unroll
      for (int i = 0; i < HG::TM; ++i)
#pragma unroll
        for (int t = 0; t < HG::TN; ++t)
          hacc[i][t] = mfma16(af[i], bf[t], hacc[i][t]);
    }
    if constexpr (!DMA) {
      __syncthreads();
      if (j + 1 < NCH) {
        wch_store_swz<C, P, HC, NT>(wr1, wr2, W1s, W2s, tid);
        __syncthreads();
      }
    }
  }

  float* ob = g.out + (long)img * g.out_bs + p0;
#pragma unroll
  for (int i = 0; i < HG::TM; ++i)
#pragma unroll
    for (int t = 0; t < HG::TN; ++t) {
      const int n = wn * (BN / HG::WN) + t * 32 + lr;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = wm * (C / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        ob[(long)c * g.HW + n] = hacc[i][t][r];
      }
    }
}

// ------------------------------------------------------------------------------------------
// LDS addressing with few live registers: every address of a slot-swizzled tile is one XOR or one
// immediate offset away from a per-lane base (the swizzles only touch the slot bits below the row
// pitch), so a loop keeps one base per operand instead of one address per fragment.
// ------------------------------------------------------------------------------------------
// byte offset of a lane's 16-byte row read (row, column 8 lh) of a slot-swizzled [rows][S*8] tile;
// column ks*16 + 8 lh is then at (this ^ 32 ks) (ks < S / 2: the XOR stays inside the row)
template <int S>
__device__ __forceinline__ unsigned swz_row_b(int row, int lh) {
  return (unsigned)(row * S * 16 + ((lh ^ slot_swz<S>(row)) << 4));
}
// byte offsets of a lane's two ds_read_b64_tr_b16 of mtr_frag_s<S>(T, k0, col0) for k0 = 0; any k0
// with k0 % 16 == 0 adds k0 * S * 16 bytes (slot_swz reads only the row's low 4 bits)
template <int S>
__device__ __forceinline__ uint2 swz_tr_b(int col0, int lane) {
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1, h = lane >> 5;
  const int col = col0 + 16 * tG + 4 * tp;
  const int rlo = 8 * h + tq, rhi = rlo + 4;
  return make_uint2((unsigned)(rlo * S * 8 + (((col >> 3) ^ slot_swz<S>(rlo)) << 3) + (col & 7)) * 2u,
                    (unsigned)(rhi * S * 8 + (((col >> 3) ^ slot_swz<S>(rhi)) << 3) + (col & 7)) * 2u);
}
template <typename T16>
__device__ __forceinline__ hx8<T16> tr_at(const T16* T, uint2 a, unsigned k_bytes) {
#if defined(__HIP_DEVICE_COMPILE__)
  const char* b = (const char*)T + k_bytes;
  ms16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(b + a.x));
  ms16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ms16x4*)(b + a.y));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(hx8<T16>, v);
#else
  return hx8<T16>{};
#endif
}

// ------------------------------------------------------------------------------------------
// backward with g / dz out at C = 256 (P = 128): the DMA form of mlp_bwd_kernel<.., GD, .., DMA>
// with the addressing made cheap.  The chunk loop runs two chunks per iteration, one per weight
// ring slot, so every LDS address is a per-lane base plus an XOR or immediate (swz_row_b,
// swz_tr_b); the LDS-DMA sources of a chunk are per-lane offsets computed once plus the chunk's
// uniform offset.  Same operands and sums in the same order: the same bits as mlp_bwd_kernel.
// ------------------------------------------------------------------------------------------
template <typename T16, int C, int P>
__global__ __launch_bounds__(256, 1) void mlp_bwd_dma_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int NW = 4, NT = 256, BN = 64, HC = 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC;
  constexpr int HSTR = BN + 32;
  constexpr int H_SZ = C * HSTR, D_SZ = P * HSTR, N_SZ = BN * HC, W1_SZ = HC * C, W2_SZ = P * HC;
  constexpr int W_SZ = W1_SZ + W2_SZ;
  static_assert(H_SZ + D_SZ >= W_SZ && NCH % 2 == 0 && (C / 8) % NW == 0 && (P / 8) % NW == 0, "shape");
  __shared__ __attribute__((aligned(1024))) T16 smem[H_SZ + D_SZ + W_SZ + 2 * N_SZ + 2 * C4];
  T16* const Hs = smem;
  T16* const Ds = Hs + H_SZ;
  T16* const Wslot0 = Ds + D_SZ;   // chunks 0, 2, 4, ...
  T16* const Wslot1 = Hs;          // chunks 1, 3, ... (the h / dy staging area, once read)
  T16* const Zn = Wslot0 + W_SZ;   // dz chunk, pixel-major [BN][HC]
  T16* const Gn = Zn + N_SZ;       // g chunk
  float* const b1s = reinterpret_cast<float*>(Gn + N_SZ);

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave >> 1, wn = wave & 1;   // z / t: hidden half x pixel half; dh: channel half x pixel half

  const int tpi = g.HW / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int img = tile / tpi, p0 = (tile - img * tpi) * BN;

  // LDS-DMA sources of a weight chunk (glds_chunk<C, P, NW, false>'s pieces), chunk-invariant parts
  constexpr int S1 = C / 8, R1 = 64 / S1, N1 = C / 8 / NW, N2 = P / 8 / NW;
  const unsigned short* const w1 = (const unsigned short*)g.w1;
  const unsigned short* const w2 = (const unsigned short*)g.w2;
  unsigned o1[N1], o2[N2];
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    const int inst = wave * N1 + i, r = inst * R1 + lane / S1, ps = lane % S1;
    o1[i] = (unsigned)(r * C + (ps ^ slot_swz<S1>(r)) * 8);
  }
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    const int inst = wave * N2 + i, r = inst * 8 + lane / 8, ps = lane % 8;
    o2[i] = (unsigned)(r * (4 * C) + (ps ^ slot_swz<8>(r)) * 8);
  }
  auto chunk_dma = [&](int j, T16* W1d) __attribute__((always_inline)) {
    unsigned short* const W1h = (unsigned short*)W1d;
    unsigned short* const W2h = W1h + W1_SZ;
#pragma unroll
    for (int i = 0; i < N1; ++i) glds16(w1 + ((unsigned)(j * 64 * C) + o1[i]), lds_addr(W1h + (wave * N1 + i) * 512));
#pragma unroll
    for (int i = 0; i < N2; ++i) glds16(w2 + ((unsigned)(j * 64) + o2[i]), lds_addr(W2h + (wave * N2 + i) * 512));
  };

  chunk_dma(0, Wslot0);
  for (int i = tid; i < C4; i += NT) b1s[i] = g.b1[i];
  stage_h<C, BN, HSTR, NT>(Hs, g, img, p0, tid);
  stage_rows<P, BN, HSTR, NT>(Ds, g.dy + (long)img * g.dy_bs + p0, g.HW, tid);

  mf32x16 hacc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[i][r] = 0.f;
  __syncthreads();
  mbf16x8 hbr[C / 16], dbr[P / 16];
#pragma unroll
  for (int ks = 0; ks < C / 16; ++ks)
    hbr[ks] = mtr_frag(Hs + (ks * 16 + 8 * lh + tq) * HSTR + wn * 32 + 16 * tG + 4 * tp, HSTR);
#pragma unroll
  for (int ks = 0; ks < P / 16; ++ks)
    dbr[ks] = mtr_frag(Ds + (ks * 16 + 8 * lh + tq) * HSTR + wn * 32 + 16 * tG + 4 * tp, HSTR);

  // per-lane LDS byte offsets (chunk-invariant)
  const unsigned a_z = swz_row_b<C / 8>(wm * 32 + lr, lh);          // W1 rows (z)
  const uint2 a_t = swz_tr_b<HC / 8>(wm * 32, lane);                 // W2 transposed (t)
  uint2 a_d[4];                                                      // W1 transposed (dh)
#pragma unroll
  for (int i = 0; i < 4; ++i) a_d[i] = swz_tr_b<C / 8>(wm * (C / 2) + i * 32, lane);
  const unsigned a_n = swz_row_b<HC / 8>(wn * 32 + lr, lh);         // Zn rows (dh B operand)
  const int chh = (wave & 1) * 32;                                   // copy-out hidden half
  const uint2 a_c = swz_tr_b<HC / 8>(chh, lane);                     // Gn / Zn transposed (copy-out)
  const unsigned a_e = (unsigned)((wn * 32 + lr) * HC * 2 + (((wm * 4) ^ slot_swz<HC / 8>(wn * 32 + lr)) << 4) + 8 * lh);
  const long gbase = (long)img * C4 * g.HW + p0;

  auto chunk = [&](int j, const T16* W1s, T16* Wnext) __attribute__((always_inline)) {
    // chunk j landed (this wave's pieces: the only LDS-DMA in flight) and every wave is done with
    // chunk j-1 (its ring slot, Zn / Gn; at j = 0 the h / dy staging area = slot 1)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (j + 1 < NCH) chunk_dma(j + 1, Wnext);
    const T16* W2s = W1s + W1_SZ;
    mf32x16 zacc, tacc;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b4 = *reinterpret_cast<const float4*>(b1s + j * HC + wm * 32 + 8 * q + 4 * lh);
      zacc[4 * q] = b4.x; zacc[4 * q + 1] = b4.y; zacc[4 * q + 2] = b4.z; zacc[4 * q + 3] = b4.w;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) tacc[r] = 0.f;
    // every A fragment of the two products read before the first MFMA: one LDS latency per chunk
    // instead of one per MFMA (the compiler otherwise waits on each fragment right before its use)
    mbf16x8 za[C / 16], ta[P / 16];
#pragma unroll
    for (int ks = 0; ks < C / 16; ++ks) za[ks] = *reinterpret_cast<const mbf16x8*>((const char*)W1s + (a_z ^ (unsigned)(32 * ks)));
#pragma unroll
    for (int ks = 0; ks < P / 16; ++ks) ta[ks] = tr_at(W2s, a_t, ks * 16 * HC * 2);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < C / 16; ++ks) zacc = mfma16(za[ks], hbr[ks], zacc);
    // gelu(z) / gelu'(z) need only z: their VALU can issue beside the t MFMAs
    f32x2 gvv[8], gpv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) mlp_gelu_pair2<true>(f32x2{zacc[2 * i], zacc[2 * i + 1]}, gvv[i], gpv[i]);
#pragma unroll
    for (int ks = 0; ks < P / 16; ++ks) tacc = mfma16(ta[ks], dbr[ks], tacc);
    // g = gelu(z), dz = t gelu'(z) -> LDS, pixel-major, 4 hidden per write
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      mbf16x4 gv4, dv4;
#pragma unroll
      for (int e = 0; e < 4; e += 2) {
        const f32x2 gv = gvv[(4 * q + e) / 2], gp = gpv[(4 * q + e) / 2];
        const f32x2 dz = mlp_mul2<true>(f32x2{tacc[4 * q + e], tacc[4 * q + e + 1]}, gp);
        gv4[e] = (T16)gv.x; gv4[e + 1] = (T16)gv.y;
        dv4[e] = (T16)dz.x; dv4[e + 1] = (T16)dz.y;
      }
      const unsigned o = a_e ^ (unsigned)(16 * q);
      *reinterpret_cast<mbf16x4*>((char*)Gn + o) = gv4;
      *reinterpret_cast<mbf16x4*>((char*)Zn + o) = dv4;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // raw barrier: chunk j+1's DMA stays in flight
    raw_barrier();
    // copy-out: 8 pixels of one hidden row per lane -> 16-byte stores; dz sums per 32 pixels
    {
      float bacc = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int pb = ((wave >> 1) * 2 + c) * 16;
        const mbf16x8 gv = tr_at(Gn, a_c, pb * HC * 2);
        const mbf16x8 dv = tr_at(Zn, a_c, pb * HC * 2);
        const long o = gbase + (long)(j * HC + chh + lr) * g.HW + pb + 8 * lh;
        *reinterpret_cast<mbf16x8*>((T16*)g.g_out + o) = gv;
        *reinterpret_cast<mbf16x8*>((T16*)g.dz_out + o) = dv;
#pragma unroll
        for (int e = 0; e < 8; ++e) bacc += (float)dv[e];
      }
      bacc += __shfl_xor(bacc, 32, 64);
      if (lh == 0 && g.bsum) g.bsum[((long)tile * (NW / 2) + (wave >> 1)) * C4 + j * HC + chh + lr] = bacc;
    }
    // dh += W1[chunk]^T dz (fragments read ahead as above)
    mbf16x8 dzb[HC / 16], w1t[HC / 16][4];
#pragma unroll
    for (int ks = 0; ks < HC / 16; ++ks) {
      dzb[ks] = *reinterpret_cast<const mbf16x8*>((const char*)Zn + (a_n ^ (unsigned)(32 * ks)));
#pragma unroll
      for (int i = 0; i < 4; ++i) w1t[ks][i] = tr_at(W1s, a_d[i], ks * 16 * C * 2);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < HC / 16; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) hacc[i] = mfma16(w1t[ks][i], dzb[ks], hacc[i]);
  };
  for (int j = 0; j < NCH; j += 2) {
    chunk(j, Wslot0, Wslot1);
    chunk(j + 1, Wslot1, Wslot0);
  }

  float* ob = g.out + (long)img * g.out_bs + p0 + wn * 32 + lr;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = wm * (C / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      ob[(long)c * g.HW] = hacc[i][r];
    }
}

// ------------------------------------------------------------------------------------------
// backward (weight path): dW1 = dz h^T, dW2 = dy g^T, db1 = sum dz -- without g / dz in HBM.
// Workgroup (hidden chunk j, pixel split s) holds chunk j's W1 rows / W2 columns in LDS for its
// whole life and walks pixel tiles s, s+S, ...: per tile it recomputes z = W1[j] h + b1 and
// t = W2[:, j]^T dy, forms g = gelu(z), dz = t gelu'(z) (bf16, LDS only) and accumulates
// dW1[j] (HC x C) and dW2[:, j] (P x HC) in registers, K = the tile's pixels.  The NCH chunk
// workgroups of one split run on the same XCD (xcd_tile, chunk index fastest) and read the same
// h / dy tiles, so HBM sees them about once.  The next tile is prefetched into registers while
// the current one computes.  Each split writes its partial dW1 / dW2 / db1 to ws (plain stores);
// a fixed-order split reduction adds them (deterministic).
// ------------------------------------------------------------------------------------------
template <int K, int BN, int NT, bool BF>
struct TileLd {   // a [K][BN] activation tile (rows strided by HW), fp32 or bf16 in HBM, via registers
  static constexpr int E = BF ? 8 : 4;                 // elements per 16-byte item
  static constexpr int N = K * BN / E / NT;
  static_assert((K * BN / E) % NT == 0, "tile split");
  mu32x4 v[N];
  __device__ __forceinline__ void load(const void* src, int HW, int tid) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int it = tid + i * NT, k = it / (BN / E), c = it % (BN / E);
      const char* p = (const char*)src + ((long)k * HW + c * E) * (BF ? 2 : 4);
      v[i] = *reinterpret_cast<const mu32x4*>(p);
    }
  }
  template <int STR, typename T16>
  __device__ __forceinline__ void store(T16* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int it = tid + i * NT, k = it / (BN / E), c = it % (BN / E);
      if constexpr (BF) *reinterpret_cast<mu32x4*>(dst + k * STR + c * E) = v[i];
      else *reinterpret_cast<hx4<T16>*>(dst + k * STR + c * E) = mcvt4<T16>(__builtin_bit_cast(float4, v[i]));
    }
  }
  // into an unpadded [K][BN] image with slot_swz<BN/8>'d 16-byte slots (a 4-element fp32 item
  // stays inside its slot)
  template <typename T16>
  __device__ __forceinline__ void store_swz(T16* dst, int tid) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int it = tid + i * NT, k = it / (BN / E), c = it % (BN / E);
      if constexpr (BF) *reinterpret_cast<mu32x4*>(dst + swz_off<BN / 8>(k, c * E)) = v[i];
      else *reinterpret_cast<hx4<T16>*>(dst + swz_off<BN / 8>(k, c * E)) = mcvt4<T16>(__builtin_bit_cast(float4, v[i]));
    }
  }
};

// wave -> (tile, k-part) split of an [M x N] weight-grad product over NW waves: TPW tiles per wave,
// or KS waves per tile each taking 1/KS of the K (pixel) range when there are fewer tiles than waves
template <int M, int N, int NW>
struct WTiles {
  static constexpr int MT = M / 32, T = MT * (N / 32);
  static constexpr int TPW = T >= NW ? T / NW : 1, KS = T >= NW ? 1 : NW / T;
  static_assert(T % NW == 0 || NW % T == 0, "weight-grad tile split");
};

template <typename T16, int C, int P, int BN, int NW, bool HBF, int MINB>
__global__ __launch_bounds__(NW * 64, MINB) void mlp_wgrad_kernel(MlpArgs g) {
  typedef hx8<T16> mbf16x8;
  typedef hx4<T16> mbf16x4;
  constexpr int HC = 64;
  constexpr int NT = NW * 64;
  constexpr int C4 = 4 * C, NCH = C4 / HC;
  // Hs / Ds are read transposed (z, t: k = channel) and row-wise (dW: k = pixel); every LDS image
  // here is unpadded with slot_swz'd 16-byte slots, conflict-free for both kinds of read and for
  // the staging / epilogue writes except the 8-byte dz / g writes (2-way; tools/lds_banks.py)
  constexpr int HSTR = BN, NSTR = HC, W1STR = C, W2STR = HC;
  constexpr int H_SZ = C * HSTR, D_SZ = P * HSTR, N_SZ = BN * NSTR, W1_SZ = HC * W1STR, W2_SZ = P * W2STR;
  __shared__ __attribute__((aligned(16))) T16 smem[H_SZ + D_SZ + 2 * N_SZ + W1_SZ + W2_SZ];
  T16* Hs = smem;
  T16* Ds = Hs + H_SZ;
  T16* Zn = Ds + D_SZ;     // dz, pixel-major [BN][NSTR]
  T16* Gn = Zn + N_SZ;     // g,  pixel-major [BN][NSTR]
  T16* W1s = Gn + N_SZ;
  T16* W2s = W1s + W1_SZ;

  using ZG = WGrid<HC, BN, NW>;    // z / t tile [HC x BN]
  using T1 = WTiles<HC, C, NW>;    // dW1[j]    [HC x C]
  using T2 = WTiles<P, HC, NW>;    // dW2[:, j] [P x HC]
  static_assert(BN % (16 * T1::KS) == 0 && BN % (16 * T2::KS) == 0, "k split");

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int tq = (lane >> 2) & 3, tp = lane & 3, tG = (lane >> 4) & 1;
  const int wm = wave / ZG::WN, wn = wave % ZG::WN;

  const int id = xcd_tile(blockIdx.x, gridDim.x);
  const int j = id % NCH, s = id / NCH;
  const int S = g.splits, tpi = g.HW / BN, ntiles = g.nb * tpi;

  {   // chunk j of the weights, once
    using WC = WCh<C, P, HC, NT>;
    mu32x4 wr1[WC::N1], wr2[WC::N2];
    wch_load<C, P, HC, NT>(wr1, wr2, g.w1, g.w2, j, tid);
    wch_store_swz<C, P, HC, NT>(wr1, wr2, W1s, W2s, tid);
  }
  float bias[ZG::TM][16];
#pragma unroll
  for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) bias[i][r] = g.b1[j * HC + wm * (HC / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh];

  mf32x16 a1[T1::TPW], a2[T2::TPW];
  float bacc[ZG::TM][16];
#pragma unroll
  for (int q = 0; q < T1::TPW; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) a1[q][r] = 0.f;
#pragma unroll
  for (int q = 0; q < T2::TPW; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) a2[q][r] = 0.f;
#pragma unroll
  for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) bacc[i][r] = 0.f;

  TileLd<C, BN, NT, HBF> hreg;
  TileLd<P, BN, NT, false> dreg;
  auto tile_src = [&](int tt, const void*& hp, const float*& dp) {
    const int img = tt / tpi, p0 = (tt - img * tpi) * BN;
    hp = HBF ? (const void*)((const T16*)g.h + (long)img * g.h_bs + p0)
             : (const void*)((const float*)g.h + (long)img * g.h_bs + p0);
    dp = g.dy + (long)img * g.dy_bs + p0;
  };
  if (s < ntiles) {
    const void* hp; const float* dp;
    tile_src(s, hp, dp);
    hreg.load(hp, g.HW, tid);
    dreg.load(dp, g.HW, tid);
  }

  for (int tt = s; tt < ntiles; tt += S) {
    __syncthreads();   // every wave is done with the previous tile's Hs / Ds / Zn / Gn
    hreg.store_swz(Hs, tid);
    dreg.store_swz(Ds, tid);
    __syncthreads();
    if (tt + S < ntiles) {   // prefetch the next tile while this one computes
      const void* hp; const float* dp;
      tile_src(tt + S, hp, dp);
      hreg.load(hp, g.HW, tid);
      dreg.load(dp, g.HW, tid);
    }
    // ---- z = W1[j] h + b1 ;  t = W2[:, j]^T dy ----
    mf32x16 zacc[ZG::TM][ZG::TN], tacc[ZG::TM][ZG::TN];
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) { zacc[i][t][r] = bias[i][r]; tacc[i][t][r] = 0.f; }
#pragma unroll 4
    for (int ks = 0; ks < C / 16; ++ks) {
      mbf16x8 af[ZG::TM], bf[ZG::TN];
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
        af[i] = *reinterpret_cast<const mbf16x8*>(W1s + swz_off<C / 8>(wm * (HC / 2) + i * 32 + lr, ks * 16 + lh * 8));
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
        bf[t] = mtr_frag_s<BN / 8>(Hs, ks * 16, wn * (BN / ZG::WN) + t * 32, lane);
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
        for (int t = 0; t < ZG::TN; ++t)
          zacc[i][t] = mfma16(af[i], bf[t], zacc[i][t]);
    }
#pragma unroll 4
    for (int ks = 0; ks < P / 16; ++ks) {
      mbf16x8 af[ZG::TM], bf[ZG::TN];
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
        af[i] = mtr_frag_s<HC / 8>(W2s, ks * 16, wm * (HC / 2) + i * 32, lane);
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t)
        bf[t] = mtr_frag_s<BN / 8>(Ds, ks * 16, wn * (BN / ZG::WN) + t * 32, lane);
#pragma unroll
      for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
        for (int t = 0; t < ZG::TN; ++t)
          tacc[i][t] = mfma16(af[i], bf[t], tacc[i][t]);
    }
    // ---- g = gelu(z), dz = t gelu'(z) -> LDS (bf16, pixel-major); b1 sums of the rounded dz ----
#pragma unroll
    for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
      for (int t = 0; t < ZG::TN; ++t) {
        const int n = wn * (BN / ZG::WN) + t * 32 + lr;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          mbf16x4 gv4, dv4;
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            f32x2 gv, gp;
            mlp_gelu_pair2<(C + P < 384)>(f32x2{zacc[i][t][4 * q + e], zacc[i][t][4 * q + e + 1]}, gv, gp);
            const f32x2 dz = mlp_mul2<(C + P < 384)>(f32x2{tacc[i][t][4 * q + e], tacc[i][t][4 * q + e + 1]}, gp);
            gv4[e] = (T16)gv.x; gv4[e + 1] = (T16)gv.y;
            dv4[e] = (T16)dz.x; dv4[e + 1] = (T16)dz.y;
            bacc[i][4 * q + e] += (float)dv4[e];
            bacc[i][4 * q + e + 1] += (float)dv4[e + 1];
          }
          const int m = wm * (HC / 2) + i * 32 + 8 * q + 4 * lh;
          *reinterpret_cast<mbf16x4*>(Gn + swz_off<HC / 8>(n, m)) = gv4;
          *reinterpret_cast<mbf16x4*>(Zn + swz_off<HC / 8>(n, m)) = dv4;
        }
      }
    __syncthreads();
    // ---- dW1[j] += dz h^T  (A = dz [hidden][px] transposed from Zn, B = h^T row-wise from Hs) ----
    if constexpr (T1::KS == 1 && NW % T1::MT == 0) {
      // the wave's TPW tiles (wave + NW q) share one row tile mt: one A fragment per k step for all of them
      const int mt = wave % T1::MT;
#pragma unroll
      for (int ks = 0; ks < BN / 16; ++ks) {
        const mbf16x8 af = mtr_frag_s<HC / 8>(Zn, ks * 16, mt * 32, lane);
#pragma unroll
        for (int q = 0; q < T1::TPW; ++q) {
          const int nt = (wave + NW * q) / T1::MT;
          const mbf16x8 bf = *reinterpret_cast<const mbf16x8*>(Hs + swz_off<BN / 8>(nt * 32 + lr, ks * 16 + lh * 8));
          a1[q] = mfma16(af, bf, a1[q]);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < T1::TPW; ++q) {
        const int ti = T1::KS == 1 ? wave + NW * q : wave % T1::T;
        const int kp = T1::KS == 1 ? 0 : wave / T1::T;
        const int mt = ti % T1::MT, nt = ti / T1::MT;
#pragma unroll
        for (int ks = kp * (BN / 16 / T1::KS); ks < (kp + 1) * (BN / 16 / T1::KS); ++ks) {
          const mbf16x8 af = mtr_frag_s<HC / 8>(Zn, ks * 16, mt * 32, lane);
          const mbf16x8 bf = *reinterpret_cast<const mbf16x8*>(Hs + swz_off<BN / 8>(nt * 32 + lr, ks * 16 + lh * 8));
          a1[q] = mfma16(af, bf, a1[q]);
        }
      }
    }
    // ---- dW2[:, j] += dy g^T  (A = dy row-wise from Ds, B = g^T transposed from Gn) ----
#pragma unroll
    for (int q = 0; q < T2::TPW; ++q) {
      const int ti = T2::KS == 1 ? wave + NW * q : wave % T2::T;
      const int kp = T2::KS == 1 ? 0 : wave / T2::T;
      const int mt = ti % T2::MT, nt = ti / T2::MT;
#pragma unroll
      for (int ks = kp * (BN / 16 / T2::KS); ks < (kp + 1) * (BN / 16 / T2::KS); ++ks) {
        const mbf16x8 af = *reinterpret_cast<const mbf16x8*>(Ds + swz_off<BN / 8>(mt * 32 + lr, ks * 16 + lh * 8));
        const mbf16x8 bf = mtr_frag_s<HC / 8>(Gn, ks * 16, nt * 32, lane);
        a2[q] = mfma16(af, bf, a2[q]);
      }
    }
  }

  // ---- partials: k-part sums through LDS (fixed order), then plain stores to this split's rows ----
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);   // [NW][64 lanes][16]
  auto kreduce = [&](mf32x16& acc, int kp, int ks_n) {
    // waves kp > 0 park their partial, wave kp == 0 of the same tile adds them in kp order
    if (kp > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(wave * 64 + lane) * 16 + r] = acc[r];
    }
    __syncthreads();
    if (kp == 0)
      for (int k = 1; k < ks_n; ++k)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += red[((wave + k * (NW / ks_n)) * 64 + lane) * 16 + r];
    __syncthreads();
  };
  float* ws1 = g.ws + (long)s * C4 * C;                                   // [S][4C][C]
  float* ws2 = g.ws + (long)S * C4 * C + (long)s * P * C4;                // [S][P][4C]
  float* ws3 = g.ws + (long)S * (C4 * C + P * C4) + (long)s * C4;         // [S][4C]
  if constexpr (T1::KS > 1) kreduce(a1[0], wave / T1::T, T1::KS);
#pragma unroll
  for (int q = 0; q < T1::TPW; ++q) {
    const int ti = T1::KS == 1 ? wave + NW * q : wave % T1::T;
    const int kp = T1::KS == 1 ? 0 : wave / T1::T;
    const int mt = ti % T1::MT, nt = ti / T1::MT;
    if (kp == 0)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ws1[(long)(j * HC + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * C + nt * 32 + lr] = a1[q][r];
  }
  if constexpr (T2::KS > 1) kreduce(a2[0], wave / T2::T, T2::KS);
#pragma unroll
  for (int q = 0; q < T2::TPW; ++q) {
    const int ti = T2::KS == 1 ? wave + NW * q : wave % T2::T;
    const int kp = T2::KS == 1 ? 0 : wave / T2::T;
    const int mt = ti % T2::MT, nt = ti / T2::MT;
    if (kp == 0)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ws2[(long)(mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * C4 + j * HC + nt * 32 + lr] = a2[q][r];
  }
  // b1: lanes lr of a half hold the same hidden rows -> butterfly, then the WN waves of a row
  // group in wn order
  float* bred = red;   // [NW][HC]
#pragma unroll
  for (int i = 0; i < ZG::TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float t = bacc[i][r];
      t += __shfl_xor(t, 1, 64); t += __shfl_xor(t, 2, 64); t += __shfl_xor(t, 4, 64);
      t += __shfl_xor(t, 8, 64); t += __shfl_xor(t, 16, 64);
      if (lr == 0) bred[wave * HC + wm * (HC / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh] = t;
    }
  __syncthreads();
  if (tid < HC) {
    const int wmr = tid / (HC / 2);
    float t = 0.f;
    for (int w = 0; w < ZG::WN; ++w) t += bred[(wmr * ZG::WN + w) * HC + tid];
    ws3[j * HC + tid] = t;
  }
}

template <typename T16>
__global__ __launch_bounds__(256) void f32_to_half_kernel(const float* __restrict__ s, T16* __restrict__ d, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) d[i] = (T16)s[i];
}

// Supported (C, P) -> pixel tile (forward and backward use the same BN); HC = 64, 8 waves.
static int mlp_bn(int C, int P) {
  if ((C == 64 && P == 128) || (C == 128 && P == 64) || (C == 128 && P == 256) || (C == 256 && P == 128)) return 128;
  return 0;
}
constexpr int MLP_NW = 8;

template <typename T16, int C, int P, int BN, int MINB>
static void fwd_lds_launch(const MlpArgs& g, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)g.nb * (g.HW / BN));
  hipLaunchKernelGGL((mlp_fwd_lds_kernel<T16, C, P, BN, 64, MLP_NW, MINB>), dim3(tiles), dim3(MLP_NW * 64), 0, st, g);
}
template <typename T16, int C, int P, int MINB>
static void fwd_launch(const MlpArgs& g, hipStream_t st) {
  const unsigned tiles = (unsigned)((long)g.nb * (g.HW / 128));
  hipLaunchKernelGGL((mlp_fwd_kernel<T16, C, P, MINB>), dim3(tiles), dim3(512), 0, st, g);
}
// backward: 8 waves x 128 pixels where the LDS tiles fit, else 4 waves x 64 pixels (same bsum
// granularity: one partial row per 32 pixels)
// Planner knob (measurement tools): key 0 = the C = 256 backward with g / dz out, 0 the LDS-DMA
// weight ring (0.831 -> 0.717 ms at uc3, B = 16, same bits; profiles/r04/mlp_micro.txt), 1 the
// register-staged weights, 2 the DMA ring with precomputed LDS / DMA addresses (mlp_bwd_dma_kernel,
// default: 0.733 -> 0.704 ms, same bits; profiles/r04/mlp_micro_b.txt).  (An 8-wave form -- two waves per SIMD, 128-row hidden chunks -- measured
// 0.977 ms: at 256 registers it spills, and it issues more VALU per MFMA.)
static int g_mlp_tune[4] = {2, 0, 0, 0};

template <typename T16, int C, int P, int BN, int NW, bool GD = true, int MINB = 1, bool DMA = false>
static void bwd_launch(const MlpArgs& g, hipStream_t st) {
  static_assert(BN / (NW / 2) == 32, "bsum granularity");
  const unsigned tiles = (unsigned)((long)g.nb * (g.HW / BN));
  hipLaunchKernelGGL((mlp_bwd_kernel<T16, C, P, BN, 64, NW, GD, MINB, DMA>), dim3(tiles), dim3(NW * 64), 0, st, g);
}

// weight-grad kernel: same pixel tile as the backward; splits so that NCH * S ~ 512 workgroups
// (2 per CU), a multiple of 8 (whole split groups per XCD), at most one tile per split
static int mlp_wgrad_splits(int C, int P, int HW, int nb) {
  const int bn = 64;
  const int nch = 4 * C / 64;
  const long ntiles = (long)nb * (HW / bn);
  long S = 512 / nch;
  S = S / 8 * 8;
  if (S < 8) S = 8;
  if (S > ntiles) S = ntiles;
  return (int)S;
}

template <typename T16, int C, int P, int BN, int NW, int MINB>
static void wgrad_launch(const MlpArgs& g, hipStream_t st) {
  const unsigned wgs = (unsigned)((4 * C / 64) * g.splits);
  if (g.h_bf16) hipLaunchKernelGGL((mlp_wgrad_kernel<T16, C, P, BN, NW, true, MINB>), dim3(wgs), dim3(NW * 64), 0, st, g);
  else hipLaunchKernelGGL((mlp_wgrad_kernel<T16, C, P, BN, NW, false, MINB>), dim3(wgs), dim3(NW * 64), 0, st, g);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// 0 if the fused kernels do not take (C, P, HW), else the number of bsum partial rows per
// image pixel: bsum has nb * HW / return rows (one per 32-pixel group of a tile x wave pair).
int dsgan_mlp_supported(int C, int P, int HW) {
  const int bn = mlp_bn(C, P);
  if (bn == 0 || HW % bn != 0) return 0;
  return 32;
}

int dsgan_mlp_fwd(const void* h, long h_bs, int h_bf16, const void* w1, const float* b1, const void* w2,
                  const float* b2, float* out, long out_bs, int nb, int C, int P, int HW,
                  int accumulate, hipStream_t st) {
  DSG_REQUIRE(h && w1 && b1 && w2 && out && nb > 0, "dsgan_mlp_fwd: bad args");
  DSG_REQUIRE(dsgan_mlp_supported(C, P, HW), "dsgan_mlp_fwd: unsupported shape C=%d P=%d HW=%d", C, P, HW);
  DSG_REQUIRE(((uintptr_t)h & 15) == 0 && (h_bs & 7) == 0 && ((uintptr_t)w1 & 15) == 0 && ((uintptr_t)w2 & 15) == 0,
              "dsgan_mlp_fwd: operands must be 16-byte aligned");
  MlpArgs g{};
  g.h = h; g.h_bs = h_bs; g.w1 = w1; g.b1 = b1; g.w2 = w2; g.b2 = b2;
  g.out = out; g.out_bs = out_bs; g.HW = HW; g.nb = nb; g.accumulate = accumulate; g.h_bf16 = h_bf16;
  // MINB = waves per SIMD: 4 (two workgroups per CU) where 128 registers hold
  with_half([&](auto* t) {
    using T16 = std::remove_pointer_t<decltype(t)>;
    if (C == 64) fwd_lds_launch<T16, 64, 128, 128, 2>(g, st);
    else if (C == 128 && P == 64) fwd_launch<T16, 128, 64, 4>(g, st);
    else if (C == 128) fwd_launch<T16, 128, 256, 2>(g, st);
    else fwd_launch<T16, 256, 128, 2>(g, st);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_mlp_bwd(const void* h, long h_bs, int h_bf16, const float* dy, long dy_bs, const void* w1, const float* b1,
                  const void* w2, float* dh, long dh_bs, void* g_out, void* dz_out, float* bsum, int nb,
                  int C, int P, int HW, hipStream_t st) {
  DSG_REQUIRE(h && dy && w1 && b1 && w2 && dh && nb > 0 && (g_out != nullptr) == (dz_out != nullptr) && (g_out || !bsum),
              "dsgan_mlp_bwd: bad args (g_out and dz_out both or neither; bsum needs them)");
  DSG_REQUIRE(dsgan_mlp_supported(C, P, HW), "dsgan_mlp_bwd: unsupported shape C=%d P=%d HW=%d", C, P, HW);
  DSG_REQUIRE(((uintptr_t)h & 15) == 0 && ((uintptr_t)dy & 15) == 0 && (h_bs & 7) == 0 && (dy_bs & 3) == 0 &&
              ((uintptr_t)g_out & 15) == 0 && ((uintptr_t)dz_out & 15) == 0,
              "dsgan_mlp_bwd: operands must be 16-byte aligned");
  MlpArgs g{};
  g.h = h; g.h_bs = h_bs; g.dy = dy; g.dy_bs = dy_bs; g.w1 = w1; g.b1 = b1;
  g.w2 = w2; g.out = dh; g.out_bs = dh_bs; g.g_out = g_out;
  g.dz_out = dz_out; g.bsum = bsum; g.HW = HW; g.nb = nb; g.h_bf16 = h_bf16;
  with_half([&](auto* t) {
    using T16 = std::remove_pointer_t<decltype(t)>;
    if (!g_out) {   // dh only: the register-chained kernel where h, dy and dh fragments fit in registers
      const unsigned tiles = (unsigned)((long)g.nb * (g.HW / 128));
      if (C == 64) hipLaunchKernelGGL((mlp_dh_kernel<T16, 64, 128, 2>), dim3(tiles), dim3(512), 0, st, g);
      else if (C == 128 && P == 64) hipLaunchKernelGGL((mlp_dh_kernel<T16, 128, 64, 2>), dim3(tiles), dim3(512), 0, st, g);
      else if (C == 128) bwd_launch<T16, 128, 256, 64, 4, false, 1>(g, st);
      else bwd_launch<T16, 256, 128, 64, 4, false, 1>(g, st);
    } else if (C == 64) bwd_launch<T16, 64, 128, 128, 8>(g, st);
    else if (C == 128 && P == 64) bwd_launch<T16, 128, 64, 128, 8>(g, st);
    else if (C == 128) bwd_launch<T16, 128, 256, 64, 4>(g, st);
    else if (g_mlp_tune[0] == 2 && P == 128)
      hipLaunchKernelGGL((mlp_bwd_dma_kernel<T16, 256, 128>), dim3((unsigned)((long)g.nb * (g.HW / 64))), dim3(256), 0,
                         st, g);
    else if (g_mlp_tune[0] == 0) bwd_launch<T16, 256, 128, 64, 4, true, 1, true>(g, st);
    else bwd_launch<T16, 256, 128, 64, 4>(g, st);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

// fp32 scratch (elements) of dsgan_mlp_wgrad
long dsgan_mlp_wgrad_workspace(int C, int P, int HW, int nb) {
  if (!dsgan_mlp_supported(C, P, HW)) return 0;
  const long S = mlp_wgrad_splits(C, P, HW, nb);
  return S * (4L * C * C + (long)P * 4 * C + 4L * C);
}

int dsgan_mlp_wgrad(const void* h, long h_bs, int h_bf16, const float* dy, long dy_bs, const void* w1,
                    const float* b1, const void* w2, float* dw1, float* db1, float* dw2, float* ws, long ws_elems,
                    int nb, int C, int P, int HW, hipStream_t st) {
  DSG_REQUIRE(h && dy && w1 && b1 && w2 && dw1 && db1 && dw2 && nb > 0, "dsgan_mlp_wgrad: bad args");
  DSG_REQUIRE(dsgan_mlp_supported(C, P, HW), "dsgan_mlp_wgrad: unsupported shape C=%d P=%d HW=%d", C, P, HW);
  DSG_REQUIRE(((uintptr_t)h & 15) == 0 && ((uintptr_t)dy & 15) == 0 && (h_bs & 7) == 0 && (dy_bs & 3) == 0,
              "dsgan_mlp_wgrad: operands must be 16-byte aligned");
  MlpArgs g{};
  g.h = h; g.h_bs = h_bs; g.h_bf16 = h_bf16; g.dy = dy; g.dy_bs = dy_bs; g.w1 = w1; g.b1 = b1;
  g.w2 = w2; g.HW = HW; g.nb = nb; g.ws = ws;
  const int S = mlp_wgrad_splits(C, P, HW, nb);
  g.splits = S;
  DSG_WS((long)S * (4L * C * C + (long)P * 4 * C + 4L * C), ws, ws_elems, "dsgan_mlp_wgrad (dsgan_mlp_wgrad_workspace)");
  with_half([&](auto* t) {
    using T16 = std::remove_pointer_t<decltype(t)>;
    if (C == 64) wgrad_launch<T16, 64, 128, 64, 4, 2>(g, st);
    else if (C == 128 && P == 64) wgrad_launch<T16, 128, 64, 64, 4, 2>(g, st);
    else if (C == 128) wgrad_launch<T16, 128, 256, 64, 4, 1>(g, st);
    else wgrad_launch<T16, 256, 128, 64, 4, 1>(g, st);
  });
  DSG_CHECK_LAUNCH();
  const long n1 = 4L * C * C, n2 = (long)P * 4 * C;
  const float* wsv[3] = {ws, ws + S * n1, ws + S * (n1 + n2)};
  const int sv[3] = {S, S, S};
  const long mv[3] = {n1, n2, 4L * C};
  float* dv[3] = {dw1, dw2, db1};
  launch_split_reduce_multi(3, wsv, sv, mv, dv, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// planner knob `key` <- val (val < 0: read only), returns the previous value (measurement tools):
// key 0 = the C = 256 backward with g / dz out: 0 LDS-DMA weight ring, 1 register-staged weights,
// 2 the ring with precomputed addresses
int dsgan_mlp_tune(int key, int val) {
  if (key < 0 || key >= 4) return -1;
  const int old = g_mlp_tune[key];
  if (val >= 0) g_mlp_tune[key] = val;
  return old;
}

int dsgan_colsum(float* part, int rows, int cols, float* out, hipStream_t st) {
  DSG_REQUIRE(part && out && rows > 0 && cols > 0, "dsgan_colsum: bad args");
  launch_split_reduce(part, rows, cols, out, st);   // rows summed in a fixed order (deterministic)
  DSG_CHECK_LAUNCH();
  return 0;
}

// (dst has the library's half type: bf16, or fp16 in --precision fp16)
int dsgan_f32_to_bf16(const float* src, void* dst, long n, hipStream_t st) {
  DSG_REQUIRE(src && dst && n > 0, "dsgan_f32_to_bf16: bad args");
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  with_half([&](auto* t) {
    using T16 = std::remove_pointer_t<decltype(t)>;
    hipLaunchKernelGGL((f32_to_half_kernel<T16>), dim3((unsigned)blocks), dim3(256), 0, st, src, (T16*)dst, n);
  });
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
