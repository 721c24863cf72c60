// Shared device helpers for libdsgan_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsg {

// dw[e] += sum_s ws[s * MN + e] for s = 0..splits-1 in a fixed order (split_reduce.hip): the
// deterministic reduction every split weight-grad (pwgemm, igemm, skinny) finishes with.
void launch_split_reduce(const float* ws, int splits, long MN, float* dw, hipStream_t st);
// ... with elements e = (c, i), i < KK1: i < KK1-1 -> dw[c*(KK1-1)+i], i == KK1-1 -> db[c]
void launch_split_reduce_kk(const float* ws, int splits, long MN, float* dw, float* db, int KK1, hipStream_t st);
// n independent reductions with disjoint outputs in one launch (split_reduce.hip: the fixed order,
// and the deferred mode that queues them for one batched flush)
void launch_split_reduce_multi(int n, const float* const* ws, const int* splits, const long* MN, float* const* dw,
                               hipStream_t st);
// out[0] = coef * sum_i part[i], i = 0..n-1 in a fixed order (losses.hip: the loss reductions' last pass)
void launch_final_sum(const float* part, int n, float coef, float* out, hipStream_t st);
// wconv.hip's weight-grad partials [splits][T][M][C] -> dw[M][C][T] (+=), C % 32 == 0, T <= 16
void launch_split_reduce_wconv(const float* ws, int splits, int T, int M, int C, float* dw, hipStream_t st);


// ---- 16-bit MFMA operand type ------------------------------------------------------------
// Every "bf16" operand / storage flag and every 16-bit MFMA of the library uses ONE 16-bit type
// per process, the library's half type (dsgan_set_half_type): bf16 (default; --precision bf16) or
// IEEE fp16 (--precision fp16, BASELINE configs[4]).  Kernels are templated on it (T16) and the
// host launchers pick the instantiation from half_type(); both MFMA forms are the gfx950
// v_mfma_f32_32x32x16_{bf16,f16} (8 operands per lane, fp32 accumulation), so tiles, LDS layouts
// and the ds_read_b64_tr_b16 transposes are identical.  Conversions from fp32 are
// round-to-nearest-even in both.
enum HalfType : int { HALF_BF16 = 0, HALF_F16 = 1 };
int half_type();   // capi.cpp

template <typename T> using hx8 = T __attribute__((ext_vector_type(8)));
template <typename T> using hx4 = T __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
// A raw workgroup barrier (no implicit s_waitcnt: the caller has issued the waits it needs, so
// LDS-DMA of later stages stays in flight across it) followed by a compiler memory fence.  LLVM
// models s_barrier as touching no memory, so without the fence the compiler could hoist the next
// stage's ds_reads above the barrier, before the other waves' DMA into that stage is ordered.
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16_t mfma16(hx8<__bf16> a, hx8<__bf16> b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t mfma16(hx8<_Float16> a, hx8<_Float16> b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// a 16-bit value from its raw bits (2-byte buffer loads)
template <typename T> __device__ __forceinline__ float h2f(unsigned short b) { return (float)__builtin_bit_cast(T, b); }
template <typename T> __device__ __forceinline__ unsigned short f2h(float v) { return __builtin_bit_cast(unsigned short, (T)v); }

// host dispatch: F(tag) with tag = (__bf16*)0 or (_Float16*)0, e.g.
//   return with_half([&](auto* t) { using T16 = std::remove_pointer_t<decltype(t)>; ... });
template <typename F> __host__ inline auto with_half(F&& f) {
  if (half_type() == HALF_F16) return f((_Float16*)nullptr);
  return f((__bf16*)nullptr);
}

// ACT_GELU_FAST: nn.GELU by the A&S 7.1.26 erfc below (|err| <= 1.5e-7), for the 16-bit modes'
// InstanceNorm epilogues (functional._in_act): the exact erf form is ~40 VALU per element and bounds
// those streaming kernels; fp32 mode keeps ACT_GELU.
enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_LRELU = 3, ACT_SIGMOID = 4, ACT_GELU_FAST = 5 };

constexpr float kInvSqrt2 = 0.70710678118654752440f;
constexpr float kInvSqrt2Pi = 0.39894228040143267794f;

// nn.GELU() (exact erf form) -- the activation of MixConvNeXtML (DSGAN/models/model/MixConvNeXtML.py:51,82,223)
// Branch-free erf: the two polynomial pieces of the device library's erff (|x| < 1 and
// |x| >= 1), both evaluated and selected.  erff itself branches on |x| < 1, which diverges
// inside a wavefront on real activations and costs exec-mask juggling per element.
__device__ __forceinline__ float erf_nb(float x) {
  const float a = fabsf(x);
  const float p = a * a;
  float r = fmaf(p, -0x1.268bc2p-11f, 0x1.420828p-8f);
  r = fmaf(p, r, -0x1.b5937p-6f);
  r = fmaf(p, r, 0x1.ce077cp-4f);
  r = fmaf(p, r, -0x1.81266p-2f);
  r = fmaf(p, r, 0x1.06eba0p-3f);
  const float small = fmaf(a, r, a);
  float q = fmaf(a, 0x1.1d3156p-16f, -0x1.8d129p-12f);
  q = fmaf(a, q, 0x1.f9a6d2p-9f);
  q = fmaf(a, q, -0x1.8c3164p-6f);
  q = fmaf(a, q, 0x1.b4e9c8p-4f);
  q = fmaf(a, q, 0x1.4515fap-1f);
  q = fmaf(a, q, 0x1.078e50p-3f);
  q = fmaf(a, q, a);
  const float large = 1.f - expf(-q);
  return copysignf(a < 1.f ? small : large, x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_nb(x * kInvSqrt2)); }
__device__ __forceinline__ float gelu_g(float x) {
  float cdf = 0.5f * (1.f + erf_nb(x * kInvSqrt2));
  return cdf + x * (kInvSqrt2Pi * __expf(-0.5f * x * x));
}

// GELU for bf16 outputs: he = erfc(|z|/sqrt2)/2 by Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7,
// far below bf16 rounding), with the 1/sqrt2 folded into p and the 1/2 into the coefficients:
// he = t (a1 + t (a2 + ...)) e, t = 1/(1 + p|z|/sqrt2), e = exp(-z^2/2) -- e is also the factor
// GELU's derivative needs.  Returns q = he - 1/2 (in [-1/2, 0]); one rcp + one exp + 9 VALU.
__device__ __forceinline__ float gelu_q(float z, float& e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * kInvSqrt2, fabsf(z), 1.f));
  float p = fmaf(t, 0.5f * 1.061405429f, 0.5f * -1.453152027f);
  p = fmaf(t, p, 0.5f * 1.421413741f);
  p = fmaf(t, p, 0.5f * -0.284496736f);
  p = fmaf(t, p, 0.5f * 0.254829592f);
  e = __builtin_amdgcn_exp2f((z * z) * -0.72134752044448170368f);   // -log2(e)/2
  return fmaf(t * p, e, -0.5f);
}
// gelu(z) = z Phi(z) = z/2 - |z| q   (z >= 0: z (1 - he); z < 0: z he)
__device__ __forceinline__ float gelu_fast(float z) {
  float e;
  const float q = gelu_q(z, e);
  return fmaf(-fabsf(z), q, 0.5f * z);
}
// gelu(z) and gelu'(z) = Phi(z) + z phi(z) together; Phi(z) = 1/2 - sign(z) q
__device__ __forceinline__ void gelu_pair_fast(float z, float& g, float& gp) {
  float e;
  const float q = gelu_q(z, e);
  const float cdf = 0.5f + copysignf(-q, z);
  g = z * cdf;
  gp = fmaf(z * kInvSqrt2Pi, e, cdf);
}

// Two-element forms of the above on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: one
// wave instruction does both elements, so outside MFMA gaps they halve the VALU issue time of
// the polynomial; rcp and exp stay per element).  Same operations per element, same results.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 gelu_nq2(f32x2 z, f32x2 az, f32x2& e) {   // -q = 1/2 - he >= 0
  const f32x2 d = pk_fma(az, f32x2(0.3275911f * kInvSqrt2), f32x2(1.f));
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = pk_fma(t, f32x2(-0.5f * 1.061405429f), f32x2(-0.5f * -1.453152027f));   // -(polynomial): exact
  p = pk_fma(t, p, f32x2(-0.5f * 1.421413741f));
  p = pk_fma(t, p, f32x2(-0.5f * -0.284496736f));
  p = pk_fma(t, p, f32x2(-0.5f * 0.254829592f));
  const f32x2 w = (z * z) * f32x2(-0.72134752044448170368f);
  e = f32x2{__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  return pk_fma(t * p, e, f32x2(0.5f));
}
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 z) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  f32x2 e;
  const f32x2 nq = gelu_nq2(z, az, e);
  return pk_fma(az, nq, f32x2(0.5f) * z);
}
__device__ __forceinline__ void gelu_pair_fast2(f32x2 z, f32x2& g, f32x2& gp) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  f32x2 e;
  const f32x2 nq = gelu_nq2(z, az, e);
  const f32x2 cdf = f32x2(0.5f) + f32x2{copysignf(nq.x, z.x), copysignf(nq.y, z.y)};
  g = z * cdf;
  gp = pk_fma(z * f32x2(kInvSqrt2Pi), e, cdf);
}

// The same two on unpacked fp32, one element at a time (identical operations, identical bits).
// Beside MFMAs a v_pk_*_f32 costs more than the two single-lane instructions it replaces
// (MI355X_MICROARCH.md, per-instruction constants: +22 cycles per v_pk_fma_f32 per MFMA gap); the
// packed forms pay off only in VALU-only phases (GEMM epilogues).
__device__ __forceinline__ float gelu_nq1(float z, float& e) {
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(z), 0.3275911f * kInvSqrt2, 1.f));
  float p = fmaf(t, -0.5f * 1.061405429f, -0.5f * -1.453152027f);
  p = fmaf(t, p, -0.5f * 1.421413741f);
  p = fmaf(t, p, -0.5f * -0.284496736f);
  p = fmaf(t, p, -0.5f * 0.254829592f);
  const float w = (z * z) * -0.72134752044448170368f;
  e = __builtin_amdgcn_exp2f(w);
  return fmaf(t * p, e, 0.5f);
}
__device__ __forceinline__ f32x2 gelu_fast1x2(f32x2 z) {
  float e0, e1;
  const float n0 = gelu_nq1(z.x, e0), n1 = gelu_nq1(z.y, e1);
  return f32x2{fmaf(fabsf(z.x), n0, 0.5f * z.x), fmaf(fabsf(z.y), n1, 0.5f * z.y)};
}
__device__ __forceinline__ void gelu_pair_fast1x2(f32x2 z, f32x2& g, f32x2& gp) {
  float e0, e1;
  const float n0 = gelu_nq1(z.x, e0), n1 = gelu_nq1(z.y, e1);
  const float c0 = 0.5f + copysignf(n0, z.x), c1 = 0.5f + copysignf(n1, z.y);
  g = f32x2{z.x * c0, z.y * c1};
  gp = f32x2{fmaf(z.x * kInvSqrt2Pi, e0, c0), fmaf(z.y * kInvSqrt2Pi, e1, c1)};
}

__device__ __forceinline__ float act_f(int act, float x, float slope) {
  switch (act) {
    case ACT_GELU: return gelu_f(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_LRELU: return x > 0.f ? x : x * slope;
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case ACT_GELU_FAST: return gelu_fast(x);
    default: return x;
  }
}
// derivative of act at pre-activation x
__device__ __forceinline__ float act_g(int act, float x, float slope) {
  switch (act) {
    case ACT_GELU: return gelu_g(x);
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_LRELU: return x > 0.f ? 1.f : slope;
    case ACT_SIGMOID: { float s = 1.f / (1.f + __expf(-x)); return s * (1.f - s); }
    case ACT_GELU_FAST: { float g, gp; gelu_pair_fast(x, g, gp); return gp; }
    default: return 1.f;
  }
}

// Array forms for GEMM epilogues: the (uniform) activation switch sits OUTSIDE the element
// loop, so each case is a straight-line unrolled block (no per-element branches / waits).
template <int N>
__device__ __forceinline__ void act_f_arr(int act, float (&v)[N], float slope) {
  switch (act) {
    case ACT_NONE: break;
    case ACT_GELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = gelu_f(v[i]);
      break;
    case ACT_RELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = fmaxf(v[i], 0.f);
      break;
    case ACT_LRELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = v[i] > 0.f ? v[i] : v[i] * slope;
      break;
    default:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = act_f(act, v[i], slope);
  }
}
// v[i] *= act'(x[i])
template <int N>
__device__ __forceinline__ void act_g_mul_arr(int act, float (&v)[N], const float (&x)[N], float slope) {
  switch (act) {
    case ACT_NONE: break;
    case ACT_GELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] *= gelu_g(x[i]);
      break;
    case ACT_RELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = x[i] > 0.f ? v[i] : 0.f;
      break;
    case ACT_LRELU:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = x[i] > 0.f ? v[i] : v[i] * slope;
      break;
    default:
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] *= act_g(act, x[i], slope);
  }
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64).  `sh` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += sh[i];
  return r;
}

}  // namespace dsg

// ---- error plumbing for the C ABI -------------------------------------------------
extern "C" const char* dsgan_last_error_string(void);
void dsgan_set_error(const char* fmt, ...);

#define DSG_CHECK_LAUNCH()                                                   \
  do {                                                                       \
    hipError_t e__ = hipGetLastError();                                      \
    if (e__ != hipSuccess) {                                                 \
      dsgan_set_error("%s: %s", __func__, hipGetErrorString(e__));           \
      return (int)e__;                                                       \
    }                                                                        \
  } while (0)

#define DSG_REQUIRE(cond, ...)                                               \
  do {                                                                       \
    if (!(cond)) {                                                           \
      dsgan_set_error(__VA_ARGS__);                                          \
      return -1;                                                             \
    }                                                                        \
  } while (0)

static inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }

// ---- scratch (workspace) contract -------------------------------------------------
// Every entry point that takes a scratch buffer also takes its size `ws_elems` (fp32 elements, or
// the buffer's own element type where stated).  The launcher plans the launch it is about to issue,
// computes the scratch that plan writes (`need`) and refuses an undersized buffer with an error
// code instead of writing past it.  In plan-only mode (dsgan_set_plan_only, thread-local; CPU
// planner tests) the entry point returns 0 right after this check: no HIP call has been made by
// then, so every planner runs without a GPU.
namespace dsg {
bool plan_only();           // capi.cpp
void note_ws_need(long n);  // capi.cpp: dsgan_last_ws_need() reports it
// Kernel-only timer (dsgan_ktimer, capi.cpp): a launcher brackets ONE kernel launch -- not the split
// reductions or finishing passes its entry point also issues -- with ktimer_mark(st, 0) / (st, 1).
// Off by default (no HIP call then); bench.py's roofline leg turns it on.
void ktimer_mark(hipStream_t st, int end);
}  // namespace dsg
#define DSG_WS(need, ws, ws_elems, name)                                                              \
  do {                                                                                               \
    const long n__ = (long)(need);                                                                   \
    dsg::note_ws_need(n__);                                                                          \
    if (n__ > 0 && ((ws) == nullptr || n__ > (long)(ws_elems))) {                                    \
      dsgan_set_error("%s: scratch of %ld elements, this launch needs %ld", name, (long)(ws_elems), n__); \
      return -1;                                                                                     \
    }                                                                                                \
    if (dsg::plan_only()) return 0;                                                                  \
  } while (0)
