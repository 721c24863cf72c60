// InstanceNorm (+per-plane scale, +residual, +activation), max-pooling with indices,
// channel attention (CA), and the small elementwise/reduction kernels of the DS-GAN step.
//
// InstanceNorm2d(affine=False, eps=1e-5, biased variance) appears 35x in the generator and
// 3x in the PatchGAN D (DSGAN/models/model/MixConvNeXtML.py:54,80,151,158,221,335-420;
// DSGAN/models/networks.py:556,565).  One plane (n,c) is one workgroup (or one wave when the
// plane is small); the activation that follows it (GELU / LeakyReLU(0.2)) and, for MidMLKA
// (:113-116), the CA scaling before it and the residual add after it, are fused in.
#include "common.h"
#include <stdlib.h>

namespace dsg {

struct INArgs {
  const float* x; long x_bs;
  const float* scale;           // per-plane multiplier [N*C] applied to x first (nullable)
  const float* res; long res_bs;  // residual added after normalisation (nullable)
  float* y; long y_bs;
  float* mean; float* rstd;     // statistics of scale*x, [N*C]
  int N, C, HW, act; float slope, eps;
  int y_bf16;                   // y is 16-bit (1 bf16, 2 fp16; y_bs in elements): the block activation h whose only
                                // consumers are bf16-operand MFMA GEMMs (v4 kernels only)
};

// Plane reduction helper: NT threads per plane (NT = 64: one wave, else the whole block).
template <int NT>
__device__ __forceinline__ float plane_sum(float v, float* sh) {
  if (NT == 64) return warp_sum(v);
  return block_sum<NT>(v, sh);
}

// One plane per workgroup (NT = 256 / 1024) or per wave (NT = 64, 4 planes per 256-thread
// block).  Planes up to NT*CACHE elements are read ONCE into registers (two-pass mean/variance
// from registers); larger planes stream three times.
template <int NT, int CACHE>
__global__ __launch_bounds__(NT == 64 ? 256 : NT) void instnorm_fwd_kernel(INArgs a) {
  __shared__ float sh[16];
  const int planes_per_block = NT == 64 ? 4 : 1;
  const int plane = blockIdx.x * planes_per_block + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= a.N * a.C) return;  // whole wave / block uniform
  const int n = plane / a.C, c = plane - n * a.C;
  const float* x = a.x + (long)n * a.x_bs + (long)c * a.HW;
  const float s = a.scale ? a.scale[plane] : 1.f;
  float* y = a.y + (long)n * a.y_bs + (long)c * a.HW;
  const float* r = a.res ? a.res + (long)n * a.res_bs + (long)c * a.HW : nullptr;
  const float inv = 1.f / (float)a.HW;
  if (CACHE > 0) {
    float rv[CACHE > 0 ? CACHE : 1];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < CACHE; ++j) {
      const int i = t + j * NT;
      rv[j] = i < a.HW ? x[i] * s : 0.f;
      sum += rv[j];
    }
    const float mean = plane_sum<NT>(sum, sh) * inv;
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < CACHE; ++j) {
      const float d = rv[j] - mean;
      if (t + j * NT < a.HW) sq += d * d;
    }
    const float rs = 1.f / sqrtf(plane_sum<NT>(sq, sh) * inv + a.eps);
    if (t == 0) { a.mean[plane] = mean; a.rstd[plane] = rs; }
#pragma unroll
    for (int j = 0; j < CACHE; ++j) {
      const int i = t + j * NT;
      if (i < a.HW) {
        float v = (rv[j] - mean) * rs;
        if (r) v += r[i];
        y[i] = act_f(a.act, v, a.slope);
      }
    }
  } else {
    float sum = 0.f;
    for (int i = t; i < a.HW; i += NT) sum += x[i] * s;
    const float mean = plane_sum<NT>(sum, sh) * inv;
    float sq = 0.f;
    for (int i = t; i < a.HW; i += NT) { const float d = x[i] * s - mean; sq += d * d; }
    const float rs = 1.f / sqrtf(plane_sum<NT>(sq, sh) * inv + a.eps);
    if (t == 0) { a.mean[plane] = mean; a.rstd[plane] = rs; }
    for (int i = t; i < a.HW; i += NT) {
      float v = (x[i] * s - mean) * rs;
      if (r) v += r[i];
      y[i] = act_f(a.act, v, a.slope);
    }
  }
}

struct INBwdArgs {
  const float* dy; long dy_bs;
  const float* x; long x_bs;
  const float* scale;
  const float* res; long res_bs;
  const float* mean; const float* rstd;
  float* dx; long dx_bs;
  float* dres; long dres_bs;   // nullable
  float* dscale;               // nullable, [N*C] (written)
  int N, C, HW, act; float slope, eps;
  void* dxh;                   // nullable: dx stored 16-bit (the library half type) here instead of dx
  float* dxsum;                // nullable, [N*C]: per-plane sum of the fp32 dx (before rounding)
  int half;                    // half type of dxh (HALF_BF16 / HALF_F16)
};

// y = act(xhat + res), xhat = (s*x - mean) * rstd
// g = dy * act'(xhat + res);  dres = g;  dxs = rstd * (g - mean(g) - xhat * mean(g * xhat))
// dx = s * dxs;  dscale = sum_p dxs * x.  The sum cancels to O(eps) (IN is scale invariant up to
// eps), so it is evaluated in closed form: sum dxs = 0 and sum xhat^2 = HW*var*rstd^2 give
//   dscale = mean(g*xhat) * HW * eps * rstd^2 / s
// which is what the fp64 reference converges to; the direct fp32 sum loses ~1e-3 relative.
// g is cached in registers (planes <= NT*CACHE); xhat is recomputed from x in the final pass.
template <int NT, int CACHE>
__global__ __launch_bounds__(NT == 64 ? 256 : NT) void instnorm_bwd_kernel(INBwdArgs a) {
  __shared__ float sh[16];
  const int planes_per_block = NT == 64 ? 4 : 1;
  const int plane = blockIdx.x * planes_per_block + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= a.N * a.C) return;
  const int n = plane / a.C, c = plane - n * a.C;
  const long po = (long)c * a.HW;
  const float* x = a.x + (long)n * a.x_bs + po;
  const float* dy = a.dy + (long)n * a.dy_bs + po;
  const float* r = a.res ? a.res + (long)n * a.res_bs + po : nullptr;
  float* dres = a.dres ? a.dres + (long)n * a.dres_bs + po : nullptr;
  const float s = a.scale ? a.scale[plane] : 1.f;
  const float mean = a.mean[plane], rs = a.rstd[plane];
  float* dx = a.dx + (long)n * a.dx_bs + po;
  auto grad_at = [&](int i, float& xh) -> float {
    xh = (x[i] * s - mean) * rs;
    float g = dy[i];
    if (a.act != ACT_NONE) g *= act_g(a.act, r ? xh + r[i] : xh, a.slope);
    if (dres) dres[i] = g;
    return g;
  };
  const float inv = 1.f / (float)a.HW;
  float sg = 0.f, sgh = 0.f;
  if (CACHE > 0) {
    float gv[CACHE > 0 ? CACHE : 1];
#pragma unroll
    for (int j = 0; j < CACHE; ++j) {
      const int i = t + j * NT;
      gv[j] = 0.f;
      if (i < a.HW) { float xh; gv[j] = grad_at(i, xh); sg += gv[j]; sgh += gv[j] * xh; }
    }
    const float mg = plane_sum<NT>(sg, sh) * inv;
    const float mgh = plane_sum<NT>(sgh, sh) * inv;
#pragma unroll
    for (int j = 0; j < CACHE; ++j) {
      const int i = t + j * NT;
      if (i < a.HW) {
        const float xh = (x[i] * s - mean) * rs;
        dx[i] = s * rs * (gv[j] - mg - xh * mgh);
      }
    }
    if (a.dscale && t == 0) a.dscale[plane] = mgh * (float)a.HW * a.eps * rs * rs / s;
  } else {
    for (int i = t; i < a.HW; i += NT) { float xh; const float g = grad_at(i, xh); sg += g; sgh += g * xh; }
    const float mg = plane_sum<NT>(sg, sh) * inv;
    const float mgh = plane_sum<NT>(sgh, sh) * inv;
    for (int i = t; i < a.HW; i += NT) {
      const float xh = (x[i] * s - mean) * rs;
      float g = dy[i];
      if (a.act != ACT_NONE) g *= act_g(a.act, r ? xh + r[i] : xh, a.slope);
      dx[i] = s * rs * (g - mg - xh * mgh);
    }
    if (a.dscale && t == 0) a.dscale[plane] = mgh * (float)a.HW * a.eps * rs * rs / s;
  }
}

// ---- float4 forms (HW % 4 == 0, 16-byte aligned planes: every G/D plane but PatchGAN's 31x31) ----
// Same math as above with 16-byte accesses: the scalar forms issue 256-byte wave loads and
// reach only 2-4 TB/s on 64K/16K-pixel planes.  C4 float4s per thread are cached in registers
// (C4 == 0: the plane streams, three passes fwd / five bwd); the bwd caches g and, with CX,
// xhat too (x is then read once).
template <int NT>
__device__ __forceinline__ float2 plane_sum2(float u, float v, float* sh) {
  u = warp_sum(u);
  v = warp_sum(v);
  if (NT == 64) return make_float2(u, v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) { sh[w] = u; sh[NT / 64 + w] = v; }
  __syncthreads();
  float2 r = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) { r.x += sh[i]; r.y += sh[NT / 64 + i]; }
  return r;
}

__device__ __forceinline__ float hsum4(float4 v) { return (v.x + v.y) + (v.z + v.w); }

template <int NT, int C4>
__global__ __launch_bounds__(NT == 64 ? 256 : NT) void instnorm_fwd_v4(INArgs a) {
  __shared__ float sh[32];
  const int plane = blockIdx.x * (NT == 64 ? 4 : 1) + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= a.N * a.C) return;
  const int n = plane / a.C, c = plane - n * a.C;
  const int HW4 = a.HW >> 2;
  const float4* x = reinterpret_cast<const float4*>(a.x + (long)n * a.x_bs + (long)c * a.HW);
  float4* y = reinterpret_cast<float4*>(a.y + (long)n * a.y_bs + (long)c * a.HW);
  const float4* r = a.res ? reinterpret_cast<const float4*>(a.res + (long)n * a.res_bs + (long)c * a.HW) : nullptr;
  const float s = a.scale ? a.scale[plane] : 1.f;
  const float inv = 1.f / (float)a.HW;
  auto out = [&](int i, float4 v, float mean, float rs) {
    v.x = (v.x - mean) * rs; v.y = (v.y - mean) * rs; v.z = (v.z - mean) * rs; v.w = (v.w - mean) * rs;
    if (r) { const float4 q = r[i]; v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w; }
    v.x = act_f(a.act, v.x, a.slope); v.y = act_f(a.act, v.y, a.slope);
    v.z = act_f(a.act, v.z, a.slope); v.w = act_f(a.act, v.w, a.slope);
    if (a.y_bf16 == 2) {   // fp16 (--precision fp16), round-to-nearest-even like the GEMMs' operand loads
      hx4<_Float16> hv = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
      reinterpret_cast<hx4<_Float16>*>(reinterpret_cast<_Float16*>(a.y) + (long)n * a.y_bs + (long)c * a.HW)[i] = hv;
    } else if (a.y_bf16) {   // bf16, round-to-nearest-even, the same rounding the GEMMs apply to fp32 operands
      hx4<__bf16> hv = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
      reinterpret_cast<hx4<__bf16>*>(reinterpret_cast<__bf16*>(a.y) + (long)n * a.y_bs + (long)c * a.HW)[i] = hv;
    } else {
      y[i] = v;
    }
  };
  auto ld = [&](int i) -> float4 {
    float4 v = x[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    return v;
  };
  if constexpr (C4 > 0) {
    float4 rv[C4];
    float sum = 0.f;
    // a plane of exactly C4 = 4 float4s per thread takes unguarded loads and stores (the same values
    // in the same order: same bits).  Build A/B on two boxes (profiles/r04/in_micro_full*.txt): the
    // 4K-pixel planes of the 256 x 4 form 45 -> 42 us (1024 @ 32^2: 24 -> 22) on both; with C4 = 16
    // the 16K-pixel planes went 108 -> 113 us on one box and the 64K-pixel ones -4 % on one box,
    // +2.5 % on the other, so those keep the guarded loop.
    const bool full = C4 <= 4 && HW4 == C4 * NT;
    if (full) {
#pragma unroll
      for (int j = 0; j < C4; ++j) rv[j] = ld(t + j * NT);
    } else {
#pragma unroll
      for (int j = 0; j < C4; ++j) {
        const int i = t + j * NT;
        rv[j] = i < HW4 ? ld(i) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < C4; ++j) sum += hsum4(rv[j]);
    const float mean = plane_sum<NT>(sum, sh) * inv;
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      if (t + j * NT < HW4) {
        const float dx = rv[j].x - mean, dy = rv[j].y - mean, dz = rv[j].z - mean, dw = rv[j].w - mean;
        sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
    }
    const float rs = 1.f / sqrtf(plane_sum<NT>(sq, sh) * inv + a.eps);
    if (t == 0) { a.mean[plane] = mean; a.rstd[plane] = rs; }
    if (full) {
#pragma unroll
      for (int j = 0; j < C4; ++j) out(t + j * NT, rv[j], mean, rs);
    } else {
#pragma unroll
      for (int j = 0; j < C4; ++j) {
        const int i = t + j * NT;
        if (i < HW4) out(i, rv[j], mean, rs);
      }
    }
  } else {
    float sum = 0.f;
    for (int i0 = t; i0 < HW4; i0 += 4 * NT) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + u * NT < HW4 ? ld(i0 + u * NT) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 4; ++u) sum += hsum4(v[u]);
    }
    const float mean = plane_sum<NT>(sum, sh) * inv;
    float sq = 0.f;
    for (int i0 = t; i0 < HW4; i0 += 4 * NT) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = i0 + u * NT < HW4 ? ld(i0 + u * NT) : make_float4(mean, mean, mean, mean);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float dx = v[u].x - mean, dy = v[u].y - mean, dz = v[u].z - mean, dw = v[u].w - mean;
        sq += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
    }
    const float rs = 1.f / sqrtf(plane_sum<NT>(sq, sh) * inv + a.eps);
    if (t == 0) { a.mean[plane] = mean; a.rstd[plane] = rs; }
    for (int i0 = t; i0 < HW4; i0 += 4 * NT) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) if (i0 + u * NT < HW4) v[u] = ld(i0 + u * NT);
#pragma unroll
      for (int u = 0; u < 4; ++u) if (i0 + u * NT < HW4) out(i0 + u * NT, v[u], mean, rs);
    }
  }
}

// XL (> 0 only with !CX): the first XL of a thread's C4 xhat float4s are parked in LDS between the
// statistics pass and the output pass instead of being recomputed from a second read of x.  The
// 64K-pixel planes (NT = 1024, C4 = 16) cannot hold xhat in registers next to g, and a plane of x
// (256 KB) does not stay in the CU's share of L2, so the second read went to HBM: XL = 8 keeps half
// of it in 128 KB of LDS (the workgroup is alone on its CU either way).  Same values, same bits.
// ACTT >= 0: the activation fixed at compile time (the launcher dispatches on a.act), so the cached
// form's loop body has no branches and the scheduler can keep several items' loads in flight.
template <int NT, int C4, bool CX, int XL = 0, int ACTT = -1>
__global__ __launch_bounds__(NT == 64 ? 256 : NT) void instnorm_bwd_v4(INBwdArgs a) {
  static_assert(XL == 0 || (!CX && XL <= C4 && NT > 64), "XL: LDS-parked xhat of the uncached form");
  __shared__ float sh[32];
  __shared__ float4 xl[XL > 0 ? XL * NT : 1];
  const int plane = blockIdx.x * (NT == 64 ? 4 : 1) + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= a.N * a.C) return;
  const int n = plane / a.C, c = plane - n * a.C;
  const long po = (long)c * a.HW;
  const int HW4 = a.HW >> 2;
  const float4* x = reinterpret_cast<const float4*>(a.x + (long)n * a.x_bs + po);
  const float4* dy = reinterpret_cast<const float4*>(a.dy + (long)n * a.dy_bs + po);
  const float4* r = a.res ? reinterpret_cast<const float4*>(a.res + (long)n * a.res_bs + po) : nullptr;
  float4* dres = a.dres ? reinterpret_cast<float4*>(a.dres + (long)n * a.dres_bs + po) : nullptr;
  float4* dx = reinterpret_cast<float4*>(a.dx + (long)n * a.dx_bs + po);
  const float s = a.scale ? a.scale[plane] : 1.f;
  const float mean = a.mean[plane], rs = a.rstd[plane];
  const float inv = 1.f / (float)a.HW;
  auto xhat = [&](int i) -> float4 {
    float4 v = x[i];
    v.x = (v.x * s - mean) * rs; v.y = (v.y * s - mean) * rs; v.z = (v.z * s - mean) * rs; v.w = (v.w * s - mean) * rs;
    return v;
  };
  auto grad = [&](int i, float4 xh) -> float4 {
    float4 g = dy[i];
    if (a.act != ACT_NONE) {
      float4 z = xh;
      if (r) { const float4 q = r[i]; z.x += q.x; z.y += q.y; z.z += q.z; z.w += q.w; }
      g.x *= act_g(a.act, z.x, a.slope); g.y *= act_g(a.act, z.y, a.slope);
      g.z *= act_g(a.act, z.z, a.slope); g.w *= act_g(a.act, z.w, a.slope);
    }
    if (dres) dres[i] = g;
    return g;
  };
  // 16-bit dx (dxh): its only readers are 16-bit-operand MFMA kernels, which round it the same way
  unsigned short* dxh = a.dxh ? reinterpret_cast<unsigned short*>(a.dxh) + (long)n * a.dx_bs + po : nullptr;
  float dsum = 0.f;
  auto fin = [&](int i, float4 g, float4 xh, float mg, float mgh) {
    const float k = s * rs;
    const float4 v = make_float4(k * (g.x - mg - xh.x * mgh), k * (g.y - mg - xh.y * mgh), k * (g.z - mg - xh.z * mgh),
                                 k * (g.w - mg - xh.w * mgh));
    if (dxh) {
      uint2 u;
      if (a.half == HALF_F16) {
        u.x = (unsigned)f2h<_Float16>(v.x) | ((unsigned)f2h<_Float16>(v.y) << 16);
        u.y = (unsigned)f2h<_Float16>(v.z) | ((unsigned)f2h<_Float16>(v.w) << 16);
      } else {
        u.x = (unsigned)f2h<__bf16>(v.x) | ((unsigned)f2h<__bf16>(v.y) << 16);
        u.y = (unsigned)f2h<__bf16>(v.z) | ((unsigned)f2h<__bf16>(v.w) << 16);
      }
      *reinterpret_cast<uint2*>(dxh + 4 * i) = u;
      dsum += hsum4(v);
    } else {
      dx[i] = v;
    }
  };
  float sg = 0.f, sgh = 0.f;
  float2 m;
  if constexpr (C4 > 0 && NT == 1024) {
    // (64K-pixel planes: the scheduled form below spills at this size's 128-register cap, so the
    // item loop keeps its guarded per-item order; XL parks half of xhat in LDS instead)
    float4 gv[C4];
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      const int i = t + j * NT;
      gv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < HW4) {
        const float4 xh = xhat(i);
        if constexpr (XL > 0) {
          if (j < XL) xl[j * NT + t] = xh;
        }
        gv[j] = grad(i, xh);
        sg += hsum4(gv[j]);
        sgh += (gv[j].x * xh.x + gv[j].y * xh.y) + (gv[j].z * xh.z + gv[j].w * xh.w);
      }
    }
    m = plane_sum2<NT>(sg, sgh, sh);
    m.x *= inv; m.y *= inv;
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      const int i = t + j * NT;
      if (i < HW4) {
        if (XL > 0 && j < XL) fin(i, gv[j], xl[j * NT + t], m.x, m.y);
        else fin(i, gv[j], xhat(i), m.x, m.y);
      }
    }
  } else if constexpr (C4 > 0) {
    // Loads through plane-sized buffer resources (an item past the plane reads 0: no guard, no
    // branch), the activation fixed at compile time, and no global store inside the statistics loop
    // (dres is written afterwards).  A guarded load sits in its own basic block, and a load after a
    // store may not be hoisted above it: each item had waited one memory latency.  Same values and
    // the same summation order (an out-of-plane item adds +0): same bits.
    const int act = ACTT >= 0 ? ACTT : a.act;
    const unsigned prange = (unsigned)a.HW * 4u;
    const __amdgpu_buffer_rsrc_t bx = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, prange, 0x00020000);
    const __amdgpu_buffer_rsrc_t bd = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, prange, 0x00020000);
    const __amdgpu_buffer_rsrc_t br =
        __builtin_amdgcn_make_buffer_rsrc(r ? (void*)r : (void*)dy, (short)0, r ? prange : 0u, 0x00020000);
    auto bld4 = [](__amdgpu_buffer_rsrc_t rc, int i) {
      return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rc, i * 16, 0, 0));
    };
    auto bxhat = [&](int i) -> float4 {
      float4 v = bld4(bx, i);
      v.x = (v.x * s - mean) * rs; v.y = (v.y * s - mean) * rs; v.z = (v.z * s - mean) * rs; v.w = (v.w * s - mean) * rs;
      return v;
    };
    float4 gv[C4];
    float4 xv[CX ? C4 : 1];
#pragma unroll
    for (int j = 0; j < C4; ++j) {
      const int i = t + j * NT;
      const float4 xh = bxhat(i);
      float4 g = bld4(bd, i);
      if (act != ACT_NONE) {
        float4 z = xh;
        // (no residual: a zero-range buffer reads 0 and z stays xhat -- no branch, no traffic)
        const float4 q = bld4(br, i);
        z.x += q.x; z.y += q.y; z.z += q.z; z.w += q.w;
        g.x *= act_g(act, z.x, a.slope); g.y *= act_g(act, z.y, a.slope);
        g.z *= act_g(act, z.z, a.slope); g.w *= act_g(act, z.w, a.slope);
      }
      gv[j] = g;
      if constexpr (CX) xv[j] = xh;
      if constexpr (XL > 0) {
        if (j < XL) xl[j * NT + t] = xh;
      }
      sg += hsum4(g);
      sgh += (g.x * xh.x + g.y * xh.y) + (g.z * xh.z + g.w * xh.w);
    }
    if (dres) {
#pragma unroll
      for (int j = 0; j < C4; ++j)
        if (t + j * NT < HW4) dres[t + j * NT] = gv[j];
    }
    m = plane_sum2<NT>(sg, sgh, sh);
    m.x *= inv; m.y *= inv;
    // the recomputed xhat of the uncached items, in groups of FG loaded before their stores
    constexpr int FG = 4;
#pragma unroll
    for (int j0 = 0; j0 < C4; j0 += FG) {
      float4 xq[FG];
      if constexpr (!CX) {
#pragma unroll
        for (int u = 0; u < FG && j0 + u < C4; ++u) {
          const int i = t + (j0 + u) * NT;
          if (!(XL > 0 && j0 + u < XL)) xq[u] = bxhat(i);
        }
      }
#pragma unroll
      for (int u = 0; u < FG && j0 + u < C4; ++u) {
        const int j = j0 + u, i = t + j * NT;
        if (i < HW4) {
          if constexpr (CX) fin(i, gv[j], xv[j], m.x, m.y);
          else if (XL > 0 && j < XL) fin(i, gv[j], xl[j * NT + t], m.x, m.y);
          else fin(i, gv[j], xq[u], m.x, m.y);
        }
      }
    }
  } else {
    for (int i0 = t; i0 < HW4; i0 += 2 * NT) {
      float4 xh[2], g[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) if (i0 + u * NT < HW4) xh[u] = xhat(i0 + u * NT);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (i0 + u * NT < HW4) {
          g[u] = grad(i0 + u * NT, xh[u]);
          sg += hsum4(g[u]);
          sgh += (g[u].x * xh[u].x + g[u].y * xh[u].y) + (g[u].z * xh[u].z + g[u].w * xh[u].w);
        }
      }
    }
    m = plane_sum2<NT>(sg, sgh, sh);
    m.x *= inv; m.y *= inv;
    for (int i0 = t; i0 < HW4; i0 += 2 * NT) {
      float4 xh[2], g[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (i0 + u * NT < HW4) {
          xh[u] = xhat(i0 + u * NT);
          g[u] = dy[i0 + u * NT];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (i0 + u * NT < HW4) {
          if (a.act != ACT_NONE) {
            float4 z = xh[u];
            if (r) { const float4 q = r[i0 + u * NT]; z.x += q.x; z.y += q.y; z.z += q.z; z.w += q.w; }
            g[u].x *= act_g(a.act, z.x, a.slope); g[u].y *= act_g(a.act, z.y, a.slope);
            g[u].z *= act_g(a.act, z.z, a.slope); g[u].w *= act_g(a.act, z.w, a.slope);
          }
          fin(i0 + u * NT, g[u], xh[u], m.x, m.y);
        }
      }
    }
  }
  if (a.dscale && t == 0) a.dscale[plane] = m.y * (float)a.HW * a.eps * rs * rs / s;
  if (a.dxsum) {   // (uniform branch: every thread of the plane's block reaches the reduction)
    const float2 ds = plane_sum2<NT>(dsum, 0.f, sh);
    if (t == 0) a.dxsum[plane] = ds.x;
  }
}

// xhat float4s per thread parked in LDS by the 64K-pixel backward (instnorm_bwd_v4 XL; A/B in
// profiles/r04/in_micro_xl.txt: 8 of 16, 128 KB of LDS)
constexpr int IN_BWD_XL = 8;

// ---- few-plane forms: one plane split over S workgroups ----
// The generator's 3-channel block (MixConvNeXtML.py:220-221 at dim 3) normalises N*3 = 48 planes
// of 64K pixels: a workgroup per plane keeps 48 of the 256 CUs busy (72.6 us at 0.35 TB/s,
// profiles/r04/launches_c.txt).  Here each plane's S chunks (IN_SPLIT_F4 float4s, 4 per thread)
// are separate workgroups; the plane statistics are summed from per-chunk partials in a fixed
// order, so the result is deterministic (it is not the one-workgroup kernel's summation order).
// fwd: partial sums -> partial squared deviations -> output; bwd: partial (sum g, sum g*xhat) -> dx.
constexpr int IN_SPLIT_F4 = 1024;

static inline int in_split_chunks(long planes, int HW) {
  if ((HW & 3) || planes >= 128 || HW < 16384) return 0;
  return (int)cdiv(HW >> 2, IN_SPLIT_F4);
}

__device__ __forceinline__ float in_split_total(const float* p, int S, int stride) {
  float r = 0.f;
  for (int k = 0; k < S; ++k) r += p[k * stride];
  return r;
}

// PASS 0: ws[plane*S + k] = sum of s*x over chunk k;  PASS 1: ws[P*S + plane*S + k] = sum of (s*x - mean)^2
template <int PASS>
__global__ __launch_bounds__(256) void in_split_stat(INArgs a, float* __restrict__ ws, int S) {
  __shared__ float sh[4];
  const int k = blockIdx.x, plane = blockIdx.y, P = a.N * a.C;
  const int n = plane / a.C, c = plane - n * a.C;
  const int HW4 = a.HW >> 2;
  const float4* x = reinterpret_cast<const float4*>(a.x + (long)n * a.x_bs + (long)c * a.HW);
  const float s = a.scale ? a.scale[plane] : 1.f;
  const float mean = PASS ? in_split_total(ws + (long)plane * S, S, 1) * (1.f / (float)a.HW) : 0.f;
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < IN_SPLIT_F4 / 256; ++j) {
    const int i = k * IN_SPLIT_F4 + j * 256 + threadIdx.x;
    if (i < HW4) {
      float4 v = x[i];
      v.x *= s; v.y *= s; v.z *= s; v.w *= s;
      if (PASS == 0) {
        acc += hsum4(v);
      } else {
        const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
        acc += (dx * dx + dy * dy) + (dz * dz + dw * dw);
      }
    }
  }
  acc = block_sum<256>(acc, sh);
  if (threadIdx.x == 0) ws[(long)PASS * P * S + (long)plane * S + k] = acc;
}

__global__ __launch_bounds__(256) void in_split_out(INArgs a, const float* __restrict__ ws, int S) {
  const int k = blockIdx.x, plane = blockIdx.y, P = a.N * a.C;
  const int n = plane / a.C, c = plane - n * a.C;
  const int HW4 = a.HW >> 2;
  const long po = (long)c * a.HW;
  const float inv = 1.f / (float)a.HW;
  const float mean = in_split_total(ws + (long)plane * S, S, 1) * inv;
  const float rs = 1.f / sqrtf(in_split_total(ws + (long)P * S + (long)plane * S, S, 1) * inv + a.eps);
  if (k == 0 && threadIdx.x == 0) { a.mean[plane] = mean; a.rstd[plane] = rs; }
  const float4* x = reinterpret_cast<const float4*>(a.x + (long)n * a.x_bs + po);
  const float4* r = a.res ? reinterpret_cast<const float4*>(a.res + (long)n * a.res_bs + po) : nullptr;
  const float s = a.scale ? a.scale[plane] : 1.f;
#pragma unroll
  for (int j = 0; j < IN_SPLIT_F4 / 256; ++j) {
    const int i = k * IN_SPLIT_F4 + j * 256 + threadIdx.x;
    if (i >= HW4) continue;
    float4 v = x[i];
    v.x = (v.x * s - mean) * rs; v.y = (v.y * s - mean) * rs; v.z = (v.z * s - mean) * rs; v.w = (v.w * s - mean) * rs;
    if (r) { const float4 q = r[i]; v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w; }
    v.x = act_f(a.act, v.x, a.slope); v.y = act_f(a.act, v.y, a.slope);
    v.z = act_f(a.act, v.z, a.slope); v.w = act_f(a.act, v.w, a.slope);
    if (a.y_bf16 == 2) {
      hx4<_Float16> hv = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
      reinterpret_cast<hx4<_Float16>*>(reinterpret_cast<_Float16*>(a.y) + (long)n * a.y_bs + po)[i] = hv;
    } else if (a.y_bf16) {
      hx4<__bf16> hv = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
      reinterpret_cast<hx4<__bf16>*>(reinterpret_cast<__bf16*>(a.y) + (long)n * a.y_bs + po)[i] = hv;
    } else {
      reinterpret_cast<float4*>(a.y + (long)n * a.y_bs + po)[i] = v;
    }
  }
}

// g = dy * act'(xhat + res) (dres = g written here);  ws[(plane*S + k)*2 + {0,1}] = chunk sums of g, g*xhat
__device__ __forceinline__ float4 in_split_g(const INBwdArgs& a, int n, long po, int i, float4 xh) {
  float4 g = reinterpret_cast<const float4*>(a.dy + (long)n * a.dy_bs + po)[i];
  if (a.act != ACT_NONE) {
    float4 z = xh;
    if (a.res) {
      const float4 q = reinterpret_cast<const float4*>(a.res + (long)n * a.res_bs + po)[i];
      z.x += q.x; z.y += q.y; z.z += q.z; z.w += q.w;
    }
    g.x *= act_g(a.act, z.x, a.slope); g.y *= act_g(a.act, z.y, a.slope);
    g.z *= act_g(a.act, z.z, a.slope); g.w *= act_g(a.act, z.w, a.slope);
  }
  return g;
}

template <int PASS>   // 0: partial sums (+ dres);  1: dx (+ dscale)
__global__ __launch_bounds__(256) void in_split_bwd(INBwdArgs a, float* __restrict__ ws, int S) {
  __shared__ float sh[8];
  const int k = blockIdx.x, plane = blockIdx.y;
  const int n = plane / a.C, c = plane - n * a.C;
  const int HW4 = a.HW >> 2;
  const long po = (long)c * a.HW;
  const float4* x = reinterpret_cast<const float4*>(a.x + (long)n * a.x_bs + po);
  const float s = a.scale ? a.scale[plane] : 1.f;
  const float mean = a.mean[plane], rs = a.rstd[plane];
  const float inv = 1.f / (float)a.HW;
  float mg = 0.f, mgh = 0.f;
  if (PASS == 1) {
    mg = in_split_total(ws + (long)plane * S * 2, S, 2) * inv;
    mgh = in_split_total(ws + (long)plane * S * 2 + 1, S, 2) * inv;
  }
  float sg = 0.f, sgh = 0.f;
#pragma unroll
  for (int j = 0; j < IN_SPLIT_F4 / 256; ++j) {
    const int i = k * IN_SPLIT_F4 + j * 256 + threadIdx.x;
    if (i >= HW4) continue;
    float4 xh = x[i];
    xh.x = (xh.x * s - mean) * rs; xh.y = (xh.y * s - mean) * rs; xh.z = (xh.z * s - mean) * rs; xh.w = (xh.w * s - mean) * rs;
    const float4 g = in_split_g(a, n, po, i, xh);
    if (PASS == 0) {
      if (a.dres) reinterpret_cast<float4*>(a.dres + (long)n * a.dres_bs + po)[i] = g;
      sg += hsum4(g);
      sgh += (g.x * xh.x + g.y * xh.y) + (g.z * xh.z + g.w * xh.w);
    } else {
      const float kk = s * rs;
      reinterpret_cast<float4*>(a.dx + (long)n * a.dx_bs + po)[i] =
          make_float4(kk * (g.x - mg - xh.x * mgh), kk * (g.y - mg - xh.y * mgh), kk * (g.z - mg - xh.z * mgh),
                      kk * (g.w - mg - xh.w * mgh));
    }
  }
  if (PASS == 0) {
    const float2 m = plane_sum2<256>(sg, sgh, sh);
    if (threadIdx.x == 0) { ws[((long)plane * S + k) * 2] = m.x; ws[((long)plane * S + k) * 2 + 1] = m.y; }
  } else if (a.dscale && k == 0 && threadIdx.x == 0) {
    a.dscale[plane] = mgh * (float)a.HW * a.eps * rs * rs / s;
  }
}

// ---------------------------------------------------------------------------------------
// MaxPool2d(k) (stride k, no padding, floor): DSGAN/models/model/MixConvNeXtML.py:71,194,333-417
// Indices are the plane-flat argmax ih*W+iw, first maximum in row-major window order, NaN wins
// (the rule of PyTorch's CPU max_pool2d) -- bit-exact with the reference's int64 indices.
// ---------------------------------------------------------------------------------------
// 2-D grid: blockIdx.y walks planes (n,c), blockIdx.x chunks of the plane; 32-bit index math.
// Fast path (H, W divisible by K, aligned rows): one thread per output window, the window rows
// moved with 8/16-byte vector accesses (consecutive lanes = consecutive windows).
template <int K>
__device__ __forceinline__ void load_row(const float* p, float* v) {
  if constexpr (K == 2) { const float2 t = *reinterpret_cast<const float2*>(p); v[0] = t.x; v[1] = t.y; }
  else {
#pragma unroll
    for (int j = 0; j < K; j += 4) {
      const float4 t = *reinterpret_cast<const float4*>(p + j);
      v[j] = t.x; v[j + 1] = t.y; v[j + 2] = t.z; v[j + 3] = t.w;
    }
  }
}
template <int K>
__device__ __forceinline__ void store_row(float* p, const float* v) {
  if constexpr (K == 2) { *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]); }
  else {
#pragma unroll
    for (int j = 0; j < K; j += 4) *reinterpret_cast<float4*>(p + j) = make_float4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  }
}

template <int K>
__global__ void maxpool_fwd_win_kernel(const float* __restrict__ x, long x_bs, float* __restrict__ y,
                                       long y_bs, int* __restrict__ idx, int N, int C, int H, int W) {
  const int Ho = H / K, Wo = W / K, Po = Ho * Wo;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* xp = x + (long)n * x_bs + (long)c * H * W;
    float* yp = y + (long)n * y_bs + (long)c * Po;
    int* ip = idx + (long)plane * Po;
    for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < Po; o += gridDim.x * blockDim.x) {
      const int oh = o / Wo, ow = o - oh * Wo;
      float best = -INFINITY; int bi = (oh * K) * W + ow * K;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        float v[K];
        load_row<K>(xp + (oh * K + i) * W + ow * K, v);
#pragma unroll
        for (int j = 0; j < K; ++j)
          if (v[j] > best || isnan(v[j])) { best = v[j]; bi = (oh * K + i) * W + ow * K + j; }
      }
      yp[o] = best;
      ip[o] = bi;
    }
  }
}

template <int K>
__global__ void maxpool_bwd_win_kernel(const float* __restrict__ dy, long dy_bs, const int* __restrict__ idx,
                                       float* __restrict__ dx, long dx_bs, int N, int C, int H, int W,
                                       int accumulate) {
  const int Ho = H / K, Wo = W / K, Po = Ho * Wo;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* gp = dy + (long)n * dy_bs + (long)c * Po;
    const int* ip = idx + (long)plane * Po;
    float* dp = dx + (long)n * dx_bs + (long)c * H * W;
    for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < Po; o += gridDim.x * blockDim.x) {
      const int oh = o / Wo, ow = o - oh * Wo;
      const int id = ip[o];
      const float gv = gp[o];
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const int rb = (oh * K + i) * W + ow * K;
        float v[K];
        if (accumulate) load_row<K>(dp + rb, v);
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const float add = (rb + j == id) ? gv : 0.f;
          v[j] = accumulate ? v[j] + add : add;
        }
        store_row<K>(dp + rb, v);
      }
    }
  }
}

// 2x2 windows, two adjacent outputs per thread: one 16-byte load from each input row, 8-byte
// value/index stores (W % 4 == 0, 16-byte aligned input planes, 8-byte aligned outputs).  The
// window is scanned in the same row-major order as maxpool_fwd_win_kernel (NaN / tie rules
// of torch's max_pool2d_with_indices are unchanged).
__device__ __forceinline__ void mp_pick(float v, int pos, float& best, int& bi) {
  if (v > best || isnan(v)) { best = v; bi = pos; }
}
__global__ void maxpool2_fwd_x2_kernel(const float* __restrict__ x, long x_bs, float* __restrict__ y, long y_bs,
                                       int* __restrict__ idx, int N, int C, int H, int W) {
  const int Wo = W / 2, Po = (H / 2) * Wo, Wq = Wo / 2, Q = Po / 2;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* xp = x + (long)n * x_bs + (long)c * H * W;
    float* yp = y + (long)n * y_bs + (long)c * Po;
    int* ip = idx + (long)plane * Po;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += gridDim.x * blockDim.x) {
      const int oh = q / Wq, qw = q - oh * Wq;
      const int r0 = 2 * oh * W + 4 * qw;
      const float4 a = *reinterpret_cast<const float4*>(xp + r0);
      const float4 b = *reinterpret_cast<const float4*>(xp + r0 + W);
      float b0 = -INFINITY, b1 = -INFINITY; int i0 = r0, i1 = r0 + 2;
      mp_pick(a.x, r0, b0, i0);     mp_pick(a.y, r0 + 1, b0, i0);
      mp_pick(b.x, r0 + W, b0, i0); mp_pick(b.y, r0 + W + 1, b0, i0);
      mp_pick(a.z, r0 + 2, b1, i1);     mp_pick(a.w, r0 + 3, b1, i1);
      mp_pick(b.z, r0 + W + 2, b1, i1); mp_pick(b.w, r0 + W + 3, b1, i1);
      *reinterpret_cast<float2*>(yp + 2 * q) = make_float2(b0, b1);
      *reinterpret_cast<int2*>(ip + 2 * q) = make_int2(i0, i1);
    }
  }
}
__global__ void maxpool2_bwd_x2_kernel(const float* __restrict__ dy, long dy_bs, const int* __restrict__ idx,
                                       float* __restrict__ dx, long dx_bs, int N, int C, int H, int W,
                                       int accumulate) {
  const int Wo = W / 2, Po = (H / 2) * Wo, Wq = Wo / 2, Q = Po / 2;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* gp = dy + (long)n * dy_bs + (long)c * Po;
    const int* ip = idx + (long)plane * Po;
    float* dp = dx + (long)n * dx_bs + (long)c * H * W;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += gridDim.x * blockDim.x) {
      const int oh = q / Wq, qw = q - oh * Wq;
      const int r0 = 2 * oh * W + 4 * qw;
      const int2 id = *reinterpret_cast<const int2*>(ip + 2 * q);
      const float2 gv = *reinterpret_cast<const float2*>(gp + 2 * q);
      float4 a = make_float4((r0 == id.x) ? gv.x : 0.f, (r0 + 1 == id.x) ? gv.x : 0.f,
                             (r0 + 2 == id.y) ? gv.y : 0.f, (r0 + 3 == id.y) ? gv.y : 0.f);
      float4 b = make_float4((r0 + W == id.x) ? gv.x : 0.f, (r0 + W + 1 == id.x) ? gv.x : 0.f,
                             (r0 + W + 2 == id.y) ? gv.y : 0.f, (r0 + W + 3 == id.y) ? gv.y : 0.f);
      float4* pa = reinterpret_cast<float4*>(dp + r0);
      float4* pb = reinterpret_cast<float4*>(dp + r0 + W);
      if (accumulate) {
        const float4 oa = *pa, ob = *pb;
        a.x += oa.x; a.y += oa.y; a.z += oa.z; a.w += oa.w;
        b.x += ob.x; b.y += ob.y; b.z += ob.z; b.w += ob.w;
      }
      *pa = a;
      *pb = b;
    }
  }
}

// KxK windows with K % 4 == 0: one 16-byte dx chunk per thread (a chunk lies in one window), so
// a wave writes 1 KB of one input row contiguously instead of K/4 strided 16-byte pieces.
// Used for K = 8, 16 (84/65 us vs 107/77 us at 16x64x256x256); at K = 4 the window kernel's
// one index load per 16 outputs wins (52 vs 56 us).
template <int K>
__global__ void maxpool_bwd_row_kernel(const float* __restrict__ dy, long dy_bs, const int* __restrict__ idx,
                                       float* __restrict__ dx, long dx_bs, int N, int C, int H, int W,
                                       int accumulate) {
  static_assert(K % 4 == 0, "16-byte chunks must not straddle windows");
  const int Wo = W / K, Po = (H / K) * Wo, W4 = W / 4, n4 = H * W4;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* gp = dy + (long)n * dy_bs + (long)c * Po;
    const int* ip = idx + (long)plane * Po;
    float* dp = dx + (long)n * dx_bs + (long)c * H * W;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
      const int h = q / W4, c4 = q - h * W4;
      const int o = (h / K) * Wo + (c4 * 4) / K;
      const int id = ip[o] - (h * W + c4 * 4);
      const float gv = gp[o];
      float4 v = make_float4(id == 0 ? gv : 0.f, id == 1 ? gv : 0.f, id == 2 ? gv : 0.f, id == 3 ? gv : 0.f);
      float4* d = reinterpret_cast<float4*>(dp) + q;
      if (accumulate) {
        const float4 u = *d;
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
      }
      *d = v;
    }
  }
}

// ---- multi-scale max-pool pyramid (the generator's skip pyramids, MixConvNeXtML.py:328-426) ----
// MaxPool2d(2), (4), (8), (16) of one tensor from ONE read of it: R1 feeds the encoder's k = 2 pool
// and downSkip's k = 4 / 8 / 16 branches, R2 k = 2 / 4 / 8, R3 k = 2 / 4.  A wave owns a 16-row x
// 64-column tile of a plane; lane (r4 = lane / 16, c4 = lane % 16) holds the 4 x 4 input block at
// rows 4 r4.., cols 4 c4.. (four 16-byte row loads).  k = 2 and k = 4 scan the lane's block in
// row-major order with torch's rule (v > best || isnan(v), initial index = the window's first
// element); k = 8 and k = 16 merge 2 x 2 neighbour lanes' results (shuffles), keeping what a
// row-major scan of the whole window keeps: any NaN beats a number and the later NaN beats an
// earlier one; otherwise the larger value, and of equal values the smaller flat index.  Each
// sub-window's result is the first max / last NaN of its own row-major scan, and a rectangular
// sub-window's elements keep their relative row-major order inside the window, so the merge is
// exactly the window's scan: bit-exact values and int32 indices.
__device__ __forceinline__ void mp_merge(float& bv, int& bi, float v, int i) {
  if (isnan(bv)) {
    if (isnan(v) && i > bi) { bv = v; bi = i; }
  } else if (isnan(v) || v > bv || (v == bv && i < bi)) {
    bv = v; bi = i;
  }
}
struct PyrPtrs {
  float* y[4]; int* idx[4];                // forward outputs (levels k = 2, 4, 8, 16), dense [N][C][H/k][W/k]
  const float* dy[4]; long dy_bs[4];       // backward: output grads (nullable = no grad), batch strides
};
template <int L>
__global__ __launch_bounds__(256) void maxpool_pyr_fwd_kernel(const float* __restrict__ x, long x_bs, PyrPtrs p,
                                                             int C, int H, int W, long nwaves) {
  const long g = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nwaves) return;   // whole waves exit; no barrier below
  const int lane = threadIdx.x & 63, r4 = lane >> 4, c4 = lane & 15;
  const int TW = W >> 6, TP = (H >> 4) * TW;
  const int plane = (int)(g / TP), t = (int)(g - (long)plane * TP);
  const int n = plane / C, c = plane - n * C;
  const int bh = (t / TW) * 16 + 4 * r4, bw = (t % TW) * 64 + 4 * c4;
  const float* xp = x + (long)n * x_bs + (long)c * H * W + (long)bh * W + bw;
  float v[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float4 q = *reinterpret_cast<const float4*>(xp + (long)r * W);
    v[r][0] = q.x; v[r][1] = q.y; v[r][2] = q.z; v[r][3] = q.w;
  }
  const int base = bh * W + bw;
  {   // k = 2: four windows, two 8-byte value / index stores per lane
    const int W2 = W >> 1;
    const long o = (long)plane * (H >> 1) * W2 + (long)(bh >> 1) * W2 + (bw >> 1);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      float bv[2]; int bi[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        bv[b] = -INFINITY; bi[b] = base + 2 * a * W + 2 * b;
#pragma unroll
        for (int r = 2 * a; r < 2 * a + 2; ++r)
#pragma unroll
          for (int j = 2 * b; j < 2 * b + 2; ++j) mp_pick(v[r][j], base + r * W + j, bv[b], bi[b]);
      }
      *reinterpret_cast<float2*>(p.y[0] + o + a * W2) = make_float2(bv[0], bv[1]);
      *reinterpret_cast<int2*>(p.idx[0] + o + a * W2) = make_int2(bi[0], bi[1]);
    }
  }
  if constexpr (L >= 2) {   // k = 4: the lane's whole block
    float bv = -INFINITY; int bi = base;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) mp_pick(v[r][j], base + r * W + j, bv, bi);
    const int W4 = W >> 2;
    const long o4 = (long)plane * (H >> 2) * W4 + (long)(bh >> 2) * W4 + (bw >> 2);
    p.y[1][o4] = bv;
    p.idx[1][o4] = bi;
    if constexpr (L >= 3) {   // k = 8: 2 x 2 lanes
      mp_merge(bv, bi, __shfl_xor(bv, 1, 64), __shfl_xor(bi, 1, 64));
      mp_merge(bv, bi, __shfl_xor(bv, 16, 64), __shfl_xor(bi, 16, 64));
      if (((r4 | c4) & 1) == 0) {
        const int W8 = W >> 3;
        const long o8 = (long)plane * (H >> 3) * W8 + (long)(bh >> 3) * W8 + (bw >> 3);
        p.y[2][o8] = bv;
        p.idx[2][o8] = bi;
      }
      if constexpr (L >= 4) {   // k = 16: 4 x 4 lanes
        mp_merge(bv, bi, __shfl_xor(bv, 2, 64), __shfl_xor(bi, 2, 64));
        mp_merge(bv, bi, __shfl_xor(bv, 32, 64), __shfl_xor(bi, 32, 64));
        if (((r4 | c4) & 3) == 0) {
          const int W16 = W >> 4;
          const long o16 = (long)plane * (H >> 4) * W16 + (long)(bh >> 4) * W16 + (bw >> 4);
          p.y[3][o16] = bv;
          p.idx[3][o16] = bi;
        }
      }
    }
  }
}
// The pyramid's backward in one pass: each lane owns its 4 x 4 block of dx and adds, per level with a
// gradient, the output grad of the window whose argmax lies in the block -- a gather, no atomics.
// Per element the order is fixed: dx (accumulate) + k=2 + k=4 + k=8 + k=16 (at most one term per level).
template <int L>
__global__ __launch_bounds__(256) void maxpool_pyr_bwd_kernel(PyrPtrs p, float* __restrict__ dx, long dx_bs, int C,
                                                             int H, int W, long nwaves, int accumulate) {
  const long g = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nwaves) return;
  const int lane = threadIdx.x & 63, r4 = lane >> 4, c4 = lane & 15;
  const int TW = W >> 6, TP = (H >> 4) * TW;
  const int plane = (int)(g / TP), t = (int)(g - (long)plane * TP);
  const int n = plane / C, c = plane - n * C;
  const int bh = (t / TW) * 16 + 4 * r4, bw = (t % TW) * 64 + 4 * c4;
  float* dp = dx + (long)n * dx_bs + (long)c * H * W + (long)bh * W + bw;
  const int base = bh * W + bw;
  float o[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (accumulate) q = *reinterpret_cast<const float4*>(dp + (long)r * W);
    o[r][0] = q.x; o[r][1] = q.y; o[r][2] = q.z; o[r][3] = q.w;
  }
  // one window's (grad, argmax) into the block: rel = argmax - base, hit where rel == r * W + j
  auto add1 = [&](float gv, int id, int r0, int r1, int j0, int j1) __attribute__((always_inline)) {
    const int rel = id - base;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (r >= r0 && r < r1 && j >= j0 && j < j1) o[r][j] += (rel == r * W + j) ? gv : 0.f;
  };
  if (p.dy[0]) {
    const int W2 = W >> 1;
    const long po = (long)(bh >> 1) * W2 + (bw >> 1);
    const float* gy = p.dy[0] + (long)n * p.dy_bs[0] + (long)c * (H >> 1) * W2 + po;
    const int* gi = p.idx[0] + (long)plane * (H >> 1) * W2 + po;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float2 gv = *reinterpret_cast<const float2*>(gy + a * W2);
      const int2 id = *reinterpret_cast<const int2*>(gi + a * W2);
      add1(gv.x, id.x, 2 * a, 2 * a + 2, 0, 2);
      add1(gv.y, id.y, 2 * a, 2 * a + 2, 2, 4);
    }
  }
#pragma unroll
  for (int l = 1; l < L; ++l) {
    if (!p.dy[l]) continue;
    const int k = 2 << l, Wk = W / k;
    const long po = (long)(bh / k) * Wk + bw / k;
    const float gv = p.dy[l][(long)n * p.dy_bs[l] + (long)c * (H / k) * Wk + po];
    const int id = p.idx[l][(long)plane * (H / k) * Wk + po];
    add1(gv, id, 0, 4, 0, 4);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) *reinterpret_cast<float4*>(dp + (long)r * W) = make_float4(o[r][0], o[r][1], o[r][2], o[r][3]);
}

// Generic fallback (any H, W): element-parallel, zero fill beyond the floor windows.
__global__ void maxpool_fwd_kernel(const float* __restrict__ x, long x_bs, float* __restrict__ y,
                                   long y_bs, int* __restrict__ idx, int N, int C, int H, int W,
                                   int k) {
  const int Ho = H / k, Wo = W / k, Po = Ho * Wo;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* xp = x + (long)n * x_bs + (long)c * H * W;
    float* yp = y + (long)n * y_bs + (long)c * Po;
    int* ip = idx + (long)plane * Po;
    for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < Po; o += gridDim.x * blockDim.x) {
      const int oh = o / Wo, ow = o - oh * Wo;
      const float* wp = xp + (oh * k) * W + ow * k;
      float best = -INFINITY; int bi = (oh * k) * W + ow * k;
      for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
          const float v = wp[i * W + j];
          if (v > best || isnan(v)) { best = v; bi = (oh * k + i) * W + ow * k + j; }
        }
      yp[o] = best;
      ip[o] = bi;
    }
  }
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, long dy_bs, const int* __restrict__ idx,
                                   float* __restrict__ dx, long dx_bs, int N, int C, int H, int W,
                                   int k, int accumulate) {
  const int Ho = H / k, Wo = W / k, Po = Ho * Wo, HW = H * W;
  for (int plane = blockIdx.y; plane < N * C; plane += gridDim.y) {
    const int n = plane / C, c = plane - n * C;
    const float* gp = dy + (long)n * dy_bs + (long)c * Po;
    const int* ip = idx + (long)plane * Po;
    float* dp = dx + (long)n * dx_bs + (long)c * HW;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < HW; e += gridDim.x * blockDim.x) {
      const int ih = e / W, iw = e - ih * W;
      const int oh = ih / k, ow = iw / k;
      float v = 0.f;
      if (oh < Ho && ow < Wo) {
        const int o = oh * Wo + ow;
        if (ip[o] == e) v = gp[o];
      }
      dp[e] = accumulate ? dp[e] + v : v;
    }
  }
}

static inline dim3 plane_grid(long per_plane, long planes) {
  long gx = (per_plane + 255) / 256;
  if (gx > 1024) gx = 1024;
  long gy = planes > 65535 ? 65535 : planes;
  return dim3((unsigned)(gx < 1 ? 1 : gx), (unsigned)gy);
}

// ---------------------------------------------------------------------------------------
// CA (DSGAN/models/model/MixConvNeXtML.py:5-22): per-plane avg/max(+argmax), then the tiny
// shared MLP fc2(prelu(fc1(.))) on both, summed, sigmoid.
// ---------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void plane_stats_kernel(const float* __restrict__ x, long x_bs,
                                                          float* avg, float* mx, int* amax, int N,
                                                          int C, int HW) {
  __shared__ float shv[4];
  __shared__ int shi[4];
  __shared__ float shs[4];
  const int ppb = 256 / NT;
  const int plane = blockIdx.x * ppb + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= N * C) return;
  const int n = plane / C, c = plane - n * C;
  const float* xp = x + (long)n * x_bs + (long)c * HW;
  float s = 0.f, best = -INFINITY; int bi = 0x7fffffff;
  for (int i = t; i < HW; i += NT) {
    const float v = xp[i];
    s += v;
    if (v > best || (isnan(v) && !isnan(best))) { best = v; bi = i; }
  }
  // reduce max with smallest index among equal maxima (first occurrence)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    const bool take = (ov > best) || (ov == best && oi < bi) || (isnan(ov) && (!isnan(best) || oi < bi));
    if (take) { best = ov; bi = oi; }
  }
  s = warp_sum(s);
  if (NT == 256) {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { shv[w] = best; shi[w] = bi; shs[w] = s; }
    __syncthreads();
    if (threadIdx.x == 0) {
      best = shv[0]; bi = shi[0]; s = shs[0];
      for (int i = 1; i < 4; ++i) {
        const bool take = (shv[i] > best) || (shv[i] == best && shi[i] < bi) ||
                          (isnan(shv[i]) && (!isnan(best) || shi[i] < bi));
        if (take) { best = shv[i]; bi = shi[i]; }
        s += shs[i];
      }
    }
  }
  if (t == 0) { avg[plane] = s / (float)HW; mx[plane] = best; amax[plane] = bi; }
}

// One block per sample n.  C <= 1024, R = C/8 <= 128.
__global__ __launch_bounds__(256) void ca_fwd_kernel(const float* avg, const float* mx,
                                                     const float* w1, const float* w2,
                                                     const float* pa, float* att, float* hsave,
                                                     int C, int R) {
  extern __shared__ float sm[];
  float* sa = sm;            // C
  float* sx = sa + C;        // C
  float* hp = sx + C;        // R : prelu(h_avg) + prelu(h_max)
  const int n = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) { sa[c] = avg[n * C + c]; sx[c] = mx[n * C + c]; }
  __syncthreads();
  const float a = pa[0];
  const int wid = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int j = wid; j < R; j += blockDim.x / 64) {
    float ha = 0.f, hm = 0.f;
    for (int c = l; c < C; c += 64) { const float w = w1[j * C + c]; ha += w * sa[c]; hm += w * sx[c]; }
    ha = warp_sum(ha); hm = warp_sum(hm);
    if (l == 0) {
      hsave[(n * R + j) * 2 + 0] = ha;
      hsave[(n * R + j) * 2 + 1] = hm;
      hp[j] = (ha >= 0.f ? ha : a * ha) + (hm >= 0.f ? hm : a * hm);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float o = 0.f;
    for (int j = 0; j < R; ++j) o += w2[c * R + j] * hp[j];
    att[n * C + c] = 1.f / (1.f + __expf(-o));
  }
}

// Backward of CA for one sample per block.  Weight grads go to per-image partials in ws, summed
// over images in a fixed order by launch_split_reduce (deterministic, no atomics).
__global__ __launch_bounds__(256) void ca_bwd_kernel(const float* datt, const float* att,
                                                     const float* avg, const float* mx,
                                                     const float* hsave, const float* w1,
                                                     const float* w2, const float* pa, float* davg,
                                                     float* dmx, float* ws, int want_w1, int want_w2,
                                                     int want_pa, int C, int R) {
  // per-image partials (summed over images in a fixed order by launch_split_reduce):
  // ws = [N][R*C] dw1 | [N][C*R] dw2 | [N] dpa
  extern __shared__ float sm[];
  __shared__ float dal_w[16];
  float* dO = sm;           // C
  float* hp = dO + C;       // R
  float* dha = hp + R;      // R
  float* dhm = dha + R;     // R
  const int n = blockIdx.x;
  const float a = pa[0];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float s = att[n * C + c];
    dO[c] = datt[n * C + c] * s * (1.f - s);
  }
  for (int j = threadIdx.x; j < R; j += blockDim.x) {
    const float ha = hsave[(n * R + j) * 2], hm = hsave[(n * R + j) * 2 + 1];
    hp[j] = (ha >= 0.f ? ha : a * ha) + (hm >= 0.f ? hm : a * hm);
  }
  __syncthreads();
  const int wid = threadIdx.x >> 6, l = threadIdx.x & 63;
  float dal = 0.f;
  for (int j = wid; j < R; j += blockDim.x / 64) {
    float dp = 0.f;
    for (int c = l; c < C; c += 64) dp += w2[c * R + j] * dO[c];
    dp = warp_sum(dp);
    if (l == 0) {
      const float ha = hsave[(n * R + j) * 2], hm = hsave[(n * R + j) * 2 + 1];
      dha[j] = ha > 0.f ? dp : a * dp;
      dhm[j] = hm > 0.f ? dp : a * dp;
      dal += (ha > 0.f ? 0.f : ha * dp) + (hm > 0.f ? 0.f : hm * dp);
    }
  }
  if (l == 0) dal_w[wid] = dal;
  __syncthreads();
  const int N = gridDim.x;
  float* ws_w1 = ws + (long)n * R * C;
  float* ws_w2 = ws + (long)N * R * C + (long)n * C * R;
  if (want_pa && threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) t += dal_w[w];
    ws[2L * N * R * C + n] = t;
  }
  if (want_w2)
    for (int e = threadIdx.x; e < C * R; e += blockDim.x) ws_w2[e] = dO[e / R] * hp[e % R];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float ga = 0.f, gm = 0.f;
    const float va = avg[n * C + c], vm = mx[n * C + c];
    for (int j = 0; j < R; ++j) {
      const float w = w1[j * C + c];
      ga += w * dha[j]; gm += w * dhm[j];
      if (want_w1) ws_w1[j * C + c] = dha[j] * va + dhm[j] * vm;
    }
    davg[n * C + c] = ga; dmx[n * C + c] = gm;
  }
}

// dx[n,c,:] += davg/HW ; dx[n,c,argmax] += dmax
// 16-byte forms (HW % 4 == 0, 16-byte aligned planes): each lane walks its float4 groups in increasing
// index order (4 loads in flight), the max / first-argmax update is branch-free with the scalar
// kernel's rule (strict >, NaN wins and sticks), and the cross-lane reduction is the same.
template <int NT>
__global__ __launch_bounds__(256) void plane_stats4_kernel(const float* __restrict__ x, long x_bs, float* avg, float* mx,
                                                           int* amax, int N, int C, int HW) {
  __shared__ float shv[4];
  __shared__ int shi[4];
  __shared__ float shs[4];
  const int ppb = 256 / NT;
  const int plane = blockIdx.x * ppb + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= N * C) return;
  const int n = plane / C, c = plane - n * C;
  const float4* xp = reinterpret_cast<const float4*>(x + (long)n * x_bs + (long)c * HW);
  const int HW4 = HW >> 2;
  float s = 0.f, best = -INFINITY;
  int bi = 0x7fffffff;
  auto upd = [&](float v, int i) {
    const bool take = v > best || (isnan(v) && !isnan(best));
    best = take ? v : best;
    bi = take ? i : bi;
  };
#pragma unroll 4
  for (int i4 = t; i4 < HW4; i4 += NT) {
    const float4 v = xp[i4];
    s += (v.x + v.y) + (v.z + v.w);
    upd(v.x, 4 * i4); upd(v.y, 4 * i4 + 1); upd(v.z, 4 * i4 + 2); upd(v.w, 4 * i4 + 3);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    const bool take = (ov > best) || (ov == best && oi < bi) || (isnan(ov) && (!isnan(best) || oi < bi));
    if (take) { best = ov; bi = oi; }
  }
  s = warp_sum(s);
  if (NT == 256) {
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { shv[w] = best; shi[w] = bi; shs[w] = s; }
    __syncthreads();
    if (threadIdx.x == 0) {
      best = shv[0]; bi = shi[0]; s = shs[0];
      for (int i = 1; i < 4; ++i) {
        const bool take = (shv[i] > best) || (shv[i] == best && shi[i] < bi) ||
                          (isnan(shv[i]) && (!isnan(best) || shi[i] < bi));
        if (take) { best = shv[i]; bi = shi[i]; }
        s += shs[i];
      }
    }
  }
  if (t == 0) { avg[plane] = s / (float)HW; mx[plane] = best; amax[plane] = bi; }
}

// dx (+)= davg / HW + (i == amax) dmx, four pixels of one plane per thread (HW % 4 == 0, aligned)
__global__ __launch_bounds__(256) void plane_stats_bwd4_kernel(const float* __restrict__ davg, const float* __restrict__ dmx,
                                                               const int* __restrict__ amax, float* __restrict__ dx,
                                                               long dx_bs, int N, int C, int HW) {
  const int HW4 = HW >> 2;
  const long total4 = (long)N * C * HW4;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total4; e += (long)gridDim.x * 256) {
    const long pl = e / HW4;
    const int i4 = (int)(e - pl * HW4);
    const int c = (int)(pl % C), n = (int)(pl / C);
    const float a = davg[pl] / (float)HW, m = dmx[pl];
    const int am = amax[pl] - 4 * i4;
    float4* o = reinterpret_cast<float4*>(dx + (long)n * dx_bs + (long)c * HW) + i4;
    float4 v = *o;
    v.x += am == 0 ? a + m : a; v.y += am == 1 ? a + m : a; v.z += am == 2 ? a + m : a; v.w += am == 3 ? a + m : a;
    *o = v;
  }
}

__global__ void plane_stats_bwd_kernel(const float* davg, const float* dmx, const int* amax,
                                       float* dx, long dx_bs, int N, int C, int HW) {
  const long total = (long)N * C * HW;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = e % HW; const long pl = e / HW;
    const int c = pl % C, n = pl / C;
    float v = davg[pl] / (float)HW;
    if (amax[pl] == i) v += dmx[pl];
    dx[(long)n * dx_bs + (long)c * HW + i] += v;
  }
}

// ---------------------------------------------------------------------------------------
// Elementwise helpers
// ---------------------------------------------------------------------------------------
struct PtrList { const float* p[8]; long bs[8]; };

// out[n, e] = sum_i in_i[n, e]   (per-sample extent E, batch strides per operand)
__global__ void add_n_kernel(PtrList in, int nin, float* out, long out_bs, int N, long E) {
  const long total = (long)N * E;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int n = t / E; const long e = t - (long)n * E;
    float s = in.p[0][(long)n * in.bs[0] + e];
    for (int i = 1; i < nin; ++i) s += in.p[i][(long)n * in.bs[i] + e];
    out[(long)n * out_bs + e] = s;
  }
}

__global__ void copy_strided_kernel(const float* src, long src_bs, float* dst, long dst_bs, int N, long E) {
  const long total = (long)N * E;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int n = t / E; const long e = t - (long)n * E;
    dst[(long)n * dst_bs + e] = src[(long)n * src_bs + e];
  }
}

// float4 forms (E, batch strides multiples of 4, 16-byte aligned): blockIdx.y is the sample, so
// no 64-bit division per element (the scalar forms above spend more time in it than in memory).
__global__ __launch_bounds__(256) void add_n4_kernel(PtrList in, int nin, float* out, long out_bs, long E4) {
  const int n = blockIdx.y;
  float4* o = reinterpret_cast<float4*>(out + (long)n * out_bs);
  for (long e = blockIdx.x * 256L + threadIdx.x; e < E4; e += (long)gridDim.x * 256) {
    float4 s = reinterpret_cast<const float4*>(in.p[0] + (long)n * in.bs[0])[e];
    for (int i = 1; i < nin; ++i) {
      const float4 v = reinterpret_cast<const float4*>(in.p[i] + (long)n * in.bs[i])[e];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    o[e] = s;
  }
}

__global__ __launch_bounds__(256) void copy4_kernel(const float* src, long src_bs, float* dst, long dst_bs, long E4) {
  const int n = blockIdx.y;
  const float4* s = reinterpret_cast<const float4*>(src + (long)n * src_bs);
  float4* d = reinterpret_cast<float4*>(dst + (long)n * dst_bs);
  for (long e = blockIdx.x * 256L + threadIdx.x; e < E4; e += (long)gridDim.x * 256) d[e] = s[e];
}

// Up to COPY_MULTI (src, dst) pairs of E floats in one launch (blockIdx.y = pair): the ImagePool's
// per-query gather / scatter (util/image_pool.py) instead of one copy launch per image.
constexpr int COPY_MULTI = 32;
struct CopyPairs {
  const float* src[COPY_MULTI];
  float* dst[COPY_MULTI];
};
__global__ __launch_bounds__(256) void copy_multi4_kernel(CopyPairs pr, long E4) {
  const float4* s = reinterpret_cast<const float4*>(pr.src[blockIdx.y]);
  float4* d = reinterpret_cast<float4*>(pr.dst[blockIdx.y]);
  for (long e = blockIdx.x * 256L + threadIdx.x; e < E4; e += (long)gridDim.x * 256) d[e] = s[e];
}
__global__ __launch_bounds__(256) void copy_multi_kernel(CopyPairs pr, long E) {
  const float* s = pr.src[blockIdx.y];
  float* d = pr.dst[blockIdx.y];
  for (long e = blockIdx.x * 256L + threadIdx.x; e < E; e += (long)gridDim.x * 256) d[e] = s[e];
}

static inline bool v4_ok(const void* p, long bs) { return (bs & 3) == 0 && (((uintptr_t)p) & 15) == 0; }
static inline dim3 grid4(int N, long E4) {
  long gx = (E4 + 255) / 256;
  if (gx > 4096) gx = 4096;
  return dim3((unsigned)(gx < 1 ? 1 : gx), (unsigned)N);
}

// Input pipeline (DSGAN/data/aligned_dataset.py:38-86): uint8 HWC crops -> ToTensor (/255) ->
// Normalize(0.5, 0.5) -> horizontal flip (per-sample flag) -> optional RGB->gray
// (0.299/0.587/0.114, evaluated in the reference's order without FMA contraction), NCHW fp32.
// One thread per output pixel, all channels; bit-exact with the torchvision/torch CPU ops.
__global__ void u8_to_image_kernel(const unsigned char* __restrict__ src, const int* __restrict__ flip,
                                   float* __restrict__ dst, int N, int H, int W, int gray) {
#pragma clang fp contract(off)   // hipcc contracts mul+add into FMA by default; torch CPU does not
  const long total = (long)N * H * W;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int n = (int)(t / ((long)H * W));
    const int r = (int)(t - (long)n * H * W), h = r / W, w = r - h * W;
    const int ws = flip[n] ? W - 1 - w : w;
    const unsigned char* px = src + (((long)n * H + h) * W + ws) * 3;
    float c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = ((float)px[k] / 255.f - 0.5f) / 0.5f;
    if (gray) {
      dst[(long)n * H * W + r] = (c[0] * 0.299f + c[1] * 0.587f) + c[2] * 0.114f;
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) dst[((long)n * 3 + k) * H * W + r] = c[k];
    }
  }
}

__global__ void scale_kernel(float* p, float a, long n) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) p[t] *= a;
}

__global__ void fill_kernel(float* p, float v, long n) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) p[t] = v;
}

// dx = dy * act'(pre)  (+ dx if accumulate)
__global__ void act_bwd_kernel(const float* dy, const float* pre, float* dx, long n, int act, float slope, int accumulate) {
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < n; t += (long)gridDim.x * blockDim.x) {
    float v = dy[t] * act_g(act, pre[t], slope);
    dx[t] = accumulate ? dx[t] + v : v;
  }
}

// part[n*C + c] = sum_p dy[n,c,p]   (bias gradient, one plane per NT threads; the sum over n is
// launch_split_reduce's fixed-order pass -- deterministic)
template <int NT>
__global__ __launch_bounds__(256) void channel_sum_kernel(const float* dy, long dy_bs, float* out, int N, int C, int HW) {
  __shared__ float sh[4];
  const int plane = blockIdx.x * (256 / NT) + (NT == 64 ? (threadIdx.x >> 6) : 0);
  const int t = NT == 64 ? (threadIdx.x & 63) : threadIdx.x;
  if (plane >= N * C) return;
  const int n = plane / C, c = plane - n * C;
  const float* p = dy + (long)n * dy_bs + (long)c * HW;
  float s = 0.f;
  if ((HW & 3) == 0 && (((uintptr_t)p) & 15) == 0) {
    const float4* p4 = reinterpret_cast<const float4*>(p);
    const int n4 = HW / 4;
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int i = t;
    for (; i + 3 * NT < n4; i += 4 * NT) {   // four independent 16-byte loads in flight
      const float4 v0 = p4[i], v1 = p4[i + NT], v2 = p4[i + 2 * NT], v3 = p4[i + 3 * NT];
      s += (v0.x + v0.y) + (v0.z + v0.w);
      s1 += (v1.x + v1.y) + (v1.z + v1.w);
      s2 += (v2.x + v2.y) + (v2.z + v2.w);
      s3 += (v3.x + v3.y) + (v3.z + v3.w);
    }
    for (; i < n4; i += NT) { const float4 v = p4[i]; s += (v.x + v.y) + (v.z + v.w); }
    s = (s + s1) + (s2 + s3);
  } else {
    for (int i = t; i < HW; i += NT) s += p[i];
  }
  s = NT == 64 ? warp_sum(s) : block_sum<NT>(s, sh);
  if (t == 0) out[plane] = s;
}

static inline unsigned grid_for(long n, int bs = 256) {
  long g = (n + bs - 1) / bs;
  if (g > 65535L * 8) g = 65535L * 8;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// the cached IN backward forms instantiated per activation (ACTT, see instnorm_bwd_v4)
template <int NT, int C4, bool CX, int XL = 0>
static void in_bwd_launch(const INBwdArgs& a, dim3 grid, dim3 block, hipStream_t st) {
  switch (a.act) {
    case ACT_NONE: hipLaunchKernelGGL((instnorm_bwd_v4<NT, C4, CX, XL, ACT_NONE>), grid, block, 0, st, a); break;
    case ACT_GELU: hipLaunchKernelGGL((instnorm_bwd_v4<NT, C4, CX, XL, ACT_GELU>), grid, block, 0, st, a); break;
    case ACT_LRELU: hipLaunchKernelGGL((instnorm_bwd_v4<NT, C4, CX, XL, ACT_LRELU>), grid, block, 0, st, a); break;
    case ACT_GELU_FAST:
      hipLaunchKernelGGL((instnorm_bwd_v4<NT, C4, CX, XL, ACT_GELU_FAST>), grid, block, 0, st, a);
      break;
    default: hipLaunchKernelGGL((instnorm_bwd_v4<NT, C4, CX, XL>), grid, block, 0, st, a); break;
  }
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// float4 InstanceNorm kernels (16-byte aligned planes); planes up to 64K pixels are cached in
// registers between the statistics and the normalise pass (measured 1.45x faster fwd and bwd
// than streaming them twice).  Unaligned planes take the scalar kernels.
static inline bool in_v4_ok(int HW, const void* p, long bs) {
  return (HW & 3) == 0 && (bs & 3) == 0 && (((uintptr_t)p) & 15) == 0;
}

int dsgan_instnorm_fwd(const float* x, long x_bs, const float* scale, const float* res, long res_bs,
                       float* y, long y_bs, float* mean, float* rstd, int N, int C, int HW, int act,
                       float slope, float eps, hipStream_t st) {
  DSG_REQUIRE(x && y && mean && rstd && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_fwd: bad args");
  INArgs a{x, x_bs, scale, res, res_bs, y, y_bs, mean, rstd, N, C, HW, act, slope, eps, 0};
  const int planes = N * C;
  const int v4 = in_v4_ok(HW, x, x_bs) && in_v4_ok(HW, y, y_bs) && (!res || in_v4_ok(HW, res, res_bs));
  if (v4) {
    if (HW <= 64 * 16)
      hipLaunchKernelGGL((instnorm_fwd_v4<64, 4>), dim3(cdiv(planes, 4)), dim3(256), 0, st, a);
    else if (HW <= 256 * 16)
      hipLaunchKernelGGL((instnorm_fwd_v4<256, 4>), dim3(planes), dim3(256), 0, st, a);
    else if (HW <= 256 * 64)
      hipLaunchKernelGGL((instnorm_fwd_v4<256, 16>), dim3(planes), dim3(256), 0, st, a);
    else if (HW <= 1024 * 64)
      hipLaunchKernelGGL((instnorm_fwd_v4<1024, 16>), dim3(planes), dim3(1024), 0, st, a);
    else
      hipLaunchKernelGGL((instnorm_fwd_v4<1024, 0>), dim3(planes), dim3(1024), 0, st, a);
    DSG_CHECK_LAUNCH();
    return 0;
  }
  if (HW <= 64 * 16)
    hipLaunchKernelGGL((instnorm_fwd_kernel<64, 16>), dim3(cdiv(planes, 4)), dim3(256), 0, st, a);
  else if (HW <= 256 * 16)
    hipLaunchKernelGGL((instnorm_fwd_kernel<256, 16>), dim3(planes), dim3(256), 0, st, a);
  else if (HW <= 1024 * 16)
    hipLaunchKernelGGL((instnorm_fwd_kernel<1024, 16>), dim3(planes), dim3(1024), 0, st, a);
  else
    hipLaunchKernelGGL((instnorm_fwd_kernel<1024, 0>), dim3(planes), dim3(1024), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

// Scratch (fp32 elements) of dsgan_instnorm_{fwd,bwd}_ws for this shape: 0 when the one-workgroup-
// per-plane kernels serve it (>= 128 planes or planes under 16K pixels), else the per-chunk partials
// of the split forms.
long dsgan_instnorm_workspace(int N, int C, int HW) {
  const int S = in_split_chunks((long)N * C, HW);
  return S ? 2L * N * C * S : 0;
}

// dsgan_instnorm_fwd with scratch: few large planes are split over several workgroups each.
int dsgan_instnorm_fwd_ws(const float* x, long x_bs, const float* scale, const float* res, long res_bs,
                          float* y, long y_bs, float* mean, float* rstd, int N, int C, int HW, int act,
                          float slope, float eps, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(x && y && mean && rstd && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_fwd_ws: bad args");
  const long planes = (long)N * C;
  const int v4 = in_v4_ok(HW, x, x_bs) && in_v4_ok(HW, y, y_bs) && (!res || in_v4_ok(HW, res, res_bs));
  const int S = v4 ? in_split_chunks(planes, HW) : 0;
  DSG_WS(S ? 2 * planes * S : 0, ws, ws_elems, "dsgan_instnorm_fwd_ws");
  if (!S) return dsgan_instnorm_fwd(x, x_bs, scale, res, res_bs, y, y_bs, mean, rstd, N, C, HW, act, slope, eps, st);
  INArgs a{x, x_bs, scale, res, res_bs, y, y_bs, mean, rstd, N, C, HW, act, slope, eps, 0};
  const dim3 g(S, (unsigned)planes);
  hipLaunchKernelGGL(in_split_stat<0>, g, dim3(256), 0, st, a, ws, S);
  hipLaunchKernelGGL(in_split_stat<1>, g, dim3(256), 0, st, a, ws, S);
  hipLaunchKernelGGL(in_split_out, g, dim3(256), 0, st, a, ws, S);
  DSG_CHECK_LAUNCH();
  return 0;
}

// y (bf16) = IN(x): the plain InstanceNorm2d(affine=False) of a ConvNeXt block
// (DSGAN/models/model/MixConvNeXtML.py:233), stored bf16 for the block's MLP GEMMs.
int dsgan_instnorm_fwd_bf16(const float* x, long x_bs, void* y, long y_bs, float* mean, float* rstd, int N, int C,
                            int HW, float eps, hipStream_t st) {
  DSG_REQUIRE(x && y && mean && rstd && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_fwd_bf16: bad args");
  DSG_REQUIRE(in_v4_ok(HW, x, x_bs) && in_v4_ok(HW, y, y_bs), "dsgan_instnorm_fwd_bf16: HW %% 4 and 16-byte alignment");
  // (y has the library's half type: y_bf16 = 1 bf16, 2 fp16)
  INArgs a{x, x_bs, nullptr, nullptr, 0, (float*)y, y_bs, mean, rstd, N, C, HW, ACT_NONE, 0.f, eps,
           half_type() == HALF_F16 ? 2 : 1};
  const int planes = N * C;
  if (HW <= 64 * 16)
    hipLaunchKernelGGL((instnorm_fwd_v4<64, 4>), dim3(cdiv(planes, 4)), dim3(256), 0, st, a);
  else if (HW <= 256 * 16)
    hipLaunchKernelGGL((instnorm_fwd_v4<256, 4>), dim3(planes), dim3(256), 0, st, a);
  else if (HW <= 256 * 64)
    hipLaunchKernelGGL((instnorm_fwd_v4<256, 16>), dim3(planes), dim3(256), 0, st, a);
  else if (HW <= 1024 * 64)
    hipLaunchKernelGGL((instnorm_fwd_v4<1024, 16>), dim3(planes), dim3(1024), 0, st, a);
  else
    hipLaunchKernelGGL((instnorm_fwd_v4<1024, 0>), dim3(planes), dim3(1024), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

// Backward with dx stored in the library's 16-bit half type (dxh, batch stride dxh_bs elements)
// plus the per-plane sums of the fp32 dx (dxsum [N*C]; nullable) -- the ConvTranspose backward's
// operand (its data-/weight-grad kernels read it as 16-bit MFMA operands) and its bias grad.
int dsgan_instnorm_bwd_h(const float* dy, long dy_bs, const float* x, long x_bs, const float* res, long res_bs,
                         const float* mean, const float* rstd, void* dxh, long dxh_bs, float* dxsum, float* dres,
                         long dres_bs, int N, int C, int HW, int act, float slope, float eps, hipStream_t st) {
  DSG_REQUIRE(dy && x && mean && rstd && dxh && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_bwd_h: bad args");
  DSG_REQUIRE(in_v4_ok(HW, dy, dy_bs) && in_v4_ok(HW, x, x_bs) && (!res || in_v4_ok(HW, res, res_bs)) &&
                  (!dres || in_v4_ok(HW, dres, dres_bs)) && ((uintptr_t)dxh & 7) == 0 && dxh_bs % 4 == 0,
              "dsgan_instnorm_bwd_h: planes must be float4-aligned (HW %% 4 == 0) and dxh 8-byte aligned");
  INBwdArgs a{dy, dy_bs, x, x_bs, nullptr, res, res_bs, mean, rstd, nullptr, dxh_bs, dres, dres_bs, nullptr,
              N, C, HW, act, slope, eps, dxh, dxsum, half_type()};
  const int planes = N * C;
  if (HW <= 64 * 16)
    in_bwd_launch<64, 4, true>(a, dim3(cdiv(planes, 4)), dim3(256), st);
  else if (HW <= 256 * 16)
    in_bwd_launch<256, 4, true>(a, dim3(planes), dim3(256), st);
  else if (HW <= 256 * 64)
    in_bwd_launch<256, 16, true>(a, dim3(planes), dim3(256), st);
  else if (HW <= 1024 * 64)
    in_bwd_launch<1024, 16, false, IN_BWD_XL>(a, dim3(planes), dim3(1024), st);
  else
    hipLaunchKernelGGL((instnorm_bwd_v4<1024, 0, false>), dim3(planes), dim3(1024), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_instnorm_bwd(const float* dy, long dy_bs, const float* x, long x_bs, const float* scale,
                       const float* res, long res_bs, const float* mean, const float* rstd,
                       float* dx, long dx_bs, float* dres, long dres_bs, float* dscale, int N,
                       int C, int HW, int act, float slope, float eps, hipStream_t st) {
  DSG_REQUIRE(dy && x && mean && rstd && dx && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_bwd: bad args");
  INBwdArgs a{dy, dy_bs, x, x_bs, scale, res, res_bs, mean, rstd, dx, dx_bs, dres, dres_bs, dscale,
              N, C, HW, act, slope, eps};
  const int planes = N * C;
  const int v4 = in_v4_ok(HW, dy, dy_bs) && in_v4_ok(HW, x, x_bs) && in_v4_ok(HW, dx, dx_bs) &&
                 (!res || in_v4_ok(HW, res, res_bs)) && (!dres || in_v4_ok(HW, dres, dres_bs));
  if (v4) {
    if (HW <= 64 * 16)
      in_bwd_launch<64, 4, true>(a, dim3(cdiv(planes, 4)), dim3(256), st);
    else if (HW <= 256 * 16)
      in_bwd_launch<256, 4, true>(a, dim3(planes), dim3(256), st);
    else if (HW <= 256 * 64)
      in_bwd_launch<256, 16, true>(a, dim3(planes), dim3(256), st);
    else if (HW <= 1024 * 64)
      in_bwd_launch<1024, 16, false, IN_BWD_XL>(a, dim3(planes), dim3(1024), st);
    else
      hipLaunchKernelGGL((instnorm_bwd_v4<1024, 0, false>), dim3(planes), dim3(1024), 0, st, a);
    DSG_CHECK_LAUNCH();
    return 0;
  }
  if (HW <= 64 * 16)
    hipLaunchKernelGGL((instnorm_bwd_kernel<64, 16>), dim3(cdiv(planes, 4)), dim3(256), 0, st, a);
  else if (HW <= 256 * 16)
    hipLaunchKernelGGL((instnorm_bwd_kernel<256, 16>), dim3(planes), dim3(256), 0, st, a);
  else if (HW <= 1024 * 16)
    hipLaunchKernelGGL((instnorm_bwd_kernel<1024, 16>), dim3(planes), dim3(1024), 0, st, a);
  else
    hipLaunchKernelGGL((instnorm_bwd_kernel<1024, 0>), dim3(planes), dim3(1024), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dsgan_instnorm_bwd with scratch (dsgan_instnorm_workspace): few large planes split as in the forward.
int dsgan_instnorm_bwd_ws(const float* dy, long dy_bs, const float* x, long x_bs, const float* scale,
                          const float* res, long res_bs, const float* mean, const float* rstd,
                          float* dx, long dx_bs, float* dres, long dres_bs, float* dscale, int N,
                          int C, int HW, int act, float slope, float eps, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(dy && x && mean && rstd && dx && N > 0 && C > 0 && HW > 0, "dsgan_instnorm_bwd_ws: bad args");
  const long planes = (long)N * C;
  const int v4 = in_v4_ok(HW, dy, dy_bs) && in_v4_ok(HW, x, x_bs) && in_v4_ok(HW, dx, dx_bs) &&
                 (!res || in_v4_ok(HW, res, res_bs)) && (!dres || in_v4_ok(HW, dres, dres_bs));
  const int S = v4 ? in_split_chunks(planes, HW) : 0;
  DSG_WS(S ? 2 * planes * S : 0, ws, ws_elems, "dsgan_instnorm_bwd_ws");
  if (!S)
    return dsgan_instnorm_bwd(dy, dy_bs, x, x_bs, scale, res, res_bs, mean, rstd, dx, dx_bs, dres, dres_bs, dscale,
                              N, C, HW, act, slope, eps, st);
  INBwdArgs a{dy, dy_bs, x, x_bs, scale, res, res_bs, mean, rstd, dx, dx_bs, dres, dres_bs, dscale,
              N, C, HW, act, slope, eps};
  const dim3 g(S, (unsigned)planes);
  hipLaunchKernelGGL(in_split_bwd<0>, g, dim3(256), 0, st, a, ws, S);
  hipLaunchKernelGGL(in_split_bwd<1>, g, dim3(256), 0, st, a, ws, S);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_maxpool_fwd(const float* x, long x_bs, float* y, long y_bs, int* idx, int N, int C, int H,
                      int W, int k, hipStream_t st) {
  DSG_REQUIRE(x && y && idx && k > 0 && H >= k && W >= k, "dsgan_maxpool_fwd: bad args");
  const dim3 grid = plane_grid((long)(H / k) * (W / k), (long)N * C);
  const bool fast = (H % k == 0) && (W % k == 0) && (k == 2 ? ((W & 1) == 0 && (x_bs & 1) == 0 && ((uintptr_t)x & 7) == 0)
                                                            : ((W & 3) == 0 && (x_bs & 3) == 0 && ((uintptr_t)x & 15) == 0));
  const bool x2 = fast && k == 2 && (W & 3) == 0 && (x_bs & 3) == 0 && ((uintptr_t)x & 15) == 0 &&
                  (y_bs & 1) == 0 && (((uintptr_t)y | (uintptr_t)idx) & 7) == 0;
  if (x2) hipLaunchKernelGGL(maxpool2_fwd_x2_kernel, plane_grid((long)(H / 2) * (W / 4), (long)N * C), dim3(256), 0, st,
                             x, x_bs, y, y_bs, idx, N, C, H, W);
  else if (fast && k == 2) hipLaunchKernelGGL(maxpool_fwd_win_kernel<2>, grid, dim3(256), 0, st, x, x_bs, y, y_bs, idx, N, C, H, W);
  else if (fast && k == 4) hipLaunchKernelGGL(maxpool_fwd_win_kernel<4>, grid, dim3(256), 0, st, x, x_bs, y, y_bs, idx, N, C, H, W);
  else if (fast && k == 8) hipLaunchKernelGGL(maxpool_fwd_win_kernel<8>, grid, dim3(256), 0, st, x, x_bs, y, y_bs, idx, N, C, H, W);
  else if (fast && k == 16) hipLaunchKernelGGL(maxpool_fwd_win_kernel<16>, grid, dim3(256), 0, st, x, x_bs, y, y_bs, idx, N, C, H, W);
  else hipLaunchKernelGGL(maxpool_fwd_kernel, grid, dim3(256), 0, st, x, x_bs, y, y_bs, idx, N, C, H, W, k);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_maxpool_bwd(const float* dy, long dy_bs, const int* idx, float* dx, long dx_bs, int N,
                      int C, int H, int W, int k, int accumulate, hipStream_t st) {
  DSG_REQUIRE(dy && idx && dx && k > 0, "dsgan_maxpool_bwd: bad args");
  const bool fast = (H % k == 0) && (W % k == 0) && (k == 2 ? ((W & 1) == 0 && (dx_bs & 1) == 0 && ((uintptr_t)dx & 7) == 0)
                                                            : ((W & 3) == 0 && (dx_bs & 3) == 0 && ((uintptr_t)dx & 15) == 0));
  const dim3 wgrid = plane_grid((long)(H / k) * (W / k), (long)N * C);
  const bool x2 = fast && k == 2 && (W & 3) == 0 && (dx_bs & 3) == 0 && ((uintptr_t)dx & 15) == 0 &&
                  (dy_bs & 1) == 0 && (((uintptr_t)dy | (uintptr_t)idx) & 7) == 0;
  if (x2) hipLaunchKernelGGL(maxpool2_bwd_x2_kernel, plane_grid((long)(H / 2) * (W / 4), (long)N * C), dim3(256), 0, st,
                             dy, dy_bs, idx, dx, dx_bs, N, C, H, W, accumulate);
  else if (fast && k == 2) hipLaunchKernelGGL(maxpool_bwd_win_kernel<2>, wgrid, dim3(256), 0, st, dy, dy_bs, idx, dx, dx_bs, N, C, H, W, accumulate);
  else if (fast && k == 4) hipLaunchKernelGGL(maxpool_bwd_win_kernel<4>, wgrid, dim3(256), 0, st, dy, dy_bs, idx, dx, dx_bs, N, C, H, W, accumulate);
  else if (fast && k == 8) hipLaunchKernelGGL(maxpool_bwd_row_kernel<8>, plane_grid((long)H * W / 4, (long)N * C), dim3(256), 0, st, dy, dy_bs, idx, dx, dx_bs, N, C, H, W, accumulate);
  else if (fast && k == 16) hipLaunchKernelGGL(maxpool_bwd_row_kernel<16>, plane_grid((long)H * W / 4, (long)N * C), dim3(256), 0, st, dy, dy_bs, idx, dx, dx_bs, N, C, H, W, accumulate);
  else hipLaunchKernelGGL(maxpool_bwd_kernel, plane_grid((long)H * W, (long)N * C), dim3(256), 0, st, dy, dy_bs,
                          idx, dx, dx_bs, N, C, H, W, k, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_maxpool_pyr_supported(int H, int W, int levels) {
  return levels >= 1 && levels <= 4 && H >= 16 && W >= 64 && H % 16 == 0 && W % 64 == 0;
}

int dsgan_maxpool_pyr_fwd(const float* x, long x_bs, int levels, float* y2, int* i2, float* y4, int* i4, float* y8, int* i8,
                          float* y16, int* i16, int N, int C, int H, int W, hipStream_t st) {
  DSG_REQUIRE(x && y2 && i2 && N > 0 && C > 0 && dsgan_maxpool_pyr_supported(H, W, levels),
              "dsgan_maxpool_pyr_fwd: bad args (levels %d, %dx%d: H %% 16, W %% 64)", levels, H, W);
  DSG_REQUIRE((levels < 2 || (y4 && i4)) && (levels < 3 || (y8 && i8)) && (levels < 4 || (y16 && i16)),
              "dsgan_maxpool_pyr_fwd: an output of a requested level is NULL");
  DSG_REQUIRE((x_bs & 3) == 0 && ((uintptr_t)x & 15) == 0 && (((uintptr_t)y2 | (uintptr_t)i2) & 7) == 0,
              "dsgan_maxpool_pyr_fwd: x rows must be 16-byte aligned, k=2 outputs 8-byte aligned");
  PyrPtrs p{};
  p.y[0] = y2; p.y[1] = y4; p.y[2] = y8; p.y[3] = y16;
  p.idx[0] = i2; p.idx[1] = i4; p.idx[2] = i8; p.idx[3] = i16;
  const long nw = (long)N * C * (H / 16) * (W / 64);
  const dim3 grid((unsigned)((nw + 3) / 4));
  switch (levels) {
    case 1: hipLaunchKernelGGL(maxpool_pyr_fwd_kernel<1>, grid, dim3(256), 0, st, x, x_bs, p, C, H, W, nw); break;
    case 2: hipLaunchKernelGGL(maxpool_pyr_fwd_kernel<2>, grid, dim3(256), 0, st, x, x_bs, p, C, H, W, nw); break;
    case 3: hipLaunchKernelGGL(maxpool_pyr_fwd_kernel<3>, grid, dim3(256), 0, st, x, x_bs, p, C, H, W, nw); break;
    default: hipLaunchKernelGGL(maxpool_pyr_fwd_kernel<4>, grid, dim3(256), 0, st, x, x_bs, p, C, H, W, nw); break;
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_maxpool_pyr_bwd(const float* dy2, long dy2_bs, const int* i2, const float* dy4, long dy4_bs, const int* i4,
                          const float* dy8, long dy8_bs, const int* i8, const float* dy16, long dy16_bs, const int* i16,
                          float* dx, long dx_bs, int levels, int N, int C, int H, int W, int accumulate, hipStream_t st) {
  DSG_REQUIRE(dx && N > 0 && C > 0 && dsgan_maxpool_pyr_supported(H, W, levels), "dsgan_maxpool_pyr_bwd: bad args");
  DSG_REQUIRE((!dy2 || i2) && (!dy4 || i4) && (!dy8 || i8) && (!dy16 || i16),
              "dsgan_maxpool_pyr_bwd: a level with a gradient needs its indices");
  DSG_REQUIRE((dx_bs & 3) == 0 && ((uintptr_t)dx & 15) == 0 && (!dy2 || ((dy2_bs & 1) == 0 && (((uintptr_t)dy2 | (uintptr_t)i2) & 7) == 0)),
              "dsgan_maxpool_pyr_bwd: dx rows must be 16-byte aligned, k=2 grads 8-byte aligned");
  PyrPtrs p{};
  const float* dys[4] = {dy2, dy4, dy8, dy16};
  const long bss[4] = {dy2_bs, dy4_bs, dy8_bs, dy16_bs};
  const int* ids[4] = {i2, i4, i8, i16};
  for (int l = 0; l < 4; ++l) {
    p.dy[l] = l < levels ? dys[l] : nullptr;
    p.dy_bs[l] = bss[l];
    p.idx[l] = const_cast<int*>(ids[l]);
  }
  const long nw = (long)N * C * (H / 16) * (W / 64);
  const dim3 grid((unsigned)((nw + 3) / 4));
  switch (levels) {
    case 1: hipLaunchKernelGGL(maxpool_pyr_bwd_kernel<1>, grid, dim3(256), 0, st, p, dx, dx_bs, C, H, W, nw, accumulate); break;
    case 2: hipLaunchKernelGGL(maxpool_pyr_bwd_kernel<2>, grid, dim3(256), 0, st, p, dx, dx_bs, C, H, W, nw, accumulate); break;
    case 3: hipLaunchKernelGGL(maxpool_pyr_bwd_kernel<3>, grid, dim3(256), 0, st, p, dx, dx_bs, C, H, W, nw, accumulate); break;
    default: hipLaunchKernelGGL(maxpool_pyr_bwd_kernel<4>, grid, dim3(256), 0, st, p, dx, dx_bs, C, H, W, nw, accumulate); break;
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_plane_stats(const float* x, long x_bs, float* avg, float* mx, int* amax, int N, int C,
                      int HW, hipStream_t st) {
  DSG_REQUIRE(x && avg && mx && amax && HW > 0, "dsgan_plane_stats: bad args");
  const int planes = N * C;
  const bool v4 = (HW & 3) == 0 && (x_bs & 3) == 0 && (((uintptr_t)x) & 15) == 0;
  if (v4 && HW <= 4096)
    hipLaunchKernelGGL(plane_stats4_kernel<64>, dim3(cdiv(planes, 4)), dim3(256), 0, st, x, x_bs, avg, mx, amax, N, C, HW);
  else if (v4)
    hipLaunchKernelGGL(plane_stats4_kernel<256>, dim3(planes), dim3(256), 0, st, x, x_bs, avg, mx, amax, N, C, HW);
  else if (HW <= 4096)
    hipLaunchKernelGGL(plane_stats_kernel<64>, dim3(cdiv(planes, 4)), dim3(256), 0, st, x, x_bs, avg, mx, amax, N, C, HW);
  else
    hipLaunchKernelGGL(plane_stats_kernel<256>, dim3(planes), dim3(256), 0, st, x, x_bs, avg, mx, amax, N, C, HW);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_plane_stats_bwd(const float* davg, const float* dmx, const int* amax, float* dx,
                          long dx_bs, int N, int C, int HW, hipStream_t st) {
  const long total = (long)N * C * HW;
  if ((HW & 3) == 0 && (dx_bs & 3) == 0 && (((uintptr_t)dx) & 15) == 0)
    hipLaunchKernelGGL(plane_stats_bwd4_kernel, dim3(grid_for(total / 4)), dim3(256), 0, st, davg, dmx, amax, dx, dx_bs,
                       N, C, HW);
  else
    hipLaunchKernelGGL(plane_stats_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, st, davg, dmx,
                       amax, dx, dx_bs, N, C, HW);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_ca_fwd(const float* avg, const float* mx, const float* w1, const float* w2,
                 const float* prelu_a, float* att, float* hsave, int N, int C, int R,
                 hipStream_t st) {
  DSG_REQUIRE(C > 0 && R > 0 && C <= 4096, "dsgan_ca_fwd: bad dims");
  const size_t shm = (2 * C + R) * sizeof(float);
  hipLaunchKernelGGL(ca_fwd_kernel, dim3(N), dim3(256), shm, st, avg, mx, w1, w2, prelu_a, att, hsave, C, R);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_ca_bwd(const float* datt, const float* att, const float* avg, const float* mx,
                 const float* hsave, const float* w1, const float* w2, const float* prelu_a,
                 float* davg, float* dmx, float* dw1, float* dw2, float* dprelu_a, int N, int C,
                 int R, float* ws, long ws_elems, hipStream_t st) {
  DSG_REQUIRE(N > 0 && C > 0 && R > 0 && C <= 4096, "dsgan_ca_bwd: bad dims");
  DSG_WS((long)N * (2L * R * C + 1), ws, ws_elems, "dsgan_ca_bwd (N*(2*R*C+1) floats)");
  const size_t shm = (C + 3 * R) * sizeof(float);
  hipLaunchKernelGGL(ca_bwd_kernel, dim3(N), dim3(256), shm, st, datt, att, avg, mx, hsave, w1, w2,
                     prelu_a, davg, dmx, ws, dw1 != nullptr, dw2 != nullptr, dprelu_a != nullptr, C, R);
  {   // the three parameter-grad reductions in one launch
    const float* wsv[3];
    int sv[3];
    long mv[3];
    float* dv[3];
    int n = 0;
    if (dw1) { wsv[n] = ws; sv[n] = N; mv[n] = (long)R * C; dv[n] = dw1; ++n; }
    if (dw2) { wsv[n] = ws + (long)N * R * C; sv[n] = N; mv[n] = (long)C * R; dv[n] = dw2; ++n; }
    if (dprelu_a) { wsv[n] = ws + 2L * N * R * C; sv[n] = N; mv[n] = 1; dv[n] = dprelu_a; ++n; }
    if (n) launch_split_reduce_multi(n, wsv, sv, mv, dv, st);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_add_n(const float* const* ins, const long* in_bs, int nin, float* out, long out_bs, int N,
                long E, hipStream_t st) {
  DSG_REQUIRE(nin >= 1 && nin <= 8 && ins && out, "dsgan_add_n: 1..8 inputs");
  PtrList pl{};
  bool v4 = (E & 3) == 0 && v4_ok(out, out_bs) && N <= 65535;
  for (int i = 0; i < nin; ++i) { pl.p[i] = ins[i]; pl.bs[i] = in_bs[i]; v4 = v4 && v4_ok(ins[i], in_bs[i]); }
  if (v4) {
    hipLaunchKernelGGL(add_n4_kernel, grid4(N, E / 4), dim3(256), 0, st, pl, nin, out, out_bs, E / 4);
    DSG_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(add_n_kernel, dim3(grid_for((long)N * E)), dim3(256), 0, st, pl, nin, out, out_bs, N, E);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_copy_strided(const float* src, long src_bs, float* dst, long dst_bs, int N, long E,
                       hipStream_t st) {
  if ((E & 3) == 0 && v4_ok(src, src_bs) && v4_ok(dst, dst_bs) && N <= 65535) {
    hipLaunchKernelGGL(copy4_kernel, grid4(N, E / 4), dim3(256), 0, st, src, src_bs, dst, dst_bs, E / 4);
    DSG_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(copy_strided_kernel, dim3(grid_for((long)N * E)), dim3(256), 0, st, src, src_bs, dst, dst_bs, N, E);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dst[i][0..E) <- src[i][0..E) for i < count (host arrays of device pointers); pairs must not
// overlap each other (the ImagePool orders its gather and scatter as two calls)
int dsgan_copy_multi(const float* const* src, float* const* dst, int count, long E, hipStream_t st) {
  DSG_REQUIRE(src && dst && count >= 0 && E >= 0, "dsgan_copy_multi: bad args");
  for (int b = 0; b < count; b += COPY_MULTI) {
    const int n = count - b < COPY_MULTI ? count - b : COPY_MULTI;
    CopyPairs pr{};
    bool v4 = (E & 3) == 0;
    for (int i = 0; i < n; ++i) {
      DSG_REQUIRE(src[b + i] && dst[b + i], "dsgan_copy_multi: null pointer in pair %d", b + i);
      pr.src[i] = src[b + i];
      pr.dst[i] = dst[b + i];
      v4 = v4 && v4_ok(src[b + i], 0) && v4_ok(dst[b + i], 0);
    }
    if (v4) hipLaunchKernelGGL(copy_multi4_kernel, grid4(n, E / 4), dim3(256), 0, st, pr, E / 4);
    else hipLaunchKernelGGL(copy_multi_kernel, grid4(n, E), dim3(256), 0, st, pr, E);
    DSG_CHECK_LAUNCH();
  }
  return 0;
}

int dsgan_u8_to_image(const unsigned char* src, const int* flip, float* dst, int N, int H, int W, int gray,
                      hipStream_t st) {
  DSG_REQUIRE(src && flip && dst && N > 0 && H > 0 && W > 0, "dsgan_u8_to_image: bad args");
  hipLaunchKernelGGL(u8_to_image_kernel, dim3(grid_for((long)N * H * W)), dim3(256), 0, st, src, flip, dst, N, H, W,
                     gray);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_fill(float* p, float v, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, v, n);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_scale(float* p, float a, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, a, n);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_act_bwd(const float* dy, const float* pre, float* dx, long n, int act, float slope,
                  int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, st, dy, pre, dx, n, act, slope, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}

int dsgan_channel_sum(const float* dy, long dy_bs, float* out, int N, int C, int HW, float* ws, long ws_elems,
                      hipStream_t st) {
  DSG_REQUIRE(dy && out && N > 0 && C > 0 && HW > 0, "dsgan_channel_sum: bad args");
  DSG_WS((long)N * C, ws, ws_elems, "dsgan_channel_sum (N*C floats)");
  if (HW <= 8192)
    hipLaunchKernelGGL(channel_sum_kernel<64>, dim3(cdiv((long)N * C, 4)), dim3(256), 0, st, dy, dy_bs, ws, N, C, HW);
  else
    hipLaunchKernelGGL(channel_sum_kernel<256>, dim3(N * C), dim3(256), 0, st, dy, dy_bs, ws, N, C, HW);
  launch_split_reduce(ws, N, C, out, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
