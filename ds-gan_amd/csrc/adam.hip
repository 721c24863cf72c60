// Fused Adam over a flat parameter buffer (torch.optim.Adam semantics, amsgrad=False,
// weight_decay=0; used by DSGAN/models/pix2pix_model.py:122-125 with lr=2e-4, betas=(0.5,0.999)).
// Every generator (or discriminator) parameter is a view into one contiguous fp32 buffer, so
// one launch updates all 188 (or 10) tensors.  Arithmetic mirrors torch's single-tensor path:
//   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
#include "common.h"

namespace dsg {
// The optimizer's scalars as torch hands them to its fp32 kernels: python doubles, each rounded
// to fp32 once (lerp weight 1 - b1, addcmul value 1 - b2, addcdiv value lr / (1 - b1^t), the
// bias_correction2 sqrt divisor, eps).
struct AdamScal {
  float w1, b2, omb2, step_size, bc2s, eps;
};

static AdamScal adam_scal(double lr, double b1, double b2, double eps, double t) {
  AdamScal a;
  a.w1 = (float)(1.0 - b1);
  a.b2 = (float)b2;
  a.omb2 = (float)(1.0 - b2);
  a.step_size = (float)(lr / (1.0 - pow(b1, t)));
  a.bc2s = (float)sqrt(1.0 - pow(b2, t));
  a.eps = (float)eps;
  return a;
}

// One element (shared by the float4 body and the tail / unaligned body so both round identically):
//   m.lerp_(g, w1); v.mul_(b2).addcmul_(g, g, 1 - b2); p.addcdiv_(m, sqrt(v) / bc2s + eps, -step_size)
__device__ __forceinline__ void adam_elem(float& p, float gr, float& m, float& v, const AdamScal& a) {
  float mm = m;
  // at::lerp: weight < 0.5 ? a + w*(b-a) : b - (b-a)*(1-w)
  mm = a.w1 < 0.5f ? mm + a.w1 * (gr - mm) : gr - (gr - mm) * (1.f - a.w1);
  const float vv = v * a.b2 + a.omb2 * gr * gr;
  m = mm; v = vv;
  const float denom = sqrtf(vv) / a.bc2s + a.eps;
  p = p - a.step_size * (mm / denom);
}

// VEC: p, g, m, v 16-byte aligned -- each lane moves float4s, the n % 4 tail elements go to the
// first threads.  Otherwise one element per lane.
// AMP: g is scaled by st[3] (1 / loss scale), the step count is st[4] (the scalars are formed here
// from the doubles, as on the host for the plain form), and the whole update is skipped when
// st[1] != 0.
template <bool VEC, bool AMP>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long n, AdamScal a,
                                                   double lr, double b1, double b2, double eps,
                                                   const float* __restrict__ st) {
  float inv = 1.f;
  if constexpr (AMP) {
    if (st[1] != 0.f) return;   // overflowed step: parameters and moments untouched
    inv = st[3];
    const double t = (double)st[4];
    a.w1 = (float)(1.0 - b1);
    a.b2 = (float)b2;
    a.omb2 = (float)(1.0 - b2);
    a.step_size = (float)(lr / (1.0 - pow(b1, t)));
    a.bc2s = (float)sqrt(1.0 - pow(b2, t));
    a.eps = (float)eps;
  }
  const long tid = blockIdx.x * 256L + threadIdx.x, stride = (long)gridDim.x * 256;
  if constexpr (VEC) {
    const long n4 = n >> 2;
    for (long i = tid; i < n4; i += stride) {
      float4 pp = reinterpret_cast<const float4*>(p)[i];
      float4 gg = reinterpret_cast<const float4*>(g)[i];
      float4 mm = reinterpret_cast<const float4*>(m)[i];
      float4 vv = reinterpret_cast<const float4*>(v)[i];
      if constexpr (AMP) { gg.x *= inv; gg.y *= inv; gg.z *= inv; gg.w *= inv; }
      adam_elem(pp.x, gg.x, mm.x, vv.x, a);
      adam_elem(pp.y, gg.y, mm.y, vv.y, a);
      adam_elem(pp.z, gg.z, mm.z, vv.z, a);
      adam_elem(pp.w, gg.w, mm.w, vv.w, a);
      reinterpret_cast<float4*>(m)[i] = mm;
      reinterpret_cast<float4*>(v)[i] = vv;
      reinterpret_cast<float4*>(p)[i] = pp;
    }
    const long e = (n4 << 2) + tid;
    if (e < n) {
      float gr = g[e];
      if constexpr (AMP) gr *= inv;
      adam_elem(p[e], gr, m[e], v[e], a);
    }
  } else {
    for (long e = tid; e < n; e += stride) {
      float gr = g[e];
      if constexpr (AMP) gr *= inv;
      adam_elem(p[e], gr, m[e], v[e], a);
    }
  }
}

static bool adam_vec_ok(const float* p, const float* g, const float* m, const float* v) {
  return (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
}

template <bool AMP>
static void adam_launch(float* p, const float* g, float* m, float* v, long n, const AdamScal& a, double lr, double b1,
                        double b2, double eps, const float* state, hipStream_t st) {
  long blocks = (n + 1023) / 1024;
  if (blocks > 8192) blocks = 8192;
  if (adam_vec_ok(p, g, m, v))
    hipLaunchKernelGGL((adam_kernel<true, AMP>), dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, a, lr, b1,
                       b2, eps, state);
  else
    hipLaunchKernelGGL((adam_kernel<false, AMP>), dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, a, lr, b1,
                       b2, eps, state);
}
}  // namespace dsg

using namespace dsg;
extern "C" int dsgan_adam(float* p, const float* g, float* m, float* v, long n, double lr, double beta1,
                          double beta2, double eps, int step, hipStream_t st) {
  DSG_REQUIRE(p && g && m && v && n >= 0 && step >= 1, "dsgan_adam: bad args");
  if (n == 0) return 0;
  adam_launch<false>(p, g, m, v, n, adam_scal(lr, beta1, beta2, eps, step), lr, beta1, beta2, eps, nullptr, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

// ---- fp16 mode (--precision fp16): dynamic loss scaling, device-resident ----------------------
// torch.cuda.amp.GradScaler semantics without a host sync: the loss is multiplied by state[0]
// before backward, so every gradient -- including the fp16 MFMA operands of the backward
// (upstream grads, dz, the VGG data-grads) -- is scaled out of the fp16 subnormal range.  After
// the backward (and the DDP all-reduce) amp_check scans the flat gradient for inf / nan, amp_update
// records {skip, 1/scale} for this step and updates the scale (x backoff on overflow, x growth
// after `interval` clean steps) and the optimizer's step count, and adam_amp_kernel applies the
// update with g / scale -- or nothing when the step overflowed (its step count is not advanced,
// as GradScaler skips optimizer.step()).
// state (fp32[5]): [0] scale, [1] skip (this step), [2] clean steps since the last change,
//                  [3] 1/scale of this step, [4] applied optimizer steps.
namespace dsg {
constexpr int AMP_PARTS = 1024;
__global__ __launch_bounds__(256) void amp_check_kernel(const float* __restrict__ g, long n, int* __restrict__ part) {
  __shared__ int sh[4];
  int bad = 0;
  const long n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = g4[i];
    bad |= !isfinite(v.x) | !isfinite(v.y) | !isfinite(v.z) | !isfinite(v.w);
  }
  for (long i = (n4 << 2) + blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) bad |= !isfinite(g[i]);
  bad = __any(bad) ? 1 : 0;
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = bad;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] | sh[1] | sh[2] | sh[3];
}
__global__ __launch_bounds__(64) void amp_update_kernel(const int* __restrict__ part, int nparts, float* __restrict__ st,
                                                        float backoff, float growth, int interval) {
  int bad = 0;
  for (int i = threadIdx.x; i < nparts; i += 64) bad |= part[i];
  bad = __any(bad) ? 1 : 0;
  if (threadIdx.x == 0) {
    const float scale = st[0];
    st[1] = bad ? 1.f : 0.f;
    st[3] = 1.f / scale;
    if (bad) {
      st[0] = scale * backoff;
      st[2] = 0.f;
    } else {
      st[4] += 1.f;
      const float good = st[2] + 1.f;
      if (good >= (float)interval) { st[0] = scale * growth; st[2] = 0.f; }
      else st[2] = good;
    }
  }
}
}  // namespace dsg

extern "C" {
// scratch ints dsgan_amp_check needs
long dsgan_amp_parts(void) { return AMP_PARTS; }
// scan the flat gradient for inf/nan and update the scaler state (see above); part: dsgan_amp_parts() ints
int dsgan_amp_check(const float* grad, long n, int* part, float* state, float backoff, float growth, int interval,
                    hipStream_t st) {
  DSG_REQUIRE(grad && part && state && n > 0 && ((uintptr_t)grad & 15) == 0 && interval > 0, "dsgan_amp_check: bad args");
  long blocks = (n / 4 + 255) / 256;
  if (blocks > AMP_PARTS) blocks = AMP_PARTS;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(amp_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, grad, n, part);
  hipLaunchKernelGGL(amp_update_kernel, dim3(1), dim3(64), 0, st, part, (int)blocks, state, backoff, growth, interval);
  DSG_CHECK_LAUNCH();
  return 0;
}
// Adam on the unscaled gradient g * state[3], skipped when state[1] != 0; step count = state[4]
int dsgan_adam_amp(float* p, const float* g, float* m, float* v, long n, double lr, double beta1, double beta2,
                   double eps, const float* state, hipStream_t st) {
  DSG_REQUIRE(p && g && m && v && state && n >= 0, "dsgan_adam_amp: bad args");
  if (n == 0) return 0;
  adam_launch<true>(p, g, m, v, n, AdamScal{}, lr, beta1, beta2, eps, state, st);
  DSG_CHECK_LAUNCH();
  return 0;
}
}
