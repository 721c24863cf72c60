// Fused Adam over a flat parameter buffer (torch.optim.Adam semantics, amsgrad=False,
// weight_decay=0; used by DSGAN/models/pix2pix_model.py:122-125 with lr=2e-4, betas=(0.5,0.999)).
// Every generator (or discriminator) parameter is a view into one contiguous fp32 buffer, so
// one launch updates all 188 (or 10) tensors.  Arithmetic mirrors torch's single-tensor path:
//   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g
//   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
#include "common.h"

namespace dsg {
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long n, float w1, float b2, float step_size,
                            float bc2_sqrt, float eps) {
  const long i0 = (blockIdx.x * 256L + threadIdx.x) * 4;
  for (long i = i0; i < n; i += (long)gridDim.x * 256 * 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long e = i + j;
      if (e >= n) break;
      const float gr = g[e];
      float mm = m[e];
      // at::lerp: weight < 0.5 ? a + w*(b-a) : b - (b-a)*(1-w)
      mm = w1 < 0.5f ? mm + w1 * (gr - mm) : gr - (gr - mm) * (1.f - w1);
      const float vv = v[e] * b2 + (1.f - b2) * gr * gr;
      m[e] = mm; v[e] = vv;
      const float denom = sqrtf(vv) / bc2_sqrt + eps;
      p[e] = p[e] - step_size * (mm / denom);
    }
  }
}
}  // namespace dsg

using namespace dsg;
extern "C" int dsgan_adam(float* p, const float* g, float* m, float* v, long n, float lr, float beta1,
                          float beta2, float eps, int step, hipStream_t st) {
  DSG_REQUIRE(p && g && m && v && n >= 0 && step >= 1, "dsgan_adam: bad args");
  if (n == 0) return 0;
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  long blocks = (n + 1023) / 1024;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, 1.f - beta1,
                     beta2, step_size, bc2s, eps);
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
__global__ void adam_amp_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, long n, float lr, float beta1, float beta2, float eps,
                                const float* __restrict__ st) {
  if (st[1] != 0.f) return;   // overflowed step: parameters and moments untouched
  const float inv = st[3];
  const double t = (double)st[4];
  // torch's bias corrections (python doubles), rounded to fp32 as torch hands them to the update
  const float step_size = (float)((double)lr / (1.0 - pow((double)beta1, t)));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, t));
  const float w1 = 1.f - beta1;
  const long i0 = (blockIdx.x * 256L + threadIdx.x) * 4;
  for (long i = i0; i < n; i += (long)gridDim.x * 256 * 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long e = i + j;
      if (e >= n) break;
      const float gr = g[e] * inv;
      float mm = m[e];
      mm = w1 < 0.5f ? mm + w1 * (gr - mm) : gr - (gr - mm) * (1.f - w1);
      const float vv = v[e] * beta2 + (1.f - beta2) * gr * gr;
      m[e] = mm; v[e] = vv;
      const float denom = sqrtf(vv) / bc2s + eps;
      p[e] = p[e] - step_size * (mm / denom);
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
int dsgan_adam_amp(float* p, const float* g, float* m, float* v, long n, float lr, float beta1, float beta2, float eps,
                   const float* state, hipStream_t st) {
  DSG_REQUIRE(p && g && m && v && state && n >= 0, "dsgan_adam_amp: bad args");
  if (n == 0) return 0;
  long blocks = (n + 1023) / 1024;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(adam_amp_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2, eps,
                     state);
  DSG_CHECK_LAUNCH();
  return 0;
}
}
