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
