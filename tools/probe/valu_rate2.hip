// VALU issue-rate probe: gelu_fast on 16 independent registers per lane, ITER times, at W waves per
// SIMD (grid = 256 CUs x 4 SIMDs x W waves).  Prints ns and VALU instructions per SIMD-cycle.
#include "../../ds-gan_amd/csrc/common.h"
#include <cstdio>
using namespace dsg;
template <int E>
__global__ __launch_bounds__(256) void k_gelu(float* out, int iters, float s) {
  float v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = (threadIdx.x + e) * 1e-3f - 0.5f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int e = 0; e < E; e += 2) {
      f32x2 r = gelu_fast2(f32x2{v[e], v[e + 1]}) * s - 0.25f;
      v[e] = r.x; v[e + 1] = r.y;
    }
  }
  float a = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) a += v[e];
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float s) {
  float v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) v[e] = (threadIdx.x + e) * 1e-3f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] = fmaf(v[e], s, 0.125f);
  }
  float a = 0.f;
#pragma unroll
  for (int e = 0; e < 16; ++e) a += v[e];
  out[blockIdx.x * 256 + threadIdx.x] = a;
}
int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 16 * 256 * sizeof(float));
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 2000;
  for (int W = 1; W <= 8; W *= 2) {
    // 256 threads = 4 waves per block; 256 CUs x W blocks -> W waves per SIMD
    const int blocks = 256 * W;
    for (int kind = 0; kind < 2; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        if (kind == 0) hipLaunchKernelGGL(k_gelu<16>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
        else hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      // per SIMD: W waves x iters x (16 elements x VALU-per-element) instructions
      const double elems = (double)W * iters * 16 * (kind == 0 ? 1 : 8);
      printf("%s W=%d  %.3f ms  %.3f ns per element-instr-group per SIMD (elements/SIMD %.3g)\n",
             kind == 0 ? "gelu" : "fma ", W, best, best * 1e6 / elems, elems);
    }
  }
  return 0;
}
