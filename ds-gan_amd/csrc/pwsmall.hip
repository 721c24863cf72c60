// Pointwise (1x1) contractions with a handful of channels on one side (gfx950, fp32 VALU).
//
// At 256x256 the generator's first layers are 1x1 convs from / to a 3- or 12-channel tensor:
// c1.pwconv1 3->12, c1.pwconv2 12->64, c1.shortcut 3->64 (MixConvNeXtML.py:218-224 on the
// 3-channel input), OriginMLKA.to32 / shortcut 3->32/64 (:122,145), and the data-grads into the
// 12-channel hidden.  A 128-wide MFMA tile wastes >90% of its work on K = 3 or M = 12, and the
// layers are pure HBM streams (268 MB written for 64 channels at 16x256^2), so this is a
// streaming VALU kernel: thread = 4 consecutive pixels (float4 in, float4 out), weights through
// scalar loads (uniform indices), exact fp32 FMAs in a fixed order -- the same result in the
// bf16 and the fp32 parity modes.
//
//   Y[b][m][p] (+)= act( bias[m] + sum_k W[m*wm + k*wk] * xact(X[b][k][p]) ) (* gact'(G[b][m][p]))
#include "common.h"

namespace dsg {

struct PsArgs {
  const float* X; long x_bs;
  const float* W; int wm, wk;
  const float* X2; long x2_bs;    // optional second input (K2 channels, xact applies to it only)
  const float* W2; int K2;        // W2[m][k2] row-major
  const float* bias;
  float* Y; long y_bs;
  const float* G; long g_bs;
  int nb, K, M, P;
  int act, xact, gact, accumulate; float slope;
};

constexpr int PS_MAXK = 256;           // M-small kernel: weights of up to 256 reduction channels in LDS
constexpr int PS_MAXM = 256;           // K-small kernel: weights of up to 256 output channels in LDS

template <int MC>
__global__ __launch_bounds__(256) void pw_small_kernel(PsArgs a) {
  // weights [k][MC] in LDS (broadcast reads; scalar loads in the k loop serialise on latency)
  __shared__ __attribute__((aligned(16))) float wl[PS_MAXK * MC];
  const int P4 = a.P >> 2;
  const long total = (long)a.nb * P4;
  for (int m0 = 0; m0 < a.M; m0 += MC) {          // chunks outside the pixel loop: uniform barriers
    __syncthreads();
    for (int e = threadIdx.x; e < a.K * MC; e += 256) {
      const int k = e / MC, i = e - k * MC;
      wl[e] = m0 + i < a.M ? a.W[(m0 + i) * a.wm + k * a.wk] : 0.f;
    }
    __syncthreads();
    for (long q = blockIdx.x * 256L + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
      const int b = (int)(q / P4), p = (int)(q - (long)b * P4) * 4;
      const float* xb = a.X + (long)b * a.x_bs + p;
      float* yb = a.Y + (long)b * a.y_bs + p;
      const float* gb = a.G ? a.G + (long)b * a.g_bs + p : nullptr;
      float4 acc[MC];
#pragma unroll
      for (int i = 0; i < MC; ++i) {
        const float bv = (a.bias && m0 + i < a.M) ? a.bias[m0 + i] : 0.f;
        acc[i] = make_float4(bv, bv, bv, bv);
      }
      auto step = [&](int k, float4 x) __attribute__((always_inline)) {
        if (a.xact) { x.x = act_f(a.xact, x.x, a.slope); x.y = act_f(a.xact, x.y, a.slope);
                      x.z = act_f(a.xact, x.z, a.slope); x.w = act_f(a.xact, x.w, a.slope); }
#pragma unroll
        for (int i = 0; i < MC; ++i) {
          const float w = wl[k * MC + i];
          acc[i].x = fmaf(w, x.x, acc[i].x); acc[i].y = fmaf(w, x.y, acc[i].y);
          acc[i].z = fmaf(w, x.z, acc[i].z); acc[i].w = fmaf(w, x.w, acc[i].w);
        }
      };
      // KU input channels' loads in flight per step (one load per step left the walk latency-bound:
      // 2.6 TB/s on the 64 -> 12 data-grad at 256^2); the channels still enter each sum in order
      constexpr int KU = MC > 8 ? 4 : 8;   // (8 at MC = 16 hoists 128 weight reads: 246 VGPRs)
      int k = 0;
      for (; k + KU <= a.K; k += KU) {
        float4 xv[KU];
#pragma unroll
        for (int u = 0; u < KU; ++u) xv[u] = *reinterpret_cast<const float4*>(xb + (long)(k + u) * a.P);
#pragma unroll
        for (int u = 0; u < KU; ++u) step(k + u, xv[u]);
      }
      for (; k < a.K; ++k) step(k, *reinterpret_cast<const float4*>(xb + (long)k * a.P));
#pragma unroll
      for (int i = 0; i < MC; ++i) {
        const int m = m0 + i;
        if (m >= a.M) break;
        float4 v = acc[i];
        if (a.act) { v.x = act_f(a.act, v.x, a.slope); v.y = act_f(a.act, v.y, a.slope);
                     v.z = act_f(a.act, v.z, a.slope); v.w = act_f(a.act, v.w, a.slope); }
        if (gb) {
          const float4 gv = *reinterpret_cast<const float4*>(gb + (long)m * a.P);
          v.x *= act_g(a.gact, gv.x, a.slope); v.y *= act_g(a.gact, gv.y, a.slope);
          v.z *= act_g(a.gact, gv.z, a.slope); v.w *= act_g(a.gact, gv.w, a.slope);
        }
        float4* dst = reinterpret_cast<float4*>(yb + (long)m * a.P);
        if (a.accumulate) { const float4 o = *dst; v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
        *dst = v;
      }
    }
  }
}

// K <= 16 input channels: the thread's 4 pixels x K inputs are loaded (and xact applied) once,
// then every output channel is one K-term dot product stored immediately.
// ACC / GP: accumulate into Y / multiply by gact'(G) (compile-time, so the plain forward carries
// no registers for the preloaded operands of either).
template <int KC, bool ACC, bool GP>
__global__ __launch_bounds__(256) void pw_small_k_kernel(PsArgs a) {
  __shared__ __attribute__((aligned(16))) float wl[PS_MAXM * KC];   // [m][KC] (W then W2 columns)
  for (int e = threadIdx.x; e < a.M * KC; e += 256) {
    const int m = e / KC, k = e - m * KC;
    wl[e] = k < a.K ? a.W[m * a.wm + k * a.wk] : (a.X2 && k < a.K + a.K2 ? a.W2[m * a.K2 + (k - a.K)] : 0.f);
  }
  __syncthreads();
  const int P4 = a.P >> 2;
  const long total = (long)a.nb * P4;
  for (long q = blockIdx.x * 256L + threadIdx.x; q < total; q += (long)gridDim.x * 256) {
    const int b = (int)(q / P4), p = (int)(q - (long)b * P4) * 4;
    const float* xb = a.X + (long)b * a.x_bs + p;
    float* yb = a.Y + (long)b * a.y_bs + p;
    const float* gb = GP ? a.G + (long)b * a.g_bs + p : nullptr;
    // inputs: K channels of X (xact applied when there is no X2), then K2 channels of X2 (xact)
    float4 xs[KC];
    const float* x2b = a.X2 ? a.X2 + (long)b * a.x2_bs + p : nullptr;
    const int xact1 = a.X2 ? 0 : a.xact;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      int xa = 0;
      if (k < a.K) { x = *reinterpret_cast<const float4*>(xb + (long)k * a.P); xa = xact1; }
      else if (x2b && k < a.K + a.K2) { x = *reinterpret_cast<const float4*>(x2b + (long)(k - a.K) * a.P); xa = a.xact; }
      if (xa) { x.x = act_f(xa, x.x, a.slope); x.y = act_f(xa, x.y, a.slope);
                x.z = act_f(xa, x.z, a.slope); x.w = act_f(xa, x.w, a.slope); }
      xs[k] = x;
    }
    // output channels in chunks of 8: the chunk's accumulate / act' operands are loaded up front
    // so their latencies overlap (a load after the previous channel's store could alias it)
    for (int m0 = 0; m0 < a.M; m0 += 8) {
      float4 old[ACC ? 8 : 1], gv[GP ? 8 : 1];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + i < a.M ? m0 + i : a.M - 1;
        if (ACC) old[i] = *reinterpret_cast<const float4*>(yb + (long)m * a.P);
        if (GP) gv[i] = *reinterpret_cast<const float4*>(gb + (long)m * a.P);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = m0 + i;
        if (m >= a.M) break;
        const float bv = a.bias ? a.bias[m] : 0.f;
        float4 v = make_float4(bv, bv, bv, bv);
#pragma unroll
        for (int k = 0; k < KC; ++k) {
          const float w = wl[m * KC + k];
          v.x = fmaf(w, xs[k].x, v.x); v.y = fmaf(w, xs[k].y, v.y);
          v.z = fmaf(w, xs[k].z, v.z); v.w = fmaf(w, xs[k].w, v.w);
        }
        if (a.act) { v.x = act_f(a.act, v.x, a.slope); v.y = act_f(a.act, v.y, a.slope);
                     v.z = act_f(a.act, v.z, a.slope); v.w = act_f(a.act, v.w, a.slope); }
        if constexpr (GP) {
          v.x *= act_g(a.gact, gv[i].x, a.slope); v.y *= act_g(a.gact, gv[i].y, a.slope);
          v.z *= act_g(a.gact, gv[i].z, a.slope); v.w *= act_g(a.gact, gv[i].w, a.slope);
        }
        if constexpr (ACC) { v.x += old[i].x; v.y += old[i].y; v.z += old[i].z; v.w += old[i].w; }
        *reinterpret_cast<float4*>(yb + (long)m * a.P) = v;
      }
    }
  }
}

}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_pw_small_supported(int K, int M, int P, long x_bs, long y_bs) {
  return ((K <= 16 && M <= PS_MAXM) || (M <= 16 && K <= PS_MAXK)) && K >= 1 && M >= 1 && P % 4 == 0 &&
         x_bs % 4 == 0 && y_bs % 4 == 0;
}

// Y[b][m][p] (+)= act(bias[m] + sum_k W[m*wm + k*wk] * xact(X[b][k][p])) (* gact'(G[b][m][p])):
// forward (wm = K, wk = 1) or data-grad (W^T: wm = 1, wk = M_fwd) of a 1x1 conv with <= 16
// channels on one side.  16-byte aligned rows, P % 4 == 0.
int dsgan_pw_small2(const float* X, long x_bs, const float* W, int wm, int wk, const float* X2, long x2_bs,
                    const float* W2, int K2, const float* bias, float* Y, long y_bs, const float* G, long g_bs,
                    int nb, int K, int M, int P, int act, int xact, int gact, int accumulate, float slope,
                    hipStream_t st);

int dsgan_pw_small(const float* X, long x_bs, const float* W, int wm, int wk, const float* bias, float* Y,
                   long y_bs, const float* G, long g_bs, int nb, int K, int M, int P, int act, int xact, int gact,
                   int accumulate, float slope, hipStream_t st) {
  return dsgan_pw_small2(X, x_bs, W, wm, wk, nullptr, 0, nullptr, 0, bias, Y, y_bs, G, g_bs, nb, K, M, P, act, xact,
                         gact, accumulate, slope, st);
}

// Two-input form: Y = act(bias + W X + W2 xact(X2)) -- the c1 Block tail in one pass
// (shortcut(x) over the 3 input channels + pwconv2(gelu(z)) over the 12 hidden ones).
int dsgan_pw_small2(const float* X, long x_bs, const float* W, int wm, int wk, const float* X2, long x2_bs,
                    const float* W2, int K2, const float* bias, float* Y, long y_bs, const float* G, long g_bs,
                    int nb, int K, int M, int P, int act, int xact, int gact, int accumulate, float slope,
                    hipStream_t st) {
  DSG_REQUIRE(X && W && Y && nb > 0, "dsgan_pw_small: bad args");
  DSG_REQUIRE(!X2 || (W2 && K2 > 0 && K + K2 <= 16 && x2_bs % 4 == 0 && ((uintptr_t)X2 & 15) == 0),
              "dsgan_pw_small2: second input needs K + K2 <= 16 and 16-byte rows");
  DSG_REQUIRE(dsgan_pw_small_supported(K, M, P, x_bs, y_bs) && (!G || g_bs % 4 == 0) &&
                  ((uintptr_t)X & 15) == 0 && ((uintptr_t)Y & 15) == 0 && (!G || ((uintptr_t)G & 15) == 0),
              "dsgan_pw_small: unsupported K=%d M=%d P=%d (K or M <= 16, P %% 4 == 0, 16-byte rows)", K, M, P);
  PsArgs a{X, x_bs, W, wm, wk, X2, x2_bs, W2, X2 ? K2 : 0, bias, Y, y_bs, G, g_bs, nb, K, M, P, act, xact, gact,
           accumulate, slope};
  const int Kt = K + (X2 ? K2 : 0);
  const long total = (long)nb * (P / 4);
  long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  const int sel = (accumulate ? 1 : 0) + (G ? 2 : 0);
#define PSK(KC_)                                                                                        \
  switch (sel) {                                                                                        \
    case 0: hipLaunchKernelGGL((pw_small_k_kernel<KC_, false, false>), dim3((unsigned)blocks), dim3(256), 0, st, a); break; \
    case 1: hipLaunchKernelGGL((pw_small_k_kernel<KC_, true, false>), dim3((unsigned)blocks), dim3(256), 0, st, a); break;  \
    case 2: hipLaunchKernelGGL((pw_small_k_kernel<KC_, false, true>), dim3((unsigned)blocks), dim3(256), 0, st, a); break;  \
    default: hipLaunchKernelGGL((pw_small_k_kernel<KC_, true, true>), dim3((unsigned)blocks), dim3(256), 0, st, a); break;  \
  }
  if (Kt <= 4) { PSK(4) }
  else if (Kt <= 16) { PSK(16) }
#undef PSK
  else if (M <= 4) hipLaunchKernelGGL((pw_small_kernel<4>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((pw_small_kernel<16>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
