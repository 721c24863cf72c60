// Loss kernels of backward_D / backward_G (DSGAN/models/pix2pix_model.py:141-199):
//   BCE-with-logits vs a constant label (GANLoss, DSGAN/models/networks.py:143-163),
//   L1 mean (:177, :182-186), TV sum (:189-191), and the fused gaussian SSIM
//   (DSGAN/MS_SSIM.py:26-150) forward + analytic backward.
// Scalar results are written to device memory; backward kernels read the upstream gradient
// from device memory, so nothing here forces a host synchronisation.
#include "common.h"

namespace dsg {

static inline unsigned red_grid(long n) {
  long g = (n + 2047) / 2048;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---- BCE with logits, mean over n, target t -----------------------------------------
__global__ __launch_bounds__(256) void bce_fwd_kernel(const float* x, long n, float t, float* out, float coef) {
  __shared__ float sh[4];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float v = x[i];
    s += fmaxf(v, 0.f) - v * t + log1pf(__expf(-fabsf(v)));
  }
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = s;   // block partial (final_sum_kernel adds them in order)
}
__global__ void bce_bwd_kernel(const float* x, long n, float t, const float* gout, float coef, float* dx, int accumulate) {
  const float g = gout[0] * coef;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float v = (1.f / (1.f + __expf(-x[i])) - t) * g;
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

// ---- L1 mean ------------------------------------------------------------------------
__global__ __launch_bounds__(256) void l1_fwd_kernel(const float* a, const float* b, long n, float* out, float coef) {
  __shared__ float sh[4];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += fabsf(a[i] - b[i]);
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}
// 16-byte form (both operands 16-byte aligned): float4 pairs, two in flight per thread; the
// n % 4 tail is summed by block 0.
__global__ __launch_bounds__(256) void l1_fwd_v4_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                       long n4, const float* __restrict__ ta,
                                                       const float* __restrict__ tb, int tail, float* out, float coef) {
  __shared__ float sh[4];
  float s0 = 0.f, s1 = 0.f;
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const float4 x0 = a[i], y0 = b[i], x1 = a[i + stride], y1 = b[i + stride];
    s0 += fabsf(x0.x - y0.x) + fabsf(x0.y - y0.y) + fabsf(x0.z - y0.z) + fabsf(x0.w - y0.w);
    s1 += fabsf(x1.x - y1.x) + fabsf(x1.y - y1.y) + fabsf(x1.z - y1.z) + fabsf(x1.w - y1.w);
  }
  if (i < n4) {
    const float4 x0 = a[i], y0 = b[i];
    s0 += fabsf(x0.x - y0.x) + fabsf(x0.y - y0.y) + fabsf(x0.z - y0.z) + fabsf(x0.w - y0.w);
  }
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) s1 += fabsf(ta[threadIdx.x] - tb[threadIdx.x]);
  float s = block_sum<256>(s0 + s1, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}
__global__ void l1_bwd_kernel(const float* a, const float* b, long n, const float* gout, float coef, float* da, int accumulate) {
  const float g = gout[0] * coef;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float d = a[i] - b[i];
    const float v = d > 0.f ? g : (d < 0.f ? -g : 0.f);
    da[i] = accumulate ? da[i] + v : v;
  }
}

// ---- TV: (sum |y[..,w+1]-y[..,w]| + sum |y[..,h+1,:]-y[..,h,:]|) * coef ----------------
__global__ __launch_bounds__(256) void tv_fwd_kernel(const float* y, long planes, int H, int W, float* out, float coef) {
  __shared__ float sh[4];
  const long n = planes * H * W;
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int w = i % W; const int h = (i / W) % H;
    const float v = y[i];
    if (w + 1 < W) s += fabsf(y[i + 1] - v);
    if (h + 1 < H) s += fabsf(y[i + W] - v);
  }
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// out[0] = coef * sum_i part[i], i in a fixed order (deterministic loss values)
__global__ __launch_bounds__(256) void final_sum_kernel(const float* __restrict__ part, int n, float coef,
                                                        float* __restrict__ out) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) out[0] = s * coef;
}

// Two-level form for many partials (the 512^2 VGG pool-L1 taps have tens of thousands,
// a long serial tail for one workgroup): chunk c = part[c * ch .. c * ch + ch) is summed by workgroup
// c in a fixed order and written back over its first element; then one workgroup sums the chunk
// sums (stride ch) in order.  In place: no scratch beyond the partials themselves.
__global__ __launch_bounds__(256) void chunk_sum_kernel(float* __restrict__ part, int n, int ch) {
  __shared__ float sh[4];
  const long b0 = (long)blockIdx.x * ch;
  const int m = (int)min((long)ch, (long)n - b0);
  float s = 0.f;
  for (int i = threadIdx.x; i < m; i += 256) s += part[b0 + i];
  s = block_sum<256>(s, sh);   // (every read of the chunk precedes the block's barriers)
  if (threadIdx.x == 0) part[b0] = s;
}
__global__ __launch_bounds__(256) void strided_sum_kernel(const float* __restrict__ part, int nc, int ch, float coef,
                                                          float* __restrict__ out) {
  __shared__ float sh[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nc; i += 256) s += part[(long)i * ch];
  s = block_sum<256>(s, sh);
  if (threadIdx.x == 0) out[0] = s * coef;
}

constexpr int FS_TWO_LEVEL = 16384, FS_CHUNK = 1024;
void launch_final_sum(const float* part, int n, float coef, float* out, hipStream_t st) {
  if (n > FS_TWO_LEVEL) {   // (the partials are the caller's scratch: overwritten in place)
    const int nc = (n + FS_CHUNK - 1) / FS_CHUNK;
    hipLaunchKernelGGL(chunk_sum_kernel, dim3((unsigned)nc), dim3(256), 0, st, const_cast<float*>(part), n, FS_CHUNK);
    hipLaunchKernelGGL(strided_sum_kernel, dim3(1), dim3(256), 0, st, part, nc, FS_CHUNK, coef, out);
    return;
  }
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, n, coef, out);
}

// stats[p][j] = sum over the tiles t of part[p][t][j], j in {0, 1} (fixed order)
__global__ void plane_tile_sum_kernel(const float* __restrict__ part, int planes, int tiles, float* __restrict__ stats) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= planes * 2) return;
  const int p = t >> 1, j = t & 1;
  const float* q = part + (long)p * tiles * 2 + j;
  float s = 0.f;
  for (int i = 0; i < tiles; ++i) s += q[2L * i];
  stats[t] = s;
}
__device__ __forceinline__ float sgnf(float d) { return d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f); }

// ---- VGG perceptual tap backward (DSGAN/models/vgg.py:30-42 + pix2pix_model.py:182-186) -----
// Gradient w.r.t. the pre-ReLU activation of a tapped VGG conv whose post-ReLU output y is both
// an L1 feature (vs the real-image feature r) and the input of a 2x2 MaxPool (or the top):
//   dx = (maxpool_bwd(dpool, idx) + g*coef*sign(y - r)) * (y > 0)
// fusing the L1 backward, the autograd sum of the two consumers' grads and the ReLU backward.
// y, r, dx: contiguous [planes][H][W]; dpool/idx: [planes][H/2][W/2] (plane-flat argmax).
__global__ void vgg_tap_bwd_pool_kernel(const float* __restrict__ dpool, const int* __restrict__ idx,
                                        const float* __restrict__ y, const float* __restrict__ r, long npool,
                                        int H, int W, const float* __restrict__ gout, float coef,
                                        float* __restrict__ dx) {
  const float g = gout[0] * coef;
  const int Wo = W / 2, Po = (H / 2) * Wo;
  for (long o = blockIdx.x * 256L + threadIdx.x; o < npool; o += (long)gridDim.x * 256) {
    const long plane = o / Po;
    const int p = (int)(o - plane * Po), oh = p / Wo, ow = p - oh * Wo;
    const int id = idx[o];
    const float gp = dpool[o];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rb = (2 * oh + i) * W + 2 * ow;
      const long e = plane * H * W + rb;
      const float2 yv = *reinterpret_cast<const float2*>(y + e);
      const float2 rv = *reinterpret_cast<const float2*>(r + e);
      float2 v;
      v.x = (rb == id ? gp : 0.f) + g * sgnf(yv.x - rv.x);
      v.y = (rb + 1 == id ? gp : 0.f) + g * sgnf(yv.y - rv.y);
      v.x = yv.x > 0.f ? v.x : 0.f;
      v.y = yv.y > 0.f ? v.y : 0.f;
      *reinterpret_cast<float2*>(dx + e) = v;
    }
  }
}
// top tap (no pool above): dx = g*coef*sign(y - r) * (y > 0)
__global__ void vgg_tap_bwd_top_kernel(const float* __restrict__ y, const float* __restrict__ r, long n4,
                                       const float* __restrict__ gout, float coef, float* __restrict__ dx) {
  const float g = gout[0] * coef;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 yv = reinterpret_cast<const float4*>(y)[i];
    const float4 rv = reinterpret_cast<const float4*>(r)[i];
    float4 v;
    v.x = yv.x > 0.f ? g * sgnf(yv.x - rv.x) : 0.f;
    v.y = yv.y > 0.f ? g * sgnf(yv.y - rv.y) : 0.f;
    v.z = yv.z > 0.f ? g * sgnf(yv.z - rv.z) : 0.f;
    v.w = yv.w > 0.f ? g * sgnf(yv.w - rv.w) : 0.f;
    reinterpret_cast<float4*>(dx)[i] = v;
  }
}
__global__ void tv_bwd_kernel(const float* y, long planes, int H, int W, const float* gout, float coef, float* dy, int accumulate) {
  const float g = gout[0] * coef;
  const long n = planes * H * W;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int w = i % W; const int h = (i / W) % H;
    const float v = y[i];
    float d = 0.f;
    if (w + 1 < W) d -= sgnf(y[i + 1] - v);
    if (w > 0) d += sgnf(v - y[i - 1]);
    if (h + 1 < H) d -= sgnf(y[i + W] - v);
    if (h > 0) d += sgnf(v - y[i - W]);
    dy[i] = accumulate ? dy[i] + g * d : g * d;
  }
}

// ---- SSIM ---------------------------------------------------------------------------
// X = a*real + b, Y = a*fake + b (a=b=0.5 for (t+1)/2, :193-194).  11-tap gaussian (sigma 1.5),
// valid filtering; per output pixel S = A1*A2/(B1*B2).  The forward also writes the three
// per-pixel coefficient maps of dS/dY used by the backward:
//   dS/dmu2 = S*(2mu1/A1 - 2mu1/A2 - 2mu2/B1 + 2mu2/B2), dS/dE[YY] = -S/B2, dS/dE[XY] = 2S/A2
// and dL/dY = G^T*(c_mu) + 2Y*G^T*(c_yy) + X*G^T*(c_xy)   (G^T = adjoint "full" filtering).
constexpr int SS_T = 32, SS_K = 11, SS_E = SS_T + SS_K - 1;

struct SSIMArgs {
  const float* real; const float* fake; float a, b;
  int planes, H, W;
  const float* win;   // 11 taps
  float C1, C2;
  float* coef;        // [3][planes][Ho][Wo]
  float* out;         // sum of S (nullable: coefficient maps only)
  const float* kscale;  // per-plane factor of the coefficient maps (nullable = 1)
  int cs_mode;          // coefficient maps of the contrast-structure term cs instead of S (MS-SSIM)
};

__global__ __launch_bounds__(256) void ssim_fwd_kernel(SSIMArgs s, int tiles_w) {
  __shared__ float xs[SS_E][SS_E + 1], ys[SS_E][SS_E + 1];
  __shared__ float hb[5][SS_E][SS_T + 1];  // blurred along H first (reference order: dim 2 then 3)
  __shared__ float wsh[SS_K];
  __shared__ float sh[4];
  const int plane = blockIdx.y;
  const int Ho = s.H - SS_K + 1, Wo = s.W - SS_K + 1;
  const int oh0 = (blockIdx.x / tiles_w) * SS_T, ow0 = (blockIdx.x % tiles_w) * SS_T;
  const float* rp = s.real + (long)plane * s.H * s.W;
  const float* fp = s.fake + (long)plane * s.H * s.W;
  if (threadIdx.x < SS_K) wsh[threadIdx.x] = s.win[threadIdx.x];
  for (int i = threadIdx.x; i < SS_E * SS_E; i += 256) {
    const int r = i / SS_E, q = i - r * SS_E;
    const int h = oh0 + r, w = ow0 + q;
    const bool ok = h < s.H && w < s.W;
    xs[r][q] = ok ? rp[(long)h * s.W + w] * s.a + s.b : 0.f;
    ys[r][q] = ok ? fp[(long)h * s.W + w] * s.a + s.b : 0.f;
  }
  __syncthreads();
  // vertical (H) pass: hb[k][out_row r][col q] for r in [0,32), q in [0,42)
  for (int i = threadIdx.x; i < SS_T * SS_E; i += 256) {
    const int r = i / SS_E, q = i - r * SS_E;
    float m1 = 0, m2 = 0, e11 = 0, e22 = 0, e12 = 0;
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float g = wsh[k], xv = xs[r + k][q], yv = ys[r + k][q];
      m1 += g * xv; m2 += g * yv; e11 += g * (xv * xv); e22 += g * (yv * yv); e12 += g * (xv * yv);
    }
    hb[0][q][r] = m1; hb[1][q][r] = m2; hb[2][q][r] = e11; hb[3][q][r] = e22; hb[4][q][r] = e12;
  }
  __syncthreads();
  float ssum = 0.f;
  const long plane_out = (long)Ho * Wo;
  for (int i = threadIdx.x; i < SS_T * SS_T; i += 256) {
    const int r = i >> 5, q = i & 31;
    const int oh = oh0 + r, ow = ow0 + q;
    if (oh >= Ho || ow >= Wo) continue;
    float v[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float g = wsh[k];
#pragma unroll
      for (int j = 0; j < 5; ++j) v[j] += g * hb[j][q + k][r];
    }
    const float mu1 = v[0], mu2 = v[1];
    const float s11 = v[2] - mu1 * mu1, s22 = v[3] - mu2 * mu2, s12 = v[4] - mu1 * mu2;
    const float A1 = 2.f * mu1 * mu2 + s.C1, A2 = 2.f * s12 + s.C2;
    const float B1 = mu1 * mu1 + mu2 * mu2 + s.C1, B2 = s11 + s22 + s.C2;
    const float cs = A2 / B2, l = A1 / B1;
    const float S = l * cs;
    ssum += S;
    const long o = (long)plane * plane_out + (long)oh * Wo + ow;
    const long stride = (long)s.planes * plane_out;
    if (s.cs_mode) {   // d cs: cs = (2 s12 + C2) / (s11 + s22 + C2)
      const float k = s.kscale[plane];
      s.coef[o] = k * ((2.f * mu2 * cs - 2.f * mu1) / B2);
      s.coef[o + stride] = k * (-cs / B2);
      s.coef[o + 2 * stride] = k * (2.f / B2);
    } else {
      const float k = s.kscale ? s.kscale[plane] : 1.f;
      // S / A1 = cs / B1 and S / A2 = l / B2, written without the division by A1 or A2: those
      // cross zero (a negative local mean of fake, a covariance of -C2/2), where S * (1/A) is 0 * inf
      // = NaN although the derivative is finite -- the reference's autograd of A/B never divides by A
      s.coef[o] = k * (2.f * mu1 * (cs / B1 - l / B2) + 2.f * mu2 * (S / B2 - S / B1));
      s.coef[o + stride] = k * (-S / B2);
      s.coef[o + 2 * stride] = k * (2.f * l / B2);
    }
  }
  if (s.out) {   // per-tile partial sum of S (final_sum_kernel)
    ssum = block_sum<256>(ssum, sh);
    if (threadIdx.x == 0) s.out[(long)blockIdx.y * gridDim.x + blockIdx.x] = ssum;
  }
}

// ---- train.py per-iteration metrics (DSGAN/train.py:27-44, 110-124) ----------------------------
// The reference converts image 0 of fake_B / real_B to uint8 HWC on the host ((t+1)/2*255, clip,
// truncate) and calls skimage's structural_similarity (uniform 7x7 window, sample covariance,
// data_range 255, border-cropped mean, channel mean) and PSNR.  Here both run on the device on
// the same uint8 values; the per-call results are accumulated in device memory so the loop
// needs no host sync per iteration.  acc[0] += ssim, acc[1] += psnr, acc[2] += 1.
__device__ __forceinline__ float to_u8f(float t) {
  const float v = ((t + 1.f) / 2.f) * 255.f;
  return truncf(fminf(fmaxf(v, 0.f), 255.f));
}

__global__ __launch_bounds__(256) void img_metrics_kernel(const float* __restrict__ fake, const float* __restrict__ real,
                                                          int C, int H, int W, double* part) {
  __shared__ double sh[2][4];
  const int Hc = H - 6, Wc = W - 6;
  const long tot = (long)C * Hc * Wc;
  double ssum = 0.0, se = 0.0;
  const double NP = 49.0, cov = NP / (NP - 1.0), C1 = (0.01 * 255.0) * (0.01 * 255.0), C2 = (0.03 * 255.0) * (0.03 * 255.0);
  for (long t = blockIdx.x * 256L + threadIdx.x; t < tot; t += (long)gridDim.x * 256) {
    const int c = (int)(t / ((long)Hc * Wc));
    const int r = (int)(t - (long)c * Hc * Wc), h = r / Wc + 3, w = r - (r / Wc) * Wc + 3;
    const float* fp = fake + (long)c * H * W;
    const float* rp = real + (long)c * H * W;
    double sx = 0, sy = 0, sxx = 0, syy = 0, sxy = 0;
    for (int dh = -3; dh <= 3; ++dh)
      for (int dw = -3; dw <= 3; ++dw) {
        const long o = (long)(h + dh) * W + (w + dw);
        const double x = to_u8f(rp[o]), y = to_u8f(fp[o]);   // img1 = label, img2 = result
        sx += x; sy += y; sxx += x * x; syy += y * y; sxy += x * y;
      }
    const double ux = sx / NP, uy = sy / NP;
    const double vx = cov * (sxx / NP - ux * ux), vy = cov * (syy / NP - uy * uy), vxy = cov * (sxy / NP - ux * uy);
    ssum += ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux * ux + uy * uy + C1) * (vx + vy + C2));
  }
  for (long t = blockIdx.x * 256L + threadIdx.x; t < (long)C * H * W; t += (long)gridDim.x * 256) {
    const double d = (double)to_u8f(real[t]) - (double)to_u8f(fake[t]);
    se += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) { ssum += __shfl_xor(ssum, o, 64); se += __shfl_xor(se, o, 64); }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[0][wv] = ssum; sh[1][wv] = se; }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    part[2 * blockIdx.x + 1] = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
  }
}

__global__ void img_metrics_final_kernel(const double* part, int nblk, int C, int H, int W, float* acc) {
  if (threadIdx.x != 0) return;
  double s = 0, e = 0;
  for (int i = 0; i < nblk; ++i) { s += part[2 * i]; e += part[2 * i + 1]; }
  const double ssim = s / ((double)C * (H - 6) * (W - 6));
  const double mse = e / ((double)C * H * W);
  const double psnr = mse / (255.0 * 255.0) < 1e-10 ? 100.0 : 10.0 * log10(255.0 * 255.0 / mse);
  acc[0] += (float)ssim; acc[1] += (float)psnr; acc[2] += 1.f;
}

// ---- MS-SSIM evaluation (DSGAN/MS_SSIM.py:153-225; no gradient) ---------------------------
// One scale: per plane the sums of the SSIM map and of the contrast-structure map cs
// (_ssim, :55-92) -- same tiling and filter order as ssim_fwd_kernel, no backward coefficients.
__global__ __launch_bounds__(256) void ssim_eval_kernel(SSIMArgs s, int tiles_w, float* stats) {
  __shared__ float xs[SS_E][SS_E + 1], ys[SS_E][SS_E + 1];
  __shared__ float hb[5][SS_E][SS_T + 1];
  __shared__ float wsh[SS_K];
  __shared__ float sh[8];
  const int plane = blockIdx.y;
  const int Ho = s.H - SS_K + 1, Wo = s.W - SS_K + 1;
  const int oh0 = (blockIdx.x / tiles_w) * SS_T, ow0 = (blockIdx.x % tiles_w) * SS_T;
  const float* rp = s.real + (long)plane * s.H * s.W;
  const float* fp = s.fake + (long)plane * s.H * s.W;
  if (threadIdx.x < SS_K) wsh[threadIdx.x] = s.win[threadIdx.x];
  for (int i = threadIdx.x; i < SS_E * SS_E; i += 256) {
    const int r = i / SS_E, q = i - r * SS_E;
    const int h = oh0 + r, w = ow0 + q;
    const bool ok = h < s.H && w < s.W;
    xs[r][q] = ok ? rp[(long)h * s.W + w] * s.a + s.b : 0.f;
    ys[r][q] = ok ? fp[(long)h * s.W + w] * s.a + s.b : 0.f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SS_T * SS_E; i += 256) {
    const int r = i / SS_E, q = i - r * SS_E;
    float m1 = 0, m2 = 0, e11 = 0, e22 = 0, e12 = 0;
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float g = wsh[k], xv = xs[r + k][q], yv = ys[r + k][q];
      m1 += g * xv; m2 += g * yv; e11 += g * (xv * xv); e22 += g * (yv * yv); e12 += g * (xv * yv);
    }
    hb[0][q][r] = m1; hb[1][q][r] = m2; hb[2][q][r] = e11; hb[3][q][r] = e22; hb[4][q][r] = e12;
  }
  __syncthreads();
  float ssum = 0.f, csum = 0.f;
  for (int i = threadIdx.x; i < SS_T * SS_T; i += 256) {
    const int r = i >> 5, q = i & 31;
    if (oh0 + r >= Ho || ow0 + q >= Wo) continue;
    float v[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float g = wsh[k];
#pragma unroll
      for (int j = 0; j < 5; ++j) v[j] += g * hb[j][q + k][r];
    }
    const float mu1 = v[0], mu2 = v[1];
    const float s11 = v[2] - mu1 * mu1, s22 = v[3] - mu2 * mu2, s12 = v[4] - mu1 * mu2;
    const float cs = (2.f * s12 + s.C2) / (s11 + s22 + s.C2);
    ssum += ((2.f * mu1 * mu2 + s.C1) / (mu1 * mu1 + mu2 * mu2 + s.C1)) * cs;
    csum += cs;
  }
  ssum = block_sum<256>(ssum, sh);
  csum = block_sum<256>(csum, sh + 4);
  if (threadIdx.x == 0) {   // per-(plane, tile) partials, summed over tiles by plane_tile_sum_kernel
    float* q = stats + ((long)plane * gridDim.x + blockIdx.x) * 2;
    q[0] = ssum; q[1] = csum;
  }
}

// F.avg_pool2d(a*x+b, 2, padding=(H%2, W%2)) with count_include_pad (divisor 4), :213-215
__global__ void avgpool2_pad_kernel(const float* __restrict__ x, float* __restrict__ y, int planes, int H, int W,
                                    int Ho, int Wo, int ph, int pw, float a, float b) {
  const long total = (long)planes * Ho * Wo;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int p = (int)(t / ((long)Ho * Wo));
    const int r = (int)(t - (long)p * Ho * Wo), oh = r / Wo, ow = r - oh * Wo;
    const float* xp = x + (long)p * H * W;
    float acc = 0.f;
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int h = 2 * oh - ph + dh, w = 2 * ow - pw + dw;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) acc += xp[(long)h * W + w] * a + b;
      }
    y[t] = 0.25f * acc;
  }
}

struct MsArgs { float inv_cnt[8]; float wt[8]; };

// out[n] = mean_c prod_l relu(v_l[n][c])^w_l, v_l = cs (l < L-1) or ssim (l = L-1) -- :218-225;
// out[N] = mean over n.  One workgroup.
__global__ __launch_bounds__(256) void ms_ssim_combine_kernel(const float* stats, int levels, int N, int C,
                                                              MsArgs m, float* out) {
  __shared__ float sh[4];
  float tot = 0.f;
  for (int n = 0; n < N; ++n) {
    float acc = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) {
      float prod = 1.f;
      for (int l = 0; l < levels; ++l) {
        const float* st = stats + ((long)l * N * C + (long)n * C + c) * 2;
        const float v = fmaxf((l < levels - 1 ? st[1] : st[0]) * m.inv_cnt[l], 0.f);
        prod *= powf(v, m.wt[l]);
      }
      acc += prod;
    }
    acc = block_sum<256>(acc, sh) / (float)C;
    if (threadIdx.x == 0) out[n] = acc;
    tot += acc;
  }
  if (threadIdx.x == 0) out[N] = tot / (float)N;
}

// ---- MS-SSIM as a loss (backward of DSGAN/MS_SSIM.py:153-225 through its 5-level pyramid) ----
// Per plane p and level l the forward keeps the map sums (ssim_eval_kernel).  The loss is
// mean_p prod_l V_l^w_l with V_l = relu(mean cs_l) (l < L-1), relu(mean S_{L-1}); so
//   dL/d(map_l pixel) = gout/P * w_l * prod / V_l / count_l     (0 where the relu clips)
// = kscale[l][p]; the coefficient maps of level l are scaled by it and adjoint-filtered into
// dY_l, which also receives 1/4 of dY_{l+1} through the padded 2x2 average pool.
__global__ void ms_ssim_kscale_kernel(const float* stats, int levels, int planes, MsArgs m, const float* gout,
                                      float inv_planes, float* kscale) {
  for (int p = blockIdx.x * 256 + threadIdx.x; p < planes; p += gridDim.x * 256) {
    float v[8], pw[8];
    float prod = 1.f;
    for (int l = 0; l < levels; ++l) {
      const float* st = stats + ((long)l * planes + p) * 2;
      v[l] = (l < levels - 1 ? st[1] : st[0]) * m.inv_cnt[l];
      pw[l] = powf(fmaxf(v[l], 0.f), m.wt[l]);
      prod *= pw[l];
    }
    const float g = gout[0] * inv_planes;
    for (int l = 0; l < levels; ++l) {
      float others = 1.f;
      for (int k = 0; k < levels; ++k)
        if (k != l) others *= pw[k];
      // d V^w / dV = w V^(w-1), only where relu passes
      const float d = v[l] > 0.f ? m.wt[l] * powf(v[l], m.wt[l] - 1.f) * others : 0.f;
      kscale[(long)l * planes + p] = g * d * m.inv_cnt[l];
    }
  }
}

// dy[p][h][w] = scale * dup[p][(h+ph)/2][(w+pw)/2]  (adjoint of the count_include_pad 2x2 pool)
__global__ void avgpool2_pad_bwd_kernel(const float* __restrict__ dup, float* __restrict__ dy, int planes, int H,
                                        int W, int Ho, int Wo, int ph, int pw, float scale) {
  const long total = (long)planes * H * W;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
    const int p = (int)(t / ((long)H * W));
    const int r = (int)(t - (long)p * H * W), h = r / W, w = r - h * W;
    dy[t] = scale * dup[((long)p * Ho + (h + ph) / 2) * Wo + (w + pw) / 2];
  }
}

// dfake[h,w] = g * a * ( G^T c_mu + 2Y G^T c_yy + X G^T c_xy )  over input tile 32x32
__global__ __launch_bounds__(256) void ssim_bwd_kernel(SSIMArgs s, const float* gout, float gcoef,
                                                       float* dfake, int tiles_w, int accumulate) {
  __shared__ float cs[3][SS_E][SS_E + 1];
  __shared__ float vb[3][SS_T][SS_E + 1];
  __shared__ float wsh[SS_K];
  const int plane = blockIdx.y;
  const int Ho = s.H - SS_K + 1, Wo = s.W - SS_K + 1;
  const int h0 = (blockIdx.x / tiles_w) * SS_T, w0 = (blockIdx.x % tiles_w) * SS_T;
  if (threadIdx.x < SS_K) wsh[threadIdx.x] = s.win[threadIdx.x];
  const long plane_out = (long)Ho * Wo, stride = (long)s.planes * plane_out;
  // coefficient window: output rows h0-10 .. h0+31
  for (int i = threadIdx.x; i < SS_E * SS_E; i += 256) {
    const int r = i / SS_E, q = i - r * SS_E;
    const int oh = h0 - (SS_K - 1) + r, ow = w0 - (SS_K - 1) + q;
    const bool ok = oh >= 0 && ow >= 0 && oh < Ho && ow < Wo;
    const long o = (long)plane * plane_out + (long)oh * Wo + ow;
#pragma unroll
    for (int j = 0; j < 3; ++j) cs[j][r][q] = ok ? s.coef[o + j * stride] : 0.f;
  }
  __syncthreads();
  // adjoint of the W pass: vb[j][r][c] = sum_k g[k] * cs[j][r][c + 10 - k]  (rows r of the window)
  for (int i = threadIdx.x; i < SS_E * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    float a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float g = wsh[k];
      a0 += g * cs[0][r][c + SS_K - 1 - k];
      a1 += g * cs[1][r][c + SS_K - 1 - k];
      a2 += g * cs[2][r][c + SS_K - 1 - k];
    }
    vb[0][c][r] = a0; vb[1][c][r] = a1; vb[2][c][r] = a2;
  }
  __syncthreads();
  const float g = (gout ? gout[0] : 1.f) * gcoef * s.a;
  const float* rp = s.real + (long)plane * s.H * s.W;
  const float* fp = s.fake + (long)plane * s.H * s.W;
  float* dp = dfake + (long)plane * s.H * s.W;
  for (int i = threadIdx.x; i < SS_T * SS_T; i += 256) {
    const int r = i >> 5, c = i & 31;
    const int h = h0 + r, w = w0 + c;
    if (h >= s.H || w >= s.W) continue;
    float a0 = 0, a1 = 0, a2 = 0;
#pragma unroll
    for (int k = 0; k < SS_K; ++k) {
      const float gk = wsh[k];
      a0 += gk * vb[0][c][r + SS_K - 1 - k];
      a1 += gk * vb[1][c][r + SS_K - 1 - k];
      a2 += gk * vb[2][c][r + SS_K - 1 - k];
    }
    const long e = (long)h * s.W + w;
    const float X = rp[e] * s.a + s.b, Y = fp[e] * s.a + s.b;
    const float v = g * (a0 + 2.f * Y * a1 + X * a2);
    dp[e] = accumulate ? dp[e] + v : v;
  }
}


// The scalar loss combination of a training step in one launch (instead of one torch launch per
// multiply / add, pix2pix_model.py:141-151, 193-199): out = scale * (t_0 + t_1 + ... ) summed left to
// right, t_i = a_i * (b_i + c_i * x_i) with c_i in {1, -1} -- every product / sum rounded to fp32
// once, as the chain of torch scalar ops rounds it (no contraction).
constexpr int LOSS_TERMS = 8;
struct LossTerms {
  const float* x[LOSS_TERMS];
  float a[LOSS_TERMS], b[LOSS_TERMS], c[LOSS_TERMS];
  int n;
  float scale;
};
__global__ void loss_combine_kernel(LossTerms t, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < t.n; ++i) {
    const float xi = t.x[i][0];
    const float u = t.b[i] == 0.f ? (t.c[i] < 0.f ? -xi : xi) : __fadd_rn(t.b[i], t.c[i] < 0.f ? -xi : xi);
    const float v = t.a[i] == 1.f ? u : __fmul_rn(t.a[i], u);
    s = i == 0 ? v : __fadd_rn(s, v);
  }
  out[0] = t.scale == 1.f ? s : __fmul_rn(s, t.scale);
}
// gx[i] = ((gout * scale) * a_i) * c_i: the upstream grad of each term (torch's mul / rsub backward)
__global__ void loss_combine_bwd_kernel(LossTerms t, const float* __restrict__ gout, float* __restrict__ gx) {
  const int i = threadIdx.x;
  if (i >= t.n) return;
  float g = gout[0];
  if (t.scale != 1.f) g = __fmul_rn(g, t.scale);
  if (t.a[i] != 1.f) g = __fmul_rn(g, t.a[i]);
  gx[i] = t.c[i] < 0.f ? -g : g;
}
}  // namespace dsg

using namespace dsg;

extern "C" {

// out[0] = scale * sum_i a_i * (b_i + c_i * x_i[0]) (device scalars x_i; host arrays a, b, c; c_i = +-1)
int dsgan_loss_combine(const float* const* x, const float* a, const float* b, const float* c, int n, float scale,
                       float* out, hipStream_t st) {
  DSG_REQUIRE(out && x && a && b && c && n >= 1 && n <= LOSS_TERMS, "dsgan_loss_combine: 1..%d terms", LOSS_TERMS);
  LossTerms t{};
  for (int i = 0; i < n; ++i) {
    DSG_REQUIRE(x[i] != nullptr && (c[i] == 1.f || c[i] == -1.f), "dsgan_loss_combine: term %d", i);
    t.x[i] = x[i]; t.a[i] = a[i]; t.b[i] = b[i]; t.c[i] = c[i];
  }
  t.n = n;
  t.scale = scale;
  hipLaunchKernelGGL(loss_combine_kernel, dim3(1), dim3(64), 0, st, t, out);
  DSG_CHECK_LAUNCH();
  return 0;
}
// gx[i] = gout[0] * scale * a_i * c_i (n floats), each product rounded in that order
int dsgan_loss_combine_bwd(const float* gout, const float* a, const float* c, int n, float scale, float* gx,
                           hipStream_t st) {
  DSG_REQUIRE(gout && gx && a && c && n >= 1 && n <= LOSS_TERMS, "dsgan_loss_combine_bwd: bad args");
  LossTerms t{};
  for (int i = 0; i < n; ++i) { t.a[i] = a[i]; t.c[i] = c[i]; }
  t.n = n;
  t.scale = scale;
  hipLaunchKernelGGL(loss_combine_bwd_kernel, dim3(1), dim3(64), 0, st, t, gout, gx);
  DSG_CHECK_LAUNCH();
  return 0;
}

// scratch floats the loss reductions below need for their block partials
long dsgan_loss_parts(void) { return 4096; }

int dsgan_bce_logits_fwd(const float* x, long n, float target, float* out, float* part, hipStream_t st) {
  DSG_REQUIRE(x && out && part && n > 0, "dsgan_bce_logits_fwd: bad args");
  const unsigned g = red_grid(n);
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(g), dim3(256), 0, st, x, n, target, part, 1.f);
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, (int)g, 1.f / (float)n, out);
  DSG_CHECK_LAUNCH();
  return 0;
}
int dsgan_bce_logits_bwd(const float* x, long n, float target, const float* gout, float* dx,
                         int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(red_grid(n) * 8), dim3(256), 0, st, x, n, target, gout, 1.f / (float)n, dx, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}
int dsgan_l1_fwd(const float* a, const float* b, long n, float* out, float* part, hipStream_t st) {
  DSG_REQUIRE(a && b && out && part && n > 0, "dsgan_l1_fwd: bad args");
  long g;
  if ((((uintptr_t)a | (uintptr_t)b) & 15) == 0) {
    const long n4 = n / 4;
    g = (n4 + 511) / 512;
    if (g > 2048) g = 2048;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(l1_fwd_v4_kernel, dim3((unsigned)g), dim3(256), 0, st, (const float4*)a, (const float4*)b, n4,
                       a + n4 * 4, b + n4 * 4, (int)(n - n4 * 4), part, 1.f);
  } else {
    g = red_grid(n);
    hipLaunchKernelGGL(l1_fwd_kernel, dim3((unsigned)g), dim3(256), 0, st, a, b, n, part, 1.f);
  }
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, (int)g, 1.f / (float)n, out);
  DSG_CHECK_LAUNCH();
  return 0;
}
int dsgan_l1_bwd(const float* a, const float* b, long n, const float* gout, float* da,
                 int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(l1_bwd_kernel, dim3(red_grid(n) * 8), dim3(256), 0, st, a, b, n, gout, 1.f / (float)n, da, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}
// dx = (maxpool_bwd(dpool, idx) [dpool != NULL] + gout*sign(y - r)/n) * (y > 0), n = planes*H*W
int dsgan_vgg_tap_bwd(const float* dpool, const int* idx, const float* y, const float* r, float* dx, long planes,
                      int H, int W, const float* gout, hipStream_t st) {
  DSG_REQUIRE(y && r && dx && gout && planes > 0 && H > 0 && W > 0, "dsgan_vgg_tap_bwd: bad args");
  const long n = planes * H * W;
  const float coef = 1.f / (float)n;
  if (dpool) {
    DSG_REQUIRE(idx && H % 2 == 0 && W % 2 == 0, "dsgan_vgg_tap_bwd: pool needs idx and even H, W");
    const long np = n / 4;
    long blocks = (np + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(vgg_tap_bwd_pool_kernel, dim3((unsigned)blocks), dim3(256), 0, st, dpool, idx, y, r, np, H, W,
                       gout, coef, dx);
  } else {
    DSG_REQUIRE(n % 4 == 0, "dsgan_vgg_tap_bwd: top tap needs numel % 4 == 0");
    long blocks = (n / 4 + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(vgg_tap_bwd_top_kernel, dim3((unsigned)blocks), dim3(256), 0, st, y, r, n / 4, gout, coef, dx);
  }
  DSG_CHECK_LAUNCH();
  return 0;
}
int dsgan_tv_fwd(const float* y, long planes, int H, int W, float coef, float* out, float* part, hipStream_t st) {
  DSG_REQUIRE(y && out && part && planes > 0, "dsgan_tv_fwd: bad args");
  const unsigned g = red_grid(planes * H * W);
  hipLaunchKernelGGL(tv_fwd_kernel, dim3(g), dim3(256), 0, st, y, planes, H, W, part, 1.f);
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, (int)g, coef, out);
  DSG_CHECK_LAUNCH();
  return 0;
}
int dsgan_tv_bwd(const float* y, long planes, int H, int W, float coef, const float* gout, float* dy,
                 int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(tv_bwd_kernel, dim3(red_grid(planes * H * W) * 8), dim3(256), 0, st, y, planes, H, W, gout, coef, dy, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}

// acc[3] (device, float) += {ssim, psnr, 1} of one [C][H][W] image pair in [-1, 1] (see
// img_metrics_kernel); part: 2*64 doubles of scratch.
int dsgan_img_metrics(const float* fake, const float* real, int C, int H, int W, double* part, float* acc,
                      hipStream_t st) {
  DSG_REQUIRE(fake && real && part && acc && C > 0 && H > 6 && W > 6, "dsgan_img_metrics: bad args (H, W > 6)");
  hipLaunchKernelGGL(img_metrics_kernel, dim3(64), dim3(256), 0, st, fake, real, C, H, W, part);
  hipLaunchKernelGGL(img_metrics_final_kernel, dim3(1), dim3(64), 0, st, part, 64, C, H, W, acc);
  DSG_CHECK_LAUNCH();
  return 0;
}

static inline int ms_half(int h) { return (h + 2 * (h % 2) - 2) / 2 + 1; }

// per-(plane, tile) partials of the first (largest) scale: the fixed-order plane sums
static long ms_tile_parts(long planes, int H, int W) {
  return planes * cdiv(H - SS_K + 1, SS_T) * cdiv(W - SS_K + 1, SS_T) * 2;
}

// floats of `work` dsgan_ms_ssim needs: the two largest pyramid levels of X and Y (ping-pong),
// then the tile partials
long dsgan_ms_ssim_workspace(int N, int C, int H, int W) {
  const long p = (long)N * C;
  const int h1 = ms_half(H), w1 = ms_half(W), h2 = ms_half(h1), w2 = ms_half(w1);
  return 2 * p * ((long)h1 * w1 + (long)h2 * w2) + ms_tile_parts(p, H, W);
}

// MS-SSIM of (a*real+b, a*fake+b): levels = number of weights (host array, <= 8), each scale
// but the last followed by the padded 2x2 average pool (the affine map is applied inside the
// first pool, before the zero padding, as the reference maps before calling ms_ssim).
// out[n] per image (size_average=False), out[N] the batch mean (size_average=True).
int dsgan_ms_ssim(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                  const float* win11, float C1, float C2, const float* weights_host, int levels, float* work,
                  long work_elems, float* stats, float* out, hipStream_t st) {
  DSG_REQUIRE(real && fake && win11 && weights_host && stats && out && N > 0 && C > 0 && levels >= 1 &&
                  levels <= 8 && N * C <= 65535,
              "dsgan_ms_ssim: bad args");
  DSG_REQUIRE(((H < W ? H : W) > (SS_K - 1) * (1 << (levels - 1))),
              "dsgan_ms_ssim: image smaller than the (win_size-1)*2^(levels-1) ms-ssim minimum");
  DSG_WS(dsgan_ms_ssim_workspace(N, C, H, W), work, work_elems, "dsgan_ms_ssim (dsgan_ms_ssim_workspace)");
  const int planes = N * C;
  MsArgs m{};
  const float* xr = real;
  const float* yr = fake;
  float ca = a, cb = b;
  const long big = 2L * planes * ms_half(H) * ms_half(W);
  float* bufs[2] = {work, work + big};
  const int h1 = ms_half(H), w1 = ms_half(W);
  float* tparts = work + 2L * planes * ((long)h1 * w1 + (long)ms_half(h1) * ms_half(w1));
  int h = H, w = W;
  for (int l = 0; l < levels; ++l) {
    const int Ho = h - SS_K + 1, Wo = w - SS_K + 1;
    SSIMArgs s{xr, yr, ca, cb, planes, h, w, win11, C1, C2, nullptr, nullptr, nullptr, 0};
    const int tw = cdiv(Wo, SS_T), th = cdiv(Ho, SS_T);
    hipLaunchKernelGGL(ssim_eval_kernel, dim3(tw * th, planes), dim3(256), 0, st, s, tw, tparts);
    hipLaunchKernelGGL(plane_tile_sum_kernel, dim3(cdiv(2 * planes, 256)), dim3(256), 0, st, tparts, planes, tw * th,
                       stats + (long)l * planes * 2);
    m.inv_cnt[l] = 1.f / ((float)Ho * (float)Wo);
    m.wt[l] = weights_host[l];
    if (l < levels - 1) {
      const int h2 = ms_half(h), w2 = ms_half(w);
      float* nx = bufs[l & 1];
      float* ny = nx + (long)planes * h2 * w2;
      const long n2 = (long)planes * h2 * w2;
      hipLaunchKernelGGL(avgpool2_pad_kernel, dim3(red_grid(n2)), dim3(256), 0, st, xr, nx, planes, h, w, h2, w2,
                         h % 2, w % 2, ca, cb);
      hipLaunchKernelGGL(avgpool2_pad_kernel, dim3(red_grid(n2)), dim3(256), 0, st, yr, ny, planes, h, w, h2, w2,
                         h % 2, w % 2, ca, cb);
      xr = nx; yr = ny; h = h2; w = w2; ca = 1.f; cb = 0.f;
    }
  }
  hipLaunchKernelGGL(ms_ssim_combine_kernel, dim3(1), dim3(256), 0, st, stats, levels, N, C, m, out);
  DSG_CHECK_LAUNCH();
  return 0;
}

// ---- MS-SSIM loss (forward keeping the pyramid, backward) ------------------------------------
// work layout (floats): X_1, Y_1, X_2, Y_2, ... X_{L-1}, Y_{L-1} (each planes*h_l*w_l), then two
// dY ping-pong buffers of level-1 size, then the kscale table [L][planes], then the coefficient
// maps [3][planes][Ho_0][Wo_0].
static void ms_dims(int H, int W, int levels, int* hs, int* ws) {
  hs[0] = H; ws[0] = W;
  for (int l = 1; l < levels; ++l) { hs[l] = ms_half(hs[l - 1]); ws[l] = ms_half(ws[l - 1]); }
}
long dsgan_ms_ssim_train_workspace(int N, int C, int H, int W, int levels) {
  if (levels < 1 || levels > 8) return -1;
  int hs[8], ws[8];
  ms_dims(H, W, levels, hs, ws);
  const long p = (long)N * C;
  long n = 0;
  for (int l = 1; l < levels; ++l) n += 2 * p * hs[l] * ws[l];
  if (levels > 1) n += 2 * p * hs[1] * ws[1];
  n += (long)levels * p;
  n += 3 * p * (long)(H - SS_K + 1) * (W - SS_K + 1);
  n += ms_tile_parts(p, H, W);
  return n;
}

static MsArgs ms_args(int levels, const int* hs, const int* ws, const float* weights_host) {
  MsArgs m{};
  for (int l = 0; l < levels; ++l) {
    m.inv_cnt[l] = 1.f / ((float)(hs[l] - SS_K + 1) * (float)(ws[l] - SS_K + 1));
    m.wt[l] = weights_host[l];
  }
  return m;
}

// Same value as dsgan_ms_ssim (out[N] = batch mean, out[n] per image), keeping every pyramid
// level in `work` for dsgan_ms_ssim_bwd.  stats: [levels][planes][2] map sums.
int dsgan_ms_ssim_fwd_train(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                            const float* win11, float C1, float C2, const float* weights_host, int levels, float* work,
                            long work_elems, float* stats, float* out, hipStream_t st) {
  DSG_REQUIRE(real && fake && win11 && weights_host && stats && out && N > 0 && C > 0 && levels >= 1 &&
                  levels <= 8 && N * C <= 65535,
              "dsgan_ms_ssim_fwd_train: bad args");
  DSG_REQUIRE(((H < W ? H : W) > (SS_K - 1) * (1 << (levels - 1))),
              "dsgan_ms_ssim_fwd_train: image smaller than the (win_size-1)*2^(levels-1) ms-ssim minimum");
  DSG_WS(dsgan_ms_ssim_train_workspace(N, C, H, W, levels), work, work_elems,
         "dsgan_ms_ssim_fwd_train (dsgan_ms_ssim_train_workspace)");
  const int planes = N * C;
  int hs[8], ws[8];
  ms_dims(H, W, levels, hs, ws);
  const float* xr = real;
  const float* yr = fake;
  float ca = a, cb = b;
  float* lvl = work;
  // tile partials live at the end of the workspace (layout of dsgan_ms_ssim_train_workspace)
  float* tparts = work + dsgan_ms_ssim_train_workspace(N, C, H, W, levels) - ms_tile_parts(planes, H, W);
  for (int l = 0; l < levels; ++l) {
    const int h = hs[l], w = ws[l];
    const int Ho = h - SS_K + 1, Wo = w - SS_K + 1;
    SSIMArgs s{xr, yr, ca, cb, planes, h, w, win11, C1, C2, nullptr, nullptr, nullptr, 0};
    const int tw = cdiv(Wo, SS_T), th = cdiv(Ho, SS_T);
    hipLaunchKernelGGL(ssim_eval_kernel, dim3(tw * th, planes), dim3(256), 0, st, s, tw, tparts);
    hipLaunchKernelGGL(plane_tile_sum_kernel, dim3(cdiv(2 * planes, 256)), dim3(256), 0, st, tparts, planes, tw * th,
                       stats + (long)l * planes * 2);
    if (l < levels - 1) {
      const int h2 = hs[l + 1], w2 = ws[l + 1];
      const long n2 = (long)planes * h2 * w2;
      float* nx = lvl;
      float* ny = lvl + n2;
      hipLaunchKernelGGL(avgpool2_pad_kernel, dim3(red_grid(n2)), dim3(256), 0, st, xr, nx, planes, h, w, h2, w2,
                         h % 2, w % 2, ca, cb);
      hipLaunchKernelGGL(avgpool2_pad_kernel, dim3(red_grid(n2)), dim3(256), 0, st, yr, ny, planes, h, w, h2, w2,
                         h % 2, w % 2, ca, cb);
      xr = nx; yr = ny; ca = 1.f; cb = 0.f;
      lvl += 2 * n2;
    }
  }
  hipLaunchKernelGGL(ms_ssim_combine_kernel, dim3(1), dim3(256), 0, st, stats, levels, N, C,
                     ms_args(levels, hs, ws, weights_host), out);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dfake (+)= d(gout[0] * batch-mean MS-SSIM)/d(fake); work/stats as left by dsgan_ms_ssim_fwd_train.
int dsgan_ms_ssim_bwd(const float* real, const float* fake, float a, float b, int N, int C, int H, int W,
                      const float* win11, float C1, float C2, const float* weights_host, int levels, float* work,
                      long work_elems, const float* stats, const float* gout, float* dfake, int accumulate,
                      hipStream_t st) {
  DSG_REQUIRE(real && fake && win11 && weights_host && stats && gout && dfake && N > 0 && C > 0 &&
                  levels >= 1 && levels <= 8 && N * C <= 65535,
              "dsgan_ms_ssim_bwd: bad args");
  DSG_WS(dsgan_ms_ssim_train_workspace(N, C, H, W, levels), work, work_elems,
         "dsgan_ms_ssim_bwd (dsgan_ms_ssim_train_workspace)");
  DSG_REQUIRE(!accumulate || levels == 1, "dsgan_ms_ssim_bwd: accumulate needs levels == 1 (dfake is staged)");
  const int planes = N * C;
  int hs[8], ws[8];
  ms_dims(H, W, levels, hs, ws);
  const float* xs[8];
  const float* ys[8];
  xs[0] = real; ys[0] = fake;
  float* lvl = work;
  for (int l = 1; l < levels; ++l) {
    const long n = (long)planes * hs[l] * ws[l];
    xs[l] = lvl; ys[l] = lvl + n;
    lvl += 2 * n;
  }
  float* dbuf[2] = {lvl, levels > 1 ? lvl + (long)planes * hs[1] * ws[1] : lvl};
  if (levels > 1) lvl += 2L * planes * hs[1] * ws[1];
  float* kscale = lvl;
  lvl += (long)levels * planes;
  float* coef = lvl;
  const MsArgs m = ms_args(levels, hs, ws, weights_host);
  hipLaunchKernelGGL(ms_ssim_kscale_kernel, dim3(cdiv(planes, 256)), dim3(256), 0, st, stats, levels, planes, m, gout,
                     1.f / (float)planes, kscale);
  const float* dup = nullptr;
  for (int l = levels - 1; l >= 0; --l) {
    const int h = hs[l], w = ws[l];
    const int Ho = h - SS_K + 1, Wo = w - SS_K + 1;
    float* dy = l == 0 ? dfake : dbuf[l & 1];
    const float sa = l == 0 ? a : 1.f, sb = l == 0 ? b : 0.f;
    int acc = 0;
    if (dup) {   // 1/4 of the level above through the padded pool (times a at the image level)
      const long n = (long)planes * h * w;
      hipLaunchKernelGGL(avgpool2_pad_bwd_kernel, dim3(red_grid(n)), dim3(256), 0, st, dup, dy, planes, h, w, hs[l + 1],
                         ws[l + 1], h % 2, w % 2, 0.25f * sa);
      acc = 1;
    } else {
      acc = l == 0 ? accumulate : 0;
    }
    SSIMArgs s{xs[l], ys[l], sa, sb, planes, h, w, win11, C1, C2, coef, nullptr, kscale + (long)l * planes,
               l < levels - 1 ? 1 : 0};
    const int tw = cdiv(Wo, SS_T), th = cdiv(Ho, SS_T);
    hipLaunchKernelGGL(ssim_fwd_kernel, dim3(tw * th, planes), dim3(256), 0, st, s, tw);
    const int tw2 = cdiv(w, SS_T), th2 = cdiv(h, SS_T);
    hipLaunchKernelGGL(ssim_bwd_kernel, dim3(tw2 * th2, planes), dim3(256), 0, st, s, (const float*)nullptr, 1.f, dy,
                       tw2, acc);
    dup = dy;
  }
  DSG_CHECK_LAUNCH();
  return 0;
}

// out = sum of the SSIM map (caller divides by planes*Ho*Wo); coef: [3][planes][Ho][Wo] scratch
// tile partials dsgan_ssim_fwd needs (one per 32x32 output tile and plane)
long dsgan_ssim_parts(int planes, int H, int W) {
  return (long)planes * cdiv(H - SS_K + 1, SS_T) * cdiv(W - SS_K + 1, SS_T);
}

int dsgan_ssim_fwd(const float* real, const float* fake, float a, float b, int planes, int H, int W,
                   const float* win11, float C1, float C2, float* coef, float* out, float* part, hipStream_t st) {
  DSG_REQUIRE(real && fake && win11 && coef && out && part && H >= SS_K && W >= SS_K && planes > 0 && planes <= 65535,
              "dsgan_ssim_fwd: bad args (H,W >= 11 required)");
  SSIMArgs s{real, fake, a, b, planes, H, W, win11, C1, C2, coef, part, nullptr, 0};
  const int Ho = H - SS_K + 1, Wo = W - SS_K + 1;
  const int tw = cdiv(Wo, SS_T), th = cdiv(Ho, SS_T);
  hipLaunchKernelGGL(ssim_fwd_kernel, dim3(tw * th, planes), dim3(256), 0, st, s, tw);
  hipLaunchKernelGGL(final_sum_kernel, dim3(1), dim3(256), 0, st, part, tw * th * planes, 1.f, out);
  DSG_CHECK_LAUNCH();
  return 0;
}

// dfake = gout[0] * gcoef * d(sum S)/d(fake)
int dsgan_ssim_bwd(const float* real, const float* fake, float a, float b, int planes, int H, int W,
                   const float* win11, const float* coef, const float* gout, float gcoef,
                   float* dfake, int accumulate, hipStream_t st) {
  DSG_REQUIRE(real && fake && win11 && coef && gout && dfake, "dsgan_ssim_bwd: bad args");
  SSIMArgs s{real, fake, a, b, planes, H, W, win11, 0.f, 0.f, const_cast<float*>(coef), nullptr, nullptr, 0};
  const int tw = cdiv(W, SS_T), th = cdiv(H, SS_T);
  hipLaunchKernelGGL(ssim_bwd_kernel, dim3(tw * th, planes), dim3(256), 0, st, s, gout, gcoef, dfake, tw, accumulate);
  DSG_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
