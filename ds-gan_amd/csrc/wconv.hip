// Patch-staged weight-gradient of KxK, pad-1 convolutions (gfx950, bf16 MFMA, fp32 accumulate).
//
//   dW[m][c][kh][kw] += sum_{b, oh, ow} D[b][m][oh][ow] * X[b][c][oh*S - 1 + kh][ow*S - 1 + kw]
//
// Covers the weight-grads of the ConvTranspose2d 3x3/s2 layers (as the equivalent stride-2
// conv with D = ConvT input, X = ConvT output grad; DSGAN/models/model/MixConvNeXtML.py:53,149-152)
// and of the PatchGAN 4x4 s2/s1 convs (DSGAN/models/networks.py:543-569).  The reduction runs
// over N*Ho*Wo pixels into a small output; with fp32 activations these contractions are
// HBM-bound, so the kernel streams D and X once per (M, C) tile pair (the tiles of one pixel
// range are adjacent workgroups on one XCD and share the reads in L2).
//
// Workgroup = 64 m x 32 c x all T taps, over a run of pixel blocks (4 output rows x 16 columns).
// Per block:
//   * D[64 m][64 px] -> LDS bf16, row per m (float4 global loads);
//   * the 32-channel input patch -> LDS bf16 as S column-parity planes per patch row, plane p
//     holding X[c][ih0 + r][iw0 + S*j + p] (float4 global loads, paired dword LDS writes;
//     plane p is stored at element offset OFF_p so every staging write is aligned);
// MFMA 32x32x16: A = D (m x 16 px of one output row), B = X patch (16 px x c) for one tap.  Tap
// (kh, kw) of output row r reads plane kw % S of patch row S*r + kh at element shift
// kw / S + OFF: shift 0 is one aligned 16-byte LDS read, other shifts two reads and a
// v_alignbit funnel (shifts are compile-time: wave w owns taps w, w+4, ...).
// Partial sums per split -> workspace [splits][T][M][C]; launch_split_reduce_wconv (split_reduce.hip)
// sums the splits in a fixed order into dW (deterministic, no atomics; queued in deferred mode).
#include "common.h"
#include <type_traits>

namespace dsg {

typedef f32x16_t wf32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int wu32x4;

struct WcArgs {
  const float* D; long d_bs;   // conv output grad  [nb][M][Ho][Wo]
  const float* X; long x_bs;   // conv input        [nb][C][H][W]
  float* P;                    // partials          [splits][T][M][C]
  int nb, M, C, H, W, Ho, Wo;
  int nbw, nbh, nblk, bps;     // pixel blocks per row / per column / total, blocks per split
  int mt, ct;                  // M tiles (64), C tiles (32)
  int vec_d;                   // D rows float4-loadable
  float* dbp;                  // (nullable) bias-grad partials [splits][M] = sum over the split's pixels of D
};

constexpr int WC_TW = 16, WC_TH = 4;
constexpr int WC_BM = 64, WC_BC = 32;
constexpr int WC_JW = 24;      // stored elements per plane row (48 B)

template <int S> struct WcGeo;
// S = 2, pad 1: float4 q of a patch row covers t = col - iw0 = 4q-3 .. 4q; its two odd-t
// elements are plane 1, j = 2q-2, 2q-1 (stored at j); its even-t elements plane 0,
// j = 2q-1, 2q (stored at j+1).  Planes hold j = 0..16.
template <> struct WcGeo<2> {
  static constexpr int NQ = 10;
  static constexpr int OFF0 = 1, OFF1 = 0;
  __device__ static constexpr int shift(int kw) { return (kw >> 1) + ((kw & 1) ? OFF1 : OFF0); }
};
// S = 1, pad 1: one plane, t = 4q-3+e stored at t+3 = 4q+e; holds t = 0..18.
template <> struct WcGeo<1> {
  static constexpr int NQ = 6;
  __device__ static constexpr int shift(int kw) { return kw + 3; }
};

// 8 consecutive bf16 starting SH elements after the 16-byte aligned p.
template <int SH, typename T16>
__device__ __forceinline__ hx8<T16> frag_at(const T16* p) {
  typedef hx8<T16> wbf16x8;
  if constexpr (SH == 0) {
    return *reinterpret_cast<const wbf16x8*>(p);
  } else {
    const wu32x4 a = *reinterpret_cast<const wu32x4*>(p);
    const wu32x4 b = *reinterpret_cast<const wu32x4*>(p + 8);
    const unsigned d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    constexpr int q = SH >> 1;
    wu32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      r[i] = (SH & 1) ? __builtin_amdgcn_alignbit(d[q + i + 1], d[q + i], 16) : d[q + i];
    return __builtin_bit_cast(wbf16x8, r);
  }
}

// XH: X is 16-bit (the half type; the ConvTranspose backward's output grad from
// dsgan_instnorm_bwd_h): 8-byte loads of the same four columns, no conversion, half the staging
// registers.
template <typename T16, int KH, int KW, int S, bool XH = false>
__global__ __launch_bounds__(256, XH ? 2 : 1) void wconv_kernel(WcArgs g) {
  typedef hx8<T16> wbf16x8;
  typedef hx4<T16> wbf16x4;
  typedef T16 wbf16x2 __attribute__((ext_vector_type(2)));
  constexpr int T = KH * KW, NT4 = (T + 3) / 4;
  constexpr int PX = WC_TH * WC_TW;
  constexpr int PH = (WC_TH - 1) * S + KH;
  constexpr int NQ = WcGeo<S>::NQ;
  constexpr int A_STR = PX + 8;                           // bf16 per m row; /8 odd -> conflict-free b128
  static_assert(((A_STR / 8) & 1) == 1, "A row stride");
  constexpr int C_DW0 = PH * S * (WC_JW / 2);             // dwords per channel
  constexpr int C_DW = ((C_DW0 / 4) & 1) ? C_DW0 : C_DW0 + 4;
  constexpr int C_STR = C_DW * 2;                         // bf16 per channel
  constexpr int A_IT = WC_BM * PX / 4 / 256;              // float4 items per thread
  constexpr int B_ITEMS = WC_BC * PH * NQ;                // (c, patch row, float4) items
  constexpr int B_IT = (B_ITEMS + 255) / 256;
  static_assert(A_IT * 256 * 4 == WC_BM * PX, "A items");
  __shared__ __attribute__((aligned(16))) T16 As[WC_BM * A_STR];
  __shared__ __attribute__((aligned(16))) T16 Bs[WC_BC * C_STR];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;

  int tile;
  {
    const int nwg = gridDim.x, id = blockIdx.x;
    const int xcd = id & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (id >> 3);
  }
  const int ntile = g.mt * g.ct;
  const int split = tile / ntile, tmc = tile - split * ntile;
  const int m_t = tmc % g.mt, c_t = tmc / g.mt;
  const int m0 = m_t * WC_BM, c0 = c_t * WC_BC;
  const int qbeg = split * g.bps;
  const int qend = min(g.nblk, qbeg + g.bps);
  const int HWo = g.Ho * g.Wo, HW = g.H * g.W;
  const int per_img = g.nbh * g.nbw;

  float4 ra[A_IT], rb[XH ? 1 : B_IT];
  uint2 rh[XH ? B_IT : 1];
  // dbp: the c-tile-0 workgroups also sum their staged fp32 D rows (the conv's bias grad), per
  // thread in block order, then over the 16 lanes of a row (fixed order: deterministic)
  // (compiled out of the 16-bit-X ConvTranspose form, which never folds a bias: its codegen is tight)
  float asr[XH ? 1 : A_IT];
#pragma unroll
  for (int i = 0; i < (XH ? 1 : A_IT); ++i) asr[i] = 0.f;
  const bool want_db = !XH && g.dbp != nullptr && c_t == 0;

  auto load = [&](int q) __attribute__((always_inline)) {
    const int b = q / per_img, rem = q - b * per_img;
    const int oh0 = (rem / g.nbw) * WC_TH, ow0 = (rem % g.nbw) * WC_TW;
    const float* db = g.D + (long)b * g.d_bs;
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256, mm = it / (PX / 4), qq = it % (PX / 4);
      const int oh = oh0 + (qq >> 2), ow = ow0 + (qq & 3) * 4;
      float4 v = {0.f, 0.f, 0.f, 0.f};
      if (m0 + mm < g.M && oh < g.Ho) {
        const float* src = db + (long)(m0 + mm) * HWo + (long)oh * g.Wo + ow;
        if (g.vec_d && ow + 3 < g.Wo) {
          v = *reinterpret_cast<const float4*>(src);
        } else {
          if (ow < g.Wo) v.x = src[0];
          if (ow + 1 < g.Wo) v.y = src[1];
          if (ow + 2 < g.Wo) v.z = src[2];
          if (ow + 3 < g.Wo) v.w = src[3];
        }
      }
      ra[i] = v;
    }
    // input patch rows: float4 q covers cols a0 + 4q .. a0 + 4q + 3, a0 = iw0 - 3 (16-byte aligned)
    const int ih0 = oh0 * S - 1, a0 = ow0 * S - 4;
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + i * 256;
      const int q4 = it % NQ, rest = it / NQ;
      const int pr = rest % PH, c = rest / PH;
      const int ih = ih0 + pr, col = a0 + 4 * q4;
      const bool ok = it < B_ITEMS && (unsigned)ih < (unsigned)g.H && (unsigned)col < (unsigned)g.W;
      const long e = (long)b * g.x_bs + (long)(c0 + c) * HW + (long)ih * g.W + col;
      if constexpr (XH) {
        uint2 v = {0u, 0u};
        if (ok) v = *reinterpret_cast<const uint2*>(reinterpret_cast<const unsigned short*>(g.X) + e);
        rh[i] = v;
      } else {
        float4 v = {0.f, 0.f, 0.f, 0.f};
        if (ok) v = *reinterpret_cast<const float4*>(g.X + e);
        rb[i] = v;
      }
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      const int it = tid + i * 256, mm = it / (PX / 4), qq = it % (PX / 4);
      const wbf16x4 v = {(T16)ra[i].x, (T16)ra[i].y, (T16)ra[i].z, (T16)ra[i].w};
      *reinterpret_cast<wbf16x4*>(As + mm * A_STR + qq * 4) = v;
      if constexpr (!XH)
        if (want_db) asr[i] += (ra[i].x + ra[i].y) + (ra[i].z + ra[i].w);
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int it = tid + i * 256;
      if (it < B_ITEMS) {
        const int q4 = it % NQ, rest = it / NQ;
        const int pr = rest % PH, c = rest / PH;
        T16* row = Bs + c * C_STR + pr * (S * WC_JW);
        if constexpr (XH) {   // elements e0..e3 = u.x lo, u.x hi, u.y lo, u.y hi
          const uint2 u = rh[i];
          if constexpr (S == 2) {
            if (q4 > 0) *reinterpret_cast<unsigned*>(row + WC_JW + 2 * q4 - 2) = (u.x & 0xffffu) | (u.y << 16);
            *reinterpret_cast<unsigned*>(row + 2 * q4) = (u.x >> 16) | (u.y & 0xffff0000u);
          } else {
            *reinterpret_cast<uint2*>(row + 4 * q4) = u;
          }
        } else if constexpr (S == 2) {
          // plane 1 <- (x, z) at j = 2q-2 (skip q = 0: j < 0); plane 0 <- (y, w) stored at 2q
          if (q4 > 0) *reinterpret_cast<wbf16x2*>(row + WC_JW + 2 * q4 - 2) = wbf16x2{(T16)rb[i].x, (T16)rb[i].z};
          *reinterpret_cast<wbf16x2*>(row + 2 * q4) = wbf16x2{(T16)rb[i].y, (T16)rb[i].w};
        } else {
          *reinterpret_cast<wbf16x4*>(row + 4 * q4) =
              wbf16x4{(T16)rb[i].x, (T16)rb[i].y, (T16)rb[i].z, (T16)rb[i].w};
        }
      }
    }
  };

  // Each wave runs its own instantiation of the block loop: wave WV owns taps WV, WV+4, ...,
  // so every tap's plane and shift are compile-time (the barriers are reached by all four
  // waves once per block in every instantiation).
  auto run = [&](auto wtag) __attribute__((always_inline)) {
    constexpr int WV = decltype(wtag)::value;
    wf32x16 acc[2][NT4];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < NT4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[s][i][r] = 0.f;

    if (qbeg < qend) load(qbeg);
    for (int q = qbeg; q < qend; ++q) {
      __syncthreads();   // LDS free (previous block consumed)
      store();
      __syncthreads();
      if (q + 1 < qend) load(q + 1);
#pragma unroll
      for (int r = 0; r < WC_TH; ++r) {
        const wbf16x8 a0 = *reinterpret_cast<const wbf16x8*>(As + lr * A_STR + r * 16 + lh * 8);
        const wbf16x8 a1 = *reinterpret_cast<const wbf16x8*>(As + (32 + lr) * A_STR + r * 16 + lh * 8);
#pragma unroll
        for (int i = 0; i < NT4; ++i) {
          if (WV + 4 * i < T) {
            const int t = WV + 4 * i, kh = t / KW, kw = t % KW;
            const T16* row = Bs + lr * C_STR + (S * r + kh) * (S * WC_JW) + (kw % S) * WC_JW + lh * 8;
            wbf16x8 bf;
            switch (WcGeo<S>::shift(kw)) {   // folds: t, kw are compile-time after unrolling
              case 0: bf = frag_at<0>(row); break;
              case 1: bf = frag_at<1>(row); break;
              case 2: bf = frag_at<2>(row); break;
              case 3: bf = frag_at<3>(row); break;
              case 4: bf = frag_at<4>(row); break;
              case 5: bf = frag_at<5>(row); break;
              default: bf = frag_at<6>(row); break;
            }
            acc[0][i] = mfma16(a0, bf, acc[0][i]);
            acc[1][i] = mfma16(a1, bf, acc[1][i]);
          }
        }
      }
    }

    // partials: P[split][t][m][c], lanes along c (coalesced)
    const int c = c0 + lr;
#pragma unroll
    for (int i = 0; i < NT4; ++i) {
      const int t = WV + 4 * i;
      if (t < T) {
        float* pt = g.P + ((long)split * T + t) * g.M * g.C;
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + s * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
            if (m < g.M) pt[(long)m * g.C + c] = acc[s][i][r];
          }
      }
    }
    if constexpr (!XH) if (want_db) {
      static_assert(PX / 4 == 16, "a D row is 16 consecutive items");
#pragma unroll
      for (int i = 0; i < A_IT; ++i) {
        float t = asr[i];
        t += __shfl_xor(t, 1, 64); t += __shfl_xor(t, 2, 64); t += __shfl_xor(t, 4, 64); t += __shfl_xor(t, 8, 64);
        const int it = tid + i * 256, m = m0 + it / (PX / 4);
        if ((it & 15) == 0 && m < g.M) g.dbp[(long)split * g.M + m] = t;
      }
    }
  };
  switch (wave) {
    case 0: run(std::integral_constant<int, 0>{}); break;
    case 1: run(std::integral_constant<int, 1>{}); break;
    case 2: run(std::integral_constant<int, 2>{}); break;
    default: run(std::integral_constant<int, 3>{}); break;
  }
}

// fp32 X: one resident workgroup per CU (next block prefetched into registers); 16-bit X (half the
// staging registers): two, so one workgroup's MFMAs cover the other's block loads.
constexpr int WC_TARGET_WG = 256, WC_TARGET_WG_XH = 512;

struct WcPlan { int nbw, nbh, nblk, mt, ct, splits, bps; };

static WcPlan wc_plan(int nb, int C, int M, int Ho, int Wo, int target = WC_TARGET_WG) {
  WcPlan p;
  p.nbw = (Wo + WC_TW - 1) / WC_TW;
  p.nbh = (Ho + WC_TH - 1) / WC_TH;
  p.nblk = nb * p.nbw * p.nbh;
  p.mt = (M + WC_BM - 1) / WC_BM;
  p.ct = C / WC_BC;
  const int tiles = p.mt * p.ct;
  int splits = (target + tiles - 1) / tiles;
  if (splits > p.nblk) splits = p.nblk;
  if (splits < 1) splits = 1;
  p.bps = (p.nblk + splits - 1) / splits;
  p.splits = (p.nblk + p.bps - 1) / p.bps;   // no empty splits
  return p;
}

template <typename T16, int K, int S>
static void wc_launch(WcArgs& g, int grid, bool xh, hipStream_t st) {
  if constexpr (K == 3 && S == 2) {   // 16-bit X: the ConvTranspose 3x3/s2 weight-grads only
    if (xh) { hipLaunchKernelGGL((wconv_kernel<T16, K, K, S, true>), dim3((unsigned)grid), dim3(256), 0, st, g); return; }
  }
  hipLaunchKernelGGL((wconv_kernel<T16, K, K, S>), dim3((unsigned)grid), dim3(256), 0, st, g);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

int dsgan_wconv_supported(int C, int KH, int KW, int stride) {
  if (C <= 0 || C % WC_BC != 0 || KH != KW) return 0;
  return (KH == 3 || KH == 4) && (stride == 1 || stride == 2);
}

// fp32 workspace elements dsgan_wconv needs for this problem
long dsgan_wconv_workspace(int nb, int C, int M, int Ho, int Wo, int KH, int KW) {
  // (enough for either form: the 16-bit-X launches plan for twice the workgroups)
  const WcPlan p = wc_plan(nb, C, M, Ho, Wo), q = wc_plan(nb, C, M, Ho, Wo, WC_TARGET_WG_XH);
  // (+ splits * M: the bias-grad partials of dsgan_wconv_db)
  return (long)(p.splits > q.splits ? p.splits : q.splits) * ((long)KH * KW * M * C + M);
}

// dw[M][C][KH][KW] += weight-grad of y = conv(x, w, stride, pad = 1): D = dy [nb][M][Ho][Wo],
// X = x [nb][C][H][W] (batch strides d_bs / x_bs; X 16-byte aligned rows: W % 4 == 0);
// ws: dsgan_wconv_workspace() floats.
}  // extern "C"

static int wconv_impl(const float* D, long d_bs, const void* X, long x_bs, bool xh, float* dw, float* db, float* ws,
                      long ws_elems, int nb, int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride,
                      int pad, hipStream_t st) {
  DSG_REQUIRE(D && X && dw && nb > 0 && M > 0 && Ho > 0 && Wo > 0, "dsgan_wconv: bad args");
  DSG_REQUIRE(dsgan_wconv_supported(C, KH, KW, stride) && pad == 1, "dsgan_wconv: unsupported C=%d K=%dx%d stride=%d pad=%d",
              C, KH, KW, stride, pad);
  DSG_REQUIRE(W % 4 == 0 && x_bs % 4 == 0 && ((uintptr_t)X & (xh ? 7 : 15)) == 0,
              "dsgan_wconv: X rows must be 4-element aligned");
  DSG_REQUIRE((Ho - 1) * stride - pad + KH <= H + pad && (Wo - 1) * stride - pad + KW <= W + pad,
              "dsgan_wconv: output size inconsistent with input/pad");
  DSG_REQUIRE(!xh || (KH == 3 && stride == 2), "dsgan_wconv_xh: 3x3 stride-2 only");
  const WcPlan p = wc_plan(nb, C, M, Ho, Wo, xh ? WC_TARGET_WG_XH : WC_TARGET_WG);
  // weight partials [splits][T][M][C], then (db) the bias partials [splits][M]
  DSG_WS((long)p.splits * ((long)KH * KW * M * C + (db ? M : 0)), ws, ws_elems, "dsgan_wconv (dsgan_wconv_workspace)");
  WcArgs g{};
  g.D = D; g.d_bs = d_bs; g.X = (const float*)X; g.x_bs = x_bs; g.P = ws;
  g.nb = nb; g.M = M; g.C = C; g.H = H; g.W = W; g.Ho = Ho; g.Wo = Wo;
  g.nbw = p.nbw; g.nbh = p.nbh; g.nblk = p.nblk; g.bps = p.bps; g.mt = p.mt; g.ct = p.ct;
  g.vec_d = ((uintptr_t)D % 16 == 0) && (d_bs % 4 == 0) && (Wo % 4 == 0);
  g.dbp = db ? ws + (long)p.splits * KH * KW * M * C : nullptr;
  const int grid = p.splits * p.mt * p.ct;
  with_half([&](auto* t_) {
    using T16 = std::remove_pointer_t<decltype(t_)>;
    if (KH == 3 && stride == 2) wc_launch<T16, 3, 2>(g, grid, xh, st);
    else if (KH == 3 && stride == 1) wc_launch<T16, 3, 1>(g, grid, xh, st);
    else if (KH == 4 && stride == 2) wc_launch<T16, 4, 2>(g, grid, xh, st);
    else wc_launch<T16, 4, 1>(g, grid, xh, st);
  });
  DSG_CHECK_LAUNCH();
  // dw[m][c][t] += sum_s P[s][t][m][c] in a fixed order (split_reduce.hip; queued in deferred mode)
  launch_split_reduce_wconv(ws, p.splits, KH * KW, M, C, dw, st);
  if (db) launch_split_reduce(g.dbp, p.splits, M, db, st);
  DSG_CHECK_LAUNCH();
  return 0;
}

extern "C" {

int dsgan_wconv(const float* D, long d_bs, const float* X, long x_bs, float* dw, float* ws, long ws_elems, int nb, int C,
                int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride, int pad, hipStream_t st) {
  return wconv_impl(D, d_bs, X, x_bs, false, dw, nullptr, ws, ws_elems, nb, C, M, H, W, Ho, Wo, KH, KW, stride, pad, st);
}

// Same, plus the conv's bias grad db[m] += sum_{b, oh, ow} D[b][m][oh][ow] from the staged D tiles
// (fp32 values, fixed order) -- no separate channel-sum pass over D.
int dsgan_wconv_db(const float* D, long d_bs, const float* X, long x_bs, float* dw, float* db, float* ws, long ws_elems,
                   int nb, int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride, int pad,
                   hipStream_t st) {
  DSG_REQUIRE(db, "dsgan_wconv_db: db is NULL");
  return wconv_impl(D, d_bs, X, x_bs, false, dw, db, ws, ws_elems, nb, C, M, H, W, Ho, Wo, KH, KW, stride, pad, st);
}

// Same with X in the library's 16-bit half type (x_bs in elements; rows 8-byte aligned): the
// ConvTranspose weight-grad on dsgan_instnorm_bwd_h's output.
int dsgan_wconv_xh(const float* D, long d_bs, const void* Xh, long x_bs, float* dw, float* ws, long ws_elems, int nb,
                   int C, int M, int H, int W, int Ho, int Wo, int KH, int KW, int stride, int pad, hipStream_t st) {
  return wconv_impl(D, d_bs, Xh, x_bs, true, dw, nullptr, ws, ws_elems, nb, C, M, H, W, Ho, Wo, KH, KW, stride, pad, st);
}

}  // extern "C"
