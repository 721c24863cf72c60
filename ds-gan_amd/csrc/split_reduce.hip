// Split partial reductions of every weight-grad of the library (pwgemm, pwf32, igemm, skinny, thin3,
// dwconv, MLP, channel attention, channel sums, PatchGAN stem / head, wconv's bias partials):
//   dw[e] += sum_s ws[s][e],  s = 0 .. S-1, in ONE fixed order (deterministic, no atomics).
//
// The canonical order of one reduction (S splits over MN elements, row stride MN):
//   rows   : S > 64 and MN < 65536 ("many splits over few elements"): G = ceil(S / 16) groups, the
//            row of group g = ((p0 + p1) + p2) + p3 with p_j = the in-order sum of ws[s][e] over
//            s = 16g + j, 16g + j + 4, ... < min(S, 16g + 16); otherwise the S splits themselves;
//   lanes  : J = (rows <= 8) ? 4 : 16; lane q sums rows q, q + J, q + 2J, ... in order (from 0);
//   result : t = lane 0 + lane 1 + ... + lane J-1 (in order), then dw[e] += t.
// (The round-4 library ran the group sums as a separate pre-pass launch; this is the same order of
// additions in one launch: a workgroup lane computes its groups' sums from the partials directly.)
// KK1 > 0 (depthwise / stem / head weight + bias vectors): element e = (c, i), i < KK1, goes to
// dw[c * (KK1 - 1) + i] for i < KK1 - 1 and to db[c] for i == KK1 - 1.
//
// Deferred mode (dsgan_split_defer): the weight-grad launchers then queue their reductions instead
// of launching them, and dsgan_split_flush issues the whole queue as a few multi-segment launches
// (segments whose outputs overlap go to different launches, in queue order).  The training step
// runs each backward pass deferred and flushes at its end (and before every DDP bucket hook), so
// ~160 small reduction launches per step become a handful; the caller keeps every queued scratch
// buffer and output alive until the flush (dsgan_hip/functional.py: wsa / deferred_splits).
#include <mutex>
#include "common.h"

#include <stdlib.h>

#include <type_traits>
#include <vector>

namespace dsg {

struct RSeg {
  const float* ws;
  float* dw;
  float* db;
  long MN;
  int S, KK1, form, b0;   // form: bit 0 = 16 lanes (else 4), bit 1 = float4 elements, bit 2 = group rows,
                          //       bit 3 = wconv layout (bit 4: 4 rows m per workgroup, else 1)
  int T, M, C;            // wconv layout: partials [S][T][M][C] -> dw [M][C][T]
};
constexpr int RS_MAX = 20;
struct RSegs { RSeg s[RS_MAX]; int n; };

template <typename V> __device__ __forceinline__ V rz();
template <> __device__ __forceinline__ float rz<float>() { return 0.f; }
template <> __device__ __forceinline__ float4 rz<float4>() { return make_float4(0.f, 0.f, 0.f, 0.f); }
__device__ __forceinline__ void radd(float& a, float v) { a += v; }
__device__ __forceinline__ void radd(float4& a, const float4 v) { a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w; }

template <int J, bool V4>
__device__ __forceinline__ void canon_body(const RSeg& g, int blk, float4* shm) {
  using V = typename std::conditional<V4, float4, float>::type;
  constexpr int EL = 256 / J, VW = V4 ? 4 : 1;
  V (*sh)[EL + 1] = reinterpret_cast<V (*)[EL + 1]>(shm);
  const int el = threadIdx.x % EL, j = threadIdx.x / EL;
  const long e = ((long)blk * EL + el) * VW;
  const long MN = g.MN;
  const int S = g.S;
  V a = rz<V>();
  if (e < MN) {
    const V* p = reinterpret_cast<const V*>(g.ws + e);
    const long rs = MN / VW;   // row stride in V units
    if (!(g.form & 4)) {
      int s = j;
      for (; s + 3 * J < S; s += 4 * J) {
        const V v0 = p[(long)s * rs], v1 = p[(long)(s + J) * rs];
        const V v2 = p[(long)(s + 2 * J) * rs], v3 = p[(long)(s + 3 * J) * rs];
        radd(a, v0); radd(a, v1); radd(a, v2); radd(a, v3);
      }
      for (; s < S; s += J) radd(a, p[(long)s * rs]);
    } else {
      const int G = (S + 15) / 16;
      for (int r = j; r < G; r += J) {
        const int s0 = r * 16, n = min(16, S - s0);
        V q[4] = {rz<V>(), rz<V>(), rz<V>(), rz<V>()};
        if (n == 16) {
          V v[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) v[i] = p[(long)(s0 + i) * rs];
#pragma unroll
          for (int i = 0; i < 16; ++i) radd(q[i & 3], v[i]);
        } else {   // the last, partial group
          int i = 0;
          for (; i + 4 <= n; i += 4) {
            const V v0 = p[(long)(s0 + i) * rs], v1 = p[(long)(s0 + i + 1) * rs];
            const V v2 = p[(long)(s0 + i + 2) * rs], v3 = p[(long)(s0 + i + 3) * rs];
            radd(q[0], v0); radd(q[1], v1); radd(q[2], v2); radd(q[3], v3);
          }
          if (i < n) radd(q[0], p[(long)(s0 + i) * rs]);
          if (i + 1 < n) radd(q[1], p[(long)(s0 + i + 1) * rs]);
          if (i + 2 < n) radd(q[2], p[(long)(s0 + i + 2) * rs]);
        }
        V gs = q[0];
        radd(gs, q[1]);
        radd(gs, q[2]);
        radd(gs, q[3]);
        radd(a, gs);
      }
    }
  }
  sh[j][el] = a;
  __syncthreads();
  if (j == 0 && e < MN) {
    V t = rz<V>();
#pragma unroll
    for (int q = 0; q < J; ++q) radd(t, sh[q][el]);
    if constexpr (V4) {
      float4* d = reinterpret_cast<float4*>(g.dw + e);
      float4 o = *d;
      radd(o, t);
      *d = o;
    } else if (g.KK1 == 0) {
      g.dw[e] += t;
    } else {
      const long c = e / g.KK1;
      const int i = (int)(e - c * g.KK1);
      if (i < g.KK1 - 1) g.dw[c * (g.KK1 - 1) + i] += t;
      else if (g.db) g.db[c] += t;
    }
  }
}

// The weight-grad partials of wconv.hip (ConvTranspose 3x3 and PatchGAN 4x4 weight-grads):
// dW[m][c][t] += sum_s P[s][t][m][c].  Workgroup = MB rows m x 32 channels c: the partial rows are
// read coalesced along c, the sums go through LDS and leave as the contiguous dw block
// [m][c0..c0+31][0..T-1] (coalesced read-modify-write, no T-strided scatter).  Per element, the
// order of additions: 4 running sums over splits s = u mod 4 (the tail splits on sum 0), combined as
// (s0 + s1) + (s2 + s3).
template <int MB>
__device__ __forceinline__ void wc_body(const RSeg& g, int blk, float* sh) {
  const int T = g.T, M = g.M, C = g.C, splits = g.S;
  const int cbs = C / 32;
  const int c0 = (blk % cbs) * 32, m0 = (blk / cbs) * MB;
  const long plane = (long)M * C, sstride = plane * T;
  const int n = MB * 32 * T;
  for (int q = threadIdx.x; q < n; q += 256) {
    const int c = q & 31, mi = (q >> 5) & (MB - 1), t = q / (32 * MB);
    const int m = m0 + mi;
    float r = 0.f;
    if (m < M) {
      const float* p = g.ws + (long)t * plane + (long)m * C + c0 + c;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      int sp = 0;
      for (; sp + 16 <= splits; sp += 16) {   // 16 loads in flight, added in the 4-sum order
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = p[(long)(sp + u) * sstride];
#pragma unroll
        for (int u = 0; u < 16; u += 4) { s0 += v[u]; s1 += v[u + 1]; s2 += v[u + 2]; s3 += v[u + 3]; }
      }
      for (; sp + 4 <= splits; sp += 4) {
        s0 += p[(long)sp * sstride]; s1 += p[(long)(sp + 1) * sstride];
        s2 += p[(long)(sp + 2) * sstride]; s3 += p[(long)(sp + 3) * sstride];
      }
      for (; sp < splits; ++sp) s0 += p[(long)sp * sstride];
      r = (s0 + s1) + (s2 + s3);
    }
    sh[(mi * 32 + c) * (T + 1) + t] = r;
  }
  __syncthreads();
  const int rowlen = 32 * T;
  for (int j = threadIdx.x; j < n; j += 256) {
    const int mi = j / rowlen, rr = j - mi * rowlen;
    if (m0 + mi >= M) break;
    const int c = rr / T, t = rr - c * T;
    g.dw[((long)(m0 + mi) * C + c0) * T + rr] += sh[(mi * 32 + c) * (T + 1) + t];
  }
}

// up to RS_MAX reductions with disjoint outputs: segment i owns blocks [b0[i], b0[i+1])
__global__ __launch_bounds__(256) void split_canon_kernel(RSegs R) {
  // >= J * (256 / J + 1) float4 of the widest lane form, 4 x 32 x 17 floats of the wconv form
  __shared__ float4 sh[4 * 32 * 17 / 4];
  int i = 0;
  for (int q = 1; q < RS_MAX; ++q)
    if (q < R.n && (int)blockIdx.x >= R.s[q].b0) i = q;
  const RSeg g = R.s[i];
  const int blk = blockIdx.x - g.b0;
  if (g.form & 8) {
    if (g.form & 16) wc_body<4>(g, blk, reinterpret_cast<float*>(sh));
    else wc_body<1>(g, blk, reinterpret_cast<float*>(sh));
    return;
  }
  switch (g.form & 3) {
    case 3: canon_body<16, true>(g, blk, sh); break;
    case 2: canon_body<4, true>(g, blk, sh); break;
    case 1: canon_body<16, false>(g, blk, sh); break;
    default: canon_body<4, false>(g, blk, sh); break;
  }
}

static RSeg make_seg(const float* ws, int S, long MN, float* dw, float* db, int KK1) {
  RSeg s{};
  s.ws = ws; s.dw = dw; s.db = db; s.MN = MN; s.S = S; s.KK1 = KK1;
  const bool pre = S > 64 && MN < 65536;
  const int rows = pre ? (S + 15) / 16 : S;
  const bool v4 = KK1 == 0 && (MN & 3) == 0 && ((((uintptr_t)ws) | ((uintptr_t)dw)) & 15) == 0;
  s.form = (rows > 8 ? 1 : 0) | (v4 ? 2 : 0) | (pre ? 4 : 0);
  return s;
}
static long seg_blocks(const RSeg& s) {
  if (s.form & 8) return (long)((s.M + ((s.form & 16) ? 3 : 0)) / ((s.form & 16) ? 4 : 1)) * (s.C / 32);
  const long per = (long)(256 / ((s.form & 1) ? 16 : 4)) * ((s.form & 2) ? 4 : 1);
  return (s.MN + per - 1) / per;
}

// n <= RS_MAX segments (disjoint outputs) in one launch
static void launch_segs(const RSeg* v, int n, hipStream_t st) {
  RSegs R{};
  long b = 0;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    if (v[i].MN <= 0 || v[i].S <= 0) continue;
    R.s[k] = v[i];
    R.s[k].b0 = (int)b;
    b += seg_blocks(v[i]);
    ++k;
  }
  if (!k) return;
  R.n = k;
  hipLaunchKernelGGL(split_canon_kernel, dim3((unsigned)b), dim3(256), 0, st, R);
}

// ---- deferred mode ----------------------------------------------------------------------
// The queue is process state shared by the host threads that launch (the main thread and autograd's
// backward thread, which flushes before a DDP bucket's all-reduce): every access holds g_qmu.
static std::vector<RSeg> g_queue;
static hipStream_t g_queue_st = nullptr;
static int g_defer = 0;
static std::mutex g_qmu;

// output byte ranges of a segment: dw (and db)
static void seg_ranges(const RSeg& s, uintptr_t r[4]) {
  const long nd = s.KK1 ? (s.MN / s.KK1) * (s.KK1 - 1) : s.MN;
  r[0] = (uintptr_t)s.dw; r[1] = r[0] + (uintptr_t)nd * 4;
  r[2] = (uintptr_t)s.db; r[3] = s.db ? r[2] + (uintptr_t)(s.MN / s.KK1) * 4 : r[2];
}
static bool overlaps(const RSeg& a, const RSeg& b) {
  uintptr_t x[4], y[4];
  seg_ranges(a, x);
  seg_ranges(b, y);
  for (int i = 0; i < 4; i += 2)
    for (int k = 0; k < 4; k += 2)
      if (x[i] < x[i + 1] && y[k] < y[k + 1] && x[i] < y[k + 1] && y[k] < x[i + 1]) return true;
  return false;
}

static int flush_queue() {
  const int n = (int)g_queue.size();
  int i = 0;
  while (i < n) {
    int k = i + 1;
    while (k < n && k - i < RS_MAX) {
      bool clash = false;
      for (int q = i; q < k && !clash; ++q) clash = overlaps(g_queue[q], g_queue[k]);
      if (clash) break;
      ++k;
    }
    launch_segs(g_queue.data() + i, k - i, g_queue_st);
    i = k;
  }
  g_queue.clear();
  return n;
}

// Deferred mode keeps a reduction in the queue only when its partials are at most this many MB:
// larger ones run at once, while their partials are still cache-resident (DSGAN_SPLIT_DEFER_MAX_MB;
// unset = every reduction deferred).
static long defer_max_bytes() {
  static long v = -2;
  if (v == -2) {
    const char* e = getenv("DSGAN_SPLIT_DEFER_MAX_MB");
    v = (e && *e) ? (long)(atof(e) * 1048576.0) : -1;
  }
  return v;
}

static void submit(const RSeg* v, int n, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_qmu);
  if (!g_defer) {
    launch_segs(v, n, st);
    return;
  }
  if (!g_queue.empty() && st != g_queue_st) flush_queue();
  g_queue_st = st;
  const long lim = defer_max_bytes();
  for (int i = 0; i < n; ++i) {
    if (lim >= 0 && (long)v[i].S * v[i].MN * 4 > lim) {
      // run now; a queued reduction into the same output goes first (queue order = addition order)
      for (const RSeg& q : g_queue)
        if (overlaps(q, v[i])) { flush_queue(); break; }
      launch_segs(&v[i], 1, st);
    } else {
      g_queue.push_back(v[i]);
    }
  }
  if (g_queue.size() >= 4096) flush_queue();
}

void launch_split_reduce_kk(const float* ws, int splits, long MN, float* dw, float* db, int KK1, hipStream_t st) {
  const RSeg s = make_seg(ws, splits, MN, dw, db, KK1);
  submit(&s, 1, st);
}
// wconv.hip's partial layout [splits][T][M][C] -> dw[M][C][T] (+=), C % 32 == 0, T <= 16
void launch_split_reduce_wconv(const float* ws, int splits, int T, int M, int C, float* dw, hipStream_t st) {
  RSeg s{};
  s.ws = ws; s.dw = dw; s.db = nullptr; s.MN = (long)T * M * C; s.S = splits; s.KK1 = 0;
  s.T = T; s.M = M; s.C = C;
  s.form = 8 | ((long)M * (C / 32) >= 4096 ? 16 : 0);
  submit(&s, 1, st);
}
void launch_split_reduce(const float* ws, int splits, long MN, float* dw, hipStream_t st) {
  launch_split_reduce_kk(ws, splits, MN, dw, nullptr, 0, st);
}
// n (<= RS_MAX) independent reductions with disjoint outputs: one launch (or n queued segments)
void launch_split_reduce_multi(int n, const float* const* ws, const int* splits, const long* MN, float* const* dw,
                               hipStream_t st) {
  RSeg v[RS_MAX];
  int k = 0;
  for (int i = 0; i < n; ++i) {
    v[k++] = make_seg(ws[i], splits[i], MN[i], dw[i], nullptr, 0);
    if (k == RS_MAX) { submit(v, k, st); k = 0; }
  }
  if (k) submit(v, k, st);
}

}  // namespace dsg

using namespace dsg;

extern "C" {

// Deferred split reductions on (1) / off (0); returns the previous setting.  Turning it off does not
// flush: call dsgan_split_flush.
int dsgan_split_defer(int on) {
  std::lock_guard<std::mutex> lk(g_qmu);
  const int old = g_defer;
  g_defer = on ? 1 : 0;
  return old;
}

// Reductions queued and not yet launched.
int dsgan_split_pending(void) {
  std::lock_guard<std::mutex> lk(g_qmu);
  return (int)g_queue.size();
}

// Launch every queued reduction on the stream its producers ran on and empty the queue.  When `st`
// is another stream, it is made to wait for those launches (an event), so whatever `st` runs next
// sees the reduced gradients.  Returns 0, or an error code (the queue is empty either way: a
// reduction is never left queued to read scratch its caller has since released).
int dsgan_split_flush(hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_qmu);
  if (g_queue.empty()) return 0;   // (no HIP call at all)
  const hipStream_t qst = g_queue_st;
  flush_queue();
  DSG_CHECK_LAUNCH();
  if (st != qst) {
    static hipEvent_t ev = nullptr;
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      ev = nullptr;
      dsgan_set_error("dsgan_split_flush: no event to order stream %p after the reductions on %p", (void*)st,
                      (void*)qst);
      return -1;
    }
    if (hipEventRecord(ev, qst) != hipSuccess || hipStreamWaitEvent(st, ev, 0) != hipSuccess) {
      dsgan_set_error("dsgan_split_flush: could not order stream %p after the reductions on %p", (void*)st,
                      (void*)qst);
      return -1;
    }
  }
  return 0;
}

}  // extern "C"
