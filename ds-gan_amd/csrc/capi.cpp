// C-ABI plumbing shared by every entry point of libdsgan_hip.so: thread-local last error,
// library version, the process-wide 16-bit operand type (common.h HalfType), and a
// device-count probe used by the host side to fail loudly.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <atomic>
#include <vector>

static thread_local char g_err[512] = "";
// The one piece of library state besides the error string: which 16-bit type the "bf16" operand
// flags and the 16-bit MFMAs mean.  Set by the host when it selects a precision
// (dsgan_hip.functional.set_precision) and read by every launcher when it picks a kernel
// instantiation; launches are stream-ordered, so a change applies to launches issued after it.
static std::atomic<int> g_half{0};

void dsgan_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// Plan-only mode (common.h DSG_WS): entry points validate, plan and check their scratch, then
// return before any launch.  Thread-local, off by default; the CPU planner tests switch it on.
static thread_local int g_plan_only = 0;
static thread_local long g_ws_need = 0;

// Kernel-only timer: event pairs recorded around the pointwise GEMM kernel launches (pw_launch), so
// the bench's roofline figure is the GEMM kernel's own duration -- the one rocprofv3 reports -- and
// not the C-ABI call's, which also holds a split-K finishing pass.  Host-thread state: the training
// step issues its launches from the main thread and autograd's thread, never at once.
static std::vector<hipEvent_t> g_kt_ev;   // [2 i] before, [2 i + 1] after launch i
static size_t g_kt_n = 0;                 // pairs recorded since the last reset
static int g_kt_on = 0;
static bool g_kt_bad = false;             // an event could not be created / recorded

namespace dsg {
int half_type() { return g_half.load(std::memory_order_relaxed); }
bool plan_only() { return g_plan_only != 0; }
void note_ws_need(long n) { g_ws_need = n; }
void ktimer_mark(hipStream_t st, int end) {
  if (!g_kt_on || g_plan_only) return;
  const size_t i = 2 * g_kt_n + (end ? 1 : 0);
  while (g_kt_ev.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) { g_kt_bad = true; return; }
    g_kt_ev.push_back(e);
  }
  if (hipEventRecord(g_kt_ev[i], st) != hipSuccess) g_kt_bad = true;
  if (end) ++g_kt_n;
}
}  // namespace dsg

extern "C" {
const char* dsgan_last_error_string(void) { return g_err; }
int dsgan_abi_version(void) { return 3; }
int dsgan_set_plan_only(int on) {
  const int old = g_plan_only;
  g_plan_only = on ? 1 : 0;
  return old;
}
long dsgan_last_ws_need(void) { return g_ws_need; }
int dsgan_set_half_type(int t) {
  if (t != 0 && t != 1) {
    dsgan_set_error("dsgan_set_half_type: %d is not 0 (bf16) or 1 (fp16)", t);
    return -1;
  }
  g_half.store(t, std::memory_order_relaxed);
  return 0;
}
int dsgan_get_half_type(void) { return g_half.load(std::memory_order_relaxed); }
// Reads and clears the HIP runtime's last launch error (0 = none).  A stream capture that was
// invalidated leaves its error pending; every entry point checks hipGetLastError() after its
// launches, so the first eager launch after a failed capture would report it as its own.
int dsgan_clear_launch_error(void) { return (int)hipGetLastError(); }

// Kernel-only timer: on = 1 starts recording (the pair count is kept), 0 stops, -1 resets the count
// to 0 (the events are reused).  Returns the number of recorded pairs.
int dsgan_ktimer(int on) {
  if (on < 0) { g_kt_n = 0; g_kt_bad = false; }
  else g_kt_on = on ? 1 : 0;
  return (int)g_kt_n;
}
// Elapsed ms of the first min(n, max) recorded pairs into ms[] (the caller synchronises first);
// returns the number written, or -1 (error string set) when an event could not be recorded or read
// -- e.g. events recorded by the nodes of a replayed HIP graph.
int dsgan_ktimer_read(float* ms, int max) {
  if (g_kt_bad) { dsgan_set_error("dsgan_ktimer_read: an event could not be created or recorded"); return -1; }
  const int n = (int)(g_kt_n < (size_t)max ? g_kt_n : (size_t)max);
  for (int i = 0; i < n; ++i) {
    const hipError_t e = hipEventElapsedTime(&ms[i], g_kt_ev[2 * i], g_kt_ev[2 * i + 1]);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      dsgan_set_error("dsgan_ktimer_read: pair %d: %s", i, hipGetErrorString(e));
      return -1;
    }
  }
  return n;
}
}
