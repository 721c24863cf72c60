// C-ABI plumbing shared by every entry point of libdsgan_hip.so: thread-local last error,
// library version, and a device-count probe used by the host side to fail loudly.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

static thread_local char g_err[512] = "";

void dsgan_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" {
const char* dsgan_last_error_string(void) { return g_err; }
int dsgan_abi_version(void) { return 1; }
}
