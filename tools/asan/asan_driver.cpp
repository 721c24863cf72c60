// Host-side AddressSanitizer driver for the C-ABI shim (CPU only, no kernel launch).
//
// Built by tools/asan/build_asan.sh with -fsanitize=address on the HOST side of hipcc only
// (device code is compiled normally), linked against the small sources whose host logic is the
// most arithmetic-heavy: the error plumbing (capi.cpp), the thin 3x3 planners (thin3.hip), the
// split-K planner of tconv.hip, the pixel-chunk planner of skinny.hip and the pwsmall.hip
// dispatch checks.  Every call below either returns a plan or fails its argument validation
// BEFORE any HIP call, so the driver needs no GPU.  Exit 0 + "ASAN OK" = no finding.
#include <stdio.h>
#include <string.h>

typedef struct ihipStream_t* hipStream_t;
extern "C" {
const char* dsgan_last_error_string(void);
int dsgan_abi_version(void);
int dsgan_thin3_supported(int M, int H, int W, long bs_small, long bs_big);
long dsgan_thin3_wgrad_workspace(int nb, int K, int M, int H, int W);
int dsgan_thin3_fwd(const float* x, long x_bs, const float* w, const float* bias, float* y, long y_bs, int nb, int K,
                    int M, int H, int W, int accumulate, hipStream_t st);
int dsgan_thin3_dgrad(const float* dy, long dy_bs, const float* w, float* dx, long dx_bs, int nb, int K, int M, int H,
                      int W, int accumulate, hipStream_t st);
long dsgan_tconv_workspace(int nb, int K, int M, int Hout, int Wout, int ntaps);
int dsgan_tconv(const float* X, long x_bs, const float* Wt, const float* bias, float* Y, long y_bs,
                const float* gpre, long gpre_bs, int nb, int K, int M, int Hin, int Win, int Hout,
                int Wout, int stride, int ntaps, const int* dh, const int* dw, int Hdst, int Wdst,
                int os, int ph, int pw, int act, int gact, float slope, hipStream_t st);
long dsgan_conv_wgrad_small_workspace(int N, int Cin, int Cout, int KH, int KW, int Ho, int Wo);
int dsgan_conv_small_out(const float* x, long x_bs, const float* w, long wm, long wk, long wh, long ww,
                         const float* bias, float* y, long y_bs, int nb, int K, int M, int Hin, int Win,
                         int Ho, int Wo, int KH, int KW, int stride, int pad, int transposed,
                         int accumulate, hipStream_t st);
int dsgan_conv_wgrad_small(const float* dy, long dy_bs, const float* x, long x_bs, float* dw, int N,
                           int Cin, int H, int W, int Cout, int KH, int KW, int stride, int pad, int Ho,
                           int Wo, float* ws, long ws_elems, hipStream_t st);
int dsgan_pw_small_supported(int K, int M, int P, long x_bs, long y_bs);
int dsgan_pw_small(const float* X, long x_bs, const float* W, int wm, int wk, const float* bias, float* Y,
                   long y_bs, const float* G, long g_bs, int nb, int K, int M, int P, int act, int xact, int gact,
                   int accumulate, float slope, hipStream_t st);
}
void dsgan_set_error(const char* fmt, ...);
extern "C" int dsgan_set_half_type(int t);
extern "C" int dsgan_get_half_type(void);

static int fails = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

static bool err_has(const char* s) { return strstr(dsgan_last_error_string(), s) != nullptr; }

int main() {
  CHECK(dsgan_abi_version() == 3);
  // the process-wide 16-bit operand type: 0 bf16 / 1 fp16, anything else refused with a message
  CHECK(dsgan_get_half_type() == 0);
  CHECK(dsgan_set_half_type(1) == 0 && dsgan_get_half_type() == 1);
  CHECK(dsgan_set_half_type(7) == -1 && err_has("dsgan_set_half_type") && dsgan_get_half_type() == 1);
  CHECK(dsgan_set_half_type(0) == 0 && dsgan_get_half_type() == 0);
  // error string: formatting and truncation at the buffer size
  char big[2048];
  memset(big, 'x', sizeof(big) - 1);
  big[sizeof(big) - 1] = 0;
  dsgan_set_error("%s/%d", big, 7);
  CHECK(strlen(dsgan_last_error_string()) == 511);

  // thin3 planners and validation
  CHECK(dsgan_thin3_supported(3, 256, 256, 3 * 65536, 64 * 65536));
  CHECK(!dsgan_thin3_supported(5, 256, 256, 0, 0));
  CHECK(!dsgan_thin3_supported(3, 254, 256, 0, 0));
  CHECK(!dsgan_thin3_supported(3, 256, 200, 0, 0));
  for (int nb = 1; nb <= 16; nb *= 2)
    for (int K = 1; K <= 129; K += 32) {
      const long n = dsgan_thin3_wgrad_workspace(nb, K, 3, 256, 512);
      CHECK(n > 0 && n % (3L * K * 9) == 0);
    }
  CHECK(dsgan_thin3_fwd(nullptr, 0, nullptr, nullptr, nullptr, 0, 1, 64, 3, 256, 256, 0, nullptr) == -1);
  CHECK(err_has("dsgan_thin3_fwd"));
  float dummy[4] __attribute__((aligned(16)));
  CHECK(dsgan_thin3_dgrad(dummy, 0, dummy, dummy, 0, 1, 64, 9, 256, 256, 0, nullptr) == -1);
  CHECK(err_has("dsgan_thin3_dgrad"));

  // tconv split-K planner: under-filled launches split, filled ones do not
  CHECK(dsgan_tconv_workspace(16, 512, 1024, 16, 16, 9) > 0);     // 256 tiles of 144 K steps
  CHECK(dsgan_tconv_workspace(16, 64, 128, 128, 128, 9) == 0);    // 2048 tiles
  CHECK(dsgan_tconv_workspace(1, 33, 64, 8, 8, 9) == 0);          // K not a multiple of 32
  for (int K = 32; K <= 2048; K *= 2)
    for (int hw = 4; hw <= 64; hw *= 2) {
      const long n = dsgan_tconv_workspace(2, K, 256, hw, hw, 9);
      CHECK(n == 0 || n % (2L * 256 * hw * hw) == 0);
    }
  const int dh[1] = {0}, dw[1] = {0};
  CHECK(dsgan_tconv(dummy, 0, dummy, nullptr, dummy, 0, nullptr, 0, 1, 33, 8, 4, 4, 4, 4, 1, 1, dh, dw, 4, 4, 1, 0,
                    0, 0, 0, 0.f, nullptr) == -1);
  CHECK(err_has("multiple of 32"));

  // skinny: chunk planner and validation
  for (int big_side = 1; big_side <= 1024; big_side *= 4)
    CHECK(dsgan_conv_wgrad_small_workspace(16, big_side, 3, 3, 3, 256, 256) >= 0);
  CHECK(dsgan_conv_small_out(dummy, 0, dummy, 1, 1, 1, 1, nullptr, dummy, 0, 1, 4, 9, 8, 8, 8, 8, 3, 3, 1, 1, 0, 0,
                             nullptr) == -1);
  CHECK(err_has("dsgan_conv_small_out"));
  CHECK(dsgan_conv_wgrad_small(dummy, 0, dummy, 0, dummy, 1, 16, 8, 8, 16, 5, 5, 1, 2, 8, 8, nullptr, 0, nullptr) == -1);
  CHECK(err_has("KH*KW"));

  // pwsmall dispatch checks
  CHECK(dsgan_pw_small_supported(3, 64, 65536, 3 * 65536, 64 * 65536));
  CHECK(!dsgan_pw_small_supported(64, 64, 65536, 0, 0));
  CHECK(dsgan_pw_small(dummy, 0, dummy, 1, 1, nullptr, dummy, 0, nullptr, 0, 1, 64, 64, 64, 0, 0, 0, 0, 0.f,
                       nullptr) == -1);
  CHECK(err_has("dsgan_pw_small"));

  if (fails) { printf("%d check(s) failed\n", fails); return 1; }
  printf("ASAN OK\n");
  return 0;
}
