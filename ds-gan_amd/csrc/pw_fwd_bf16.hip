// bf16-operand forward instantiations of the pointwise GEMM (pw_impl.h; host side and C ABI in pwgemm.hip):
// one translation unit per (operand type, mode) so the kernel families compile in parallel.
#include "pw_impl.h"

namespace dsg {
template void pw_fd_launch_m<__bf16, PW_FWD>(const PwArgs&, int, int, int, int, hipStream_t);
}  // namespace dsg
