// fp16-operand data-grad instantiations of the pointwise GEMM (pw_impl.h; host side and C ABI in pwgemm.hip):
// one translation unit per (operand type, mode) so the kernel families compile in parallel.
#include "pw_impl.h"

namespace dsg {
template void pw_fd_launch_m<_Float16, PW_DGRAD>(const PwArgs&, int, int, int, int, hipStream_t);
}  // namespace dsg
