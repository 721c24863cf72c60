// bf16-operand weight-grad instantiations of the pointwise GEMM (pw_impl.h; host side and C ABI in pwgemm.hip):
// one translation unit per (operand type, mode) so the kernel families compile in parallel.
#include "pw_impl.h"

namespace dsg {
template void pw_wgrad_launch<__bf16>(const PwArgs&, int, int, int, int, hipStream_t);
}  // namespace dsg
