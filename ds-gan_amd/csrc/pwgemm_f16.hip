// fp16-operand instantiations of the pointwise GEMM (pw_impl.h), a translation unit of its own so
// that the two 16-bit types compile in parallel (--precision fp16, BASELINE configs[4]).
#include "pw_impl.h"

namespace dsg {
template void pw_fd_launch<_Float16>(int, const PwArgs&, int, int, int, hipStream_t);
template void pw_wgrad_launch<_Float16>(const PwArgs&, int, int, int, int, hipStream_t);
}  // namespace dsg
