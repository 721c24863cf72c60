// Instantiations of the persistent LDS-DMA ring pointwise GEMM (pw_ring.h) for f16 operands.
#include "pw_ring.h"

namespace dsg {
template bool pw_ring_launch<_Float16, PW_FWD, 0>(const PwArgs&, hipStream_t);
template bool pw_ring_launch<_Float16, PW_FWD, 1>(const PwArgs&, hipStream_t);
template bool pw_ring_launch<_Float16, PW_DGRAD, 0>(const PwArgs&, hipStream_t);
template bool pw_ring_launch<_Float16, PW_DGRAD, 1>(const PwArgs&, hipStream_t);
}  // namespace dsg
