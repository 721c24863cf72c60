// The split reductions live in pwgemm.hip (a long device compile); the ASan driver never reaches a
// launch, so these definitions only satisfy the linker and abort if anything ever calls them.
#include <hip/hip_runtime.h>
#include <stdlib.h>
namespace dsg {
void launch_split_reduce(const float*, int, long, float*, hipStream_t) { abort(); }
void launch_split_reduce_kk(const float*, int, long, float*, float*, int, hipStream_t) { abort(); }
}  // namespace dsg
