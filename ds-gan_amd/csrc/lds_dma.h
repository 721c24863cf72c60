// LDS-DMA helpers (gfx950): global -> LDS copies that bypass the VGPRs.
#pragma once
#include "common.h"

namespace dsg {

// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): lane l's 16 bytes land at LDS byte address
// lds + 16 l (the destination is wave-uniform base + lane-linear; the global SOURCE is per lane, so a
// gather or a swizzle goes on the source address).  Issued from asm so that hipcc neither counts it
// nor drains it with a vmcnt(0) in front of every LDS read of the other buffer: the issuing wave waits
// for it by hand (s_waitcnt vmcnt) and a barrier orders it for the other waves' ds_reads.  M0 is
// written and restored in the same statement (it is compiler-reserved).
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds)
               : "memory");
}
// LDS byte offset of a __shared__ pointer (wave-uniform)
__device__ __forceinline__ unsigned lds_off(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)p);
}
// every LDS-DMA this wave issued has landed in LDS
__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 16 zero bytes in global memory: the source of the LDS-DMA lanes whose element lies outside the
// tensor (image borders), so a patch image is filled whole by lane-linear DMA without masking
static __device__ __attribute__((aligned(16))) unsigned int g_dma_zero16[4] = {0u, 0u, 0u, 0u};

}  // namespace dsg
