// LDS-DMA helpers shared by the GEMV translation units (device code only; gemv.hip,
// gemv_exact.hip). `__builtin_amdgcn_global_load_lds` moves 16 B per lane from global memory
// straight into LDS (wave-uniform destination, lane l at +16*l), holding no VGPRs while in
// flight; hipcc does not track its completion, so the kernels wait for it explicitly.
#pragma once
#include <hip/hip_runtime.h>

namespace mvg {

typedef __attribute__((address_space(3))) void* lds_void_t;
typedef __attribute__((address_space(1))) void* gbl_void_t;

// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt[6:4], lgkmcnt[11:8]; the
// others left at "no wait"), fenced against compiler reordering of memory operations: the
// LDS-DMA writes of the tile about to be read are complete once at most N vector-memory
// operations of this wave are outstanding.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits on gfx950");
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void wait_lgkmcnt0() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

}  // namespace mvg
