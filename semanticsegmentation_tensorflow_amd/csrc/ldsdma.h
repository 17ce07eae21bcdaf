// LDS-DMA helpers shared by the gfx950 GEMM / direct-conv kernels.
#pragma once
#include "common.h"

namespace seg {

// One wave instruction moves 64 lanes x 16 B from per-lane global addresses
// into 1 KiB of contiguous LDS at M0.  Issued from inline asm so the compiler
// does not drain vmcnt before every later ds_read.
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Bijective remap so that consecutive logical workgroups land on the same XCD
// (hardware dispatches round-robin over the 8 XCDs).
__device__ __forceinline__ int xcd_remap2(int bid, int nwg) {
    const int xcd = bid & 7;
    const int q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

}  // namespace seg
