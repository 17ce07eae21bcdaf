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

// Raw buffer resource (gfx9 V#: 48-bit base, stride 0, num_records bytes) for
// the offset-addressed LDS DMA below; offsets >= num_records read as zero.
typedef int seg_i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ seg_i32x4 make_rsrc(const void* base, unsigned bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    seg_i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
    r.y = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffffu));
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

// One wave instruction moves 64 lanes x 16 B from rsrc + voff + soff into
// 1 KiB of contiguous LDS at lds_dst: the per-lane part of the address is a
// 32-bit VGPR that stays fixed across k steps (the step's offset is the
// scalar soff), and an out-of-range voff (0x80000000) lands zeros -- no
// 64-bit address arithmetic and no zero page per piece.  M0 is written
// without being restored: nothing in the gfx950 kernels that use this reads
// M0 (DS instructions do not).
__device__ __forceinline__ void bglds16(seg_i32x4 rsrc, unsigned voff, unsigned soff, unsigned lds_dst) {
    asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds_dst)
                 : "memory");
}

// As bglds16 with the LDS destination lds_base + OFF (OFF a compile-time byte
// offset folded into the M0 write).
template <int OFF>
__device__ __forceinline__ void bglds16_at(seg_i32x4 rsrc, unsigned voff, unsigned soff, unsigned lds_base) {
    asm volatile("s_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds_base), "n"(OFF)
                 : "memory");
}

template <int N>
__device__ __forceinline__ void wait_lgkmcnt() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
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
