// Shared device/host helpers for the gfx950 segmentation kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/segkern.h"
#include "knobs.h"

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define SEG_LDS __attribute__((address_space(3)))

template <typename T> struct dt_traits;
template <> struct dt_traits<float> {
    static constexpr int EPC = 4;  // elements per 16-byte chunk
    static constexpr int id = SEG_F32;
};
template <> struct dt_traits<bf16> {
    static constexpr int EPC = 8;
    static constexpr int id = SEG_BF16;
};
template <> struct dt_traits<f16> {
    static constexpr int EPC = 8;
    static constexpr int id = SEG_F16;
};
template <typename T> inline constexpr bool is_bf16_v = false;
template <> inline constexpr bool is_bf16_v<bf16> = true;
template <typename T> inline constexpr bool is_f16_v = false;
template <> inline constexpr bool is_f16_v<f16> = true;

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
__device__ __forceinline__ float to_f32(f16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }
template <> __device__ __forceinline__ f16 from_f32<f16>(float v) { return (f16)v; }

// 8-lane 16-bit vector of T (MFMA operand) and one element's bits -> fp32
template <typename T> struct vec8 { typedef bf16x8 type; };
template <> struct vec8<f16> { typedef f16x8 type; };
template <typename T> using vec8_t = typename vec8<T>::type;
template <typename T>
__device__ __forceinline__ float bits16_to_f32(unsigned short u) {
    if constexpr (is_f16_v<T>) return (float)__builtin_bit_cast(f16, u);
    else return __uint_as_float((unsigned)u << 16);
}
template <typename T>
__device__ __forceinline__ f32x4 mfma_v8(const vec8_t<T>& a, const vec8_t<T>& b, const f32x4& c) {
    if constexpr (is_f16_v<T>) return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16x16x32 MFMA on eight packed 16-bit elements per lane (A, B as loaded from
// LDS), fp32 accumulation: bf16 or IEEE half operands
template <typename T>
__device__ __forceinline__ f32x4 mfma16x16x32(const uint4& a, const uint4& b, const f32x4& c) {
    if constexpr (is_f16_v<T>)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                       c, 0, 0, 0);
}

// 16-byte chunk <-> floats
template <typename T> struct Chunk;
template <> struct Chunk<float> {
    static constexpr int N = 4;
    __device__ __forceinline__ static void unpack(const uint4& u, float* f) {
        f[0] = __uint_as_float(u.x); f[1] = __uint_as_float(u.y);
        f[2] = __uint_as_float(u.z); f[3] = __uint_as_float(u.w);
    }
    __device__ __forceinline__ static uint4 pack(const float* f) {
        return make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                          __float_as_uint(f[3]));
    }
};
template <> struct Chunk<bf16> {
    static constexpr int N = 8;
    __device__ __forceinline__ static void unpack(const uint4& u, float* f) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = __uint_as_float(w[i] << 16);
            f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
    __device__ __forceinline__ static uint4 pack(const float* f) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf16 lo = (bf16)f[2 * i], hi = (bf16)f[2 * i + 1];
            w[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) |
                   ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
};

template <> struct Chunk<f16> {
    static constexpr int N = 8;
    __device__ __forceinline__ static void unpack(const uint4& u, float* f) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = (float)__builtin_bit_cast(f16, (uint16_t)(w[i] & 0xffffu));
            f[2 * i + 1] = (float)__builtin_bit_cast(f16, (uint16_t)(w[i] >> 16));
        }
    }
    __device__ __forceinline__ static uint4 pack(const float* f) {
        uint32_t w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f16 lo = (f16)f[2 * i], hi = (f16)f[2 * i + 1];
            w[i] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
        return make_uint4(w[0], w[1], w[2], w[3]);
    }
};

// Counter-based uniform in [0,1) for TF1 dropout, in groups of 8 counters:
// counter idx = 8 q + j.  The group hash of q is a lowbias32-style finalizer
// (xorshift-multiply, 32-bit multiplies: quarter rate on CDNA) of q (high word
// folded in first) with the seed key -- itself fully avalanched, a loop
// invariant -- XORed in after the first multiply; mixing the key
// non-additively keeps the streams of different seeds (layers, steps,
// data-parallel ranks) from being shifted copies of one another.  Each element
// then takes one more xorshift-multiply-xorshift of (group hash + j * golden
// ratio), so a lane that owns 4 or 8 consecutive counters (the conv
// epilogues' column chunks) pays ONE multiply per element plus the group hash
// once (SegDropRun), instead of the three multiplies per element of a
// per-counter finalizer.  Restated in numpy by the tests.
__host__ __device__ __forceinline__ uint32_t seg_avalanche32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ uint32_t seg_drop_key(uint64_t seed) {
    return seg_avalanche32((uint32_t)(seed ^ (seed >> 32)) ^ 0x632BE59Bu);
}

__host__ __device__ __forceinline__ uint32_t seg_grp_hash(uint32_t key, uint64_t q) {
    uint32_t x = (uint32_t)q ^ ((uint32_t)(q >> 32) * 0x85EBCA6Bu);
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= key;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ __forceinline__ float seg_grp_uniform(uint32_t h, uint32_t j) {
    uint32_t x = h + j * 0x9E3779B9u;
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    return (float)(x >> 8) * (1.0f / 16777216.0f);
}

__host__ __device__ __forceinline__ float seg_uniform(uint64_t seed, uint64_t idx) {
    return seg_grp_uniform(seg_grp_hash(seg_drop_key(seed), idx >> 3), (uint32_t)idx & 7u);
}

// TF1 dropout of one element, x / kp * floor(kp + U(seed, idx)), with the
// division as a multiply by 1/kp (within 1 ulp; the reciprocal is
// loop-invariant, an IEEE divide per element is not free in an epilogue).
__host__ __device__ __forceinline__ float seg_dropout(float x, float kp, uint64_t seed, uint64_t idx) {
    return (x * (1.f / kp)) * floorf(kp + seg_uniform(seed, idx));
}

// Dropout of N <= 8 consecutive counters base .. base + N - 1 (one lane's
// column chunk): the one or two group hashes they touch computed once.
// Same values as seg_dropout element by element.
template <int N>
struct SegDropRun {
    static_assert(N >= 1 && N <= 8, "at most one group boundary");
    uint32_t h0, h1, off;
    // on == false (keep_prob 1): no hashing; operator() must not be called
    __host__ __device__ __forceinline__ SegDropRun(uint64_t seed, uint64_t base, bool on = true) {
        h0 = h1 = off = 0u;
        if (!on) return;
        const uint32_t key = seg_drop_key(seed);
        off = (uint32_t)base & 7u;
        h0 = seg_grp_hash(key, base >> 3);
        h1 = off + N > 8 ? seg_grp_hash(key, (base >> 3) + 1) : h0;
    }
    __host__ __device__ __forceinline__ float operator()(float x, float kp, int j) const {
        const uint32_t jj = off + (uint32_t)j;
        return (x * (1.f / kp)) * floorf(kp + seg_grp_uniform(jj < 8u ? h0 : h1, jj & 7u));
    }
};

#define SEG_CHECK_LAUNCH()                                     \
    do {                                                       \
        if (hipGetLastError() != hipSuccess) return SEG_ELAUNCH; \
    } while (0)

static inline int seg_grid_1d(long n, int block, int cap = 2048 * 8) {
    long g = (n + block - 1) / block;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}
