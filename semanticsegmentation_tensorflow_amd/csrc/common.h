// Shared device/host helpers for the gfx950 segmentation kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "../../include/segkern.h"

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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

__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

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

// Counter-based uniform in [0,1) for TF1 dropout: splitmix64 of (seed, idx),
// top 24 bits.  Restated in numpy by the tests.
__host__ __device__ __forceinline__ float seg_uniform(uint64_t seed, uint64_t idx) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + idx + 0x632BE59BD9B4E019ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

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
