// Multi-tensor TF1 Adam fused with the bf16/fp32 compute-copy packing.
//
// The reference's AdamOptimizer.minimize (Network/model/FCN.py:338-340) updates
// every variable; the conv kernels then need the new weights in their packed
// layouts ([K][R][S][C] forward, HWIO dgrad, tconv variants).  Running Adam and
// then a pack pass re-reads all fp32 weights once per layout.  Here one launch
// walks a device-resident segment table: each block owns a TA x TB [a][b] tile
// of one variable viewed as [rs][a][b] (TB = 128 fp32 = 512-byte runs per
// array row, so HBM rows are streamed, not hopped), applies Adam to params /
// m / v, and
// writes the packed copies of the updated values:
//   rows copy       dst[(rs * ap + a) * bp + b]      (HWIO, tconv-forward)
//   transposed copy dst[(b * RS + rs) * ap + a]      (KRSC, tconv-input-grad)
// the transposed one through an LDS tile so both stores stay coalesced.
// Padding entries of the copies are never written (they keep the zeros of the
// initial pack).  Elementwise arithmetic is identical to adam_k (eltwise.hip).
// With G == null the same walk only rewrites the copies from P (no update):
// the repack after a data-parallel all-gather of sharded Adam results.
#include "common.h"

namespace {

constexpr int TA = 32, TB = 128;   // tile [a][b]; 256 threads = 32 lanes x float4 per b-row

template <typename T>
__device__ __forceinline__ uint2 pack4_16(const float* v) {   // four 16-bit (bf16 / half) values
    T h[4] = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
    return *reinterpret_cast<const uint2*>(h);
}

__device__ __forceinline__ int find_segment(const seg_adam_segment* segs, int nsegs, int tile) {
    int lo = 0, hi = nsegs - 1;
    while (lo < hi) {   // last segment with tile_begin <= tile
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].tile_begin <= tile) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <typename T>
__device__ __forceinline__ void adam_pack_tile(float* __restrict__ P, const float* __restrict__ G,
                                               float* __restrict__ Mm, float* __restrict__ Vv,
                                               const seg_adam_segment* __restrict__ segs, int nsegs, int tile,
                                               float lr_t, float b1, float b2, float eps, float gs,
                                               float (*lds)[TA + 1]) {
    const int si = find_segment(segs, nsegs, tile);
    const seg_adam_segment sg = segs[si];
    const int ta = (sg.a + TA - 1) / TA, tb = (sg.b + TB - 1) / TB;
    int t = tile - sg.tile_begin;
    const int rs = t / (ta * tb);
    t -= rs * ta * tb;
    const int a0 = (t / tb) * TA, b0 = (t - (t / tb) * tb) * TB;
    const int tid = threadIdx.x;
    const int bl = (tid & 31) * 4;
    const bool vec = ((sg.b & 3) == 0) && ((sg.offset & 3) == 0);
    T* rows = reinterpret_cast<T*>(sg.rows_dst);
#pragma unroll
    for (int i = 0; i < TA / 8; ++i) {
        const int al = (tid >> 5) + 8 * i;
        const int a = a0 + al, b = b0 + bl;
        float pv[4] = {0.f, 0.f, 0.f, 0.f};
        if (a < sg.a && b < sg.b) {
            const long e = sg.offset + ((long)rs * sg.a + a) * sg.b + b;
            if (!G) {    // pack only
                if (vec) {
                    const float4 pp = *reinterpret_cast<const float4*>(P + e);
                    pv[0] = pp.x; pv[1] = pp.y; pv[2] = pp.z; pv[3] = pp.w;
                } else {
                    for (int j = 0; j < 4 && b + j < sg.b; ++j) pv[j] = P[e + j];
                }
            } else if (vec) {   // b + 4 <= B since B % 4 == 0
                float4 pp = *reinterpret_cast<float4*>(P + e);
                const float4 gg = *reinterpret_cast<const float4*>(G + e);
                float4 mm = *reinterpret_cast<float4*>(Mm + e);
                float4 vv = *reinterpret_cast<float4*>(Vv + e);
#define ADAM1(c)                                                  \
    {                                                             \
        const float gc = gg.c * gs;                               \
        mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
        vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                  \
        pp.c = pp.c - lr_t * mm.c / (sqrtf(vv.c) + eps);          \
    }
                ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
                *reinterpret_cast<float4*>(P + e) = pp;
                *reinterpret_cast<float4*>(Mm + e) = mm;
                *reinterpret_cast<float4*>(Vv + e) = vv;
                pv[0] = pp.x; pv[1] = pp.y; pv[2] = pp.z; pv[3] = pp.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (b + j >= sg.b) break;
                    const long ej = e + j;
                    const float gc = G[ej] * gs;
                    const float mj = b1 * Mm[ej] + (1.f - b1) * gc;
                    const float vj = b2 * Vv[ej] + (1.f - b2) * gc * gc;
                    const float pj = P[ej] - lr_t * mj / (sqrtf(vj) + eps);
                    Mm[ej] = mj;
                    Vv[ej] = vj;
                    P[ej] = pj;
                    pv[j] = pj;
                }
            }
            if (rows) {
                T* d = rows + ((long)rs * sg.rows_ap + a) * sg.rows_bp + b;
                if (b + 4 <= sg.b) {
                    if constexpr (sizeof(T) == 2) {
                        *reinterpret_cast<uint2*>(d) = pack4_16<T>(pv);
                    } else {
                        *reinterpret_cast<float4*>(d) = float4{pv[0], pv[1], pv[2], pv[3]};
                    }
                } else {
                    for (int j = 0; j < 4 && b + j < sg.b; ++j) d[j] = from_f32<T>(pv[j]);
                }
            }
        }
        if (sg.tr_dst) {
#pragma unroll
            for (int j = 0; j < 4; ++j) lds[bl + j][al] = pv[j];
        }
    }
    if (!sg.tr_dst) return;
    __syncthreads();
    // transposed copy: thread -> (b row, 16 consecutive a)
    T* tr = reinterpret_cast<T*>(sg.tr_dst);
    const int RS = sg.rs;
    const int blr = tid >> 1, ab = (tid & 1) * 16;
    const int b = b0 + blr;
    if (b >= sg.b) return;
    T* d = tr + ((long)b * RS + rs) * sg.tr_ap + a0 + ab;
    const int na = min(16, sg.a - (a0 + ab));
    if (na <= 0) return;
    if (na == 16) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = lds[blr][ab + j];
        if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4*>(d) = Chunk<T>::pack(v);
            *reinterpret_cast<uint4*>(d + 8) = Chunk<T>::pack(v + 8);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<float4*>(d + 4 * q) = float4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
        }
    } else {
        for (int j = 0; j < na; ++j) d[j] = from_f32<T>(lds[blr][ab + j]);
    }
}

// one tile per block (full grid), or -- capped grid -- each block walks tiles
// blockIdx.x, +gridDim.x, ...: a low-occupancy update that streams HBM beside
// MFMA-bound kernels on another stream instead of taking their CUs
template <typename T>
__global__ __launch_bounds__(256) void adam_pack_k(float* __restrict__ P, const float* __restrict__ G,
                                                    float* __restrict__ Mm, float* __restrict__ Vv,
                                                    const seg_adam_segment* __restrict__ segs, int nsegs,
                                                    int total_tiles, float lr_t, float b1, float b2, float eps,
                                                    float gs) {
    __shared__ float lds[TB][TA + 1];
    for (int tile = blockIdx.x; tile < total_tiles; tile += gridDim.x) {
        adam_pack_tile<T>(P, G, Mm, Vv, segs, nsegs, tile, lr_t, b1, b2, eps, gs, lds);
        __syncthreads();          // the LDS transpose tile is reused by the next tile
    }
}

}  // namespace



extern "C" int seg_adam_segments_plan(seg_adam_segment* segs, int nsegs) {
    if (!segs || nsegs <= 0) return -SEG_EINVAL;
    long total = 0;
    for (int i = 0; i < nsegs; ++i) {
        seg_adam_segment& s = segs[i];
        if (s.rs <= 0 || s.a <= 0 || s.b <= 0) return -SEG_EINVAL;
        if (s.rows_dst && (s.rows_ap < s.a || s.rows_bp < s.b)) return -SEG_EINVAL;
        if (s.tr_dst && s.tr_ap < s.a) return -SEG_EINVAL;
        s.tile_begin = (int)total;
        total += (long)s.rs * ((s.a + TA - 1) / TA) * ((s.b + TB - 1) / TB);
        if (total > 0x7fffffff) return -SEG_EINVAL;
    }
    return (int)total;
}

extern "C" int seg_pack_segments(const float* p, const seg_adam_segment* dev_segs, int nsegs, int total_tiles,
                                  int dtype, void* stream) {
    if (!p || !dev_segs || nsegs <= 0 || total_tiles <= 0) return SEG_EINVAL;
    if ((uintptr_t)p & 15) return SEG_EALIGN;
    hipStream_t st = (hipStream_t)stream;
    float* P = const_cast<float*>(p);    // read only on this path
    if (dtype == SEG_BF16)
        hipLaunchKernelGGL(adam_pack_k<bf16>, dim3(total_tiles), dim3(256), 0, st, P, nullptr, nullptr, nullptr,
                           dev_segs, nsegs, total_tiles, 0.f, 0.f, 0.f, 0.f, 0.f);
    else if (dtype == SEG_F32)
        hipLaunchKernelGGL(adam_pack_k<float>, dim3(total_tiles), dim3(256), 0, st, P, nullptr, nullptr, nullptr,
                           dev_segs, nsegs, total_tiles, 0.f, 0.f, 0.f, 0.f, 0.f);
    else if (dtype == SEG_F16)
        hipLaunchKernelGGL(adam_pack_k<f16>, dim3(total_tiles), dim3(256), 0, st, P, nullptr, nullptr, nullptr,
                           dev_segs, nsegs, total_tiles, 0.f, 0.f, 0.f, 0.f, 0.f);
    else
        return SEG_EINVAL;
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_adam_tf1_pack(float* p, const float* g, float* m, float* v, const seg_adam_segment* dev_segs,
                                 int nsegs, int total_tiles, float lr, float b1, float b2, float eps, int t,
                                 float gs, int dtype, void* stream) {
    if (!p || !g || !m || !v || !dev_segs || nsegs <= 0 || total_tiles <= 0 || t < 1) return SEG_EINVAL;
    if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return SEG_EALIGN;
    const double lr_t = (double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
    hipStream_t st = (hipStream_t)stream;
    const int grid = g_adam_blocks > 0 ? std::min(total_tiles, g_adam_blocks) : total_tiles;
    if (dtype == SEG_BF16)
        hipLaunchKernelGGL(adam_pack_k<bf16>, dim3(grid), dim3(256), 0, st, p, g, m, v, dev_segs, nsegs, total_tiles,
                           (float)lr_t, b1, b2, eps, gs);
    else if (dtype == SEG_F32)
        hipLaunchKernelGGL(adam_pack_k<float>, dim3(grid), dim3(256), 0, st, p, g, m, v, dev_segs, nsegs, total_tiles,
                           (float)lr_t, b1, b2, eps, gs);
    else if (dtype == SEG_F16)
        hipLaunchKernelGGL(adam_pack_k<f16>, dim3(grid), dim3(256), 0, st, p, g, m, v, dev_segs, nsegs, total_tiles,
                           (float)lr_t, b1, b2, eps, gs);
    else
        return SEG_EINVAL;
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}
