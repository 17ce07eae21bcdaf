// HBM-bound kernels of the training path: bias/ReLU gradients, pooling,
// dropout, frozen-stat BatchNorm+ReLU, bilinear resize, softmax
// cross-entropy, argmax / confusion counts, TF1 Adam, and small utilities.
// All per-pixel work moves 16-byte chunks (8 bf16 / 4 fp32) per lane;
// channel reductions are two-stage (per-workgroup partials in a caller
// workspace, then one ordered pass) so results are run-to-run deterministic.
#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ uint4 ldc(const T* p) { return *reinterpret_cast<const uint4*>(p); }
template <typename T>
__device__ __forceinline__ void stc(T* p, const uint4& v) { *reinterpret_cast<uint4*>(p) = v; }

constexpr int RED_BLOCKS = 1024;

// ---------------------------------------------------------------------------
// channel-reduction skeleton: each workgroup covers a contiguous pixel range
// and all K channels; LPP lanes span the channel chunks of one pixel.
// ---------------------------------------------------------------------------
struct RedGeom {
    int CK, LPP, rows, iters;
};
__host__ __device__ inline RedGeom red_geom(int K, int epc) {
    RedGeom g;
    g.CK = K / epc;
    g.LPP = g.CK < 256 ? g.CK : 256;
    g.rows = 256 / g.LPP;
    g.iters = (g.CK + 255) / 256;
    return g;
}

// ReluGrad + BiasAddGrad
template <typename T>
__global__ __launch_bounds__(256) void bias_relu_bwd_k(const T* __restrict__ dy, int ld_dy, const T* __restrict__ y,
                                                       int ld_y, T* __restrict__ dz, int ld_dz, float* __restrict__ part,
                                                       long P, int K, int relu, float scale) {
    constexpr int EPC = dt_traits<T>::EPC;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const RedGeom g = red_geom(K, EPC);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    const bool active = prow < g.rows;
    const long per = (P + gridDim.x - 1) / gridDim.x;
    const long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
    constexpr int MAXIT = 16 / EPC;
    float acc[MAXIT][EPC];
#pragma unroll
    for (int j = 0; j < MAXIT; ++j)
#pragma unroll
        for (int e = 0; e < EPC; ++e) acc[j][e] = 0.f;
    if (active) {
        for (long pix = p0 + prow; pix < p1; pix += g.rows) {
#pragma unroll
            for (int j = 0; j < MAXIT; ++j) {
                if (j >= g.iters) break;
                const int cc = c8 + j * g.LPP;
                if (cc >= g.CK) break;
                float d[EPC];
                Chunk<T>::unpack(ldc(dy + pix * ld_dy + cc * EPC), d);
                if (relu) {
                    float yy[EPC];
                    Chunk<T>::unpack(ldc(y + pix * ld_y + cc * EPC), yy);
#pragma unroll
                    for (int e = 0; e < EPC; ++e) d[e] = yy[e] > 0.f ? d[e] * scale : 0.f;
                    stc(dz + pix * ld_dz + cc * EPC, Chunk<T>::pack(d));
                } else if (scale != 1.f) {
#pragma unroll
                    for (int e = 0; e < EPC; ++e) d[e] *= scale;
                    stc(dz + pix * ld_dz + cc * EPC, Chunk<T>::pack(d));
                } else if (dz != dy) {
                    stc(dz + pix * ld_dz + cc * EPC, Chunk<T>::pack(d));
                }
#pragma unroll
                for (int e = 0; e < EPC; ++e) acc[j][e] += d[e];
            }
        }
    }
    // block reduction over prow: red[prow][K]
#pragma unroll
    for (int j = 0; j < MAXIT; ++j) {
        const int cc = c8 + j * g.LPP;
        if (active && j < g.iters && cc < g.CK)
#pragma unroll
            for (int e = 0; e < EPC; ++e) red[prow * K + cc * EPC + e] = acc[j][e];
    }
    __syncthreads();
    for (int k = t; k < K; k += 256) {
        float s = 0.f;
        for (int r = 0; r < g.rows; ++r) s += red[r * K + k];
        part[(long)blockIdx.x * K + k] = s;
    }
}

// BiasAddGrad of a wide dy (K >= 512: conv6 / conv7, 4096 channels over a few
// thousand pixels): workgroup (64 chunks of 8 channels) x (row range), four
// row lanes with four rows in flight each, so every wave streams 1 KiB rows
// instead of the one-row-per-block walk of bias_relu_bwd_k at K = 4096
// (65.7 us for 3.8 MB in the C2 step).  part[blockIdx.y][K], summed by
// reduce_rows_k; fixed order, deterministic.
template <typename T>
__global__ __launch_bounds__(256) void col_sum_k(const T* __restrict__ dy, int ld_dy, float* __restrict__ part,
                                                 long P, int K, int per) {
    constexpr int EPC = dt_traits<T>::EPC;
    __shared__ float red[3][64 * EPC];
    const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int cc = blockIdx.x * 64 + cl;
    const bool live = cc < K / EPC;
    const long p0 = (long)blockIdx.y * per, p1 = min(P, p0 + per);
    float acc[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[e] = 0.f;
    if (live) {
        const T* src = dy + cc * EPC;
        long pix = p0 + rl;
        for (; pix + 12 < p1; pix += 16) {
            float d[4][EPC];
#pragma unroll
            for (int u = 0; u < 4; ++u) Chunk<T>::unpack(ldc(src + (pix + 4 * u) * ld_dy), d[u]);
#pragma unroll
            for (int e = 0; e < EPC; ++e) acc[e] += (d[0][e] + d[1][e]) + (d[2][e] + d[3][e]);
        }
        for (; pix < p1; pix += 4) {
            float d[EPC];
            Chunk<T>::unpack(ldc(src + pix * ld_dy), d);
#pragma unroll
            for (int e = 0; e < EPC; ++e) acc[e] += d[e];
        }
    }
    if (rl > 0) {
#pragma unroll
        for (int e = 0; e < EPC; ++e) red[rl - 1][e * 64 + cl] = acc[e];
    }
    __syncthreads();
    if (rl == 0 && live) {
        float o[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) o[e] = (acc[e] + red[0][e * 64 + cl]) + (red[1][e * 64 + cl] + red[2][e * 64 + cl]);
        float* dst = part + (long)blockIdx.y * K + cc * EPC;
#pragma unroll
        for (int e = 0; e < EPC; e += 4) *reinterpret_cast<float4*>(dst + e) = make_float4(o[e], o[e + 1], o[e + 2], o[e + 3]);
    }
}

// Column sums of a [nrows][K] fp32 partial matrix: 8 channels x 32 row groups
// per workgroup, so even K = 64 spreads 1024 rows over 2048 threads.
__global__ __launch_bounds__(256) void reduce_rows_k(const float* __restrict__ part, int nrows, int K, int k_valid,
                                                     float* __restrict__ out) {
    __shared__ float s[32][9];
    const int cl = threadIdx.x & 7, rg = threadIdx.x >> 3;
    const int c = blockIdx.x * 8 + cl;
    float acc = 0.f;
    if (c < k_valid)
        for (int r = rg; r < nrows; r += 32) acc += part[(long)r * K + c];
    s[rg][cl] = acc;
    __syncthreads();
    if (threadIdx.x < 8 && c < k_valid) {
        float t = 0.f;
        for (int r = 0; r < 32; ++r) t += s[r][cl];
        out[c] = t;
    }
}

// ---------------------------------------------------------------------------
// 2x2 pooling
// ---------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int ldx, int ldy) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2, OW = W / 2, CK = C / EPC;
    const long total = (long)N * OH * OW * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cc = (int)(i % CK);
        long t = i / CK;
        const int ow = (int)(t % OW);
        t /= OW;
        const int oh = (int)(t % OH);
        const int n = (int)(t / OH);
        const T* b = x + (((long)n * H + 2 * oh) * W + 2 * ow) * ldx + cc * EPC;
        float v0[EPC], v1[EPC], v2[EPC], v3[EPC];
        Chunk<T>::unpack(ldc(b), v0);
        Chunk<T>::unpack(ldc(b + ldx), v1);
        Chunk<T>::unpack(ldc(b + (long)W * ldx), v2);
        Chunk<T>::unpack(ldc(b + (long)W * ldx + ldx), v3);
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            float m = v0[e];
            m = v1[e] > m ? v1[e] : m;
            m = v2[e] > m ? v2[e] : m;
            m = v3[e] > m ? v3[e] : m;
            v0[e] = m;
        }
        stc(y + (((long)n * OH + oh) * OW + ow) * ldy + cc * EPC, Chunk<T>::pack(v0));
    }
}

// One thread per (2x2 input block, chunk); blocks past the pooled region
// (odd H / W) receive zero gradient.
template <typename T>
__global__ void maxpool_bwd_k(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ dx, int N, int H,
                              int W, int C, int ldx, int ldy, int relu) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2, OW = W / 2, BH = (H + 1) / 2, BW = (W + 1) / 2, CK = C / EPC;
    const long total = (long)N * BH * BW * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cc = (int)(i % CK);
        long t = i / CK;
        const int bw = (int)(t % BW);
        t /= BW;
        const int bh = (int)(t % BH);
        const int n = (int)(t / BH);
        const long base = (((long)n * H + 2 * bh) * W + 2 * bw) * ldx + cc * EPC;
        float o[4][EPC];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < EPC; ++e) o[q][e] = 0.f;
        if (bh < OH && bw < OW) {
            float v[4][EPC], d[EPC];
            Chunk<T>::unpack(ldc(x + base), v[0]);
            Chunk<T>::unpack(ldc(x + base + ldx), v[1]);
            Chunk<T>::unpack(ldc(x + base + (long)W * ldx), v[2]);
            Chunk<T>::unpack(ldc(x + base + (long)W * ldx + ldx), v[3]);
            Chunk<T>::unpack(ldc(dy + (((long)n * OH + bh) * OW + bw) * ldy + cc * EPC), d);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                int a = 0;
                float m = v[0][e];
                if (v[1][e] > m) { m = v[1][e]; a = 1; }
                if (v[2][e] > m) { m = v[2][e]; a = 2; }
                if (v[3][e] > m) { m = v[3][e]; a = 3; }
                // relu: ReluGrad of the post-ReLU input -> nothing flows where the max is 0
                const float g = (relu && !(m > 0.f)) ? 0.f : d[e];
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q][e] = (q == a) ? g : 0.f;
            }
        }
        const bool h1 = 2 * bh + 1 < H, w1 = 2 * bw + 1 < W;
        stc(dx + base, Chunk<T>::pack(o[0]));
        if (w1) stc(dx + base + ldx, Chunk<T>::pack(o[1]));
        if (h1) stc(dx + base + (long)W * ldx, Chunk<T>::pack(o[2]));
        if (h1 && w1) stc(dx + base + (long)W * ldx + ldx, Chunk<T>::pack(o[3]));
    }
}

// MaxPool with its switches recorded (training path): besides y, one byte per
// pooled element -- bits 0-1 the first-max position q (0 = (0,0), 1 = (0,1),
// 2 = (1,0), 3 = (1,1), TF's tie rule as maxpool_fwd_k), bit 2 set when the max
// is > 0 (the ReluGrad of a post-ReLU input, !(m > 0) for NaN as well).  The
// gradient then reads dy + 1 B/elem instead of the 4x-sized input x.  32-bit
// index math (the host checks the element count).  idx row stride = C.
template <typename T>
__global__ void maxpool_fwd_idx_k(const T* __restrict__ x, T* __restrict__ y, unsigned char* __restrict__ idx, int H,
                                  int W, int C, int ldx, int ldy, unsigned OW, unsigned CK, unsigned total) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned cc = i % CK, pix = i / CK;
        const unsigned ow = pix % OW, t = pix / OW;
        const unsigned oh = t % (unsigned)OH, n = t / (unsigned)OH;
        const T* b = x + ((long)(n * (unsigned)H + 2 * oh) * W + 2 * ow) * ldx + cc * EPC;
        float v0[EPC], v1[EPC], v2[EPC], v3[EPC];
        Chunk<T>::unpack(ldc(b), v0);
        Chunk<T>::unpack(ldc(b + ldx), v1);
        Chunk<T>::unpack(ldc(b + (long)W * ldx), v2);
        Chunk<T>::unpack(ldc(b + (long)W * ldx + ldx), v3);
        unsigned long long code = 0;
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            unsigned a = 0;
            float m = v0[e];
            if (v1[e] > m) { m = v1[e]; a = 1; }
            if (v2[e] > m) { m = v2[e]; a = 2; }
            if (v3[e] > m) { m = v3[e]; a = 3; }
            v0[e] = m;
            code |= (unsigned long long)(a | (m > 0.f ? 4u : 0u)) << (8 * e);
        }
        stc(y + (long)pix * ldy + cc * EPC, Chunk<T>::pack(v0));
        unsigned char* q = idx + (long)pix * C + cc * EPC;
        if constexpr (EPC == 8) *reinterpret_cast<unsigned long long*>(q) = code;
        else *reinterpret_cast<unsigned*>(q) = (unsigned)code;
    }
}

// MaxPoolGrad from the recorded switches: one thread per (2x2 input block,
// chunk); blocks past the pooled region (odd H / W) receive zero gradient.
template <typename T>
__global__ void maxpool_bwd_idx_k(const unsigned char* __restrict__ idx, const T* __restrict__ dy, T* __restrict__ dx,
                                  int H, int W, int C, int ldx, int ldy, int relu, unsigned BW, unsigned CK,
                                  unsigned total) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2, OW = W / 2, BH = (H + 1) / 2;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const unsigned cc = i % CK, blk = i / CK;
        const unsigned bw = blk % BW, t = blk / BW;
        const unsigned bh = t % (unsigned)BH, n = t / (unsigned)BH;
        const long base = ((long)(n * (unsigned)H + 2 * bh) * W + 2 * bw) * ldx + cc * EPC;
        float o[4][EPC];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < EPC; ++e) o[q][e] = 0.f;
        if (bh < (unsigned)OH && bw < (unsigned)OW) {
            const unsigned pix = (n * (unsigned)OH + bh) * (unsigned)OW + bw;
            const unsigned char* q = idx + (long)pix * C + cc * EPC;
            unsigned long long code;
            if constexpr (EPC == 8) code = *reinterpret_cast<const unsigned long long*>(q);
            else code = *reinterpret_cast<const unsigned*>(q);
            float d[EPC];
            Chunk<T>::unpack(ldc(dy + (long)pix * ldy + cc * EPC), d);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                const unsigned c8 = (unsigned)(code >> (8 * e)) & 7u;
                const float g = (relu && !(c8 & 4u)) ? 0.f : d[e];
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) o[qq][e] = ((c8 & 3u) == (unsigned)qq) ? g : 0.f;
            }
        }
        const bool h1 = 2 * bh + 1 < (unsigned)H, w1 = 2 * bw + 1 < (unsigned)W;
        stc(dx + base, Chunk<T>::pack(o[0]));
        if (w1) stc(dx + base + ldx, Chunk<T>::pack(o[1]));
        if (h1) stc(dx + base + (long)W * ldx, Chunk<T>::pack(o[2]));
        if (h1 && w1) stc(dx + base + (long)W * ldx + ldx, Chunk<T>::pack(o[3]));
    }
}

template <typename T>
__global__ void avgpool_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int ldx, int ldy) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2, OW = W / 2, CK = C / EPC;
    const long total = (long)N * OH * OW * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cc = (int)(i % CK);
        long t = i / CK;
        const int ow = (int)(t % OW);
        t /= OW;
        const int oh = (int)(t % OH);
        const int n = (int)(t / OH);
        const T* b = x + (((long)n * H + 2 * oh) * W + 2 * ow) * ldx + cc * EPC;
        float v0[EPC], v1[EPC], v2[EPC], v3[EPC];
        Chunk<T>::unpack(ldc(b), v0);
        Chunk<T>::unpack(ldc(b + ldx), v1);
        Chunk<T>::unpack(ldc(b + (long)W * ldx), v2);
        Chunk<T>::unpack(ldc(b + (long)W * ldx + ldx), v3);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v0[e] = ((v0[e] + v1[e]) + (v2[e] + v3[e])) * 0.25f;
        stc(y + (((long)n * OH + oh) * OW + ow) * ldy + cc * EPC, Chunk<T>::pack(v0));
    }
}

template <typename T>
__global__ void avgpool_bwd_k(const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int ldx, int ldy) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int OH = H / 2, OW = W / 2, BH = (H + 1) / 2, BW = (W + 1) / 2, CK = C / EPC;
    const long total = (long)N * BH * BW * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int cc = (int)(i % CK);
        long t = i / CK;
        const int bw = (int)(t % BW);
        t /= BW;
        const int bh = (int)(t % BH);
        const int n = (int)(t / BH);
        const long base = (((long)n * H + 2 * bh) * W + 2 * bw) * ldx + cc * EPC;
        float d[EPC];
        if (bh < OH && bw < OW) {
            Chunk<T>::unpack(ldc(dy + (((long)n * OH + bh) * OW + bw) * ldy + cc * EPC), d);
#pragma unroll
            for (int e = 0; e < EPC; ++e) d[e] *= 0.25f;
        } else {
#pragma unroll
            for (int e = 0; e < EPC; ++e) d[e] = 0.f;
        }
        const uint4 v = Chunk<T>::pack(d);
        const bool h1 = 2 * bh + 1 < H, w1 = 2 * bw + 1 < W;
        stc(dx + base, v);
        if (w1) stc(dx + base + ldx, v);
        if (h1) stc(dx + base + (long)W * ldx, v);
        if (h1 && w1) stc(dx + base + (long)W * ldx + ldx, v);
    }
}

// ---------------------------------------------------------------------------
// elementwise
// ---------------------------------------------------------------------------
template <typename T>
__global__ void add_k(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f32<T>(to_f32(a[i]) + to_f32(b[i]));
}

template <typename T>
__global__ void dropout_k(const T* __restrict__ x, T* __restrict__ y, long n, float kp, uint64_t seed) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float u = seg_uniform(seed, (uint64_t)i);
        y[i] = from_f32<T>((to_f32(x[i]) * (1.f / kp)) * floorf(kp + u));
    }
}

// TF1 dropout gradient of a conv whose forward epilogue applied the dropout
// (no ReLU after it): element (pixel p, channel c < cv) uses the epilogue's
// counter index p * cv + c; padding channels are zeroed.  Lanes own fixed
// 8-channel chunks and walk pixels (bn_relu_fwd_k's geometry): the flat
// element loop paid a 64-bit division per 16-byte chunk.
template <typename T>
__global__ __launch_bounds__(256) void dropout_ch_k(const T* __restrict__ dy, int ldy, T* __restrict__ dz, int ldz,
                                                    long P, int C, int cv, float kp, uint64_t seed) {
    constexpr int EPC = dt_traits<T>::EPC;
    constexpr int MAXIT = 16 / EPC;
    const RedGeom g = red_geom(C, EPC);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    if (prow >= g.rows) return;
    const long step = (long)gridDim.x * g.rows;
    for (long pix = (long)blockIdx.x * g.rows + prow; pix < P; pix += step) {
        const uint64_t base = (uint64_t)pix * cv;
#pragma unroll
        for (int j = 0; j < MAXIT; ++j) {
            if (j >= g.iters) break;
            const int cc = c8 + j * g.LPP;
            if (cc >= g.CK) break;
            float v[EPC];
            Chunk<T>::unpack(ldc(dy + pix * ldy + cc * EPC), v);
            const SegDropRun<EPC> drop(seed, base + cc * EPC);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                const int c = cc * EPC + e;
                v[e] = c < cv ? drop(v[e], kp, e) : 0.f;
            }
            stc(dz + pix * ldz + cc * EPC, Chunk<T>::pack(v));
        }
    }
}

// The same re-draw with one 8-channel chunk per thread over a grid of all
// (pixel, chunk) pairs: no grid-stride loop, the chunk's loads issued at once
// (the loop form above ran FC-DenseNet's 16-channel growth outputs at ~1.5-2
// TB/s, instruction-bound like smallk_nt's first forms)
template <typename T>
__global__ __launch_bounds__(256) void dropout_ch_flat_k(const T* __restrict__ dy, int ldy, T* __restrict__ dz, int ldz,
                                                         int P, int CK, int cv, float kp, uint64_t seed) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= P * CK) return;
    const int pix = q / CK, cc = q - pix * CK;
    const uint64_t base = (uint64_t)pix * cv;
    float v[EPC];
    Chunk<T>::unpack(ldc(dy + (long)pix * ldy + cc * EPC), v);
    const SegDropRun<EPC> drop(seed, base + cc * EPC);
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
        const int c = cc * EPC + e;
        v[e] = c < cv ? drop(v[e], kp, e) : 0.f;
    }
    stc(dz + (long)pix * ldz + cc * EPC, Chunk<T>::pack(v));
}

template <typename T>
__global__ void fill_k(T* y, long n, float v) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f32<T>(v);
}

// y += alpha * x, fp32 (accumulate template: accum.assign_add(const * g), Network/main.py:92-95)
__global__ void axpy_k(float* __restrict__ y, const float* __restrict__ x, float alpha, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = fmaf(alpha, x[i], y[i]);
}

template <typename A, typename B>
__global__ void cast_k(const A* __restrict__ x, B* __restrict__ y, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f32<B>(to_f32(x[i]));
}

template <typename T>
__global__ void copy_channels_k(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy, long P, int C) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int CK = C / EPC;
    const long total = P * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long p = i / CK;
        const int cc = (int)(i - p * CK);
        stc(y + p * ldy + cc * EPC, ldc(x + p * ldx + cc * EPC));
    }
}


// ---------------------------------------------------------------------------
// tf.concat over channels with unaligned part offsets (FC-DenseNet)
// ---------------------------------------------------------------------------
struct ConcatArgs {
    seg_concat_part part[SEG_CONCAT_MAX];
    int off[SEG_CONCAT_MAX + 1];
    int n;
};

template <typename T>
__global__ void concat_fwd_k(ConcatArgs a, T* __restrict__ y, int ldy, int yc8, long P) {
    const long total = P * yc8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long p = i / yc8;
        const int k = (int)(i - p * yc8);
        float v[8];
        int src = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = k * 8 + j;
            while (src < a.n && c >= a.off[src + 1]) ++src;
            v[j] = 0.f;
            if (src < a.n) {
                const T* xp = reinterpret_cast<const T*>(a.part[src].ptr);
                v[j] = to_f32(xp[p * a.part[src].ld + (c - a.off[src])]);
            }
        }
        T* yp = y + p * ldy + k * 8;
        if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
        } else {
            *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
            *reinterpret_cast<uint4*>(yp + 4) = Chunk<T>::pack(v + 4);
        }
    }
}

// one thread per (pixel, 8-channel chunk of a destination part)
template <typename T>
__global__ void concat_bwd_k(const T* __restrict__ dy, int ldy, ConcatArgs a, const int* __restrict__ dummy,
                             long P, int chunks_per_px) {
    (void)dummy;
    const long total = P * chunks_per_px;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long p = i / chunks_per_px;
        int k = (int)(i - p * chunks_per_px);
        int d = 0;
        while (d < a.n && k >= (a.part[d].channels + 7) / 8) { k -= (a.part[d].channels + 7) / 8; ++d; }
        if (d >= a.n) continue;
        const seg_concat_part& pt = a.part[d];
        T* xp = reinterpret_cast<T*>(const_cast<void*>(pt.ptr)) + p * pt.ld + k * 8;
        float v[8];
        if (pt.accumulate) {
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xp), v);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(xp + 4), v + 4);
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = k * 8 + j;
            if (c < pt.channels) v[j] += to_f32(dy[p * ldy + a.off[d] + c]);
        }
        *reinterpret_cast<uint4*>(xp) = Chunk<T>::pack(v);
        if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(xp + 4) = Chunk<T>::pack(v + 4);
    }
}

// bf16 fast paths when every part starts on an 8-channel boundary: a lane owns
// one output chunk (its source part found once), pixels are walked with
// 16-byte loads / stores (the element loops above run at a fraction of HBM)
__global__ __launch_bounds__(256) void concat_fwd_fast_k(ConcatArgs a, bf16* __restrict__ y, int ldy, int yc8,
                                                         long P) {
    const RedGeom g = red_geom(yc8 * 8, 8);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    if (prow >= g.rows) return;
    const long step = (long)gridDim.x * g.rows;
    for (int j = 0; j < g.iters; ++j) {
        const int k = c8 + j * g.LPP;
        if (k >= yc8) break;
        int src = 0;
        while (src < a.n && k * 8 >= a.off[src + 1]) ++src;
        const bf16* xp = src < a.n ? reinterpret_cast<const bf16*>(a.part[src].ptr) + (k * 8 - a.off[src]) : nullptr;
        const int ld = src < a.n ? a.part[src].ld : 0;
        for (long p = (long)blockIdx.x * g.rows + prow; p < P; p += step) {
            const uint4 v = xp ? *reinterpret_cast<const uint4*>(xp + p * ld) : uint4{0u, 0u, 0u, 0u};
            *reinterpret_cast<uint4*>(y + p * ldy + k * 8) = v;
        }
    }
}

__global__ __launch_bounds__(256) void concat_bwd_fast_k(const bf16* __restrict__ dy, int ldy, ConcatArgs a,
                                                         int chunks, long P) {
    const RedGeom g = red_geom(chunks * 8, 8);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    if (prow >= g.rows) return;
    const long step = (long)gridDim.x * g.rows;
    for (int j = 0; j < g.iters; ++j) {
        int k = c8 + j * g.LPP;
        if (k >= chunks) break;
        int d = 0;
        while (d < a.n && k >= (a.part[d].channels + 7) / 8) { k -= (a.part[d].channels + 7) / 8; ++d; }
        if (d >= a.n) break;
        const seg_concat_part& pt = a.part[d];
        bf16* xp = reinterpret_cast<bf16*>(const_cast<void*>(pt.ptr)) + k * 8;
        const bf16* sp = dy + a.off[d] + k * 8;
        const int nv = min(8, pt.channels - k * 8);   // valid channels of this chunk
        for (long p = (long)blockIdx.x * g.rows + prow; p < P; p += step) {
            float v[8], d8[8];
            Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(sp + p * ldy), d8);
            if (pt.accumulate) {
                Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(xp + p * pt.ld), v);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += e < nv ? d8[e] : 0.f;
            *reinterpret_cast<uint4*>(xp + p * pt.ld) = Chunk<bf16>::pack(v);
        }
    }
}

template <typename T, typename S = float>
__global__ void prepare_input_k(const S* __restrict__ img, T* __restrict__ x, int N, int H, int W, int cin, int HP,
                                int WP, int CP) {
    // one thread per output pixel: its cin fp32 values (contiguous) -> one
    // 16-byte chunk per 8 channels (zeros in channel / spatial padding)
    constexpr int EPC = dt_traits<T>::EPC;
    const long total = (long)N * HP * WP;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int w = (int)(i % WP);
        const long t = i / WP;
        const int h = (int)(t % HP);
        const int n = (int)(t / HP);
        const bool in = h < H && w < W;
        const S* src = img + (((long)n * H + (in ? h : 0)) * W + (in ? w : 0)) * cin;
        T* dst = x + i * CP;
        for (int c0 = 0; c0 < CP; c0 += EPC) {
            float v[EPC];
#pragma unroll
            for (int e = 0; e < EPC; ++e) v[e] = (in && c0 + e < cin) ? (float)src[c0 + e] : 0.f;
            *reinterpret_cast<uint4*>(dst + c0) = Chunk<T>::pack(v);
        }
    }
}

// ---------------------------------------------------------------------------
// frozen-stat BatchNorm (+ ReLU)
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void bn_relu_fwd_k(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float inv, long P, int C, int cv, int relu) {
    // lane -> fixed 8-channel chunk(s) of a pixel (the bwd kernel's geometry):
    // the affine is loaded once per lane and the pixel walk has no 64-bit
    // division (the flat element loop ran at 1.4-2.1 TB/s)
    constexpr int EPC = dt_traits<T>::EPC;
    constexpr int MAXIT = 16 / EPC;
    const RedGeom g = red_geom(C, EPC);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    if (prow >= g.rows) return;
    float sc[MAXIT][EPC], sh[MAXIT][EPC];
#pragma unroll
    for (int j = 0; j < MAXIT; ++j)
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            const int c = (c8 + j * g.LPP) * EPC + e;
            const bool ok = j < g.iters && c < cv;
            sc[j][e] = ok ? gamma[c] * inv : 0.f;
            sh[j][e] = ok ? beta[c] : 0.f;
        }
    const long step = (long)gridDim.x * g.rows;
    for (long pix = (long)blockIdx.x * g.rows + prow; pix < P; pix += step) {
#pragma unroll
        for (int j = 0; j < MAXIT; ++j) {
            if (j >= g.iters) break;
            const int cc = c8 + j * g.LPP;
            if (cc >= g.CK) break;
            float v[EPC];
            Chunk<T>::unpack(ldc(x + pix * ldx + cc * EPC), v);
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                // one fma: the conv epilogues' second output (EpiParams.y2) computes the same
                float o = __builtin_fmaf(v[e], sc[j][e], sh[j][e]);
                if (relu) o = fmaxf(o, 0.f);
                v[e] = o;
            }
            stc(y + pix * ldy + cc * EPC, Chunk<T>::pack(v));
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_relu_bwd_k(const T* __restrict__ x, int ldx, const T* __restrict__ y, int ldy,
                                                     const T* __restrict__ dy, int lddy, T* __restrict__ dx, int lddx,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float inv, float* __restrict__ part, long P, int C, int cv,
                                                     int flags, float dkp, uint64_t dseed, int dcv) {
    // ReLU mask from y, or (y == null) re-derived from x with the forward's
    // own arithmetic (x * gamma*inv + beta > 0): 2 bytes per element less
    constexpr int EPC = dt_traits<T>::EPC;
    const bool relu = flags & 1, acc = flags & 2, remask = relu && !y;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const RedGeom g = red_geom(C, EPC);
    const int t = threadIdx.x;
    const int c8 = t % g.LPP, prow = t / g.LPP;
    const bool active = prow < g.rows;
    const long per = (P + gridDim.x - 1) / gridDim.x;
    const long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
    constexpr int MAXIT = 16 / EPC;
    float sg[MAXIT][EPC], sb[MAXIT][EPC], sc[MAXIT][EPC], sh[MAXIT][EPC];
#pragma unroll
    for (int j = 0; j < MAXIT; ++j)
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
            sg[j][e] = sb[j][e] = 0.f;
            // the per-lane affine, loaded once (channels >= cv: scale 0)
            const int c = (c8 + j * g.LPP) * EPC + e;
            const bool ok = j < g.iters && c < cv;
            sc[j][e] = ok ? gamma[c] * inv : 0.f;
            sh[j][e] = ok && remask ? beta[c] : 0.f;
        }
    if (active) {
        for (long pix = p0 + prow; pix < p1; pix += g.rows) {
            const uint64_t dbase = (uint64_t)pix * dcv;
#pragma unroll
            for (int j = 0; j < MAXIT; ++j) {
                if (j >= g.iters) break;
                const int cc = c8 + j * g.LPP;
                if (cc >= g.CK) break;
                float xv[EPC], yv[EPC], d[EPC], old[EPC];
                Chunk<T>::unpack(ldc(x + pix * ldx + cc * EPC), xv);
                if (relu && !remask) Chunk<T>::unpack(ldc(y + pix * ldy + cc * EPC), yv);
                Chunk<T>::unpack(ldc(dy + pix * lddy + cc * EPC), d);
                if (acc) Chunk<T>::unpack(ldc(dx + pix * lddx + cc * EPC), old);
                const SegDropRun<EPC> drop(dseed, dbase + cc * EPC, dkp < 1.f);
#pragma unroll
                for (int e = 0; e < EPC; ++e) {
                    const int c = cc * EPC + e;
                    if (remask) yv[e] = xv[e] * sc[j][e] + sh[j][e];
                    float dz = (relu && !(yv[e] > 0.f)) ? 0.f : d[e];
                    if (c >= cv) dz = 0.f;
                    sb[j][e] += dz;
                    sg[j][e] += dz * xv[e];
                    d[e] = dz * sc[j][e];
                    if (acc) d[e] += old[e];
                    // dropout of the conv epilogue that produced x (no ReLU
                    // between): its gradient, same counter as the forward draw
                    if (dkp < 1.f) d[e] = c < dcv ? drop(d[e], dkp, e) : 0.f;
                }
                stc(dx + pix * lddx + cc * EPC, Chunk<T>::pack(d));
            }
        }
    }
#pragma unroll
    for (int j = 0; j < MAXIT; ++j) {
        const int cc = c8 + j * g.LPP;
        if (active && j < g.iters && cc < g.CK)
#pragma unroll
            for (int e = 0; e < EPC; ++e) {
                red[prow * 2 * C + cc * EPC + e] = sg[j][e];
                red[prow * 2 * C + C + cc * EPC + e] = sb[j][e];
            }
    }
    __syncthreads();
    for (int k = t; k < 2 * C; k += 256) {
        float s = 0.f;
        for (int r = 0; r < g.rows; ++r) s += red[r * 2 * C + k];
        part[(long)blockIdx.x * 2 * C + k] = s;
    }
}

// dgamma / dbeta from the per-block partial rows: 8 channels per block, the
// rows split over 32 thread groups (a thread per channel looping over all
// rows serialised ~2k dependent loads: 170 us per BN layer)
__global__ __launch_bounds__(256) void bn_finish_k(const float* __restrict__ part, int nrows, int C, int cv,
                                                   float inv, float* dgamma, float* dbeta) {
    __shared__ float sg[32][9], sb[32][9];
    const int cl = threadIdx.x & 7, rg = threadIdx.x >> 3;
    const int k = blockIdx.x * 8 + cl;
    float g = 0.f, b = 0.f;
    if (k < cv)
        for (int r = rg; r < nrows; r += 32) {
            g += part[(long)r * 2 * C + k];
            b += part[(long)r * 2 * C + C + k];
        }
    sg[rg][cl] = g;
    sb[rg][cl] = b;
    __syncthreads();
    if (threadIdx.x < 8 && k < cv) {
        float tg = 0.f, tb = 0.f;
        for (int r = 0; r < 32; ++r) {
            tg += sg[r][cl];
            tb += sb[r][cl];
        }
        dgamma[k] = tg * inv;
        dbeta[k] = tb;
    }
}

// per-tile partial rows [nrows][width] -> [groups][width]: rows r = g, g + groups, ...
__global__ __launch_bounds__(256) void part_rows_reduce_k(const float* __restrict__ part, int nrows, int width,
                                                          float* __restrict__ out, int groups) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    const int gi = blockIdx.y;
    if (c >= width) return;
    float s = 0.f;
    for (int r = gi; r < nrows; r += groups) s += part[(long)r * width + c];
    out[(long)gi * width + c] = s;
}

// ---------------------------------------------------------------------------
// resize_bilinear(align_corners=True)
// ---------------------------------------------------------------------------
// One block row = one output row (n, oy): the row's source rows and weight
// are computed once, threads walk (ox, c) with 32-bit index math (the 64-bit
// divisions of a flat-index decomposition dominated this pass).
template <typename T>
__global__ __launch_bounds__(256) void resize_fwd_k(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W,
                                                    int C, int OH, int OW) {
    const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
    const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
    const int row = blockIdx.x;                   // n * OH + oy
    const int n = row / OH, oh = row - n * OH;
    const float fy = oh * sh;
    const int y0 = (int)floorf(fy);
    const int y1 = min(y0 + 1, H - 1);
    const float ly = fy - y0;
    const T* r0 = x + ((long)n * H + y0) * W * C;
    const T* r1 = x + ((long)n * H + y1) * W * C;
    T* yr = y + (long)row * OW * C;
    const int rowlen = OW * C;
    for (int j = blockIdx.y * blockDim.x + threadIdx.x; j < rowlen; j += gridDim.y * blockDim.x) {
        const int ow = j / C, c = j - (j / C) * C;
        const float fx = ow * sw;
        const int x0 = (int)floorf(fx);
        const int x1 = min(x0 + 1, W - 1);
        const float lx = fx - x0;
        const float tl = to_f32(r0[x0 * C + c]), tr = to_f32(r0[x1 * C + c]);
        const float bl = to_f32(r1[x0 * C + c]), br = to_f32(r1[x1 * C + c]);
        // explicit fmas (the 8-channel kernel's arithmetic, whatever the contraction)
        // (the fp32 result is pinned before the 16-bit rounding: hipcc would
        // otherwise fold fma + fp16 conversion into one v_fma_mixlo_f16, a
        // single rounding the 8-channel kernel's packed form does not get)
        const float top = __builtin_fmaf(tr - tl, lx, tl), bot = __builtin_fmaf(br - bl, lx, bl);
        float r = __builtin_fmaf(bot - top, ly, top);
        asm volatile("" : "+v"(r));
        yr[j] = from_f32<T>(r);
    }
}

// The same with 8 channels per thread (C % 8 == 0, 16-byte aligned rows):
// 16-byte gathers and stores instead of 2-byte ones -- DeepLab's logits (2
// classes padded to 8) made the scalar form a 2-byte store stream at 0.15
// TB/s.  Per-channel arithmetic identical to resize_fwd_k (explicit fmas in
// both, so the compiler's contraction choices cannot differ).
template <typename T>
__global__ __launch_bounds__(256) void resize_fwd8_k(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W,
                                                     int C, int OH, int OW) {
    const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
    const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
    const int row = blockIdx.x;                   // n * OH + oy
    const int n = row / OH, oh = row - n * OH;
    const float fy = oh * sh;
    const int y0 = (int)floorf(fy);
    const int y1 = min(y0 + 1, H - 1);
    const float ly = fy - y0;
    const T* r0 = x + ((long)n * H + y0) * W * C;
    const T* r1 = x + ((long)n * H + y1) * W * C;
    T* yr = y + (long)row * OW * C;
    const int c8 = C / 8, nch = OW * c8;
    for (int j = blockIdx.y * blockDim.x + threadIdx.x; j < nch; j += gridDim.y * blockDim.x) {
        const int ow = j / c8, c = (j - ow * c8) * 8;
        const float fx = ow * sw;
        const int x0 = (int)floorf(fx);
        const int x1 = min(x0 + 1, W - 1);
        const float lx = fx - x0;
        float tl[8], tr[8], bl[8], br[8], o[8];
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(r0 + x0 * C + c), tl);
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(r0 + x1 * C + c), tr);
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(r1 + x0 * C + c), bl);
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(r1 + x1 * C + c), br);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float top = __builtin_fmaf(tr[k] - tl[k], lx, tl[k]), bot = __builtin_fmaf(br[k] - bl[k], lx, bl[k]);
            o[k] = __builtin_fmaf(bot - top, ly, top);
            asm volatile("" : "+v"(o[k]));
        }
        *reinterpret_cast<uint4*>(yr + ow * C + c) = Chunk<T>::pack(o);
    }
}

// Output positions o (of n_out) whose bilinear source pair (floor(o*s),
// min(floor(o*s)+1, n_in-1)) includes i: a contiguous range, found from a
// generous analytic bracket and then tested with the forward's own float
// arithmetic, so weights match resize_fwd_k exactly.
__device__ __forceinline__ void resize_src_range(int i, float s, int n_out, int& lo, int& hi) {
    if (s <= 0.f) {
        lo = 0;
        hi = n_out - 1;
        return;
    }
    lo = max(0, (int)floorf((i - 1) / s) - 1);
    hi = min(n_out - 1, (int)ceilf((i + 1) / s) + 1);
}

__device__ __forceinline__ float resize_weight(int o, int i, float s, int n_in) {
    const float f = o * s;
    const int a = (int)floorf(f);
    const int b = min(a + 1, n_in - 1);
    const float l = f - a;
    return (a == i ? 1.f - l : 0.f) + (b == i ? l : 0.f);
}

// Gradient as a gather (deterministic, no atomics): dx[n, y, x, c] =
// sum over the output rows / columns that read (y, x) of wy * wx * dy.
template <typename T>
__global__ __launch_bounds__(256) void resize_bwd_k(const T* __restrict__ dy, float* __restrict__ dx, int N, int H,
                                                    int W, int C, int OH, int OW) {
    const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
    const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
    const int row = blockIdx.x;                   // n * H + y
    const int n = row / H, yy = row - n * H;
    int oy_lo, oy_hi;
    resize_src_range(yy, sh, OH, oy_lo, oy_hi);
    const int rowlen = W * C;
    for (int j = blockIdx.y * blockDim.x + threadIdx.x; j < rowlen; j += gridDim.y * blockDim.x) {
        const int xx = j / C, c = j - (j / C) * C;
        int ox_lo, ox_hi;
        resize_src_range(xx, sw, OW, ox_lo, ox_hi);
        float acc = 0.f;
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const float wy = resize_weight(oy, yy, sh, H);
            if (wy == 0.f) continue;
            const T* dr = dy + ((long)n * OH + oy) * OW * C + c;
            float racc = 0.f;
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const float wx = resize_weight(ox, xx, sw, W);
                if (wx != 0.f) racc = __builtin_fmaf(wx, to_f32(dr[ox * C]), racc);
            }
            acc = __builtin_fmaf(wy, racc, acc);
        }
        dx[(long)row * rowlen + j] = acc;
    }
}

// The gather with 8 channels per thread (C % 8 == 0): 16-byte dy loads, two
// 16-byte dx stores; per-channel summation order identical to resize_bwd_k.
template <typename T>
__global__ __launch_bounds__(256) void resize_bwd8_k(const T* __restrict__ dy, float* __restrict__ dx, int N, int H,
                                                     int W, int C, int OH, int OW) {
    const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
    const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
    const int row = blockIdx.x;                   // n * H + y
    const int n = row / H, yy = row - n * H;
    int oy_lo, oy_hi;
    resize_src_range(yy, sh, OH, oy_lo, oy_hi);
    const int c8 = C / 8, nch = W * c8;
    for (int j = blockIdx.y * blockDim.x + threadIdx.x; j < nch; j += gridDim.y * blockDim.x) {
        const int xx = j / c8, c = (j - xx * c8) * 8;
        int ox_lo, ox_hi;
        resize_src_range(xx, sw, OW, ox_lo, ox_hi);
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const float wy = resize_weight(oy, yy, sh, H);
            if (wy == 0.f) continue;
            const T* dr = dy + ((long)n * OH + oy) * OW * C + c;
            float racc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const float wx = resize_weight(ox, xx, sw, W);
                if (wx != 0.f) {
                    float d[8];
                    Chunk<T>::unpack(*reinterpret_cast<const uint4*>(dr + ox * C), d);
#pragma unroll
                    for (int k = 0; k < 8; ++k) racc[k] = __builtin_fmaf(wx, d[k], racc[k]);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = __builtin_fmaf(wy, racc[k], acc[k]);
        }
        float* dp = dx + ((long)row * W + xx) * C + c;
        *reinterpret_cast<float4*>(dp) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(dp + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
}

// ---------------------------------------------------------------------------
// softmax cross-entropy (fused forward + backward) and prediction
// ---------------------------------------------------------------------------
constexpr int XENT_MAXC = 16;

template <typename T, bool SOFT>
__global__ __launch_bounds__(256) void xent_k(const T* __restrict__ logits, int ld, const uint8_t* __restrict__ lab_idx,
                                              const float* __restrict__ lab_soft, int N, int H, int W, int C,
                                              int vh, int vw, float scale, T* __restrict__ dlog, int ldd,
                                              float* __restrict__ part) {
    __shared__ float wsum[4];
    const long P = (long)N * H * W;
    float lsum = 0.f;
    for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
        const int w = (int)(p % W);
        const int h = (int)((p / W) % H);
        const bool valid = h < vh && w < vw;
        float z[XENT_MAXC];
        float mx = -INFINITY;
        for (int c = 0; c < C; ++c) {
            z[c] = to_f32(logits[p * ld + c]);
            mx = fmaxf(mx, z[c]);
        }
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += __expf(z[c] - mx);
        const float lse = mx + __logf(se);
        const float inv = 1.f / se;
        float ysum = 0.f, yz = 0.f;
        for (int c = 0; c < C; ++c) {
            float yc;
            if (SOFT) yc = lab_soft[p * C + c];
            else yc = (lab_idx[p] == c) ? 1.f : 0.f;
            ysum += yc;
            yz += yc * z[c];
        }
        for (int c = 0; c < C; ++c) {
            float yc;
            if (SOFT) yc = lab_soft[p * C + c];
            else yc = (lab_idx[p] == c) ? 1.f : 0.f;
            const float g = valid ? (__expf(z[c] - mx) * inv * ysum - yc) * scale : 0.f;
            dlog[p * ldd + c] = from_f32<T>(g);
        }
        for (int c = C; c < ldd; ++c) dlog[p * ldd + c] = from_f32<T>(0.f);
        if (valid) lsum += ysum * lse - yz;
    }
    // wave64 then workgroup reduction
    for (int off = 32; off > 0; off >>= 1) lsum += __shfl_down(lsum, off, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = lsum;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

__global__ void sum_k(const float* __restrict__ part, int n, float* out) {
    __shared__ float s[256];
    float v = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) v += part[i];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = s[0];
}

template <typename T>
__global__ void argmax_k(const T* __restrict__ logits, int ld, int C, long P, int64_t* __restrict__ pred) {
    for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
        float best = to_f32(logits[p * ld]);
        int arg = 0;
        for (int c = 1; c < C; ++c) {
            const float v = to_f32(logits[p * ld + c]);
            if (v > best) { best = v; arg = c; }
        }
        pred[p] = arg;
    }
}

// tf.nn.softmax over the channel dim (Network/utils/utils.py:54 eval path):
// max-subtracted, padding channels >= C written as 0.
template <typename T>
__global__ void softmax_k(const T* __restrict__ x, int ldx, int C, long P, T* __restrict__ y, int ldy) {
    for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
        float mx = to_f32(x[p * ldx]);
        for (int c = 1; c < C; ++c) mx = fmaxf(mx, to_f32(x[p * ldx + c]));
        float s = 0.f;
        for (int c = 0; c < C; ++c) s += expf(to_f32(x[p * ldx + c]) - mx);
        const float inv = 1.f / s;
        for (int c = 0; c < ldy; ++c)
            y[p * ldy + c] = from_f32<T>(c < C ? expf(to_f32(x[p * ldx + c]) - mx) * inv : 0.f);
    }
}

__global__ void confusion_k(const int64_t* __restrict__ pred, const uint8_t* __restrict__ lab, int N, int H, int W,
                            int vh, int vw, int C, unsigned long long* conf) {
    const long P = (long)N * H * W;
    for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
        const int w = (int)(p % W);
        const int h = (int)((p / W) % H);
        if (h >= vh || w >= vw) continue;
        const int t = lab[p], q = (int)pred[p];
        if (t < C && q < C) atomicAdd(conf + t * C + q, 1ull);
    }
}

// ---------------------------------------------------------------------------
// TF1 Adam over a flat fp32 buffer (4 params / lane / iteration)
// ---------------------------------------------------------------------------
__global__ void adam_k(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                       long n, float lr_t, float b1, float b2, float eps, float gs) {
    const long n4 = n / 4;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
        float4 pp = reinterpret_cast<float4*>(p)[i];
        const float4 gg = reinterpret_cast<const float4*>(g)[i];
        float4 mm = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
#define ADAM1(c)                                                  \
    {                                                             \
        const float gc = gg.c * gs;                               \
        mm.c = b1 * mm.c + (1.f - b1) * gc;                       \
        vv.c = b2 * vv.c + (1.f - b2) * gc * gc;                  \
        pp.c = pp.c - lr_t * mm.c / (sqrtf(vv.c) + eps);          \
    }
        ADAM1(x) ADAM1(y) ADAM1(z) ADAM1(w)
#undef ADAM1
        reinterpret_cast<float4*>(p)[i] = pp;
        reinterpret_cast<float4*>(m)[i] = mm;
        reinterpret_cast<float4*>(v)[i] = vv;
    }
    for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const float gc = g[i] * gs;
        m[i] = b1 * m[i] + (1.f - b1) * gc;
        v[i] = b2 * v[i] + (1.f - b2) * gc * gc;
        p[i] = p[i] - lr_t * m[i] / (sqrtf(v[i]) + eps);
    }
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
#define DISPATCH_T(dtype, KERNEL_CALL)                  \
    do {                                                \
        if ((dtype) == SEG_BF16) {                      \
            typedef bf16 T;                             \
            KERNEL_CALL;                                \
        } else if ((dtype) == SEG_F32) {                \
            typedef float T;                            \
            KERNEL_CALL;                                \
        } else if ((dtype) == SEG_F16) {                \
            typedef f16 T;                              \
            KERNEL_CALL;                                \
        } else                                          \
            return SEG_EINVAL;                          \
    } while (0)

static inline int epc_of(int dtype) { return dtype == SEG_F32 ? 4 : 8; }

extern "C" size_t seg_bias_grad_workspace(long P, int K) {
    (void)P;
    return (size_t)RED_BLOCKS * 2 * K * sizeof(float);
}

// Enough workgroups to keep many rows in flight: each covers about two passes
// of its row groups (64 pixels at K = 64, 2 pixels at K = 4096), capped.
static int red_blocks(long P, int K, int epc) {
    const RedGeom g = red_geom(K, epc);
    const long per = 2L * g.rows;
    long b = (P + per - 1) / per;
    // the fp32 partial rows (blocks x K) are written and read back: for wide
    // K cap them at ~4 MB (conv6 / conv7 BiasAddGrad, K = 4096: 936 blocks of
    // 2 pixels each wrote 15 MB of partials for a 3.8 MB input)
    const long cap = std::max(64L, std::min((long)RED_BLOCKS, (1L << 20) / K));
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

extern "C" int seg_bias_relu_bwd(const void* dy, int ld_dy, const void* y, int ld_y, void* dz, int ld_dz, float* dbias,
                                 long P, int K, int k_valid, int relu, float scale, int dtype, void* ws,
                                 size_t ws_bytes, void* stream) {
    if (!dy || !dz || (relu && !y) || (K & 7) || P <= 0) return SEG_EINVAL;
    if (K > 4096) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (dbias && !relu && scale == 1.f && dz == dy && K / epc_of(dtype) >= 64 && (ld_dy % epc_of(dtype)) == 0) {
        // plain column sums of a wide dy
        const int gx = (K / epc_of(dtype) + 63) / 64;
        long rs = std::max(1L, std::min((long)RED_BLOCKS, std::min(2048L / gx, (P + 63) / 64)));
        const int per = (int)((P + rs - 1) / rs);
        rs = (P + per - 1) / per;
        float* part = (float*)ws;
        if (!ws || ws_bytes < (size_t)rs * K * sizeof(float)) return SEG_EWORKSPACE;
        DISPATCH_T(dtype, hipLaunchKernelGGL(col_sum_k<T>, dim3(gx, (unsigned)rs), dim3(256), 0, s, (const T*)dy, ld_dy,
                                             part, P, K, per));
        SEG_CHECK_LAUNCH();
        hipLaunchKernelGGL(reduce_rows_k, dim3((k_valid + 7) / 8), dim3(256), 0, s, part, (int)rs, K, k_valid, dbias);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const int nb = red_blocks(P, K, epc_of(dtype));
    const RedGeom g = red_geom(K, epc_of(dtype));
    const size_t shm = (size_t)g.rows * K * sizeof(float);
    float* part = (float*)ws;
    if (!ws || ws_bytes < (size_t)nb * K * sizeof(float)) return SEG_EWORKSPACE;
    DISPATCH_T(dtype, hipLaunchKernelGGL(bias_relu_bwd_k<T>, dim3(nb), dim3(256), shm, s, (const T*)dy, ld_dy,
                                         (const T*)y, ld_y, (T*)dz, ld_dz, part, P, K, relu, scale));
    SEG_CHECK_LAUNCH();
    if (dbias) {
        hipLaunchKernelGGL(reduce_rows_k, dim3((k_valid + 7) / 8), dim3(256), 0, s, part, nb, K, k_valid, dbias);
        SEG_CHECK_LAUNCH();
    }
    return SEG_OK;
}

extern "C" int seg_maxpool2x2_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int ldy, int dtype,
                                  void* stream) {
    if (!x || !y || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2) return SEG_EINVAL;
    const long total = (long)N * (H / 2) * (W / 2) * (C / epc_of(dtype));
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, (T*)y, N, H, W, C, ldx, ldy));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_maxpool2x2_bwd(const void* x, const void* y, const void* dy, void* dx, int N, int H, int W, int C,
                                  int ldx, int ldy, int relu_mask, int dtype, void* stream) {
    (void)y;
    if (!x || !dy || !dx || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2) return SEG_EINVAL;
    const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / epc_of(dtype));
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, (const T*)dy, (T*)dx, N, H, W, C, ldx, ldy,
                                         relu_mask));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_maxpool2x2_fwd_argmax(const void* x, void* y, void* idx, int N, int H, int W, int C, int ldx,
                                         int ldy, int dtype, void* stream) {
    if (!x || !y || !idx || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2 || N < 1 || (uintptr_t)idx % 8)
        return SEG_EINVAL;
    const long total = (long)N * (H / 2) * (W / 2) * (C / epc_of(dtype));
    if ((long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / epc_of(dtype)) >= (1L << 31)) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_fwd_idx_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, (T*)y, (unsigned char*)idx, H, W, C, ldx,
                                         ldy, (unsigned)(W / 2), (unsigned)(C / epc_of(dtype)), (unsigned)total));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_maxpool2x2_bwd_argmax(const void* idx, const void* dy, void* dx, int N, int H, int W, int C,
                                         int ldx, int ldy, int relu_mask, int dtype, void* stream) {
    if (!idx || !dy || !dx || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2 || N < 1 || (uintptr_t)idx % 8)
        return SEG_EINVAL;
    const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / epc_of(dtype));
    if (total >= (1L << 31)) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(maxpool_bwd_idx_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const unsigned char*)idx, (const T*)dy, (T*)dx, H, W,
                                         C, ldx, ldy, relu_mask, (unsigned)((W + 1) / 2),
                                         (unsigned)(C / epc_of(dtype)), (unsigned)total));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_avgpool2x2_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int ldy, int dtype,
                                  void* stream) {
    if (!x || !y || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2) return SEG_EINVAL;
    const long total = (long)N * (H / 2) * (W / 2) * (C / epc_of(dtype));
    DISPATCH_T(dtype, hipLaunchKernelGGL(avgpool_fwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, (T*)y, N, H, W, C, ldx, ldy));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_avgpool2x2_bwd(const void* dy, void* dx, int N, int H, int W, int C, int ldx, int ldy, int dtype,
                                  void* stream) {
    if (!dy || !dx || (C & 7) || (ldx & 7) || (ldy & 7) || H < 2 || W < 2) return SEG_EINVAL;
    const long total = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / epc_of(dtype));
    DISPATCH_T(dtype, hipLaunchKernelGGL(avgpool_bwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)dy, (T*)dx, N, H, W, C, ldx, ldy));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_add(const void* a, const void* b, void* y, long n, int dtype, void* stream) {
    if (!a || !b || !y || n < 0) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(add_k<T>, dim3(seg_grid_1d(n, 256)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)a, (const T*)b, (T*)y, n));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_dropout_fwd(const void* x, void* y, long n, float kp, uint64_t seed, int dtype, void* stream) {
    if (!x || !y || !(kp > 0.f) || kp > 1.f) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(dropout_k<T>, dim3(seg_grid_1d(n, 256)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, (T*)y, n, kp, seed));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_dropout_bwd(const void* dy, void* dx, long n, float kp, uint64_t seed, int dtype, void* stream) {
    // the same mask and 1/kp scale: dx = dy / kp * floor(kp + U)
    return seg_dropout_fwd(dy, dx, n, kp, seed, dtype, stream);
}

namespace seg {
}

extern "C" int seg_dropout_bwd_ch(const void* dy, int ldy, void* dz, int ldz, long P, int C, int cv, float kp,
                                  uint64_t seed, int dtype, void* stream) {
    if (!dy || !dz || !(kp > 0.f) || kp > 1.f || (C & 7) || cv > C || ldy < C || ldz < C) return SEG_EINVAL;
    if (C > 4096) return SEG_EINVAL;
    const RedGeom g = red_geom(C, epc_of(dtype));
    const long chunks = P * (long)g.CK;
    if (g_dropout_flat && chunks < (1L << 31) - 256) {
        const int CK = g.CK;
        DISPATCH_T(dtype, hipLaunchKernelGGL(dropout_ch_flat_k<T>, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0,
                                             (hipStream_t)stream, (const T*)dy, ldy, (T*)dz, ldz, (int)P, CK, cv, kp,
                                             seed));
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const long blocks = std::max<long>(1, std::min<long>((P + g.rows - 1) / g.rows, 16384));
    DISPATCH_T(dtype, hipLaunchKernelGGL(dropout_ch_k<T>, dim3((unsigned)blocks), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)dy, ldy, (T*)dz, ldz, P, C, cv, kp, seed));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_fill(void* y, long n, float v, int dtype, void* stream) {
    if (!y) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(fill_k<T>, dim3(seg_grid_1d(n, 256)), dim3(256), 0, (hipStream_t)stream,
                                         (T*)y, n, v));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

// any non-finite element of n fp32 values -> *flag = 1 (dynamic loss scaling:
// a step whose scaled gradients overflowed is skipped)
__global__ void check_finite_k(const float* __restrict__ g, long n, int* __restrict__ flag) {
    bool bad = false;
    const long n4 = n / 4;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
        const float4 v = reinterpret_cast<const float4*>(g)[i];
        bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        bad |= !isfinite(g[i]);
    if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1;
}

extern "C" int seg_check_finite(const float* g, long n, int* flag, void* stream) {
    if (!g || !flag || n < 0 || ((uintptr_t)g & 15)) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(flag, 0, sizeof(int), s) != hipSuccess) return SEG_ELAUNCH;
    if (n == 0) return SEG_OK;
    hipLaunchKernelGGL(check_finite_k, dim3(seg_grid_1d(n / 4 + 1, 256, 4096)), dim3(256), 0, s, g, n, flag);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_axpy(float* y, const float* x, float alpha, long n, void* stream) {
    if (!y || !x || n < 0) return SEG_EINVAL;
    if (n == 0) return SEG_OK;
    hipLaunchKernelGGL(axpy_k, dim3(seg_grid_1d(n, 256)), dim3(256), 0, (hipStream_t)stream, y, x, alpha, n);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_cast(const void* x, int xd, void* y, int yd, long n, void* stream) {
    if (!x || !y) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int g = seg_grid_1d(n, 256);
    if (xd == SEG_F32 && yd == SEG_BF16) hipLaunchKernelGGL((cast_k<float, bf16>), dim3(g), dim3(256), 0, s, (const float*)x, (bf16*)y, n);
    else if (xd == SEG_BF16 && yd == SEG_F32) hipLaunchKernelGGL((cast_k<bf16, float>), dim3(g), dim3(256), 0, s, (const bf16*)x, (float*)y, n);
    else if (xd == SEG_F32 && yd == SEG_F32) hipLaunchKernelGGL((cast_k<float, float>), dim3(g), dim3(256), 0, s, (const float*)x, (float*)y, n);
    else if (xd == SEG_BF16 && yd == SEG_BF16) hipLaunchKernelGGL((cast_k<bf16, bf16>), dim3(g), dim3(256), 0, s, (const bf16*)x, (bf16*)y, n);
    else if (xd == SEG_F32 && yd == SEG_F16) hipLaunchKernelGGL((cast_k<float, f16>), dim3(g), dim3(256), 0, s, (const float*)x, (f16*)y, n);
    else if (xd == SEG_F16 && yd == SEG_F32) hipLaunchKernelGGL((cast_k<f16, float>), dim3(g), dim3(256), 0, s, (const f16*)x, (float*)y, n);
    else if (xd == SEG_F16 && yd == SEG_F16) hipLaunchKernelGGL((cast_k<f16, f16>), dim3(g), dim3(256), 0, s, (const f16*)x, (f16*)y, n);
    else return SEG_EINVAL;
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_copy_channels(const void* x, int ldx, void* y, int ldy, long P, int C, int dtype, void* stream) {
    if (!x || !y || (C & 7) || (ldx & 7) || (ldy & 7)) return SEG_EINVAL;
    const long total = P * (C / epc_of(dtype));
    DISPATCH_T(dtype, hipLaunchKernelGGL(copy_channels_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, ldx, (T*)y, ldy, P, C));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}


static int concat_args(const seg_concat_part* parts, int n, ConcatArgs* a) {
    if (!parts || n <= 0 || n > SEG_CONCAT_MAX) return SEG_EINVAL;
    a->n = n;
    a->off[0] = 0;
    for (int i = 0; i < n; ++i) {
        if (!parts[i].ptr || parts[i].channels <= 0 || (parts[i].ld & 7) || parts[i].ld < parts[i].channels)
            return SEG_EINVAL;
        a->part[i] = parts[i];
        a->off[i + 1] = a->off[i] + parts[i].channels;
    }
    return SEG_OK;
}

extern "C" int seg_concat_fwd(const seg_concat_part* parts, int nparts, void* y, int ldy, int ychannels, long P,
                              int dtype, void* stream) {
    ConcatArgs a;
    int st = concat_args(parts, nparts, &a);
    if (st) return st;
    if (!y || (ldy & 7) || (ychannels & 7) || ychannels < a.off[nparts] || ldy < ychannels) return SEG_EINVAL;
    bool aligned = dtype == SEG_BF16;
    for (int i = 0; i < nparts; ++i) aligned = aligned && (a.off[i] & 7) == 0;
    if (aligned) {
        const RedGeom g = red_geom(ychannels, 8);
        const long blocks = std::max<long>(1, std::min<long>((P + g.rows - 1) / g.rows, 16384));
        hipLaunchKernelGGL(concat_fwd_fast_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, (bf16*)y,
                           ldy, ychannels / 8, P);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const long total = P * (ychannels / 8);
    DISPATCH_T(dtype, hipLaunchKernelGGL(concat_fwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, a, (T*)y, ldy, ychannels / 8, P));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_concat_bwd(const void* dy, int ldy, const seg_concat_part* parts, int nparts, long P, int dtype,
                              void* stream) {
    ConcatArgs a;
    int st = concat_args(parts, nparts, &a);
    if (st) return st;
    if (!dy || ldy < a.off[nparts]) return SEG_EINVAL;
    int chunks = 0;
    for (int i = 0; i < nparts; ++i) chunks += (parts[i].channels + 7) / 8;
    bool aligned = dtype == SEG_BF16 && (ldy & 7) == 0;
    for (int i = 0; i < nparts; ++i) aligned = aligned && (a.off[i] & 7) == 0;
    if (aligned) {
        const RedGeom g = red_geom(chunks * 8, 8);
        const long blocks = std::max<long>(1, std::min<long>((P + g.rows - 1) / g.rows, 16384));
        hipLaunchKernelGGL(concat_bwd_fast_k, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                           (const bf16*)dy, ldy, a, chunks, P);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const long total = P * chunks;
    DISPATCH_T(dtype, hipLaunchKernelGGL(concat_bwd_k<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)dy, ldy, a, (const int*)nullptr, P, chunks));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_prepare_input(const float* img, void* x, int N, int H, int W, int cin, int HP, int WP, int CP,
                                 int dtype, void* stream) {
    if (!img || !x || HP < H || WP < W || CP < cin || CP % (dtype == SEG_F32 ? 4 : 8)) return SEG_EINVAL;
    const long total = (long)N * HP * WP * CP;
    DISPATCH_T(dtype, hipLaunchKernelGGL(prepare_input_k<T>, dim3(seg_grid_1d(total / CP + 1, 256)), dim3(256), 0,
                                         (hipStream_t)stream, img, (T*)x, N, H, W, cin, HP, WP, CP));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_prepare_input_u8(const uint8_t* img, void* x, int N, int H, int W, int cin, int HP, int WP, int CP,
                                    int dtype, void* stream) {
    if (!img || !x || HP < H || WP < W || CP < cin || CP % (dtype == SEG_F32 ? 4 : 8)) return SEG_EINVAL;
    const long total = (long)N * HP * WP * CP;
    DISPATCH_T(dtype, hipLaunchKernelGGL((prepare_input_k<T, uint8_t>), dim3(seg_grid_1d(total / CP + 1, 256)),
                                         dim3(256), 0, (hipStream_t)stream, img, (T*)x, N, H, W, cin, HP, WP, CP));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_bn_relu_fwd(const void* x, int ldx, void* y, int ldy, const float* gamma, const float* beta,
                               float eps, long P, int C, int cv, int relu, int dtype, void* stream) {
    if (!x || !y || !gamma || !beta || (C & 7) || C > 4096) return SEG_EINVAL;
    const float inv = 1.0f / sqrtf(1.0f + eps);
    const RedGeom g = red_geom(C, epc_of(dtype));
    const long blocks = std::min<long>((P + g.rows - 1) / g.rows, 16384);
    DISPATCH_T(dtype, hipLaunchKernelGGL(bn_relu_fwd_k<T>, dim3((unsigned)std::max<long>(blocks, 1)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, ldx, (T*)y, ldy, gamma, beta, inv, P, C, cv,
                                         relu));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

static int bn_relu_bwd_impl(const void* x, int ldx, const void* y, int ldy, const void* dy, int lddy, void* dx,
                            int lddx, const float* gamma, const float* beta, float eps, float* dgamma, float* dbeta,
                            long P, int C, int cv, int flags, int dtype, void* ws, size_t ws_bytes, void* stream,
                            float dkp, uint64_t dseed, int dcv) {
    if (!x || !dy || !dx || !gamma || !dgamma || !dbeta || (C & 7) || (flags & ~3)) return SEG_EINVAL;
    if ((flags & 1) && !y && !beta) return SEG_EINVAL;
    if (C > 4096) return SEG_EINVAL;
    const int nb = red_blocks(P, C, epc_of(dtype));
    if (!ws || ws_bytes < (size_t)nb * 2 * C * sizeof(float)) return SEG_EWORKSPACE;
    const float inv = 1.0f / sqrtf(1.0f + eps);
    const RedGeom g = red_geom(C, epc_of(dtype));
    const size_t shm = (size_t)g.rows * 2 * C * sizeof(float);
    if (shm > 64 * 1024) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    DISPATCH_T(dtype, hipLaunchKernelGGL(bn_relu_bwd_k<T>, dim3(nb), dim3(256), shm, s, (const T*)x, ldx, (const T*)y,
                                         ldy, (const T*)dy, lddy, (T*)dx, lddx, gamma, beta, inv, (float*)ws, P, C, cv, flags,
                                         dkp, dseed, dcv));
    SEG_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_finish_k, dim3((cv + 7) / 8), dim3(256), 0, s, (const float*)ws, nb, C, cv, inv, dgamma, dbeta);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_bn_relu_bwd(const void* x, int ldx, const void* y, int ldy, const void* dy, int lddy, void* dx,
                               int lddx, const float* gamma, const float* beta, float eps, float* dgamma,
                               float* dbeta, long P, int C, int cv, int flags, int dtype, void* ws, size_t ws_bytes,
                               void* stream) {
    return bn_relu_bwd_impl(x, ldx, y, ldy, dy, lddy, dx, lddx, gamma, beta, eps, dgamma, dbeta, P, C, cv, flags,
                            dtype, ws, ws_bytes, stream, 1.f, 0, 0);
}

extern "C" int seg_bn_relu_dropout_bwd(const void* x, int ldx, const void* y, int ldy, const void* dy, int lddy,
                                       void* dx, int lddx, const float* gamma, const float* beta, float eps,
                                       float* dgamma, float* dbeta, long P, int C, int cv, int flags,
                                       float keep_prob, uint64_t seed, int drop_c_valid, int dtype, void* ws,
                                       size_t ws_bytes, void* stream) {
    // the dropout gradient applies to this BN's contribution alone: no accumulation
    if ((flags & 2) || !(keep_prob > 0.f && keep_prob <= 1.f) || drop_c_valid <= 0 || drop_c_valid > C)
        return SEG_EINVAL;
    return bn_relu_bwd_impl(x, ldx, y, ldy, dy, lddy, dx, lddx, gamma, beta, eps, dgamma, dbeta, P, C, cv, flags,
                            dtype, ws, ws_bytes, stream, keep_prob, seed, drop_c_valid);
}

// ---------------------------------------------------------------------------
// Global average pooling (tflearn global_avg_pool = tf.reduce_mean(x, [1, 2]),
// Network/utils/utils.py:312; DeepLab's image-pooling ASPP branch,
// Network/model/DeepLabv3Plus.py:215-225) and its broadcast counterpart.
// reduce: grid (N, slices); a thread owns one 8-channel chunk and a strided
// pixel subset, the block combines equal chunks through LDS and adds its
// partial sum into an fp32 workspace (one atomic per channel per block); a
// second pass writes scale * sum in the compute dtype.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void spatial_sum_k(const T* __restrict__ x, int ldx, float* __restrict__ acc,
                                                     int HW, int C) {
    constexpr int EPC = dt_traits<T>::EPC;
    __shared__ float red[256][EPC + 1];
    const int CK = C / EPC;                       // <= 256 (checked by the entry point)
    const int n = blockIdx.y;
    const int prow = 256 / CK;                    // pixel rows per block step
    const int t = threadIdx.x, ck = t % CK, pr = t / CK;
    float a[EPC];
#pragma unroll
    for (int e = 0; e < EPC; ++e) a[e] = 0.f;
    if (pr < prow) {
        for (long pix = (long)blockIdx.x * prow + pr; pix < HW; pix += (long)gridDim.x * prow) {
            float v[EPC];
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(x + ((long)n * HW + pix) * ldx + ck * EPC), v);
#pragma unroll
            for (int e = 0; e < EPC; ++e) a[e] += v[e];
        }
    }
#pragma unroll
    for (int e = 0; e < EPC; ++e) red[t][e] = a[e];
    __syncthreads();
    if (t < CK) {
        for (int r = 1; r < prow; ++r)
#pragma unroll
            for (int e = 0; e < EPC; ++e) a[e] += red[t + r * CK][e];
#pragma unroll
        for (int e = 0; e < EPC; ++e) atomicAdd(acc + (long)n * C + t * EPC + e, a[e]);
    }
}

template <typename T>
__global__ void scale_cast_k(const float* __restrict__ acc, T* __restrict__ y, long n, float scale) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = from_f32<T>(acc[i] * scale);
}

template <typename T>
__global__ void spatial_bcast_k(const T* __restrict__ x, T* __restrict__ y, int ldy, long NHW, int HW, int C,
                                float scale) {
    constexpr int EPC = dt_traits<T>::EPC;
    const int CK = C / EPC;
    const long total = NHW * CK;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const long p = i / CK;
        const int cc = (int)(i - p * CK);
        const long n = p / HW;
        float v[EPC];
        Chunk<T>::unpack(*reinterpret_cast<const uint4*>(x + n * C + cc * EPC), v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) v[e] *= scale;
        *reinterpret_cast<uint4*>(y + p * ldy + cc * EPC) = Chunk<T>::pack(v);
    }
}

extern "C" int seg_spatial_reduce(const void* x, int ldx, void* y, int N, int H, int W, int C, float scale,
                                  float* ws, int dtype, void* stream) {
    if (!x || !y || !ws || N <= 0 || H <= 0 || W <= 0 || (C & 7) || ldx < C || (ldx & 7)) return SEG_EINVAL;
    if (C / epc_of(dtype) > 256) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(ws, 0, (size_t)N * C * sizeof(float), s) != hipSuccess) return SEG_ELAUNCH;
    const int HW = H * W;
    const int slices = std::max(1, std::min(256, (HW + 255) / 256));
    DISPATCH_T(dtype, hipLaunchKernelGGL(spatial_sum_k<T>, dim3(slices, N), dim3(256), 0, s, (const T*)x, ldx, ws,
                                         HW, C));
    DISPATCH_T(dtype, hipLaunchKernelGGL(scale_cast_k<T>, dim3(seg_grid_1d((long)N * C, 256)), dim3(256), 0, s, ws,
                                         (T*)y, (long)N * C, scale));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_spatial_broadcast(const void* x, void* y, int ldy, int N, int H, int W, int C, float scale,
                                     int dtype, void* stream) {
    if (!x || !y || N <= 0 || H <= 0 || W <= 0 || (C & 7) || ldy < C || (ldy & 7)) return SEG_EINVAL;
    const long NHW = (long)N * H * W;
    DISPATCH_T(dtype, hipLaunchKernelGGL(spatial_bcast_k<T>, dim3(seg_grid_1d(NHW * (C / 8), 256)), dim3(256), 0,
                                         (hipStream_t)stream, (const T*)x, (T*)y, ldy, NHW, H * W, C, scale));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_resize_bilinear_fwd(const void* x, void* y, int N, int H, int W, int C, int OH, int OW, int dtype,
                                       void* stream) {
    if (!x || !y || N <= 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0) return SEG_EINVAL;
    if ((long)W * C > 0x7fffffffL || (long)OW * C > 0x7fffffffL || (long)N * OH > 0x7fffffffL) return SEG_EINVAL;
    const int rowlen = OW * C;
    if (dtype != SEG_F32 && C % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
        const dim3 grid8((unsigned)(N * OH), (unsigned)std::min((rowlen / 8 + 255) / 256, 64));
        if (dtype == SEG_BF16)
            hipLaunchKernelGGL(resize_fwd8_k<bf16>, grid8, dim3(256), 0, (hipStream_t)stream, (const bf16*)x, (bf16*)y,
                               N, H, W, C, OH, OW);
        else
            hipLaunchKernelGGL(resize_fwd8_k<f16>, grid8, dim3(256), 0, (hipStream_t)stream, (const f16*)x, (f16*)y, N,
                               H, W, C, OH, OW);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const dim3 grid((unsigned)(N * OH), (unsigned)std::min((rowlen + 255) / 256, 64));
    DISPATCH_T(dtype, hipLaunchKernelGGL(resize_fwd_k<T>, grid, dim3(256), 0, (hipStream_t)stream, (const T*)x, (T*)y,
                                         N, H, W, C, OH, OW));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_resize_bilinear_bwd(const void* dy, float* dx, int N, int H, int W, int C, int OH, int OW,
                                       int dtype, void* stream) {
    if (!dy || !dx || N <= 0 || H <= 0 || W <= 0 || C <= 0 || OH <= 0 || OW <= 0) return SEG_EINVAL;
    if ((long)W * C > 0x7fffffffL || (long)OW * C > 0x7fffffffL || (long)N * H > 0x7fffffffL) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int rowlen = W * C;                       // every dx element is written: no memset
    if (dtype != SEG_F32 && C % 8 == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0) {
        const dim3 grid8((unsigned)(N * H), (unsigned)std::min((rowlen / 8 + 255) / 256, 64));
        if (dtype == SEG_BF16)
            hipLaunchKernelGGL(resize_bwd8_k<bf16>, grid8, dim3(256), 0, s, (const bf16*)dy, dx, N, H, W, C, OH, OW);
        else
            hipLaunchKernelGGL(resize_bwd8_k<f16>, grid8, dim3(256), 0, s, (const f16*)dy, dx, N, H, W, C, OH, OW);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    const dim3 grid((unsigned)(N * H), (unsigned)std::min((rowlen + 255) / 256, 64));
    DISPATCH_T(dtype, hipLaunchKernelGGL(resize_bwd_k<T>, grid, dim3(256), 0, s, (const T*)dy, dx, N, H, W, C, OH,
                                         OW));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" size_t seg_xent_workspace(int N, int H, int W) {
    (void)N; (void)H; (void)W;
    return 2048 * sizeof(float);
}

static int xent_launch(const void* logits, int ld, const uint8_t* li, const float* ls, int N, int H, int W, int C,
                       int vh, int vw, float scale, float* loss, void* dl, int ldd, void* ws, size_t wsb,
                       void* stream, int dtype) {
    if (!logits || !loss || !dl || C < 1 || C > XENT_MAXC || ld < C || ldd < C) return SEG_EINVAL;
    if (!ws || wsb < 2048 * sizeof(float)) return SEG_EWORKSPACE;
    const long P = (long)N * H * W;
    int nb = seg_grid_1d(P, 256, 2048);
    hipStream_t s = (hipStream_t)stream;
    if (ls) {
        DISPATCH_T(dtype, hipLaunchKernelGGL((xent_k<T, true>), dim3(nb), dim3(256), 0, s, (const T*)logits, ld, li,
                                             ls, N, H, W, C, vh, vw, scale, (T*)dl, ldd, (float*)ws));
    } else {
        DISPATCH_T(dtype, hipLaunchKernelGGL((xent_k<T, false>), dim3(nb), dim3(256), 0, s, (const T*)logits, ld, li,
                                             ls, N, H, W, C, vh, vw, scale, (T*)dl, ldd, (float*)ws));
    }
    SEG_CHECK_LAUNCH();
    hipLaunchKernelGGL(sum_k, dim3(1), dim3(256), 0, s, (const float*)ws, nb, loss);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_softmax_xent_fwd_bwd(const void* logits, int ld, const uint8_t* labels, int N, int H, int W, int C,
                                        int vh, int vw, float scale, float* loss, void* dl, int ldd, int dtype,
                                        void* ws, size_t wsb, void* stream) {
    if (!labels) return SEG_EINVAL;
    return xent_launch(logits, ld, labels, nullptr, N, H, W, C, vh, vw, scale, loss, dl, ldd, ws, wsb, stream,
                       dtype);
}

extern "C" int seg_softmax_xent_soft_fwd_bwd(const void* logits, int ld, const float* labels, int N, int H, int W,
                                             int C, int vh, int vw, float scale, float* loss, void* dl, int ldd,
                                             int dtype, void* ws, size_t wsb, void* stream) {
    if (!labels) return SEG_EINVAL;
    return xent_launch(logits, ld, nullptr, labels, N, H, W, C, vh, vw, scale, loss, dl, ldd, ws, wsb, stream,
                       dtype);
}

extern "C" int seg_argmax(const void* logits, int ld, int C, long P, int64_t* pred, int dtype, void* stream) {
    if (!logits || !pred || C < 1) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(argmax_k<T>, dim3(seg_grid_1d(P, 256)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)logits, ld, C, P, pred));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_softmax(const void* x, int ldx, int C, long P, void* y, int ldy, int dtype, void* stream) {
    if (!x || !y || C < 1 || ldx < C || ldy < C) return SEG_EINVAL;
    DISPATCH_T(dtype, hipLaunchKernelGGL(softmax_k<T>, dim3(seg_grid_1d(P, 256)), dim3(256), 0, (hipStream_t)stream,
                                         (const T*)x, ldx, C, P, (T*)y, ldy));
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_confusion(const int64_t* pred, const uint8_t* labels, int N, int H, int W, int vh, int vw, int C,
                             unsigned long long* conf, void* stream) {
    if (!pred || !labels || !conf) return SEG_EINVAL;
    const long P = (long)N * H * W;
    hipLaunchKernelGGL(confusion_k, dim3(seg_grid_1d(P, 256)), dim3(256), 0, (hipStream_t)stream, pred, labels, N, H,
                       W, vh, vw, C, conf);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_adam_tf1_step(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                                 float eps, int t, float gs, void* stream) {
    if (!p || !g || !m || !v || t < 1) return SEG_EINVAL;
    if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return SEG_EALIGN;
    const double lr_t = (double)lr * sqrt(1.0 - pow((double)b2, t)) / (1.0 - pow((double)b1, t));
    hipLaunchKernelGGL(adam_k, dim3(seg_grid_1d(n / 4 + 1, 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                       (float)lr_t, b1, b2, eps, gs);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" const char* seg_status_string(int s) {
    switch (s) {
        case SEG_OK: return "ok";
        case SEG_EINVAL: return "invalid argument";
        case SEG_ESHAPE: return "shape rule violated (TF InvalidArgumentError)";
        case SEG_EALIGN: return "channel count / stride / pointer not 16-byte aligned";
        case SEG_EWORKSPACE: return "workspace too small";
        case SEG_ELAUNCH: return "HIP kernel launch failed";
    }
    return "unknown status";
}

extern "C" int seg_version(void) { return 1; }

namespace seg {

constexpr int kBnFinishGroups = 128;

size_t bn_grad_finish_scratch(int C) { return (size_t)kBnFinishGroups * 2 * C * sizeof(float); }

int bn_grad_finish(const float* part, int nrows, int C, int cv, float inv, float* dgamma, float* dbeta,
                   float* scratch, hipStream_t s) {
    if (!part || !dgamma || !dbeta || !scratch || nrows <= 0 || C <= 0 || cv > C) return SEG_EINVAL;
    const float* rows = part;
    int n = nrows;
    if (nrows > kBnFinishGroups) {   // thousands of tile rows: fold them first (coalesced)
        const int width = 2 * C;
        hipLaunchKernelGGL(part_rows_reduce_k, dim3((width + 255) / 256, kBnFinishGroups), dim3(256), 0, s, part,
                           nrows, width, scratch, kBnFinishGroups);
        SEG_CHECK_LAUNCH();
        rows = scratch;
        n = kBnFinishGroups;
    }
    hipLaunchKernelGGL(bn_finish_k, dim3((cv + 7) / 8), dim3(256), 0, s, rows, n, C, cv, inv, dgamma, dbeta);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}


// ---- many BN backward finishes in two launches (seg_bn_grad_finish_batch):
// the same two stages and summation order as bn_grad_finish per segment
__device__ __forceinline__ int bnb_seg(const seg_bn_finish_segment* sg, int n, int b, bool stage_a) {
    int s = 0;
    for (int i = 1; i < n; ++i)
        if ((stage_a ? sg[i].a_blk0 : sg[i].b_blk0) <= b) s = i;
    return s;
}

__global__ __launch_bounds__(256) void bn_fold_batch_k(const seg_bn_finish_segment* __restrict__ sg, int n) {
    __shared__ int ss;
    if (threadIdx.x == 0) ss = bnb_seg(sg, n, blockIdx.x, true);
    __syncthreads();
    const seg_bn_finish_segment& g = sg[ss];
    const int local = blockIdx.x - g.a_blk0;
    const int cbs = (2 * g.C + 255) / 256;
    const int gi = local / cbs, cb = local - gi * cbs;
    const int width = 2 * g.C;
    const int c = cb * 256 + threadIdx.x;
    if (c >= width) return;
    float s = 0.f;
    for (int r = gi; r < g.nrows; r += kBnFinishGroups) s += g.part[(long)r * width + c];
    g.scratch[(long)gi * width + c] = s;
}

__global__ __launch_bounds__(256) void bn_finish_batch_k(const seg_bn_finish_segment* __restrict__ sg, int n) {
    __shared__ int ss;
    __shared__ float sgm[32][9], sbt[32][9];
    if (threadIdx.x == 0) ss = bnb_seg(sg, n, blockIdx.x, false);
    __syncthreads();
    const seg_bn_finish_segment& g = sg[ss];
    const float* part = g.nrows > kBnFinishGroups ? g.scratch : g.part;
    const int nrows = g.nrows > kBnFinishGroups ? kBnFinishGroups : g.nrows;
    const int C = g.C;
    const int cl = threadIdx.x & 7, rg = threadIdx.x >> 3;
    const int k = (blockIdx.x - g.b_blk0) * 8 + cl;
    float a = 0.f, b = 0.f;
    if (k < g.cv)
        for (int r = rg; r < nrows; r += 32) {
            a += part[(long)r * 2 * C + k];
            b += part[(long)r * 2 * C + C + k];
        }
    sgm[rg][cl] = a;
    sbt[rg][cl] = b;
    __syncthreads();
    if (threadIdx.x < 8 && k < g.cv) {
        float tg = 0.f, tb = 0.f;
        for (int r = 0; r < 32; ++r) {
            tg += sgm[r][cl];
            tb += sbt[r][cl];
        }
        g.dgamma[k] = tg * g.inv;
        g.dbeta[k] = tb;
    }
}

}  // namespace seg

extern "C" size_t seg_bn_finish_batch_plan(seg_bn_finish_segment* segs, int nsegs, float* scratch, int* a_blocks,
                                           int* b_blocks) {
    size_t bytes = 0;
    int a = 0, b = 0;
    for (int i = 0; i < nsegs; ++i) {
        seg_bn_finish_segment& g = segs[i];
        g.a_blk0 = a;
        g.a_nblk = 0;
        g.scratch = nullptr;
        if (g.nrows > seg::kBnFinishGroups) {
            g.a_nblk = ((2 * g.C + 255) / 256) * seg::kBnFinishGroups;
            g.scratch = scratch ? reinterpret_cast<float*>(reinterpret_cast<char*>(scratch) + bytes) : nullptr;
            bytes += (size_t)seg::kBnFinishGroups * 2 * g.C * sizeof(float);
        }
        a += g.a_nblk;
        g.b_blk0 = b;
        g.b_nblk = (g.cv + 7) / 8;
        b += g.b_nblk;
    }
    if (a_blocks) *a_blocks = a;
    if (b_blocks) *b_blocks = b;
    return bytes;
}

extern "C" int seg_bn_grad_finish_batch(const seg_bn_finish_segment* dev_segs, int nsegs, int a_blocks, int b_blocks,
                                        void* stream) {
    if (!dev_segs || nsegs <= 0 || b_blocks <= 0) return SEG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (a_blocks > 0) {
        hipLaunchKernelGGL(seg::bn_fold_batch_k, dim3(a_blocks), dim3(256), 0, s, dev_segs, nsegs);
        SEG_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(seg::bn_finish_batch_k, dim3(b_blocks), dim3(256), 0, s, dev_segs, nsegs);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}
