// Shared pieces of the halo-tiled direct-conv kernels (halo.hip, halo4.hip).
#pragma once
#include "common.h"
#include "igemm.h"

namespace seg {

struct HaloGeom {
    int taps_h, tiles_x, tiles_y, nimg;
    int hwd, hrows, hy0, hx0;   // halo width, rows, origin offset vs tap (0,0)
    int nchunks, kc_per_split;
};

// Output pixel (within its image) of GEMM grid point (oy, ox) on the Ha x Wa
// grid: (oy * osh + ooh, ox * osw + oow).  halo_plan admits only convs
// (Ha = OH, Wa = OW, stride 1, offset 0: the identity map); a transposed
// conv's 2x2-tap phases do not fit the halo pipelines, which spread a chunk's
// halo DMA over at least hi + 1 (conv_halo) / 7 (conv_halo2) taps.
__device__ __forceinline__ long halo_opix(const NTParams& p, int oy, int ox) {
    return (long)(oy * p.osh + p.ooh) * p.OW + (ox * p.osw + p.oow);
}

// MaxPool 2x2 / stride 2 fused into the LDS-staged epilogue (TF's MaxPool after
// conv_layer's bias + ReLU, Network/model/FCN.py:55-100 / :158-160): wbuf holds
// this wave's HR staged fp32 rows [rr][SROW] (8 column chunks of 8), row rr =
// tile pixel ml0 + rr = (oy0 + ml / BW, ox0 + ml % BW), ml0 on an even tile
// row.  Each lane keeps its column chunk (col0); items = (pooled pixel, chunk).
// Every value is rounded to T before the comparison, so the pooled map and the
// switches equal seg_maxpool2x2_fwd_argmax of the unfused conv output bit for
// bit (first max in (0,0) (0,1) (1,0) (1,1) order; bit 2 = max > 0).
template <typename T, int BW, int HR>
__device__ __forceinline__ void pool_epi_rows(const NTParams& p, const char* wbuf, int srow, int ml0, int oy0, int ox0,
                                              int img, int col0, int lane, const float* bias, const float* scl,
                                              const float* shf) {
    static_assert(HR % (2 * BW) == 0 && (HR / 4 * 8) % 64 == 0, "whole pooled rows per half, 64-lane items");
    constexpr int PPR = BW / 2, NPP = HR / 4;
    const EpiParams& e = p.epi;
    const int PH = p.OH >> 1, PW = p.OW >> 1;
#pragma unroll
    for (int k = 0; k < NPP * 8 / 64; ++k) {
        const int pp = (lane >> 3) + 8 * k;
        const int prow = pp / PPR, pcol = pp - (pp / PPR) * PPR;
        const int r00 = 2 * prow * BW + 2 * pcol;
        const int ml = ml0 + r00;
        const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
        if (oy + 1 >= p.OH || ox + 1 >= p.OW || col0 >= p.N) continue;
        float v[4][8];
        splitk_lds8(wbuf + r00 * srow, v[0]);
        splitk_lds8(wbuf + (r00 + 1) * srow, v[1]);
        splitk_lds8(wbuf + (r00 + BW) * srow, v[2]);
        splitk_lds8(wbuf + (r00 + BW + 1) * srow, v[3]);
        float m[8];
        unsigned long long code = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const bool cv = col0 + j < e.n_valid;
            float q[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                float x = v[t][j] * scl[j] + shf[j] + bias[j];
                if (e.relu) x = fmaxf(x, 0.f);
                q[t] = cv ? to_f32(from_f32<T>(x)) : 0.f;
            }
            unsigned a = 0;
            float mx = q[0];
            if (q[1] > mx) { mx = q[1]; a = 1; }
            if (q[2] > mx) { mx = q[2]; a = 2; }
            if (q[3] > mx) { mx = q[3]; a = 3; }
            m[j] = mx;
            code |= (unsigned long long)(a | (mx > 0.f ? 4u : 0u)) << (8 * j);
        }
        const long pix = ((long)img * PH + (oy >> 1)) * PW + (ox >> 1);
        *reinterpret_cast<uint4*>(reinterpret_cast<T*>(e.pool_y) + pix * e.ld_pool + col0) = Chunk<T>::pack(m);
        if (e.pool_idx) *reinterpret_cast<unsigned long long*>(e.pool_idx + pix * e.ld_idx + col0) = code;
    }
}

// conv_halo4 (halo4.hip): 256 x 256 plans at one wave per SIMD
bool halo4_ok(const NTParams& p, const HaloPlan& hp);
void launch_halo4(NTParams& p, const HaloPlan& hp, const HaloGeom& g, hipStream_t s, int dtype);

}  // namespace seg
