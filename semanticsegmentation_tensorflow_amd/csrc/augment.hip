// KITTI training-data augmentation on the GPU: the three samples
// gen_batch_function makes per file (Network/model/FCN.py:235-307) --
// resized original + bc_img, resized crop_image window, resized flip_image --
// and process_gt_image's class labels, computed from the decoded uint8
// images resident in HBM.
//
// The resize is scipy.misc.imresize(..., 'bilinear') = PIL Image.resize
// BILINEAR: Pillow's two-pass ImagingResample (antialiased triangle filter,
// float64 coefficients rounded to 22-bit fixed point, 8-bit clip after each
// pass; unchanged size = copy; RGBA premultiplied around the resample).  One
// thread makes one output pixel: it derives its own horizontal and vertical
// coefficient rows in float64 (the same operation sequence as Pillow, FP
// contraction off so no fma changes a rounding) and runs the horizontal pass
// for each source row its vertical filter reads.  Results are bit-exact with
// PIL (tests/golden/augment.npz via oracle/augment.py).
#include <cmath>

#include "common.h"

namespace {

constexpr int PB = 22;      // PRECISION_BITS = 32 - 8 - 2
constexpr int MAXV = 24;    // views per launch (kernel-argument block)

struct AugView {
    const uint8_t* src;
    int H0, W0, x0, y0, w, h, flip, bc, bright;
    double contrast;
};
struct AugSet {
    AugView v[MAXV];
};

// precompute_coeffs (support 1, box (0, in_size)) for output index xx,
// then normalize_coeffs_8bpc: first source index, tap count, int taps.
template <int K>
__device__ __forceinline__ int pil_coeffs(int in_size, int out_size, int xx, int* k, int* xmin_out) {
#pragma clang fp contract(off)
    const double scale = (double)((float)in_size - 0.0f) / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 1.0 * filterscale;
    const double center = 0.0 + (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double w[K];
    double ww = 0.0;
#pragma unroll
    for (int x = 0; x < K; ++x) {
        double t = ((double)(x + xmin) - center + 0.5) * ss;
        if (t < 0.0) t = -t;
        w[x] = (x < xmax && t < 1.0) ? 1.0 - t : 0.0;
        ww += w[x];
    }
#pragma unroll
    for (int x = 0; x < K; ++x) {
        const double kx = ww != 0.0 ? w[x] / ww : w[x];
        k[x] = x < xmax ? (int)(0.5 + kx * (double)(1 << PB)) : 0;
    }
    *xmin_out = xmin;
    return xmax;
}

__device__ __forceinline__ int clip8(int v) {
    if (v >= (1 << PB << 8)) return 255;
    if (v <= 0) return 0;
    return v >> PB;
}

template <int C, int KH, int KV, bool LABELS>
__global__ __launch_bounds__(256) void augment_k(AugSet set, int OH, int OW, uint8_t* __restrict__ out) {
#pragma clang fp contract(off)
    const AugView& V = set.v[blockIdx.y];
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= OH * OW) return;
    const int oy = idx / OW, ox = idx - oy * OW;
    const bool same = V.w == OW && V.h == OH;
    const bool needh = V.w != OW, needv = V.h != OH;
    const uint8_t* __restrict__ src = V.src;

    // window / mirror / premultiply ('RGBa') view of the source
    auto fetch = [&](int y, int x, int* px) {
        const int sx = V.flip ? V.x0 + V.w - 1 - x : V.x0 + x;
        const uint8_t* s = src + ((long)(V.y0 + y) * V.W0 + sx) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) px[c] = s[c];
        if (C == 4 && !same) {
            const int a = px[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int t = px[c] * a + 128;
                px[c] = ((t >> 8) + t) >> 8;
            }
        }
    };

    int res[C];
    if (same) {
        fetch(oy, ox, res);
    } else {
        int kh[KH], kv[KV], xmin = 0, ymin = oy, ch = 0, cv = 1;
        if (needh) ch = pil_coeffs<KH>(V.w, OW, ox, kh, &xmin);
        if (needv) {
            cv = pil_coeffs<KV>(V.h, OH, oy, kv, &ymin);
        } else {
#pragma unroll
            for (int t = 0; t < KV; ++t) kv[t] = 0;
        }
        int accv[C];
#pragma unroll
        for (int c = 0; c < C; ++c) accv[c] = 1 << (PB - 1);
        int hv[C];
#pragma unroll
        for (int t = 0; t < KV; ++t) {
            if (t >= cv) break;
            const int y = ymin + t;
            if (needh) {
                int acc[C];
#pragma unroll
                for (int c = 0; c < C; ++c) acc[c] = 1 << (PB - 1);
#pragma unroll
                for (int x = 0; x < KH; ++x) {
                    if (x >= ch) break;
                    int px[C];
                    fetch(y, xmin + x, px);
#pragma unroll
                    for (int c = 0; c < C; ++c) acc[c] += px[c] * kh[x];
                }
#pragma unroll
                for (int c = 0; c < C; ++c) hv[c] = clip8(acc[c]);
            } else {
                fetch(y, ox, hv);
            }
#pragma unroll
            for (int c = 0; c < C; ++c) accv[c] += hv[c] * kv[t];
        }
#pragma unroll
        for (int c = 0; c < C; ++c) res[c] = needv ? clip8(accv[c]) : hv[c];
        if (C == 4) {   // 'RGBa' -> 'RGBA'
            const int a = res[3];
            if (a != 0 && a != 255) {
#pragma unroll
                for (int c = 0; c < 3; ++c) res[c] = min(255, (255 * res[c]) / a);
            }
        }
    }
    if (LABELS) {   // process_gt_image: background = exactly (255, 0, 0)
        out[(long)blockIdx.y * OH * OW + idx] = (res[0] == 255 && res[1] == 0 && res[2] == 0) ? 0 : 1;
        return;
    }
    uint8_t* o = out + ((long)blockIdx.y * OH * OW + idx) * C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        int v = res[c];
        if (V.bc) {   // bc_img: int64 * s + m in float64, clip, truncate
            double d = (double)v * V.contrast;
            d = d + (double)V.bright;
            if (d > 255.0) d = 255.0;
            if (d < 0.0) d = 0.0;
            v = (int)d;
        }
        o[c] = (uint8_t)v;
    }
}

int taps_for(int in_size, int out_size) {
    const double scale = (double)in_size / out_size;
    const double support = scale < 1.0 ? 1.0 : scale;
    return (int)std::ceil(support) * 2 + 1;
}

template <int C, bool LABELS>
int launch_aug(const AugSet& set, int nv, int OH, int OW, int kmax, uint8_t* out, hipStream_t s) {
    const dim3 g((OH * OW + 255) / 256, nv), b(256);
#define AUG(K) hipLaunchKernelGGL((augment_k<C, K, K, LABELS>), g, b, 0, s, set, OH, OW, out)
    if (kmax <= 3) AUG(3);
    else if (kmax <= 5) AUG(5);
    else if (kmax <= 7) AUG(7);
    else if (kmax <= 9) AUG(9);
    else if (kmax <= 13) AUG(13);
    else if (kmax <= 17) AUG(17);
    else return SEG_ESHAPE;   // downscale beyond 8x
#undef AUG
    return SEG_OK;
}

}  // namespace

extern "C" int seg_augment(const seg_aug_view* views, int nviews, int C, int OH, int OW, int labels, void* out,
                           void* stream) {
    if (!views || nviews < 0 || !out || OH < 1 || OW < 1 || (C != 3 && C != 4) || (labels && C != 3))
        return SEG_EINVAL;
    if ((long)OH * OW >= (1L << 31)) return SEG_EINVAL;
    const long per = (long)OH * OW * (labels ? 1 : C);
    for (int v0 = 0; v0 < nviews; v0 += MAXV) {
        AugSet set;
        const int nv = std::min(MAXV, nviews - v0);
        int kmax = 3;
        for (int i = 0; i < nv; ++i) {
            const seg_aug_view& a = views[v0 + i];
            if (!a.src) return SEG_EINVAL;
            if (a.w < 1 || a.h < 1 || a.x0 < 0 || a.y0 < 0 || a.x0 + a.w > a.W0 || a.y0 + a.h > a.H0)
                return SEG_ESHAPE;   // window outside the source image
            set.v[i] = AugView{static_cast<const uint8_t*>(a.src), a.H0, a.W0, a.x0, a.y0, a.w, a.h, a.flip ? 1 : 0,
                               a.bc ? 1 : 0, a.bright, a.contrast};
            kmax = std::max(kmax, std::max(taps_for(a.w, OW), taps_for(a.h, OH)));
        }
        if (nv == 0) break;
        uint8_t* o = static_cast<uint8_t*>(out) + v0 * per;
        int st;
        if (labels) st = launch_aug<3, true>(set, nv, OH, OW, kmax, o, (hipStream_t)stream);
        else if (C == 3) st = launch_aug<3, false>(set, nv, OH, OW, kmax, o, (hipStream_t)stream);
        else st = launch_aug<4, false>(set, nv, OH, OW, kmax, o, (hipStream_t)stream);
        if (st) return st;
        SEG_CHECK_LAUNCH();
    }
    return SEG_OK;
}
