// C-ABI convolution entry points: Conv2D / Conv2DBackpropInput /
// Conv2DBackpropFilter and conv2d_transpose (forward + both gradients),
// each mapped onto the implicit-GEMM kernels of igemm.hip.
#include "common.h"
#include "igemm.h"
#include "halo.h"
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <math.h>

using seg::NTParams;
using seg::TNParams;

static inline int round8(int c) { return (c + 7) & ~7; }

static int same_pads(int in, int k, int s, int d, int* out, int* pb, int* pa) {
    const int keff = k + (k - 1) * (d - 1);
    *out = (in + s - 1) / s;
    int total = (*out - 1) * s + keff - in;
    if (total < 0) total = 0;
    *pb = total / 2;
    *pa = total - total / 2;
    return 0;
}

static int valid_out(int in, int k, int s, int d) {
    const int keff = k + (k - 1) * (d - 1);
    return (in - keff) / s + 1;
}

static int check_desc(const seg_conv_desc* d) {
    if (!d) return SEG_EINVAL;
    if (d->dtype != SEG_F32 && d->dtype != SEG_BF16 && d->dtype != SEG_F16) return SEG_EINVAL;
    if (d->N <= 0 || d->H <= 0 || d->W <= 0 || d->OH <= 0 || d->OW <= 0 || d->R <= 0 || d->S <= 0) return SEG_ESHAPE;
    if ((d->C & 7) || (d->K & 7) || (d->ldx & 7) || (d->ldy & 7)) return SEG_EALIGN;
    if (d->ldx < d->C || d->ldy < d->K) return SEG_EALIGN;
    if (d->c_valid > d->C || d->k_valid > d->K || d->c_valid <= 0 || d->k_valid <= 0) return SEG_EINVAL;
    return SEG_OK;
}

extern "C" int seg_conv_desc_init(seg_conv_desc* d, int N, int H, int W, int C, int K, int R, int S,
                                  int stride, int dilation, int padding, int dtype) {
    if (!d || stride <= 0 || dilation <= 0 || N <= 0 || H <= 0 || W <= 0 || C <= 0 || K <= 0) return SEG_EINVAL;
    seg_conv_desc z = {};
    z.N = N; z.H = H; z.W = W;
    z.C = round8(C); z.K = round8(K);
    z.c_valid = C; z.k_valid = K;
    z.R = R; z.S = S;
    z.stride_h = z.stride_w = stride;
    z.dil_h = z.dil_w = dilation;
    if (padding == 0) {
        same_pads(H, R, stride, dilation, &z.OH, &z.pad_top, &z.pad_bottom);
        same_pads(W, S, stride, dilation, &z.OW, &z.pad_left, &z.pad_right);
    } else {
        z.OH = valid_out(H, R, stride, dilation);
        z.OW = valid_out(W, S, stride, dilation);
        if (z.OH <= 0 || z.OW <= 0) return SEG_ESHAPE;
    }
    z.ldx = z.C; z.ldy = z.K;
    z.dtype = dtype;
    *d = z;
    return SEG_OK;
}

extern "C" int seg_tconv_desc_init(seg_conv_desc* d, int N, int H, int W, int C, int OH, int OW, int K,
                                   int R, int S, int stride, int padding, int dtype) {
    if (!d || stride <= 0 || N <= 0 || H <= 0 || W <= 0 || C <= 0 || K <= 0 || OH <= 0 || OW <= 0) return SEG_EINVAL;
    seg_conv_desc z = {};
    z.N = N; z.H = H; z.W = W; z.OH = OH; z.OW = OW;
    z.C = round8(C); z.K = round8(K);
    z.c_valid = C; z.k_valid = K;
    z.R = R; z.S = S;
    z.stride_h = z.stride_w = stride;
    z.dil_h = z.dil_w = 1;
    // TF: the forward conv of the output shape must give the input shape
    int eh, ew;
    if (padding == 0) {
        same_pads(OH, R, stride, 1, &eh, &z.pad_top, &z.pad_bottom);
        same_pads(OW, S, stride, 1, &ew, &z.pad_left, &z.pad_right);
    } else {
        eh = valid_out(OH, R, stride, 1);
        ew = valid_out(OW, S, stride, 1);
    }
    if (eh != H || ew != W) return SEG_ESHAPE;
    z.ldx = z.C; z.ldy = z.K;
    z.dtype = dtype;
    *d = z;
    return SEG_OK;
}

static seg::EpiParams make_epi(const seg_epilogue* e, int n_valid, long res_img, long pix_per_img = 0, int ld_out = 0) {
    seg::EpiParams r = {};
    r.n_valid = n_valid;
    r.keep_prob = 1.f;
    r.mask_scale = 1.f;
    if (e) {
        r.bias = e->bias; r.scale = e->scale; r.shift = e->shift;
        r.residual = e->residual; r.ld_res = e->ld_residual; r.res_img = res_img;
        r.relu = e->relu; r.keep_prob = e->keep_prob > 0.f ? e->keep_prob : 1.f; r.seed = e->seed;
        if (e->relu_mask) {
            r.mask = e->relu_mask;
            r.ld_mask = e->ld_relu_mask > 0 ? e->ld_relu_mask : ld_out;
            r.mask_img = pix_per_img * r.ld_mask;
            r.mask_scale = e->mask_scale != 0.f ? e->mask_scale : 1.f;
        }
    }
    return r;
}

// ---------------------------------------------------------------------------
// parameter builders (shared by the launchers and the workspace queries)
// ---------------------------------------------------------------------------
// diagnostics only: extra elements of row padding in the packed KRSC (fwd) /
// HWIO (dgrad) filter copies the caller allocated (L2 channel-stride probe)

static NTParams conv_fwd_params(const seg_conv_desc* d) {
    NTParams p = {};
    p.M = d->N * d->OH * d->OW; p.N = d->K; p.K = d->R * d->S * d->C;
    p.x_img = (long)d->H * d->W * d->ldx; p.IH = d->H; p.IW = d->W; p.C = d->C; p.ldx = d->ldx;
    p.Ha = d->OH; p.Wa = d->OW; p.ish = d->stride_h; p.isw = d->stride_w;
    p.ioh = -d->pad_top; p.iow = -d->pad_left; p.tsh = d->dil_h; p.tsw = d->dil_w; p.taps_w = d->S;
    p.w_col = (long)d->R * d->S * (d->C + g_wpad); p.w_tap = d->C + g_wpad; p.rstep = 1; p.sstep = 1; p.Sfull = d->S;
    p.y_img = (long)d->OH * d->OW * d->ldy; p.OH = d->OH; p.OW = d->OW; p.ldy = d->ldy; p.osh = 1; p.osw = 1;
    return p;
}

static NTParams conv_bwd_data_params(const seg_conv_desc* d) {
    NTParams p = {};
    p.M = d->N * d->H * d->W; p.N = d->C; p.K = d->R * d->S * d->K;
    p.x_img = (long)d->OH * d->OW * d->ldy; p.IH = d->OH; p.IW = d->OW; p.C = d->K; p.ldx = d->ldy;
    p.Ha = d->H; p.Wa = d->W; p.ish = 1; p.isw = 1;
    p.ioh = d->pad_top; p.iow = d->pad_left; p.tsh = -d->dil_h; p.tsw = -d->dil_w; p.taps_w = d->S;
    p.w_col = d->K + g_wpad; p.w_tap = (long)d->C * (d->K + g_wpad); p.rstep = 1; p.sstep = 1; p.Sfull = d->S;
    p.y_img = (long)d->H * d->W * d->ldx; p.OH = d->H; p.OW = d->W; p.ldy = d->ldx; p.osh = 1; p.osw = 1;
    p.epi.n_valid = d->C; p.epi.keep_prob = 1.f;
    p.kv = d->k_valid;
    return p;
}

static int bwd_data_bn_params(const seg_conv_desc* d, NTParams& p);

static TNParams conv_bwd_filter_params(const seg_conv_desc* d) {
    TNParams p = {};
    p.M = d->R * d->S * d->C; p.N = d->K; p.P = d->N * d->OH * d->OW;
    p.x_img = (long)d->H * d->W * d->ldx; p.IH = d->H; p.IW = d->W; p.Cg = d->C; p.ldx = d->ldx;
    p.Ha = d->OH; p.Wa = d->OW; p.ish = d->stride_h; p.isw = d->stride_w;
    p.ioh = -d->pad_top; p.iow = -d->pad_left; p.tsh = d->dil_h; p.tsw = d->dil_w; p.taps_w = d->S;
    p.ldb = d->ldy;
    p.o_tap = (long)d->c_valid * d->k_valid; p.o_c = d->k_valid; p.o_n = 1;
    p.c_valid = d->c_valid; p.n_valid = d->k_valid;
    return p;
}

static NTParams tconv_fwd_params(const seg_conv_desc* d) {
    NTParams p = {};
    const int sh = d->stride_h, sw = d->stride_w;
    p.N = d->K; p.K = (d->R / sh) * (d->S / sw) * d->C;
    p.x_img = (long)d->H * d->W * d->ldx; p.IH = d->H; p.IW = d->W; p.C = d->C; p.ldx = d->ldx;
    p.ish = 1; p.isw = 1; p.tsh = -1; p.tsw = -1; p.taps_w = d->S / sw;
    p.w_col = d->C; p.w_tap = (long)d->K * d->C; p.rstep = sh; p.sstep = sw; p.Sfull = d->S;
    p.y_img = (long)d->OH * d->OW * d->ldy; p.OH = d->OH; p.OW = d->OW; p.ldy = d->ldy; p.osh = sh; p.osw = sw;
    p.phase = 1; p.st_h = sh; p.st_w = sw; p.pad_t = d->pad_top; p.pad_l = d->pad_left; p.Nimg = d->N;
    p.M = d->N * ((d->OH + sh - 1) / sh) * ((d->OW + sw - 1) / sw);   // max over phases
    p.Ha = (d->OH + sh - 1) / sh; p.Wa = (d->OW + sw - 1) / sw;
    return p;
}

static NTParams tconv_bwd_data_params(const seg_conv_desc* d) {
    NTParams p = {};
    p.M = d->N * d->H * d->W; p.N = d->C; p.K = d->R * d->S * d->K;
    p.x_img = (long)d->OH * d->OW * d->ldy; p.IH = d->OH; p.IW = d->OW; p.C = d->K; p.ldx = d->ldy;
    p.Ha = d->H; p.Wa = d->W; p.ish = d->stride_h; p.isw = d->stride_w;
    p.ioh = -d->pad_top; p.iow = -d->pad_left; p.tsh = 1; p.tsw = 1; p.taps_w = d->S;
    p.w_col = (long)d->R * d->S * d->K; p.w_tap = d->K; p.rstep = 1; p.sstep = 1; p.Sfull = d->S;
    p.y_img = (long)d->H * d->W * d->ldx; p.OH = d->H; p.OW = d->W; p.ldy = d->ldx; p.osh = 1; p.osw = 1;
    p.epi.n_valid = d->C; p.epi.keep_prob = 1.f;
    return p;
}

static TNParams tconv_bwd_filter_params(const seg_conv_desc* d) {
    TNParams p = {};
    p.M = d->R * d->S * d->K; p.N = d->C; p.P = d->N * d->H * d->W;
    p.x_img = (long)d->OH * d->OW * d->ldy; p.IH = d->OH; p.IW = d->OW; p.Cg = d->K; p.ldx = d->ldy;
    p.Ha = d->H; p.Wa = d->W; p.ish = d->stride_h; p.isw = d->stride_w;
    p.ioh = -d->pad_top; p.iow = -d->pad_left; p.tsh = 1; p.tsw = 1; p.taps_w = d->S;
    p.ldb = d->ldx;
    p.o_tap = (long)d->k_valid * d->c_valid; p.o_c = d->c_valid; p.o_n = 1;
    p.c_valid = d->k_valid; p.n_valid = d->c_valid;
    return p;
}


// conv2d_transpose with few output channels and a large stride (FCN conv_t3:
// 256 -> 2, k16 s8): the "tap-dense" path.  Its packed filters keep the true
// output-channel count Kq (even, <= 8) instead of padding it to 8, so no MFMA
// work is spent on padding channels:
//   forward   Z[p_in][(r,s,k)] = sum_c x[p_in][c] W[r][s][k][c]  (dense GEMM,
//             N = R*S*Kq), then every output pixel gathers its (R/st)*(S/st)
//             taps: y[oh][ow][k] = b[k] + res + sum Z[ih][iw][(r,s,k)];
//   input grad  D[p_in][(r,s,k)] = dy[ih*st - pt + r][iw*st - pl + s][k] (gather),
//             dx = D . Wt^T with Wt = [c][(r,s,k)] (dense GEMM, K = R*S*Kq);
//   filter grad dW[(r,s,k)][c] = sum_p D[p][(r,s,k)] x[p][c] (dense TN GEMM).
template <typename T, int KQ>
__global__ void tconv_col2im_k(const T* __restrict__ Z, T* __restrict__ y, int N, int H, int W, int OH, int OW,
                               int kv, int R, int S, int st, int pt, int pl, int ldy,
                               const float* __restrict__ bias, const T* __restrict__ res, int ldr) {
    static_assert(KQ == 2 || KQ == 4 || KQ == 8, "tap-dense channel counts");
    const long total = (long)N * OH * OW;
    const int zrow = R * S * KQ;
    float b8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) b8[k] = (bias && k < kv) ? bias[k] : 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int ow = (int)(i % OW);
        const long t = i / OW;
        const int oh = (int)(t % OH);
        const int n = (int)(t / OH);
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
        const int rh = (oh + pt) % st, rw = (ow + pl) % st;
        for (int r = rh; r < R; r += st) {
            const int ih = (oh + pt - r) / st;
            if (ih < 0 || ih >= H) continue;
            for (int s2 = rw; s2 < S; s2 += st) {
                const int iw = (ow + pl - s2) / st;
                if (iw < 0 || iw >= W) continue;
                const T* zp = Z + (((long)n * H + ih) * W + iw) * zrow + (r * S + s2) * KQ;
                if constexpr (is_bf16_v<T> && KQ == 2) {
                    const unsigned u = *reinterpret_cast<const unsigned*>(zp);
                    acc[0] += __uint_as_float(u << 16);
                    acc[1] += __uint_as_float(u & 0xffff0000u);
                } else {
#pragma unroll
                    for (int k = 0; k < KQ; ++k) acc[k] += to_f32(zp[k]);
                }
            }
        }
        float r8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (res) {
            const T* rp = res + i * ldr;
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), r8);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp + 4), r8 + 4);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = k < kv ? acc[k] + b8[k] + r8[k] : 0.f;
        T* yp = y + i * ldy;
        *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(acc);
        if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(yp + 4) = Chunk<T>::pack(acc + 4);
    }
}

// D[p_in][(r,s,k)] for the tap-dense input / filter gradients.  One thread per
// 16-byte chunk of a row = 8 / KQ consecutive taps (r, s..s+8/KQ-1) of one
// input pixel: KQ-channel reads (4 bytes for bf16 KQ=2) of consecutive output
// pixels, so a wave covers 16 output pixels of each of 2..8 filter rows.
template <typename T, int KQ>
__global__ void tconv_gather_dy_k(const T* __restrict__ dy, T* __restrict__ D, int N, int H, int W, int OH, int OW,
                                  int ldy, int R, int S, int st, int pt, int pl) {
    constexpr int TPC = 8 / KQ;                       // taps per 16-byte chunk
    const int row = R * S * KQ, r8 = row / 8;
    const long total = (long)N * H * W * r8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int q = (int)(i % r8);
        const long pix = i / r8;
        const int iw = (int)(pix % W);
        const long t = pix / W;
        const int ih = (int)(t % H);
        const int n = (int)(t / H);
        const int tap0 = q * TPC;
        const int r = tap0 / S, s0 = tap0 - (tap0 / S) * S;   // S % TPC == 0: one filter row
        const int oh = ih * st - pt + r;
        const bool rok = (unsigned)oh < (unsigned)OH;
        const T* src = dy + ((long)n * OH + (rok ? oh : 0)) * OW * ldy;
        float v[8];
#pragma unroll
        for (int j = 0; j < TPC; ++j) {
            const int ow = iw * st - pl + s0 + j;
            const bool ok = rok && (unsigned)ow < (unsigned)OW;
            if constexpr (is_bf16_v<T> && KQ == 2) {
                const unsigned u = ok ? *reinterpret_cast<const unsigned*>(src + (long)ow * ldy) : 0u;
                v[2 * j] = __uint_as_float(u << 16);
                v[2 * j + 1] = __uint_as_float(u & 0xffff0000u);
            } else {
#pragma unroll
                for (int k = 0; k < KQ; ++k) v[j * KQ + k] = ok ? to_f32(src[(long)ow * ldy + k]) : 0.f;
            }
        }
        T* dp = D + pix * row + q * 8;
        *reinterpret_cast<uint4*>(dp) = Chunk<T>::pack(v);
        if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(dp + 4) = Chunk<T>::pack(v + 4);
    }
}

// tap-dense applies: few (even) output channels, K padded to 8, stride >= 4, square kernel
static int tconv_dense_kq(const seg_conv_desc* d) {
    if (d->K != 8 || d->stride_h != d->stride_w || d->stride_h < 4 || d->R != d->S) return 0;
    const int kq = d->k_valid;
    if (kq != 2 && kq != 4 && kq != 8) return 0;
    if ((d->R * d->S * kq) % 8 || d->S % (8 / kq)) return 0;
    return kq;
}

static size_t tconv_dense_zbytes(const seg_conv_desc* d) {
    const size_t esz = d->dtype == SEG_F32 ? 4 : 2;
    return ((size_t)d->N * d->H * d->W * d->R * d->S * tconv_dense_kq(d) * esz + 255) & ~(size_t)255;
}

// the dense GEMM over the Z / D matrix viewed as a 1x1 "conv" of C_g channels
static NTParams dense_nt(int M, int N, int K, const void* x, int ldx, const void* w, void* y, int ldy) {
    NTParams g = {};
    g.M = M; g.N = N; g.K = K;
    g.x = x; g.x_img = (long)M * ldx; g.IH = 1; g.IW = M; g.C = K; g.ldx = ldx;
    g.Ha = 1; g.Wa = M; g.ish = 1; g.isw = 1; g.ioh = 0; g.iow = 0; g.tsh = 1; g.tsw = 1; g.taps_w = 1;
    g.w = w; g.w_col = K; g.w_tap = K; g.rstep = 1; g.sstep = 1; g.Sfull = 1;
    g.y = y; g.y_img = (long)M * ldy; g.OH = 1; g.OW = M; g.ldy = ldy; g.osh = 1; g.osw = 1;
    g.epi.n_valid = N; g.epi.keep_prob = 1.f;
    return g;
}

static int launch_gather_dy(const seg_conv_desc* d, const void* dy, void* D, hipStream_t st) {
    const int kq = tconv_dense_kq(d);
    const long total = (long)d->N * d->H * d->W * (d->R * d->S * kq / 8);
    const int grid = seg_grid_1d(total, 256);
#define GATHER(T, KQ) hipLaunchKernelGGL((tconv_gather_dy_k<T, KQ>), dim3(grid), dim3(256), 0, st, (const T*)dy, (T*)D, \
                                         d->N, d->H, d->W, d->OH, d->OW, d->ldy, d->R, d->S, d->stride_h, d->pad_top, d->pad_left)
    if (d->dtype == SEG_BF16) {
        if (kq == 2) GATHER(bf16, 2); else if (kq == 4) GATHER(bf16, 4); else GATHER(bf16, 8);
    } else if (d->dtype == SEG_F16) {
        if (kq == 2) GATHER(f16, 2); else if (kq == 4) GATHER(f16, 4); else GATHER(f16, 8);
    } else {
        if (kq == 2) GATHER(float, 2); else if (kq == 4) GATHER(float, 4); else GATHER(float, 8);
    }
#undef GATHER
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_tconv_filter_apad(const seg_conv_desc* d) {
    if (check_desc(d)) return -SEG_EINVAL;
    const int kq = tconv_dense_kq(d);
    return kq ? kq : d->K;
}

extern "C" size_t seg_conv_workspace(const seg_conv_desc* d, int op) {
    if (check_desc(d) != SEG_OK) return 0;
    switch (op) {
        case 0: { NTParams p = conv_fwd_params(d); return seg::nt_workspace(p.M, p.N, p.K, d->dtype, 0); }
        case 1: { NTParams p = conv_bwd_data_params(d); return seg::nt_workspace(p.M, p.N, p.K, d->dtype, 0); }
        case 2: {
            TNParams p = conv_bwd_filter_params(d);
            size_t need = seg::tn_workspace(p.M, p.N, p.P, d->dtype);
            seg::WgradPlan wp;
            if (g_tn_variant == 2 && seg::wgrad_plan(p, d->dtype, seg::device_cus(), &wp))
                need = std::max(need, seg::wgrad_workspace(wp, p));
            if (seg::smallc_wgrad_ok(p, d->dtype))
                need = std::max(need, (size_t)seg::smallc_wgrad_splits(p, seg::device_cus()) * (p.M + 1) * p.N *
                                          sizeof(float));
            return std::max(need, seg_bias_grad_workspace((long)d->N * d->OH * d->OW, d->K));
        }
        case 3:
            if (tconv_dense_kq(d)) {
                const int M = d->N * d->H * d->W, Nn = d->R * d->S * tconv_dense_kq(d);
                return tconv_dense_zbytes(d) + seg::nt_workspace(M, Nn, d->C, d->dtype, 0);
            }
            return 0;
        case 4: {
            if (tconv_dense_kq(d)) {
                const int M = d->N * d->H * d->W, Kd = d->R * d->S * tconv_dense_kq(d);
                return tconv_dense_zbytes(d) + seg::nt_workspace(M, d->C, Kd, d->dtype, 0);
            }
            NTParams p = tconv_bwd_data_params(d);
            return seg::nt_workspace(p.M, p.N, p.K, d->dtype, 0);
        }
        case 5: {
            if (tconv_dense_kq(d)) {
                const int P = d->N * d->H * d->W, Md = d->R * d->S * tconv_dense_kq(d);
                return tconv_dense_zbytes(d) + std::max(seg::tn_workspace(Md, d->C, P, d->dtype),
                                                        seg_bias_grad_workspace((long)d->N * d->OH * d->OW, d->K));
            }
            TNParams p = tconv_bwd_filter_params(d);
            return std::max(seg::tn_workspace(p.M, p.N, p.P, d->dtype),
                            seg_bias_grad_workspace((long)d->N * d->OH * d->OW, d->K));
        }
    }
    return 0;
}

extern "C" int seg_conv_kernel_info(const seg_conv_desc* d, int op, char* name, int len, int* splits,
                                    double* flops) {
    int st = check_desc(d);
    if (st) return st;
    int bm = 0, bn = 0, sp = 1;
    const char* fam = "igemm_nt";
    const char* ty = d->dtype == SEG_BF16 ? "bf16" : d->dtype == SEG_F16 ? "f16" : "f32";
    const double macs_conv = (double)d->N * d->OH * d->OW * d->R * d->S * d->c_valid * d->k_valid;
    // conv2d_transpose MACs: every input pixel meets every tap
    const double macs_t = (double)d->N * d->H * d->W * d->R * d->S * d->c_valid * d->k_valid;
    double macs = 0;
    switch (op) {
        case 0:
        case 1: {
            NTParams p = op == 0 ? conv_fwd_params(d) : conv_bwd_data_params(d);
            p.epi.keep_prob = 1.f;
            macs = macs_conv;
            if (op == 0 && d->dil_w == d->dil_h && seg::smallc_fwd_ok(p, d->dtype, d->R, d->S, d->dil_h)) {
                fam = "conv_c8"; bm = 512; bn = d->K; sp = 1;
                break;
            }
            fam = seg::nt_choice(p, d->dtype, 1, p.M, &bm, &bn, &sp);
            break;
        }
        case 2: {
            TNParams p = conv_bwd_filter_params(d);
            seg::tn_info(p.M, p.N, p.P, d->dtype, &bm, &bn, &sp);
            fam = "igemm_tn";
            seg::WgradPlan wp;
            if (seg::smallc_wgrad_ok(p, d->dtype)) {
                fam = "wgrad_c8"; bm = 72; bn = p.N; sp = seg::smallc_wgrad_splits(p, seg::device_cus());
            } else if (g_tn_variant == 2 && seg::wgrad_plan(p, d->dtype, seg::device_cus(), &wp)) {
                fam = "wgrad_halo"; bm = 576; bn = wp.nt; sp = wp.splits;
            } else if (g_tn_variant == 2 && seg::tn3_ok(p, d->dtype)) {
                fam = "igemm_tn3"; bm = bn = 256; seg::tn3_info(p.M, p.N, p.P, seg::device_cus(), &sp);
            } else if (g_tn_variant == 2 && d->dtype != SEG_F32 && p.M >= 128) {
                fam = "igemm_tn2";
            }
            macs = macs_conv;
            break;
        }
        case 3: {
            macs = macs_t;
            if (const int kq = tconv_dense_kq(d)) {
                const int M = d->N * d->H * d->W, Nn = d->R * d->S * kq;
                NTParams g = dense_nt(M, Nn, d->C, nullptr, d->ldx, nullptr, nullptr, Nn);
                g.IH = d->H; g.IW = d->W; g.Ha = d->H; g.Wa = d->W; g.OH = d->H; g.OW = d->W;
                fam = seg::nt_choice(g, d->dtype, 1, g.M, &bm, &bn, &sp);
            } else {
                NTParams p = tconv_fwd_params(d);
                fam = seg::nt_choice(p, d->dtype, d->stride_h * d->stride_w, p.M, &bm, &bn, &sp);
            }
            break;
        }
        case 4: {
            macs = macs_t;
            if (const int kq = tconv_dense_kq(d)) {
                const int M = d->N * d->H * d->W, Kd = d->R * d->S * kq;
                NTParams g = dense_nt(M, d->C, Kd, nullptr, Kd, nullptr, nullptr, d->ldx);
                g.IH = d->H; g.IW = d->W; g.Ha = d->H; g.Wa = d->W; g.OH = d->H; g.OW = d->W;
                fam = seg::nt_choice(g, d->dtype, 1, g.M, &bm, &bn, &sp);
            } else {
                NTParams p = tconv_bwd_data_params(d);
                fam = seg::nt_choice(p, d->dtype, 1, p.M, &bm, &bn, &sp);
            }
            break;
        }
        case 5: {
            const int Mt = tconv_dense_kq(d) ? d->R * d->S * tconv_dense_kq(d) : d->R * d->S * d->K;
            seg::tn_info(Mt, d->C, d->N * d->H * d->W, d->dtype, &bm, &bn, &sp);
            fam = (g_tn_variant == 2 && d->dtype != SEG_F32 && Mt >= 128) ? "igemm_tn2" : "igemm_tn";
            if (g_tn_variant == 2 && seg::tn3_applies(Mt, d->C, d->dtype)) {
                fam = "igemm_tn3"; bm = bn = 256; seg::tn3_info(Mt, d->C, d->N * d->H * d->W, seg::device_cus(), &sp);
            }
            macs = macs_t;
            break;
        }
        case 6: {        // Conv2DBackpropInput through the BN(+ReLU) backward (seg_conv2d_bwd_data_bn)
            NTParams p;
            const int kind = bwd_data_bn_params(d, p);
            if (!kind) return SEG_EINVAL;
            macs = macs_conv;
            if (kind == 1 && seg::bn1x1s_ok(p, d->dtype)) { fam = "bn1x1_stream"; bm = 128; bn = 64; }
            else if (kind == 1) { fam = "igemm_nt2_bn"; bm = 256; bn = 64; }
            else { fam = "conv_res16c_bn"; bm = 256; bn = 64; }
            break;
        }
        case 7: {        // Conv2D over relu(BN(x)) (seg_conv2d_fwd_pro)
            NTParams p = conv_fwd_params(d);
            macs = macs_conv;
            if (seg::s1x1_ok(p, d->dtype, 1)) {
                fam = "conv1x1_stream"; bm = 128; bn = 64;
            } else if (g_nt_variant == 2 && seg::nt2_pro_ok(p, d->dtype, 1)) {
                fam = "igemm_nt2_pro"; bm = 192; bn = p.N <= 64 ? 64 : 128;
            } else {
                fam = "igemm_nt_pro"; bm = 128; bn = p.N <= 64 ? 64 : 128;
            }
            break;
        }
        case 8: {        // Conv2DBackpropFilter with relu(BN(x)) recomputed (seg_conv2d_bwd_filter_pro)
            TNParams p = conv_bwd_filter_params(d);
            macs = macs_conv;
            seg::tn_info(p.M, p.N, p.P, d->dtype, &bm, &bn, &sp);
            fam = (d->dtype != SEG_F32 && g_tn_variant == 2 && p.M == p.Cg) ? "igemm_tn2_pro" : "igemm_tn_pro";
            break;
        }
        default: return SEG_EINVAL;
    }
    if (name && len > 0) snprintf(name, len, "%s<%s,%d,%d>", fam, ty, bm, bn);
    if (splits) *splits = sp;
    if (flops) *flops = 2.0 * macs;
    return SEG_OK;
}

// Kernel-selection knobs (A/B runs and the variant parity tests): every value
// an entry accepts selects a parity-tested kernel or schedule.  The ablation
// modes behind kernel diagnostics (no DMA / no MFMA / no stores: garbage
// results) exist only in the diagnostic build (-DSEG_DIAG, _lib.build(diag=True)
// -> libsegkern_diag.so), never in libsegkern.so.
namespace {
struct Knob {
    const char* name;
    std::atomic<int> seg::KnobSet::*var;
    int lo, hi;        // accepted range ...
    int step;          // ... in multiples of step (0: any listed in `only`)
    int only[8];
};

std::mutex g_knob_mu;   // serialises seg_set_option writers

const Knob* find_knob(const char* name) {
    static const Knob knobs[] = {
        {"igemm_nt_variant", &seg::KnobSet::nt_variant, 1, 2, 1, {}},
        {"igemm_tn_variant", &seg::KnobSet::tn_variant, 1, 2, 1, {}},
        {"tn_nsplit", &seg::KnobSet::tn_nsplit, 0, 1, 1, {}},
        {"nt_nsplit", &seg::KnobSet::nt_nsplit, 0, 1, 1, {}},
        {"halo_duo", &seg::KnobSet::halo_duo, 0, 1, 1, {}},
        {"nt_halo", &seg::KnobSet::nt_halo, 0, 1, 1, {}},
        {"halo_wide", &seg::KnobSet::halo_wide, 0, 1, 1, {}},
        {"halo4", &seg::KnobSet::halo4, 0, 2, 1, {}},         // 2: conv_halo4 8 waves, 1: 4 waves, 0: conv_halo2
        {"halo_min_splits", &seg::KnobSet::halo_min_splits, 1, 64, 1, {}},   // force split-K in the halo planner
        {"adam_tr_fused", &seg::KnobSet::adam_tr_fused, 0, 1, 1, {}},
        {"nt2_short", &seg::KnobSet::nt2_short, 0, 64, 1, {}},                // max k tiles of the 2-stage igemm_nt2
        {"tn_fill", &seg::KnobSet::tn_fill, 1, 64, 1, {}},                   // filter-gradient split-K target, blocks/CU
        {"tn_split_cap", &seg::KnobSet::tn_split_cap, 1, 4096, 1, {}},
        {"tn_reduce_sl", &seg::KnobSet::tn_reduce_sl, 0, 0, 0, {1, 2, 4, 8, 16, 32, 64}},
        {"tn2_smallm", &seg::KnobSet::tn2_smallm, 0, 1, 1, {}},
        {"adam_blocks", &seg::KnobSet::adam_blocks, 0, 1 << 30, 1, {}},           // grid cap of seg_adam_tf1_pack (0: per tile)
        {"nt3_fill", &seg::KnobSet::nt3_fill, 0, 1, 1, {}},
        {"tn3_stagger_us", &seg::KnobSet::tn3_stagger_us, 0, 1000, 1, {}},
        {"s1x1", &seg::KnobSet::s1x1, 0, 1, 1, {}},
        {"tn3_half", &seg::KnobSet::tn3_half, 0, 7, 1, {}},
        {"tn3_mfast", &seg::KnobSet::tn3_mfast, 0, 1, 1, {}},
        {"tn3", &seg::KnobSet::tn3, 0, 1, 1, {}},
        {"nt3", &seg::KnobSet::nt3, 0, 1, 1, {}},
        {"wgrad_fill", &seg::KnobSet::wgrad_fill, 1, 800, 1, {}},            // filter-gradient split-K, % of the CUs
        {"wgrad_nt32", &seg::KnobSet::wgrad_nt32, 0, 1, 1, {}},
        {"wgrad_nbias", &seg::KnobSet::wgrad_nbias, 1, 4, 1, {}},
        {"wgrad_nt", &seg::KnobSet::wgrad_nt, 0, 0, 0, {64, 128}},
        {"wgrad_halo", &seg::KnobSet::wgrad_halo, 0, 1, 1, {}},
        {"wgrad_pxs", &seg::KnobSet::wgrad_pxs, 0, 1, 1, {}},         // 64-wide wgrad_halo tiles: pixel-split waves
        {"smallc_tr", &seg::KnobSet::smallc_tr, 0, 1, 1, {}},         // conv_c8_fwd: transposed accumulators, 8-byte staging
        {"res16c", &seg::KnobSet::res16c, 0, 1, 1, {}},
        {"res16", &seg::KnobSet::res16, 0, 1, 1, {}},
        {"res64", &seg::KnobSet::res64, 0, 1, 1, {}},
        {"res64_pp", &seg::KnobSet::res64_pp, 0, 2, 1, {}},
        {"res16_dma", &seg::KnobSet::res16_dma, 0, 1, 1, {}},
        {"res16c_bh", &seg::KnobSet::res16c_bh, 0, 0, 0, {4, 8}},
        {"bn1x1s", &seg::KnobSet::bn1x1s, 0, 1, 1, {}},
        {"s1x1_st", &seg::KnobSet::s1x1_st, 0, 2, 1, {}},
        {"res16c_st", &seg::KnobSet::res16c_st, 0, 1, 1, {}},
        {"dropout_flat", &seg::KnobSet::dropout_flat, 0, 1, 1, {}},
        {"smallc", &seg::KnobSet::smallc, 0, 1, 1, {}},
        {"smallk", &seg::KnobSet::smallk, 0, 1, 1, {}},
        {"wpad", &seg::KnobSet::wpad, 0, 256, 8, {}},
#ifdef SEG_DIAG
        {"tn3_abl", &seg::KnobSet::tn3_abl, 0, 3, 1, {}},
        {"smallk_abl", &seg::KnobSet::smallk_abl, 0, 3, 1, {}},
        {"tn3_adam_abl", &seg::KnobSet::tn3_adam_abl, 0, 31, 1, {}},
        {"wgrad_abl", &seg::KnobSet::wgrad_abl, 0, 3, 1, {}},
        {"nt2_ablate", &seg::KnobSet::nt2_ablate, 0, 19, 1, {}},
#endif
    };
    for (const Knob& k : knobs)
        if (!strcmp(name, k.name)) return &k;
    return nullptr;
}
}  // namespace

namespace seg {
KnobSet& knobs() {
    constexpr int MAXDEV = 64;
    static KnobSet sets[MAXDEV];
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAXDEV) d = 0;
    return sets[d];
}
}  // namespace seg

// Sets one knob for the calling thread's current device (see knobs.h).
extern "C" int seg_set_option(const char* name, int value) {
    const Knob* k = name ? find_knob(name) : nullptr;
    if (!k) return SEG_EINVAL;
    bool ok;
    if (k->step) {
        ok = value >= k->lo && value <= k->hi && (value - k->lo) % k->step == 0;
    } else {
        ok = false;
        for (int v : k->only) ok = ok || (v != 0 && v == value);
    }
    if (!ok) return SEG_EINVAL;
    std::lock_guard<std::mutex> lk(g_knob_mu);
    (seg::knobs().*(k->var)).store(value, std::memory_order_relaxed);
    return SEG_OK;
}

extern "C" int seg_get_option(const char* name, int* value) {
    const Knob* k = name ? find_knob(name) : nullptr;
    if (!k || !value) return SEG_EINVAL;
    *value = (seg::knobs().*(k->var)).load(std::memory_order_relaxed);
    return SEG_OK;
}

extern "C" int seg_conv2d_fwd(const seg_conv_desc* d, const void* x, const void* w, const seg_epilogue* epi,
                              void* y, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !w || !y) return SEG_EINVAL;
    NTParams p = conv_fwd_params(d);
    p.x = x; p.w = w; p.y = y;
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    if (d->dil_w == d->dil_h && seg::smallc_fwd_ok(p, d->dtype, d->R, d->S, d->dil_h)) {
        seg::launch_smallc_fwd(p, d->dtype, (hipStream_t)stream);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2D whose ReLU mask is also written as bits (bits[pixel * ld_bits + k/8],
// bit k & 7: stored y > 0) for the next conv's seg_conv2d_bwd_data_bits --
// conv1_1 of FCN / VGG (3 -> 64), on conv_c8_fwd, the one kernel that writes
// them: 8 bytes per pixel beside the 128 of the map.
static bool fwd_relu_bits_params(const seg_conv_desc* d, const seg_epilogue* epi, int ld_bits, NTParams* out) {
    // (K = 64: 8-byte row stores)
    if (check_desc(d) || d->dil_w != d->dil_h || ld_bits < d->K / 8 || (d->K == 64 && ld_bits % 8)) return false;
    if (epi && epi->relu_mask) return false;
    NTParams p = conv_fwd_params(d);
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    if (!seg::smallc_fwd_ok(p, d->dtype, d->R, d->S, d->dil_h)) return false;
    p.epi.ld_bits = ld_bits;
    *out = p;
    return true;
}

extern "C" int seg_conv2d_fwd_relu_bits_ok(const seg_conv_desc* d) {
    NTParams p;
    seg_epilogue e = {};
    e.relu = 1;
    e.keep_prob = 1.f;
    return d && fwd_relu_bits_params(d, &e, d->K / 8, &p) ? 1 : 0;
}

extern "C" int seg_conv2d_fwd_relu_bits(const seg_conv_desc* d, const void* x, const void* w, const seg_epilogue* epi,
                                        void* y, void* bits, int ld_bits, void* stream) {
    if (!d || !x || !w || !y || !bits) return SEG_EINVAL;
    if (d->K == 64 && ((uintptr_t)bits & 7)) return SEG_EALIGN;
    NTParams p;
    if (!fwd_relu_bits_params(d, epi, ld_bits, &p)) return SEG_EINVAL;
    p.x = x; p.w = w; p.y = y;
    p.epi.ybits = reinterpret_cast<unsigned char*>(bits);
    seg::launch_smallc_fwd(p, d->dtype, (hipStream_t)stream);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

// Conv2D reading the HWIO filter copy ([R][S][C][K], the one the input
// gradient reads) on igemm_nt3's B-transposed form: a weight with one packed
// copy instead of two (seg_conv2d_fwd_hwio_ok).
static NTParams fwd_hwio_params(const seg_conv_desc* d) {
    NTParams p = conv_fwd_params(d);
    p.bt = 1;
    // [r][s][c][k]: c rows of K (+ the diagnostic row padding, as
    // conv_bwd_data_params reads the same copy) columns.  The HWIO-only
    // forward exists only while the plan picks igemm_nt3 whole: a kernel
    // option changed after the Session planned (e.g. nt3 = 0) makes this
    // entry refuse (SEG_EINVAL) -- such filters have no KRSC copy.
    p.w_col = d->K + g_wpad;
    p.w_tap = (long)d->C * (d->K + g_wpad);
    return p;
}

extern "C" int seg_conv2d_fwd_hwio_ok(const seg_conv_desc* d) {
    if (!d || check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return 0;
    return seg::nt_fwd_bt_ok(fwd_hwio_params(d), d->dtype) ? 1 : 0;
}

extern "C" int seg_conv2d_fwd_hwio(const seg_conv_desc* d, const void* x, const void* w_hwio, const seg_epilogue* epi,
                                   void* y, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !w_hwio || !y) return SEG_EINVAL;
    if (!seg_conv2d_fwd_hwio_ok(d)) return SEG_EINVAL;
    NTParams p = fwd_hwio_params(d);
    p.x = x; p.w = w_hwio; p.y = y;
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2D + bias + ReLU + MaxPool 2x2 / 2 in one launch: the pooled epilogue of
// conv_res64 / conv_halo_duo / conv_halo2 (seg_conv2d_fwd_pool_ok).
static bool fwd_pool_params(const seg_conv_desc* d, const seg_epilogue* epi, NTParams* out) {
    if (check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return false;
    if ((d->OH & 1) || (d->OW & 1) || d->OH < 2 || d->OW < 2) return false;
    if (epi && (epi->scale || epi->shift || epi->residual || epi->relu_mask || (epi->keep_prob > 0.f && epi->keep_prob < 1.f)))
        return false;
    NTParams p = conv_fwd_params(d);
    p.epi = make_epi(epi, d->k_valid, 0);
    if (d->dil_w == d->dil_h && seg::smallc_fwd_ok(p, d->dtype, d->R, d->S, d->dil_h)) return false;
    if (!seg::nt_pool_ok(p, d->dtype)) return false;
    *out = p;
    return true;
}

extern "C" int seg_conv2d_fwd_pool_ok(const seg_conv_desc* d) {
    if (!d) return 0;
    NTParams p;
    seg_epilogue e = {};
    e.relu = 1;
    e.keep_prob = 1.f;
    return fwd_pool_params(d, &e, &p) ? 1 : 0;
}

extern "C" int seg_conv2d_fwd_pool(const seg_conv_desc* d, const void* x, const void* w, const seg_epilogue* epi,
                                   void* y_pool, int ld_pool, void* idx, int ld_idx, void* ws, size_t ws_bytes,
                                   void* stream) {
    if (!d || !x || !w || !y_pool || ld_pool < d->K || (ld_pool & 7) || (idx && (ld_idx < d->K || (ld_idx & 7))))
        return SEG_EINVAL;
    if (((uintptr_t)y_pool & 15) || ((uintptr_t)idx & 7)) return SEG_EALIGN;
    NTParams p;
    if (!fwd_pool_params(d, epi, &p)) return SEG_EINVAL;
    p.x = x; p.w = w; p.y = nullptr;
    p.epi.pool_y = y_pool;
    p.epi.pool_idx = reinterpret_cast<unsigned char*>(idx);
    p.epi.ld_pool = ld_pool;
    p.epi.ld_idx = ld_idx;
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// BiasAddGrad of dy [N*OH*OW][K] when the filter-gradient kernel did not fuse it.
static int bias_grad_fallback(const seg_conv_desc* d, const void* dy, float* dbias, void* ws, size_t ws_bytes,
                              void* stream) {
    return seg_bias_relu_bwd(dy, d->ldy, nullptr, 0, const_cast<void*>(dy), d->ldy, dbias,
                             (long)d->N * d->OH * d->OW, d->K, d->k_valid, 0, 1.f, d->dtype, ws, ws_bytes, stream);
}

static seg::ProParams make_pro(const seg_prologue* pro, int cv) {
    seg::ProParams r = {};
    if (pro) {
        r.gamma = pro->gamma;
        r.beta = pro->beta;
        r.inv = 1.0f / sqrtf(1.0f + pro->eps);   // seg_bn_relu_fwd's arithmetic
        r.relu = pro->relu;
        r.cv = cv;
    }
    return r;
}

extern "C" int seg_conv2d_fwd_pro(const seg_conv_desc* d, const void* x, const seg_prologue* pro, const void* w,
                                  const seg_epilogue* epi, void* y, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !w || !y || !pro || !pro->gamma || !pro->beta) return SEG_EINVAL;
    NTParams p = conv_fwd_params(d);
    p.x = x; p.w = w; p.y = y;
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    p.pro = make_pro(pro, d->c_valid);
    if (seg::s1x1_ok(p, d->dtype, 1)) {
        seg::launch_s1x1(p, d->dtype, seg::device_cus(), (hipStream_t)stream);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2D (operand prologue optional) whose output also feeds a frozen
// BatchNorm(+ReLU): both maps in one launch (FC-DenseNet's bottleneck conv1 ->
// dropout -> BN -> ReLU, Network/model/FCDenseNet.py:28-31).  The kernel
// chosen for the conv must be one that writes the second output.
static int fwd_bn2_params(const seg_conv_desc* d, const void* x, const seg_prologue* pro, const void* w,
                          const seg_epilogue* epi, void* y, void* y2, int ld_y2, const float* gamma2,
                          const float* beta2, float eps2, int relu2, NTParams* out, bool* stream1x1) {
    if (check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return SEG_EINVAL;
    if (ld_y2 < d->K || ld_y2 % 8) return SEG_EINVAL;
    if (pro && (!pro->gamma || !pro->beta)) return SEG_EINVAL;
    NTParams p = conv_fwd_params(d);
    p.x = x; p.w = w; p.y = y;
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    if (pro) p.pro = make_pro(pro, d->c_valid);
    p.epi.y2 = y2;
    p.epi.ld_y2 = ld_y2;
    p.epi.y2_img = (long)d->OH * d->OW * ld_y2;
    p.epi.bn2_gamma = gamma2;
    p.epi.bn2_beta = beta2;
    p.epi.bn2_inv = 1.0f / sqrtf(1.0f + eps2);   // as seg_bn_relu_fwd
    p.epi.bn2_relu = relu2 ? 1 : 0;
    p.epi.bn2_cv = d->k_valid;
    *stream1x1 = pro && seg::s1x1_ok(p, d->dtype, 1);
    if (!*stream1x1 && !seg::nt_bn2_ok(p, d->dtype)) return SEG_EINVAL;
    *out = p;
    return SEG_OK;
}

extern "C" int seg_conv2d_fwd_bn2_ok(const seg_conv_desc* d, int with_prologue) {
    static const float one = 1.f;
    static seg_prologue pro = {&one, &one, 1e-3f, 1};
    NTParams p;
    bool s1;
    // shape-only query: aligned stand-ins for the buffers
    const void* a = reinterpret_cast<const void*>(uintptr_t(1) << 20);
    return fwd_bn2_params(d, a, with_prologue ? &pro : nullptr, a, nullptr, (void*)a, (void*)a,
                          d ? d->ldy : 0, &one, &one, 1e-3f, 1, &p, &s1) == SEG_OK;
}

extern "C" int seg_conv2d_fwd_bn2(const seg_conv_desc* d, const void* x, const seg_prologue* pro, const void* w,
                                  const seg_epilogue* epi, void* y, void* y2, int ld_y2, const float* gamma2,
                                  const float* beta2, float eps2, int relu2, void* ws, size_t ws_bytes,
                                  void* stream) {
    if (!x || !w || !y || !y2 || !gamma2 || !beta2) return SEG_EINVAL;
    NTParams p;
    bool s1 = false;
    int st = fwd_bn2_params(d, x, pro, w, epi, y, y2, ld_y2, gamma2, beta2, eps2, relu2, &p, &s1);
    if (st) return st;
    if (s1) {
        seg::launch_s1x1(p, d->dtype, seg::device_cus(), (hipStream_t)stream);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int seg_conv2d_bwd_filter_pro(const seg_conv_desc* d, const void* x, const seg_prologue* pro,
                                         const void* dy, float* dw, float* dbias, void* ws, size_t ws_bytes,
                                         void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !dy || !dw || !pro || !pro->gamma || !pro->beta) return SEG_EINVAL;
    TNParams p = conv_bwd_filter_params(d);
    p.x = x; p.b = dy; p.out = dw; p.dbias = nullptr;
    p.pro = make_pro(pro, d->c_valid);
    st = seg::launch_tn(p, d->dtype, ws, ws_bytes, (hipStream_t)stream);
    if (st || !dbias) return st;
    return bias_grad_fallback(d, dy, dbias, ws, ws_bytes, stream);
}

extern "C" int seg_conv2d_bwd_data(const seg_conv_desc* d, const void* dy, const void* w, const seg_epilogue* epi,
                                   void* dx, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!dy || !w || !dx) return SEG_EINVAL;
    if (d->stride_h != 1 || d->stride_w != 1) return SEG_EINVAL;  // FCN / FC-DenseNet convs are stride 1
    NTParams p = conv_bwd_data_params(d);
    p.x = dy; p.w = w; p.y = dx;
    if (epi) {
        const int ldr = epi->ld_residual ? epi->ld_residual : d->ldx;
        p.epi = make_epi(epi, d->C, (long)d->H * d->W * ldr, (long)d->H * d->W, d->ldx);
        if (epi->residual && epi->ld_residual == 0) p.epi.ld_res = d->ldx;
    }
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2DBackpropInput with the ReluGrad mask given as seg_conv2d_fwd_relu_bits'
// bits (epi->relu_mask null; epi->mask_scale applies): conv1_2's input
// gradient reads 8 bytes per pixel instead of conv1_1's 128-byte map row.
// conv_res64pp only (64 input channels, 3x3, stride 1).
static bool bwd_data_bits_params(const seg_conv_desc* d, const seg_epilogue* epi, const void* bits, int ld_bits,
                                 NTParams* out) {
    if (check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return false;
    if (d->stride_h != 1 || d->stride_w != 1) return false;
    if (epi && (epi->relu_mask || epi->residual)) return false;
    NTParams p = conv_bwd_data_params(d);
    p.epi.mask_scale = 1.f;              // (epi NULL: the plain ReluGrad)
    if (epi) {
        p.epi = make_epi(epi, d->C, 0, (long)d->H * d->W, d->ldx);
        if (epi->mask_scale != 0.f) p.epi.mask_scale = epi->mask_scale;
    }
    p.epi.mask_bits = reinterpret_cast<const unsigned char*>(bits);
    p.epi.ld_bits = ld_bits;
    if (!seg::nt_mask_bits_ok(p, d->dtype)) return false;
    *out = p;
    return true;
}

extern "C" int seg_conv2d_bwd_data_bits_ok(const seg_conv_desc* d) {
    NTParams p;
    // shape-only query: an aligned stand-in for the bits
    const void* a = reinterpret_cast<const void*>(uintptr_t(1) << 20);
    return d && bwd_data_bits_params(d, nullptr, a, d->C / 8, &p) ? 1 : 0;
}

extern "C" int seg_conv2d_bwd_data_bits(const seg_conv_desc* d, const void* dy, const void* w, const seg_epilogue* epi,
                                        const void* bits, int ld_bits, void* dx, void* ws, size_t ws_bytes,
                                        void* stream) {
    if (!d || !dy || !w || !bits || !dx) return SEG_EINVAL;
    if ((uintptr_t)bits & 7) return SEG_EALIGN;
    NTParams p;
    if (!bwd_data_bits_params(d, epi, bits, ld_bits, &p)) return SEG_EINVAL;
    p.x = dy; p.w = w; p.y = dx;
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2DBackpropInput + MaxPoolGrad (+ the ReluGrad of the pool's post-ReLU
// input) in one launch: the MaxPoolGrad epilogue of the halo kernels
// (EpiParams::unpool_y), no split-K.
extern "C" int seg_conv2d_bwd_data_unpool_ok(const seg_conv_desc* d) {
    if (!d || check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return 0;
    if (d->stride_h != 1 || d->stride_w != 1 || (d->C & 7) || (d->ldx & 7)) return 0;
    return seg::nt_unpool_ok(conv_bwd_data_params(d), d->dtype) ? 1 : 0;
}

extern "C" int seg_conv2d_bwd_data_unpool(const seg_conv_desc* d, const void* dy, const void* w,
                                          const seg_epilogue* epi, const void* idx, int ld_idx, int relu,
                                          void* dx_full, int ld_full, void* ws, size_t ws_bytes, void* stream) {
    if (!d || !dy || !w || !idx || !dx_full || ld_full < d->C || (ld_full & 7) || ld_idx < d->C || (ld_idx & 7))
        return SEG_EINVAL;
    if (((uintptr_t)dx_full & 15) || ((uintptr_t)idx & 7)) return SEG_EALIGN;
    if (!seg_conv2d_bwd_data_unpool_ok(d)) return SEG_EINVAL;
    if (epi && (epi->bias || epi->scale || epi->shift || epi->relu || epi->relu_mask ||
                (epi->keep_prob > 0.f && epi->keep_prob < 1.f)))
        return SEG_EINVAL;
    NTParams p = conv_bwd_data_params(d);
    p.x = dy; p.w = w; p.y = nullptr;
    if (epi && epi->residual) {     // the pooled gradient of the pool's other consumers, added first
        const int ldr = epi->ld_residual ? epi->ld_residual : d->ldx;
        p.epi = make_epi(epi, d->C, (long)d->H * d->W * ldr, (long)d->H * d->W, d->ldx);
        p.epi.ld_res = ldr;
    }
    p.epi.unpool_y = dx_full;
    p.epi.unpool_idx = reinterpret_cast<const unsigned char*>(idx);
    p.epi.ld_unpool = ld_full;
    p.epi.ld_uidx = ld_idx;
    p.epi.unpool_relu = relu != 0;
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

// Conv2DBackpropInput of a 1x1 conv whose input is relu(BN(x)) with the BN
// folded into its operand prologue, continued through the BatchNorm(+ReLU)
// backward in the GEMM epilogue: dx = dL/dx of the BN input (optionally
// accumulated in place), dgamma / dbeta from per-tile column sums.  16-bit
// igemm_nt2 only (seg_conv_bwd_data_bn_workspace returns 0 where it does not
// apply).
// kind: 1 = 1x1 (short-K igemm_nt2), 2 = 3x3 over 16 output channels (conv_res16c)
static int bwd_data_bn_params(const seg_conv_desc* d, NTParams& p) {
    if (check_desc(d) || (d->dtype != SEG_BF16 && d->dtype != SEG_F16)) return 0;
    if (d->stride_h != 1 || d->stride_w != 1 || d->C % 8) return 0;
    p = conv_bwd_data_params(d);
    if (d->R == 1 && d->S == 1 && d->K <= 64 * 8) return 1;   // no split-K
    if (seg::res16c_ok(p, d->dtype)) return 2;
    return 0;
}

// per-tile (1x1) or per-block (3x3) partial rows + the finish scratch
static long bwd_data_bn_rows(const seg_conv_desc* d, const NTParams& p, int kind) {
    if (kind == 2) return seg::res16c_grid(p, seg::device_cus());
    return seg::bn1x1s_ok(p, d->dtype) ? seg::bn1x1s_rows(p, seg::device_cus()) : seg::nt2_bn_rows(p.M);
}

extern "C" size_t seg_conv_bwd_data_bn_workspace(const seg_conv_desc* d) {
    NTParams p;
    const int kind = bwd_data_bn_params(d, p);
    if (!kind) return 0;
    return (size_t)bwd_data_bn_rows(d, p, kind) * 2 * d->C * sizeof(float) + seg::bn_grad_finish_scratch(d->C);
}

extern "C" long seg_conv_bwd_data_bn_part_rows(const seg_conv_desc* d) {
    NTParams p;
    const int kind = bwd_data_bn_params(d, p);
    return kind ? bwd_data_bn_rows(d, p, kind) : 0;
}

// The input-gradient launch through the BN backward; its dgamma / dbeta
// column sums left as partial rows [nrows][2 C] in `part`.
static int bwd_data_bn_launch(const seg_conv_desc* d, const void* dy, const void* w, const seg_bn_bwd* bn, void* dx,
                              float* part, void* stream, long* rows_out) {
    NTParams p;
    const int kind = bwd_data_bn_params(d, p);
    if (!kind) return SEG_EINVAL;
    if (!dy || !w || !dx || !bn || !bn->x || !bn->gamma || !bn->beta || !part) return SEG_EINVAL;
    if (bn->ldx % 8 || bn->ldx < d->C) return SEG_EINVAL;
    const bool drop = bn->keep_prob > 0.f && bn->keep_prob < 1.f;
    if ((drop || kind == 2) && bn->accumulate) return SEG_EINVAL;   // the 3x3 / dropout forms write dx
    if (drop && kind != 2) return SEG_EINVAL;
    *rows_out = bwd_data_bn_rows(d, p, kind);
    p.x = dy; p.w = w; p.y = dx;
    const float inv = 1.0f / sqrtf(1.0f + bn->eps);
    seg::EpiParams& e = p.epi;
    e.n_valid = d->C;
    e.keep_prob = 1.f;
    e.mask_scale = 1.f;
    if (bn->accumulate) {                             // dx += ... (concat gradient slice)
        e.residual = dx; e.ld_res = d->ldx; e.res_img = (long)d->H * d->W * d->ldx;
    }
    e.bn_x = bn->x; e.ld_bn_x = bn->ldx; e.bn_x_img = (long)d->H * d->W * bn->ldx;
    e.bn_gamma = bn->gamma; e.bn_beta = bn->beta; e.bn_inv = inv; e.bn_relu = bn->relu ? 1 : 0;
    e.bn_cv = d->c_valid; e.bn_part = part; e.bn_C = d->C;
    if (drop) {          // the dropout of the conv that produced x (counter pixel * C + c)
        e.keep_prob = bn->keep_prob;
        e.seed = bn->seed;
    }
    hipStream_t s = (hipStream_t)stream;
    if (kind == 1 && seg::bn1x1s_ok(p, d->dtype)) {
        const int st = seg::launch_bn1x1s(p, d->dtype, seg::device_cus(), s);
        if (st) return st;
    } else if (kind == 1) {
        seg::launch_nt2_bn(p, d->dtype, s);
    } else {
        seg::launch_res16c_bn(p, seg::device_cus(), s, d->dtype);
    }
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

extern "C" int seg_conv2d_bwd_data_bn(const seg_conv_desc* d, const void* dy, const void* w, const seg_bn_bwd* bn,
                                      void* dx, void* ws, size_t ws_bytes, void* stream) {
    if (!bn || !bn->dgamma || !bn->dbeta) return SEG_EINVAL;
    const size_t need = seg_conv_bwd_data_bn_workspace(d);
    if (!need) return SEG_EINVAL;
    if (!ws || ws_bytes < need) return SEG_EWORKSPACE;
    float* part = reinterpret_cast<float*>(ws);
    long nrows = 0;
    int st = bwd_data_bn_launch(d, dy, w, bn, dx, part, stream, &nrows);
    if (st) return st;
    float* scratch = part + nrows * 2 * d->C;
    return seg::bn_grad_finish(part, (int)nrows, d->C, d->c_valid, 1.0f / sqrtf(1.0f + bn->eps), bn->dgamma,
                               bn->dbeta, scratch, (hipStream_t)stream);
}

extern "C" int seg_conv2d_bwd_data_bn_part(const seg_conv_desc* d, const void* dy, const void* w,
                                           const seg_bn_bwd* bn, void* dx, float* part, long part_rows, void* stream) {
    const long rows = seg_conv_bwd_data_bn_part_rows(d);
    if (!rows) return SEG_EINVAL;
    if (part_rows != rows) return SEG_EWORKSPACE;   // planned for another launch geometry
    long nrows = 0;
    return bwd_data_bn_launch(d, dy, w, bn, dx, part, stream, &nrows);
}

extern "C" int seg_conv2d_bwd_filter(const seg_conv_desc* d, const void* x, const void* dy, float* dw, float* dbias,
                                     void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !dy || !dw) return SEG_EINVAL;
    TNParams p = conv_bwd_filter_params(d);
    p.x = x; p.b = dy; p.out = dw; p.dbias = dbias;
    st = seg::launch_tn(p, d->dtype, ws, ws_bytes, (hipStream_t)stream);
    if (st || !p.dbias) return st;
    return bias_grad_fallback(d, dy, dbias, ws, ws_bytes, stream);
}

// Split form of seg_conv2d_bwd_filter: _begin runs the filter-gradient kernel
// (and any BiasAddGrad it does not fuse) and leaves a split-K reduction
// pending in `ws` (pending = {splits, slab rows}); _end performs it, on any
// stream ordered after _begin's, so it can overlap the next layer's work.
extern "C" int seg_conv2d_bwd_filter_begin(const seg_conv_desc* d, const void* x, const void* dy, float* dw,
                                           float* dbias, void* ws, size_t ws_bytes, int* pending, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !dy || !dw || !pending) return SEG_EINVAL;
    TNParams p = conv_bwd_filter_params(d);
    p.x = x; p.b = dy; p.out = dw; p.dbias = dbias;
    seg::WgradPlan wp;
    const bool fuses_bias = seg::smallc_wgrad_ok(p, d->dtype) ||
                            (g_tn_variant == 2 && seg::wgrad_plan(p, d->dtype, seg::device_cus(), &wp));
    if (dbias && !fuses_bias) {          // reduce it now, while the workspace is free
        st = bias_grad_fallback(d, dy, dbias, ws, ws_bytes, stream);
        if (st) return st;
        p.dbias = nullptr;
    }
    pending[0] = 1;
    pending[1] = 0;
    p.defer = pending;
    return seg::launch_tn(p, d->dtype, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int seg_conv2d_bwd_filter_end(const seg_conv_desc* d, float* dw, float* dbias, void* ws,
                                         const int* pending, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!dw || !pending) return SEG_EINVAL;
    if (pending[0] <= 1) return SEG_OK;
    TNParams p = conv_bwd_filter_params(d);
    p.out = dw;
    p.dbias = dbias;
    p.partial = reinterpret_cast<float*>(ws);
    p.Mp = pending[1];
    if (!ws || p.Mp < p.M || (p.Mp > p.M && !dbias)) return SEG_EINVAL;
    seg::tn_reduce(p, pending[0], (hipStream_t)stream);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

static bool wgrad_adam_params(const seg_conv_desc* d, TNParams* out) {
    if (check_desc(d) || d->dtype != SEG_BF16 || g_tn_variant != 2) return false;
    TNParams p = conv_bwd_filter_params(d);
    if (seg::smallc_wgrad_ok(p, d->dtype)) return false;
    seg::WgradPlan wp;
    if (seg::wgrad_plan(p, d->dtype, seg::device_cus(), &wp)) return false;
    if (!seg::tn3_adam_ok(p, d->dtype)) return false;
    *out = p;
    return true;
}

extern "C" int seg_conv_wgrad_adam_fusable(const seg_conv_desc* d) {
    TNParams p;
    return wgrad_adam_params(d, &p) ? 1 : 0;
}

// KRSC copy from the HWIO copy the fused-Adam epilogue wrote: tr[n][rs][c] =
// rows[rs][c][n] for c < C, n < K (padding untouched).  One wave per 64 x 64
// tile, no LDS: lane (cg, nc) loads the 8 x 8 block rows c0+8cg.., columns
// n0+8nc.. as eight 16-byte row pieces (all eight in flight), transposes it in
// registers (v_perm pairs) and stores eight 16-byte column pieces; for every
// load / store instruction the wave touches eight full 128-byte runs.  (The
// LDS-staged 64 x 64 block form moved 2.8 TB/s on conv6: two loads in flight
// per lane and eight 2-byte LDS writes per chunk.)
__global__ __launch_bounds__(256) void rows_to_tr_k(const bf16* __restrict__ rows, bf16* __restrict__ tr, int RS,
                                                    int C, int K, int rows_ap, int rows_bp, int tr_ap, int ctiles,
                                                    int tiles) {
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= tiles) return;
    const int rs = blockIdx.y;
    const int c0 = (tile % ctiles) * 64 + (lane >> 3) * 8;
    const int n0 = (tile / ctiles) * 64 + (lane & 7) * 8;
    if (c0 >= C || n0 >= K) return;
    uint4 v[8];
    const bf16* src = rows + ((long)rs * rows_ap + c0) * rows_bp + n0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = make_uint4(0u, 0u, 0u, 0u);
        if (c0 + i < C && n0 < rows_bp) v[i] = *reinterpret_cast<const uint4*>(src + (long)i * rows_bp);
    }
    const unsigned* w = reinterpret_cast<const unsigned*>(v);   // w[4 * i + k]: row c0+i, columns n0+2k, +2k+1
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int n = n0 + j;
        if (n >= K) break;
        unsigned o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned a = w[4 * (2 * q) + j / 2], b = w[4 * (2 * q + 1) + j / 2];
            o[q] = (j & 1) ? ((a >> 16) | (b & 0xffff0000u)) : ((a & 0xffffu) | (b << 16));
        }
        bf16* dst = tr + ((long)n * RS + rs) * tr_ap + c0;
        if (c0 + 8 <= C) {
            *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            unsigned short* d16 = reinterpret_cast<unsigned short*>(dst);
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (c0 + i < C) d16[i] = (unsigned short)(o[i >> 1] >> (16 * (i & 1)));
        }
    }
}

extern "C" int seg_conv2d_bwd_filter_adam(const seg_conv_desc* d, const void* x, const void* dy, float* dw,
                                          float* dbias, const seg_adam_fused* a, void* ws, size_t ws_bytes,
                                          void* stream) {
    TNParams p;
    if (!x || !dy || !a || !a->p || !a->m || !a->v || a->t < 1) return SEG_EINVAL;
    if (!wgrad_adam_params(d, &p)) return SEG_EINVAL;
    if ((((uintptr_t)a->p | (uintptr_t)a->m | (uintptr_t)a->v | (uintptr_t)dw) & 15)) return SEG_EALIGN;
    p.x = x; p.b = dy; p.out = dw; p.dbias = nullptr;
    const double lr_t = (double)a->lr * sqrt(1.0 - pow((double)a->beta2, a->t)) / (1.0 - pow((double)a->beta1, a->t));
    p.adam.p = a->p; p.adam.m = a->m; p.adam.v = a->v;
    p.adam.rows = a->rows_dst; p.adam.rows_ap = a->rows_ap; p.adam.rows_bp = a->rows_bp;
    const bool tr_after = a->tr_dst && a->rows_dst && !g_adam_tr_fused;
    p.adam.tr = tr_after ? nullptr : a->tr_dst; p.adam.tr_ap = a->tr_ap; p.adam.RS = d->R * d->S;
    p.adam.lr_t = (float)lr_t; p.adam.b1 = a->beta1; p.adam.b2 = a->beta2; p.adam.eps = a->eps;
    p.adam.gs = a->grad_scale;
    p.adam.store_grad = dw != nullptr;
#ifdef SEG_DIAG
    p.adam.abl = g_tn3_adam_abl;
#endif
    p.Mp = p.M;
    p.partial = nullptr;
    seg::launch_tn3(p, 1, (hipStream_t)stream, SEG_BF16);
    SEG_CHECK_LAUNCH();
    if (tr_after) {
        const int RS = d->R * d->S, C = d->c_valid, K = d->k_valid;
        const int ctiles = (C + 63) / 64, ntiles = (K + 63) / 64;
        const int tiles = ctiles * ntiles;
        hipLaunchKernelGGL(rows_to_tr_k, dim3((tiles + 3) / 4, RS), dim3(256), 0, (hipStream_t)stream,
                           (const bf16*)a->rows_dst, (bf16*)a->tr_dst, RS, C, K, a->rows_ap, a->rows_bp, a->tr_ap,
                           ctiles, tiles);
        SEG_CHECK_LAUNCH();
    }
    if (!dbias) return SEG_OK;
    return bias_grad_fallback(d, dy, dbias, ws, ws_bytes, stream);
}

extern "C" int seg_tconv2d_fwd(const seg_conv_desc* d, const void* x, const void* w, const seg_epilogue* epi,
                               void* y, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !w || !y) return SEG_EINVAL;
    if (d->R % d->stride_h || d->S % d->stride_w) return SEG_EINVAL;
    if (const int kq = tconv_dense_kq(d)) {
        const int M = d->N * d->H * d->W, Nn = d->R * d->S * kq;
        const size_t zbytes = tconv_dense_zbytes(d);
        if (!ws || ws_bytes < seg_conv_workspace(d, 3)) return SEG_EWORKSPACE;
        NTParams g = dense_nt(M, Nn, d->C, x, d->ldx, w, ws, Nn);
        g.x_img = (long)d->H * d->W * d->ldx; g.IH = d->H; g.IW = d->W; g.Ha = d->H; g.Wa = d->W;
        g.y_img = (long)d->H * d->W * Nn; g.OH = d->H; g.OW = d->W;
        int st2 = seg::launch_nt(g, d->dtype, 1, g.M, (char*)ws + zbytes, ws_bytes - zbytes, (hipStream_t)stream);
        if (st2) return st2;
        const long total = (long)d->N * d->OH * d->OW;
        const int grid = seg_grid_1d(total, 256);
        const float* bias = epi ? epi->bias : nullptr;
        const void* res = epi ? epi->residual : nullptr;
        const int ldr = epi ? epi->ld_residual : 0;
#define COL2IM(T, KQ) hipLaunchKernelGGL((tconv_col2im_k<T, KQ>), dim3(grid), dim3(256), 0, (hipStream_t)stream, \
                                         (const T*)ws, (T*)y, d->N, d->H, d->W, d->OH, d->OW, d->k_valid, d->R, d->S, \
                                         d->stride_h, d->pad_top, d->pad_left, d->ldy, bias, (const T*)res, ldr)
        if (d->dtype == SEG_BF16) {
            if (kq == 2) COL2IM(bf16, 2); else if (kq == 4) COL2IM(bf16, 4); else COL2IM(bf16, 8);
        } else if (d->dtype == SEG_F16) {
            if (kq == 2) COL2IM(f16, 2); else if (kq == 4) COL2IM(f16, 4); else COL2IM(f16, 8);
        } else {
            if (kq == 2) COL2IM(float, 2); else if (kq == 4) COL2IM(float, 4); else COL2IM(float, 8);
        }
#undef COL2IM
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    NTParams p = tconv_fwd_params(d);
    p.x = x; p.w = w; p.y = y;
    p.epi = make_epi(epi, d->k_valid, (long)d->OH * d->OW * (epi ? epi->ld_residual : 0));
    return seg::launch_nt(p, d->dtype, d->stride_h * d->stride_w, p.M, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int seg_tconv2d_bwd_data(const seg_conv_desc* d, const void* dy, const void* w, const seg_epilogue* epi,
                                    void* dx, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!dy || !w || !dx) return SEG_EINVAL;
    if (const int kq = tconv_dense_kq(d)) {
        const int M = d->N * d->H * d->W, Kd = d->R * d->S * kq;
        const size_t zbytes = tconv_dense_zbytes(d);
        if (!ws || ws_bytes < seg_conv_workspace(d, 4)) return SEG_EWORKSPACE;
        st = launch_gather_dy(d, dy, ws, (hipStream_t)stream);
        if (st) return st;
        NTParams g = dense_nt(M, d->C, Kd, ws, Kd, w, dx, d->ldx);
        g.x_img = (long)d->H * d->W * Kd; g.IH = d->H; g.IW = d->W; g.Ha = d->H; g.Wa = d->W;
        g.y_img = (long)d->H * d->W * d->ldx; g.OH = d->H; g.OW = d->W;
        if (epi) {
            const int ldr = epi->ld_residual ? epi->ld_residual : d->ldx;
            g.epi = make_epi(epi, d->C, (long)d->H * d->W * ldr, (long)d->H * d->W, d->ldx);
            if (epi->residual && epi->ld_residual == 0) g.epi.ld_res = d->ldx;
        }
        return seg::launch_nt(g, d->dtype, 1, g.M, (char*)ws + zbytes, ws_bytes - zbytes, (hipStream_t)stream);
    }
    NTParams p = tconv_bwd_data_params(d);
    p.x = dy; p.w = w; p.y = dx;
    if (epi) {
        const int ldr = epi->ld_residual ? epi->ld_residual : d->ldx;
        p.epi = make_epi(epi, d->C, (long)d->H * d->W * ldr, (long)d->H * d->W, d->ldx);
        if (epi->residual && epi->ld_residual == 0) p.epi.ld_res = d->ldx;
    }
    return seg::launch_nt(p, d->dtype, 1, p.M, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int seg_tconv2d_bwd_filter(const seg_conv_desc* d, const void* x, const void* dy, float* dw,
                                      float* dbias, void* ws, size_t ws_bytes, void* stream) {
    int st = check_desc(d);
    if (st) return st;
    if (!x || !dy || !dw) return SEG_EINVAL;
    if (const int kq = tconv_dense_kq(d)) {
        const int P = d->N * d->H * d->W, Md = d->R * d->S * kq;
        const size_t zbytes = tconv_dense_zbytes(d);
        if (!ws || ws_bytes < seg_conv_workspace(d, 5)) return SEG_EWORKSPACE;
        st = launch_gather_dy(d, dy, ws, (hipStream_t)stream);
        if (st) return st;
        TNParams g = {};
        g.M = Md; g.N = d->C; g.P = P;
        g.x = ws; g.x_img = (long)d->H * d->W * Md; g.IH = d->H; g.IW = d->W; g.Cg = Md; g.ldx = Md;
        g.Ha = d->H; g.Wa = d->W; g.ish = 1; g.isw = 1; g.ioh = 0; g.iow = 0; g.tsh = 1; g.tsw = 1; g.taps_w = 1;
        g.b = x; g.ldb = d->ldx;
        g.out = dw; g.o_tap = 0; g.o_c = d->c_valid; g.o_n = 1;   // [(r,s,k)][c] = TF [kh][kw][Cout][Cin]
        g.c_valid = Md; g.n_valid = d->c_valid;
        st = seg::launch_tn(g, d->dtype, (char*)ws + zbytes, ws_bytes - zbytes, (hipStream_t)stream);
        if (st || !dbias) return st;
        return bias_grad_fallback(d, dy, dbias, (char*)ws + zbytes, ws_bytes - zbytes, stream);
    }
    TNParams p = tconv_bwd_filter_params(d);
    p.x = dy; p.b = x; p.out = dw;          // dy is the gathered operand here: bias via the fallback
    st = seg::launch_tn(p, d->dtype, ws, ws_bytes, (hipStream_t)stream);
    if (st || !dbias) return st;
    return bias_grad_fallback(d, dy, dbias, ws, ws_bytes, stream);
}

// ---------------------------------------------------------------------------
// filter packing
// ---------------------------------------------------------------------------
// dst [RS][ap][bp] <- src [RS][av][bv]: one thread per 8 consecutive b.
template <typename T>
__global__ void pack_rows_k(const float* __restrict__ src, T* __restrict__ dst, int RS, int av, int bv, int ap,
                            int bp) {
    const int b8 = bp / 8;
    const long total = (long)RS * ap * b8;
    const bool vec = (bv & 3) == 0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int bc = (int)(i % b8);
        const long ra = i / b8;              // rs * ap + a
        const int a = (int)(ra % ap);
        const long rs = ra / ap;
        float v[8];
        const int b0 = bc * 8;
        const float* srow = src + (rs * av + a) * (long)bv;
        if (a < av && vec && b0 + 8 <= bv) {
            const float4 x0 = *reinterpret_cast<const float4*>(srow + b0);
            const float4 x1 = *reinterpret_cast<const float4*>(srow + b0 + 4);
            v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
            v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (a < av && b0 + e < bv) ? srow[b0 + e] : 0.f;
        }
        T* d = dst + ra * bp + b0;
        if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4*>(d) = Chunk<T>::pack(v);
        } else {
            *reinterpret_cast<uint4*>(d) = Chunk<float>::pack(v);
            *reinterpret_cast<uint4*>(d + 4) = Chunk<float>::pack(v + 4);
        }
    }
}

// dst [bp][RS][ap] <- src [RS][av][bv]: 64x64 tiles transposed through LDS.
template <typename T>
__global__ __launch_bounds__(256) void pack_transpose_k(const float* __restrict__ src, T* __restrict__ dst, int RS,
                                                        int av, int bv, int ap, int bp) {
    __shared__ float tile[64][65];
    const int tiles_a = (ap + 63) / 64;
    const int ta = blockIdx.x % tiles_a, tb = blockIdx.x / tiles_a;
    const long rs = blockIdx.y;
    const int a0 = ta * 64, b0 = tb * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {          // rows of a, coalesced along b
        const int a = a0 + r, b = b0 + tx;
        tile[r][tx] = (a < av && b < bv) ? src[(rs * av + a) * (long)bv + b] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {          // rows of b, coalesced along a
        const int b = b0 + r, a = a0 + tx;
        if (b < bp && a < ap) dst[((long)b * RS + rs) * ap + a] = from_f32<T>(tile[tx][r]);
    }
}

extern "C" int seg_pack_filter(const float* src, void* dst, int R, int S, int a_valid, int b_valid, int a_pad,
                               int b_pad, int mode, int dtype, void* stream) {
    if (!src || !dst || a_pad < a_valid || b_pad < b_valid || mode < 0 || mode > 3) return SEG_EINVAL;
    const int bmajor = (mode == 0 || mode == 3);
    hipStream_t st = (hipStream_t)stream;
    const int RS = R * S;
    // a_pad may be the true channel count of a tap-dense tconv copy (modes 2, 3:
    // seg_tconv_filter_apad); everything else is padded to 8
    if ((b_pad & 7) || ((a_pad & 7) && (mode < 2 || (a_pad & 1)))) return SEG_EALIGN;
    if (bmajor) {
        dim3 grid(((a_pad + 63) / 64) * ((b_pad + 63) / 64), RS);
        if (dtype == SEG_BF16)
            hipLaunchKernelGGL(pack_transpose_k<bf16>, grid, dim3(256), 0, st, src, (bf16*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else if (dtype == SEG_F32)
            hipLaunchKernelGGL(pack_transpose_k<float>, grid, dim3(256), 0, st, src, (float*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else if (dtype == SEG_F16)
            hipLaunchKernelGGL(pack_transpose_k<f16>, grid, dim3(256), 0, st, src, (f16*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else
            return SEG_EINVAL;
    } else {
        const long total = (long)RS * a_pad * (b_pad / 8);
        const int grid = seg_grid_1d(total, 256);
        if (dtype == SEG_BF16)
            hipLaunchKernelGGL(pack_rows_k<bf16>, dim3(grid), dim3(256), 0, st, src, (bf16*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else if (dtype == SEG_F32)
            hipLaunchKernelGGL(pack_rows_k<float>, dim3(grid), dim3(256), 0, st, src, (float*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else if (dtype == SEG_F16)
            hipLaunchKernelGGL(pack_rows_k<f16>, dim3(grid), dim3(256), 0, st, src, (f16*)dst, RS, a_valid, b_valid, a_pad, b_pad);
        else
            return SEG_EINVAL;
    }
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}
