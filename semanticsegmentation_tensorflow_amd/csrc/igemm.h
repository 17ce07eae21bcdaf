// Internal parameter blocks of the implicit-GEMM kernels (not part of the C-ABI).
#pragma once
#include "common.h"

namespace seg {

struct EpiParams {
    const float* bias;
    const float* scale;
    const float* shift;
    const void* residual;
    long res_img;     // elements per image of the residual
    int ld_res;
    int relu;
    float keep_prob;
    uint64_t seed;
    int n_valid;      // columns >= n_valid are written as 0 (padding channels)
    // ReluGrad of the layer that produced this op's input (gradient kernels):
    // v = mask[pixel, col] > 0 ? v * mask_scale : 0
    const void* mask;
    long mask_img;
    int ld_mask;
    float mask_scale;
    // BatchNorm(+ReLU) backward of the BN folded into this conv's operand
    // prologue (input gradients, igemm_nt2 only): v = acc = dL/d relu(BN(x));
    // dz = v * [x*g*inv + beta > 0 or !bn_relu]; out = dz*g*inv (+ residual);
    // column sums of dz*x and dz -> bn_part[M tile][2 * bn_C]
    const void* bn_x;
    long bn_x_img;
    int ld_bn_x;
    const float* bn_gamma;
    const float* bn_beta;
    float bn_inv;
    int bn_relu;
    int bn_cv;
    float* bn_part;
    int bn_C;
    // MaxPool 2x2 / stride 2 of this conv's output fused into the epilogue
    // (conv_res64, conv_halo_duo, conv_halo2): the conv output is not written;
    // pool_y [img][OH/2][OW/2][ld_pool] gets the pooled map, pool_idx (may be
    // null) the switches in seg_maxpool2x2_fwd_argmax's encoding (row stride
    // ld_idx bytes).  Whole windows only (OH, OW even; checked by the host).
    void* pool_y;
    unsigned char* pool_idx;
    int ld_pool, ld_idx;
    // Frozen BatchNorm(+ReLU) of this conv's output written beside it
    // (seg_conv2d_fwd_bn2: FC-DenseNet's bottleneck conv1 -> BN -> ReLU):
    // y2 = relu(fma(y, bn2_gamma * bn2_inv, bn2_beta)) from the stored
    // (rounded) y, channels >= bn2_cv 0 -- seg_bn_relu_fwd's arithmetic.
    // conv1x1_stream and igemm_nt2 (no split-K) only; 16-bit types.
    void* y2;
    long y2_img;
    int ld_y2;
    const float* bn2_gamma;
    const float* bn2_beta;
    float bn2_inv;
    int bn2_relu;
    int bn2_cv;
    // MaxPoolGrad of the 2x2 / 2 MaxPool whose output this input gradient is
    // (conv_halo / conv_halo_duo / conv_halo2, no split-K): the pooled
    // gradient is not written; each value, rounded to the storage type, goes
    // to the window element unpool_idx selects (seg_maxpool2x2_fwd_argmax's
    // switches, row stride ld_uidx bytes; 0 with unpool_relu and bit 2 clear:
    // the ReluGrad of the post-ReLU pool input), zeros to the other three, in
    // unpool_y [img][2 OH][2 OW][ld_unpool] -- bit for bit the unfused
    // output + seg_maxpool2x2_bwd_argmax.  Output dims (OH, OW) pooled, unit
    // output stride (checked by the host).
    void* unpool_y;
    const unsigned char* unpool_idx;
    int ld_unpool, ld_uidx, unpool_relu;
    // The ReLU mask as bits: bit k & 7 of byte k >> 3 of a pixel's ld_bits-byte
    // row, pixels dense over the batch (seg_conv2d_fwd_relu_bits).  ybits: a
    // forward also writes stored y > 0 there (conv_c8_fwd only); mask_bits: an
    // input gradient's ReluGrad mask in place of `mask` (conv_res64pp only) --
    // 1 bit instead of 2 bytes per element.
    unsigned char* ybits;
    const unsigned char* mask_bits;
    int ld_bits;
};

// The MaxPoolGrad store of EpiParams::unpool_y for the 8 channels col0.. of
// pooled pixel (oy, ox) of image img, v = the epilogue's fp32 values.
template <typename T>
__device__ __forceinline__ void unpool_store8(const EpiParams& e, long img, int OH, int OW, int oy, int ox, int col0,
                                              const float* v) {
    static_assert(sizeof(T) == 2, "8 channels per 16-byte chunk");
    const long pp = (img * OH + oy) * (long)OW + ox;
    const unsigned long long code = *reinterpret_cast<const unsigned long long*>(e.unpool_idx + pp * e.ld_uidx + col0);
    // the values rounded as the unfused output store rounds them, then routed
    // as 16-bit halves of the packed words (few live registers: the halo
    // kernels run at 128 VGPRs)
    const uint4 g = Chunk<T>::pack(v);
    const unsigned gw[4] = {g.x, g.y, g.z, g.w};
    unsigned live = 0;             // bit j: channel j passes the ReluGrad
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (!e.unpool_relu || ((code >> (8 * j + 2)) & 1ull)) live |= 1u << j;
    const long UW = 2L * OW;
    T* b = reinterpret_cast<T*>(e.unpool_y) + ((img * 2 * OH + 2 * oy) * UW + 2 * ox) * e.ld_unpool + col0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        unsigned o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool k0 = (live >> (2 * i) & 1u) && ((code >> (16 * i)) & 3ull) == (unsigned long long)q;
            const bool k1 = (live >> (2 * i + 1) & 1u) && ((code >> (16 * i + 8)) & 3ull) == (unsigned long long)q;
            o[i] = (k0 ? (gw[i] & 0xffffu) : 0u) | (k1 ? (gw[i] & 0xffff0000u) : 0u);
        }
        T* dst = b + ((q >> 1) * UW + (q & 1)) * e.ld_unpool;
        *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// dgamma / dbeta from per-tile partial rows [nrows][2C] (eltwise.hip);
// scratch: bn_grad_finish_scratch(C) bytes
size_t bn_grad_finish_scratch(int C);
int bn_grad_finish(const float* part, int nrows, int C, int cv, float inv, float* dgamma, float* dbeta,
                   float* scratch, hipStream_t s);

// Optional A-operand prologue: the operand is relu(x * gamma[c] * inv + beta[c])
// (frozen-statistics BatchNorm + ReLU of the producing layer, applied while
// staging; zero-padded (out-of-image) elements stay zero, as TF pads the BN
// output) -- FC-DenseNet's BN -> ReLU -> conv (Network/model/FCDenseNet.py:25-28).
struct ProParams {
    const float* gamma;   // null: off
    const float* beta;
    float inv;            // 1 / sqrt(1 + eps), as seg_bn_relu_fwd
    int relu;
    int cv;               // valid channels
};

// C[m][n] = sum_k A[m][k] B[n][k].  Row m -> (img, a, b) on an Ha x Wa grid;
// reduction k -> (tap=(j,i), channel c), taps_w taps along w.
// A element: x[img, a*ish + j*tsh + ioh, b*isw + i*tsw + iow, c]  (0 outside)
// B element: w[n*w_col + ((rb + rstep*j)*Sfull + (sb + sstep*i))*w_tap + c]
// Output   : y[img, a*osh + ooh, b*osw + oow, n]
struct NTParams {
    int M, N, K;
    const void* x;
    long x_img;
    int IH, IW, C, ldx;
    int Ha, Wa, ish, isw, ioh, iow, tsh, tsw, taps_w;
    const void* w;
    long w_col, w_tap;
    int rb, rstep, sb, sstep, Sfull;
    void* y;
    long y_img;
    int OH, OW, ldy, osh, osw, ooh, oow;
    EpiParams epi;
    float* partial;
    int kt_per_split;
    // conv2d_transpose phase split: blockIdx.z = ph*st_w + pw
    int phase, st_h, st_w, pad_t, pad_l, Nimg;
    ProParams pro;
    int kv;        // valid reduction channels per tap (0: all C; the rest are zero padding)
    // B given as [k][n] rows (w = tap * w_tap + c * w_col + n: the HWIO copy);
    // igemm_nt3 only (nt_fwd_bt_ok)
    int bt;
};

// C[m][n] = sum_p A[p][m] B[p][n].  p -> (img, a, b) on an Ha x Wa grid;
// m -> (tap=(j,i), c) with Cg channels per tap.
// A element: x[img, a*ish + j*tsh + ioh, b*isw + i*tsw + iow, c]
// B element: b[p*ldb + n]
// Output   : out[tap*o_tap + c*o_c + n*o_n] for c < c_valid, n < n_valid.
// 8 consecutive fp32 values staged in LDS (the epilogues' row reads)
__device__ __forceinline__ void splitk_lds8(const char* src, float v[8]) {
    const float4 lo = *reinterpret_cast<const float4*>(src);
    const float4 hi = *reinterpret_cast<const float4*>(src + 16);
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
}


// Pixel cursor (img, row a, col b) over the N x Ha x Wa GEMM-k grid of a TN
// (filter-gradient) kernel, advanced by a fixed step per k tile.  The step is
// split once per kernel into q rows + r columns (0 <= r < Wa), so an advance
// is two adds and at most one carry into the row and one into the image --
// instead of a divergent `while (b >= Wa)` loop (~35 VALU / SALU per DMA piece
// on conv6's 39-wide rows, ~40 % of the filter-gradient main loop's VALU).
// Exact when q + 1 <= Ha (the step spans less than an image); otherwise
// (images of fewer pixels than the step) the general loop runs.
struct PixStep {
    int q, r, fast;
    __device__ __forceinline__ PixStep(int step, int Ha, int Wa) {
        q = step / Wa;
        r = step - q * Wa;
        fast = q + 1 <= Ha;
    }
    __device__ __forceinline__ void advance(int step, int Ha, int Wa, int& img, int& a, int& b) const {
        if (fast) {
            b += r;
            a += q;
            if (b >= Wa) { b -= Wa; ++a; }
            if (a >= Ha) { a -= Ha; ++img; }
        } else {
            b += step;
            while (b >= Wa) {
                b -= Wa;
                if (++a == Ha) { a = 0; ++img; }
            }
        }
    }
};

struct TNParams {
    int M, N, P;
    const void* x;
    long x_img;
    int IH, IW, Cg, ldx;
    int Ha, Wa, ish, isw, ioh, iow, tsh, tsw, taps_w;
    const void* b;
    int ldb;
    float* out;
    long o_tap, o_c, o_n;
    int c_valid, n_valid;
    float* partial;
    int kt_per_split;
    // BiasAddGrad fused into the filter gradient: dbias[n] = sum_p b[p][n]
    // (kernels that support it clear the pointer after launching); split-K
    // slabs then carry it as an extra row M, so slabs hold Mp = M + 1 rows.
    float* dbias;
    int Mp;
    // non-null: leave a split-K reduction pending (slabs stay in the
    // workspace) and report {splits, Mp} here instead of reducing
    int* defer;
    // TF1 Adam fused into the filter-gradient epilogue (igemm_tn3 only; p == null: off)
    struct {
        float *p, *m, *v;      // fp32 master slices indexed like out
        void* rows;            // bf16 rows copy [(tap*rows_ap + c)*rows_bp + n] or null
        int rows_ap, rows_bp;
        void* tr;              // bf16 transposed copy [(n*RS + tap)*tr_ap + c] or null
        int tr_ap, RS;
        float lr_t, b1, b2, eps, gs;
        int store_grad;        // also write the gradient to out
        int abl;               // diagnostics (garbage results): g_tn3_adam_abl bits
        int stagger;           // half tiles: second block per CU starts this many 10 ns ticks late
        int first_round;       // blocks of the first dispatch round (2 per CU)
        int* cu_slots;         // per-CU arrival counters (zeroed per launch)
    } adam;
    ProParams pro;             // A = x operand prologue (igemm_tn only)
};

int launch_nt(NTParams& p, int dtype, int nphases, int max_m, void* ws, size_t ws_bytes, hipStream_t s);
bool nt_pool_ok(const NTParams& p, int dtype);   // launch_nt's kernel fuses EpiParams::pool_y
bool nt_fwd_bt_ok(const NTParams& p, int dtype);
bool nt_unpool_ok(const NTParams& p, int dtype);
bool nt_mask_bits_ok(const NTParams& p, int dtype);
int launch_tn(TNParams& p, int dtype, void* ws, size_t ws_bytes, hipStream_t s);
void tn_reduce(TNParams& p, int splits, hipStream_t s);   // a pending (p.defer) split-K reduction
size_t nt_workspace(int M, int N, int K, int dtype, int phase);
size_t tn_workspace(int M, int N, int P, int dtype);
void nt_info(int M, int N, int K, int dtype, int phase, int* bm, int* bn, int* splits);
const char* nt_choice(const NTParams& p, int dtype, int nphases, int max_m, int* bm, int* bn, int* splits);
void tn_info(int M, int N, int P, int dtype, int* bm, int* bn, int* splits);
void launch_nt2(NTParams& p, int dtype, int bn, int gridz, int max_m, hipStream_t s);
void launch_nt2_bn(NTParams& p, int dtype, hipStream_t s);
long nt2_bn_rows(int M);
// dense1x1.hip: the 1x1 BN-backward input gradient streamed (K = 64)
bool bn1x1s_ok(const NTParams& p, int dtype);
int bn1x1s_rows(const NTParams& p, int cus);
int launch_bn1x1s(NTParams& p, int dtype, int cus, hipStream_t s);
bool nt2_short(const NTParams& p, int dtype);
void launch_tn2(TNParams& p, int bm, int bn, int splits, hipStream_t s, int dtype = SEG_BF16);

// 256 x 256 NT tiles (igemm3.hip) for bf16 with N > 128
bool nt3_ok(const NTParams& p, int dtype);
// the 16-byte chunk v of channels c0..c0+EPC-1 through the prologue
template <typename T>
__device__ __forceinline__ uint4 apply_pro(const ProParams& pro, uint4 v, int c0) {
    constexpr int EPC = dt_traits<T>::EPC;
    float f[EPC];
    Chunk<T>::unpack(v, f);
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
        const int c = c0 + e;
        const float sc = c < pro.cv ? pro.gamma[c] * pro.inv : 0.f;
        const float sh = c < pro.cv ? pro.beta[c] : 0.f;
        float o = f[e] * sc + sh;
        if (pro.relu) o = fmaxf(o, 0.f);
        f[e] = o;
    }
    return Chunk<T>::pack(f);
}

// LDS-DMA kernels (igemm2.hip) apply the prologue after the LDS read, so only
// where no operand element is zero padding: single-tap (1x1) problems.
// tn2: the transposed A fragment is 8 pixels of ONE channel -> scalar pair.
template <typename T>
__device__ __forceinline__ uint4 pro_affine(uint4 v, float sc, float sh, int relu) {
    float f[8];
    Chunk<T>::unpack(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float o = f[e] * sc + sh;
        f[e] = relu ? fmaxf(o, 0.f) : o;
    }
    return Chunk<T>::pack(f);
}
// nt2: the A fragment is 8 channels of one pixel; ss = (scale, shift) x 8
template <typename T>
__device__ __forceinline__ uint4 pro_affine8(uint4 v, const float* ss, int relu) {
    float f[8];
    Chunk<T>::unpack(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float o = f[e] * ss[2 * e] + ss[2 * e + 1];
        f[e] = relu ? fmaxf(o, 0.f) : o;
    }
    return Chunk<T>::pack(f);
}
constexpr int NT2_PRO_MAXK = 1024;    // (scale, shift) table in LDS
bool nt2_pro_ok(const NTParams& p, int dtype, int nphases);
// persistent streaming 1x1 conv (dense1x1.hip): FC-DenseNet bottleneck convs
bool s1x1_ok(const NTParams& p, int dtype, int nphases);
void launch_s1x1(NTParams& p, int dtype, int cus, hipStream_t s);
void launch_nt2_pro(NTParams& p, int dtype, int gridz, int max_m, hipStream_t s);
void launch_tn2_pro(TNParams& p, int bm, int bn, int splits, hipStream_t s, int dtype);

inline bool nt3_applies(int N, int dtype) { return g_nt3 && (dtype == SEG_BF16 || dtype == SEG_F16) && N > 128; }
// Split-K count for `tiles` output tiles of a one-block-per-CU kernel: the
// s <= min(smax, ceil(cus / tiles)) minimising rounds / s, rounds =
// ceil(tiles * s / cus) (the smaller s on ties).  The plain ceil(cus / tiles)
// overshoots the CU count by a few blocks for many tile counts (C3's
// transposed-conv gradients: 20 x 13 = 260, 54 x 5 = 270, 30 x 9 = 270 blocks
// on 256 CUs), and the second round of 4-14 blocks doubles the launch.
inline int one_round_splits(long tiles, int cus, int smax) {
    if (tiles <= 0 || tiles >= cus || smax <= 1) return 1;
    const int hi = (int)std::min<long>(smax, (cus + tiles - 1) / tiles);
    int best = 1;
    double best_t = 1e30;
    for (int s = 1; s <= hi; ++s) {
        const double t = (double)((tiles * s + cus - 1) / cus) / s;
        if (t < best_t * 0.999) { best_t = t; best = s; }
    }
    return best;
}
void nt3_info(int M, int N, int K, int cus, int* splits);
void launch_nt3(NTParams& p, int gridz, int max_m, hipStream_t s, int dtype);
bool tn3_ok(const TNParams& p, int dtype);
inline bool tn3_applies(int M, int N, int dtype) {
    return g_tn3 && (dtype == SEG_BF16 || dtype == SEG_F16) && M >= 256 && N > 128;
}
void tn3_info(int M, int N, int P, int cus, int* splits);
void launch_tn3(TNParams& p, int splits, hipStream_t s, int dtype);
bool tn3_adam_ok(const TNParams& p, int dtype);

// halo-tiled direct conv (halo.hip) for stride-1 NT problems
struct HaloPlan {
    int bw, hi, bn, splits;
    long tiles;
    int geom[10];
};
int device_cus();
bool halo_plan(const NTParams& p, int dtype, int max_splits, int cus, HaloPlan* hp);
enum { HALO_K1 = 0, HALO_KDUO = 1, HALO_K2 = 2, HALO_K4 = 3 };   // conv_halo, conv_halo_duo, conv_halo2, conv_halo4
int halo_kernel(const NTParams& p, const HaloPlan& hp, int dtype);
bool halo_unpools(const HaloPlan& hp, int kernel);
bool halo_pools(const HaloPlan& hp, int kernel);
int launch_halo(NTParams& p, const HaloPlan& hp, int kernel, hipStream_t s, int dtype = SEG_BF16);
// the launch plan for p writes EpiParams.y2 (seg_conv2d_fwd_bn2)
bool nt_bn2_ok(const NTParams& p, int dtype);
bool res16c_ok(const NTParams& p, int dtype);
void launch_res16c(NTParams& p, int cus, hipStream_t s, int dtype);
int res16c_grid(const NTParams& p, int cus);
void launch_res16c_bn(NTParams& p, int cus, hipStream_t s, int dtype);
bool res64_ok(const NTParams& p, int dtype);
int launch_res64(NTParams& p, int cus, hipStream_t s, int dtype = SEG_BF16);

// 8-input-channel first layer (smallc.hip)
bool smallc_fwd_ok(const NTParams& p, int dtype, int R, int S, int dil);
void launch_smallc_fwd(NTParams& p, int dtype, hipStream_t s);
// single-tap NT with K <= 16 (a classifier head's input gradient): streaming kernel
bool smallk_ok(const NTParams& p, int dtype);
void launch_smallk(NTParams& p, int dtype, int cus, hipStream_t s);
bool smallc_wgrad_ok(const TNParams& p, int dtype);
int smallc_wgrad_splits(const TNParams& p, int cus);
void launch_smallc_wgrad(TNParams& p, int dtype, int splits, hipStream_t s);

// halo-tiled filter gradient (wgrad.hip) for stride-1 3x3 TN problems
struct WgradPlan {
    int bw, nt, splits, nbias;
    int pxs;      // pixel-split waves (wgrad_halo<64, ..., PXS>)
    int slabs;    // split-K slabs written (splits, x 2 with pxs)
    long blocks;
    int g[10];
};
bool wgrad_plan(const TNParams& p, int dtype, int cus, WgradPlan* wp);
size_t wgrad_workspace(const WgradPlan& wp, const TNParams& p);
void launch_wgrad(TNParams& p, const WgradPlan& wp, hipStream_t s, int dtype = SEG_BF16);

}  // namespace seg
