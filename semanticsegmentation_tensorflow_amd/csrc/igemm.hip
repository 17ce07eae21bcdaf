// Implicit-GEMM convolution kernels for gfx950 (MI355X / CDNA4).
//
//  igemm_nt : C[m][n] = sum_k A[m][k] * B[n][k]
//             A = activation gathered per output pixel m and filter tap,
//             reduction index k = (tap, channel) with channels contiguous;
//             B = packed filter rows (one per output channel), k contiguous.
//             Serves Conv2D forward, Conv2DBackpropInput (stride 1), the
//             strided conv that is conv2d_transpose's input gradient, and
//             conv2d_transpose forward through a sub-pixel phase split
//             (blockIdx.z = phase; every phase is a dense stride-1 GEMM).
//  igemm_tn : C[m][n] = sum_p A[p][m] * B[p][n]   (filter gradients)
//             reduction over pixels p; both operands are pixel-major in HBM,
//             so fragments are read column-wise out of LDS with
//             ds_read_b64_tr_b16 (bf16) -- no transpose pass in HBM.
//
// Tiles: BM x BN per 256-thread workgroup (2x2 waves), 16x16 MFMA tiles,
// K staged through double-buffered LDS with 16-byte register-staged loads.
// bf16 operands use v_mfma_f32_16x16x32_bf16, fp32 operands the exact-f32
// v_mfma_f32_16x16x4_f32 (parity path).  Accumulation is always fp32.
#include <mutex>
#include "common.h"
#include "igemm.h"
#include "halo.h"

namespace seg {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    // bijective remap so consecutive logical tiles share an XCD (and its L2)
    const int xcd = bid & 7;
    const int q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

__device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }

// NT epilogue, split into a per-row part (one pixel decomposition) and a
// per-element part; used by the v1 GEMM and by the split-K reducer.
struct NtRow {
    long yoff, roff, moff, y2off;
    uint64_t gidx;   // dropout counter base: (img*OH*OW + pix) * n_valid
};

__device__ __forceinline__ NtRow nt_row(const NTParams& p, int row, int Ha, int Wa, int ooh, int oow) {
    const int hw = Ha * Wa;
    const int img = row / hw;
    const int rem = row - img * hw;
    const int a = rem / Wa;
    const int b = rem - a * Wa;
    const long pix = (long)(a * p.osh + ooh) * p.OW + (b * p.osw + oow);
    NtRow r;
    r.yoff = img * p.y_img + pix * p.ldy;
    r.roff = img * p.epi.res_img + pix * p.epi.ld_res;
    r.moff = img * p.epi.mask_img + pix * p.epi.ld_mask;
    r.y2off = img * p.epi.y2_img + pix * p.epi.ld_y2;
    r.gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * p.epi.n_valid;
    return r;
}

// mk: the ReLU-mask value (e.mask) at (pixel, col), 1 when unused
__device__ __forceinline__ float nt_apply(const EpiParams& e, const NtRow& r, int col, float v, float res,
                                          float mk = 1.f) {
    if (col >= e.n_valid) return 0.f;
    if (e.scale) v *= e.scale[col];
    if (e.shift) v += e.shift[col];
    if (e.bias) v += e.bias[col];
    if (e.relu) v = fmaxf(v, 0.f);
    if (e.keep_prob < 1.f) v = seg_dropout(v, e.keep_prob, e.seed, r.gidx + col);
    v += res;
    if (e.mask) v = mk > 0.f ? v * e.mask_scale : 0.f;
    return v;
}

// ---------------------------------------------------------------------------
// NT kernel
// ---------------------------------------------------------------------------
template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void igemm_nt(NTParams p) {
    constexpr int EPC = dt_traits<T>::EPC;
    constexpr int BK = 128 / sizeof(T);          // k elements per 128-byte LDS row
    constexpr int NT = 256;
    constexpr int A_CH = BM * 8 / NT;
    constexpr int B_CH = BN * 8 / NT;
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int STAGE = (BM + BN) * 128;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    // ---- phase (conv2d_transpose sub-pixel split) ----
    int Ha = p.Ha, Wa = p.Wa, ioh = p.ioh, iow = p.iow, ooh = p.ooh, oow = p.oow;
    int rb = p.rb, sb = p.sb, M = p.M;
    if (p.phase) {
        const int ph = blockIdx.z / p.st_w, pw = blockIdx.z - (blockIdx.z / p.st_w) * p.st_w;
        const int oh0 = ((ph - p.pad_t) % p.st_h + p.st_h) % p.st_h;
        const int ow0 = ((pw - p.pad_l) % p.st_w + p.st_w) % p.st_w;
        Ha = (p.OH - oh0 + p.st_h - 1) / p.st_h;
        Wa = (p.OW - ow0 + p.st_w - 1) / p.st_w;
        ooh = oh0;
        oow = ow0;
        ioh = (oh0 + p.pad_t - ph) / p.st_h;
        iow = (ow0 + p.pad_l - pw) / p.st_w;
        rb = ph;
        sb = pw;
        M = p.Nimg * Ha * Wa;
        if (M <= 0) return;
    }
    const int tiles_n = (p.N + BN - 1) / BN;
    const int tiles_m = (M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int tm = wg / tiles_n, tn = wg - (wg / tiles_n) * tiles_n;
    if (tm >= tiles_m) return;
    const int m0 = tm * BM, n0 = tn * BN;

    const int KT = (p.K + BK - 1) / BK;
    int kt_begin = 0, kt_end = KT;
    if (p.partial) {
        kt_begin = blockIdx.z * p.kt_per_split;
        kt_end = min(KT, kt_begin + p.kt_per_split);
    }

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ch = tid & 7;

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);

    // ---- per-thread A row gather state ----
    long a_off[A_CH];
    int a_ih[A_CH], a_iw[A_CH];
    bool a_ok[A_CH];
    const int hw = Ha * Wa;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
        const int m = m0 + (tid >> 3) + 32 * i;
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int img = mm / hw;
        const int rem = mm - img * hw;
        const int a = rem / Wa;
        const int b = rem - a * Wa;
        a_off[i] = (long)img * p.x_img;
        a_ih[i] = a * p.ish + ioh;
        a_iw[i] = b * p.isw + iow;
    }
    long b_off[B_CH];
    bool b_ok[B_CH];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        b_ok[i] = n < p.N;
        b_off[i] = (long)(b_ok[i] ? n : 0) * p.w_col;
    }

    // ---- incremental (tap, channel) state of this thread's chunk ----
    int kg = kt_begin * BK + ch * EPC;
    int tap = kg / p.C;
    int cc = kg - tap * p.C;
    int tj = tap / p.taps_w;
    int ti = tap - tj * p.taps_w;

    uint4 ra[A_CH], rbv[B_CH];

    auto load_tile = [&]() {
        const bool kok = kg < p.K;
        const int dh = tj * p.tsh, dw = ti * p.tsw;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
            const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const T* src = X + a_off[i] + ((long)ih * p.IW + iw) * p.ldx + cc;
            uint4 v = ld16(ok ? src : X);
            if (p.pro.gamma && ok) v = apply_pro<T>(p.pro, v, cc);
            ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
        }
        const long wtap = (long)((rb + p.rstep * tj) * p.Sfull + (sb + p.sstep * ti)) * p.w_tap + cc;
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const bool ok = b_ok[i] && kok;
            const T* src = Wt + b_off[i] + wtap;
            uint4 v = ld16(ok ? src : Wt);
            rbv[i] = ok ? v : make_uint4(0, 0, 0, 0);
        }
        // advance to next k tile
        kg += BK;
        cc += BK;
        while (cc >= p.C) {
            cc -= p.C;
            if (++ti == p.taps_w) { ti = 0; ++tj; }
        }
    };
    auto store_tile = [&](int stage) {
        char* As = smem + stage * STAGE;
        char* Bs = As + BM * 128;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int row = (tid >> 3) + 32 * i;
            *reinterpret_cast<uint4*>(As + row * 128 + 16 * (ch ^ ((row >> 1) & 7))) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const int row = (tid >> 3) + 32 * i;
            *reinterpret_cast<uint4*>(Bs + row * 128 + 16 * (ch ^ ((row >> 1) & 7))) = rbv[i];
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (kt_begin < kt_end) {
        load_tile();
        store_tile(0);
    }
    __syncthreads();

    const int fr = lane & 15, fg = lane >> 4;
    for (int kt = kt_begin; kt < kt_end; ++kt) {
        const int cur = (kt - kt_begin) & 1;
        const bool more = kt + 1 < kt_end;
        if (more) load_tile();
        const char* As = smem + cur * STAGE;
        const char* Bs = As + BM * 128;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            uint4 af[TM], bfr[TN];
            const int chunk = ks * 4 + fg;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int row = wm * WTM + mi * 16 + fr;
                af[mi] = *reinterpret_cast<const uint4*>(As + row * 128 + 16 * (chunk ^ ((row >> 1) & 7)));
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int row = wn * WTN + ni * 16 + fr;
                bfr[ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * (chunk ^ ((row >> 1) & 7)));
            }
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    if constexpr (sizeof(T) == 2) {
                        acc[mi][ni] = mfma16x16x32<T>(af[mi], bfr[ni], acc[mi][ni]);
                    } else {
                        const f32x4 a4 = __builtin_bit_cast(f32x4, af[mi]);
                        const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[ni]);
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[t], b4[t], acc[mi][ni], 0, 0, 0);
                    }
                }
        }
        if (more) store_tile(cur ^ 1);
        __syncthreads();
    }

    // ---- epilogue ----
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm * WTM + mi * 16 + fg * 4 + r;
            if (row >= M) continue;
            if (p.partial) {
                float* prow = p.partial + ((long)blockIdx.z * M + row) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col = n0 + wn * WTN + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
                continue;
            }
            const NtRow rw = nt_row(p, row, Ha, Wa, ooh, oow);
            T* yrow = reinterpret_cast<T*>(p.y) + rw.yoff;
            const T* rrow = reinterpret_cast<const T*>(p.epi.residual) + rw.roff;
            const T* mrow = reinterpret_cast<const T*>(p.epi.mask) + rw.moff;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int col = n0 + wn * WTN + ni * 16 + fr;
                if (col >= p.N) continue;
                const float res = p.epi.residual ? to_f32(rrow[col]) : 0.f;
                const float mk = p.epi.mask ? to_f32(mrow[col]) : 1.f;
                yrow[col] = from_f32<T>(nt_apply(p.epi, rw, col, acc[mi][ni][r], res, mk));
            }
        }
}

// One thread per (row, 8 columns): sum the split-K slabs, apply the epilogue
// once per row decomposition, store 16 B (bf16) / 32 B (fp32).
// 32-bit index math (the host checks M * N / 8 < 2^31); the slabs of up to
// four splits are requested before their (split-ordered) additions.
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_nt(NTParams p, int splits) {
    const unsigned c8 = (unsigned)p.N / 8;
    const unsigned total = (unsigned)p.M * c8;
    const long slab = (long)p.M * p.N;
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const int row = (int)(i / c8);
        const int col0 = (int)(i - (unsigned)row * c8) * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const float* src = p.partial + (long)row * p.N + col0;
        int z = 0;
        for (; z + 3 < splits; z += 4) {
            float4 a[4], b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] = *reinterpret_cast<const float4*>(src + (z + q) * slab);
                b[q] = *reinterpret_cast<const float4*>(src + (z + q) * slab + 4);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[0] += a[q].x; v[1] += a[q].y; v[2] += a[q].z; v[3] += a[q].w;
                v[4] += b[q].x; v[5] += b[q].y; v[6] += b[q].z; v[7] += b[q].w;
            }
        }
        if (z + 1 < splits) {
            const float4 a0 = *reinterpret_cast<const float4*>(src + z * slab);
            const float4 b0 = *reinterpret_cast<const float4*>(src + z * slab + 4);
            const float4 a1 = *reinterpret_cast<const float4*>(src + (z + 1) * slab);
            const float4 b1 = *reinterpret_cast<const float4*>(src + (z + 1) * slab + 4);
            v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w;
            v[4] += b0.x; v[5] += b0.y; v[6] += b0.z; v[7] += b0.w;
            v[0] += a1.x; v[1] += a1.y; v[2] += a1.z; v[3] += a1.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
            z += 2;
        }
        if (z < splits) {
            const float4 a = *reinterpret_cast<const float4*>(src + z * slab);
            const float4 b = *reinterpret_cast<const float4*>(src + z * slab + 4);
            v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
            v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
        }
        const NtRow rw = nt_row(p, row, p.Ha, p.Wa, p.ooh, p.oow);
        float res[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        float mk[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
        if (p.epi.residual) {
            const T* rp = reinterpret_cast<const T*>(p.epi.residual) + rw.roff + col0;
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp + 4), res + 4);
        }
        if (p.epi.mask) {
            const T* mp = reinterpret_cast<const T*>(p.epi.mask) + rw.moff + col0;
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp), mk);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp + 4), mk + 4);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = nt_apply(p.epi, rw, col0 + j, v[j], res[j], mk[j]);
        T* yp = reinterpret_cast<T*>(p.y) + rw.yoff + col0;
        const uint4 packed = Chunk<T>::pack(v);
        *reinterpret_cast<uint4*>(yp) = packed;
        if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(yp + 4) = Chunk<T>::pack(v + 4);
        if constexpr (sizeof(T) == 2) {
            if (p.epi.y2) {      // BN2(+ReLU) of the stored values (seg_bn_relu_fwd's arithmetic, as igemm_nt2)
                const EpiParams& e = p.epi;
                float r[8], o2[8];
                Chunk<T>::unpack(packed, r);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int col = col0 + j;
                    const bool c2 = col < e.bn2_cv;
                    float v2 = __builtin_fmaf(r[j], c2 ? e.bn2_gamma[col] * e.bn2_inv : 0.f, c2 ? e.bn2_beta[col] : 0.f);
                    if (e.bn2_relu) v2 = fmaxf(v2, 0.f);
                    o2[j] = v2;
                }
                *reinterpret_cast<uint4*>(reinterpret_cast<T*>(e.y2) + rw.y2off + col0) = Chunk<T>::pack(o2);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// TN kernel (filter gradients)
// ---------------------------------------------------------------------------
template <int ROWB>
__device__ __forceinline__ int tn_swz(int row, int chunk) {
    // bf16 images: conflict-free for ds_write_b128 rows and ds_read_b64_tr_b16
    if constexpr (ROWB == 256) return chunk ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3));
    else return chunk ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2));
}

__device__ __forceinline__ float* tn_row(const TNParams& p, int m, bool& ok) {
    const int tap = m / p.Cg;
    const int c = m - tap * p.Cg;
    ok = c < p.c_valid;
    return p.out + (long)tap * p.o_tap + (long)c * p.o_c;
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void igemm_tn(TNParams p) {
    constexpr bool BF = sizeof(T) == 2;
    constexpr int EPC = dt_traits<T>::EPC;
    constexpr int NT = 256;
    constexpr int BKP = BF ? 64 : 32;                       // pixels per k tile
    constexpr int PAD = BF ? 0 : 16;                        // fp32 rows padded (no swizzle)
    constexpr int AROWB = BM * (int)sizeof(T) + PAD;
    constexpr int BROWB = BN * (int)sizeof(T) + PAD;
    constexpr int A_CPR = BM / EPC, A_RPP = NT / A_CPR, A_CH = BKP / A_RPP;
    constexpr int B_CPR = BN / EPC, B_RPP = NT / B_CPR, B_CH = BKP / B_RPP;
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int ASZ = BKP * AROWB, STAGE = BKP * (AROWB + BROWB);
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tiles_n = (p.N + BN - 1) / BN;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int tm = wg / tiles_n, tn = wg - (wg / tiles_n) * tiles_n;
    if (tm >= tiles_m) return;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = (p.P + BKP - 1) / BKP;
    int kt_begin = 0, kt_end = KT;
    if (p.partial) {
        kt_begin = blockIdx.z * p.kt_per_split;
        kt_end = min(KT, kt_begin + p.kt_per_split);
    }

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Bm = reinterpret_cast<const T*>(p.b);

    // ---- this thread's fixed A column chunk: m -> (tap, c) ----
    const int a_cch = tid % A_CPR;
    const int am = m0 + a_cch * EPC;
    const bool a_mok = am < p.M;
    const int atap = a_mok ? am / p.Cg : 0;
    const int ac = a_mok ? am - atap * p.Cg : 0;
    const int atj = atap / p.taps_w, ati = atap - atj * p.taps_w;
    const int hoff = atj * p.tsh + p.ioh, woff = ati * p.tsw + p.iow;
    // ---- A pixel rows: incremental (img, a, b) ----
    int pimg[A_CH], pa[A_CH], pb[A_CH], pp[A_CH];
    const int hw = p.Ha * p.Wa;
    const PixStep pstep(BKP, p.Ha, p.Wa);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
        const int pix = kt_begin * BKP + tid / A_CPR + A_RPP * i;
        pp[i] = pix;
        const int q = pix < p.P ? pix : 0;
        pimg[i] = q / hw;
        const int rem = q - pimg[i] * hw;
        pa[i] = rem / p.Wa;
        pb[i] = rem - pa[i] * p.Wa;
    }
    const int b_cch = tid % B_CPR;
    const int bn = n0 + b_cch * EPC;
    const bool b_nok = bn < p.N;
    int bpix = kt_begin * BKP + tid / B_CPR;

    uint4 ra[A_CH], rbv[B_CH];
    auto load_tile = [&]() {
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int ih = pa[i] * p.ish + hoff, iw = pb[i] * p.isw + woff;
            const bool ok = a_mok && pp[i] < p.P && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const T* src = X + (long)pimg[i] * p.x_img + ((long)ih * p.IW + iw) * p.ldx + ac;
            uint4 v = ld16(ok ? src : X);
            if (p.pro.gamma && ok) v = apply_pro<T>(p.pro, v, ac);
            ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
            // advance by one k tile
            pp[i] += BKP;
            pstep.advance(BKP, p.Ha, p.Wa, pimg[i], pa[i], pb[i]);
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const int pix = bpix + B_RPP * i;
            const bool ok = b_nok && pix < p.P;
            const T* src = Bm + (long)pix * p.ldb + bn;
            uint4 v = ld16(ok ? src : Bm);
            rbv[i] = ok ? v : make_uint4(0, 0, 0, 0);
        }
        bpix += BKP;
    };
    auto store_tile = [&](int stage) {
        char* As = smem + stage * STAGE;
        char* Bs = As + ASZ;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int row = tid / A_CPR + A_RPP * i;
            int off;
            if constexpr (BF) off = row * AROWB + 16 * tn_swz<AROWB>(row, a_cch);
            else off = row * AROWB + 16 * a_cch;
            *reinterpret_cast<uint4*>(As + off) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < B_CH; ++i) {
            const int row = tid / B_CPR + B_RPP * i;
            int off;
            if constexpr (BF) off = row * BROWB + 16 * tn_swz<BROWB>(row, b_cch);
            else off = row * BROWB + 16 * b_cch;
            *reinterpret_cast<uint4*>(Bs + off) = rbv[i];
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (kt_begin < kt_end) {
        load_tile();
        store_tile(0);
    }
    __syncthreads();

    const int fr = lane & 15, fg = lane >> 4;
    const int tq = (lane & 15) >> 2, tpp = lane & 3;
    for (int kt = kt_begin; kt < kt_end; ++kt) {
        const int cur = (kt - kt_begin) & 1;
        const bool more = kt + 1 < kt_end;
        if (more) load_tile();
        const char* As = smem + cur * STAGE;
        const char* Bs = As + ASZ;
        if constexpr (BF) {
#pragma unroll
            for (int ks = 0; ks < BKP / 32; ++ks) {
                uint4 af[TM], bfr[TN];
                const int r1 = ks * 32 + 8 * fg + tq;
#pragma unroll
                for (int mi = 0; mi < TM; ++mi) {
                    const int chk = ((wm * WTM + mi * 16) >> 3) + (tpp >> 1);
                    const SEG_LDS s16x4* p1 = (const SEG_LDS s16x4*)(As + r1 * AROWB + 16 * tn_swz<AROWB>(r1, chk) + 8 * (tpp & 1));
                    const SEG_LDS s16x4* p2 = (const SEG_LDS s16x4*)(As + (r1 + 4) * AROWB + 16 * tn_swz<AROWB>(r1 + 4, chk) + 8 * (tpp & 1));
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)p1);
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)p2);
                    typedef short s16x8 __attribute__((ext_vector_type(8)));
                    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    af[mi] = __builtin_bit_cast(uint4, v);
                }
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int chk = ((wn * WTN + ni * 16) >> 3) + (tpp >> 1);
                    const SEG_LDS s16x4* p1 = (const SEG_LDS s16x4*)(Bs + r1 * BROWB + 16 * tn_swz<BROWB>(r1, chk) + 8 * (tpp & 1));
                    const SEG_LDS s16x4* p2 = (const SEG_LDS s16x4*)(Bs + (r1 + 4) * BROWB + 16 * tn_swz<BROWB>(r1 + 4, chk) + 8 * (tpp & 1));
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)p1);
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)p2);
                    typedef short s16x8 __attribute__((ext_vector_type(8)));
                    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    bfr[ni] = __builtin_bit_cast(uint4, v);
                }
#pragma unroll
                for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[mi][ni] = mfma16x16x32<T>(af[mi], bfr[ni], acc[mi][ni]);
            }
        } else {
#pragma unroll
            for (int kq = 0; kq < BKP / 16; ++kq) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int row = kq * 16 + 4 * fg + t;
                    float af[TM], bfv[TN];
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
                        af[mi] = *reinterpret_cast<const float*>(As + row * AROWB + 4 * (wm * WTM + mi * 16 + fr));
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        bfv[ni] = *reinterpret_cast<const float*>(Bs + row * BROWB + 4 * (wn * WTN + ni * 16 + fr));
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni)
                            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi], bfv[ni], acc[mi][ni], 0, 0, 0);
                }
            }
        }
        if (more) store_tile(cur ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + mi * 16 + fg * 4 + r;
            if (m >= p.M) continue;
            if (p.partial) {
                float* prow = p.partial + ((long)blockIdx.z * p.Mp + m) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int n = n0 + wn * WTN + ni * 16 + fr;
                    if (n < p.N) prow[n] = acc[mi][ni][r];
                }
                continue;
            }
            bool ok;
            float* orow = tn_row(p, m, ok);
            if (!ok) continue;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int n = n0 + wn * WTN + ni * 16 + fr;
                if (n < p.n_valid) orow[(long)n * p.o_n] = acc[mi][ni][r];
            }
        }
}

// Split-K slab sum of the filter gradients.  A wave holds VW = 64 / SL output
// float4s x SL split-lanes: lane sl sums slabs sl, sl+SL, ... and the SL
// partial sums meet by cross-lane shuffles (no LDS allocation, so the reducer
// can share a CU with an LDS-heavy conv kernel when it runs on the side
// stream), so a 256-slab reduction of a small gradient (wgrad_halo: 576 x 16)
// runs on ~150 blocks instead of 9 latency-bound ones.
// Row M of the output range is the fused BiasAddGrad: slab rows M..Mp-1.
__global__ __launch_bounds__(256) void splitk_reduce_tn(TNParams p, int splits, int SL) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int VW = 64 / SL;
    const int v = lane % VW, sl = lane / VW;
    const int c4 = p.N / 4;
    const long total = (long)(p.Mp > p.M ? p.M + 1 : p.M) * c4;
    const long slab = (long)p.Mp * p.N;
    const long i = ((long)blockIdx.x * 4 + wave) * VW + v;
    const bool live = i < total;
    const int m = live ? (int)(i / c4) : 0;
    const int n0 = live ? (int)(i - (long)m * c4) * 4 : 0;
    float4 s = {0.f, 0.f, 0.f, 0.f};
    if (live) {
        const int r_end = m == p.M ? p.Mp : m + 1;     // bias row: all partial rows
        for (int r = m; r < r_end; ++r) {
            const float* src = p.partial + (long)r * p.N + n0;
            int z = sl;
            for (; z + 7 * SL < splits; z += 8 * SL) {  // 8 independent slab loads in flight
                float4 a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) a[u] = *reinterpret_cast<const float4*>(src + (z + u * SL) * slab);
                s.x += ((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x));
                s.y += ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y));
                s.z += ((a[0].z + a[1].z) + (a[2].z + a[3].z)) + ((a[4].z + a[5].z) + (a[6].z + a[7].z));
                s.w += ((a[0].w + a[1].w) + (a[2].w + a[3].w)) + ((a[4].w + a[5].w) + (a[6].w + a[7].w));
            }
            for (; z + 3 * SL < splits; z += 4 * SL) {  // 4 independent slab loads in flight
                const float4 a = *reinterpret_cast<const float4*>(src + z * slab);
                const float4 b = *reinterpret_cast<const float4*>(src + (z + SL) * slab);
                const float4 c = *reinterpret_cast<const float4*>(src + (z + 2 * SL) * slab);
                const float4 d = *reinterpret_cast<const float4*>(src + (z + 3 * SL) * slab);
                s.x += (a.x + b.x) + (c.x + d.x);
                s.y += (a.y + b.y) + (c.y + d.y);
                s.z += (a.z + b.z) + (c.z + d.z);
                s.w += (a.w + b.w) + (c.w + d.w);
            }
            for (; z < splits; z += SL) {
                const float4 a = *reinterpret_cast<const float4*>(src + z * slab);
                s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
            }
        }
    }
    for (int off = VW; off < 64; off <<= 1) {         // all lanes take part
        s.x += __shfl_xor(s.x, off);
        s.y += __shfl_xor(s.y, off);
        s.z += __shfl_xor(s.z, off);
        s.w += __shfl_xor(s.w, off);
    }
    if (!live || sl) return;
    const float vv[4] = {s.x, s.y, s.z, s.w};
    if (m == p.M) {               // fused BiasAddGrad row
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (n0 + j < p.n_valid) p.dbias[n0 + j] = vv[j];
        return;
    }
    bool ok;
    float* orow = tn_row(p, m, ok);
    if (!ok) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (n0 + j < p.n_valid) orow[(long)(n0 + j) * p.o_n] = vv[j];
}

static void launch_splitk_reduce_tn(TNParams& p, int splits, hipStream_t s) {
    int SL = 1;                  // ~8 slabs per lane, at most g_tn_reduce_sl lanes
    while (SL < g_tn_reduce_sl && SL * 8 < splits) SL *= 2;
    const long total = (long)(p.Mp > p.M ? p.M + 1 : p.M) * (p.N / 4);
    const long blocks = (total + 256 / SL - 1) / (256 / SL);
    hipLaunchKernelGGL(splitk_reduce_tn, dim3((unsigned)blocks), dim3(256), 0, s, p, splits, SL);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int num_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        hipGetDevice(&dev);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
        if (cus <= 0) cus = 256;
    }
    return cus;
}

int device_cus() { return num_cus(); }



// Kernel generation for the NT GEMMs (1 = register-staged 128-row tiles,
// 2 = LDS-DMA 3-stage ring, 256-row tiles).  Runtime-selectable for tests.

// Tile / split selection: fill >= ~2 workgroups per CU; split K only when the
// (M,N) tiling cannot, and keep >= 8 k tiles per split.
static void choose_nt(int M, int N, int K, int bk, int& bm, int& bn, int& splits) {
    bn = N <= 64 ? 64 : 128;
    bm = g_nt_variant == 2 ? 256 : 128;
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const int target = 2 * num_cus();
    const int kt = (K + bk - 1) / bk;
    splits = 1;
    if (tiles < target) {
        splits = (int)((target + tiles - 1) / tiles);
        splits = std::min(splits, std::max(1, kt / 8));
        splits = std::min(splits, 64);
    }
}

void nt_info(int M, int N, int K, int dtype, int phase, int* bm, int* bn, int* splits) {
    choose_nt(M, N, K, dtype == SEG_F32 ? 32 : 64, *bm, *bn, *splits);
    if (phase) *splits = 1;
}

int nt_variant() { return g_nt_variant; }

void tn_info(int M, int N, int P, int dtype, int* bm, int* bn, int* splits);

size_t nt_workspace(int M, int N, int K, int dtype, int phase) {
    if (phase) return 0;
    int bm, bn, splits;
    choose_nt(M, N, K, dtype == SEG_F32 ? 32 : 64, bm, bn, splits);
    if (g_nt_variant == 2 && nt3_applies(N, dtype)) {
        int s3;
        nt3_info(M, N, K, num_cus(), &s3);
        splits = std::max(splits, s3);
    }
    if (g_nt_variant == 2 && dtype != SEG_F32) splits = std::max(splits, std::min(g_halo_min_splits, K / 64));
    return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}


// 256x256 tiles only when the launch (tiles x splits x phases) fills at least
// half the CUs; narrow problems (phased conv2d_transpose, K <= 6 k-tiles) run
// more, smaller blocks on igemm_nt2 instead.
static bool nt3_pick(const NTParams& p, int dtype, int nphases, int max_m) {
    if (!nt3_ok(p, dtype)) return false;
    // one or two k tiles: the 2-stage igemm_nt2 (two blocks per CU) wins
    if (g_nt3_fill && g_nt2_short >= 2 && p.K <= 128) return false;
    if (!g_nt3_fill) return true;
    int s3;
    nt3_info(max_m, p.N, p.K, num_cus(), &s3);
    if (nphases > 1) s3 = 1;
    const long blocks = (long)((max_m + 255) / 256) * ((p.N + 255) / 256) * s3 * nphases;
    return blocks * 2 >= num_cus();
}

template <typename T, int BM, int BN>
static void launch_nt_t(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    hipLaunchKernelGGL((igemm_nt<T, BM, BN>), dim3(tiles, 1, gridz), dim3(256), 0, s, p);
}

// The ONE kernel decision for an NT problem: launch_nt_typed launches the
// plan, nt_choice names it, nt_pool_ok reads its pooled-epilogue flag, so the
// host-side checks and the launch can never disagree.
enum NTKind { NTK_SMALLK, NTK_PRO2, NTK_PRO_REG, NTK_RES16C, NTK_RES64, NTK_HALO, NTK_NT3, NTK_NT3_NSPLIT, NTK_NT2, NTK_REG };
struct NTPlan {
    int kind, bm, bn, splits;
    HaloPlan hp;
    int halo_kernel;     // NTK_HALO: halo_kernel(p, hp, dtype)
};

static NTPlan nt_plan(const NTParams& p, int dtype, int nphases, int max_m) {
    NTPlan pl = {};
    const bool h16 = dtype == SEG_BF16 || dtype == SEG_F16;
    const int bk = dtype == SEG_F32 ? 32 : 64;
    choose_nt(max_m, p.N, p.K, bk, pl.bm, pl.bn, pl.splits);
    if (nphases > 1) pl.splits = 1;
    if (h16 && nphases == 1 && smallk_ok(p, dtype)) {
        pl.kind = NTK_SMALLK;
        pl.bm = 1; pl.bn = 8; pl.splits = 1;
        return pl;
    }
    if (p.pro.gamma) {
        if (g_nt_variant == 2 && nt2_pro_ok(p, dtype, nphases)) {   // 1x1: K <= 1024, no split-K
            pl.kind = NTK_PRO2;
            pl.splits = 1;
            return pl;
        }
        pl.kind = NTK_PRO_REG;                 // operand prologue: the register-staged kernel
        pl.bm = 128;
        const long tiles = (long)((max_m + 127) / 128) * ((p.N + pl.bn - 1) / pl.bn);
        pl.splits = 1;
        if (tiles < 2 * num_cus()) {
            const int kt = (p.K + bk - 1) / bk;
            pl.splits = std::min<int>(std::max(1, kt / 8), (int)((2 * num_cus() + tiles - 1) / tiles));
        }
        return pl;
    }
    if (h16 && nphases == 1 && g_nt_variant == 2 && res16c_ok(p, dtype)) {
        pl.kind = NTK_RES16C;
        pl.bm = 256; pl.bn = 64; pl.splits = 1;
        return pl;
    }
    if (h16 && nphases == 1 && g_nt_variant == 2 && res64_ok(p, dtype)) {
        pl.kind = NTK_RES64;
        pl.bn = (p.N <= 16 && g_res16) ? 16 : 64;
        pl.splits = 1;
        return pl;
    }
    if (h16 && nphases == 1 && g_nt_variant == 2 && halo_plan(p, dtype, pl.splits, num_cus(), &pl.hp)) {
        pl.kind = NTK_HALO;
        pl.bm = 256; pl.bn = pl.hp.bn; pl.splits = pl.hp.splits;
        pl.halo_kernel = halo_kernel(p, pl.hp, dtype);
        return pl;
    }
    if (h16 && g_nt_variant == 2 && nt3_pick(p, dtype, nphases, max_m)) {
        nt3_info(max_m, p.N, p.K, num_cus(), &pl.splits);
        if (nphases > 1) pl.splits = 1;
        pl.bm = pl.bn = 256;
        // N = 256 k + a tail of <= 128 columns (FC-DenseNet's 320 / 560 / 352 /
        // 280-wide transposed-conv GEMMs): the 256-aligned head on igemm_nt3, the
        // tail on igemm_nt2 (256 x 64 / 128 tiles) instead of a 256-wide tile that
        // is 50-80 % padding.  Not with dropout (its counter uses the full row
        // width) or the BN-backward epilogue (per-tile column sums).
        pl.kind = (pl.splits == 1 && g_nt_nsplit && p.N > 256 && p.N % 256 != 0 && p.N % 256 <= 128 &&
                   p.epi.keep_prob >= 1.f && !p.epi.bn_x) ? NTK_NT3_NSPLIT : NTK_NT3;
        return pl;
    }
    pl.kind = pl.bm == 256 ? NTK_NT2 : NTK_REG;
    return pl;
}

// Whether the planned kernel has the fused MaxPool epilogue (EpiParams
// pool_y): conv_res64 with 64-wide output blocks, conv_halo_duo with 16-px
// tile rows and 128-wide blocks, conv_halo2 -- each without split-K.
static bool nt_plan_pools(const NTPlan& pl) {
    if (pl.kind == NTK_RES64) return pl.bn == 64;
    if (pl.kind == NTK_HALO) return halo_pools(pl.hp, pl.halo_kernel);
    return false;
}

// Whether the planned kernel has the fused MaxPoolGrad epilogue (EpiParams
// unpool_y): halo_unpools (no split-K slabs), unit output stride.
static bool nt_plan_unpools(const NTPlan& pl, const NTParams& p) {
    return pl.kind == NTK_HALO && halo_unpools(pl.hp, pl.halo_kernel) && p.osh == 1 && p.osw == 1 && p.ooh == 0 &&
           p.oow == 0 && !p.phase;
}

// Whether the plan for p runs igemm_nt3 whole (the kernel with the B-transposed
// form) and the reduction channels tile by 64 (a k tile never crosses a tap).
bool nt_fwd_bt_ok(const NTParams& p, int dtype) {
    if ((dtype != SEG_BF16 && dtype != SEG_F16) || p.pro.gamma || p.phase || p.C % 64 || p.kv) return false;
    return nt_plan(p, dtype, 1, p.M).kind == NTK_NT3;
}

bool nt_unpool_ok(const NTParams& p, int dtype) {
    if ((dtype != SEG_BF16 && dtype != SEG_F16) || p.pro.gamma || p.phase) return false;
    return nt_plan_unpools(nt_plan(p, dtype, 1, p.M), p);
}

// Whether the planned launch writes EpiParams.y2 (the BN(+ReLU) second
// output): igemm_nt2 with its operand prologue or without, no split-K; and
// igemm_nt3 -- unsplit in its own epilogue (round 6: DeepLab's ASPP convs ->
// BN -> ReLU at 1024 x 2048, C5), split through splitk_reduce_nt (the same
// convs on the 1/8-resolution map of a 384 x 1248 input).
static bool nt_plan_bn2(const NTPlan& pl, int dtype) {
    if (dtype == SEG_F32) return false;
    return (pl.splits == 1 && (pl.kind == NTK_PRO2 || pl.kind == NTK_NT2)) || pl.kind == NTK_NT3;
}

bool nt_bn2_ok(const NTParams& p, int dtype) { return nt_plan_bn2(nt_plan(p, dtype, 1, p.M), dtype); }

// Whether the planned launch reads the ReluGrad mask as bits
// (EpiParams::mask_bits): the 64-wide conv_res64 plan, which launch_res64 runs
// on conv_res64pp.
static bool nt_plan_mask_bits(const NTPlan& pl) { return pl.kind == NTK_RES64 && pl.bn == 64; }

bool nt_mask_bits_ok(const NTParams& p, int dtype) {
    if ((dtype != SEG_BF16 && dtype != SEG_F16) || p.pro.gamma || p.phase || !p.epi.mask_bits) return false;
    return nt_plan_mask_bits(nt_plan(p, dtype, 1, p.M));
}

template <typename T>
static int launch_nt_typed(NTParams& p, int nphases, int max_m, void* ws, size_t ws_bytes, hipStream_t s) {
    constexpr int BK = 128 / sizeof(T);
    const NTPlan pl = nt_plan(p, dt_traits<T>::id, nphases, max_m);
    // a pooled launch writes no unpooled map (p.y is null): only a kernel with
    // the pooled epilogue and no split-K slabs may run it
    if (p.epi.pool_y && !nt_plan_pools(pl)) return SEG_EINVAL;
    // likewise the MaxPoolGrad epilogue (p.y unused) and a second BN output:
    // only the kernels that write them
    if (p.epi.unpool_y && (nphases != 1 || !nt_plan_unpools(pl, p))) return SEG_EINVAL;
    if (p.bt && (nphases != 1 || pl.kind != NTK_NT3 || p.C % 64 || p.kv)) return SEG_EINVAL;
    if (p.epi.y2 && (nphases != 1 || !nt_plan_bn2(pl, dt_traits<T>::id))) return SEG_EINVAL;
    // the mask bits are read by conv_res64pp alone and written by conv_c8_fwd
    // alone (seg_conv2d_fwd_relu_bits, which does not come here)
    if (p.epi.ybits || (p.epi.mask_bits && (nphases != 1 || !nt_plan_mask_bits(pl)))) return SEG_EINVAL;
    int splits = pl.splits;
    p.partial = nullptr;
    switch (pl.kind) {
        case NTK_SMALLK:
            launch_smallk(p, dt_traits<T>::id, num_cus(), s);
            SEG_CHECK_LAUNCH();
            return SEG_OK;
        case NTK_PRO2:
            launch_nt2_pro(p, dt_traits<T>::id, 1, max_m, s);
            SEG_CHECK_LAUNCH();
            return SEG_OK;
        case NTK_PRO_REG: {
            int gridz = nphases;
            if (splits > 1) {
                const int kt = (p.K + BK - 1) / BK;
                p.kt_per_split = (kt + splits - 1) / splits;
                splits = (kt + p.kt_per_split - 1) / p.kt_per_split;
                if (!ws || ws_bytes < (size_t)splits * p.M * p.N * sizeof(float)) return SEG_EWORKSPACE;
                p.partial = reinterpret_cast<float*>(ws);
                gridz = splits;
            }
            if (pl.bn == 64) launch_nt_t<T, 128, 64>(p, gridz, max_m, s);
            else launch_nt_t<T, 128, 128>(p, gridz, max_m, s);
            SEG_CHECK_LAUNCH();
            if (p.partial) {
                const long total = (long)p.M * (p.N / 8);
                if (total >= (1L << 31)) return SEG_EINVAL;
                hipLaunchKernelGGL(splitk_reduce_nt<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0, s, p, splits);
                SEG_CHECK_LAUNCH();
                p.partial = nullptr;
            }
            return SEG_OK;
        }
        case NTK_RES16C:
            launch_res16c(p, num_cus(), s, dt_traits<T>::id);
            SEG_CHECK_LAUNCH();
            return SEG_OK;
        case NTK_RES64: {
            const int st = launch_res64(p, num_cus(), s, dt_traits<T>::id);
            if (st) return st;
            SEG_CHECK_LAUNCH();
            return SEG_OK;
        }
        case NTK_HALO: {
            if (pl.hp.splits > 1) {
                const size_t need = (size_t)pl.hp.splits * p.M * p.N * sizeof(float);
                if (!ws || ws_bytes < need) return SEG_EWORKSPACE;
                p.partial = reinterpret_cast<float*>(ws);
            }
            const int st = launch_halo(p, pl.hp, pl.halo_kernel, s, dt_traits<T>::id);
            if (st) {
                p.partial = nullptr;
                return st;
            }
            SEG_CHECK_LAUNCH();
            if (p.partial) {
                const long total = (long)p.M * (p.N / 8);
                if (total >= (1L << 31)) return SEG_EINVAL;
                hipLaunchKernelGGL(splitk_reduce_nt<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0, s, p, pl.hp.splits);
                SEG_CHECK_LAUNCH();
                p.partial = nullptr;
            }
            return SEG_OK;
        }
        case NTK_NT3_NSPLIT: {
            const int nh = p.N / 256 * 256;
            NTParams t = p;
            p.N = nh;
            launch_nt3(p, nphases, max_m, s, dt_traits<T>::id);
            SEG_CHECK_LAUNCH();
            p.N = t.N;
            t.N -= nh;
            t.w = reinterpret_cast<const T*>(t.w) + (long)nh * t.w_col;
            t.y = reinterpret_cast<T*>(t.y) + nh;
            if (t.epi.bias) t.epi.bias += nh;
            if (t.epi.scale) t.epi.scale += nh;
            if (t.epi.shift) t.epi.shift += nh;
            if (t.epi.residual) t.epi.residual = reinterpret_cast<const T*>(t.epi.residual) + nh;
            if (t.epi.mask) t.epi.mask = reinterpret_cast<const T*>(t.epi.mask) + nh;
            t.epi.n_valid = std::max(0, t.epi.n_valid - nh);
            launch_nt2(t, dt_traits<T>::id, t.N <= 64 ? 64 : 128, nphases, max_m, s);
            SEG_CHECK_LAUNCH();
            return SEG_OK;
        }
        default:
            break;
    }
    int gridz = nphases;
    if (splits > 1) {
        const int kt = (p.K + BK - 1) / BK;
        p.kt_per_split = (kt + splits - 1) / splits;
        splits = (kt + p.kt_per_split - 1) / p.kt_per_split;
        const size_t need = (size_t)splits * p.M * p.N * sizeof(float);
        if (!ws || ws_bytes < need) return SEG_EWORKSPACE;
        p.partial = reinterpret_cast<float*>(ws);
        gridz = splits;
    }
    if (pl.kind == NTK_NT3) launch_nt3(p, gridz, max_m, s, dt_traits<T>::id);
    else if (pl.kind == NTK_NT2) launch_nt2(p, dt_traits<T>::id, pl.bn, gridz, max_m, s);
    else if (pl.bn == 64) launch_nt_t<T, 128, 64>(p, gridz, max_m, s);
    else launch_nt_t<T, 128, 128>(p, gridz, max_m, s);
    SEG_CHECK_LAUNCH();
    if (p.partial) {
        const long total = (long)p.M * (p.N / 8);
        if (total >= (1L << 31)) return SEG_EINVAL;
        hipLaunchKernelGGL(splitk_reduce_nt<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0, s, p, splits);
        SEG_CHECK_LAUNCH();
    }
    p.partial = nullptr;
    return SEG_OK;
}

bool nt_pool_ok(const NTParams& p, int dtype) {
    if ((dtype != SEG_BF16 && dtype != SEG_F16) || p.pro.gamma || p.phase) return false;
    return nt_plan_pools(nt_plan(p, dtype, 1, p.M));
}

// The kernel family launch_nt runs for p (named from the same plan).
const char* nt_choice(const NTParams& p, int dtype, int nphases, int max_m, int* bm, int* bn, int* splits) {
    const NTPlan pl = nt_plan(p, dtype, nphases, max_m);
    *bm = pl.bm; *bn = pl.bn; *splits = pl.splits;
    switch (pl.kind) {
        case NTK_SMALLK: return "smallk_nt";
        case NTK_PRO2: return "igemm_nt2_pro";
        case NTK_PRO_REG: return "igemm_nt_pro";
        case NTK_RES16C: return "conv_res16c";
        case NTK_RES64: return "conv_res64";
        case NTK_HALO: return pl.halo_kernel == HALO_K4 ? "conv_halo4" : "conv_halo";
        case NTK_NT3:
        case NTK_NT3_NSPLIT: return "igemm_nt3";
        case NTK_NT2: return "igemm_nt2";
        default: return "igemm_nt";
    }
}

int launch_nt(NTParams& p, int dtype, int nphases, int max_m, void* ws, size_t ws_bytes, hipStream_t s) {
    if (dtype == SEG_BF16) return launch_nt_typed<bf16>(p, nphases, max_m, ws, ws_bytes, s);
    if (dtype == SEG_F32) return launch_nt_typed<float>(p, nphases, max_m, ws, ws_bytes, s);
    if (dtype == SEG_F16) return launch_nt_typed<f16>(p, nphases, max_m, ws, ws_bytes, s);
    return SEG_EINVAL;
}


// v2: 0 = igemm_tn tiles, 1 = igemm_tn2 tiles when M >= 128, 2 = igemm_tn2 tiles
static void choose_tn(int M, int N, int P, int bkp, int v2, int& bm, int& bn, int& splits) {
    if (g_tn_variant == 2 && (v2 == 2 || (v2 && (M >= 128 || g_tn2_smallm)))) {
        // v2 tiles: minimise padded work / relative tile efficiency
        static const int cand[5][2] = {{128, 256}, {256, 128}, {128, 128}, {256, 64}, {128, 64}};
        static const double eff[5] = {1.0, 1.0, 0.85, 0.85, 0.8};
        double best = 1e30;
        for (int i = 0; i < 5; ++i) {
            const double cost = (double)((M + cand[i][0] - 1) / cand[i][0] * cand[i][0]) *
                                ((N + cand[i][1] - 1) / cand[i][1] * cand[i][1]) / eff[i];
            if (cost < best * 0.999) { best = cost; bm = cand[i][0]; bn = cand[i][1]; }
        }
    } else {
        bm = M <= 64 ? 64 : 128;
        bn = N <= 64 ? 64 : 128;
    }
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const int target = g_tn_fill * num_cus();
    const int kt = (P + bkp - 1) / bkp;
    splits = 1;
    if (tiles < target) {
        splits = (int)((target + tiles - 1) / tiles);
        splits = std::min(splits, std::max(1, kt / 8));
        splits = std::min(splits, g_tn_split_cap);
    }
}

void tn_info(int M, int N, int P, int dtype, int* bm, int* bn, int* splits) {
    choose_tn(M, N, P, dtype == SEG_F32 ? 32 : 64, dtype != SEG_F32, *bm, *bn, *splits);
}

size_t tn_workspace(int M, int N, int P, int dtype) {
    int bm, bn, splits;
    choose_tn(M, N, P, dtype == SEG_F32 ? 32 : 64, dtype != SEG_F32, bm, bn, splits);
    if (dtype != SEG_F32) {        // prologue (folded BatchNorm) launches: tn2 tiles at any M
        int b2m, b2n, s2;
        choose_tn(M, N, P, 64, 2, b2m, b2n, s2);
        splits = std::max(splits, s2);
    }
    if (g_tn_variant == 2 && tn3_applies(M, N, dtype)) {
        int s3;
        tn3_info(M, N, P, num_cus(), &s3);
        splits = std::max(splits, s3);
    }
    return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

template <typename T, int BM, int BN>
static void launch_tn_t(TNParams& p, int gridz, hipStream_t s) {
    const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    hipLaunchKernelGGL((igemm_tn<T, BM, BN>), dim3(tiles, 1, gridz), dim3(256), 0, s, p);
}

// Split-K tail: reduce the slabs now, or leave them pending (p.defer).
static void tn_finish(TNParams& p, int splits, hipStream_t s) {
    if (p.defer) {
        p.defer[0] = p.partial ? splits : 1;
        p.defer[1] = p.Mp;
        p.partial = nullptr;
        return;
    }
    if (!p.partial) return;
    launch_splitk_reduce_tn(p, splits, s);
    p.partial = nullptr;
}

void tn_reduce(TNParams& p, int splits, hipStream_t s) { launch_splitk_reduce_tn(p, splits, s); }

template <typename T>
static int launch_tn_typed(TNParams& p, void* ws, size_t ws_bytes, hipStream_t s) {
    constexpr int BKP = sizeof(T) == 2 ? 64 : 32;
    p.partial = nullptr;
    p.Mp = p.M;
    if (p.pro.gamma) {       // operand prologue: tn2 for single-tap 16-bit problems, else igemm_tn
        const bool v2 = sizeof(T) == 2 && g_tn_variant == 2 && p.M == p.Cg;
        int bm, bn, splits;
        choose_tn(p.M, p.N, p.P, BKP, v2 ? 2 : 0, bm, bn, splits);
        int gridz = 1;
        if (splits > 1) {
            const int kt = (p.P + BKP - 1) / BKP;
            p.kt_per_split = (kt + splits - 1) / splits;
            splits = (kt + p.kt_per_split - 1) / p.kt_per_split;
            if (!ws || ws_bytes < (size_t)splits * p.M * p.N * sizeof(float)) return SEG_EWORKSPACE;
            p.partial = reinterpret_cast<float*>(ws);
            gridz = splits;
        }
        if (v2) launch_tn2_pro(p, bm, bn, gridz, s, dt_traits<T>::id);
        else if (bm == 64 && bn == 64) launch_tn_t<T, 64, 64>(p, gridz, s);
        else if (bm == 64) launch_tn_t<T, 64, 128>(p, gridz, s);
        else if (bn == 64) launch_tn_t<T, 128, 64>(p, gridz, s);
        else launch_tn_t<T, 128, 128>(p, gridz, s);
        SEG_CHECK_LAUNCH();
        tn_finish(p, splits, s);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    if (smallc_wgrad_ok(p, dt_traits<T>::id)) {
        const int splits = smallc_wgrad_splits(p, num_cus());
        if (p.dbias) p.Mp = p.M + 1;
        if (splits > 1) {
            if (!ws || ws_bytes < (size_t)splits * p.Mp * p.N * sizeof(float)) return SEG_EWORKSPACE;
            p.partial = reinterpret_cast<float*>(ws);
        }
        launch_smallc_wgrad(p, dt_traits<T>::id, splits, s);
        SEG_CHECK_LAUNCH();
        tn_finish(p, splits, s);
        SEG_CHECK_LAUNCH();
        p.dbias = nullptr;
        return SEG_OK;
    }
    WgradPlan wp;
    if (sizeof(T) == 2 && g_tn_variant == 2 && wgrad_plan(p, dt_traits<T>::id, num_cus(), &wp)) {
        if (p.dbias) p.Mp = p.M + wp.nbias;   // wgrad_halo sums dy columns too (nbias partial rows)
        if (wp.slabs > 1) {
            if (!ws || ws_bytes < wgrad_workspace(wp, p)) return SEG_EWORKSPACE;
            p.partial = reinterpret_cast<float*>(ws);
        }
        launch_wgrad(p, wp, s, dt_traits<T>::id);
        SEG_CHECK_LAUNCH();
        tn_finish(p, wp.slabs, s);
        SEG_CHECK_LAUNCH();
        p.dbias = nullptr;                    // done
        return SEG_OK;
    }
    int bm, bn, splits;
    choose_tn(p.M, p.N, p.P, BKP, sizeof(T) == 2, bm, bn, splits);
    const bool tn3 = sizeof(T) == 2 && g_tn_variant == 2 && tn3_ok(p, dt_traits<T>::id);
    if (tn3) tn3_info(p.M, p.N, p.P, num_cus(), &splits);
    // N = 256 k + a tail <= 128 (FC-DenseNet's transposed-conv filter
    // gradients, N = 320 / 560 input channels): the 256-aligned head on
    // igemm_tn3, the tail on igemm_tn2, each with its own split-K slabs in `ws`
    // (reduced in stream order, so the tail reuses the head's slab space)
    if (tn3 && g_tn_nsplit && !p.defer && !p.adam.p && p.N > 256 && p.N % 256 != 0 && p.N % 256 <= 128) {
        const int nh = p.N / 256 * 256;
        const int kt = (p.P + BKP - 1) / BKP;
        auto plan = [&](TNParams& q, int sp) {
            const long cap = ws ? (long)(ws_bytes / ((size_t)q.M * q.N * sizeof(float))) : 1;
            sp = (int)std::max(1L, std::min<long>(sp, cap));
            q.partial = nullptr;
            if (sp > 1) {
                q.kt_per_split = (kt + sp - 1) / sp;
                sp = (kt + q.kt_per_split - 1) / q.kt_per_split;
                q.partial = reinterpret_cast<float*>(ws);
            }
            return sp;
        };
        TNParams h = p;
        h.N = nh;
        h.n_valid = std::min(p.n_valid, nh);
        h.dbias = nullptr;
        int sh;
        tn3_info(h.M, h.N, h.P, num_cus(), &sh);
        sh = plan(h, sh);
        launch_tn3(h, sh, s, dt_traits<T>::id);
        SEG_CHECK_LAUNCH();
        tn_finish(h, sh, s);
        SEG_CHECK_LAUNCH();
        TNParams t = p;
        t.N = p.N - nh;
        t.n_valid = std::max(0, p.n_valid - nh);
        t.b = reinterpret_cast<const T*>(p.b) + nh;
        t.out = p.out + (long)nh * p.o_n;
        t.dbias = nullptr;
        int tbm, tbn, st;
        choose_tn(t.M, t.N, t.P, BKP, 1, tbm, tbn, st);
        st = plan(t, st);
        launch_tn2(t, tbm, tbn, st, s, dt_traits<T>::id);
        SEG_CHECK_LAUNCH();
        tn_finish(t, st, s);
        SEG_CHECK_LAUNCH();
        return SEG_OK;
    }
    int gridz = 1;
    if (splits > 1) {
        const int kt = (p.P + BKP - 1) / BKP;
        p.kt_per_split = (kt + splits - 1) / splits;
        splits = (kt + p.kt_per_split - 1) / p.kt_per_split;
        const size_t need = (size_t)splits * p.M * p.N * sizeof(float);
        if (!ws || ws_bytes < need) return SEG_EWORKSPACE;
        p.partial = reinterpret_cast<float*>(ws);
        gridz = splits;
    }
    if (tn3) {
        launch_tn3(p, gridz, s, dt_traits<T>::id);
    } else if (g_tn_variant == 2 && sizeof(T) == 2 && (bm == 256 || bn == 256 || p.M >= 128 || g_tn2_smallm)) {
        launch_tn2(p, bm, bn, gridz, s, dt_traits<T>::id);
    } else if (bm == 64 && bn == 64) launch_tn_t<T, 64, 64>(p, gridz, s);
    else if (bm == 64) launch_tn_t<T, 64, 128>(p, gridz, s);
    else if (bn == 64) launch_tn_t<T, 128, 64>(p, gridz, s);
    else launch_tn_t<T, 128, 128>(p, gridz, s);
    SEG_CHECK_LAUNCH();
    tn_finish(p, splits, s);
    SEG_CHECK_LAUNCH();
    return SEG_OK;
}

int launch_tn(TNParams& p, int dtype, void* ws, size_t ws_bytes, hipStream_t s) {
    if (dtype == SEG_BF16) return launch_tn_typed<bf16>(p, ws, ws_bytes, s);
    if (dtype == SEG_F32) return launch_tn_typed<float>(p, ws, ws_bytes, s);
    if (dtype == SEG_F16) return launch_tn_typed<f16>(p, ws, ws_bytes, s);
    return SEG_EINVAL;
}

}  // namespace seg
