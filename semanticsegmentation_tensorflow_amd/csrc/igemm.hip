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
#include "common.h"
#include "igemm.h"

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

// NT epilogue for one element; used by the GEMM and by the split-K reducer.
template <typename T>
__device__ __forceinline__ void nt_store(const NTParams& p, int row, int col, float v, int Ha,
                                         int Wa, int ooh, int oow) {
    const int hw = Ha * Wa;
    const int img = row / hw;
    const int rem = row - img * hw;
    const int a = rem / Wa;
    const int b = rem - a * Wa;
    const int oh = a * p.osh + ooh;
    const int ow = b * p.osw + oow;
    const long pix = (long)oh * p.OW + ow;
    const EpiParams& e = p.epi;
    if (col >= e.n_valid) {
        v = 0.f;
    } else {
        if (e.scale) v *= e.scale[col];
        if (e.shift) v += e.shift[col];
        if (e.bias) v += e.bias[col];
        if (e.relu) v = fmaxf(v, 0.f);
        if (e.keep_prob < 1.f) {
            const uint64_t idx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid + col;
            const float u = seg_uniform(e.seed, idx);
            v = (v / e.keep_prob) * floorf(e.keep_prob + u);
        }
        if (e.residual)
            v += to_f32(reinterpret_cast<const T*>(e.residual)[img * e.res_img + pix * e.ld_res + col]);
    }
    reinterpret_cast<T*>(p.y)[img * p.y_img + pix * p.ldy + col] = from_f32<T>(v);
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
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, af[mi]), __builtin_bit_cast(bf16x8, bfr[ni]),
                            acc[mi][ni], 0, 0, 0);
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
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int col = n0 + wn * WTN + ni * 16 + fr;
                if (col >= p.N) continue;
                const float v = acc[mi][ni][r];
                if (p.partial)
                    p.partial[((long)blockIdx.z * M + row) * p.N + col] = v;
                else
                    nt_store<T>(p, row, col, v, Ha, Wa, ooh, oow);
            }
        }
}

template <typename T>
__global__ void splitk_reduce_nt(NTParams p, int splits) {
    const long total = (long)p.M * p.N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int z = 0; z < splits; ++z) s += p.partial[(long)z * total + i];
        const int row = (int)(i / p.N), col = (int)(i - (long)(i / p.N) * p.N);
        nt_store<T>(p, row, col, s, p.Ha, p.Wa, p.ooh, p.oow);
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

__device__ __forceinline__ void tn_out(const TNParams& p, int m, int n, float v) {
    const int tap = m / p.Cg;
    const int c = m - tap * p.Cg;
    if (c < p.c_valid && n < p.n_valid) p.out[(long)tap * p.o_tap + (long)c * p.o_c + (long)n * p.o_n] = v;
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
            ra[i] = ok ? v : make_uint4(0, 0, 0, 0);
            // advance by one k tile
            pp[i] += BKP;
            pb[i] += BKP;
            while (pb[i] >= p.Wa) {
                pb[i] -= p.Wa;
                if (++pa[i] == p.Ha) { pa[i] = 0; ++pimg[i]; }
            }
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
                bf16x8 af[TM], bfr[TN];
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
                    af[mi] = __builtin_bit_cast(bf16x8, v);
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
                    bfr[ni] = __builtin_bit_cast(bf16x8, v);
                }
#pragma unroll
                for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
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
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int n = n0 + wn * WTN + ni * 16 + fr;
                if (n >= p.N) continue;
                const float v = acc[mi][ni][r];
                if (p.partial)
                    p.partial[((long)blockIdx.z * p.M + m) * p.N + n] = v;
                else
                    tn_out(p, m, n, v);
            }
        }
}

__global__ void splitk_reduce_tn(TNParams p, int splits) {
    const long total = (long)p.M * p.N;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int z = 0; z < splits; ++z) s += p.partial[(long)z * total + i];
        const int m = (int)(i / p.N), n = (int)(i - (long)(i / p.N) * p.N);
        tn_out(p, m, n, s);
    }
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

// Tile / split selection: fill >= ~2 workgroups per CU; split K only when the
// (M,N) tiling cannot, and keep >= 8 k tiles per split.
static void choose_nt(int M, int N, int K, int bk, int& bm, int& bn, int& splits) {
    bn = N <= 64 ? 64 : 128;
    bm = 128;
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
    choose_nt(M, N, K, dtype == SEG_BF16 ? 64 : 32, *bm, *bn, *splits);
    if (phase) *splits = 1;
}

void tn_info(int M, int N, int P, int dtype, int* bm, int* bn, int* splits);

size_t nt_workspace(int M, int N, int K, int dtype, int phase) {
    if (phase) return 0;
    int bm, bn, splits;
    choose_nt(M, N, K, dtype == SEG_BF16 ? 64 : 32, bm, bn, splits);
    return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

template <typename T, int BM, int BN>
static void launch_nt_t(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    hipLaunchKernelGGL((igemm_nt<T, BM, BN>), dim3(tiles, 1, gridz), dim3(256), 0, s, p);
}

template <typename T>
static int launch_nt_typed(NTParams& p, int nphases, int max_m, void* ws, size_t ws_bytes, hipStream_t s) {
    constexpr int BK = 128 / sizeof(T);
    int bm, bn, splits;
    choose_nt(max_m, p.N, p.K, BK, bm, bn, splits);
    if (nphases > 1) splits = 1;
    p.partial = nullptr;
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
    if (bn == 64) launch_nt_t<T, 128, 64>(p, gridz, max_m, s);
    else launch_nt_t<T, 128, 128>(p, gridz, max_m, s);
    SEG_CHECK_LAUNCH();
    if (p.partial) {
        const long total = (long)p.M * p.N;
        hipLaunchKernelGGL(splitk_reduce_nt<T>, dim3(seg_grid_1d(total, 256)), dim3(256), 0, s, p, splits);
        SEG_CHECK_LAUNCH();
        p.partial = nullptr;
    }
    return SEG_OK;
}

int launch_nt(NTParams& p, int dtype, int nphases, int max_m, void* ws, size_t ws_bytes, hipStream_t s) {
    if (dtype == SEG_BF16) return launch_nt_typed<bf16>(p, nphases, max_m, ws, ws_bytes, s);
    if (dtype == SEG_F32) return launch_nt_typed<float>(p, nphases, max_m, ws, ws_bytes, s);
    return SEG_EINVAL;
}

static void choose_tn(int M, int N, int P, int bkp, int& bm, int& bn, int& splits) {
    bm = M <= 64 ? 64 : 128;
    bn = N <= 64 ? 64 : 128;
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const int target = 2 * num_cus();
    const int kt = (P + bkp - 1) / bkp;
    splits = 1;
    if (tiles < target) {
        splits = (int)((target + tiles - 1) / tiles);
        splits = std::min(splits, std::max(1, kt / 8));
        splits = std::min(splits, 256);
    }
}

void tn_info(int M, int N, int P, int dtype, int* bm, int* bn, int* splits) {
    choose_tn(M, N, P, dtype == SEG_BF16 ? 64 : 32, *bm, *bn, *splits);
}

size_t tn_workspace(int M, int N, int P, int dtype) {
    int bm, bn, splits;
    choose_tn(M, N, P, dtype == SEG_BF16 ? 64 : 32, bm, bn, splits);
    return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

template <typename T, int BM, int BN>
static void launch_tn_t(TNParams& p, int gridz, hipStream_t s) {
    const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    hipLaunchKernelGGL((igemm_tn<T, BM, BN>), dim3(tiles, 1, gridz), dim3(256), 0, s, p);
}

template <typename T>
static int launch_tn_typed(TNParams& p, void* ws, size_t ws_bytes, hipStream_t s) {
    constexpr int BKP = sizeof(T) == 2 ? 64 : 32;
    int bm, bn, splits;
    choose_tn(p.M, p.N, p.P, BKP, bm, bn, splits);
    p.partial = nullptr;
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
    if (bm == 64 && bn == 64) launch_tn_t<T, 64, 64>(p, gridz, s);
    else if (bm == 64) launch_tn_t<T, 64, 128>(p, gridz, s);
    else if (bn == 64) launch_tn_t<T, 128, 64>(p, gridz, s);
    else launch_tn_t<T, 128, 128>(p, gridz, s);
    SEG_CHECK_LAUNCH();
    if (p.partial) {
        const long total = (long)p.M * p.N;
        hipLaunchKernelGGL(splitk_reduce_tn, dim3(seg_grid_1d(total, 256)), dim3(256), 0, s, p, splits);
        SEG_CHECK_LAUNCH();
        p.partial = nullptr;
    }
    return SEG_OK;
}

int launch_tn(TNParams& p, int dtype, void* ws, size_t ws_bytes, hipStream_t s) {
    if (dtype == SEG_BF16) return launch_tn_typed<bf16>(p, ws, ws_bytes, s);
    if (dtype == SEG_F32) return launch_tn_typed<float>(p, ws, ws_bytes, s);
    return SEG_EINVAL;
}

}  // namespace seg
