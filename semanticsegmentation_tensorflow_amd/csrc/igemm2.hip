// Second-generation implicit-GEMM NT kernel for gfx950.
//
// Same contract as igemm_nt (igemm.hip) but staged the CDNA4 way:
//  * operands go HBM/L2 -> LDS by LDS-DMA (`global_load_lds_dwordx4`, one
//    1 KiB wave-instruction = 8 rows x 128 B), issued from inline asm so
//    hipcc does not drain the DMA queue before every ds_read;
//  * the implicit-GEMM gather lives in the per-lane SOURCE address; zero
//    padding / tails point the lane at a zero page; the LDS XOR swizzle is
//    applied on the source side (LDS image stays lane-linear);
//  * a 3-deep LDS ring: tile t+2 is in flight while tile t is consumed; one
//    counted `s_waitcnt vmcnt(N)` + raw `s_barrier` per K tile;
//  * 8 waves (4 x 2), 64x64 (or 64x32) per wave on v_mfma_f32_16x16x32_bf16.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

__device__ uint4 g_zero_page[4];

template <typename T>
[[maybe_unused]] __device__ __forceinline__ void nt2_store(const NTParams& p, int row, int col, float v, int Ha, int Wa, int ooh,
                                          int oow) {
    const int hw = Ha * Wa;
    const int img = row / hw;
    const int rem = row - img * hw;
    const int a = rem / Wa;
    const int b = rem - a * Wa;
    const long pix = (long)(a * p.osh + ooh) * p.OW + (b * p.osw + oow);
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
            v = seg_dropout(v, e.keep_prob, e.seed, idx);
        }
        if (e.residual)
            v += to_f32(reinterpret_cast<const T*>(e.residual)[img * e.res_img + pix * e.ld_res + col]);
    }
    reinterpret_cast<T*>(p.y)[img * p.y_img + pix * p.ldy + col] = from_f32<T>(v);
}

// ABL (diagnostic builds only, results are garbage): 1 = no LDS-DMA in the
// main loop, 2 = no MFMA, 3 = trivial (row-constant) source addresses.
// NSTG = ring depth.  3 for long K; 2 for short-K problems (1x1 convs over
// <= 128 channels: one or two k tiles per block), where the smaller LDS
// footprint lets two blocks share a CU so one block's loads overlap the
// other's epilogue -- with one block per CU those blocks are pure latency.
// PRO: the A operand goes through p.pro (BatchNorm + ReLU) between the LDS
// read and the MFMA; the per-channel (scale, shift) table is staged in LDS
// once per block (single-tap problems, K <= NT2_PRO_MAXK).
// BNB: the epilogue continues through the folded BatchNorm(+ReLU) backward
// (EpiParams.bn_*): its own instantiation, so the plain kernels keep their
// register budget (two blocks per CU for the short-K form).
template <typename T, int BM, int BN, int WM, int WN, int ABL = 0, int NSTG = 3, bool PRO = false, bool BNB = false>
__global__ __launch_bounds__(WM* WN * 64, NSTG == 2 ? 2 : 1) void igemm_nt2(NTParams p) {
    constexpr int NW = WM * WN;
    constexpr int EPC = dt_traits<T>::EPC;
    constexpr int BK = 128 / sizeof(T);
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int A_INS = BM / 8 / NW, B_INS = BN / 8 / NW;
    static_assert(A_INS * 8 * NW == BM && B_INS * 8 * NW == BN, "tile rows must split into 8-row pieces per wave");
    static_assert(NW % 2 == 0, "swizzle assumes an even wave count");
    constexpr int NI = A_INS + B_INS;
    constexpr int STAGE = (BM + BN) * 128;
    constexpr int SROW = WTN * 4 + 16;               // epilogue: padded fp32 row (bytes)
    constexpr int SMEM = NSTG * STAGE > NW * WTM * SROW ? NSTG * STAGE : NW * WTM * SROW;
    static_assert(NSTG == 2 || NSTG == 3, "ring depth");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

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
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    // Few M tiles x many N tiles (conv6/7: B = 100+ MB of filter): walk M fastest
    // so all M tiles of one B panel run back to back on one XCD and share its
    // L2; otherwise N fastest (A panel shared).
    const int tiles_mg = gridDim.x / tiles_n;        // grid M tiles (max over phases)
    int tm, tn;
    if (tiles_mg <= 16 && tiles_n > tiles_mg) {
        tn = wg / tiles_mg;
        tm = wg - tn * tiles_mg;
    } else {
        tm = wg / tiles_n;
        tn = wg - tm * tiles_n;
    }
    if (tm >= tiles_m) return;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = (p.K + BK - 1) / BK;
    int kt_begin = 0, kt_end = KT;
    if (p.partial) {
        kt_begin = blockIdx.z * p.kt_per_split;
        kt_end = min(KT, kt_begin + p.kt_per_split);
    }

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const int lr = lane >> 3;
    // global k-chunk this lane stages: physical chunk (lane & 7) of its row,
    // pre-swizzled; the swizzle of row (i*NW + w)*8 + lr is i-independent.
    const int c = (lane & 7) ^ ((((w & 1) << 2) + (lr >> 1)) & 7);

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)g_zero_page;

    long a_off[A_INS];
    int a_ih[A_INS], a_iw[A_INS];
    bool a_ok[A_INS];
    const int hw = Ha * Wa;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
        const int m = m0 + (i * NW + w) * 8 + lr;
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
    long b_off[B_INS];
    bool b_ok[B_INS];
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
        const int n = n0 + (i * NW + w) * 8 + lr;
        b_ok[i] = n < p.N;
        b_off[i] = (long)(b_ok[i] ? n : 0) * p.w_col;
    }
    int kg = kt_begin * BK + c * EPC;
    int tap = kg / p.C;
    int cc = kg - tap * p.C;
    int tj = tap / p.taps_w;
    int ti = tap - tj * p.taps_w;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;

    const float* ptab = nullptr;
    if constexpr (PRO) {
        // before the first DMA: the table loads' wait drains nothing else
        __shared__ __attribute__((aligned(16))) float ptab_s[2 * NT2_PRO_MAXK];
        for (int k = tid; k < KT * BK; k += NW * 64) {
            const bool v = k < p.pro.cv;
            ptab_s[2 * k] = v ? p.pro.gamma[k] * p.pro.inv : 0.f;
            ptab_s[2 * k + 1] = v ? p.pro.beta[k] : 0.f;
        }
        ptab = ptab_s;      // visible after the first iteration's barrier
    }

    auto load_stage = [&](int stage) {
        const unsigned sb_ = lds0 + stage * STAGE;
        const bool kok = kg < p.K;
        const int dh = tj * p.tsh, dw = ti * p.tsw;
#pragma unroll
        for (int i = 0; i < A_INS; ++i) {
            const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
            const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const void* src;
            if constexpr (ABL == 3) src = (const void*)(X + a_off[i] + (long)(a_ih[i] & 7) * p.ldx + cc);
            else src = ok ? (const void*)(X + a_off[i] + ((long)ih * p.IW + iw) * p.ldx + cc) : zero;
            if constexpr (ABL != 1) glds16(src, sb_ + (i * NW + w) * 1024);
        }
        const long wtap = (long)((rb + p.rstep * tj) * p.Sfull + (sb + p.sstep * ti)) * p.w_tap + cc;
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const bool ok = b_ok[i] && kok;
            const void* src = ok ? (const void*)(Wt + b_off[i] + wtap) : zero;
            if constexpr (ABL != 1) glds16(src, sb_ + BM * 128 + (i * NW + w) * 1024);
        }
        kg += BK;
        cc += BK;
        while (cc >= p.C) {
            cc -= p.C;
            if (++ti == p.taps_w) { ti = 0; ++tj; }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // BNB: the epilogue's BN input and accumulation operands (x, old dx) for
    // this lane's rows are requested before the first DMA, so their HBM
    // latency overlaps the operand staging and MFMAs instead of following it
    constexpr int ECPR = WTN / 8, ERPP = 64 / ECPR, ENPR = WTM / ERPP;   // epilogue: rows per lane
    uint4 pfx[BNB ? ENPR : 1], pfr[BNB ? ENPR : 1];
    if constexpr (BNB) {
        static_assert(sizeof(T) == 2, "BNB epilogue: 16-bit operands");
        const int ecol0 = n0 + wn * WTN + (lane % ECPR) * 8;
        const int ersub = lane / ECPR;
#pragma unroll
        for (int k = 0; k < ENPR; ++k) {
            const int row = m0 + wm * WTM + ersub + k * ERPP;
            pfx[k] = pfr[k] = uint4{0u, 0u, 0u, 0u};
            if (row >= M || ecol0 >= p.N) continue;
            const int hw = Ha * Wa;
            const int img = row / hw;
            const int rem = row - img * hw;
            const int a = rem / Wa;
            const int b = rem - a * Wa;
            const long pix = (long)(a * p.osh + ooh) * p.OW + (b * p.osw + oow);
            pfx[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p.epi.bn_x) + img * p.epi.bn_x_img +
                                                     pix * p.epi.ld_bn_x + ecol0);
            if (p.epi.residual)
                pfr[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p.epi.residual) +
                                                         img * p.epi.res_img + pix * p.epi.ld_res + ecol0);
        }
    }

    if (kt_begin < kt_end) load_stage(0);
    if (NSTG == 3 && kt_begin + 1 < kt_end) load_stage(1);

    const int fr = lane & 15, fg = lane >> 4;
    int stage = 0;
    for (int kt = kt_begin; kt < kt_end; ++kt) {
        if (NSTG == 3 && kt + 1 < kt_end) wait_vmcnt<NI>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (kt + NSTG - 1 < kt_end) load_stage(NSTG == 3 ? (stage == 0 ? 2 : stage - 1) : stage ^ 1);
        const char* As = smem + stage * STAGE;
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
            if constexpr (PRO) {
                float ss[16];
                const float4* tp = reinterpret_cast<const float4*>(ptab + 2 * (kt * BK + chunk * 8));
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = tp[q];
                    ss[4 * q] = t.x; ss[4 * q + 1] = t.y; ss[4 * q + 2] = t.z; ss[4 * q + 3] = t.w;
                }
#pragma unroll
                for (int mi = 0; mi < TM; ++mi) af[mi] = pro_affine8<T>(af[mi], ss, p.pro.relu);
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
                    if constexpr (ABL == 2) {
                        asm volatile("" ::"v"(af[mi].x), "v"(af[mi].w), "v"(bfr[ni].x), "v"(bfr[ni].w));
                    } else if constexpr (sizeof(T) == 2) {
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
        stage = stage == NSTG - 1 ? 0 : stage + 1;
    }

    if (p.partial) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * WTM + mi * 16 + fg * 4 + r;
                if (row >= M) continue;
                float* prow = p.partial + ((long)blockIdx.z * M + row) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col = n0 + wn * WTN + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
            }
        return;
    }
    // ---- epilogue: stage the wave's fp32 tile in LDS, then each lane
    // finishes 8 consecutive columns of a row (one pixel decomposition per
    // row, 16-byte bf16 / 32-byte fp32 stores).
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    char* wbuf = smem + w * WTM * SROW;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
                *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) = acc[mi][ni][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own wave's rows only
    constexpr int CPR = WTN / 8;                      // 8-column chunks per row
    constexpr int RPP = 64 / CPR;                     // rows per pass of the wave
    const int cch = lane % CPR, rsub = lane / CPR;
    const int col0 = n0 + wn * WTN + cch * 8;
    const EpiParams& e = p.epi;
    float bias[8], scl[8], shf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        const bool cv = col < e.n_valid;
        bias[j] = (e.bias && cv) ? e.bias[col] : 0.f;
        scl[j] = (e.scale && cv) ? e.scale[col] : 1.f;
        shf[j] = (e.shift && cv) ? e.shift[col] : 0.f;
    }
    constexpr bool bnb = BNB;                          // folded BatchNorm backward (see EpiParams)
    float bsc[8], bsh[8], sgm[8], sbt[8];
    if constexpr (BNB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int col = col0 + j;
            const bool cv = col < e.bn_cv;
            bsc[j] = cv ? e.bn_gamma[col] * e.bn_inv : 0.f;
            bsh[j] = cv ? e.bn_beta[col] : 0.f;
            sgm[j] = sbt[j] = 0.f;
        }
    }
    const int hw2 = Ha * Wa;
    auto erow = [&](const int rr, const int k) {
        const int row = m0 + wm * WTM + rr;
        if (row >= M || col0 >= p.N) return;
        const int img = row / hw2;
        const int rem = row - img * hw2;
        const int a = rem / Wa;
        const int b = rem - a * Wa;
        const long pix = (long)(a * p.osh + ooh) * p.OW + (b * p.osw + oow);
        const float4 lo = *reinterpret_cast<const float4*>(wbuf + rr * SROW + cch * 32);
        const float4 hi = *reinterpret_cast<const float4*>(wbuf + rr * SROW + cch * 32 + 16);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        float res[8], mk[8];
        if (e.mask) {
            const T* mp = reinterpret_cast<const T*>(e.mask) + img * e.mask_img + pix * e.ld_mask + col0;
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp), mk);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp + 4), mk + 4);
        }
        if constexpr (BNB) {
            if (e.residual) Chunk<T>::unpack(pfr[k], res);
        } else if (e.residual) {
            const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
            Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            if constexpr (sizeof(T) == 4) Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp + 4), res + 4);
        }
        const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
        if constexpr (BNB) {
            // dL/da -> dL/dx of a = relu(BN(x)): mask re-derived from x with
            // the forward's arithmetic, BN scale, accumulation, column sums
            float xv[8];
            Chunk<T>::unpack(pfx[k], xv);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                const bool on = col < e.bn_cv && (!e.bn_relu || xv[j] * bsc[j] + bsh[j] > 0.f);
                const float dz = on ? v[j] : 0.f;
                sgm[j] += dz * xv[j];
                sbt[j] += dz;
                float x = dz * bsc[j];
                if (e.residual) x += res[j];
                v[j] = col < e.n_valid ? x : 0.f;
            }
        } else {
            const SegDropRun<8> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                float x = v[j] * scl[j] + shf[j] + bias[j];
                if (e.relu) x = fmaxf(x, 0.f);
                if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                if (e.residual) x += res[j];
                if (e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                v[j] = col < e.n_valid ? x : 0.f;
            }
        }
        T* yp = reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0;
        const uint4 packed = Chunk<T>::pack(v);
        *reinterpret_cast<uint4*>(yp) = packed;
        if constexpr (sizeof(T) == 4) *reinterpret_cast<uint4*>(yp + 4) = Chunk<T>::pack(v + 4);
        if constexpr (!BNB && sizeof(T) == 2) {
            if (e.y2) {      // BN2(+ReLU) of the stored values (seg_bn_relu_fwd's arithmetic)
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
                *reinterpret_cast<uint4*>(reinterpret_cast<T*>(e.y2) + img * e.y2_img + pix * e.ld_y2 + col0) =
                    Chunk<T>::pack(o2);
            }
        }
    };
    if constexpr (BNB) {
        static_assert(ERPP == RPP && ENPR * RPP == WTM, "prefetch rows = epilogue rows");
#pragma unroll
        for (int k = 0; k < ENPR; ++k) erow(rsub + k * RPP, k);
    } else {
#pragma unroll 2
        for (int rr = rsub; rr < WTM; rr += RPP) erow(rr, 0);
    }
    if constexpr (BNB) {
        // block column sums of dz*x / dz -> one partial row per M tile
        constexpr int WMW = NW / WN;
        __syncthreads();                              // staging reads done: reuse smem
        float* red = reinterpret_cast<float*>(smem);  // [NW * 64][16]
        static_assert(NW * 64 * 16 * 4 <= SMEM, "column-sum staging must fit");
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[tid * 16 + j] = sgm[j];
            red[tid * 16 + 8 + j] = sbt[j];
        }
        __syncthreads();
        for (int q = tid; q < 2 * BN; q += NW * 64) {
            const int kind = q / BN, lc = q - (q / BN) * BN;
            const int wn_ = lc / WTN, cch_ = (lc % WTN) / 8, j = lc % 8;
            float sum = 0.f;
            for (int wm_ = 0; wm_ < WMW; ++wm_)
                for (int rs = 0; rs < RPP; ++rs)
                    sum += red[((wm_ * WN + wn_) * 64 + rs * CPR + cch_) * 16 + kind * 8 + j];
            const int col = n0 + lc;
            if (col < e.bn_C) e.bn_part[(long)tm * 2 * e.bn_C + kind * e.bn_C + col] = sum;
        }
    }
}

// ---------------------------------------------------------------------------
// TN v2: filter gradients C[m][n] = sum_p A[p][m] B[p][n] with LDS-DMA staging.
// LDS image per stage: A [64 px][BM] and B [64 px][BN] bf16 rows, 16-byte
// chunks XOR-swizzled so the column-wise ds_read_b64_tr_b16 fragment reads
// are conflict-free.  Grid = splits x tiles flattened so that all tiles of one
// pixel range (split) are consecutive after the XCD remap -> they share the
// XCD's L2 for the x / dy rows of that range.
// ---------------------------------------------------------------------------
template <int ROWB>
__device__ __forceinline__ int tn2_swz(int row) {
    // conflict-free ds_read_b64_tr_b16 images: even XOR values that stay inside
    // the row's 16-chunk (256 B) half, or inside the row for 128 B rows
    if constexpr (ROWB >= 256) return ((row & 3) << 1) | (((row >> 3) & 1) << 3);
    else return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

// PRO: A (= x) through p.pro after the transposed LDS read; a lane's A rows
// are fixed channels, so its (scale, shift) pairs load once (single-tap only).
template <typename T, int BM, int BN, int WM, int WN, bool PRO = false>
__global__ __launch_bounds__(WM* WN * 64) void igemm_tn2(TNParams p, int tiles_m, int tiles_n, int splits) {
    constexpr int NW = WM * WN;
    constexpr int BKP = 64;
    constexpr int AROWB = BM * 2, BROWB = BN * 2;
    constexpr int A_RPI = 1024 / AROWB, B_RPI = 1024 / BROWB;     // rows per glds instruction
    constexpr int A_INS = BKP / A_RPI / NW, B_INS = BKP / B_RPI / NW;
    static_assert(A_INS * A_RPI * NW == BKP && B_INS * B_RPI * NW == BKP, "rows must split per wave");
    constexpr int A_CPR = AROWB / 16, B_CPR = BROWB / 16;       // 16-byte chunks per row
    constexpr int NI = A_INS + B_INS;
    constexpr int ASZ = BKP * AROWB, STAGE = BKP * (AROWB + BROWB);
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    __shared__ __attribute__((aligned(16))) char smem[3 * STAGE];

    const int ntile = tiles_m * tiles_n;
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int split = wg / ntile;
    const int tile = wg - split * ntile;
    if (split >= splits) return;
    const int tm = tile / tiles_n, tn = tile - (tile / tiles_n) * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = (p.P + BKP - 1) / BKP;
    int kt_begin = 0, kt_end = KT;
    if (p.partial) {
        kt_begin = split * p.kt_per_split;
        kt_end = min(KT, kt_begin + p.kt_per_split);
    }

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Bm = reinterpret_cast<const T*>(p.b);
    const void* zero = (const void*)g_zero_page;

    // ---- A: lane -> (row within instruction, physical chunk) -> global chunk
    const int a_rsub = lane / A_CPR, a_pc = lane % A_CPR;
    const int a_row0 = w * A_RPI + a_rsub;                // row of instruction 0
    const int a_c = (a_pc & ~15) | ((a_pc & 15) ^ tn2_swz<AROWB>(a_row0));   // swizzle i-independent
    const int am = m0 + a_c * 8;
    const bool a_mok = am < p.M;
    const int atap = a_mok ? am / p.Cg : 0;
    const int ac = a_mok ? am - atap * p.Cg : 0;
    const int atj = atap / p.taps_w, ati = atap - atj * p.taps_w;
    const int hoff = atj * p.tsh + p.ioh, woff = ati * p.tsw + p.iow;
    int pimg[A_INS], pa[A_INS], pb[A_INS], pp[A_INS];
    const int hw = p.Ha * p.Wa;
    const PixStep pstep(BKP, p.Ha, p.Wa);
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
        const int pix = kt_begin * BKP + (i * NW) * A_RPI + a_row0;
        pp[i] = pix;
        const int q = pix < p.P ? pix : 0;
        pimg[i] = q / hw;
        const int rem = q - pimg[i] * hw;
        pa[i] = rem / p.Wa;
        pb[i] = rem - pa[i] * p.Wa;
    }
    // ---- B
    const int b_rsub = lane / B_CPR, b_pc = lane % B_CPR;
    const int b_row0 = w * B_RPI + b_rsub;
    const int b_c = (b_pc & ~15) | ((b_pc & 15) ^ tn2_swz<BROWB>(b_row0));
    const int bn = n0 + b_c * 8;
    const bool b_nok = bn < p.N;
    int bpix = kt_begin * BKP + b_row0;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    auto load_stage = [&](int stage) {
        const unsigned sb_ = lds0 + stage * STAGE;
#pragma unroll
        for (int i = 0; i < A_INS; ++i) {
            const int ih = pa[i] * p.ish + hoff, iw = pb[i] * p.isw + woff;
            const bool ok = a_mok && pp[i] < p.P && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const void* src = ok ? (const void*)(X + (long)pimg[i] * p.x_img + ((long)ih * p.IW + iw) * p.ldx + ac) : zero;
            glds16(src, sb_ + (i * NW + w) * 1024);
            pp[i] += BKP;
            pstep.advance(BKP, p.Ha, p.Wa, pimg[i], pa[i], pb[i]);
        }
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const int pix = bpix + (i * NW) * B_RPI;
            const bool ok = b_nok && pix < p.P;
            const void* src = ok ? (const void*)(Bm + (long)pix * p.ldb + bn) : zero;
            glds16(src, sb_ + ASZ + (i * NW + w) * 1024);
        }
        bpix += BKP;
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float psc[PRO ? TM : 1], psh[PRO ? TM : 1];
    if constexpr (PRO) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
            const int m = m0 + wm * WTM + mi * 16 + (lane & 15);
            const bool v = m < p.M && m < p.pro.cv;
            psc[mi] = v ? p.pro.gamma[m] * p.pro.inv : 0.f;
            psh[mi] = v ? p.pro.beta[m] : 0.f;
            asm volatile("" ::"v"(psc[mi]), "v"(psh[mi]));   // loaded before the first DMA
        }
    }
    if (kt_begin < kt_end) load_stage(0);
    if (kt_begin + 1 < kt_end) load_stage(1);
    const int fr = lane & 15, fg = lane >> 4;
    const int tq = (lane & 15) >> 2, tpp = lane & 3;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    int stage = 0;
    for (int kt = kt_begin; kt < kt_end; ++kt) {
        if (kt + 1 < kt_end) wait_vmcnt<NI>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (kt + 2 < kt_end) load_stage(stage == 0 ? 2 : stage - 1);
        const char* As = smem + stage * STAGE;
        const char* Bs = As + ASZ;
#pragma unroll
        for (int ks = 0; ks < BKP / 32; ++ks) {
            uint4 af[TM], bfr[TN];
            const int r1 = ks * 32 + 8 * fg + tq;
            const int s1 = tn2_swz<AROWB>(r1), s2 = tn2_swz<AROWB>(r1 + 4);
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int chk = ((wm * WTM + mi * 16) >> 3) + (tpp >> 1);
                const int c1 = (chk & ~15) | ((chk & 15) ^ s1), c2 = (chk & ~15) | ((chk & 15) ^ s2);
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(As + r1 * AROWB + 16 * c1 + 8 * (tpp & 1)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(As + (r1 + 4) * AROWB + 16 * c2 + 8 * (tpp & 1)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                af[mi] = __builtin_bit_cast(uint4, v);
                if constexpr (PRO) af[mi] = pro_affine<T>(af[mi], psc[mi], psh[mi], p.pro.relu);
            }
            const int t1 = tn2_swz<BROWB>(r1), t2 = tn2_swz<BROWB>(r1 + 4);
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int chk = ((wn * WTN + ni * 16) >> 3) + (tpp >> 1);
                const int c1 = (chk & ~15) | ((chk & 15) ^ t1), c2 = (chk & ~15) | ((chk & 15) ^ t2);
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Bs + r1 * BROWB + 16 * c1 + 8 * (tpp & 1)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Bs + (r1 + 4) * BROWB + 16 * c2 + 8 * (tpp & 1)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bfr[ni] = __builtin_bit_cast(uint4, v);
            }
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    acc[mi][ni] = mfma16x16x32<T>(af[mi], bfr[ni], acc[mi][ni]);
        }
        stage = stage == 2 ? 0 : stage + 1;
    }

#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + mi * 16 + fg * 4 + r;
            if (m >= p.M) continue;
            if (p.partial) {
                float* prow = p.partial + ((long)split * p.Mp + m) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int n = n0 + wn * WTN + ni * 16 + fr;
                    if (n < p.N) prow[n] = acc[mi][ni][r];
                }
                continue;
            }
            const int tap = m / p.Cg;
            const int c = m - tap * p.Cg;
            if (c >= p.c_valid) continue;
            float* orow = p.out + (long)tap * p.o_tap + (long)c * p.o_c;
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int n = n0 + wn * WTN + ni * 16 + fr;
                if (n < p.n_valid) orow[(long)n * p.o_n] = acc[mi][ni][r];
            }
        }
}

template <typename T, int BM, int BN, int WM, int WN, bool PRO = false>
void launch_tn2_t(TNParams& p, int splits, hipStream_t s) {
    const int tm = (p.M + BM - 1) / BM, tn = (p.N + BN - 1) / BN;
    hipLaunchKernelGGL((igemm_tn2<T, BM, BN, WM, WN, PRO>), dim3(tm * tn * splits), dim3(WM * WN * 64), 0, s, p, tm,
                       tn, splits);
}

template <typename T, bool PRO = false>
static void launch_tn2_typed(TNParams& p, int bm, int bn, int splits, hipStream_t s) {
    if (bm == 256 && bn == 128) launch_tn2_t<T, 256, 128, 4, 2, PRO>(p, splits, s);
    else if (bm == 128 && bn == 256) launch_tn2_t<T, 128, 256, 2, 4, PRO>(p, splits, s);
    else if (bm == 256 && bn == 64) launch_tn2_t<T, 256, 64, 4, 2, PRO>(p, splits, s);
    else if (bm == 128 && bn == 64) launch_tn2_t<T, 128, 64, 4, 2, PRO>(p, splits, s);
    else launch_tn2_t<T, 128, 128, 2, 4, PRO>(p, splits, s);
}

void launch_tn2(TNParams& p, int bm, int bn, int splits, hipStream_t s, int dtype) {
    if (dtype == SEG_F16) launch_tn2_typed<f16>(p, bm, bn, splits, s);
    else launch_tn2_typed<bf16>(p, bm, bn, splits, s);
}

void launch_tn2_pro(TNParams& p, int bm, int bn, int splits, hipStream_t s, int dtype) {
    if (dtype == SEG_F16) launch_tn2_typed<f16, true>(p, bm, bn, splits, s);
    else launch_tn2_typed<bf16, true>(p, bm, bn, splits, s);
}


template <typename T, int BM, int BN, int WM, int WN>
void launch_nt2_t(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    const dim3 g(tiles, 1, gridz), b(WM * WN * 64);
#ifdef SEG_DIAG   // ablation builds (garbage results): tools/ only
    if constexpr (is_bf16_v<T> && BN == 128) {
        switch (g_nt2_ablate) {
            case 1: hipLaunchKernelGGL((igemm_nt2<T, BM, BN, WM, WN, 1>), g, b, 0, s, p); return;
            case 2: hipLaunchKernelGGL((igemm_nt2<T, BM, BN, WM, WN, 2>), g, b, 0, s, p); return;
            case 3: hipLaunchKernelGGL((igemm_nt2<T, BM, BN, WM, WN, 3>), g, b, 0, s, p); return;
        }
    }
#endif
    hipLaunchKernelGGL((igemm_nt2<T, BM, BN, WM, WN>), g, b, 0, s, p);
}

// Short-K bf16 problems (<= g_nt2_short 64-deep k tiles, no split-K) on the
// 2-stage ring with 64-column tiles: two blocks per CU.  0 = off (tests / A-B).

bool nt2_short(const NTParams& p, int dtype) {
    return dtype == SEG_BF16 && !p.partial && p.K <= 64 * g_nt2_short && g_nt2_ablate == 0;
}

// input gradient + folded BN backward (EpiParams.bn_*): short-K 2-stage form,
// 256-row tiles of 8 waves (two blocks per CU); one bn_part row per M tile
long nt2_bn_rows(int M) { return (M + 255) / 256; }

void launch_nt2_bn(NTParams& p, int dtype, hipStream_t s) {
    const int tiles = ((p.M + 255) / 256) * ((p.N + 63) / 64);
    if (dtype == SEG_F16)
        hipLaunchKernelGGL((igemm_nt2<f16, 256, 64, 4, 2, 0, 2, false, true>), dim3(tiles), dim3(512), 0, s, p);
    else
        hipLaunchKernelGGL((igemm_nt2<bf16, 256, 64, 4, 2, 0, 2, false, true>), dim3(tiles), dim3(512), 0, s, p);
}

bool nt2_pro_ok(const NTParams& p, int dtype, int nphases) {
    return (dtype == SEG_BF16 || dtype == SEG_F16) && nphases == 1 && g_nt2_ablate == 0 && p.K == p.C &&
           (p.K + 63) / 64 * 64 <= NT2_PRO_MAXK;
}

// 192-row tiles: the 2-stage ring (64 KiB) + the 8 KiB table leave room for
// two blocks per CU at 64 columns.
template <typename T>
static void launch_nt2_pro_t(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tm = (max_m + 191) / 192;
    if (p.N <= 64)
        hipLaunchKernelGGL((igemm_nt2<T, 192, 64, 4, 2, 0, 2, true>), dim3(tm, 1, gridz), dim3(512), 0, s, p);
    else
        hipLaunchKernelGGL((igemm_nt2<T, 192, 128, 4, 2, 0, 3, true>), dim3(tm * ((p.N + 127) / 128), 1, gridz),
                           dim3(512), 0, s, p);
}

void launch_nt2_pro(NTParams& p, int dtype, int gridz, int max_m, hipStream_t s) {
    if (dtype == SEG_F16) launch_nt2_pro_t<f16>(p, gridz, max_m, s);
    else launch_nt2_pro_t<bf16>(p, gridz, max_m, s);
}

void launch_nt2(NTParams& p, int dtype, int bn, int gridz, int max_m, hipStream_t s) {
    if (dtype == SEG_BF16) {
        if (nt2_short(p, dtype)) {
            const int tiles = ((max_m + 255) / 256) * ((p.N + 63) / 64);
            hipLaunchKernelGGL((igemm_nt2<bf16, 256, 64, 4, 2, 0, 2>), dim3(tiles, 1, gridz), dim3(512), 0, s, p);
        } else if (bn == 64) launch_nt2_t<bf16, 256, 64, 4, 2>(p, gridz, max_m, s);
        else launch_nt2_t<bf16, 256, 128, 4, 2>(p, gridz, max_m, s);
    } else if (dtype == SEG_F16) {
        if (bn == 64) launch_nt2_t<f16, 256, 64, 4, 2>(p, gridz, max_m, s);
        else launch_nt2_t<f16, 256, 128, 4, 2>(p, gridz, max_m, s);
    } else {
        if (bn == 64) launch_nt2_t<float, 256, 64, 4, 2>(p, gridz, max_m, s);
        else launch_nt2_t<float, 256, 128, 4, 2>(p, gridz, max_m, s);
    }
}

}  // namespace seg
