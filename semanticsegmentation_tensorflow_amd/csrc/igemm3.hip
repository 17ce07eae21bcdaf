// Third-generation implicit-GEMM NT kernel for gfx950: 256 x 256 tiles.
//
// Same contract as igemm_nt / igemm_nt2 (NTParams, igemm.h) for bf16, built on
// the schedule the halo direct conv (halo.hip, conv_halo2) measured best, but
// with the implicit-GEMM gather of igemm_nt2 on BOTH operands:
//  * 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave (LDS bytes per MFMA
//    FLOP 0.75x of igemm_nt2's 64 x 64 wave tiles);
//  * each 64-deep K tile is two phases: h0 reads A rows 0..127 of the wave's
//    half + the whole B slice and issues the LDS-DMA of B(t+1); h1 reads A
//    rows 128..255 and issues A(t+2); each phase = 32 MFMAs between barriers;
//  * the upper M wave group runs one barrier behind, so on every SIMD
//    one wave's MFMA cluster overlaps the other wave's LDS reads;
//  * LDS: A in a 3-stage ring (3 x 32 KiB), B in a 2-stage ring (2 x 32 KiB)
//    = 160 KiB, one block per CU.  Every buffer is restaged >= 2 phases after
//    its last reads (retired with lgkmcnt(0) before a barrier both wave
//    groups pass), and every DMA is retired by its issuing wave's counted
//    vmcnt before a barrier that precedes (by one more for the lagging group)
//    the first read of its data;
//  * source-side XOR swizzle of the 16-byte chunks (LDS image lane-linear,
//    conflict-free ds_read_b128), zero page for padding / tails, split-K and
//    conv2d_transpose phases as in igemm_nt2, LDS-staged row epilogue.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

__device__ uint4 g_nt3_zero[4];

// XOR swizzle of the 16-byte chunks of a [k][n] row image (512-byte rows):
// the column-wise ds_read_b64_tr_b16 fragment reads are conflict-free
// (igemm_tn3's operands, igemm_nt3's B-transposed form)
__device__ __forceinline__ int tn3_swz(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

// BT: B given as [k][n] rows (n contiguous: the HWIO filter copy, the one the
// input gradient reads) instead of [n][k]: staged as 64 x 512-byte k rows like
// igemm_tn3's operands and read with transposing ds_read_b64_tr_b16, so one
// packed copy serves the forward and the input gradient (FCN conv6 / conv7:
// no KRSC copy, no rows_to_tr after their fused Adam).  Needs C % 64 == 0
// (a k tile never crosses a tap).
template <typename T = bf16, bool BT = false>
__global__ __launch_bounds__(512) void igemm_nt3(NTParams p) {
    constexpr int NW = 8, BM = 256, BN = 256, BK = 64;
    constexpr int WTM = 128, WTN = 64, TN = WTN / 16;   // TM = 8 (two halves of 4)
    constexpr int A_INS = BM / 8 / NW, B_INS = BN / 8 / NW;   // 4 + 4 DMA pieces per wave per tile
    constexpr int ABUF = BM * 128, BBUF = BN * 128;
    __shared__ __attribute__((aligned(16))) char smem[3 * ABUF + 2 * BBUF];

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
    const int tiles_mg = gridDim.x / tiles_n;
    int tm, tn;
    if (tiles_mg <= 16 && tiles_n > tiles_mg) {   // few M tiles: share each B panel on one XCD
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
    const int nk = kt_end - kt_begin;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 2, wn = w & 3;
    const int lr = lane >> 3;
    const int c = (lane & 7) ^ ((((w & 1) << 2) + (lr >> 1)) & 7);

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)g_nt3_zero;

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
    // BT: lane -> (row of the 2-row DMA piece, physical chunk) -> column bn;
    // pieces differ by 16 rows, which the swizzle ignores
    const int rsubb = lane >> 5, pcb = lane & 31;
    const int rowb0 = w * 2 + rsubb;
    const int bn_bt = n0 + ((pcb & ~15) | ((pcb & 15) ^ tn3_swz(rowb0))) * 8;
    const bool bnok_bt = bn_bt < p.N;
    int bt_cc = 0, bt_ti = 0, bt_tj = 0, bt_kg = kt_begin * BK;
    if constexpr (BT) {
        const int tap = bt_kg / p.C;
        bt_cc = bt_kg - tap * p.C;
        bt_tj = tap / p.taps_w;
        bt_ti = tap - bt_tj * p.taps_w;
    }
    // independent k trackers: A runs two tiles ahead, B one
    struct KState { int kg, cc, ti, tj; };
    auto kinit = [&](int kt) {
        KState s;
        s.kg = kt * BK + c * 8;
        const int tap = s.kg / p.C;
        s.cc = s.kg - tap * p.C;
        s.tj = tap / p.taps_w;
        s.ti = tap - s.tj * p.taps_w;
        return s;
    };
    auto kadv = [&](KState& s) {
        s.kg += BK;
        s.cc += BK;
        while (s.cc >= p.C) {
            s.cc -= p.C;
            if (++s.ti == p.taps_w) { s.ti = 0; ++s.tj; }
        }
    };
    KState ka = kinit(kt_begin), kb = ka;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + 3 * ABUF;
    auto issue_a = [&](int buf) {
        const bool kok = ka.kg < p.K;
        const int dh = ka.tj * p.tsh, dw = ka.ti * p.tsw;
#pragma unroll
        for (int i = 0; i < A_INS; ++i) {
            const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
            const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const void* src = ok ? (const void*)(X + a_off[i] + ((long)ih * p.IW + iw) * p.ldx + ka.cc) : zero;
            glds16(src, lds0 + buf * ABUF + (i * NW + w) * 1024);
        }
        kadv(ka);
    };
    auto issue_b = [&](int buf) {
        if constexpr (BT) {
            const bool kok = bt_kg < p.K;
            const long wtap = (long)((rb + p.rstep * bt_tj) * p.Sfull + (sb + p.sstep * bt_ti)) * p.w_tap +
                              (long)(bt_cc + rowb0) * p.w_col + bn_bt;
#pragma unroll
            for (int i = 0; i < B_INS; ++i) {
                const void* src = (kok && bnok_bt) ? (const void*)(Wt + wtap + (long)(i * NW * 2) * p.w_col) : zero;
                glds16(src, ldsB + buf * BBUF + (i * NW + w) * 1024);
            }
            bt_kg += BK;
            bt_cc += BK;
            if (bt_cc >= p.C) {
                bt_cc -= p.C;
                if (++bt_ti == p.taps_w) { bt_ti = 0; ++bt_tj; }
            }
            return;
        }
        const bool kok = kb.kg < p.K;
        const long wtap = (long)((rb + p.rstep * kb.tj) * p.Sfull + (sb + p.sstep * kb.ti)) * p.w_tap + kb.cc;
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const bool ok = b_ok[i] && kok;
            const void* src = ok ? (const void*)(Wt + b_off[i] + wtap) : zero;
            glds16(src, ldsB + buf * BBUF + (i * NW + w) * 1024);
        }
        kadv(kb);
    };

    f32x4 acc[8][TN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) {
        issue_a(0);
        issue_b(0);
        if (nk > 1) {
            issue_a(1);
            wait_vmcnt<A_INS>();
        } else {
            wait_vmcnt<0>();
        }
    }
    lds_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();

    const int fr = lane & 15, fg = lane >> 4;
    // BT fragment offsets (igemm_tn3's B reads): row fr1 = 8 fg + tq, chunk of
    // column col0 + ..., the second 4 rows at +4 * 512
    unsigned boff_bt[TN];
    if constexpr (BT) {
        const int tq = (lane & 15) >> 2, tpp = lane & 3;
        const int fr1 = 8 * fg + tq, fsw = tn3_swz(fr1);
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
            const int chk = ((wn * WTN + ni * 16) >> 3) + (tpp >> 1);
            boff_bt[ni] = (unsigned)(fr1 * 512 + 16 * ((chk & ~15) | ((chk & 15) ^ fsw)) + 8 * (tpp & 1));
        }
    }
    int abuf = 0, bbuf = 0;
    for (int it = 0; it < nk; ++it) {
        const char* As = smem + abuf * ABUF;
        const char* Bs = smem + 3 * ABUF + bbuf * BBUF;
        uint4 af[2][4], bq[2][TN];
        auto read_a = [&](int mh) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const int row = wm * WTM + mh * 64 + mi * 16 + fr;
                    af[ks][mi] = *reinterpret_cast<const uint4*>(As + row * 128 + 16 * ((ks * 4 + fg) ^ ((row >> 1) & 7)));
                }
        };
        auto mma = [&](int mh) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[mh * 4 + mi][ni] = mfma16x16x32<T>(af[ks][mi], bq[ks][ni], acc[mh * 4 + mi][ni]);
            __builtin_amdgcn_s_setprio(0);
        };
        // h0: A half 0 + B slice; B(t+1) into the other B buffer (last read at h0(t-1))
        read_a(0);
        if constexpr (BT) {
            typedef short s16x8 __attribute__((ext_vector_type(8)));
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    SEG_LDS char* a = (SEG_LDS char*)Bs + boff_bt[ni] + ks * 32 * 512;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)a);
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(a + 4 * 512));
                    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    bq[ks][ni] = __builtin_bit_cast(uint4, v);
                }
        } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int row = wn * WTN + ni * 16 + fr;
                    bq[ks][ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * ((ks * 4 + fg) ^ ((row >> 1) & 7)));
                }
        }
        if (it + 1 < nk) issue_b(bbuf ^ 1);
        __builtin_amdgcn_s_barrier();
        mma(0);
        __builtin_amdgcn_s_barrier();
        // h1: A half 1; A(t+2) into the A buffer of t-1 (last read at h1(t-1));
        // then A(t+1) and B(t+1) must have landed before the next h0
        read_a(1);
        const int anext = abuf == 0 ? 2 : abuf - 1;   // (abuf + 2) % 3
        if (it + 2 < nk) issue_a(anext);
        // the wait precedes the barrier the lagging group passes before its
        // next reads (half an iteration for B(t+1) to land)
        if (it + 2 < nk) wait_vmcnt<A_INS>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        mma(1);
        __builtin_amdgcn_s_barrier();
        abuf = abuf == 2 ? 0 : abuf + 1;
        bbuf ^= 1;
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();

    if (p.partial) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
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
    // ---- epilogue in two 64-row halves per wave (LDS holds 8 x 64 x WTN fp32)
    constexpr int SROW = WTN * 4 + 16;
    constexpr int CPR = WTN / 8, RPP = 64 / CPR;
    static_assert(NW * 64 * SROW <= 3 * ABUF + 2 * BBUF, "epilogue staging must fit");
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
    char* wbuf = smem + w * 64 * SROW;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
        lds_barrier();
        {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                            acc[mh * 4 + mi][ni][r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 2
        for (int rr = rsub; rr < 64; rr += RPP) {
            const int row = m0 + wm * WTM + mh * 64 + rr;
            if (row >= M || col0 >= p.N) continue;
            const int img = row / hw;
            const int rem = row - img * hw;
            const int a = rem / Wa;
            const int b = rem - a * Wa;
            const long pix = (long)(a * p.osh + ooh) * p.OW + (b * p.osw + oow);
            float v[8];
            splitk_lds8(wbuf + rr * SROW + cch * 32, v);
            float res[8], mk[8];
            if (e.mask) {
                const T* mp = reinterpret_cast<const T*>(e.mask) + img * e.mask_img + pix * e.ld_mask + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp), mk);
            }
            if (e.residual) {
                const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            }
            const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
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
            T* yp = reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0;
            const uint4 packed = Chunk<T>::pack(v);
            *reinterpret_cast<uint4*>(yp) = packed;
            if (e.y2) {      // BN2(+ReLU) of the stored values (seg_bn_relu_fwd's arithmetic, as igemm_nt2)
                float r2[8], o2[8];
                Chunk<T>::unpack(packed, r2);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int col = col0 + j;
                    const bool c2 = col < e.bn2_cv;
                    float v2 = __builtin_fmaf(r2[j], c2 ? e.bn2_gamma[col] * e.bn2_inv : 0.f, c2 ? e.bn2_beta[col] : 0.f);
                    if (e.bn2_relu) v2 = fmaxf(v2, 0.f);
                    o2[j] = v2;
                }
                *reinterpret_cast<uint4*>(reinterpret_cast<T*>(e.y2) + img * e.y2_img + pix * e.ld_y2 + col0) =
                    Chunk<T>::pack(o2);
            }
        }
    }
}

// 256 x 256 tiles, one block per CU: split K until the grid covers the CUs in
// one round (keeping >= 6 K tiles per split), never past 64 slabs.
void nt3_info(int M, int N, int K, int cus, int* splits) {
    const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
    const int kt = (K + 63) / 64;
    *splits = one_round_splits(tiles, cus, std::min(64, std::max(1, kt / 6)));
}

bool nt3_ok(const NTParams& p, int dtype) {
    return g_nt3 && (dtype == SEG_BF16 || dtype == SEG_F16) && p.N > 128;
}

template <typename T>
static void launch_nt3_t(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + 255) / 256) * ((p.N + 255) / 256);
    if (p.bt) hipLaunchKernelGGL((igemm_nt3<T, true>), dim3(tiles, 1, gridz), dim3(512), 0, s, p);
    else hipLaunchKernelGGL((igemm_nt3<T>), dim3(tiles, 1, gridz), dim3(512), 0, s, p);
}

void launch_nt3(NTParams& p, int gridz, int max_m, hipStream_t s, int dtype) {
    if (dtype == SEG_F16) launch_nt3_t<f16>(p, gridz, max_m, s);
    else launch_nt3_t<bf16>(p, gridz, max_m, s);
}


// ---------------------------------------------------------------------------
// TN v3: filter gradients C[m][n] = sum_p A[p][m] B[p][n] on 256 x 256 tiles.
// LDS image per stage: 64 pixel rows x 512 B for A (gathered x columns) and
// for B (dy columns); 16-byte chunks XOR-swizzled within 256-byte halves so
// the column-wise ds_read_b64_tr_b16 fragment reads are conflict-free (as
// igemm_tn2).  Same wave layout, rings and staggered two-phase schedule as
// igemm_nt3.  Epilogue: fp32 tile staged in LDS, 32-byte row-contiguous
// stores (filter gradient or split-K slab).
// ---------------------------------------------------------------------------

// Main loop unstaggered: the DMA wait for slice t+1 sits at the end of the
// iteration, a full iteration after its issue.  The dy / x slices of a filter
// gradient miss L2 far more often than a forward conv's filter slices, so the
// longer window beats conv_halo2's wave-group stagger here (conv6 main loop
// 445 -> 307 us measured with the staggered form, since removed).
__device__ int g_tn3_cu_slots[4096];

// ABL: see g_tn3_abl.  MFAST: consecutive tiles walk M (share the dy panel).
// ADAM: TF1 Adam on the parameters of the tile (p.adam) instead of (or besides)
// storing the gradient -- the filter gradient never round-trips through HBM.
// BN / BKP: 256 / 64 is the one-block-per-CU tile (8 waves, 160 KiB rings);
// 128 / 32 is the half tile (4 waves, 64 KiB rings + 68 KiB epilogue staging)
// that runs two blocks per CU, so one block's HBM-bound epilogue (the fused
// Adam) overlaps the other block's MFMA main loop.
template <int ABL = 0, bool MFAST = false, bool ADAM = false, int BN = 256, int BKP = 64, typename T = bf16>
__global__ __launch_bounds__(BN * 2, 2) void igemm_tn3(TNParams p, int tiles_m, int tiles_n, int splits) {
    static_assert(!ADAM || is_bf16_v<T>, "the fused Adam epilogue writes bf16 weight copies");
    constexpr int BM = 256, WTM = 128, WTN = 64, TN = WTN / 16;
    constexpr int NWN = BN / WTN, NW = 2 * NWN;                      // waves: 2 (M) x NWN (N)
    constexpr int ROWB = BM * 2, RPI = 1024 / ROWB, CPR = ROWB / 16; // A: 2 rows / DMA piece, 32 chunks / row
    constexpr int ROWBB = BN * 2, RPIB = 1024 / ROWBB, CPRB = ROWBB / 16;
    constexpr int A_INS = BKP / RPI / NW, B_INS = BKP / RPIB / NW;
    constexpr int KS = BKP / 32;
    constexpr int ABUF = BKP * ROWB, BBUF = BKP * ROWBB;
    // B (dy) ring depth: 3 stages for the half tile (B(t+2) issued at t, two
    // iterations to land; its 32-deep iterations are short), else 2
    constexpr int BST = BN == 128 ? 3 : 2;
    constexpr int RING = 3 * ABUF + BST * BBUF;
    constexpr int EPI = ADAM ? NW * (32 * (WTN * 4 + 16) + WTN * (32 * 2 + 16)) : NW * 64 * (WTN * 4 + 16);
    constexpr int SMEM = RING > EPI ? RING : EPI;
    static_assert(A_INS * NW * RPI == BKP && B_INS * NW * RPIB == BKP, "DMA pieces must tile the stage");
    static_assert(NW == 8 || (NW == 4 && BKP == 32), "A-piece row map");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    typedef short s16x8 __attribute__((ext_vector_type(8)));

    if constexpr (ADAM && BN == 128) {
        // The two blocks resident on a CU start together and would stay in
        // lock step (both in the MFMA loop, then both in the HBM-bound
        // update).  The second arrival on each CU in the first round starts
        // late, seeding the alternation main loop <-> update across the pair.
        if (p.adam.stagger > 0 && (int)blockIdx.x < p.adam.first_round) {
            __shared__ int late;
            if (threadIdx.x == 0) {
                const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_ID
                const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // XCC_ID
                const int cu = (int)(((xcc & 15u) << 8) | ((hw >> 8) & 255u));
                late = atomicAdd(&p.adam.cu_slots[cu], 1) & 1;
            }
            __syncthreads();
            if (late) {
                const unsigned long long t0 = wall_clock64();
                while (wall_clock64() - t0 < (unsigned long long)p.adam.stagger) __builtin_amdgcn_s_sleep(16);
            }
        }
    }
    const int ntile = tiles_m * tiles_n;
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int split = wg / ntile;
    const int tile = wg - split * ntile;
    if (split >= splits) return;
    int tm, tn;
    if (MFAST) {
        tn = tile / tiles_m;
        tm = tile - tn * tiles_m;
    } else {
        tm = tile / tiles_n;
        tn = tile - tm * tiles_n;
    }
    const int m0 = tm * BM, n0 = tn * BN;
    const int KT = (p.P + BKP - 1) / BKP;
    int kt_begin = 0, kt_end = KT;
    if (p.partial) {
        kt_begin = split * p.kt_per_split;
        kt_end = min(KT, kt_begin + p.kt_per_split);
    }
    const int nk = max(0, kt_end - kt_begin);

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / NWN, wn = w % NWN;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Bm = reinterpret_cast<const T*>(p.b);
    const void* zero = (const void*)g_nt3_zero;

    // first stage row of A piece i (2 rows): the pieces of one wave differ
    // only in row bits the swizzle ignores (bits 4+ for 8 waves; bits 2 and
    // 4 for 4 waves), so one swizzled column serves all of them
    auto arow = [&](int i) {
        return NW == 8 ? (i * NW + w) * RPI : 2 * (w & 1) + 8 * (w >> 1) + 4 * (i & 1) + 16 * (i >> 1);
    };
    // lane -> (row of the DMA piece, physical chunk) -> global chunk
    const int rsub = lane / CPR, pc = lane % CPR;
    const int row0 = arow(0) + rsub;
    const int gc = (pc & ~15) | ((pc & 15) ^ tn3_swz(row0));
    // A: column m = m0 + gc*8 .. +7 -> (tap, channel)
    const int am = m0 + gc * 8;
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
        const int pix = kt_begin * BKP + arow(i) + rsub;
        pp[i] = pix;
        const int q = pix < p.P ? pix : 0;
        pimg[i] = q / hw;
        const int rem = q - pimg[i] * hw;
        pa[i] = rem / p.Wa;
        pb[i] = rem - pa[i] * p.Wa;
    }
    // B: column n = n0 + gcb*8 (B pieces differ by 16 rows: swizzle-invariant)
    const int rsubb = lane / CPRB, pcb = lane % CPRB;
    const int rowb0 = w * RPIB + rsubb;
    const int gcb = (pcb & ~15) | ((pcb & 15) ^ tn3_swz(rowb0));
    const int bn = n0 + gcb * 8;
    const bool b_nok = bn < p.N;
    int bpix = kt_begin * BKP + rowb0;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + 3 * ABUF;
    auto issue_a = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_INS; ++i) {
            const int ih = pa[i] * p.ish + hoff, iw = pb[i] * p.isw + woff;
            const bool ok = a_mok && pp[i] < p.P && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const void* src = ok ? (const void*)(X + (long)pimg[i] * p.x_img + ((long)ih * p.IW + iw) * p.ldx + ac) : zero;
            glds16(src, lds0 + buf * ABUF + arow(i) * ROWB);
            pp[i] += BKP;
            pstep.advance(BKP, p.Ha, p.Wa, pimg[i], pa[i], pb[i]);
        }
    };
    auto issue_b = [&](int buf) {
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const int pix = bpix + (i * NW) * RPIB;
            const bool ok = b_nok && pix < p.P;
            const void* src = ok ? (const void*)(Bm + (long)pix * p.ldb + bn) : zero;
            glds16(src, ldsB + buf * BBUF + (i * NW + w) * 1024);
        }
        bpix += BKP;
    };

    f32x4 acc[8][TN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) {
        issue_a(0);
        issue_b(0);
        if (nk > 1) {
            issue_a(1);
            if constexpr (BST == 3) {
                issue_b(1);
                wait_vmcnt<A_INS + B_INS>();
            } else {
                wait_vmcnt<A_INS>();
            }
        } else {
            wait_vmcnt<0>();
        }
    }
    lds_barrier();

    const int fg = lane >> 4;
    const int tq = (lane & 15) >> 2, tpp = lane & 3;
    // Per-lane LDS byte offsets of the fragment reads, hoisted out of the
    // loop: row r1 = 8 fg + tq has bit 2 clear, so rows r1 + 4 and
    // r1 + 32 ks share its swizzle and are immediate offsets of one address.
    const int fr1 = 8 * fg + tq, fsw = tn3_swz(fr1);
    auto lane_off = [&](int col0, int rowb) {
        const int chk = (col0 >> 3) + (tpp >> 1);
        return (unsigned)(fr1 * rowb + 16 * ((chk & ~15) | ((chk & 15) ^ fsw)) + 8 * (tpp & 1));
    };
    unsigned aoff[2][4], boff[TN];
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) aoff[mh][mi] = lane_off(wm * WTM + mh * 64 + mi * 16, ROWB);
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) boff[ni] = lane_off(wn * WTN + ni * 16, ROWBB);
    int abuf = 0, bbuf = 0;
    for (int it = 0; it < nk; ++it) {
        SEG_LDS char* As = (SEG_LDS char*)smem + abuf * ABUF;
        SEG_LDS char* Bs = (SEG_LDS char*)smem + 3 * ABUF + bbuf * BBUF;
        vec8_t<T> af[KS][4], bq[KS][TN];
        // 16 columns x 32 pixel rows fragment at lane offset `off`, k rows ks*32 ..
        auto frag = [&](SEG_LDS char* base, int rowb, unsigned off, int ks) {
            SEG_LDS char* a = base + off + ks * 32 * rowb;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)a);
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(a + 4 * rowb));
            s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            return __builtin_bit_cast(vec8_t<T>, v);
        };
        auto read_a = [&](int mh) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) af[ks][mi] = frag(As, ROWB, aoff[mh][mi], ks);
        };
        auto mma = [&](int mh) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[mh * 4 + mi][ni] = mfma_v8<T>(af[ks][mi], bq[ks][ni], acc[mh * 4 + mi][ni]);
            __builtin_amdgcn_s_setprio(0);
        };
        if constexpr (ABL == 0) {
            // Unstaggered: ONE barrier per iteration.  Every buffer a DMA of
            // this iteration writes was last read in an earlier iteration (the
            // previous end barrier retired those reads), and slice t+1 is
            // waited for right before this iteration's barrier.  All fragment
            // reads are issued up front; the first half's MFMAs wait only for
            // their own reads (the compiler counts lgkmcnt), the second half's
            // A reads stay in flight beneath them.
            // (64-deep full tiles: no room for both A halves, the second is
            // read after the first half's MFMAs)
            constexpr int KS1 = KS == 1 ? 1 : 0;
            vec8_t<T> af1[KS1 ? KS : 1][4];
            read_a(0);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) bq[ks][ni] = frag(Bs, ROWBB, boff[ni], ks);
            if constexpr (KS1) {
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) af1[0][mi] = frag(As, ROWB, aoff[1][mi], 0);
            }
            if constexpr (BST == 3) {
                if (it + 2 < nk) issue_b(bbuf == 0 ? 2 : bbuf - 1);
            } else {
                if (it + 1 < nk) issue_b(bbuf ^ 1);
            }
            const bool more = it + 2 < nk;
            if (more) issue_a(abuf == 0 ? 2 : abuf - 1);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[mi][ni] = mfma_v8<T>(af[ks][mi], bq[ks][ni], acc[mi][ni]);
            if constexpr (!KS1) read_a(1);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        acc[4 + mi][ni] = mfma_v8<T>(KS1 ? af1[0][mi] : af[ks][mi], bq[ks][ni], acc[4 + mi][ni]);
            __builtin_amdgcn_s_setprio(0);
            if (more) wait_vmcnt<BST == 3 ? A_INS + B_INS : A_INS>();
            else wait_vmcnt<0>();
            lds_barrier();
            abuf = abuf == 2 ? 0 : abuf + 1;
            bbuf = bbuf == BST - 1 ? 0 : bbuf + 1;
            continue;
        }
        read_a(0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) bq[ks][ni] = frag(Bs, ROWBB, boff[ni], ks);
        if constexpr (BST == 3) {
            if (ABL != 1 && it + 2 < nk) issue_b(bbuf == 0 ? 2 : bbuf - 1);
        } else {
            if (ABL != 1 && it + 1 < nk) issue_b(bbuf ^ 1);
        }
        __builtin_amdgcn_s_barrier();
        if (ABL != 2) mma(0);
        else asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(af[0][0]), "v"(af[KS - 1][3]), "v"(bq[0][0]), "v"(bq[KS - 1][3]) : "memory");
        __builtin_amdgcn_s_barrier();
        read_a(1);
        const int anext = abuf == 0 ? 2 : abuf - 1;
        const bool more = ABL != 1 && it + 2 < nk;
        if (more) issue_a(anext);
        // the wait sits right before the iteration's last barrier (a full
        // iteration after the slice's issue)
        __builtin_amdgcn_s_barrier();
        if (ABL != 2) mma(1);
        else asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(af[0][0]), "v"(af[KS - 1][3]) : "memory");
        // newest: B(t+2) (3-stage B ring) and A(t+2); A(t+1), B(t+1) landed
        if (more) wait_vmcnt<BST == 3 ? A_INS + B_INS : A_INS>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        abuf = abuf == 2 ? 0 : abuf + 1;
        bbuf = bbuf == BST - 1 ? 0 : bbuf + 1;
    }
    if (ABL == 3) {   // every accumulator feeds the (never taken) store: no MFMA is dead code
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        if (sum == 12345.f) p.out[tid] = sum;
        return;
    }

    if constexpr (ADAM) {
        // ---- fused Adam epilogue, per wave in four 32-row quarters (waves
        // work independently: no block barrier after the first): the fp32
        // gradient rows go through the wave's LDS slice so each lane owns 8
        // consecutive columns (n) of a row (tap, c); all p/m/v loads of a
        // quarter are in flight before the update; the transposed (KRSC) copy
        // is re-staged as bf16 [n][32 rows] and stored as 16-byte runs along c.
        // (A block-wide variant with 1 KiB row runs measured slower: the
        // epilogue is latency-, not DRAM-page-bound.)
        constexpr int QR = 32, SROWF = WTN * 4 + 16, SROWT = QR * 2 + 16;
        constexpr int WB = QR * SROWF + WTN * SROWT;
        static_assert(NW * WB <= SMEM, "fused epilogue staging must fit");
        const auto& A = p.adam;
#ifdef SEG_DIAG
        const int abl = A.abl;     // ablation bits (garbage results): diagnostic build only
#else
        constexpr int abl = 0;
#endif
        if (abl & 16) {
            if (acc[0][0][0] == 12345.f && acc[7][3][3] == 54321.f) p.out[tid] = acc[3][1][2];
            return;
        }
        const int fr = lane & 15;
        const int cch = lane & 7, esub = lane >> 3;          // 8 lanes x 8 columns per row, 8 rows per pass
        const int col0 = n0 + wn * WTN + cch * 8;
        char* fbuf = smem + w * WB;
        char* tbuf = fbuf + QR * SROWF;
        lds_barrier();                                       // ring buffers are dead for every wave
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni)
                        *reinterpret_cast<float*>(fbuf + (mi * 16 + fg * 4 + r) * SROWF + (ni * 16 + fr) * 4) =
                            acc[q * 2 + mi][ni][r];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            float pv[4][8], mv[4][8], vv[4][8];
            long eo[4];
            bool ok[4];
            int tp[4], cc[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int rr = esub + 8 * i;
                const int m = m0 + wm * WTM + q * QR + rr;
                tp[i] = m / p.Cg;
                cc[i] = m - tp[i] * p.Cg;
                ok[i] = m < p.M && cc[i] < p.c_valid && col0 + 8 <= p.n_valid;
                eo[i] = (long)tp[i] * p.o_tap + (long)cc[i] * p.o_c + col0;
                if (ok[i] && (abl & 1)) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) pv[i][j] = mv[i][j] = vv[i][j] = 0.f;
                } else if (ok[i]) {
                    *reinterpret_cast<float4*>(pv[i]) = *reinterpret_cast<const float4*>(A.p + eo[i]);
                    *reinterpret_cast<float4*>(pv[i] + 4) = *reinterpret_cast<const float4*>(A.p + eo[i] + 4);
                    *reinterpret_cast<float4*>(mv[i]) = *reinterpret_cast<const float4*>(A.m + eo[i]);
                    *reinterpret_cast<float4*>(mv[i] + 4) = *reinterpret_cast<const float4*>(A.m + eo[i] + 4);
                    *reinterpret_cast<float4*>(vv[i]) = *reinterpret_cast<const float4*>(A.v + eo[i]);
                    *reinterpret_cast<float4*>(vv[i] + 4) = *reinterpret_cast<const float4*>(A.v + eo[i] + 4);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int rr = esub + 8 * i;
                const float4 g0 = *reinterpret_cast<const float4*>(fbuf + rr * SROWF + cch * 32);
                const float4 g1 = *reinterpret_cast<const float4*>(fbuf + rr * SROWF + cch * 32 + 16);
                const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
                float np[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if (ok[i]) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float gc = gg[j] * A.gs;
                        const float mj = A.b1 * mv[i][j] + (1.f - A.b1) * gc;
                        const float vj = A.b2 * vv[i][j] + (1.f - A.b2) * gc * gc;
                        np[j] = pv[i][j] - A.lr_t * mj / (sqrtf(vj) + A.eps);
                        mv[i][j] = mj;
                        vv[i][j] = vj;
                    }
                    if (!(abl & 2)) {
                        *reinterpret_cast<float4*>(A.p + eo[i]) = *reinterpret_cast<const float4*>(np);
                        *reinterpret_cast<float4*>(A.p + eo[i] + 4) = *reinterpret_cast<const float4*>(np + 4);
                        *reinterpret_cast<float4*>(A.m + eo[i]) = *reinterpret_cast<const float4*>(mv[i]);
                        *reinterpret_cast<float4*>(A.m + eo[i] + 4) = *reinterpret_cast<const float4*>(mv[i] + 4);
                        *reinterpret_cast<float4*>(A.v + eo[i]) = *reinterpret_cast<const float4*>(vv[i]);
                        *reinterpret_cast<float4*>(A.v + eo[i] + 4) = *reinterpret_cast<const float4*>(vv[i] + 4);
                    }
                    if (A.store_grad) {
                        *reinterpret_cast<float4*>(p.out + eo[i]) = g0;
                        *reinterpret_cast<float4*>(p.out + eo[i] + 4) = g1;
                    }
                    if (A.rows && !(abl & 4))
                        *reinterpret_cast<uint4*>(reinterpret_cast<bf16*>(A.rows) +
                                                  ((long)tp[i] * A.rows_ap + cc[i]) * A.rows_bp + col0) = Chunk<bf16>::pack(np);
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    *reinterpret_cast<bf16*>(tbuf + (cch * 8 + j) * SROWT + rr * 2) = (bf16)np[j];
            }
            if (A.tr && !(abl & 8)) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const int n = n0 + wn * WTN + lane;              // one transposed row per lane
#pragma unroll
                for (int k = 0; k < QR / 8; ++k) {
                    const int m = m0 + wm * WTM + q * QR + 8 * k;
                    const int tap = m / p.Cg, c = m - (m / p.Cg) * p.Cg;
                    if (m >= p.M || n >= p.n_valid || c >= p.c_valid) continue;
                    const uint4 v8 = *reinterpret_cast<const uint4*>(tbuf + lane * SROWT + k * 16);
                    bf16* dst = reinterpret_cast<bf16*>(A.tr) + ((long)n * A.RS + tap) * A.tr_ap + c;
                    if (c + 8 <= p.c_valid && ((((uintptr_t)dst) & 15) == 0)) {
                        *reinterpret_cast<uint4*>(dst) = v8;
                    } else {
                        const bf16* h = reinterpret_cast<const bf16*>(&v8);
                        for (int j = 0; j < 8 && c + j < p.c_valid; ++j) dst[j] = h[j];
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tbuf / fbuf reads done before the next quarter
        }
        return;
    }
    // ---- epilogue: two 64-row halves per wave staged in LDS, then each lane
    // stores 8 consecutive columns of a row (filter gradient or split slab)
    constexpr int SROW = WTN * 4 + 16;
    constexpr int ECPR = WTN / 8, RPP = 64 / ECPR;
    const int fr = lane & 15;
    const int cch = lane % ECPR, esub = lane / ECPR;
    const int col0 = n0 + wn * WTN + cch * 8;
    char* wbuf = smem + w * 64 * SROW;
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
        lds_barrier();
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                        acc[mh * 4 + mi][ni][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 2
        for (int rr = esub; rr < 64; rr += RPP) {
            const int m = m0 + wm * WTM + mh * 64 + rr;
            if (m >= p.M || col0 >= p.N) continue;
            const float4 lo = *reinterpret_cast<const float4*>(wbuf + rr * SROW + cch * 32);
            const float4 hi = *reinterpret_cast<const float4*>(wbuf + rr * SROW + cch * 32 + 16);
            if (p.partial) {
                float* dst = p.partial + ((long)split * p.Mp + m) * p.N + col0;
                *reinterpret_cast<float4*>(dst) = lo;
                *reinterpret_cast<float4*>(dst + 4) = hi;
                continue;
            }
            const int tap = m / p.Cg;
            const int c = m - tap * p.Cg;
            if (c >= p.c_valid) continue;
            float* orow = p.out + (long)tap * p.o_tap + (long)c * p.o_c;
            const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            if (p.o_n == 1 && col0 + 8 <= p.n_valid && ((((uintptr_t)(orow + col0)) & 15) == 0)) {
                *reinterpret_cast<float4*>(orow + col0) = lo;
                *reinterpret_cast<float4*>(orow + col0 + 4) = hi;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (col0 + j < p.n_valid) orow[(long)(col0 + j) * p.o_n] = v[j];
            }
        }
    }
}

bool tn3_ok(const TNParams& p, int dtype) { return tn3_applies(p.M, p.N, dtype); }

void tn3_info(int M, int N, int P, int cus, int* splits) {
    const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
    const int kt = (P + 63) / 64;
    *splits = one_round_splits(tiles, cus, std::min(64, std::max(1, kt / 6)));
}

void launch_tn3(TNParams& p, int splits, hipStream_t s, int dtype) {
    const int tm = (p.M + 255) / 256;
    if (dtype == SEG_F16) {   // half storage: plain filter gradients only (loss scaling keeps Adam separate)
        if (splits == 1 && (g_tn3_half & 2)) {
            const int tn = (p.N + 127) / 128;
            hipLaunchKernelGGL((igemm_tn3<0, false, false, 128, 32, f16>), dim3(tm * tn), dim3(256), 0, s, p, tm, tn, 1);
            return;
        }
        const int tn = (p.N + 255) / 256;
        hipLaunchKernelGGL((igemm_tn3<0, false, false, 256, 64, f16>), dim3(tm * tn * splits), dim3(512), 0, s, p, tm,
                           tn, splits);
        return;
    }
    const bool multi_round = (long)tm * ((p.N + 255) / 256) > device_cus();
    if (splits == 1 && !g_tn3_abl && (g_tn3_half & (p.adam.p ? 1 : 2)) && (multi_round || !p.adam.p || (g_tn3_half & 4))) {
        // 256 x 128 tiles, two blocks per CU
        const int tn = (p.N + 127) / 128;
        const dim3 g(tm * tn), b(256);
        const bool mfast = g_tn3_mfast && tm > tn;
        if (p.adam.p && g_tn3_stagger_us > 0 && tm * tn > 4 * device_cus()) {
            static int* slots = nullptr;
            if (!slots) (void)hipGetSymbolAddress((void**)&slots, HIP_SYMBOL(g_tn3_cu_slots));
            (void)hipMemsetAsync(slots, 0, sizeof(int) * 4096, s);
            p.adam.cu_slots = slots;
            p.adam.stagger = g_tn3_stagger_us * 100;
            p.adam.first_round = 2 * device_cus();
        } else {
            p.adam.stagger = 0;
        }
#define TN3H(MF, AD) hipLaunchKernelGGL((igemm_tn3<0, MF, AD, 128, 32>), g, b, 0, s, p, tm, tn, 1)
        if (p.adam.p) {
            if (mfast) TN3H(true, true);
            else TN3H(false, true);
        } else {
            if (mfast) TN3H(true, false);
            else TN3H(false, false);
        }
#undef TN3H
        return;
    }
    const int tn = (p.N + 255) / 256;
    const dim3 g(tm * tn * splits), b(512);
    const bool mfast = g_tn3_mfast && tm > tn;
#define TN3(A, MF) hipLaunchKernelGGL((igemm_tn3<A, MF>), g, b, 0, s, p, tm, tn, splits)
#ifdef SEG_DIAG   // ablation builds (garbage results): tools/ only
    switch (g_tn3_abl) {
        case 1: TN3(1, false); return;
        case 2: TN3(2, false); return;
        case 3: TN3(3, false); return;
    }
#endif
    if (p.adam.p) {
        if (mfast) hipLaunchKernelGGL((igemm_tn3<0, true, true>), g, b, 0, s, p, tm, tn, splits);
        else hipLaunchKernelGGL((igemm_tn3<0, false, true>), g, b, 0, s, p, tm, tn, splits);
        return;
    }
    if (mfast) TN3(0, true);
    else TN3(0, false);
#undef TN3
}

// the fused-Adam epilogue needs the whole reduction in one tile (no split-K
// slabs), vector-aligned rows (o_n = 1, n_valid % 8 == 0) and 8-aligned taps
bool tn3_adam_ok(const TNParams& p, int dtype) {
    if (!tn3_ok(p, dtype) || p.o_n != 1 || (p.n_valid & 7) || (p.Cg & 7) || (p.o_c & 7) || (p.o_tap & 7)) return false;
    int sp;
    tn3_info(p.M, p.N, p.P, device_cus(), &sp);
    return sp == 1;
}

}  // namespace seg
