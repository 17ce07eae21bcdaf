// Fourth-generation implicit-GEMM NT kernel for gfx950: 256 x 256 tiles with
// FOUR waves of 128 x 128 (one wave per SIMD).
//
// Same contract as igemm_nt3 (NTParams, igemm.h; bf16).  What changes is the
// wave tile: igemm_nt3's eight 128 x 64 waves read 384 LDS bytes per MFMA
// (12 fragments per 32 MFMAs); a 128 x 128 wave reads 256 (16 per 64), so the
// LDS port that bounds the 8-wave kernels carries a third less per FLOP.  The
// price is 256 accumulator registers per wave (AGPRs) and one wave per SIMD,
// so the latency hiding the 8-wave kernels get from a second wave comes from
// inside the wave instead:
//  * K stages of 32 (one MFMA k-step): A and B each 256 rows x 64 B per
//    stage, a 4-deep LDS-DMA ring (4 x 32 KiB = 128 KiB);
//  * iteration j: one barrier (after this wave's counted vmcnt for stage j+1),
//    then the DMA of stage j+3 into the buffer of stage j-1, then the 16
//    fragment reads of stage j+1 into the idle register set while the 64
//    MFMAs of stage j run from the other -- reads and MFMAs of one wave
//    overlap, and every DMA has two iterations to land;
//  * 64-byte LDS rows, chunk XOR (row >> 1) & 2: conflict-free ds_read_b128
//    lane groups (gfx950 b128 groups {0-3,12-15,20-27}, ...);
//  * gather / zero page / split-K / conv2d_transpose phases / epilogue as
//    igemm_nt3 (epilogue staged through LDS in four 32-row passes).
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

int g_nt4 = 0;
int g_nt4_abl = 0;   // diagnostics (garbage results): 1 = no DMA in the main loop
__device__ uint4 g_nt4_zero[4];

__global__ __launch_bounds__(256) void igemm_nt4(NTParams p, int abl) {
    using T = bf16;
    constexpr int NW = 4, BM = 256, BN = 256, BK = 32, NST = 5;
    constexpr int ROWB = 64, STG = BM * ROWB;                 // 16 KiB per operand per stage
    constexpr int INS = BM * ROWB / 1024 / NW;                // 4 DMA pieces per wave per operand
    constexpr int TM = 8, TN = 8;                             // 128 x 128 per wave
    __shared__ __attribute__((aligned(16))) char smem[2 * NST * STG];

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
    if (tiles_mg <= 16 && tiles_n > tiles_mg) {
        tn = wg / tiles_mg;
        tm = wg - tn * tiles_mg;
    } else {
        // groups of 8 M tiles walked M-fastest: the 32 blocks an XCD runs at
        // once share 8 A and 4 B k-slices in its L2
        constexpr int GM = 8;
        const int grp = wg / (GM * tiles_n);
        const int gm = min(GM, tiles_mg - grp * GM);
        const int r = wg - grp * GM * tiles_n;
        tm = grp * GM + r % gm;
        tn = r / gm;
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
    const int wm = w >> 1, wn = w & 1;
    // DMA piece i of wave w: rows (i*NW + w)*16 + lr, lr = lane >> 2; the
    // lane's physical chunk (lane & 3) holds global chunk c (row-swizzled)
    const int lr = lane >> 2;
    const int c = (lane & 3) ^ ((lr >> 1) & 2);

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)g_nt4_zero;

    // per-piece base pointers and pixel coordinates (C % 32 == 0: a 32-deep
    // stage never crosses a tap, so the k state is wave-uniform)
    const T* a_base[INS];
    int a_ih[INS], a_iw[INS];
    bool a_ok[INS];
    const int hw = Ha * Wa;
#pragma unroll
    for (int i = 0; i < INS; ++i) {
        const int m = m0 + (i * NW + w) * 16 + lr;
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int img = mm / hw;
        const int rem = mm - img * hw;
        const int a = rem / Wa;
        const int b = rem - a * Wa;
        a_base[i] = X + (long)img * p.x_img + c * 8;
        a_ih[i] = a * p.ish + ioh;
        a_iw[i] = b * p.isw + iow;
    }
    const T* b_base[INS];
    bool b_ok[INS];
#pragma unroll
    for (int i = 0; i < INS; ++i) {
        const int n = n0 + (i * NW + w) * 16 + lr;
        b_ok[i] = n < p.N;
        b_base[i] = Wt + (long)(b_ok[i] ? n : 0) * p.w_col + c * 8;
    }
    // wave-uniform k state of the next stage to issue
    int k_kg = kt_begin * BK;
    int k_tap = k_kg / p.C;
    int k_cc = k_kg - k_tap * p.C;
    int k_tj = k_tap / p.taps_w, k_ti = k_tap - (k_tap / p.taps_w) * p.taps_w;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + NST * STG;
    // DMA piece q of a stage (q < INS: A rows, else B rows) into ring slot
    // `buf`; branch-free so the pieces can sit between MFMAs
    auto issue_piece = [&](int buf, int q) {
        const bool kok = k_kg < p.K;
        if (q < INS) {
            const int i = q;
            const int ih = a_ih[i] + k_tj * p.tsh, iw = a_iw[i] + k_ti * p.tsw;
            const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const T* ptr = a_base[i] + ((ih * p.IW + iw) * p.ldx + k_cc);
            glds16(ok ? (const void*)ptr : zero, lds0 + buf * STG + (i * NW + w) * 1024);
        } else {
            const int i = q - INS;
            const long wtap = (long)((rb + p.rstep * k_tj) * p.Sfull + (sb + p.sstep * k_ti)) * p.w_tap + k_cc;
            const bool ok = b_ok[i] && kok;
            glds16(ok ? (const void*)(b_base[i] + wtap) : zero, ldsB + buf * STG + (i * NW + w) * 1024);
        }
    };
    auto kstep = [&]() {
        k_kg += BK;
        k_cc += BK;
        const bool wrap = k_cc >= p.C;
        k_cc = wrap ? k_cc - p.C : k_cc;
        const int ti = k_ti + (wrap ? 1 : 0);
        const bool wrap2 = ti == p.taps_w;
        k_ti = wrap2 ? 0 : ti;
        k_tj += wrap2 ? 1 : 0;
    };
    auto issue = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 2 * INS; ++q) issue_piece(buf, q);
        kstep();
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // fragment reads: row r = base + fr, 16 bytes at chunk fg ^ swz(r)
    const int fr = lane & 15, fg = lane >> 4;
    const unsigned foff = fr * ROWB + 16 * (fg ^ ((fr >> 1) & 2));   // base rows are multiples of 16
    // two register sets, selected at compile time (the loop is unrolled by 2)
    uint4 ra0[TM], rb0[TN], ra1[TM], rb1[TN];
    auto read_stage = [&](int buf, uint4* ra, uint4* rb) {
        const char* As = smem + buf * STG + wm * 128 * ROWB + foff;
        const char* Bs = smem + NST * STG + buf * STG + wn * 128 * ROWB + foff;
#pragma unroll
        for (int i = 0; i < TM; ++i) ra[i] = *reinterpret_cast<const uint4*>(As + i * 16 * ROWB);
#pragma unroll
        for (int j = 0; j < TN; ++j) rb[j] = *reinterpret_cast<const uint4*>(Bs + j * 16 * ROWB);
    };

    // prologue: stages 0..2 in flight, stage 0 landed, its fragments in set 0
    constexpr int PER = 2 * INS;   // DMA instructions per stage per wave
    // (stages past the end are zero-page stages into free slots, so every
    // vmcnt count below is uniform)
    for (int s = 0; s < NST - 1; ++s) issue(s);
    wait_vmcnt<3 * PER>();
    lds_barrier();
    if (nk > 0) read_stage(0, ra0, rb0);

    // iteration j: stage j+1 must have landed (stage j+2 may be in flight);
    // the barrier also retires every wave's reads of stage j-1, whose ring
    // slot the DMA of stage j+3 then reuses; stage j+1's fragments are read
    // into the other register set while stage j's MFMAs run
    auto step = [&](int j, uint4* ca, uint4* cb, uint4* na, uint4* nb) {
        wait_vmcnt<2 * PER>();    // stages j+2, j+3 may still be in flight
        __builtin_amdgcn_s_barrier();
        const int slot4 = (j + 4) % NST;   // stage j+4 goes where stage j-1 was
        // fragment reads of stage j+1 (a harmless re-read of stage j on the
        // last iteration) interleaved with stage j's MFMAs: 2 ds_read_b128
        // per 8 MFMAs keeps lgkmcnt within its 4-bit range and the LDS port
        // busy under the MFMA pipe
        const int nbuf = (j + 1 < nk ? j + 1 : j) % NST;
        const char* As = smem + nbuf * STG + wm * 128 * ROWB + foff;
        const char* Bs = smem + NST * STG + nbuf * STG + wn * 128 * ROWB + foff;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            na[i] = *reinterpret_cast<const uint4*>(As + i * 16 * ROWB);
            nb[i] = *reinterpret_cast<const uint4*>(Bs + i * 16 * ROWB);
#pragma unroll
            for (int jj = 0; jj < TN; ++jj)
                acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, ca[i]),
                                                                     __builtin_bit_cast(bf16x8, cb[jj]), acc[i][jj],
                                                                     0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, 8, 0);
            if (!abl) issue_piece(slot4, i);
        }
        kstep();
        __builtin_amdgcn_s_setprio(0);
    };
    for (int j = 0; j < nk; j += 2) {
        step(j, ra0, rb0, ra1, rb1);
        if (j + 1 < nk) step(j + 1, ra1, rb1, ra0, rb0);
    }
    wait_vmcnt<0>();          // trailing zero-page stages land before LDS is reused
    __builtin_amdgcn_s_barrier();

    if (p.partial) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * 128 + mi * 16 + fg * 4 + r;
                if (row >= M) continue;
                float* prow = p.partial + ((long)blockIdx.z * M + row) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col = n0 + wn * 128 + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
            }
        return;
    }
    // ---- epilogue in four 32-row passes per wave (LDS holds 4 x 32 x 128 fp32)
    constexpr int WTN = 128, SROW = WTN * 4 + 16;
    constexpr int CPR = WTN / 8, RPP = 64 / CPR;   // 16 lanes per row, 4 rows per pass
    static_assert(NW * 32 * SROW <= 2 * NST * STG, "epilogue staging must fit");
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
    char* wbuf = smem + w * 32 * SROW;
#pragma unroll
    for (int mq = 0; mq < 4; ++mq) {
        lds_barrier();
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                        acc[mq * 2 + mi][ni][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 2
        for (int rr = rsub; rr < 32; rr += RPP) {
            const int row = m0 + wm * 128 + mq * 32 + rr;
            if (row >= M || col0 >= p.N) continue;
            const int img = row / hw;
            const int rem = row - img * hw;
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
            }
            if (e.residual) {
                const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            }
            const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                float x = v[j] * scl[j] + shf[j] + bias[j];
                if (e.relu) x = fmaxf(x, 0.f);
                if (e.keep_prob < 1.f) x = seg_dropout(x, e.keep_prob, e.seed, gidx + col);
                if (e.residual) x += res[j];
                if (e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                v[j] = col < e.n_valid ? x : 0.f;
            }
            T* yp = reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0;
            *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
        }
    }
}

bool nt4_ok(const NTParams& p, int dtype) { return g_nt4 && dtype == SEG_BF16 && p.N > 128 && p.C % 32 == 0; }

// same split rule as igemm_nt3 with 32-deep K tiles (>= 12 per split)
void nt4_info(int M, int N, int K, int cus, int* splits) {
    const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
    const int kt = (K + 31) / 32;
    int s = 1;
    if (tiles < cus) {
        s = (int)((cus + tiles - 1) / tiles);
        s = std::min(s, std::max(1, kt / 12));
        s = std::min(s, 64);
    }
    *splits = s;
}

void launch_nt4(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + 255) / 256) * ((p.N + 255) / 256);
    hipLaunchKernelGGL(igemm_nt4, dim3(tiles, 1, gridz), dim3(256), 0, s, p, g_nt4_abl);
}

}  // namespace seg
