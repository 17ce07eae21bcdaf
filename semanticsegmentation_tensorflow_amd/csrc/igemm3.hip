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
//  * the upper M wave group runs one barrier behind (STAG), so on every SIMD
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

int g_nt3 = 1;
__device__ uint4 g_nt3_zero[4];

template <bool STAG>
__global__ __launch_bounds__(512) void igemm_nt3(NTParams p) {
    using T = bf16;
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
    if (STAG && wm == 1) __builtin_amdgcn_s_barrier();

    const int fr = lane & 15, fg = lane >> 4;
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
                        acc[mh * 4 + mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8, af[ks][mi]), __builtin_bit_cast(bf16x8, bq[ks][ni]),
                            acc[mh * 4 + mi][ni], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        };
        // h0: A half 0 + B slice; B(t+1) into the other B buffer (last read at h0(t-1))
        read_a(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int row = wn * WTN + ni * 16 + fr;
                bq[ks][ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * ((ks * 4 + fg) ^ ((row >> 1) & 7)));
            }
        if (it + 1 < nk) issue_b(bbuf ^ 1);
        __builtin_amdgcn_s_barrier();
        mma(0);
        __builtin_amdgcn_s_barrier();
        // h1: A half 1; A(t+2) into the A buffer of t-1 (last read at h1(t-1));
        // then A(t+1) and B(t+1) must have landed before the next h0
        read_a(1);
        const int anext = abuf == 0 ? 2 : abuf - 1;   // (abuf + 2) % 3
        if (it + 2 < nk) {
            issue_a(anext);
            wait_vmcnt<A_INS>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        mma(1);
        __builtin_amdgcn_s_barrier();
        abuf = abuf == 2 ? 0 : abuf + 1;
        bbuf ^= 1;
    }
    if (STAG && wm == 0) __builtin_amdgcn_s_barrier();

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
        for (int rr = rsub; rr < 64; rr += RPP) {
            const int row = m0 + wm * WTM + mh * 64 + rr;
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
                if (e.keep_prob < 1.f) x = (x / e.keep_prob) * floorf(e.keep_prob + seg_uniform(e.seed, gidx + col));
                if (e.residual) x += res[j];
                if (e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                v[j] = col < e.n_valid ? x : 0.f;
            }
            T* yp = reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0;
            *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
        }
    }
}

// 256 x 256 tiles, one block per CU: split K until the grid covers the CUs
// (keeping >= 6 K tiles per split), never past 64 slabs.
void nt3_info(int M, int N, int K, int cus, int* splits) {
    const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
    const int kt = (K + 63) / 64;
    int s = 1;
    if (tiles < cus) {
        s = (int)((cus + tiles - 1) / tiles);
        s = std::min(s, std::max(1, kt / 6));
        s = std::min(s, 64);
    }
    *splits = s;
}

bool nt3_ok(const NTParams& p, int dtype) {
    return g_nt3 && dtype == SEG_BF16 && p.N > 128;
}

void launch_nt3(NTParams& p, int gridz, int max_m, hipStream_t s) {
    const int tiles = ((max_m + 255) / 256) * ((p.N + 255) / 256);
    hipLaunchKernelGGL((igemm_nt3<true>), dim3(tiles, 1, gridz), dim3(512), 0, s, p);
}

}  // namespace seg
