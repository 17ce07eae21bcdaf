// conv_halo4: the 256 x 256 halo-tiled 3x3 conv (Conv2D forward and
// Conv2DBackpropInput, stride 1) at ONE wave per SIMD.
//
// conv_halo2 (halo.hip) runs 8 waves of 128 px x 64 ch in two wave groups
// that trade MFMA and LDS phases between four barriers per (tap, 64-channel)
// step: every phase ends when its slowest wave does, and a third of the wave
// cycles were parked at those barriers.  Here 4 waves (one per SIMD) each own
// a 128 px x 128 ch quadrant -- 64 accumulators = 256 AGPRs -- and the
// step has ONE barrier.  The step's fragments are software-pipelined by half
// a step:
//
//   after barrier s:   MFMA  ks1 of slice s-1   (fragments already in VGPRs)
//                        + ds_read ks0 of slice s, filter DMA of slice s+1
//                      MFMA  ks0 of slice s
//                        + ds_read ks1 of slice s, halo DMA of the next chunk
//                      lgkmcnt(0), vmcnt(own slice s+1 pieces), barrier s+1
//
// so every LDS read has half a step (64 MFMAs) to land and no MFMA waits for
// one, and the filter slice issued right after the barrier has the whole
// step.  The accumulation order per output element is conv_halo2's ((chunk,
// tap) outer, ks inner), so the two kernels agree bit for bit.
//
// LDS: two halo buffers of 44 pieces x 8 rows (352 rows of 128 B: (BH+2) x
// (BW+2) = 324 / 340 for BW = 16 / 32) + two 32 KiB filter slices = 152 KiB;
// the next chunk's halo pieces are issued two per tap over taps 0-5 of the
// current chunk into the idle buffer.  Fragment reads use conv_halo2's
// swizzle (chunk XOR row & 6), applied on the DMA source side.
//
// Epilogue as conv_halo2: LDS-staged 16-byte stores with bias / BN affine /
// ReLU / dropout / residual / ReluGrad mask, the fused MaxPool (pooled map +
// switches) or MaxPoolGrad (unpool routing), or fp32 split-K slabs.
//
// Reference layers: Network/model/FCN.py:55-99 (conv3_1 ... conv5_3), the
// input gradients TF derives for them, FC-DenseNet / DeepLab 3x3 convs with
// > 128 output channels.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"
#include "halo.h"

namespace seg {

static __device__ uint4 h4_zero_page[4];


// Geometry per wave count: NW = 4 (one wave per SIMD, 128 px x 128 ch per
// wave) or NW = 8 (two waves per SIMD, 128 px x 64 ch: one wave's DMA /
// LDS-read issue runs beside the other's MFMAs).  HP halo pieces of 8 rows
// per wave: the halo buffer holds HP * NW * 8 rows (>= 340).
template <int NW> struct H4Geo {
    static constexpr int WN = NW / 2;                 // waves along N (2 along M)
    static constexpr int WTN = 256 / WN;              // columns per wave
    static constexpr int NF = WTN / 16;               // n-fragments per wave
    static constexpr int HP = NW == 4 ? 11 : 6;       // halo pieces per wave
    static constexpr int HPT = NW == 4 ? 2 : 1;       // halo pieces per tap (taps 0-5)
    static constexpr int HBUF = HP * NW * 1024;
    static constexpr int BBUF = 256 * 128;            // 256 filter rows x 64 channels
    static constexpr int SMEM = 2 * HBUF + 2 * BBUF;  // 152 / 160 KiB
    static constexpr int B_INS = 256 / 8 / NW;        // filter pieces per wave per slice
    static_assert(HP * NW * 8 >= 340 && HPT * 6 >= HP, "halo pieces");
    static_assert(SMEM <= 160 * 1024, "LDS");
};

// ABL (diagnostic builds, garbage results; tools/kbench.py --opts nt2_ablate=1N):
// 1 no barrier in the loop, 2 no end-of-step waits, 3 no DMA in the loop,
// 4 no fragment reads, 5 no MFMA, 6 no barrier and no waits.
// (Measured within noise and removed in round 6: the second wave of each
// SIMD issuing its DMA in other MFMA groups than the first, s_setprio around
// each MFMA group, fragment reads placed between the MFMAs of a group; the
// same tile on 32x32x16 MFMAs -- 4.6 % fewer wave cycles but a 3 % lower
// clock, 2-5 % slower per launch.)
template <int BW, int NW, typename T = bf16, bool UNP = false, int ABL = 0>
__global__ __launch_bounds__(NW * 64) void conv_halo4(NTParams p, HaloGeom g) {
    using G = H4Geo<NW>;
    constexpr int BM = 256, BN = 256, BH = BM / BW;
    constexpr int WN = G::WN, WTN = G::WTN, NF = G::NF, B_INS = G::B_INS;
    constexpr int HWD = BW + 2, HROWS = HWD * (BH + 2);   // 3x3 stride-1 halo: 324 / 340 rows
    static_assert(HROWS <= G::HP * NW * 8, "halo fits the LDS buffer");
    static_assert(BW % 16 == 0 && BM % BW == 0, "fragments are 16 px of one tile row");
    __shared__ __attribute__((aligned(16))) char smem[G::SMEM];

    const int tiles_n = (p.N + BN - 1) / BN;
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int tsp = wg / tiles_n, tn = wg - (wg / tiles_n) * tiles_n;
    const int tpi = g.tiles_x * g.tiles_y;
    const int img = tsp / tpi;
    if (img >= g.nimg) return;
    const int trem = tsp - img * tpi;
    const int ty = trem / g.tiles_x, tx = trem - (trem / g.tiles_x) * g.tiles_x;
    const int oy0 = ty * BH, ox0 = tx * BW, n0 = tn * BN;
    int kc_begin = 0, kc_end = g.nchunks;
    if (p.partial) {
        kc_begin = blockIdx.z * g.kc_per_split;
        kc_end = min(g.nchunks, kc_begin + g.kc_per_split);
    }
    const int iters = (kc_end - kc_begin) * 9;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w % WN;
    const int lr = lane >> 3;
    const int c = (lane & 7) ^ (lr & 6);   // filter rows: source chunk of this lane's 16 LDS bytes

    const T* __restrict__ Xi = reinterpret_cast<const T*>(p.x) + (long)img * p.x_img;
    const seg_i32x4 rs_x = make_rsrc(Xi, 0x80000000u);
    const seg_i32x4 rs_w = make_rsrc(p.w, 0x80000000u);
    constexpr unsigned OOB = 0x80000000u;   // reads as zero (>= num_records)

    // halo piece h of this wave: rows (h * NW + w) * 8 + lr of the (BH+2) x
    // HWD halo; LDS row hr keeps its 8 chunks XOR-swizzled by (hx & 6) (the
    // halo COLUMN: a tap shift moves every fragment row by the same column
    // offset, so the swizzle of all 8 m-fragments follows from the tap alone),
    // i.e. LDS slot q holds source chunk q ^ (hx & 6).  Byte offset in the
    // image (the host checks 2 IH IW ldx < 2^31); out-of-image rows OOB.
    // Computed per issue (HWD is a compile-time divisor): no register array
    // indexed by a runtime piece number.
    const int hoy = oy0 + p.ioh + g.hy0, hox = ox0 + p.iow + g.hx0;
    auto halo_v = [&](int h) -> unsigned {
        const int hr = (h * NW + w) * 8 + lr;
        const int hy = hr / HWD, hx = hr - (hr / HWD) * HWD;
        const int ih = hoy + hy, iw = hox + hx;
        const bool ok = hr < HROWS && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
        const int cs = (lane & 7) ^ (hx & 6);
        return ok ? (unsigned)(((ih * p.IW + iw) * p.ldx + cs * 8) * 2) : OOB;
    };
    constexpr int H_N_MAX = (HROWS + NW * 8 - 1) / (NW * 8);
    static_assert(H_N_MAX <= G::HP, "halo pieces");
    const int h_n = HROWS > w * 8 ? min(H_N_MAX, (HROWS - w * 8 + NW * 8 - 1) / (NW * 8)) : 0;
    // filter piece i of this wave: rows (i * NW + w) * 8 + lr of the 256-row
    // slice, chunks swizzled by (row & 6); rows past N OOB
    unsigned bv[B_INS];
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
        const int n = n0 + (i * NW + w) * 8 + lr;
        bv[i] = n < p.N ? (unsigned)((n * (int)p.w_col + c * 8) * 2) : OOB;
    }
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + 2 * G::HBUF;

    auto load_halo = [&](int h, int kc, int buf) {
        bglds16(rs_x, halo_v(h), (unsigned)kc * 128u, lds0 + buf * G::HBUF + (h * NW + w) * 1024);
    };
    // filter slice cursor (chunk, tap row, tap col) of the next slice to issue;
    // byte offset ((rb + rstep j) Sfull + sb + sstep i) w_tap + 64 kc elements
    int b_kc = kc_begin, b_j = 0, b_i = 0;
    auto slice_off = [&]() -> unsigned {
        return (unsigned)((((p.rb + p.rstep * b_j) * p.Sfull + (p.sb + p.sstep * b_i)) * (int)p.w_tap + b_kc * 64) * 2);
    };
    auto b_advance = [&]() {
        if (++b_i == 3) {
            b_i = 0;
            if (++b_j == 3) { b_j = 0; ++b_kc; }
        }
    };

    f32x4 acc[8][NF];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: the first chunk's halo and slice 0
    if (iters > 0) {
#pragma unroll
        for (int h = 0; h < H_N_MAX; ++h)
            if (h < h_n) load_halo(h, kc_begin, 0);
        const unsigned so = slice_off();
        const unsigned bdst = ldsB + (unsigned)(w * 1024);
#pragma unroll
        for (int i = 0; i < B_INS; ++i) bglds16(rs_w, bv[i], so, bdst + i * NW * 1024);
        b_advance();
    }
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();

    const int fr = lane & 15, fg = lane >> 4;
    // A fragment mi: halo rows rowbase(mi) + toff(tap) .. + 15 (lane fr);
    // rowbase(mi) - rowbase(0) is a compile-time byte offset (ds_read immediate)
    constexpr int TR0 = 128 / BW;   // tile rows per wave half
    const int arow0 = ((wm * TR0) * HWD + fr) * 128;
    auto a_imm = [](int mi) constexpr -> int { return (((mi * 16) / BW) * HWD + (mi * 16) % BW) * 128; };
    // B fragment ni: row wn*WTN + ni*16 + fr, 16-B chunk (ks*4 + fg) ^ (fr & 6);
    // ks = 1 flips bit 6 of the chunk offset
    const unsigned vbase = 2 * G::HBUF + (wn * WTN + fr) * 128 + 16 * (fg ^ (fr & 6));

    uint4 a0[8], b0[NF], a1[8], b1[NF];
    int t_j = 0, t_i = 0, tap = 0, kc = kc_begin, hbuf = 0, bbuf = 0;

    // fragment read at byte offset off + imm of the block's LDS
    auto rd = [&](unsigned off, int imm) -> uint4 {
        if constexpr (ABL == 4) {
            uint4 u;
            asm volatile("" : "=v"(u.x), "=v"(u.y), "=v"(u.z), "=v"(u.w));
            return u;
        }
        return *reinterpret_cast<const uint4*>(smem + off + imm);
    };
    auto mma = [&](const uint4& a, const uint4& b, f32x4& cc) __attribute__((always_inline)) {
        if constexpr (ABL == 5) asm volatile("" ::"v"(a.x), "v"(b.x));
        else cc = mfma16x16x32<T>(a, b, cc);
    };
    // the fragment reads of one k-step half: NF B fragments (the next half's
    // first MFMA group needs them all) then the 8 A fragments in the order the
    // next half consumes them, spread over the 8 MFMA groups
    constexpr int NR = NF + 8;
    auto reads = [&](auto q_tag, uint4* aa, uint4* bb, unsigned va, unsigned vb) __attribute__((always_inline)) {
        constexpr int Q = decltype(q_tag)::value;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            if (k * 8 / NR != Q) continue;
            if (k < NF) bb[k] = rd(vb, k * 2048);
            else aa[k - NF] = rd(va, a_imm(k - NF));
        }
    };
    // one (tap, chunk) step; FIRST: no ks1 of a previous slice to finish
    auto step = [&](auto first_tag) __attribute__((always_inline)) {
        constexpr bool FIRST = decltype(first_tag)::value;
        const bool next_ok = b_kc < kc_end;   // a slice s+1 exists
        // past the last slice: a harmless re-read of the chunk's first slice
        const unsigned so = next_ok ? slice_off() : (unsigned)((p.rb * p.Sfull + p.sb) * (int)p.w_tap * 2);
        // this step's A base: tap shift (dy, dx) and the column swizzle of dx
        const int dx = t_i * p.tsw - g.hx0;
        const int toff = (t_j * p.tsh - g.hy0) * HWD + dx;
        const unsigned va0 = (unsigned)(arow0 + toff * 128 + hbuf * G::HBUF) + 16u * (unsigned)(fg ^ ((fr + dx) & 6));
        const unsigned vb0 = vbase + (unsigned)(bbuf * G::BBUF);
        const unsigned va1 = va0 ^ 64u, vb1 = vb0 ^ 64u;
        // half 1: MFMA ks1 of the previous slice.  Beside it: the filter DMA
        // of slice s+1 (groups 0-3: the slice has the rest of the step to
        // land), then this slice's ks0 fragments.
        const unsigned bdst = ldsB + (unsigned)((bbuf ^ 1) * G::BBUF + w * 1024);
        auto issue_b = [&](auto q_tag) __attribute__((always_inline)) {
            constexpr int Q = decltype(q_tag)::value;
            constexpr int PER = B_INS / 4;    // pieces per group, groups 0-3
            bglds16_at<(Q * PER) * NW * 1024>(rs_w, bv[Q * PER], so, bdst);
            if constexpr (PER >= 2) bglds16_at<(Q * PER + 1) * NW * 1024>(rs_w, bv[Q * PER + (PER >= 2)], so, bdst);
        };
        auto half1 = [&](auto q_tag) __attribute__((always_inline)) {
            constexpr int Q = decltype(q_tag)::value;
            if constexpr (!FIRST) {
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) mma(a1[Q], b1[ni], acc[Q][ni]);
            }
            __builtin_amdgcn_sched_barrier(0);
            reads(q_tag, a0, b0, va0, vb0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ABL != 3 && Q < 4) issue_b(q_tag);
            __builtin_amdgcn_sched_barrier(0);
        };
        half1(std::integral_constant<int, 0>{});
        half1(std::integral_constant<int, 1>{});
        half1(std::integral_constant<int, 2>{});
        half1(std::integral_constant<int, 3>{});
        half1(std::integral_constant<int, 4>{});
        half1(std::integral_constant<int, 5>{});
        half1(std::integral_constant<int, 6>{});
        half1(std::integral_constant<int, 7>{});
        if (next_ok) b_advance();
        // half 2: MFMA ks0 of this slice; ds_read ks1; the next chunk's halo
        // pieces HPT tap .. HPT tap + HPT - 1 (taps 0-5)
        const bool hp = kc + 1 < kc_end;
        const int h0 = G::HPT * tap;
        const int nh = hp ? max(0, min(G::HPT, h_n - h0)) : 0;
        auto half2 = [&](auto q_tag) __attribute__((always_inline)) {
            constexpr int Q = decltype(q_tag)::value;
#pragma unroll
            for (int ni = 0; ni < NF; ++ni) mma(a0[Q], b0[ni], acc[Q][ni]);
            __builtin_amdgcn_sched_barrier(0);
            reads(q_tag, a1, b1, va1, vb1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (ABL != 3 && Q >= 1 && Q <= G::HPT) {
                if (Q - 1 < nh) load_halo(h0 + Q - 1, kc + 1, hbuf ^ 1);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        half2(std::integral_constant<int, 0>{});
        half2(std::integral_constant<int, 1>{});
        half2(std::integral_constant<int, 2>{});
        half2(std::integral_constant<int, 3>{});
        half2(std::integral_constant<int, 4>{});
        half2(std::integral_constant<int, 5>{});
        half2(std::integral_constant<int, 6>{});
        half2(std::integral_constant<int, 7>{});
        // slice s+1 (issued before this step's halo pieces) must have landed;
        // at a chunk's last tap the next chunk's halo too.  Before the
        // barrier only the reads of this slice's FILTER buffer must be done
        // (the next step's DMA overwrites it): the 8 ks1 A reads of the halo
        // stay in flight into the next step's half 1 -- except at the chunk's
        // last tap, whose halo buffer the next chunk's DMA refills.
        const bool last_tap = t_i == 2 && t_j == 2;
        if constexpr (ABL != 2 && ABL != 6) {
            if (last_tap || nh == 0) wait_vmcnt<0>();
            else if (nh == 1) wait_vmcnt<1>();
            else wait_vmcnt<2>();
            if (last_tap) wait_lgkmcnt<0>();
            else wait_lgkmcnt<8>();
        }
        if constexpr (ABL != 1 && ABL != 6) __builtin_amdgcn_s_barrier();
        bbuf ^= 1;
        ++tap;
        if (++t_i == 3) {
            t_i = 0;
            if (++t_j == 3) {
                t_j = 0;
                tap = 0;
                ++kc;
                hbuf ^= 1;
            }
        }
    };
    if (iters > 0) {
        step(std::true_type{});
        for (int it = 1; it < iters; ++it) step(std::false_type{});
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int ni = 0; ni < NF; ++ni) acc[q][ni] = mfma16x16x32<T>(a1[q], b1[ni], acc[q][ni]);
    }

    if (p.partial) {
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ml = wm * 128 + mi * 16 + fg * 4 + r;
                const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
                if (oy >= p.Ha || ox >= p.Wa) continue;
                const long m = ((long)img * p.Ha + oy) * p.Wa + ox;
                float* prow = p.partial + ((long)blockIdx.z * p.M + m) * p.N;
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) {
                    const int col = n0 + wn * WTN + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
            }
        return;
    }
    // ---- epilogue in two 64-row halves per wave (LDS: NW x 64 rows x WTN fp32)
    constexpr int SROW = WTN * 4 + 16;
    constexpr int CPR = WTN / 8, RPP = 64 / CPR, NRR = 64 / RPP;
    static_assert(NW * 64 * SROW <= G::SMEM, "epilogue staging must fit");
    const int cch = lane % CPR, rsub = lane / CPR;
    const int col0 = n0 + wn * WTN + cch * 8;
    const EpiParams& e = p.epi;
    char* wbuf = smem + w * 64 * SROW;
    // stage rows mh * 64 .. + 63 of this wave's tile (compile-time mh: acc
    // stays in registers)
    auto stage = [&](auto mh_tag) __attribute__((always_inline)) {
        constexpr int mh = decltype(mh_tag)::value;
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ni = 0; ni < NF; ++ni)
                    *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                        acc[mh * 4 + mi][ni][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    if (!UNP && e.pool_y) {     // MaxPool fused: pooled map + switches, 64 columns per call
        auto pool_half = [&](auto mh_tag) __attribute__((always_inline)) {
            constexpr int mh = decltype(mh_tag)::value;
            stage(mh_tag);
#pragma unroll
            for (int ch = 0; ch < WTN / 64; ++ch) {
                const int pc0 = n0 + wn * WTN + ch * 64 + (lane & 7) * 8;
                float pb[8], ps[8], pf[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool cv = pc0 + j < e.n_valid;
                    pb[j] = (e.bias && cv) ? e.bias[pc0 + j] : 0.f;
                    ps[j] = (e.scale && cv) ? e.scale[pc0 + j] : 1.f;
                    pf[j] = (e.shift && cv) ? e.shift[pc0 + j] : 0.f;
                }
                pool_epi_rows<T, BW, 64>(p, wbuf + ch * 256 + (lane & 7) * 32, SROW, wm * 128 + mh * 64, oy0, ox0,
                                         img, pc0, lane, pb, ps, pf);
            }
        };
        pool_half(std::integral_constant<int, 0>{});
        pool_half(std::integral_constant<int, 1>{});
        return;
    }
    float bias[8], scl[8], shf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        const bool cv = col < e.n_valid;
        bias[j] = (e.bias && cv) ? e.bias[col] : 0.f;
        scl[j] = (e.scale && cv) ? e.scale[col] : 1.f;
        shf[j] = (e.shift && cv) ? e.shift[col] : 0.f;
    }
    // ReluGrad mask rows: the first half's requested before its staging, the
    // second half's row by row as the first half's are consumed
    uint4 mkv[NRR];
    auto load_mask = [&](int mh, int k) {
        const int ml = wm * 128 + mh * 64 + rsub + k * RPP;
        const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
        mkv[k] = uint4{0u, 0u, 0u, 0u};
        if (oy < p.Ha && ox < p.Wa && col0 < p.N)
            mkv[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(e.mask) + img * e.mask_img +
                                                     halo_opix(p, oy, ox) * e.ld_mask + col0);
    };
    if (!UNP && e.mask) {
#pragma unroll
        for (int k = 0; k < NRR; ++k) load_mask(0, k);
    }
    auto epi_half = [&](auto mh_tag) __attribute__((always_inline)) {
        constexpr int mh = decltype(mh_tag)::value;
        stage(mh_tag);
#pragma unroll
        for (int k = 0; k < NRR; ++k) {
            const int rr = rsub + k * RPP;
            const int ml = wm * 128 + mh * 64 + rr;
            const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
            float mk[8];
            if (!UNP && e.mask) {
                Chunk<T>::unpack(mkv[k], mk);
                if (mh == 0) load_mask(1, k);
            }
            if (oy >= p.Ha || ox >= p.Wa || col0 >= p.N) continue;
            const long pix = halo_opix(p, oy, ox);
            float v[8];
            splitk_lds8(wbuf + rr * SROW + cch * 32, v);
            float res[8];
            if (e.residual) {
                const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            }
            const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
            const SegDropRun<8> drop(e.seed, gidx + col0, !UNP && e.keep_prob < 1.f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                float x = v[j] * scl[j] + shf[j] + bias[j];
                if (e.relu) x = fmaxf(x, 0.f);
                if (!UNP && e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                if (e.residual) x += res[j];
                if (!UNP && e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                v[j] = col < e.n_valid ? x : 0.f;
            }
            if constexpr (UNP) {     // MaxPoolGrad fused: the pooled gradient is not written
                unpool_store8<T>(e, img, p.OH, p.OW, oy, ox, col0, v);
                continue;
            }
            T* yp = reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0;
            *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
        }
    };
    epi_half(std::integral_constant<int, 0>{});
    epi_half(std::integral_constant<int, 1>{});
}

// The plan hp (a 256-wide halo2 plan) runs on conv_halo4: 3 x 3 taps at
// unit spacing (halo (BH + 2) x (BW + 2)), byte offsets < 2^31.
bool halo4_ok(const NTParams& p, const HaloPlan& hp) {
    if (!g_halo4 || hp.bn != 256 || (hp.bw != 16 && hp.bw != 32)) return false;
    return hp.geom[0] == 3 && p.taps_w == 3 && (p.tsh == 1 || p.tsh == -1) && (p.tsw == 1 || p.tsw == -1) &&
           hp.geom[4] == hp.bw + 2 && 2L * ((long)p.IH * p.IW * p.ldx + 64L * hp.geom[8]) < (1L << 31) &&
           2L * ((long)p.N * p.w_col + 9L * p.w_tap + 64L * hp.geom[8]) < (1L << 31) && p.rb >= 0 && p.sb >= 0;
}

template <int NW>
static void launch_halo4_t(NTParams& p, const HaloPlan& hp, const HaloGeom& g, hipStream_t s, int dtype) {
    const dim3 grid((unsigned)hp.tiles, 1, hp.splits), block(NW * 64);
#ifdef SEG_DIAG   // ablation builds (garbage results): tools/ only
    if (g_nt2_ablate > 10 && hp.bw == 16 && dtype == SEG_BF16 && !p.epi.unpool_y) {
        switch (g_nt2_ablate - 10) {
            case 1: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 1>), grid, block, 0, s, p, g); return;
            case 2: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 2>), grid, block, 0, s, p, g); return;
            case 3: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 3>), grid, block, 0, s, p, g); return;
            case 4: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 4>), grid, block, 0, s, p, g); return;
            case 5: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 5>), grid, block, 0, s, p, g); return;
            case 6: hipLaunchKernelGGL((conv_halo4<16, NW, bf16, false, 6>), grid, block, 0, s, p, g); return;
        }
    }
#endif
    if (p.epi.unpool_y) {
        if (dtype == SEG_F16) hipLaunchKernelGGL((conv_halo4<16, NW, f16, true>), grid, block, 0, s, p, g);
        else hipLaunchKernelGGL((conv_halo4<16, NW, bf16, true>), grid, block, 0, s, p, g);
        return;
    }
    if (dtype == SEG_F16) {
        if (hp.bw == 16) hipLaunchKernelGGL((conv_halo4<16, NW, f16>), grid, block, 0, s, p, g);
        else hipLaunchKernelGGL((conv_halo4<32, NW, f16>), grid, block, 0, s, p, g);
    } else {
        if (hp.bw == 16) hipLaunchKernelGGL((conv_halo4<16, NW, bf16>), grid, block, 0, s, p, g);
        else hipLaunchKernelGGL((conv_halo4<32, NW, bf16>), grid, block, 0, s, p, g);
    }
}

void launch_halo4(NTParams& p, const HaloPlan& hp, const HaloGeom& g, hipStream_t s, int dtype) {
    if (g_halo4 >= 2) launch_halo4_t<8>(p, hp, g, s, dtype);
    else launch_halo4_t<4>(p, hp, g, s, dtype);
}

}  // namespace seg
