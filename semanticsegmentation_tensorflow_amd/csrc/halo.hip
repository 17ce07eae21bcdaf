// Halo-tiled direct convolution for stride-1 convs (bf16, gfx950).
//
// The implicit-GEMM NT kernel (igemm2.hip) re-gathers every input pixel once
// per filter tap: for a 3x3 conv each activation byte crosses L2 -> LDS nine
// times, and ablation shows that DMA stream (not the MFMA) bounds it.  Here a
// block owns a BH x BW tile of output pixels (256 px) x BN output channels and,
// per 64-channel chunk, stages the tile's input HALO
// ((BH + (taps_h-1)|tsh|) x (BW + (taps_w-1)|tsw|) pixels x 128 B) in LDS once;
// all taps of that chunk read their A fragments from the halo at a per-tap row
// offset.  Only the filter slice (BN x 128 B) is streamed per tap.
//
//  * k order: channel chunk outer, tap inner (iteration = (chunk, tap)).
//  * filter slices: 3-deep LDS ring, slice it+2 in flight while it is consumed.
//  * halos: double buffered; halo chunk c+1 is staged one 8-row-per-wave piece
//    per tap iteration of chunk c (pieces h < HI, HI <= taps-1), so every
//    iteration issues at most B_INS + 1 DMA instructions per wave and one
//    counted `s_waitcnt vmcnt` + barrier per iteration suffices.
//  * A fragment = 16 consecutive output px of one tile row = 16 consecutive
//    halo rows starting at ANY row (taps shift it): the chunk XOR (row & 6)
//    keeps every ds_read_b128 lane group (gfx950: lanes {0-3,12-15,20-27},
//    ...) on 16 distinct 16-byte slots for every start row -- the
//    (row >> 1) & 7 XOR is 2-way conflicted whenever start row % 4 != 0.
//  * output: same LDS-staged 16-byte epilogue as igemm_nt2 (bias / BN-affine /
//    ReLU / dropout / residual), or fp32 split-K slabs over channel chunks.
//
// Covers Conv2D fwd and Conv2DBackpropInput of stride-1 convs (dilation any)
// with C % 64 == 0 -- conv1_2 ... conv5_3 of FCN (Network/model/FCN.py:55-99)
// and the FC-DenseNet 3x3 layers.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"
#include "halo.h"

namespace seg {

static __device__ uint4 halo_zero_page[4];

// 64-wide blocks on the two-group ping-pong conv_res64pp: 0 never, 1 for the
// pooled forward and the ReluGrad-masked input gradient (conv1_2: 191 vs 192
// and 259 vs 277 us; the plain forward measured 214 vs 202 on it), 2 always



// value of lane ^ 1 (DPP quad_perm [1, 0, 3, 2]: no LDS crossbar traffic)
__device__ __forceinline__ float dpp_swap1(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}


template <int BW, int HI, int BN, typename T = bf16>
__global__ __launch_bounds__(512) void conv_halo(NTParams p, HaloGeom g) {
    constexpr int NW = 8, WM = 4, WN = 2, BM = 256, BH = BM / BW;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int B_INS = BN / 8 / NW;
    constexpr int HBUF = HI * NW * 1024;
    constexpr int BSTAGE = BN * 128;
    constexpr int SMEM = 2 * HBUF + 3 * BSTAGE;
    static_assert(BW % 16 == 0 && BM % BW == 0, "fragments are 16 px of one tile row");
    static_assert(B_INS >= 1 && B_INS <= 2, "wait counts below assume B_INS + 1 <= 3");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

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
    const int ntaps = g.taps_h * p.taps_w;
    const int iters = (kc_end - kc_begin) * ntaps;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const int lr = lane >> 3;
    // physical 16-byte chunk (lane & 7) of LDS row (q*8 + lr) holds global
    // chunk c; the swizzle row & 6 depends on lr only.
    const int c = (lane & 7) ^ (lr & 6);   // halo row (h*NW + w)*8 + lr: swizzle row & 6

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)halo_zero_page;

    // ---- halo rows this lane stages: row (h*NW + w)*8 + lr, h < h_n
    long h_off[HI];
    const long xbase = (long)img * p.x_img + c * 8;
#pragma unroll
    for (int h = 0; h < HI; ++h) {
        const int hr = (h * NW + w) * 8 + lr;
        const int hy = hr / g.hwd, hx = hr - (hr / g.hwd) * g.hwd;
        const int ih = oy0 + p.ioh + g.hy0 + hy, iw = ox0 + p.iow + g.hx0 + hx;
        const bool ok = hr < g.hrows && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
        h_off[h] = ok ? xbase + ((long)ih * p.IW + iw) * p.ldx : -1;
    }
    // wave-uniform: instructions whose 8 rows start below hrows
    const int h_n = g.hrows > w * 8 ? min(HI, (g.hrows - w * 8 + NW * 8 - 1) / (NW * 8)) : 0;

    long b_off[B_INS];
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
        const int n = n0 + (i * NW + w) * 8 + lr;
        b_off[i] = n < p.N ? (long)n * p.w_col + c * 8 : -1;
    }

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + 2 * HBUF;

    auto load_halo = [&](int h, int kc, int buf) {
        const void* src = h_off[h] >= 0 ? (const void*)(X + h_off[h] + kc * 64) : zero;
        glds16(src, lds0 + buf * HBUF + (h * NW + w) * 1024);
    };
    // B issue cursor (chunk, tap j/i)
    int b_kc = kc_begin, b_j = 0, b_i = 0;
    auto issue_b = [&](int stage) {
        const long wtap = (long)((p.rb + p.rstep * b_j) * p.Sfull + (p.sb + p.sstep * b_i)) * p.w_tap + b_kc * 64;
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const void* src = b_off[i] >= 0 ? (const void*)(Wt + b_off[i] + wtap) : zero;
            glds16(src, ldsB + stage * BSTAGE + (i * NW + w) * 1024);
        }
        if (++b_i == p.taps_w) {
            b_i = 0;
            if (++b_j == g.taps_h) { b_j = 0; ++b_kc; }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (iters > 0) {
        for (int h = 0; h < h_n; ++h) load_halo(h, kc_begin, 0);
        issue_b(0);
    }
    if (iters > 1) issue_b(1);
    int last = iters > 1 ? B_INS : 0;   // DMA instructions of the newest batch

    const int fr = lane & 15, fg = lane >> 4;
    int rowbase[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int ml = wm * WTM + mi * 16;
        rowbase[mi] = (ml / BW) * g.hwd + (ml % BW) + fr;
    }
    int t_j = 0, t_i = 0, kc = kc_begin, stage = 0, hbuf = 0, tap = 0;
    for (int it = 0; it < iters; ++it) {
        // everything but the newest batch (slice it+1, next-halo piece) landed
        if (last == 0) wait_vmcnt<0>();
        else if (last == 1) wait_vmcnt<1>();
        else if (last == 2) wait_vmcnt<2>();
        else wait_vmcnt<3>();
        lds_barrier();
        int issued = 0;
        if (it + 2 < iters) {
            issue_b(stage == 0 ? 2 : stage - 1);
            issued = B_INS;
        }
        if (tap < h_n && kc + 1 < kc_end) {
            load_halo(tap, kc + 1, hbuf ^ 1);
            ++issued;
        }
        last = issued;

        const char* Hs = smem + hbuf * HBUF;
        const char* Bs = smem + 2 * HBUF + stage * BSTAGE;
        const int toff = (t_j * p.tsh - g.hy0) * g.hwd + t_i * p.tsw - g.hx0;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            uint4 af[TM], bfr[TN];
            const int chunk = ks * 4 + fg;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int row = rowbase[mi] + toff;
                af[mi] = *reinterpret_cast<const uint4*>(Hs + row * 128 + 16 * (chunk ^ (row & 6)));
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int row = wn * WTN + ni * 16 + fr;
                bfr[ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * (chunk ^ (row & 6)));
            }
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    acc[mi][ni] = mfma16x16x32<T>(af[mi], bfr[ni], acc[mi][ni]);
        }
        stage = stage == 2 ? 0 : stage + 1;
        ++tap;
        if (++t_i == p.taps_w) {
            t_i = 0;
            if (++t_j == g.taps_h) {
                t_j = 0;
                tap = 0;
                ++kc;
                hbuf ^= 1;
            }
        }
    }

    if (p.partial) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ml = wm * WTM + mi * 16 + fg * 4 + r;
                const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
                if (oy >= p.Ha || ox >= p.Wa) continue;
                const long m = ((long)img * p.Ha + oy) * p.Wa + ox;
                float* prow = p.partial + ((long)blockIdx.z * p.M + m) * p.N;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col = n0 + wn * WTN + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
            }
        return;
    }
    // ---- epilogue: wave tile -> LDS (fp32), then 8 columns x one row per lane
    constexpr int SROW = WTN * 4 + 16;
    static_assert(NW * WTM * SROW <= SMEM, "epilogue staging must fit");
    constexpr int CPR = WTN / 8;
    constexpr int RPP = 64 / CPR, NRR = WTM / RPP;
    const int cch = lane % CPR, rsub = lane / CPR;
    const int col0 = n0 + wn * WTN + cch * 8;
    const EpiParams& e = p.epi;
    // 16-bit ReluGrad mask rows of this lane, requested before the staging
    uint4 mkv[NRR];
    if constexpr (sizeof(T) == 2) {
        if (e.mask) {
#pragma unroll
            for (int k = 0; k < NRR; ++k) {
                const int ml = wm * WTM + rsub + k * RPP;
                const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
                mkv[k] = uint4{0u, 0u, 0u, 0u};
                if (oy < p.Ha && ox < p.Wa && col0 < p.N)
                    mkv[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(e.mask) + img * e.mask_img +
                                                             halo_opix(p, oy, ox) * e.ld_mask + col0);
            }
        }
    }
    lds_barrier();
    char* wbuf = smem + w * WTM * SROW;
    {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                        acc[mi][ni][r];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float bias[8], scl[8], shf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        const bool cv = col < e.n_valid;
        bias[j] = (e.bias && cv) ? e.bias[col] : 0.f;
        scl[j] = (e.scale && cv) ? e.scale[col] : 1.f;
        shf[j] = (e.shift && cv) ? e.shift[col] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NRR; ++k) {
        const int rr = rsub + k * RPP;
        const int ml = wm * WTM + rr;
        const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
        if (oy >= p.Ha || ox >= p.Wa || col0 >= p.N) continue;
        const long pix = halo_opix(p, oy, ox);
        float v[8];
        splitk_lds8(wbuf + rr * SROW + cch * 32, v);
        float res[8], mk[8];
        if (e.mask) {
            if constexpr (sizeof(T) == 2) {
                Chunk<T>::unpack(mkv[k], mk);
            } else {
                const T* mp = reinterpret_cast<const T*>(e.mask) + img * e.mask_img + pix * e.ld_mask + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp), mk);
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(mp + 4), mk + 4);
            }
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
        *reinterpret_cast<uint4*>(yp) = Chunk<T>::pack(v);
    }
}


// ---------------------------------------------------------------------------
// Two blocks per CU (N <= 128): conv_halo's tile and fragment layout with ONE
// halo buffer and a 2-stage filter ring (BN = 128: 48 + 32 KiB; BN = 64: 48 +
// 16 KiB) and the epilogue staged in two 32-row halves, so two blocks share a
// CU (<= 128 VGPRs: 4 waves per SIMD).  One block's pipeline bubbles -- the
// halo of each channel chunk is loaded after the previous chunk's last tap and
// waited for before its first; the filter slice of iteration it+1 is in flight
// during iteration it only -- are the other block's MFMA time.  On conv2_x of
// FCN (C = 64 / 128: one or two chunks per tile, 1872 tiles) conv_halo left
// each block ~80 % of its time waiting on a single in-order pipeline.
// No split-K (the host uses it only for splits == 1).
// UNP: the MaxPoolGrad epilogue (EpiParams::unpool_y), no ReluGrad mask /
// dropout paths (its own instantiation: the 128-VGPR budget of two blocks
// per CU has no room for both).
template <int BW, int HI, int BN, typename T = bf16, bool UNP = false>
__global__ __launch_bounds__(512, 4) void conv_halo_duo(NTParams p, HaloGeom g) {
    constexpr int NW = 8, WM = 4, WN = 2, BM = 256, BH = BM / BW;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int B_INS = BN / 8 / NW;
    constexpr int HBUF = HI * NW * 1024;
    constexpr int BSTAGE = BN * 128;
    constexpr int SMEM = HBUF + 2 * BSTAGE;
    static_assert(BW % 16 == 0 && BM % BW == 0, "fragments are 16 px of one tile row");
    static_assert(SMEM <= 80 * 1024, "two blocks per CU");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

    const int tiles_n = (p.N + BN - 1) / BN;
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int tsp = wg / tiles_n, tn = wg - (wg / tiles_n) * tiles_n;
    const int tpi = g.tiles_x * g.tiles_y;
    const int img = tsp / tpi;
    if (img >= g.nimg) return;
    const int trem = tsp - img * tpi;
    const int ty = trem / g.tiles_x, tx = trem - (trem / g.tiles_x) * g.tiles_x;
    const int oy0 = ty * BH, ox0 = tx * BW, n0 = tn * BN;
    const int ntaps = g.taps_h * p.taps_w;
    const int iters = g.nchunks * ntaps;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const int lr = lane >> 3;
    const int c = (lane & 7) ^ (lr & 6);   // halo row (h*NW + w)*8 + lr: swizzle row & 6

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)halo_zero_page;

    // 32-bit element offsets within the (block-uniform) image: fits 128 VGPRs
    const T* __restrict__ Ximg = X + (long)img * p.x_img;
    int h_off[HI];
#pragma unroll
    for (int h = 0; h < HI; ++h) {
        const int hr = (h * NW + w) * 8 + lr;
        const int hy = hr / g.hwd, hx = hr - (hr / g.hwd) * g.hwd;
        const int ih = oy0 + p.ioh + g.hy0 + hy, iw = ox0 + p.iow + g.hx0 + hx;
        const bool ok = hr < g.hrows && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
        h_off[h] = ok ? (ih * p.IW + iw) * p.ldx + c * 8 : -1;
    }
    const int h_n = g.hrows > w * 8 ? min(HI, (g.hrows - w * 8 + NW * 8 - 1) / (NW * 8)) : 0;
    int b_off[B_INS];
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
        const int n = n0 + (i * NW + w) * 8 + lr;
        b_off[i] = n < p.N ? n * (int)p.w_col + c * 8 : -1;
    }
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + HBUF;
    auto load_halo = [&](int kc) {
        for (int h = 0; h < h_n; ++h) {
            const void* src = h_off[h] >= 0 ? (const void*)(Ximg + h_off[h] + kc * 64) : zero;
            glds16(src, lds0 + (h * NW + w) * 1024);
        }
    };
    int b_kc = 0, b_j = 0, b_i = 0;
    auto issue_b = [&](int stage) {
        const long wtap = (long)((p.rb + p.rstep * b_j) * p.Sfull + (p.sb + p.sstep * b_i)) * p.w_tap + b_kc * 64;
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const void* src = b_off[i] >= 0 ? (const void*)(Wt + b_off[i] + wtap) : zero;
            glds16(src, ldsB + stage * BSTAGE + (i * NW + w) * 1024);
        }
        if (++b_i == p.taps_w) {
            b_i = 0;
            if (++b_j == g.taps_h) { b_j = 0; ++b_kc; }
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (iters > 0) {
        load_halo(0);
        issue_b(0);
    }
    const int fr = lane & 15, fg = lane >> 4;
    int rowbase[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int ml = wm * WTM + mi * 16;
        rowbase[mi] = (ml / BW) * g.hwd + (ml % BW) + fr;
    }
    int t_j = 0, t_i = 0, kc = 0, stage = 0;
    for (int it = 0; it < iters; ++it) {
        wait_vmcnt<0>();            // slice it (and, at it = 0, the first halo) landed
        lds_barrier();              // ... for every wave; slice it-1 / the old halo are dead
        if (it > 0 && t_j == 0 && t_i == 0) {
            // first tap of chunk kc: its halo replaces the previous chunk's
            load_halo(kc);
            if (it + 1 < iters) issue_b(stage ^ 1);
            if (it + 1 < iters) wait_vmcnt<B_INS>();
            else wait_vmcnt<0>();
            lds_barrier();
        } else if (it + 1 < iters) {
            issue_b(stage ^ 1);
        }
        const char* Bs = smem + HBUF + stage * BSTAGE;
        const int toff = (t_j * p.tsh - g.hy0) * g.hwd + t_i * p.tsw - g.hx0;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            uint4 af[TM], bfr[TN];
            const int chunk = ks * 4 + fg;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int row = rowbase[mi] + toff;
                af[mi] = *reinterpret_cast<const uint4*>(smem + row * 128 + 16 * (chunk ^ (row & 6)));
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int row = wn * WTN + ni * 16 + fr;
                bfr[ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * (chunk ^ (row & 6)));
            }
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    acc[mi][ni] = mfma16x16x32<T>(af[mi], bfr[ni], acc[mi][ni]);
        }
        stage ^= 1;
        if (++t_i == p.taps_w) {
            t_i = 0;
            if (++t_j == g.taps_h) {
                t_j = 0;
                ++kc;
            }
        }
    }

    // ---- epilogue in two 32-row halves per wave: wave tile -> LDS (fp32),
    // then 8 columns x one row per lane (conv_halo's arithmetic)
    constexpr int SROW = WTN * 4 + 16, HR = WTM / 2;
    static_assert(NW * HR * SROW <= SMEM, "epilogue staging must fit");
    constexpr int CPR = WTN / 8;
    constexpr int RPP = 64 / CPR, NRH = HR / RPP;
    const int cch = lane % CPR, rsub = lane / CPR;
    const int col0 = n0 + wn * WTN + cch * 8;
    const EpiParams& e = p.epi;
    float bias[8];     // BN scale / shift (rare here) are read per row: 128 VGPRs
#pragma unroll
    for (int j = 0; j < 8; ++j) bias[j] = (e.bias && col0 + j < e.n_valid) ? e.bias[col0 + j] : 0.f;
    char* wbuf = smem + w * HR * SROW;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        uint4 mkv[NRH];          // ReluGrad mask rows of this half, requested before the staging
        if (!UNP && e.mask) {
#pragma unroll
            for (int k = 0; k < NRH; ++k) {
                const int ml = wm * WTM + hh * HR + rsub + k * RPP;
                const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
                mkv[k] = uint4{0u, 0u, 0u, 0u};
                if (oy < p.Ha && ox < p.Wa && col0 < p.N)
                    mkv[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(e.mask) + img * e.mask_img +
                                                             halo_opix(p, oy, ox) * e.ld_mask + col0);
            }
        }
        lds_barrier();
#pragma unroll
        for (int mi = 0; mi < TM / 2; ++mi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)
                    *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                        acc[hh * (TM / 2) + mi][ni][r];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (BW == 16 && HR == 32 && CPR == 8) {
            if (!UNP && e.pool_y) {      // MaxPool fused (bias + ReLU only: no scale / shift here)
                const float one[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
                const float nil[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                pool_epi_rows<T, BW, HR>(p, wbuf + cch * 32, SROW, wm * WTM + hh * HR, oy0, ox0, img, col0, lane,
                                         bias, one, nil);
                continue;
            }
        }
#pragma unroll
        for (int k = 0; k < NRH; ++k) {
            const int rr = rsub + k * RPP;
            const int ml = wm * WTM + hh * HR + rr;
            const int oy = oy0 + ml / BW, ox = ox0 + ml % BW;
            if (oy >= p.Ha || ox >= p.Wa || col0 >= p.N) continue;
            const long pix = halo_opix(p, oy, ox);
            float v[8];
            splitk_lds8(wbuf + rr * SROW + cch * 32, v);
            float res[8], mk[8];
            if (!UNP && e.mask) Chunk<T>::unpack(mkv[k], mk);
            if (e.residual) {
                const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
                Chunk<T>::unpack(*reinterpret_cast<const uint4*>(rp), res);
            }
            const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
            const SegDropRun<8> drop(e.seed, gidx + col0, !UNP && e.keep_prob < 1.f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                const bool cv = col < e.n_valid;
                const float sc = (e.scale && cv) ? e.scale[col] : 1.f, sh = (e.shift && cv) ? e.shift[col] : 0.f;
                float x = v[j] * sc + sh + bias[j];
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
    }
}

// ---------------------------------------------------------------------------
// 256 x 256 variant (N > 128): 8 waves as 2 (M) x 4 (N), 128 x 64 per wave.
// Each (chunk, tap) iteration is two phases of 32 MFMAs between barriers:
//   h0: A rows of the wave's first M half + the WHOLE filter slice into
//       registers, barrier, 32 MFMAs, barrier;
//   h1: A rows of the second half, the next chunk's halo piece (taps < h_n),
//       filter slice it+2 into the buffer slice it just left, barrier, 32
//       MFMAs, barrier.
// The upper M wave group runs one barrier behind (waves w and w+4 share a
// SIMD, so one wave's MFMA cluster overlaps the other's LDS reads).  Slice
// it+2's DMA is issued after both groups' h0 reads of slice it retired (the
// lagging group's at the barrier after its h0 MFMAs): the leading group
// issues it after its h1 pre-MFMA barrier, the lagging group before it, and
// each waits for everything but those pieces before the barrier after which
// the leading group reads slice it+1 -- five barrier intervals of DMA
// latency per slice.  LDS: 2 halo buffers + 2 filter slices (160 KiB).
// ABL (diagnostic builds, garbage results): 1 = no DMA in the loop, 2 = no
// MFMA, 3 = no LDS fragment reads, 4 = no halo DMA in the loop, 5 = no filter
// DMA in the loop, 7 = every DMA piece reads the zero page (same
// instructions, no L2 traffic), 9 = every filter slice from the first slice's
// address (L1/L2-hot).  Measured (conv4_2 fwd, 4 x 48 x 156 x 512): 116 us;
// no DMA 99, zero page 97, hot slice 108, no filter DMA 100 -- the filter
// stream's L2 round trips, not the DMA instructions, cost the difference.
template <int BW, int ABL = 0, typename T = bf16, bool UNP = false>
__global__ __launch_bounds__(512) void conv_halo2(NTParams p, HaloGeom g) {
    constexpr int NW = 8, BM = 256, BN = 256, BH = BM / BW, HI = 6;
    constexpr int WTN = BN / 4, NFH = WTN / 32;   // per-wave columns, n-fragments per B half
    constexpr int HBUF = HI * NW * 1024;
    constexpr int BBUF = BN * 128;
    constexpr int SMEM = 2 * HBUF + 2 * BBUF;
    constexpr int B_INS = BN / 8 / NW;   // 4
    static_assert(BW % 16 == 0 && BM % BW == 0, "fragments are 16 px of one tile row");
    __shared__ __attribute__((aligned(16))) char smem[SMEM];

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
    const int ntaps = g.taps_h * p.taps_w;
    const int iters = (kc_end - kc_begin) * ntaps;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 2, wn = w & 3;
    const int lr = lane >> 3;
    const int c = (lane & 7) ^ (lr & 6);   // halo row (h*NW + w)*8 + lr: swizzle row & 6

    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)halo_zero_page;

    long h_off[HI];
    const long xbase = (long)img * p.x_img + c * 8;
#pragma unroll
    for (int h = 0; h < HI; ++h) {
        const int hr = (h * NW + w) * 8 + lr;
        const int hy = hr / g.hwd, hx = hr - (hr / g.hwd) * g.hwd;
        const int ih = oy0 + p.ioh + g.hy0 + hy, iw = ox0 + p.iow + g.hx0 + hx;
        const bool ok = hr < g.hrows && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
        h_off[h] = ok ? xbase + ((long)ih * p.IW + iw) * p.ldx : -1;
    }
    const int h_n = g.hrows > w * 8 ? min(HI, (g.hrows - w * 8 + NW * 8 - 1) / (NW * 8)) : 0;
    long b_off[B_INS];
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
        const int n = n0 + (i * NW + w) * 8 + lr;
        b_off[i] = n < p.N ? (long)n * p.w_col + c * 8 : -1;
    }
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsB = lds0 + 2 * HBUF;

    auto load_halo = [&](int h, int kc, int buf) {
        const void* src = (ABL != 7 && h_off[h] >= 0) ? (const void*)(X + h_off[h] + kc * 64) : zero;
        glds16(src, lds0 + buf * HBUF + (h * NW + w) * 1024);
    };
    int b_kc = kc_begin, b_j = 0, b_i = 0;
    auto issue_b = [&](int buf) {
        const long wtap = ABL == 9 ? 0L : (long)((p.rb + p.rstep * b_j) * p.Sfull + (p.sb + p.sstep * b_i)) * p.w_tap + b_kc * 64;
#pragma unroll
        for (int i = 0; i < B_INS; ++i) {
            const void* src = (ABL != 7 && b_off[i] >= 0) ? (const void*)(Wt + b_off[i] + wtap) : zero;
            glds16(src, ldsB + buf * BBUF + (i * NW + w) * 1024);
        }
        if (++b_i == p.taps_w) {
            b_i = 0;
            if (++b_j == g.taps_h) { b_j = 0; ++b_kc; }
        }
    };

    f32x4 acc[8][2 * NFH];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2 * NFH; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (iters > 0) {
        for (int h = 0; h < h_n; ++h) load_halo(h, kc_begin, 0);
        issue_b(0);
    }
    if (iters > 1 && ABL != 1 && ABL != 5) {   // slice 1 stays in flight
        issue_b(1);
        wait_vmcnt<B_INS>();
    } else {
        wait_vmcnt<0>();
    }
    lds_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();

    const int fr = lane & 15, fg = lane >> 4;
    int rowbase[8];
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
        const int ml = wm * 128 + mi * 16;
        rowbase[mi] = (ml / BW) * g.hwd + (ml % BW) + fr;
    }
    int t_j = 0, t_i = 0, kc = kc_begin, hbuf = 0, tap = 0, bbuf = 0;
    for (int it = 0; it < iters; ++it) {
        const char* Hs = smem + hbuf * HBUF;
        const char* Bs = smem + 2 * HBUF + bbuf * BBUF;
        const int toff = (t_j * p.tsh - g.hy0) * g.hwd + t_i * p.tsw - g.hx0;
        uint4 af[2][4], bq[2][2][NFH];   // A half [ks][mi]; B [nh][ks][ni]
        auto read_a = [&](int mh) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const int row = rowbase[mh * 4 + mi] + toff;
                    if constexpr (ABL == 3) af[ks][mi] = uint4{(unsigned)row, (unsigned)ks, 0u, (unsigned)mi};
                    else af[ks][mi] = *reinterpret_cast<const uint4*>(Hs + row * 128 + 16 * ((ks * 4 + fg) ^ (row & 6)));
                }
        };
        auto read_b = [&](int nh) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int ni = 0; ni < NFH; ++ni) {
                    const int row = wn * WTN + nh * (WTN / 2) + ni * 16 + fr;
                    if constexpr (ABL == 3) bq[nh][ks][ni] = uint4{(unsigned)row, (unsigned)it, 1u, (unsigned)ni};
                    else bq[nh][ks][ni] = *reinterpret_cast<const uint4*>(Bs + row * 128 + 16 * ((ks * 4 + fg) ^ (row & 6)));
                }
        };
        auto mma = [&](int mh, int nh) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NFH; ++ni) {
                        if constexpr (ABL == 2) {
                            asm volatile("" ::"v"(af[ks][mi].x), "v"(af[ks][mi].w), "v"(bq[nh][ks][ni].x), "v"(bq[nh][ks][ni].w));
                        } else {
                            acc[mh * 4 + mi][nh * NFH + ni] = mfma16x16x32<T>(
                                af[ks][mi], bq[nh][ks][ni], acc[mh * 4 + mi][nh * NFH + ni]);
                        }
                    }
            __builtin_amdgcn_s_setprio(0);
        };
        read_a(0);
        read_b(0);
        read_b(1);
        __builtin_amdgcn_s_barrier();
        mma(0, 0);
        mma(0, 1);
        __builtin_amdgcn_s_barrier();
        read_a(1);
        const bool hp = ABL != 1 && ABL != 4 && tap < h_n && kc + 1 < kc_end;
        const bool bp = ABL != 1 && ABL != 5 && it + 2 < iters;
        if (wm == 1 && bp) issue_b(bbuf);
        if (hp) load_halo(tap, kc + 1, hbuf ^ 1);
        if (wm == 1) {
            if (bp) {
                if (hp) wait_vmcnt<B_INS + 1>();
                else wait_vmcnt<B_INS>();
            } else {
                if (hp) wait_vmcnt<1>();
                else wait_vmcnt<0>();
            }
        }
        __builtin_amdgcn_s_barrier();
        if (wm == 0 && bp) issue_b(bbuf);
        mma(1, 1);
        mma(1, 0);
        if (wm == 0) {
            if (bp) wait_vmcnt<B_INS>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        bbuf ^= 1;
        ++tap;
        if (++t_i == p.taps_w) {
            t_i = 0;
            if (++t_j == g.taps_h) {
                t_j = 0;
                tap = 0;
                ++kc;
                hbuf ^= 1;
            }
        }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();

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
                for (int ni = 0; ni < 2 * NFH; ++ni) {
                    const int col = n0 + wn * WTN + ni * 16 + fr;
                    if (col < p.N) prow[col] = acc[mi][ni][r];
                }
            }
        return;
    }
    // ---- epilogue in two 64-row halves per wave (LDS holds 8 x 64 x WTN fp32)
    constexpr int SROW = WTN * 4 + 16;
    constexpr int CPR = WTN / 8, RPP = 64 / CPR;
    static_assert(NW * 64 * SROW <= SMEM, "epilogue staging must fit");
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
    // ReluGrad mask rows: the first half's requested before its staging, the
    // second half's row by row as the first half's are consumed
    constexpr int NRR = 64 / RPP;
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
#pragma unroll
    for (int mh = 0; mh < 2; ++mh) {
        lds_barrier();
        {
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int ni = 0; ni < 2 * NFH; ++ni)
                        *reinterpret_cast<float*>(wbuf + (mi * 16 + fg * 4 + r) * SROW + (ni * 16 + fr) * 4) =
                            acc[mh * 4 + mi][ni][r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (CPR == 8) {
            if (!UNP && e.pool_y) {      // MaxPool fused: pooled map + switches only
                pool_epi_rows<T, BW, 64>(p, wbuf + cch * 32, SROW, wm * 128 + mh * 64, oy0, ox0, img, col0, lane,
                                         bias, scl, shf);
                continue;
            }
        }
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
    }
}



// ---------------------------------------------------------------------------
// Persistent variant for a single 64-channel chunk with N <= 64 (conv1_2 fwd
// and its input gradient: 384 x 1248 px, C = K = 64).  The whole 3x3 filter
// (9 x 64 rows x 128 B = 72 KB) is loaded into LDS once per block; the block
// then walks tiles t = blockIdx.x, +gridDim.x, ...: the 8 x 32 tile's halo
// (10 x 34 px x 128 B) sits in LDS, all 9 taps run without a barrier, and the
// NEXT tile's halo is prefetched into VGPRs (6 x 16 B per thread) while the
// current one computes.  The epilogue is staged in the (dead) halo buffer.
// ---------------------------------------------------------------------------
constexpr int R64_BH = 8, R64_BW = 32, R64_HW = R64_BW + 2, R64_HROWS = (R64_BH + 2) * R64_HW;   // 340
constexpr int R64_PER = (R64_HROWS * 8 + 511) / 512;                                             // 6
constexpr int RPP_PIECES = (R64_HROWS + 7) / 8;     // halo LDS-DMA pieces of 8 rows (43: 340 rows used)

// ABL (diagnostics only, garbage results): 1 no halo fetch, 2 no MFMA,
// 3 no epilogue stores, 4 no LDS fragment reads.
// NB = output channels per block: 64, or 16 for N <= 16 (FC-DenseNet's
// growth convs, 64 -> 16): one 16-row filter fragment, all 8 waves along the
// pixels, a quarter of the MFMAs and a 18 KB filter, so two blocks share a CU.
// DMA (NB = 16): the halo comes by LDS DMA into one buffer instead of through
// 24 prefetch VGPRs per thread -- that register staging held the 16-wide
// kernel at 145 VGPRs, one block per CU; without it the kernel fits the 128
// that two resident blocks need, and the other block's MFMAs cover each
// block's DMA round trip.
template <int ABL = 0, typename T = bf16, int NB = 64, bool DMA = false>
__global__ __launch_bounds__(512, NB == 16 ? (DMA ? 4 : 2) : 1) void conv_res64(NTParams p, int tiles_x, int tiles_y,
                                                                                int ntiles) {
    static_assert(NB == 64 || NB == 16, "output block width");
    static_assert(!DMA || (NB == 16 && ABL == 0), "the DMA halo is the 16-wide form");
    constexpr int NW = 8, WN = NB == 64 ? 2 : 1, WTM = 256 / (NW / WN), WTN = NB / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int BS = 9 * NB * 128;                 // resident filter
    constexpr int HS = DMA ? RPP_PIECES * 8 * 128 : R64_HROWS * 128;   // halo (DMA: 43 whole 8-row pieces)
    __shared__ __attribute__((aligned(16))) char smem[BS + HS];
    char* Bs = smem;
    char* Hs = smem + BS;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const int fr = lane & 15, fg = lane >> 4;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const int hy0 = p.tsh < 0 ? 2 * p.tsh : 0, hx0 = p.tsw < 0 ? 2 * p.tsw : 0;
    const int tpi = tiles_x * tiles_y;

    // ---- filter: Bs[tap][n][chunk ^ swz(n)]
    for (int i = tid; i < 9 * NB * 8; i += 512) {
        const int c8 = i & 7, n = (i >> 3) % NB, tap = i / (NB * 8);
        const int j = tap / 3, ii = tap - (tap / 3) * 3;
        uint4 v = {0u, 0u, 0u, 0u};
        if (n < p.N)
            v = *reinterpret_cast<const uint4*>(Wt + (long)n * p.w_col +
                                                (long)((p.rb + p.rstep * j) * p.Sfull + (p.sb + p.sstep * ii)) * p.w_tap +
                                                c8 * 8);
        *reinterpret_cast<uint4*>(Bs + (tap * NB + n) * 128 + 16 * (c8 ^ (n & 6))) = v;
    }
    // ---- halo fetch into registers: slot q -> (row q / 8, chunk q % 8)
    uint4 hv[R64_PER];
    auto fetch = [&](int t) {
        if constexpr (ABL == 1) return;
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
        const int oy0 = ty * R64_BH, ox0 = tx * R64_BW;
#pragma unroll
        for (int k = 0; k < R64_PER; ++k) {
            const int q = tid + k * 512;
            const int hr = q >> 3, c8 = q & 7;
            uint4 v = {0u, 0u, 0u, 0u};
            if (hr < R64_HROWS) {
                const int hy = hr / R64_HW, hx = hr - (hr / R64_HW) * R64_HW;
                const int ih = oy0 + p.ioh + hy0 + hy, iw = ox0 + p.iow + hx0 + hx;
                if ((unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW)
                    v = *reinterpret_cast<const uint4*>(X + (long)img * p.x_img + ((long)ih * p.IW + iw) * p.ldx + c8 * 8);
            }
            hv[k] = v;
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int k = 0; k < R64_PER; ++k) {
            const int q = tid + k * 512;
            const int hr = q >> 3, c8 = q & 7;
            if (hr < R64_HROWS) *reinterpret_cast<uint4*>(Hs + hr * 128 + 16 * (c8 ^ (hr & 6))) = hv[k];
        }
    };
    // DMA: halo piece i = w + 8 k holds rows 8 i .. 8 i + 7; lane -> (row
    // lane >> 3, LDS chunk lane & 7) = logical chunk (lane & 7) ^ (row & 6)
    const void* zero = (const void*)halo_zero_page;
    const unsigned hbase = (unsigned)(uintptr_t)(SEG_LDS char*)smem + BS;
    auto dma = [&](int t) {
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
        const int oy0 = ty * R64_BH + p.ioh + hy0, ox0 = tx * R64_BW + p.iow + hx0;
        const int lr = lane >> 3;
        const T* xb = X + (long)img * p.x_img + ((lane & 7) ^ (lr & 6)) * 8;
#pragma unroll 1
        for (int k = 0; k < (RPP_PIECES + NW - 1) / NW; ++k) {
            const int i = w + NW * k;
            if (i < RPP_PIECES) {
                const int hr = i * 8 + lr;
                const int hy = hr / R64_HW, hx = hr - (hr / R64_HW) * R64_HW;
                const int ih = oy0 + hy, iw = ox0 + hx;
                const bool ok = hr < R64_HROWS && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
                glds16(ok ? (const void*)(xb + ((long)ih * p.IW + iw) * p.ldx) : zero, hbase + i * 1024);
            }
        }
    };

    int rowbase[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int ml = wm * WTM + mi * 16;
        rowbase[mi] = (ml / R64_BW) * R64_HW + (ml % R64_BW) + fr;
    }
    int toff[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) toff[tap] = ((tap / 3) * p.tsh - hy0) * R64_HW + (tap % 3) * p.tsw - hx0;

    // epilogue constants: the MFMA computes D^T (filter rows x pixels), so a
    // lane holds 4 consecutive channels of one pixel -> 8-byte stores.  The
    // per-column scale / (shift + bias) sit in LDS (read as float4 per
    // fragment), not in 24 VGPRs across the whole kernel.
    const EpiParams& e = p.epi;
    __shared__ __attribute__((aligned(16))) float etab[2][NB];
    if (tid < NB) {
        const bool cv = tid < e.n_valid;
        etab[0][tid] = (e.scale && cv) ? e.scale[tid] : 1.f;
        etab[1][tid] = ((e.shift && cv) ? e.shift[tid] : 0.f) + ((e.bias && cv) ? e.bias[tid] : 0.f);
    }

    int t = blockIdx.x;
    if constexpr (DMA) {
        if (t < ntiles) dma(t);
        wait_vmcnt<0>();
    } else {
        if (t < ntiles) fetch(t);
        commit();
    }
    __syncthreads();
    for (; t < ntiles; t += gridDim.x) {
        const int tn = t + gridDim.x;
        // ReluGrad mask of this tile (the input gradient's epilogue), requested
        // before the next tile's halo so the epilogue waits only for it
        uint2 mpre[TM][TN];
        if (e.mask) {
            const int img = t / tpi;
            const int rem = t - img * tpi;
            const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int ml = wm * WTM + mi * 16 + fr;
                const int oy = ty * R64_BH + ml / R64_BW, ox = tx * R64_BW + ml % R64_BW;
                const bool ok = oy < p.OH && ox < p.OW;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col0 = wn * WTN + ni * 16 + 4 * fg;
                    mpre[mi][ni] = uint2{0u, 0u};
                    if (ok && col0 < p.N)
                        mpre[mi][ni] = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(e.mask) + img * e.mask_img +
                                                                       ((long)oy * p.OW + ox) * e.ld_mask + col0);
                }
            }
        }
        if (!DMA && tn < ntiles) fetch(tn);          // in flight during this tile's MFMAs
        f32x4 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
        // software pipeline over the 18 (tap, k-half) steps: fragments of step
        // s+1 are read while the MFMAs of step s issue
        uint4 fa[2][TM], fb[2][TN];
        auto load_step = [&](int st, uint4* a, uint4* b) {
            const int tap = st >> 1, chunk = (st & 1) * 4 + fg;
            if constexpr (ABL == 4) {
#pragma unroll
                for (int mi = 0; mi < TM; ++mi) a[mi] = uint4{(unsigned)st, (unsigned)mi, 0u, (unsigned)tap};
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) b[ni] = uint4{(unsigned)chunk, (unsigned)ni, 1u, 0u};
                return;
            }
            const char* Bt = Bs + tap * NB * 128;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int row = rowbase[mi] + toff[tap];
                a[mi] = *reinterpret_cast<const uint4*>(Hs + row * 128 + 16 * (chunk ^ (row & 6)));
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int row = wn * WTN + ni * 16 + fr;
                b[ni] = *reinterpret_cast<const uint4*>(Bt + row * 128 + 16 * (chunk ^ (row & 6)));
            }
        };
        load_step(0, fa[0], fb[0]);
#pragma unroll
        for (int st = 0; st < 18; ++st) {
            const int cur = st & 1;
            if (st + 1 < 18) load_step(st + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {  // D^T[n][px] += W[n][k] X[px][k]
                    if constexpr (ABL == 2) {
                        asm volatile("" ::"v"(fb[cur][ni].x), "v"(fa[cur][mi].x), "v"(fb[cur][ni].w), "v"(fa[cur][mi].w));
                    } else {
                        acc[mi][ni] = mfma16x16x32<T>(fb[cur][ni], fa[cur][mi], acc[mi][ni]);
                    }
                }
        }
        if constexpr (DMA) {       // every wave is done with the halo: the next one may land
            __syncthreads();
            if (tn < ntiles) dma(tn);
        }
        // ---- MaxPool 2x2 / 2 fused (conv1_2 -> pool1, Network/model/FCN.py:56-57): a
        // wave's 64 pixels are image rows 2 wm (mi 0, 1) and 2 wm + 1 (mi 2, 3), so a
        // window's vertical pair sits in one lane (mi, mi + 2) and its horizontal
        // pair in lanes fr, fr ^ 1; even-fr lanes store 4 pooled channels + switches
        // (values rounded to T before comparing: bit-equal to the unfused pool).
        if constexpr (NB == 64 && ABL == 0) {
            if (e.pool_y) {
                const int img = t / tpi;
                const int rem = t - img * tpi;
                const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
                const int oy = ty * R64_BH + 2 * wm;
                const int PH = p.OH >> 1, PW = p.OW >> 1;
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    const int ox = tx * R64_BW + mi * 16 + fr;
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const int col0 = wn * WTN + ni * 16 + 4 * fg;
                        const f32x4 sc4 = *reinterpret_cast<const f32x4*>(&etab[0][col0]);
                        const f32x4 ad4 = *reinterpret_cast<const f32x4*>(&etab[1][col0]);
                        T o[4];
                        unsigned code = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float raw[4] = {acc[mi][ni][j], dpp_swap1(acc[mi][ni][j]),
                                                  acc[mi + 2][ni][j], dpp_swap1(acc[mi + 2][ni][j])};
                            const bool cv = col0 + j < e.n_valid;
                            float q[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                float x = raw[u] * sc4[j] + ad4[j];
                                if (e.relu) x = fmaxf(x, 0.f);
                                q[u] = cv ? to_f32(from_f32<T>(x)) : 0.f;
                            }
                            unsigned a = 0;
                            float mx = q[0];
                            if (q[1] > mx) { mx = q[1]; a = 1; }
                            if (q[2] > mx) { mx = q[2]; a = 2; }
                            if (q[3] > mx) { mx = q[3]; a = 3; }
                            o[j] = from_f32<T>(mx);
                            code |= (a | (mx > 0.f ? 4u : 0u)) << (8 * j);
                        }
                        if ((fr & 1) || oy + 1 >= p.OH || ox + 1 >= p.OW || col0 >= p.N) continue;
                        const long pix = ((long)img * PH + (oy >> 1)) * PW + (ox >> 1);
                        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(e.pool_y) + pix * e.ld_pool + col0) =
                            *reinterpret_cast<const uint2*>(o);
                        if (e.pool_idx) *reinterpret_cast<unsigned*>(e.pool_idx + pix * e.ld_idx + col0) = code;
                    }
                }
                __syncthreads();                     // all taps read the halo
                commit();                            // next tile's halo (waits for its loads)
                __syncthreads();
                continue;
            }
        }
        // ---- epilogue straight from registers: pixel (mi, fr), channels 4*fg..+3 of (ni)
        {
            const int img = t / tpi;
            const int rem = t - img * tpi;
            const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
            const int oy0 = ty * R64_BH, ox0 = tx * R64_BW;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int ml = wm * WTM + mi * 16 + fr;
                const int oy = oy0 + ml / R64_BW, ox = ox0 + ml % R64_BW;
                if (oy >= p.OH || ox >= p.OW) continue;
                const long pix = (long)oy * p.OW + ox;
                const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col0 = wn * WTN + ni * 16 + 4 * fg;
                    if (col0 >= p.N) continue;
                    float mk[4] = {1.f, 1.f, 1.f, 1.f}, res[4] = {0.f, 0.f, 0.f, 0.f};
                    if (e.mask) {
                        const unsigned short* mh = reinterpret_cast<const unsigned short*>(&mpre[mi][ni]);
#pragma unroll
                        for (int j = 0; j < 4; ++j) mk[j] = bits16_to_f32<T>(mh[j]);
                    }
                    if (e.residual) {
                        const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) res[j] = to_f32(rp[j]);
                    }
                    T o[4];
                    const f32x4 sc4 = *reinterpret_cast<const f32x4*>(&etab[0][col0]);
                    const f32x4 ad4 = *reinterpret_cast<const f32x4*>(&etab[1][col0]);
                    const SegDropRun<4> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int col = col0 + j;
                        float x = acc[mi][ni][j] * sc4[j] + ad4[j];
                        if (e.relu) x = fmaxf(x, 0.f);
                        if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                        x += res[j];
                        if (e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                        o[j] = from_f32<T>(col < e.n_valid ? x : 0.f);
                    }
                    if constexpr (ABL == 3) {
                        asm volatile("" ::"v"(o[0]), "v"(o[3]));
                    } else {
                        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0) =
                            *reinterpret_cast<const uint2*>(o);
                    }
                }
            }
        }
        if constexpr (DMA) {
            wait_vmcnt<0>();                         // the next halo landed (and this tile's stores left)
            __syncthreads();
        } else {
            __syncthreads();                         // all taps read the halo
            commit();                                // next tile's halo (waits for its loads)
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// Ping-pong form of conv_res64 for 64 output channels (conv1_2 fwd + pool1 and
// its input gradient, Network/model/FCN.py:55-57).  conv_res64 runs one
// 8-wave pipeline per CU, so a tile's epilogue, its halo commit and the load
// latency of the next halo all sit between two tiles' MFMAs: ~7.5 us per
// 256-px tile against ~2.2 us of MFMA.  Here the block's waves form two
// groups of four (one wave of each on every SIMD); each wave owns 64 px x 64
// channels (4 x 4 fragments) and a group owns a whole 8 x 32 tile, with its
// own halo buffer filled by LDS DMA.  The block's tiles k = 0, 1, ... go to
// group k % 2; tile k is computed in phase k and finished in phase k + 1, so
// in every phase one group issues MFMAs while the other runs the epilogue of
// its previous tile, DMAs its next halo and waits for it:
//
//   phase   0        1        2        3      ...
//   group0  mma t0   epi t0   mma t2   epi t2
//                    dma t2            dma t4
//   group1  -        mma t1   epi t1   mma t3
//                             dma t3
//
// One block-wide barrier per phase (both groups, nt + 1 phases): it retires
// the computing group's halo reads before the group's next DMA overwrites
// the buffer (issued one phase later), and the DMA-ing group's vmcnt(0) before
// it publishes the new halo for the next phase's MFMAs.  LDS: filter 72 KB +
// 2 halo buffers (43 DMA pieces of 8 rows) + the epilogue table = 162,304 B.
// The ReluGrad mask of a tile is requested at the start of its compute phase
// and reduced to one bit per output (mask > 0) after its MFMAs, so no wait for
// it lands behind the epilogue phase's DMA (vmcnt retires in issue order).
// Given as bits (EpiParams::mask_bits, round 6: conv_c8_fwd writes them with
// conv1_1's map) it is 8 B per pixel instead of 128: four 8-byte loads per
// lane and tile instead of sixteen.
// ---------------------------------------------------------------------------
constexpr int RPP_HS = RPP_PIECES * 8 * 128;         // 44,032 B per halo buffer

template <typename T = bf16>
__global__ __launch_bounds__(512, 1) void conv_res64pp(NTParams p, int tiles_x, int tiles_y, int ntiles) {
    constexpr int NB = 64, TM = 4, TN = 4;
    constexpr int BS = 9 * NB * 128;
    __shared__ __attribute__((aligned(16))) char smem[BS + 2 * RPP_HS + 2 * NB * 4];
    char* Bs = smem;
    float* etab = reinterpret_cast<float*>(smem + BS + 2 * RPP_HS);   // [0][NB] scale, [1][NB] shift + bias

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = w >> 2, wm = w & 3;
    const int fr = lane & 15, fg = lane >> 4;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const void* zero = (const void*)halo_zero_page;
    const int hy0 = p.tsh < 0 ? 2 * p.tsh : 0, hx0 = p.tsw < 0 ? 2 * p.tsw : 0;
    const int tpi = tiles_x * tiles_y;
    const int nt = (int)blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const unsigned hbuf = (unsigned)(uintptr_t)(SEG_LDS char*)smem + BS + g * RPP_HS;
    const char* Hs = smem + BS + g * RPP_HS;
    const EpiParams& e = p.epi;

    // halo of tile t into this group's buffer: piece i = wm + 4 k holds halo
    // rows 8 i .. 8 i + 7; lane -> (row lr, LDS chunk lane & 7), which holds
    // logical chunk (lane & 7) ^ (row & 6) (the swizzle the fragment reads use)
    const int lr = lane >> 3;
    const int hc = (lane & 7) ^ (lr & 6);
    auto dma = [&](int t) {
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
        const int oy0 = ty * R64_BH + p.ioh + hy0, ox0 = tx * R64_BW + p.iow + hx0;
        const T* xb = X + (long)img * p.x_img + hc * 8;
#pragma unroll 1
        for (int k = 0; k < (RPP_PIECES + 3) / 4; ++k) {
            const int i = wm + 4 * k;
            if (i < RPP_PIECES) {
                const int hr = i * 8 + lr;
                const int hy = hr / R64_HW, hx = hr - (hr / R64_HW) * R64_HW;
                const int ih = oy0 + hy, iw = ox0 + hx;
                const bool ok = hr < R64_HROWS && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
                glds16(ok ? (const void*)(xb + ((long)ih * p.IW + iw) * p.ldx) : zero, hbuf + i * 1024);
            }
        }
    };
    auto tile_of = [&](int k) { return (int)blockIdx.x + k * (int)gridDim.x; };

    if (g < nt) dma(tile_of(g));
    // ---- filter: Bs[tap][n][chunk ^ swz(n)] (resident for the whole launch)
    for (int i = tid; i < 9 * NB * 8; i += 512) {
        const int c8 = i & 7, n = (i >> 3) % NB, tap = i / (NB * 8);
        const int j = tap / 3, ii = tap - (tap / 3) * 3;
        uint4 v = {0u, 0u, 0u, 0u};
        if (n < p.N)
            v = *reinterpret_cast<const uint4*>(Wt + (long)n * p.w_col +
                                                (long)((p.rb + p.rstep * j) * p.Sfull + (p.sb + p.sstep * ii)) * p.w_tap +
                                                c8 * 8);
        *reinterpret_cast<uint4*>(Bs + (tap * NB + n) * 128 + 16 * (c8 ^ (n & 6))) = v;
    }
    if (tid < NB) {
        const bool cv = tid < e.n_valid;
        etab[tid] = (e.scale && cv) ? e.scale[tid] : 1.f;
        etab[NB + tid] = ((e.shift && cv) ? e.shift[tid] : 0.f) + ((e.bias && cv) ? e.bias[tid] : 0.f);
    }
    wait_vmcnt<0>();
    lds_barrier();

    int rowbase[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int ml = wm * 64 + mi * 16;
        rowbase[mi] = (ml / R64_BW) * R64_HW + (ml % R64_BW) + fr;
    }
    f32x4 acc[TM][TN];
    uint2 mpre[TM][TN];
    uint64_t mbits = 0;     // ReluGrad mask > 0, bit (mi * TN + ni) * 4 + j
    for (int ph = 0; ph <= nt; ++ph) {
        if ((ph & 1) == g) {
            if (ph < nt) {   // ---- compute phase: tile ph
                const int t = tile_of(ph);
                const int img = t / tpi;
                const int rem = t - img * tpi;
                const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
                if (e.mask_bits) {  // the same as bits: one 8-byte row per pixel (64 channels)
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi) {
                        const int ml = wm * 64 + mi * 16 + fr;
                        const int oy = ty * R64_BH + ml / R64_BW, ox = tx * R64_BW + ml % R64_BW;
                        mpre[mi][0] = uint2{0u, 0u};
                        if (oy < p.OH && ox < p.OW)
                            mpre[mi][0] = *reinterpret_cast<const uint2*>(
                                e.mask_bits + (((long)img * p.OH + oy) * p.OW + ox) * e.ld_bits);
                    }
                } else if (e.mask) {       // ReluGrad mask rows, used in the next phase
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi) {
                        const int ml = wm * 64 + mi * 16 + fr;
                        const int oy = ty * R64_BH + ml / R64_BW, ox = tx * R64_BW + ml % R64_BW;
                        const bool ok = oy < p.OH && ox < p.OW;
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni) {
                            const int col0 = ni * 16 + 4 * fg;
                            mpre[mi][ni] = uint2{0u, 0u};
                            if (ok && col0 < p.N)
                                mpre[mi][ni] = *reinterpret_cast<const uint2*>(
                                    reinterpret_cast<const T*>(e.mask) + img * e.mask_img + ((long)oy * p.OW + ox) * e.ld_mask + col0);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
                // fragment addresses are recomputed in every compute phase (the
                // laundered bases stop the compiler hoisting all 18 x 8 of them
                // out of the phase loop into registers)
                int rb[TM], brow = fr * 128;
#pragma unroll
                for (int mi = 0; mi < TM; ++mi) {
                    rb[mi] = rowbase[mi];
                    asm volatile("" : "+v"(rb[mi]));
                }
                asm volatile("" : "+v"(brow));
                uint4 fa[2][TM], fb[2][TN];
                auto load_step = [&](int st, uint4* a, uint4* b) {
                    const int tap = st >> 1, chunk = (st & 1) * 4 + fg;
                    const char* Bt = Bs + tap * NB * 128;
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi) {
                        const int row = rb[mi] + ((tap / 3) * p.tsh - hy0) * R64_HW + (tap % 3) * p.tsw - hx0;
                        a[mi] = *reinterpret_cast<const uint4*>(Hs + row * 128 + 16 * (chunk ^ (row & 6)));
                    }
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        // row ni * 16 + fr: (row & 6) == (fr & 6)
                        b[ni] = *reinterpret_cast<const uint4*>(Bt + ni * 2048 + brow + 16 * (chunk ^ (fr & 6)));
                    }
                };
                load_step(0, fa[0], fb[0]);
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int st = 0; st < 18; ++st) {
                    const int cur = st & 1;
                    if (st + 1 < 18) load_step(st + 1, fa[cur ^ 1], fb[cur ^ 1]);
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni)   // D^T[n][px] += W[n][k] X[px][k]
                            acc[mi][ni] = mfma16x16x32<T>(fb[cur][ni], fa[cur][mi], acc[mi][ni]);
                }
                __builtin_amdgcn_s_setprio(0);
                if (e.mask_bits) {  // channels ni * 16 + 4 fg .. + 3: one nibble per (mi, ni)
                    mbits = 0;
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi) {
                        const uint64_t row = (uint64_t)mpre[mi][0].x | ((uint64_t)mpre[mi][0].y << 32);
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni)
                            mbits |= ((row >> (ni * 16 + 4 * fg)) & 0xFull) << ((mi * TN + ni) * 4);
                    }
                } else if (e.mask) {       // the loads had the whole MFMA loop to land
                    mbits = 0;
#pragma unroll
                    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                        for (int ni = 0; ni < TN; ++ni) {
                            const unsigned short* mh = reinterpret_cast<const unsigned short*>(&mpre[mi][ni]);
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                if (bits16_to_f32<T>(mh[j]) > 0.f) mbits |= 1ull << ((mi * TN + ni) * 4 + j);
                        }
                }
            }
        } else if (ph >= 1) {   // ---- epilogue phase: tile ph - 1, then the DMA of tile ph + 1
            const int t = tile_of(ph - 1);
            const int img = t / tpi;
            const int rem = t - img * tpi;
            const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
            if (ph + 1 < nt) dma(tile_of(ph + 1));
            if (e.pool_y) {    // MaxPool 2x2 / 2 fused (as conv_res64: rows 2 wm, 2 wm + 1 per wave)
                const int oy = ty * R64_BH + 2 * wm;
                const int PH = p.OH >> 1, PW = p.OW >> 1;
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    const int ox = tx * R64_BW + mi * 16 + fr;
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const int col0 = ni * 16 + 4 * fg;
                        const f32x4 sc4 = *reinterpret_cast<const f32x4*>(etab + col0);
                        const f32x4 ad4 = *reinterpret_cast<const f32x4*>(etab + NB + col0);
                        T o[4];
                        unsigned code = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float raw[4] = {acc[mi][ni][j], dpp_swap1(acc[mi][ni][j]),
                                                  acc[mi + 2][ni][j], dpp_swap1(acc[mi + 2][ni][j])};
                            const bool cv = col0 + j < e.n_valid;
                            float q[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                float x = raw[u] * sc4[j] + ad4[j];
                                if (e.relu) x = fmaxf(x, 0.f);
                                q[u] = cv ? to_f32(from_f32<T>(x)) : 0.f;
                            }
                            unsigned a = 0;
                            float mx = q[0];
                            if (q[1] > mx) { mx = q[1]; a = 1; }
                            if (q[2] > mx) { mx = q[2]; a = 2; }
                            if (q[3] > mx) { mx = q[3]; a = 3; }
                            o[j] = from_f32<T>(mx);
                            code |= (a | (mx > 0.f ? 4u : 0u)) << (8 * j);
                        }
                        if ((fr & 1) || oy + 1 >= p.OH || ox + 1 >= p.OW || col0 >= p.N) continue;
                        const long pix = ((long)img * PH + (oy >> 1)) * PW + (ox >> 1);
                        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(e.pool_y) + pix * e.ld_pool + col0) =
                            *reinterpret_cast<const uint2*>(o);
                        if (e.pool_idx) *reinterpret_cast<unsigned*>(e.pool_idx + pix * e.ld_idx + col0) = code;
                    }
                }
            } else {           // straight from registers: pixel (mi, fr), channels 4 fg .. + 3 of (ni)
                const int oy0 = ty * R64_BH, ox0 = tx * R64_BW;
#pragma unroll
                for (int mi = 0; mi < TM; ++mi) {
                    const int ml = wm * 64 + mi * 16 + fr;
                    const int oy = oy0 + ml / R64_BW, ox = ox0 + ml % R64_BW;
                    if (oy >= p.OH || ox >= p.OW) continue;
                    const long pix = (long)oy * p.OW + ox;
                    const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
#pragma unroll
                    for (int ni = 0; ni < TN; ++ni) {
                        const int col0 = ni * 16 + 4 * fg;
                        if (col0 >= p.N) continue;
                        float res[4] = {0.f, 0.f, 0.f, 0.f};
                        if (e.residual) {
                            const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
#pragma unroll
                            for (int j = 0; j < 4; ++j) res[j] = to_f32(rp[j]);
                        }
                        T o[4];
                        const f32x4 sc4 = *reinterpret_cast<const f32x4*>(etab + col0);
                        const f32x4 ad4 = *reinterpret_cast<const f32x4*>(etab + NB + col0);
                        const SegDropRun<4> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int col = col0 + j;
                            float x = acc[mi][ni][j] * sc4[j] + ad4[j];
                            if (e.relu) x = fmaxf(x, 0.f);
                            if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                            x += res[j];
                            if (e.mask || e.mask_bits) x = (mbits >> ((mi * TN + ni) * 4 + j)) & 1 ? x * e.mask_scale : 0.f;
                            o[j] = from_f32<T>(col < e.n_valid ? x : 0.f);
                        }
                        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0) =
                            *reinterpret_cast<const uint2*>(o);
                    }
                }
            }
            wait_vmcnt<0>();   // this group's next halo has landed (and its stores left)
        }
        lds_barrier();
    }
}

// ---------------------------------------------------------------------------
// Resident-filter direct conv for 16 input channels: the input gradient of
// FC-DenseNet's 64 -> 16 growth convs (dz: 16 channels, dx: 64), which the
// implicit GEMM ran at ~1.7 TB/s.  One v_mfma_f32_16x16x32 k-step covers two
// taps x 16 channels, so the 9 taps take 5 steps (tap 8 pairs with a zero
// filter tap).  Filter [5 steps][64 n][64 B] = 20 KB and the 10 x 34 px halo
// of 32-byte rows (10.9 KB) stay in LDS; tiles, prefetch and epilogue as
// conv_res64.  Swizzles: filter rows chunk ^ ((n >> 2) & 3), halo rows
// chunk ^ ((row >> 3) & 1).
// ---------------------------------------------------------------------------
// BNB: the epilogue continues through the BatchNorm(+ReLU) backward of the
// layer whose output this conv read (EpiParams.bn_*; then the standard
// dropout fields re-draw the dropout of the conv before that BN), and the
// block's column sums of dz*x / dz over all its tiles go to bn_part[block].
// BH: tile rows (tile BH x 32 px, BH waves of 64 px x 32 channels).  The BNB
// epilogue (BN-input reads, the dropout hash and the BN sums per element)
// holds the kernel at 160 VGPRs, three waves per SIMD: 8-row tiles (8-wave
// blocks) fit one block per CU, 4-row tiles (4-wave blocks) three, and the
// blocks' epilogues, MFMAs and loads then overlap.
// ST: the wave's 64 px x 32 ch output tile goes through a per-wave LDS
// buffer and leaves as 16-byte stores of 64-byte row halves (4 per lane per
// tile) instead of 8-byte stores of 32-byte pieces (8 per lane)
template <typename T = bf16, bool BNB = false, int BH = 8, bool ST = false>
__global__ __launch_bounds__(BH * 64, BNB ? (BH == 8 ? 2 : 3) : 4) void conv_res16c(NTParams p, int tiles_x, int tiles_y,
                                                                                  int ntiles) {
    static_assert(BH == 8 || BH == 4 || BH == 2, "tile rows");
    constexpr int NT = BH * 64, NW = BH;
    constexpr int HROWS = (BH + 2) * R64_HW;
    constexpr int R16_PER = (HROWS * 2 + NT - 1) / NT;   // halo chunks per thread
    constexpr int WN = 2, WTM = 64, WTN = 32, TM = 4, TN = 2, KS = 5;
    constexpr int BS = KS * 64 * 64;
    constexpr int HS = HROWS * 32 > NW * 2 * 32 * 4 ? HROWS * 32 : NW * 2 * 32 * 4;
    __shared__ __attribute__((aligned(16))) char smem[BS + HS];
    __shared__ __attribute__((aligned(16))) char stg[ST ? NW * 4096 : 16];
    char* Bs = smem;
    char* Hs = smem + BS;

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w / WN, wn = w - (w / WN) * WN;
    const int fr = lane & 15, fg = lane >> 4;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const int hy0 = p.tsh < 0 ? 2 * p.tsh : 0, hx0 = p.tsw < 0 ? 2 * p.tsw : 0;
    const int tpi = tiles_x * tiles_y;

    // ---- filter: Bs[ks][n][q ^ swz(n)], chunk q = (tap 2ks + (q >> 1), channels 8 (q & 1)..)
    for (int i = tid; i < KS * 64 * 4; i += NT) {
        const int q = i & 3, n = (i >> 2) & 63, ks = i >> 8;
        const int tap = 2 * ks + (q >> 1), c8 = q & 1;
        uint4 v = {0u, 0u, 0u, 0u};
        if (n < p.N && tap < 9) {
            const int j = tap / 3, ii = tap - (tap / 3) * 3;
            v = *reinterpret_cast<const uint4*>(Wt + (long)n * p.w_col +
                                                (long)((p.rb + p.rstep * j) * p.Sfull + (p.sb + p.sstep * ii)) * p.w_tap +
                                                c8 * 8);
        }
        *reinterpret_cast<uint4*>(Bs + (ks * 64 + n) * 64 + 16 * (q ^ ((n >> 2) & 3))) = v;
    }
    // ---- halo fetch into registers: slot q -> (row q / 2, chunk q % 2)
    uint4 hv[R16_PER];
    auto fetch = [&](int t) {
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
        const int oy0 = ty * BH, ox0 = tx * R64_BW;
#pragma unroll
        for (int k = 0; k < R16_PER; ++k) {
            const int q = tid + k * NT;
            const int hr = q >> 1, c8 = q & 1;
            uint4 v = {0u, 0u, 0u, 0u};
            if (hr < HROWS) {
                const int hy = hr / R64_HW, hx = hr - (hr / R64_HW) * R64_HW;
                const int ih = oy0 + p.ioh + hy0 + hy, iw = ox0 + p.iow + hx0 + hx;
                if ((unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW)
                    v = *reinterpret_cast<const uint4*>(X + (long)img * p.x_img + ((long)ih * p.IW + iw) * p.ldx + c8 * 8);
            }
            hv[k] = v;
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int k = 0; k < R16_PER; ++k) {
            const int q = tid + k * NT;
            const int hr = q >> 1, c8 = q & 1;
            if (hr < HROWS) *reinterpret_cast<uint4*>(Hs + hr * 32 + 16 * (c8 ^ ((hr >> 3) & 1))) = hv[k];
        }
    };

    int rowbase[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
        const int ml = wm * WTM + mi * 16;
        rowbase[mi] = (ml / R64_BW) * R64_HW + (ml % R64_BW) + fr;
    }
    int toff[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) toff[tap] = ((tap / 3) * p.tsh - hy0) * R64_HW + (tap % 3) * p.tsw - hx0;

    // per-column epilogue constants in LDS (float4 per fragment): scale,
    // shift + bias, and for BNB the BN's gamma * inv and beta
    const EpiParams& e = p.epi;
    __shared__ __attribute__((aligned(16))) float etab[4][64];
    if (tid < 64) {
        const bool cv = tid < e.n_valid;
        etab[0][tid] = (e.scale && cv) ? e.scale[tid] : 1.f;
        etab[1][tid] = ((e.shift && cv) ? e.shift[tid] : 0.f) + ((e.bias && cv) ? e.bias[tid] : 0.f);
        if constexpr (BNB) {
            const bool bv = tid < e.bn_cv;
            etab[2][tid] = bv ? e.bn_gamma[tid] * e.bn_inv : 0.f;
            etab[3][tid] = bv ? e.bn_beta[tid] : 0.f;
        }
    }
    float sgm[TN][4], sbt[TN][4];
    if constexpr (BNB) {
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) sgm[ni][j] = sbt[ni][j] = 0.f;
    }

    int t = blockIdx.x;
    if (t < ntiles) fetch(t);
    commit();
    __syncthreads();
    const int hi_tap = fg >> 1, ach = fg & 1;
    for (; t < ntiles; t += gridDim.x) {
        const int tn = t + gridDim.x;
        if (tn < ntiles) fetch(tn);                  // in flight during this tile's MFMAs
        // BNB: this tile's BN inputs for the lane's epilogue elements, also
        // requested now so their latency hides under the MFMAs
        uint2 pxb[BNB ? TM : 1][BNB ? TN : 1];
        if constexpr (BNB) {
            const int img = t / tpi;
            const int rem = t - img * tpi;
            const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int ml = wm * WTM + mi * 16 + fr;
                const int oy = ty * BH + ml / R64_BW, ox = tx * R64_BW + ml % R64_BW;
                const bool ok = oy < p.OH && ox < p.OW;
                const long pix = ok ? (long)oy * p.OW + ox : 0;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col0 = wn * WTN + ni * 16 + 4 * fg;
                    pxb[mi][ni] = uint2{0u, 0u};
                    if (ok && col0 < p.N)
                        pxb[mi][ni] = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(e.bn_x) +
                                                                       img * e.bn_x_img + pix * e.ld_bn_x + col0);
                }
            }
        }
        f32x4 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jj = 0; jj < TN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            // this lane's k group reads tap 2ks (groups 0, 1) or 2ks + 1 (2, 3)
            const int to = hi_tap ? toff[ks * 2 + 1 < 9 ? ks * 2 + 1 : 8] : toff[ks * 2];
            uint4 fa[TM], fb[TN];
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int row = rowbase[mi] + to;
                fa[mi] = *reinterpret_cast<const uint4*>(Hs + row * 32 + 16 * (ach ^ ((row >> 3) & 1)));
            }
#pragma unroll
            for (int ni = 0; ni < TN; ++ni) {
                const int n = wn * WTN + ni * 16 + fr;
                fb[ni] = *reinterpret_cast<const uint4*>(Bs + (ks * 64 + n) * 64 + 16 * (fg ^ ((n >> 2) & 3)));
            }
#pragma unroll
            for (int mi = 0; mi < TM; ++mi)
#pragma unroll
                for (int ni = 0; ni < TN; ++ni)   // D^T[n][px] += W[n][k] X[px][k]
                    acc[mi][ni] = mfma16x16x32<T>(fb[ni], fa[mi], acc[mi][ni]);
        }
        {
            const int img = t / tpi;
            const int rem = t - img * tpi;
            const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
            const int oy0 = ty * BH, ox0 = tx * R64_BW;
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) {
                const int ml = wm * WTM + mi * 16 + fr;
                const int oy = oy0 + ml / R64_BW, ox = ox0 + ml % R64_BW;
                if (oy >= p.OH || ox >= p.OW) continue;
                const long pix = (long)oy * p.OW + ox;
                const uint64_t gidx = ((uint64_t)((long)img * p.OH * p.OW + pix)) * e.n_valid;
#pragma unroll
                for (int ni = 0; ni < TN; ++ni) {
                    const int col0 = wn * WTN + ni * 16 + 4 * fg;
                    if (col0 >= p.N) continue;
                    float mk[4] = {1.f, 1.f, 1.f, 1.f}, res[4] = {0.f, 0.f, 0.f, 0.f};
                    if (e.mask) {
                        const T* mp = reinterpret_cast<const T*>(e.mask) + img * e.mask_img + pix * e.ld_mask + col0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) mk[j] = to_f32(mp[j]);
                    }
                    if (e.residual) {
                        const T* rp = reinterpret_cast<const T*>(e.residual) + img * e.res_img + pix * e.ld_res + col0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) res[j] = to_f32(rp[j]);
                    }
                    T o[4];
                    if constexpr (BNB) {
                        const uint2 xr = pxb[mi][ni];
                        const T* xh = reinterpret_cast<const T*>(&xr);
                        const f32x4 bs4 = *reinterpret_cast<const f32x4*>(&etab[2][col0]);
                        const f32x4 bb4 = *reinterpret_cast<const f32x4*>(&etab[3][col0]);
                        const SegDropRun<4> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int col = col0 + j;
                            const float xv = to_f32(xh[j]);
                            const bool on = col < e.bn_cv && (!e.bn_relu || xv * bs4[j] + bb4[j] > 0.f);
                            const float dz = on ? acc[mi][ni][j] : 0.f;
                            sgm[ni][j] += dz * xv;
                            sbt[ni][j] += dz;
                            float x = dz * bs4[j];
                            if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                            o[j] = from_f32<T>(col < e.n_valid ? x : 0.f);
                        }
                    } else {
                        const f32x4 sc4 = *reinterpret_cast<const f32x4*>(&etab[0][col0]);
                        const f32x4 ad4 = *reinterpret_cast<const f32x4*>(&etab[1][col0]);
                        const SegDropRun<4> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int col = col0 + j;
                            float x = acc[mi][ni][j] * sc4[j] + ad4[j];
                            if (e.relu) x = fmaxf(x, 0.f);
                            if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                            x += res[j];
                            if (e.mask) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                            o[j] = from_f32<T>(col < e.n_valid ? x : 0.f);
                        }
                    }
                    if constexpr (ST) {
                        const int r = mi * 16 + fr;
                        *reinterpret_cast<uint2*>(stg + w * 4096 + r * 64 + 16 * ((ni * 2 + (fg >> 1)) ^ ((r >> 2) & 3)) +
                                                  8 * (fg & 1)) = *reinterpret_cast<const uint2*>(o);
                    } else {
                        *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.y) + img * p.y_img + pix * p.ldy + col0) =
                            *reinterpret_cast<const uint2*>(o);
                    }
                }
            }
            if constexpr (ST) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const int c = lane & 3;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = q * 16 + (lane >> 2);
                    const uint4 v = *reinterpret_cast<const uint4*>(stg + w * 4096 + r * 64 + 16 * (c ^ ((r >> 2) & 3)));
                    const int ml = wm * WTM + r;
                    const int oy = oy0 + ml / R64_BW, ox = ox0 + ml % R64_BW;
                    const int col = wn * WTN + c * 8;
                    if (oy < p.OH && ox < p.OW && col < p.N)
                        *reinterpret_cast<uint4*>(reinterpret_cast<T*>(p.y) + img * p.y_img +
                                                  ((long)oy * p.OW + ox) * p.ldy + col) = v;
                }
            }
        }
        __syncthreads();                             // all steps read the halo
        commit();                                    // next tile's halo (waits for its loads)
        __syncthreads();
    }
    if constexpr (BNB) {
        // lanes fr = 0..15 share channels: butterfly over them, then the
        // M waves of each column half meet in LDS (the halo is free)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int off = 1; off < 16; off <<= 1) {
                    sgm[ni][j] += __shfl_xor(sgm[ni][j], off);
                    sbt[ni][j] += __shfl_xor(sbt[ni][j], off);
                }
        float* red = reinterpret_cast<float*>(Hs);   // [NW waves][2 kinds][32 columns]
        if (fr == 0) {
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int lc = ni * 16 + 4 * fg + j;
                    red[(w * 2 + 0) * 32 + lc] = sgm[ni][j];
                    red[(w * 2 + 1) * 32 + lc] = sbt[ni][j];
                }
        }
        __syncthreads();
        if (tid < 2 * 64) {
            const int kind = tid / 64, c = tid % 64, wn_ = c / 32, lc = c % 32;
            float sum = 0.f;
            for (int wm_ = 0; wm_ < NW / WN; ++wm_) sum += red[((wm_ * WN + wn_) * 2 + kind) * 32 + lc];
            if (c < e.bn_C) e.bn_part[(long)blockIdx.x * 2 * e.bn_C + kind * e.bn_C + c] = sum;
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static constexpr int kHaloBW[3] = {16, 32, 64};

bool halo_plan(const NTParams& p, int dtype, int max_splits, int cus, HaloPlan* hp) {
    if (!g_nt_halo || (dtype != SEG_BF16 && dtype != SEG_F16)) return false;
    if (p.phase || p.ish != 1 || p.isw != 1 || p.osh != 1 || p.osw != 1 || p.ooh != 0 || p.oow != 0) return false;
    if (p.Ha != p.OH || p.Wa != p.OW || p.rb != 0 || p.sb != 0) return false;
    if (p.C % 64 != 0 || p.K % p.C != 0 || p.taps_w <= 0) return false;
    const int ntaps = p.K / p.C;
    if (ntaps % p.taps_w) return false;
    const int taps_h = ntaps / p.taps_w;
    if (p.OH <= 0 || p.OW <= 0 || p.M % (p.OH * p.OW)) return false;
    const int nimg = p.M / (p.OH * p.OW);
    long best = -1;
    for (int k = 0; k < 3; ++k) {
        const int bw = kHaloBW[k], bh = 256 / bw;
        const int hwd = bw + (p.taps_w - 1) * std::abs(p.tsw);
        const int hht = bh + (taps_h - 1) * std::abs(p.tsh);
        const int hrows = hwd * hht;
        const int hi = (hrows + 63) / 64;
        if (hi > 7 || hi > ntaps - 1) continue;
        const int tx = (p.OW + bw - 1) / bw, ty = (p.OH + bh - 1) / bh;
        // padded output work + halo staging (~1/9 of the per-tap filter stream)
        const long cost = (long)tx * ty * (256 * 16 + hrows);
        if (best < 0 || cost < best) {
            best = cost;
            hp->bw = bw;
            hp->hi = hi <= 6 ? 6 : 7;
            hp->geom[0] = taps_h; hp->geom[1] = tx; hp->geom[2] = ty; hp->geom[3] = nimg;
            hp->geom[4] = hwd; hp->geom[5] = hrows;
            hp->geom[6] = std::min(0, (taps_h - 1) * p.tsh);
            hp->geom[7] = std::min(0, (p.taps_w - 1) * p.tsw);
        }
    }
    if (best < 0) return false;
    hp->bn = p.N <= 64 ? 64 : 128;
    if (p.N > 128 && g_halo_wide) {
        // 256 x 256 four-phase kernel: halo must fit 6 pieces (384 rows)
        long best2 = -1;
        for (int k = 0; k < 2; ++k) {
            const int bw = kHaloBW[k], bh = 256 / bw;
            const int hwd = bw + (p.taps_w - 1) * std::abs(p.tsw);
            const int hht = bh + (taps_h - 1) * std::abs(p.tsh);
            if (hwd * hht > 384 || 6 > ntaps - 1) continue;
            const int tx = (p.OW + bw - 1) / bw, ty = (p.OH + bh - 1) / bh;
            const long cost = (long)tx * ty * (256 * 16 + hwd * hht);
            if (best2 < 0 || cost < best2) {
                best2 = cost;
                hp->bw = bw;
                hp->hi = 6;
                hp->geom[1] = tx; hp->geom[2] = ty;
                hp->geom[4] = hwd; hp->geom[5] = hwd * hht;
            }
        }
        if (best2 >= 0) hp->bn = 256;
    }
    const int nchunks = p.C / 64;
    const long tiles = (long)hp->geom[1] * hp->geom[2] * nimg * ((p.N + hp->bn - 1) / hp->bn);
    // split-K over channel chunks: minimise (block rounds x chunks per split),
    // +4% per extra split for the fp32 slab round trip and reduce
    const int lo = std::min(nchunks, std::max(1, g_halo_min_splits));
    const int cap = std::max(lo, std::min(nchunks, std::max(1, max_splits)));
    int kps = (nchunks + lo - 1) / lo;
    double best_t = 1e30;
    for (int sp = lo; sp <= cap; ++sp) {
        const int k = (nchunks + sp - 1) / sp;
        const int s2 = (nchunks + k - 1) / k;
        const long rounds = (tiles * s2 + cus - 1) / cus;
        const double t = (double)rounds * k * (1.0 + 0.04 * (s2 - 1));
        if (t < best_t * 0.999) { best_t = t; kps = k; }
    }
    hp->splits = (nchunks + kps - 1) / kps;
    hp->geom[8] = nchunks;
    hp->geom[9] = kps;
    hp->tiles = tiles;
    return true;
}

template <int BW, int HI, int BN>
static void launch_halo_t(NTParams& p, const HaloGeom& g, long tiles, int gridz, hipStream_t s, int dtype) {
    if (dtype == SEG_F16)
        hipLaunchKernelGGL((conv_halo<BW, HI, BN, f16>), dim3((unsigned)tiles, 1, gridz), dim3(512), 0, s, p, g);
    else
        hipLaunchKernelGGL((conv_halo<BW, HI, BN>), dim3((unsigned)tiles, 1, gridz), dim3(512), 0, s, p, g);
}

template <int BW, int HI, int BN>
static void launch_halo_duo_t(NTParams& p, const HaloGeom& g, long tiles, hipStream_t s, int dtype) {
    if constexpr (BW == 16 && HI == 6) {
        if (p.epi.unpool_y) {     // MaxPoolGrad epilogue (halo_unpools)
            if (dtype == SEG_F16)
                hipLaunchKernelGGL((conv_halo_duo<BW, HI, BN, f16, true>), dim3((unsigned)tiles), dim3(512), 0, s, p, g);
            else
                hipLaunchKernelGGL((conv_halo_duo<BW, HI, BN, bf16, true>), dim3((unsigned)tiles), dim3(512), 0, s, p, g);
            return;
        }
    }
    if (dtype == SEG_F16)
        hipLaunchKernelGGL((conv_halo_duo<BW, HI, BN, f16>), dim3((unsigned)tiles), dim3(512), 0, s, p, g);
    else
        hipLaunchKernelGGL((conv_halo_duo<BW, HI, BN>), dim3((unsigned)tiles), dim3(512), 0, s, p, g);
}

template <int BW, int HI>
static void launch_halo_bn(NTParams& p, const HaloGeom& g, int bn, long tiles, int gridz, bool duo, hipStream_t s,
                           int dtype) {
    if (duo) {
        if (bn == 64) launch_halo_duo_t<BW, HI, 64>(p, g, tiles, s, dtype);
        else launch_halo_duo_t<BW, 6, 128>(p, g, tiles, s, dtype);
        return;
    }
    if (bn == 64) launch_halo_t<BW, HI, 64>(p, g, tiles, gridz, s, dtype);
    else launch_halo_t<BW, HI, 128>(p, g, tiles, gridz, s, dtype);
}

// Which halo kernel runs plan hp: conv_halo2 for 256-wide blocks; for 64 / 128
// conv_halo_duo at two blocks per CU when there is no split-K (its 80 KiB LDS
// takes HI = 7 halos for BN = 64 only; 32-bit in-image offsets; the f16 BW = 32 /
// BN = 128 instance spills), else conv_halo.
int halo_kernel(const NTParams& p, const HaloPlan& hp, int dtype) {
    if (hp.bn == 256) return halo4_ok(p, hp) ? HALO_K4 : HALO_K2;
    if (g_halo_duo && hp.splits == 1 && (hp.bn == 64 || hp.hi == 6) && (long)p.IH * p.IW * p.ldx < (1L << 31) &&
        !(dtype == SEG_F16 && hp.bw == 32 && hp.bn == 128))
        return HALO_KDUO;
    return HALO_K1;
}

// The kernel has the fused MaxPool epilogue for this plan: conv_halo2 (16- and
// 32-px tile rows, 64-column wave tiles), conv_halo_duo<16, 6, 128> (32-row
// staging halves, 8 column chunks per row) -- never with split-K slabs.
// The kernel has the MaxPoolGrad epilogue (EpiParams::unpool_y) for this
// plan: conv_halo2 with 16-px tile rows, conv_halo_duo<16, 6, *> -- never
// with split-K slabs.
bool halo_unpools(const HaloPlan& hp, int kernel) {
    if (hp.splits != 1 || hp.bw != 16) return false;
    return kernel == HALO_K2 || kernel == HALO_K4 || (kernel == HALO_KDUO && hp.hi == 6);
}

bool halo_pools(const HaloPlan& hp, int kernel) {
    if (hp.splits != 1) return false;
    if (kernel == HALO_K2 || kernel == HALO_K4) return true;
    return kernel == HALO_KDUO && hp.bw == 16 && hp.bn == 128 && hp.hi == 6;
}

bool res16c_ok(const NTParams& p, int dtype) {
    return g_res16c && g_nt_halo && (dtype == SEG_BF16 || dtype == SEG_F16) && !p.phase && p.ish == 1 &&
           p.isw == 1 && p.osh == 1 && p.osw == 1 && p.ooh == 0 && p.oow == 0 && p.Ha == p.OH && p.Wa == p.OW &&
           p.C == 16 && p.K == 9 * 16 && p.taps_w == 3 && (p.tsh == 1 || p.tsh == -1) &&
           (p.tsw == 1 || p.tsw == -1) && p.N <= 64 && p.N % 8 == 0 && p.ldx % 8 == 0 && p.OH > 0 && p.OW > 0 &&
           p.M % (p.OH * p.OW) == 0;
}

void launch_res16c(NTParams& p, int cus, hipStream_t s, int dtype) {
    const int tx = (p.OW + R64_BW - 1) / R64_BW, ty = (p.OH + R64_BH - 1) / R64_BH;
    const int ntiles = (p.M / (p.OH * p.OW)) * tx * ty;
    const int grid = std::min(ntiles, 2 * cus);
    if (dtype == SEG_F16) hipLaunchKernelGGL((conv_res16c<f16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
    else hipLaunchKernelGGL((conv_res16c<bf16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
}

// grid of the BN-backward form (= its bn_part rows): tiles of g_res16c_bh rows,
// two rounds of the resident blocks (8 rows: one per CU, 4 rows: three)
int res16c_grid(const NTParams& p, int cus) {
    const int bh = g_res16c_bh;
    const int tx = (p.OW + R64_BW - 1) / R64_BW, ty = (p.OH + bh - 1) / bh;
    return std::min((p.M / (p.OH * p.OW)) * tx * ty, (bh == 8 ? 2 : 6) * cus);
}

// staged 16-byte dx stores in the BN-backward form: 403 -> 336 us at
// 384x1248x8, C3 213 -> 215.8 img/s (0: 8-byte stores from the accumulators)

template <typename T, int BH>
static void launch_res16c_bn_t(NTParams& p, int grid, hipStream_t s) {
    const int tx = (p.OW + R64_BW - 1) / R64_BW, ty = (p.OH + BH - 1) / BH;
    const int ntiles = (p.M / (p.OH * p.OW)) * tx * ty;
    const bool st = g_res16c_st && p.ldy % 8 == 0 && p.y_img % 8 == 0 && ((uintptr_t)p.y % 16) == 0;
    if (st) hipLaunchKernelGGL((conv_res16c<T, true, BH, true>), dim3(grid), dim3(BH * 64), 0, s, p, tx, ty, ntiles);
    else hipLaunchKernelGGL((conv_res16c<T, true, BH>), dim3(grid), dim3(BH * 64), 0, s, p, tx, ty, ntiles);
}

void launch_res16c_bn(NTParams& p, int cus, hipStream_t s, int dtype) {
    const int grid = res16c_grid(p, cus);
    const bool h = dtype == SEG_F16;
    switch (g_res16c_bh) {
        case 8: h ? launch_res16c_bn_t<f16, 8>(p, grid, s) : launch_res16c_bn_t<bf16, 8>(p, grid, s); break;
        default: h ? launch_res16c_bn_t<f16, 4>(p, grid, s) : launch_res16c_bn_t<bf16, 4>(p, grid, s); break;
    }
}

bool res64_ok(const NTParams& p, int dtype) {
    return g_res64 && g_nt_halo && (dtype == SEG_BF16 || dtype == SEG_F16) && !p.phase && p.ish == 1 && p.isw == 1 && p.osh == 1 &&
           p.osw == 1 && p.ooh == 0 && p.oow == 0 && p.Ha == p.OH && p.Wa == p.OW && p.C == 64 && p.K == 9 * 64 &&
           p.taps_w == 3 && (p.tsh == 1 || p.tsh == -1) && (p.tsw == 1 || p.tsw == -1) && p.N <= 64 &&
           p.N % 8 == 0 && p.OH > 0 && p.OW > 0 && p.M % (p.OH * p.OW) == 0 &&
           (!p.epi.mask || ((uintptr_t)p.epi.mask % 8 == 0 && p.epi.ld_mask % 4 == 0 && p.epi.mask_img % 4 == 0)) &&
           (!p.epi.mask_bits || (p.N == 64 && !p.epi.mask && (uintptr_t)p.epi.mask_bits % 8 == 0 &&
                                 p.epi.ld_bits >= 8 && p.epi.ld_bits % 8 == 0));
}

int launch_res64(NTParams& p, int cus, hipStream_t s, int dtype) {
    const int tx = (p.OW + R64_BW - 1) / R64_BW, ty = (p.OH + R64_BH - 1) / R64_BH;
    const int ntiles = (p.M / (p.OH * p.OW)) * tx * ty;
    if (p.N <= 16 && g_res16) {
        if (p.epi.pool_y || p.epi.mask_bits) return SEG_EINVAL;  // no pooled epilogue / mask bits in the 16-wide form
        const int grid = std::min(ntiles, 2 * cus);
        if (g_res16_dma) {                    // two blocks per CU (launch bounds: 4 waves / SIMD)
            if (dtype == SEG_F16)
                hipLaunchKernelGGL((conv_res64<0, f16, 16, true>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
            else
                hipLaunchKernelGGL((conv_res64<0, bf16, 16, true>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
        } else if (dtype == SEG_F16) {
            hipLaunchKernelGGL((conv_res64<0, f16, 16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
        } else {
            hipLaunchKernelGGL((conv_res64<0, bf16, 16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
        }
        return SEG_OK;
    }
    const int grid = std::min(ntiles, cus);
    if (g_res64_pp == 2 || (g_res64_pp == 1 && (p.epi.pool_y || p.epi.mask)) || p.epi.mask_bits) {
        if (dtype == SEG_F16) hipLaunchKernelGGL((conv_res64pp<f16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
        else hipLaunchKernelGGL((conv_res64pp<bf16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
        return SEG_OK;
    }
    if (dtype == SEG_F16) hipLaunchKernelGGL((conv_res64<0, f16>), dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
    else hipLaunchKernelGGL(conv_res64<0>, dim3(grid), dim3(512), 0, s, p, tx, ty, ntiles);
    return SEG_OK;
}

// Launch plan hp on the kernel halo_kernel() chose.  A pooled launch (p.y
// null) on a kernel without the pooled epilogue, or with split-K slabs, is
// refused here, at the kernel choice itself.
int launch_halo(NTParams& p, const HaloPlan& hp, int kernel, hipStream_t s, int dtype) {
    if (p.epi.pool_y && !halo_pools(hp, kernel)) return SEG_EINVAL;
    if (p.epi.unpool_y && !halo_unpools(hp, kernel)) return SEG_EINVAL;
    if (hp.splits > 1 && !p.partial) return SEG_EINVAL;
    HaloGeom g;
    g.taps_h = hp.geom[0]; g.tiles_x = hp.geom[1]; g.tiles_y = hp.geom[2]; g.nimg = hp.geom[3];
    g.hwd = hp.geom[4]; g.hrows = hp.geom[5]; g.hy0 = hp.geom[6]; g.hx0 = hp.geom[7];
    g.nchunks = hp.geom[8]; g.kc_per_split = hp.geom[9];
    const int gridz = hp.splits;
    if (kernel == HALO_K4) {
        launch_halo4(p, hp, g, s, dtype);
        return SEG_OK;
    }
    if (kernel == HALO_K2) {
        const dim3 grid((unsigned)hp.tiles, 1, gridz);
#ifdef SEG_DIAG   // ablation builds (garbage results): tools/ only
        if (g_nt2_ablate && hp.bw == 16 && dtype == SEG_BF16) {
            switch (g_nt2_ablate) {
                case 1: hipLaunchKernelGGL((conv_halo2<16, 1>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 2: hipLaunchKernelGGL((conv_halo2<16, 2>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 3: hipLaunchKernelGGL((conv_halo2<16, 3>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 4: hipLaunchKernelGGL((conv_halo2<16, 4>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 5: hipLaunchKernelGGL((conv_halo2<16, 5>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 7: hipLaunchKernelGGL((conv_halo2<16, 7>), grid, dim3(512), 0, s, p, g); return SEG_OK;
                case 9: hipLaunchKernelGGL((conv_halo2<16, 9>), grid, dim3(512), 0, s, p, g); return SEG_OK;
            }
        }
#endif
        if (p.epi.unpool_y) {
            if (dtype == SEG_F16) hipLaunchKernelGGL((conv_halo2<16, 0, f16, true>), grid, dim3(512), 0, s, p, g);
            else hipLaunchKernelGGL((conv_halo2<16, 0, bf16, true>), grid, dim3(512), 0, s, p, g);
            return SEG_OK;
        }
        if (dtype == SEG_F16) {
            if (hp.bw == 16) hipLaunchKernelGGL((conv_halo2<16, 0, f16>), grid, dim3(512), 0, s, p, g);
            else hipLaunchKernelGGL((conv_halo2<32, 0, f16>), grid, dim3(512), 0, s, p, g);
        } else {
            if (hp.bw == 16) hipLaunchKernelGGL((conv_halo2<16>), grid, dim3(512), 0, s, p, g);
            else hipLaunchKernelGGL((conv_halo2<32>), grid, dim3(512), 0, s, p, g);
        }
        return SEG_OK;
    }
    const bool duo = kernel == HALO_KDUO;
    switch (hp.bw * 10 + hp.hi) {
        case 166: launch_halo_bn<16, 6>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
        case 167: launch_halo_bn<16, 7>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
        case 326: launch_halo_bn<32, 6>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
        case 327: launch_halo_bn<32, 7>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
        case 646: launch_halo_bn<64, 6>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
        default: launch_halo_bn<64, 7>(p, g, hp.bn, hp.tiles, gridz, duo, s, dtype); break;
    }
    return SEG_OK;
}

}  // namespace seg
