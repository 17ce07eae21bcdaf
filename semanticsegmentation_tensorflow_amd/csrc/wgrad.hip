// Halo-tiled filter gradient (Conv2DBackpropFilter) for stride-1 3x3 convs,
// bf16 operands, fp32 accumulation (gfx950).
//
//   dW[r][s][c][n] = sum_p x[p + (r*dil_h - pad_t, s*dil_w - pad_l)][c] * dy[p][n]
//
// The implicit-GEMM TN kernel (igemm_tn2) re-gathers the shifted activation
// rows once per tap.  Here a block owns one 64-channel chunk c0 x NT output
// channels with ALL 9 taps accumulated in registers (M tile = 9 x 64 rows) and
// walks a contiguous range of 128-pixel tiles (BH x BW output pixels).  Per
// tile it LDS-DMAs the x halo ((BH+2dil) x (BW+2dil) px x 128 B) and the dy
// tile (128 px x NT) once; every tap reads its A fragments from the halo at a
// row offset, so each activation byte crosses L2 -> LDS once per tile instead
// of nine times.
//
//  * fragments: ds_read_b64_tr_b16 on pixel-major images (k = pixels), the
//    same operand maps as igemm_tn2; 128 B / 256 B rows XOR-swizzled on the
//    DMA source side.
//  * waves: 4 (16-channel fragment of the chunk) x 2 (N halves); per 32-pixel
//    substep a wave issues 9 x 2 A + NF x 2 B transposed reads for 9 x NF MFMAs.
//  * pipeline: 2 LDS stages, tile t+1 staged right after the barrier that
//    retires tile t; one barrier per tile (36 x NF MFMAs per wave between).
//  * split-K over pixel-tile ranges -> fp32 slabs + splitk_reduce_tn.
//  * PXS (64-wide dy tiles, round 6): the waves split the tile's pixels
//    instead of its columns -- wave (cf, ph) owns all 64 columns for
//    substeps 2 ph, 2 ph + 1 -- so each A fragment read feeds 4 MFMAs instead
//    of 2 (conv1_2's filter gradient, 64 -> 64, was bound by the LDS fragment
//    reads: 22 per 18 MFMAs); each half writes its own split-K slab (slab
//    2 split + ph), so the reducer adds twice the partials.  (Adding the
//    halves through LDS instead spilled 48-65 VGPRs.)
//
// Covers the 3x3 layers of FCN (Network/model/FCN.py:55-99) and FC-DenseNet.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

static __device__ uint4 wg_zero_page[4];


struct WGGeom {
    int tiles_x, tiles_y, nimg, hwd, hrows;
    int nct, nnt, splits, tps, ptiles;
    int nbias;    // fused BiasAddGrad spread over the first nbias channel blocks
};

template <int ROWB>
__device__ __forceinline__ int wg_swz(int row) {
    if constexpr (ROWB >= 256) return ((row & 3) << 1) | (((row >> 3) & 1) << 3);
    else if constexpr (ROWB == 64) return 0;     // 4-chunk dy rows (NT = 32): unswizzled
    else return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

// NST LDS stages (tile t+NST-1 in flight while t is consumed); HI halo DMA
// pieces per wave (8 rows each): 4 covers dilation 1, 5 dilation 2.
// ABL (diagnostic builds, garbage results): 1 no DMA in the loop, 2 no MFMA,
// 3 no LDS fragment reads.
template <int NT, int NST, int HI, int ABL = 0, typename T = bf16, bool PXS = false>
__global__ __launch_bounds__(512) void wgrad_halo(TNParams p, WGGeom g) {
    constexpr int BW = 16;
    using V8 = vec8_t<T>;
    constexpr int NW = 8, BH = 128 / BW;
    constexpr int NF = PXS ? NT / 16 : NT / 32;   // n fragments per wave
    static_assert(!PXS || NT == 64, "pixel-split waves hold all 64 columns");
    constexpr int DROWB = NT * 2;             // dy tile row bytes
    constexpr int D_RPI = 1024 / DROWB;       // dy rows per DMA instruction
    constexpr int D_INS = 128 / D_RPI / NW;   // dy DMA instructions per wave
    constexpr int D_CPR = DROWB / 16;
    constexpr int HBUF = HI * NW * 1024;
    constexpr int DBUF = 128 * DROWB;
    constexpr int STAGE = HBUF + DBUF;
    static_assert(BW == 16 || BW == 32, "8-pixel fragment groups must stay in one tile row");
    __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

    const int nout = g.nct * g.nnt;
    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int split = wg / nout, ot = wg - (wg / nout) * nout;
    if (split >= g.splits) return;
    const int ct = ot / g.nnt, nt = ot - (ot / g.nnt) * g.nnt;
    const int c0 = ct * 64, n0 = nt * NT;
    const int t_begin = split * g.tps, t_end = min(g.ptiles, t_begin + g.tps);

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cf = w & 3;
    const int nh = PXS ? 0 : w >> 2;          // column half (PXS: all columns)
    const int ph = PXS ? w >> 2 : 0;          // PXS: pixel half (substeps 2 ph, 2 ph + 1)
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Dy = reinterpret_cast<const T*>(p.b);
    const void* zero = (const void*)wg_zero_page;

    // ---- halo DMA: row (h*NW + w)*8 + lr, global chunk hc (swizzle is h-independent)
    const int lr = lane >> 3;
    const int hc = (lane & 7) ^ ((((lr >> 1) & 1) << 1) | ((w & 1) << 2));
    int h_hy[HI], h_hx[HI];
#pragma unroll
    for (int h = 0; h < HI; ++h) {
        const int hr = (h * NW + w) * 8 + lr;
        h_hy[h] = hr < g.hrows ? hr / g.hwd : -(1 << 20);
        h_hx[h] = hr < g.hrows ? hr - (hr / g.hwd) * g.hwd : 0;
    }
    const int h_n = g.hrows > w * 8 ? min(HI, (g.hrows - w * 8 + NW * 8 - 1) / (NW * 8)) : 0;
    // ---- dy DMA: row (i*NW + w)*D_RPI + dr, global chunk dc
    const int dr = lane / D_CPR, dpc = lane % D_CPR;
    int dc;
    if constexpr (DROWB >= 256) dc = dpc ^ (((dr & 3) << 1) | (((w >> 1) & 1) << 3));
    else if constexpr (DROWB == 64) dc = dpc;
    else dc = dpc ^ ((((dr >> 1) & 1) << 1) | ((w & 1) << 2));
    const bool d_nok = n0 + dc * 8 < p.N;

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    auto stage_tile = [&](int t, int buf) {
        const int tpi = g.tiles_x * g.tiles_y;
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / g.tiles_x, tx = rem - (rem / g.tiles_x) * g.tiles_x;
        const int oy0 = ty * BH, ox0 = tx * BW;
        const long xb = (long)img * p.x_img + c0 + hc * 8;
        const unsigned sb = lds0 + buf * STAGE;
#pragma unroll
        for (int h = 0; h < HI; ++h) {
            if (h < h_n) {
                const int ih = oy0 + p.ioh + h_hy[h], iw = ox0 + p.iow + h_hx[h];
                const bool ok = (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
                const void* src = ok ? (const void*)(X + xb + ((long)ih * p.IW + iw) * p.ldx) : zero;
                glds16(src, sb + (h * NW + w) * 1024);
            }
        }
#pragma unroll
        for (int i = 0; i < D_INS; ++i) {
            const int r = (i * NW + w) * D_RPI + dr;
            const int oy = oy0 + r / BW, ox = ox0 + r % BW;
            const bool ok = d_nok && oy < p.Ha && ox < p.Wa;
            const void* src =
                ok ? (const void*)(Dy + (((long)img * p.Ha + oy) * p.Wa + ox) * p.ldb + n0 + dc * 8) : zero;
            glds16(src, sb + HBUF + (i * NW + w) * 1024);
        }
    };

    f32x4 acc[9][NF];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fused BiasAddGrad, spread so no wave carries much extra VALU (a block
    // waits for its slowest wave at every tile barrier, and the kernel for its
    // slowest block): channel block ct < nbias sums the dy fragments of the
    // substeps ss = ct (mod nbias), and within it wave cf only fragment ni = cf
    // (8 pixels x column fr per lane).  Each (ct, n) partial goes to its own
    // split-K slab row M + ct (or straight to dbias when nbias == 1).
    const bool do_bias = p.dbias != nullptr && ct < g.nbias && cf < NF;
    float dsum[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) dsum[j] = 0.f;

    const int fg = lane >> 4, tq = (lane & 15) >> 2, tpp = lane & 3;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    int tapoff[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) tapoff[r * 3 + s] = r * p.tsh * g.hwd + s * p.tsw;

    // per-lane LDS byte offsets of every tap's A fragment and of every B
    // fragment, packed two per register (rows kk and kk + 4 as lo | hi << 16;
    // BW = 16, hwd % 8 == 0 so substeps only add a wave-uniform base): one
    // VALU op per fragment read instead of the index / swizzle arithmetic
    unsigned a_pk[9], b_pk[NF];
    {
        const int kk = 8 * fg + tq;
        const int py = kk / BW, px = kk - (kk / BW) * BW;
        const int achk = cf * 2 + (tpp >> 1);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int r1 = py * g.hwd + px + tapoff[t];
            const unsigned lo = r1 * 128 + 16 * (achk ^ wg_swz<128>(r1)) + 8 * (tpp & 1);
            const unsigned hi = (r1 + 4) * 128 + 16 * (achk ^ wg_swz<128>(r1 + 4)) + 8 * (tpp & 1);
            a_pk[t] = lo | (hi << 16);
        }
        const int d1 = wg_swz<DROWB>(kk), d2 = wg_swz<DROWB>(kk + 4);
#pragma unroll
        for (int ni = 0; ni < NF; ++ni) {
            const int chk = ((nh * (NT / 2) + ni * 16) >> 3) + (tpp >> 1);
            const unsigned lo = kk * DROWB + 16 * ((chk & ~15) | ((chk & 15) ^ d1)) + 8 * (tpp & 1);
            const unsigned hi = (kk + 4) * DROWB + 16 * ((chk & ~15) | ((chk & 15) ^ d2)) + 8 * (tpp & 1);
            b_pk[ni] = lo | (hi << 16);
        }
    }
    // per-wave DMA instructions per tile (wave-uniform, tile-independent)
    const int per_tile = h_n + D_INS;
    for (int i = 0; i < NST - 1; ++i)
        if (t_begin + i < t_end) stage_tile(t_begin + i, i);
    int buf = 0;
    for (int t = t_begin; t < t_end; ++t) {
        // tile t landed; the NST-2 younger tiles may still be in flight
        const int younger = min(NST - 2, t_end - 1 - t);
        const int allow = younger * per_tile;
        if (allow <= 0) wait_vmcnt<0>();
        else if (allow <= 2) wait_vmcnt<2>();
        else if (allow <= 3) wait_vmcnt<3>();
        else if (allow <= 4) wait_vmcnt<4>();
        else if (allow <= 5) wait_vmcnt<5>();
        else if (allow <= 6) wait_vmcnt<6>();
        else if (allow <= 7) wait_vmcnt<7>();
        else if (allow <= 8) wait_vmcnt<8>();
        else if (allow <= 9) wait_vmcnt<9>();
        else if (allow <= 10) wait_vmcnt<10>();
        else if (allow <= 11) wait_vmcnt<11>();
        else wait_vmcnt<12>();
        lds_barrier();
        if (ABL != 1 && t + NST - 1 < t_end) stage_tile(t + NST - 1, buf == 0 ? NST - 1 : buf - 1);
        // flat software pipeline over the 36 (substep, tap) steps of the tile:
        // the A fragment of step s+1 (and the B fragments of the next substep)
        // are read while the MFMAs of step s issue
        auto read_b = [&](int ss, V8* bo) {
            if constexpr (ABL == 3) {
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) {
                    s16x8 v = {(short)ss, (short)ni, 1, 2, 3, 4, 5, (short)lane};
                    bo[ni] = __builtin_bit_cast(V8, v);
                }
                return;
            }
#pragma unroll
            for (int ni = 0; ni < NF; ++ni) {
                SEG_LDS char* dbs = (SEG_LDS char*)smem + buf * STAGE + HBUF + ss * 32 * DROWB;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(dbs + (b_pk[ni] & 0xffffu)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(dbs + (b_pk[ni] >> 16)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bo[ni] = __builtin_bit_cast(V8, v);
                if (do_bias && ni == cf && ss % g.nbias == ct) {
#pragma unroll
                    for (int e = 0; e < 8; ++e)
                        dsum[ni] += bits16_to_f32<T>((unsigned short)v[e]);
                }
            }
        };
        auto read_a = [&](int ss, int tap) {
            if constexpr (ABL == 3) {
                s16x8 v = {(short)ss, (short)tap, 1, 2, 3, 4, 5, (short)lane};
                return __builtin_bit_cast(V8, v);
            }
            SEG_LDS char* hb = (SEG_LDS char*)smem + buf * STAGE + ss * (32 / BW) * g.hwd * 128;
            const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(hb + (a_pk[tap] & 0xffffu)));
            const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(hb + (a_pk[tap] >> 16)));
            s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            return __builtin_bit_cast(V8, v);
        };
        const int ss0 = 2 * ph;
        V8 b0[NF], b1[NF];
        read_b(ss0, b0);
        V8 a_cur = read_a(ss0, 0);
        // one substep: 9 taps, A(tap+1) read ahead, next substep's B at tap 4
        // (more: a next substep follows in this wave)
        auto substep = [&](int ss, V8* bc, V8* bn, bool more) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                V8 a_nxt = a_cur;
                if (tap < 8) a_nxt = read_a(ss, tap + 1);
                else if (more) a_nxt = read_a(ss + 1, 0);
                if (tap == 4 && more) read_b(ss + 1, bn);
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) {
                    if constexpr (ABL == 2) asm volatile("" ::"v"(a_cur), "v"(bc[ni]));
                    else acc[tap][ni] = mfma_v8<T>(a_cur, bc[ni], acc[tap][ni]);
                }
                a_cur = a_nxt;
            }
        };
        if constexpr (PXS) {
            substep(ss0, b0, b1, true);
            substep(ss0 + 1, b1, b0, false);
        } else {
#pragma unroll 1
            for (int ss = 0; ss < 4; ss += 2) {
                substep(ss, b0, b1, true);
                substep(ss + 1, b1, b0, ss + 2 < 4);
            }
        }
        buf = buf == NST - 1 ? 0 : buf + 1;
    }
    const int fr = lane & 15;
    const int slab = PXS ? 2 * split + ph : split;
    if (do_bias) {
#pragma unroll
        for (int ni = 0; ni < NF; ++ni) {
            dsum[ni] += __shfl_xor(dsum[ni], 16);
            dsum[ni] += __shfl_xor(dsum[ni], 32);
        }
        if (fg == 0) {
#pragma unroll
            for (int ni = 0; ni < NF; ++ni) {
                if (ni != cf) continue;
                const int n = n0 + nh * (NT / 2) + ni * 16 + fr;
                if (p.partial) {
                    if (n < p.N) p.partial[((long)slab * p.Mp + p.M + ct) * p.N + n] = dsum[ni];
                } else if (n < p.n_valid) {
                    p.dbias[n] = dsum[ni];
                }
            }
        }
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + cf * 16 + fg * 4 + j;
            const int m = tap * p.Cg + c;
            if (p.partial) {
                float* prow = p.partial + ((long)slab * p.Mp + m) * p.N;
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) {
                    const int n = n0 + nh * (NT / 2) + ni * 16 + fr;
                    if (n < p.N) prow[n] = acc[tap][ni][j];
                }
            } else if (c < p.c_valid) {
                float* orow = p.out + (long)tap * p.o_tap + (long)c * p.o_c;
#pragma unroll
                for (int ni = 0; ni < NF; ++ni) {
                    const int n = n0 + nh * (NT / 2) + ni * 16 + fr;
                    if (n < p.n_valid) orow[(long)n * p.o_n] = acc[tap][ni][j];
                }
            }
        }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool wgrad_plan(const TNParams& p, int dtype, int cus, WgradPlan* wp) {
    if (!g_wgrad_halo || (dtype != SEG_BF16 && dtype != SEG_F16)) return false;
    if (p.ish != 1 || p.isw != 1 || p.taps_w != 3 || p.Cg % 64 != 0 || p.M != 9 * p.Cg) return false;
    if (p.tsh <= 0 || p.tsw <= 0 || p.N % 8 != 0 || p.ldb % 8 != 0 || p.ldx % 8 != 0) return false;
    if (p.Ha <= 0 || p.Wa <= 0 || p.P % (p.Ha * p.Wa) != 0) return false;
    const int nimg = p.P / (p.Ha * p.Wa);
    // 16 x 8-pixel tiles (the packed per-lane fragment offsets need 16-pixel
    // rows); halo rows padded to a multiple of 8 so substep shifts keep the swizzle
    const int bw = 16, bh = 128 / bw;
    const int hwd = (bw + 2 * p.tsw + 7) & ~7;
    const int hrows = hwd * (bh + 2 * p.tsh);
    if (hrows > 5 * 64) return false;
    wp->bw = bw;
    wp->g[0] = (p.Wa + bw - 1) / bw; wp->g[1] = (p.Ha + bh - 1) / bh; wp->g[3] = hwd; wp->g[4] = hrows;
    // 128-wide dy tiles (2 LDS stages, 4 halo pieces) when N allows and the halo fits
    wp->nt = (g_wgrad_nt == 128 && p.N > 64 && wp->g[4] <= 4 * 64) ? 128 : 64;
    // <= 32 output channels (FC-DenseNet growth convs, 64 -> 16): 32-wide dy
    // tiles instead of padding to 64 (half the MFMAs, a quarter of the dy LDS)
    if (g_wgrad_nt32 && p.N <= 32) wp->nt = 32;
    wp->g[2] = nimg;
    const int nct = p.Cg / 64, nnt = (p.N + wp->nt - 1) / wp->nt;
    const int nout = nct * nnt;
    const int ptiles = nimg * wp->g[0] * wp->g[1];
    const int tcus = std::max(1, cus * g_wgrad_fill / 100);
    int splits = std::max(1, std::min(ptiles, one_round_splits(nout, tcus, ptiles)));
    const int tps = (ptiles + splits - 1) / splits;
    splits = (ptiles + tps - 1) / tps;
    wp->g[5] = nct; wp->g[6] = nnt; wp->g[7] = splits; wp->g[8] = tps; wp->g[9] = ptiles;
    wp->splits = splits;
    // 64-wide dy tiles (no second column block to share an A fragment read):
    // pixel-split waves, two slabs per split
    wp->pxs = wp->nt == 64 && g_wgrad_pxs && splits > 1;
    wp->slabs = splits * (wp->pxs ? 2 : 1);
    wp->nbias = splits > 1 ? std::max(1, std::min(nct, g_wgrad_nbias)) : 1;
    wp->blocks = (long)nout * splits;
    return true;
}

size_t wgrad_workspace(const WgradPlan& wp, const TNParams& p) {
    // + nbias slab rows for the fused BiasAddGrad partials
    return wp.slabs > 1 ? (size_t)wp.slabs * (p.M + wp.nbias) * p.N * sizeof(float) : 0;
}

void launch_wgrad(TNParams& p, const WgradPlan& wp, hipStream_t s, int dtype) {
    WGGeom g;
    g.tiles_x = wp.g[0]; g.tiles_y = wp.g[1]; g.nimg = wp.g[2]; g.hwd = wp.g[3]; g.hrows = wp.g[4];
    g.nct = wp.g[5]; g.nnt = wp.g[6]; g.splits = wp.g[7]; g.tps = wp.g[8]; g.ptiles = wp.g[9];
    g.nbias = wp.nbias;
    const dim3 grid((unsigned)wp.blocks), block(512);
    const bool small = g.hrows <= 4 * 64;     // 4 halo pieces -> 3 stages fit
#ifdef SEG_DIAG   // ablation builds (garbage results): tools/ only
    if (g_wgrad_abl && wp.nt == 128 && dtype == SEG_BF16) {
        if (g_wgrad_abl == 1) hipLaunchKernelGGL((wgrad_halo<128, 2, 4, 1>), grid, block, 0, s, p, g);
        if (g_wgrad_abl == 2) hipLaunchKernelGGL((wgrad_halo<128, 2, 4, 2>), grid, block, 0, s, p, g);
        if (g_wgrad_abl == 3) hipLaunchKernelGGL((wgrad_halo<128, 2, 4, 3>), grid, block, 0, s, p, g);
        return;
    }
#endif
    if (wp.pxs) {
        if (dtype == SEG_F16) {
            if (small) hipLaunchKernelGGL((wgrad_halo<64, 3, 4, 0, f16, true>), grid, block, 0, s, p, g);
            else hipLaunchKernelGGL((wgrad_halo<64, 2, 5, 0, f16, true>), grid, block, 0, s, p, g);
        } else {
            if (small) hipLaunchKernelGGL((wgrad_halo<64, 3, 4, 0, bf16, true>), grid, block, 0, s, p, g);
            else hipLaunchKernelGGL((wgrad_halo<64, 2, 5, 0, bf16, true>), grid, block, 0, s, p, g);
        }
        return;
    }
    if (dtype == SEG_F16) {
        if (wp.nt == 128) hipLaunchKernelGGL((wgrad_halo<128, 2, 4, 0, f16>), grid, block, 0, s, p, g);
        else if (wp.nt == 32 && small) hipLaunchKernelGGL((wgrad_halo<32, 3, 4, 0, f16>), grid, block, 0, s, p, g);
        else if (wp.nt == 32) hipLaunchKernelGGL((wgrad_halo<32, 2, 5, 0, f16>), grid, block, 0, s, p, g);
        else if (small) hipLaunchKernelGGL((wgrad_halo<64, 3, 4, 0, f16>), grid, block, 0, s, p, g);
        else hipLaunchKernelGGL((wgrad_halo<64, 2, 5, 0, f16>), grid, block, 0, s, p, g);
        return;
    }
    if (wp.nt == 128) hipLaunchKernelGGL((wgrad_halo<128, 2, 4>), grid, block, 0, s, p, g);
    else if (wp.nt == 32 && small) hipLaunchKernelGGL((wgrad_halo<32, 3, 4>), grid, block, 0, s, p, g);
    else if (wp.nt == 32) hipLaunchKernelGGL((wgrad_halo<32, 2, 5>), grid, block, 0, s, p, g);
    else if (small) hipLaunchKernelGGL((wgrad_halo<64, 3, 4>), grid, block, 0, s, p, g);
    else hipLaunchKernelGGL((wgrad_halo<64, 2, 5>), grid, block, 0, s, p, g);
}

}  // namespace seg
