// Whole-image filter gradient (Conv2DBackpropFilter) for large filters on
// small feature maps -- FCN's conv6, 7x7 over 12x39 at batch 4
// (Network/model/FCN.py:78) -- optionally fused with TF1 Adam on the filter
// (Network/model/FCN.py:338-340), bf16 operands, fp32 accumulation (gfx950).
//
//   dW[r][s][c][n] = sum_p x[p + (r*dil - pad_t, s*dil - pad_l)][c] * dy[p][n]
//
// The implicit-GEMM TN kernel (igemm_tn3) gathers the im2col'd activation
// panel from L2 once per output tile: for conv6 that is 3 GB of L2 -> LDS
// traffic for 385 GFLOP, and the 256x128 tiles that let the fused Adam's HBM
// update overlap another block's MFMAs were bound by it.  Here a block owns
// ALL R*S taps x 16 input channels x 32 output channels (25,088 fp32
// accumulators for 7x7) and stages, per image, the whole zero-padded input
// image of its 16 channels in LDS (18 x 45 px x 32 B = 26 KB for conv6); every
// tap reads its A fragments from that image at a per-tap row offset, and only
// dy (64 B per pixel) is streamed.  L2 -> LDS traffic per block: 104 KB of
// images + 120 KB of dy for 94 MFLOP (~8x less per FLOP than the tiles), so
// the MFMA phase leaves the memory path to the other block on the CU, whose
// epilogue streams its 25,088 parameters' p / m / v from HBM (two 256-thread
// blocks per CU, 72 KiB LDS each).
//
//  * waves: 4; wave w owns taps w, w+4, w+8, ... (13 or 12 of 49) x 2 n
//    fragments of 16 columns; per 32-pixel k-step a wave reads 2 B and one A
//    fragment per tap (ds_read_b64_tr_b16, as wgrad_halo) for 2 MFMAs per tap.
//  * pixels: images concatenated, each padded to a multiple of 32 pixel
//    slots; slots past OH*OW read dy = 0 (the A row is clamped in range).
//  * LDS: two image buffers (image i+1 staged while i is consumed) and a
//    4-stage dy ring of 64-pixel stages (1 KiB DMA piece per wave per stage);
//    one counted `s_waitcnt vmcnt` + barrier per stage.  Images: 32-byte rows,
//    byte address a stored at a ^ ((a >> 1) & 128) (rows 8 apart land on
//    different bank halves); dy: 64-byte rows, a ^ ((a >> 4) & 32).  Both
//    swizzles are involutions applied on the DMA source side.
//  * epilogue: per accumulator element, fp32 gradient store, or TF1 Adam
//    (p, m, v read-modify-write in HWIO order + the bf16 HWIO copy) -- 16
//    lanes cover 64 contiguous bytes of a (tap, c) row.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

static __device__ uint4 wi_zero_page[4];

int g_wgrad_img = 1;

struct WIGeom {
    int hh, hw;          // staged image: rows (OH + (R-1) dil) x cols (OW + (S-1) dil)
    int kpi;             // 32-pixel k-steps per image
    int nimg, rs, S, dil;
    int nst;             // 64-pixel dy stages over all images
    int nct, nnt;        // channel tiles (16), column tiles (32)
};

constexpr int WI_NW = 4, WI_CB = 16, WI_NB = 32, WI_TPW = 13;   // taps per wave (max)
constexpr int WI_XP = 7;                                          // image DMA pieces per wave
constexpr int WI_XBUF = WI_XP * WI_NW * 1024;                     // 28 KiB
constexpr int WI_NST = 4;                                         // dy ring stages
constexpr int WI_DBUF = 64 * WI_NB * 2;                           // 4 KiB
constexpr int WI_SMEM = 2 * WI_XBUF + WI_NST * WI_DBUF;           // 72 KiB

__device__ __forceinline__ unsigned wi_xswz(unsigned a) { return a ^ ((a >> 1) & 128u); }
__device__ __forceinline__ unsigned wi_dswz(unsigned a) { return a ^ ((a >> 4) & 32u); }

template <int N>
__device__ __forceinline__ void wi_wait_upto(int allow) {
    if constexpr (N == 0) {
        wait_vmcnt<0>();
    } else {
        if (allow >= N) wait_vmcnt<N>();
        else wi_wait_upto<N - 1>(allow);
    }
}

// image i + 1 is staged at the first dy stage whose two k-steps both belong to
// images >= i (image i - 1, which shares its buffer, is then fully consumed)
__device__ __forceinline__ int wi_xstage(int i, int kpi) { return (i * kpi + 1) >> 1; }

template <bool ADAM>
__global__ __launch_bounds__(256, 2) void wgrad_img(TNParams p, WIGeom g) {
    using V8 = vec8_t<bf16>;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    __shared__ __attribute__((aligned(1024))) char smem[WI_SMEM];

    const int wg = xcd_remap2(blockIdx.x, gridDim.x);
    const int nt = wg / g.nct, ct = wg - (wg / g.nct) * g.nct;   // consecutive blocks share dy columns
    if (nt >= g.nnt) return;
    const int c0 = ct * WI_CB, n0 = nt * WI_NB;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bf16* __restrict__ X = reinterpret_cast<const bf16*>(p.x);
    const bf16* __restrict__ Dy = reinterpret_cast<const bf16*>(p.b);
    const void* zero = (const void*)wi_zero_page;
    const int OHW = p.Ha * p.Wa;
    const int hrows = g.hh * g.hw;
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
    const unsigned ldsD = lds0 + 2 * WI_XBUF;

    // ---- staging: image img of this block's 16 channels into buffer buf
    auto stage_image = [&](int img, int buf) {
        const long xb = (long)img * p.x_img + c0;
#pragma unroll
        for (int k = 0; k < WI_XP; ++k) {
            const unsigned P = (unsigned)((k * WI_NW + w) * 1024 + lane * 16);
            const unsigned a = wi_xswz(P);
            const int row = (int)(a >> 5), half = (int)((a >> 4) & 1u);
            const void* src = zero;
            if (row < hrows) {
                const int hy = row / g.hw, hx = row - (row / g.hw) * g.hw;
                const int iy = hy + p.ioh, ix = hx + p.iow;
                if ((unsigned)iy < (unsigned)p.IH && (unsigned)ix < (unsigned)p.IW)
                    src = (const void*)(X + xb + ((long)iy * p.IW + ix) * p.ldx + half * 8);
            }
            glds16(src, lds0 + buf * WI_XBUF + (k * WI_NW + w) * 1024);
        }
    };
    // ---- staging: dy stage st (64 pixel slots x 32 columns) into its ring slot
    auto stage_dy = [&](int st) {
        const unsigned P = (unsigned)(w * 1024 + lane * 16);
        const unsigned a = wi_dswz(P);
        const int r = (int)(a >> 6), chunk = (int)((a >> 4) & 3u);
        const int ks = st * 2 + (r >> 5);
        const int img = ks / g.kpi;
        const int pix = (ks - img * g.kpi) * 32 + (r & 31);
        const void* src = zero;
        if (img < g.nimg && pix < OHW)
            src = (const void*)(Dy + ((long)img * OHW + pix) * p.ldb + n0 + chunk * 8);
        glds16(src, ldsD + (st % WI_NST) * WI_DBUF + w * 1024);
    };
    // outstanding DMA pieces of this wave younger than dy stage st's
    auto younger = [&](int st) {
        int n = 0;
        const int j0 = st - (WI_NST - 1);          // stage that issued dy(st); -1 = prologue
        auto ximg_at = [&](int j) {                // image staged at stage j (>= 1) or -1
            for (int i = 1; i + 1 < g.nimg; ++i)
                if (wi_xstage(i, g.kpi) == j) return i + 1;
            return -1;
        };
        if (j0 < 0) {
            n += max(0, min(WI_NST - 2, g.nst - 1) - st);   // later prologue dy stages
            if (g.nimg > 1) n += WI_XP;            // image 1
            for (int j = 0; j < st; ++j) {
                if (j + WI_NST - 1 < g.nst) ++n;
                if (ximg_at(j) >= 0) n += WI_XP;
            }
        } else {
            if (ximg_at(j0) >= 0) n += WI_XP;
            for (int j = j0 + 1; j < st; ++j) {
                if (j + WI_NST - 1 < g.nst) ++n;
                if (ximg_at(j) >= 0) n += WI_XP;
            }
        }
        return n;
    };

    // ---- prologue: image 0, dy stages 0 .. NST-2, image 1
    stage_image(0, 0);
    for (int j = 0; j < WI_NST - 1; ++j)
        if (j < g.nst) stage_dy(j);
    if (g.nimg > 1) stage_image(1, 1);

    // ---- per-lane fragment geometry (wgrad_halo's transposed-read maps)
    const int fg = lane >> 4, tq = (lane & 15) >> 2, tpp = lane & 3;
    const int kk = 8 * fg + tq;                    // pixel rows kk and kk + 4 of a k-step
    const int ntap = (g.rs - w + WI_NW - 1) / WI_NW;
    int toff[WI_TPW];
#pragma unroll
    for (int i = 0; i < WI_TPW; ++i) {
        const int t = w + WI_NW * i;
        const int r = t / g.S, s = t - (t / g.S) * g.S;
        toff[i] = (r * g.hw + s) * g.dil;
    }
    unsigned dlo[2], dhi[2];                       // dy fragment byte offsets in a stage (k-step 0)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        dlo[ni] = wi_dswz((unsigned)(kk * 64 + 32 * ni + 8 * tpp));
        dhi[ni] = wi_dswz((unsigned)((kk + 4) * 64 + 32 * ni + 8 * tpp));
    }
    f32x4 acc[WI_TPW][2];
#pragma unroll
    for (int i = 0; i < WI_TPW; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    int oh_lo = 0, ow_lo = 0, oh_hi = 0, ow_hi = 0, pix_lo = 0;
    for (int st = 0; st < g.nst; ++st) {
        wi_wait_upto<16>(younger(st));
        lds_barrier();
        if (st + WI_NST - 1 < g.nst) stage_dy(st + WI_NST - 1);
        for (int i = 1; i + 1 < g.nimg; ++i)
            if (wi_xstage(i, g.kpi) == st) stage_image(i + 1, (i + 1) & 1);
        SEG_LDS char* Ds = (SEG_LDS char*)smem + 2 * WI_XBUF + (st % WI_NST) * WI_DBUF;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ks = st * 2 + h;
            const int img = ks / g.kpi, kin = ks - img * g.kpi;
            if (img >= g.nimg) continue;
            if (kin == 0) {                         // first k-step of an image
                pix_lo = kk;
                oh_lo = kk / p.Wa; ow_lo = kk - oh_lo * p.Wa;
                oh_hi = (kk + 4) / p.Wa; ow_hi = (kk + 4) - oh_hi * p.Wa;
            } else {
                pix_lo += 32;
                ow_lo += 32; while (ow_lo >= p.Wa) { ow_lo -= p.Wa; ++oh_lo; }
                ow_hi += 32; while (ow_hi >= p.Wa) { ow_hi -= p.Wa; ++oh_hi; }
            }
            // slots past the image: any in-range row (their dy rows are zero)
            const int blo = pix_lo < OHW ? oh_lo * g.hw + ow_lo : 0;
            const int bhi = pix_lo + 4 < OHW ? oh_hi * g.hw + ow_hi : 0;
            SEG_LDS char* Xs = (SEG_LDS char*)smem + (img & 1) * WI_XBUF;
            V8 bq[2];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Ds + h * 2048 + dlo[ni]));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Ds + h * 2048 + dhi[ni]));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bq[ni] = __builtin_bit_cast(V8, v);
            }
            auto afrag = [&](int i) {
                const unsigned alo = wi_xswz((unsigned)((blo + toff[i]) * 32 + 8 * tpp));
                const unsigned ahi = wi_xswz((unsigned)((bhi + toff[i]) * 32 + 8 * tpp));
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Xs + alo));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Xs + ahi));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                return __builtin_bit_cast(V8, v);
            };
            V8 a_cur = afrag(0);
#pragma unroll
            for (int i = 0; i < WI_TPW; ++i) {
                V8 a_nxt = a_cur;
                if (i + 1 < WI_TPW && i + 1 < ntap) a_nxt = afrag(i + 1);
                if (i < ntap) {
                    acc[i][0] = mfma_v8<bf16>(a_cur, bq[0], acc[i][0]);
                    acc[i][1] = mfma_v8<bf16>(a_cur, bq[1], acc[i][1]);
                }
                a_cur = a_nxt;
            }
        }
    }

    // ---- epilogue: element (tap, c, n) = acc[i][ni][j], c = c0 + 4 fg + j, n = n0 + 16 ni + (lane & 15)
    const int fr = lane & 15;
    const auto& A = p.adam;
#pragma unroll
    for (int i = 0; i < WI_TPW; ++i) {
        if (i >= ntap) continue;
        const int tap = w + WI_NW * i;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = c0 + 4 * fg + j;
            if (c >= p.c_valid) continue;
            const long eo = (long)tap * p.o_tap + (long)c * p.o_c + n0 + fr;
            if constexpr (ADAM) {
                float pv[2], mv[2], vv[2];
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    if (n0 + 16 * ni + fr >= p.n_valid) continue;
                    pv[ni] = A.p[eo + 16 * ni];
                    mv[ni] = A.m[eo + 16 * ni];
                    vv[ni] = A.v[eo + 16 * ni];
                }
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    const int n = n0 + 16 * ni + fr;
                    if (n >= p.n_valid) continue;
                    const float gc = acc[i][ni][j] * A.gs;
                    const float mj = A.b1 * mv[ni] + (1.f - A.b1) * gc;
                    const float vj = A.b2 * vv[ni] + (1.f - A.b2) * gc * gc;
                    const float np = pv[ni] - A.lr_t * mj / (sqrtf(vj) + A.eps);
                    A.p[eo + 16 * ni] = np;
                    A.m[eo + 16 * ni] = mj;
                    A.v[eo + 16 * ni] = vj;
                    if (A.store_grad) p.out[eo + 16 * ni] = acc[i][ni][j];
                    if (A.rows)
                        reinterpret_cast<bf16*>(A.rows)[((long)tap * A.rows_ap + c) * A.rows_bp + n] = (bf16)np;
                }
            } else {
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    if (n0 + 16 * ni + fr < p.n_valid) p.out[eo + 16 * ni] = acc[i][ni][j];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool wgrad_img_geom(const TNParams& p, int dtype, WIGeom* g) {
    if (!g_wgrad_img || dtype != SEG_BF16) return false;
    if (p.ish != 1 || p.isw != 1 || p.tsh != p.tsw || p.tsh < 1 || p.o_n != 1) return false;
    const int S = p.taps_w, RS = p.M / p.Cg, R = RS / S;
    // 3x3 filters stay on wgrad_halo (pixel tiles, split-K): this path is for
    // the 5x5 .. 7x7 filters whose im2col panel the TN tiles re-gather per tap
    if (R * S * p.Cg != p.M || RS > WI_NW * WI_TPW || RS <= 9) return false;
    if (p.Cg % WI_CB || p.N % WI_NB || p.ldx % 8 || p.ldb % 8 || p.c_valid != p.Cg || p.n_valid != p.N) return false;
    if (p.Ha <= 0 || p.Wa <= 0 || p.P % (p.Ha * p.Wa)) return false;
    const int hh = p.Ha + (R - 1) * p.tsh, hw = p.Wa + (S - 1) * p.tsw;
    // the staged image covers every tap's input window: SAME / VALID padding only
    if (p.ioh > 0 || p.iow > 0 || hh * hw * 32 > WI_XBUF) return false;
    g->hh = hh; g->hw = hw;
    g->kpi = (p.Ha * p.Wa + 31) / 32;
    g->nimg = p.P / (p.Ha * p.Wa);
    g->rs = RS; g->S = S; g->dil = p.tsh;
    g->nst = (g->nimg * g->kpi + 1) / 2;
    g->nct = p.Cg / WI_CB; g->nnt = p.N / WI_NB;
    // the image DMA schedule: image 1 (prologue) and image i + 1 (staged at
    // wi_xstage(i)) must be older than the dy stage waited for before their
    // first k-step -- images of at least 2 * NST k-steps
    if (g->nimg > 1 && (g->kpi >> 1) < WI_NST - 1) return false;
    for (int i = 1; i + 1 < g->nimg; ++i)
        if ((((i + 1) * g->kpi) >> 1) < ((i * g->kpi + 1) >> 1) + WI_NST) return false;
    return g->nimg >= 1;
}

bool wgrad_img_ok(const TNParams& p, int dtype) {
    WIGeom g;
    return wgrad_img_geom(p, dtype, &g);
}

void launch_wgrad_img(TNParams& p, hipStream_t s) {
    WIGeom g;
    wgrad_img_geom(p, SEG_BF16, &g);
    const dim3 grid((unsigned)(g.nct * g.nnt)), block(256);
    if (p.adam.p) hipLaunchKernelGGL(wgrad_img<true>, grid, block, 0, s, p, g);
    else hipLaunchKernelGGL(wgrad_img<false>, grid, block, 0, s, p, g);
}

}  // namespace seg
