// First-layer convolution with 8 (padded) input channels: conv1_1 of FCN
// (Network/model/FCN.py:55, 3 -> 64, 3x3 SAME) and the FC-DenseNet stem.
//
// K = 9 taps x 8 channels = 72 is far too shallow for the implicit-GEMM
// kernels (a whole block lives for ~2 k-tiles), and the layer is bound by its
// output write (4 x 384 x 1248 x 64 x 2 B = 123 MB).  Direct form:
//  * v_mfma_f32_16x16x32_bf16 with k = 4 taps x 8 channels: lane group g of an
//    A fragment is ONE tap's 8 channels of one pixel = one 16-byte ds_read_b128
//    from the LDS input halo (taps 9..11 read a zero slot);
//  * the filter (3 k-steps x K/16 fragments) stays in VGPRs for the block;
//  * block = 8 x 64 output pixels, 4 waves x 2 rows, one 16-pixel fragment
//    at a time; bias + ReLU, staged through LDS into 16-byte row stores;
//  * optionally the ReLU mask as bits beside the map (EpiParams::ybits: one
//    byte per 16-byte chunk), read by the next conv's input gradient instead
//    of the 2-byte map (seg_conv2d_fwd_relu_bits).
#include "common.h"
#include "igemm.h"

namespace seg {

namespace {

constexpr int SC_BH = 8, SC_BW = 64;
constexpr int SC_HW = SC_BW + 2;                       // halo width (3x3, dilation 1)
constexpr int SC_HROWS = (SC_BH + 2) * SC_HW;          // 660 halo pixels

// TR (round 6): D^T = W . X^T, so a lane holds 4 consecutive channels of one
// pixel and stages them with one 8-byte LDS write per fragment column block
// instead of four 2-byte ones per channel row (16 -> 4 LDS writes per lane
// and fragment)
template <int NF, typename T, bool TR = false>
__global__ __launch_bounds__(256) void conv_c8_fwd(NTParams p, int tiles_x, int tiles_y) {
    constexpr int KN = NF * 16;
    constexpr int SROW = KN + 8;                       // staged bf16 row (pad vs bank conflicts)
    __shared__ __attribute__((aligned(16))) uint4 halo[SC_HROWS + 1];    // + zero slot
    __shared__ __attribute__((aligned(16))) T stage[4][16 * SROW];

    const int tpi = tiles_x * tiles_y;
    const int img = blockIdx.x / tpi;
    const int rem = blockIdx.x - img * tpi;
    const int ty = rem / tiles_x, tx = rem - (rem / tiles_x) * tiles_x;
    const int oy0 = ty * SC_BH, ox0 = tx * SC_BW;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);

    // ---- halo: pixel (hy, hx) <- x[oy0 + ioh + hy, ox0 + iow + hx, 0..7]
    for (int i = tid; i < SC_HROWS + 1; i += 256) {
        uint4 v = {0u, 0u, 0u, 0u};
        if (i < SC_HROWS) {
            const int hy = i / SC_HW, hx = i - (i / SC_HW) * SC_HW;
            const int ih = oy0 + p.ioh + hy, iw = ox0 + p.iow + hx;
            if ((unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW)
                v = *reinterpret_cast<const uint4*>(X + (long)img * p.x_img + ((long)ih * p.IW + iw) * p.ldx);
        }
        halo[i] = v;
    }
    // ---- filter fragments: lane -> n = nf*16 + (lane&15), tap = ks*4 + (lane>>4)
    const int fr = lane & 15, fg = lane >> 4;
    uint4 bw[3][NF];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
        const int t = ks * 4 + fg;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
            const int n = nf * 16 + fr;
            uint4 v = {0u, 0u, 0u, 0u};
            if (t < 9 && n < p.N) v = *reinterpret_cast<const uint4*>(Wt + (long)n * p.w_col + t * 8);
            bw[ks][nf] = v;
        }
    }
    const EpiParams& e = p.epi;
    float bv[NF][4];        // TR: bias of the lane's channels nf * 16 + 4 fg + j
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = nf * 16 + 4 * fg + j;
            bv[nf][j] = (TR && e.bias && n < e.n_valid) ? e.bias[n] : 0.f;
        }
    __syncthreads();

    // A address of this lane for k-step ks: tap (r, s) of pixel (py, px)
    int toff[3];
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
        const int t = ks * 4 + fg;
        toff[ks] = t < 9 ? (t / 3) * SC_HW + (t % 3) : -1;
    }
    T* st = stage[w];
#pragma unroll 1
    for (int f = 0; f < 2 * SC_BW / 16; ++f) {         // 8 fragments of 16 px per wave
        const int py = w * 2 + f / (SC_BW / 16);
        const int px0 = (f % (SC_BW / 16)) * 16;
        f32x4 acc[NF];
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const int hr = toff[ks] < 0 ? SC_HROWS : py * SC_HW + px0 + fr + toff[ks];
            const uint4 a = halo[hr];
#pragma unroll
            for (int nf = 0; nf < NF; ++nf)
                acc[nf] = TR ? mfma16x16x32<T>(bw[ks][nf], a, acc[nf]) : mfma16x16x32<T>(a, bw[ks][nf], acc[nf]);
        }
        if constexpr (TR) {
            // D^T: lane holds channels n0 + j (n0 = nf*16 + 4*fg) of pixel fr
#pragma unroll
            for (int nf = 0; nf < NF; ++nf) {
                const int n0 = nf * 16 + 4 * fg;
                T o[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = acc[nf][j] + bv[nf][j];
                    if (e.relu) v = fmaxf(v, 0.f);
                    o[j] = from_f32<T>(n0 + j < e.n_valid ? v : 0.f);
                }
                *reinterpret_cast<uint2*>(st + fr * SROW + n0) = *reinterpret_cast<const uint2*>(o);
            }
        } else {
        // D: lane holds rows (pixels) 4*fg + j, column n = nf*16 + fr
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
            const int n = nf * 16 + fr;
            const float b = (e.bias && n < e.n_valid) ? e.bias[n] : 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[nf][j] + b;
                if (e.relu) v = fmaxf(v, 0.f);
                st[(4 * fg + j) * SROW + n] = from_f32<T>(n < e.n_valid ? v : 0.f);
            }
        }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own wave's stage writes
        // 16 px x KN/8 chunks of 16 B
        const int oy = oy0 + py;
#pragma unroll
        for (int q = lane; q < 16 * (KN / 8); q += 64) {
            const int px = q / (KN / 8), ch = q - (q / (KN / 8)) * (KN / 8);
            const int ox = ox0 + px0 + px;
            const bool inb = oy < p.OH && ox < p.OW;
            const uint4 v = *reinterpret_cast<const uint4*>(st + px * SROW + ch * 8);
            if (inb)
                *reinterpret_cast<uint4*>(reinterpret_cast<T*>(p.y) + (long)img * p.y_img +
                                          ((long)oy * p.OW + ox) * p.ldy + ch * 8) = v;
            if (e.ybits) {         // ReLU mask bits of the stored values: byte ch of the pixel's row
                const T* tv = reinterpret_cast<const T*>(&v);
                unsigned b = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) b |= (to_f32(tv[i]) > 0.f ? 1u : 0u) << i;
                unsigned char* row = e.ybits + (((long)img * p.OH + oy) * p.OW + ox) * e.ld_bits;
                if constexpr (KN == 64) {
                    // a pixel's 8 chunks are 8 consecutive lanes: gather its
                    // 64 bits into lane ch == 0 (two quad swaps, one shift by
                    // 4 lanes) for one 8-byte store instead of eight 1-byte ones
                    unsigned wd = b << (8 * (ch & 3));
                    wd |= (unsigned)__builtin_amdgcn_mov_dpp((int)wd, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
                    wd |= (unsigned)__builtin_amdgcn_mov_dpp((int)wd, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
                    const unsigned hi = __shfl_down(wd, 4);
                    if (inb && ch == 0) *reinterpret_cast<uint2*>(row) = uint2{wd, hi};
                } else if (inb) {
                    row[ch] = (unsigned char)b;
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next writes
    }
}

}  // namespace


bool smallc_fwd_ok(const NTParams& p, int dtype, int R, int S, int dil) {
    return g_smallc && (dtype == SEG_BF16 || dtype == SEG_F16) && p.C == 8 && p.K == 72 && R == 3 && S == 3 && dil == 1 && p.ish == 1 &&
           p.isw == 1 && !p.phase && p.N % 16 == 0 && p.N <= 64 && p.N >= 16 && p.ldx == 8 &&
           p.ldy % 8 == 0 && !p.epi.residual && !p.epi.mask && !p.epi.scale && !p.epi.shift &&
           p.epi.keep_prob >= 1.f;
}

template <typename T>
void launch_smallc_fwd_t(NTParams& p, hipStream_t s) {
    const int tx = (p.OW + SC_BW - 1) / SC_BW, ty = (p.OH + SC_BH - 1) / SC_BH;
    const int nimg = p.M / (p.OH * p.OW);
    const dim3 grid(nimg * tx * ty), block(256);
    if (g_smallc_tr) {
        switch (p.N / 16) {
            case 1: hipLaunchKernelGGL((conv_c8_fwd<1, T, true>), grid, block, 0, s, p, tx, ty); break;
            case 2: hipLaunchKernelGGL((conv_c8_fwd<2, T, true>), grid, block, 0, s, p, tx, ty); break;
            case 3: hipLaunchKernelGGL((conv_c8_fwd<3, T, true>), grid, block, 0, s, p, tx, ty); break;
            default: hipLaunchKernelGGL((conv_c8_fwd<4, T, true>), grid, block, 0, s, p, tx, ty); break;
        }
        return;
    }
    switch (p.N / 16) {
        case 1: hipLaunchKernelGGL((conv_c8_fwd<1, T>), grid, block, 0, s, p, tx, ty); break;
        case 2: hipLaunchKernelGGL((conv_c8_fwd<2, T>), grid, block, 0, s, p, tx, ty); break;
        case 3: hipLaunchKernelGGL((conv_c8_fwd<3, T>), grid, block, 0, s, p, tx, ty); break;
        default: hipLaunchKernelGGL((conv_c8_fwd<4, T>), grid, block, 0, s, p, tx, ty); break;
    }
}

void launch_smallc_fwd(NTParams& p, int dtype, hipStream_t s) {
    if (dtype == SEG_F16) launch_smallc_fwd_t<f16>(p, s);
    else launch_smallc_fwd_t<bf16>(p, s);
}

// ---------------------------------------------------------------------------
// Single-tap NT problems with a reduction of K <= 16: y[m][n] =
// epilogue(sum_k x[m][k] w[n][k]).  The input gradient of a classifier head
// over a few classes (FC-DenseNet final_conv 256 -> 2, Network/model/
// FCDenseNet.py:160: dx[3.8 M px][256] from dlogits[.][2]) is a pure write
// stream -- 2 B read per 256 B written -- that the 256 x 64 tile kernel ran
// at 1.6 TB/s.  Here a thread owns 8 consecutive columns of one pixel
// (consecutive threads walk the columns: 16-byte stores, 8 threads per 128 B),
// the filter sits in LDS as fp32 [k][n] (a k step reads 32 contiguous bytes per
// lane, consecutive lanes adjacent: no bank conflicts), the sum runs in k
// order, and the epilogue is igemm_nt2's (bias, BN affine, ReLU, dropout,
// residual, ReluGrad).
// ---------------------------------------------------------------------------
namespace {
constexpr int SK_MAXK = 16, SK_MAXN = 1024, SK_RPT = 16, SK_UNR = 4;

// KK: the reduction rounded up to 2, 4, 8 or 16 (filter zero-padded), so the
// k loop unrolls without per-k branches
// abl (diagnostic build only, garbage results): 1 no operand loads, 2 no stores
template <typename T, int KK>
__global__ __launch_bounds__(256) void smallk_nt_k(NTParams p, int abl) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];   // [KK][N]
    const int K = p.K, NN = p.N;
    const EpiParams& e = p.epi;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ RS = reinterpret_cast<const T*>(e.residual);
    const T* __restrict__ MK = reinterpret_cast<const T*>(e.mask);
    // thread -> (pixel row, 8-column chunk); the block owns SK_RPT x PB
    // consecutive pixels (pass r: pixels base + r * PB .. + PB - 1, one
    // contiguous run of output rows), SK_UNR passes' loads in flight at once,
    // the filter staged once per block
    const int CK = p.N / 8, PB = 256 / CK;
    const int prow = threadIdx.x / CK, ck = threadIdx.x - prow * CK;
    const int col0 = ck * 8;
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    for (int i = threadIdx.x; i < NN * KK; i += 256) {
        const int n = i / KK, k = i - (i / KK) * KK;
        wsm[k * NN + n] = k < K ? to_f32(Wt[(long)n * p.w_col + k]) : 0.f;
    }
    __syncthreads();
    if (prow >= PB) return;
    float sc[8], ad[8], bs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int col = col0 + j;
        const bool cv = col < e.n_valid;
        sc[j] = (e.scale && cv) ? e.scale[col] : 1.f;
        ad[j] = (e.shift && cv) ? e.shift[col] : 0.f;
        bs[j] = (e.bias && cv) ? e.bias[col] : 0.f;
    }
    constexpr int XQ = (KK + 7) / 8;
    const int base = blockIdx.x * (SK_RPT * PB) + prow;
    T* __restrict__ Y = reinterpret_cast<T*>(p.y);
    for (int r0 = 0; r0 < SK_RPT; r0 += SK_UNR) {
        uint4 xq[SK_UNR][XQ], rq[SK_UNR], mq[SK_UNR];
#pragma unroll
        for (int u = 0; u < SK_UNR; ++u) {
            const long m = base + (r0 + u) * PB;
            const bool ok = m < p.M && !(abl & 1);
            const long mm = ok ? m : 0;             // dense pixel rows (smallk_ok)
#pragma unroll
            for (int q = 0; q < XQ; ++q)
                xq[u][q] = ok ? *reinterpret_cast<const uint4*>(X + mm * p.ldx + q * 8) : uint4{0u, 0u, 0u, 0u};
            rq[u] = mq[u] = uint4{0u, 0u, 0u, 0u};
            if (ok && RS) rq[u] = *reinterpret_cast<const uint4*>(RS + mm * e.ld_res + col0);
            if (ok && MK) mq[u] = *reinterpret_cast<const uint4*>(MK + mm * e.ld_mask + col0);
        }
#pragma unroll
        for (int u = 0; u < SK_UNR; ++u) {
            const long m = base + (r0 + u) * PB;
            if (m >= p.M) break;
            float xv[XQ * 8];
#pragma unroll
            for (int q = 0; q < XQ; ++q) Chunk<T>::unpack(xq[u][q], xv + q * 8);
            float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < KK; ++k) {
                const float4 w0 = *reinterpret_cast<const float4*>(wsm + k * NN + col0);
                const float4 w1 = *reinterpret_cast<const float4*>(wsm + k * NN + col0 + 4);
                const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] += xv[k] * wk[j];
            }
            float res[8], mk[8];
            Chunk<T>::unpack(rq[u], res);
            Chunk<T>::unpack(mq[u], mk);
            const uint64_t gidx = ((uint64_t)m) * e.n_valid;
            const SegDropRun<8> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int col = col0 + j;
                const bool cv = col < e.n_valid;
                float x = v[j] * sc[j] + ad[j] + bs[j];
                if (e.relu) x = fmaxf(x, 0.f);
                if (e.keep_prob < 1.f) x = drop(x, e.keep_prob, j);
                if (RS) x += res[j];
                if (MK) x = mk[j] > 0.f ? x * e.mask_scale : 0.f;
                v[j] = cv ? x : 0.f;
            }
            if (!(abl & 2) || v[0] == -1234.5f) *reinterpret_cast<uint4*>(Y + m * p.ldy + col0) = Chunk<T>::pack(v);
        }
    }
}
}  // namespace


bool smallk_ok(const NTParams& p, int dtype) {
    return g_smallk && (dtype == SEG_BF16 || dtype == SEG_F16) && !p.phase && p.taps_w == 1 && p.K == p.C &&
           p.K <= SK_MAXK && p.K > 0 && p.N % 8 == 0 && p.N <= SK_MAXN && p.ish == 1 && p.isw == 1 && p.ioh == 0 &&
           p.iow == 0 && p.osh == 1 && p.osw == 1 && p.ooh == 0 && p.oow == 0 && p.IH == p.Ha && p.IW == p.Wa &&
           p.OH == p.Ha && p.OW == p.Wa && p.M > 0 && p.M % (p.OH * p.OW) == 0 && p.ldx % 8 == 0 &&
           p.ldy % 8 == 0 && !p.pro.gamma && !p.epi.bn_x && !p.epi.pool_y && !p.epi.y2 &&
           p.x_img == (long)p.OH * p.OW * p.ldx && p.y_img == (long)p.OH * p.OW * p.ldy &&
           (!p.epi.residual || p.epi.res_img == (long)p.OH * p.OW * p.epi.ld_res) &&
           (!p.epi.mask || p.epi.mask_img == (long)p.OH * p.OW * p.epi.ld_mask) &&
           (!p.epi.residual || p.epi.ld_res % 8 == 0) && (!p.epi.mask || p.epi.ld_mask % 8 == 0);
}

template <typename T>
static void launch_smallk_t(NTParams& p, int grid, hipStream_t s) {
    // the valid reduction only: the padded channels' products are exact zeros
    // added to a +0-started sum, so dropping them changes no bit
    const int kr = p.kv > 0 && p.kv < p.K ? p.kv : p.K;
    const int kk = kr <= 2 ? 2 : kr <= 4 ? 4 : kr <= 8 ? 8 : 16;
    const size_t lds = (size_t)p.N * kk * sizeof(float);
    switch (kk) {
        case 2: hipLaunchKernelGGL((smallk_nt_k<T, 2>), dim3(grid), dim3(256), lds, s, p, g_smallk_abl); break;
        case 4: hipLaunchKernelGGL((smallk_nt_k<T, 4>), dim3(grid), dim3(256), lds, s, p, g_smallk_abl); break;
        case 8: hipLaunchKernelGGL((smallk_nt_k<T, 8>), dim3(grid), dim3(256), lds, s, p, g_smallk_abl); break;
        default: hipLaunchKernelGGL((smallk_nt_k<T, 16>), dim3(grid), dim3(256), lds, s, p, g_smallk_abl); break;
    }
}

void launch_smallk(NTParams& p, int dtype, int cus, hipStream_t s) {
    const int pb = 256 / (p.N / 8);                  // pixels per block pass
    const int grid = (p.M + pb * SK_RPT - 1) / (pb * SK_RPT);
    (void)cus;
    if (dtype == SEG_F16) launch_smallk_t<f16>(p, grid, s);
    else launch_smallk_t<bf16>(p, grid, s);
}


// ---------------------------------------------------------------------------
// Filter gradient of the same layer: dW[r][s][c][n] = sum_p x[p + (r,s)][c] dz[p][n]
// computed as D[n][j] = sum_p dz[p][n] * X2[p][j] with k = pixels, where a
// 16-column B fragment j = (s_off, c) of tap pair (r, s0..s0+1) is 32
// contiguous bytes of the [px][8] halo starting at pixel (py + r, px + s0):
// taps are paired horizontally, the s0+1 == 3 half is computed and dropped.
// Both operands come from LDS with ds_read_b64_tr_b16 (k = pixels).
//  * tile = 4 x 64 output pixels; halo (4+2) x (64+2) px x 16 B; dz tile
//    256 px x N x 2 B; both staged by LDS-DMA, double buffered.
//  * 4 waves = (N half) x (tap-pair half): 2 n-fragments x 3 pair fragments.
//  * split-K over tile ranges -> fp32 slabs (+ BiasAddGrad row) -> reducer.
// ---------------------------------------------------------------------------
namespace {

constexpr int WC_BH = 4, WC_BW = 64, WC_TP = WC_BH * WC_BW;      // 256 px per tile
constexpr int WC_HW = WC_BW + 2;
constexpr int WC_HROWS = (WC_BH + 2) * WC_HW;                     // 396
constexpr int WC_HPAD = 448;                                      // 7 x 64 DMA rows (>= 396 + 1)

struct WCGeom {
    int tiles_x, tiles_y, ptiles, tps, splits;
};

__device__ __forceinline__ void wc_glds16(const void* gsrc, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

__device__ uint4 wc_zero_page[4];

// N <= 64 (4 n fragments; columns >= N staged as zeros); 6 tap-pair fragments: (r, 0..1), (r, 2..3*) for r = 0..2
template <typename T>
__global__ __launch_bounds__(256) void wgrad_c8(TNParams p, WCGeom g) {
    constexpr int DROWB = 128;                          // 64 dz channels
    constexpr int HBUF = WC_HPAD * 16, DBUF = WC_TP * DROWB, STAGE = HBUF + DBUF;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int split = blockIdx.x;
    const int t_begin = split * g.tps, t_end = min(g.ptiles, t_begin + g.tps);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nh = w & 1, mh = w >> 1;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Dz = reinterpret_cast<const T*>(p.b);
    const void* zero = (const void*)wc_zero_page;
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;

    // DMA: halo 7 instructions per block (1.75 per wave -> waves 0..2 take 2, 3 takes 1),
    // dz: 256 rows x 128 B = 32 instructions (8 per wave), lane -> (row lane>>3, chunk lane&7)
    auto stage_tile = [&](int t, int buf) {
        const int tpi = g.tiles_x * g.tiles_y;
        const int img = t / tpi;
        const int rem = t - img * tpi;
        const int ty = rem / g.tiles_x, tx = rem - (rem / g.tiles_x) * g.tiles_x;
        const int oy0 = ty * WC_BH, ox0 = tx * WC_BW;
        const unsigned sb = lds0 + buf * STAGE;
        for (int q = w; q < WC_HPAD / 64; q += 4) {
            const int hr = q * 64 + lane;
            const int hy = hr / WC_HW, hx = hr - (hr / WC_HW) * WC_HW;
            const int ih = oy0 + p.ioh + hy, iw = ox0 + p.iow + hx;
            const bool ok = hr < WC_HROWS && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
            const void* src = ok ? (const void*)(X + (long)img * p.x_img + ((long)ih * p.IW + iw) * p.ldx) : zero;
            wc_glds16(src, sb + q * 1024);
        }
        const int lr = lane >> 3, pc = lane & 7;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int r = (i * 4 + w) * 8 + lr;                 // dz tile row (pixel)
            const int ch = pc ^ ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2));
            const int oy = oy0 + r / WC_BW, ox = ox0 + r % WC_BW;
            const bool ok = oy < p.Ha && ox < p.Wa && ch * 8 < p.N;     // N < 64: zero columns
            const void* src = ok ? (const void*)(Dz + (((long)img * p.Ha + oy) * p.Wa + ox) * p.ldb + ch * 8) : zero;
            wc_glds16(src, sb + HBUF + (i * 4 + w) * 1024);
        }
    };

    f32x4 acc[2][3];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = p.dbias != nullptr && mh == 0;
    float dsum[2] = {0.f, 0.f};
    const int fg = lane >> 4, tq = (lane & 15) >> 2, tpp = lane & 3;
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    // tap-pair fragments of this wave: mf = mh*3 + i -> (r = mf / 2, s0 = (mf % 2) * 2)
    int poff[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int mf = mh * 3 + i;
        poff[i] = (mf >> 1) * WC_HW + (mf & 1) * 2;
    }

    if (t_begin < t_end) stage_tile(t_begin, 0);
    int buf = 0;
    for (int t = t_begin; t < t_end; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (t + 1 < t_end) stage_tile(t + 1, buf ^ 1);
        const char* Hs = smem + buf * STAGE;
        const char* Ds = Hs + HBUF;
#pragma unroll 2
        for (int ks = 0; ks < WC_TP / 32; ++ks) {
            const int kk = ks * 32 + 8 * fg + tq;                  // pixel of this lane's lo row
            const int py = kk / WC_BW, px = kk - (kk / WC_BW) * WC_BW;
            vec8_t<T> af[2], bfr[3];
            const int d1 = (((kk >> 1) & 1) << 1) | (((kk >> 3) & 1) << 2);
            const int d2 = ((((kk + 4) >> 1) & 1) << 1) | ((((kk + 4) >> 3) & 1) << 2);
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int chk = nh * 4 + ni * 2 + (tpp >> 1);
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Ds + kk * DROWB + 16 * (chk ^ d1) + 8 * (tpp & 1)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Ds + (kk + 4) * DROWB + 16 * (chk ^ d2) + 8 * (tpp & 1)));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                af[ni] = __builtin_bit_cast(vec8_t<T>, v);
                if (do_bias) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) dsum[ni] += bits16_to_f32<T>((unsigned short)v[e]);
                }
            }
            const int hb = py * WC_HW + px;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int h1 = hb + poff[i];
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Hs + h1 * 16 + 8 * tpp));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(Hs + (h1 + 4) * 16 + 8 * tpp));
                s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bfr[i] = __builtin_bit_cast(vec8_t<T>, v);
            }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    acc[ni][i] = mfma_v8<T>(af[ni], bfr[i], acc[ni][i]);
        }
        buf ^= 1;
    }

    // D[n][j]: lane holds n = nfrag*16 + 4*fg + jj, j = lane & 15 -> (s_off = j >> 3, c = j & 7)
    const int j = lane & 15, soff = j >> 3, c = j & 7;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int mf = mh * 3 + i, r = mf >> 1, s = (mf & 1) * 2 + soff;
        if (s >= 3) continue;
        const int m = (r * 3 + s) * p.Cg + c;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int n = nh * 32 + ni * 16 + 4 * fg + jj;
                const float v = acc[ni][i][jj];
                if (p.partial) {
                    if (n < p.N) p.partial[((long)split * p.Mp + m) * p.N + n] = v;
                } else if (c < p.c_valid && n < p.n_valid) {
                    p.out[(long)(r * 3 + s) * p.o_tap + (long)c * p.o_c + (long)n * p.o_n] = v;
                }
            }
    }
    if (do_bias) {
        const int fr = lane & 15;
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            dsum[ni] += __shfl_xor(dsum[ni], 16);
            dsum[ni] += __shfl_xor(dsum[ni], 32);
            const int n = nh * 32 + ni * 16 + fr;
            if (fg == 0) {
                if (p.partial) {
                    if (n < p.N) p.partial[((long)split * p.Mp + p.M) * p.N + n] = dsum[ni];
                } else if (n < p.n_valid) {
                    p.dbias[n] = dsum[ni];
                }
            }
        }
    }
}

}  // namespace

bool smallc_wgrad_ok(const TNParams& p, int dtype) {
    return g_smallc && (dtype == SEG_BF16 || dtype == SEG_F16) && p.Cg == 8 && p.M == 72 && p.taps_w == 3 && p.ish == 1 && p.isw == 1 &&
           p.tsh == 1 && p.tsw == 1 && p.N % 16 == 0 && p.N >= 16 && p.N <= 64 && p.ldx == 8 && p.ldb % 8 == 0 &&
           p.ldb >= p.N && p.Ha > 0 && p.Wa > 0 &&
           p.P % (p.Ha * p.Wa) == 0;
}

int smallc_wgrad_splits(const TNParams& p, int cus) {
    const int nimg = p.P / (p.Ha * p.Wa);
    const int ptiles = nimg * ((p.Wa + WC_BW - 1) / WC_BW) * ((p.Ha + WC_BH - 1) / WC_BH);
    const int want = std::min(ptiles, 2 * cus);
    const int tps = (ptiles + want - 1) / want;
    return (ptiles + tps - 1) / tps;
}

void launch_smallc_wgrad(TNParams& p, int dtype, int splits, hipStream_t s) {
    WCGeom g;
    g.tiles_x = (p.Wa + WC_BW - 1) / WC_BW;
    g.tiles_y = (p.Ha + WC_BH - 1) / WC_BH;
    g.ptiles = (p.P / (p.Ha * p.Wa)) * g.tiles_x * g.tiles_y;
    g.tps = (g.ptiles + splits - 1) / splits;
    g.splits = splits;
    if (dtype == SEG_F16) hipLaunchKernelGGL(wgrad_c8<f16>, dim3(splits), dim3(256), 0, s, p, g);
    else hipLaunchKernelGGL(wgrad_c8<bf16>, dim3(splits), dim3(256), 0, s, p, g);
}

}  // namespace seg
