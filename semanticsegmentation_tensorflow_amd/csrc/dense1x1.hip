// Persistent streaming 1x1 convolution for FC-DenseNet's bottleneck layers
// (Network/model/FCDenseNet.py:23-35: BN -> ReLU -> 1x1 conv (4*growth = 64
// filters) -> dropout over the dense block's concat).  The op is HBM-bound:
// per pixel it reads C <= 256 input channels and writes <= 64 outputs, at
// ~2*64 MACs per byte.  The tile-per-block implicit GEMM (igemm_nt2_pro) spends
// most of each short block in load latency (1.9-2.7 TB/s); here one block per
// CU streams pixel tiles through a 6-deep LDS-DMA ring that does not drain at
// tile boundaries:
//  * step s = (pixel tile i, 64-channel k tile kk) of the block's tiles
//    t = blockIdx.x + i * gridDim.x; the DMA of step s + 5 is issued when
//    step s starts, so ~5 k tiles (up to 80 KiB) per CU are always in flight;
//    each wave stages and consumes its own 16 pixel rows: no barriers;
//  * the filter (<= 64 x 256) and the BatchNorm (scale, shift) table stay in
//    LDS for the whole kernel;
//  * MFMA on D^T = W . relu(BN(x))^T, so a lane holds 4 consecutive output
//    channels of one pixel: the epilogue (bias / ReLU / dropout, TF1 counter
//    mask) stores 8 bytes per lane straight from the accumulators, no LDS
//    staging; lanes past the last pixel store into a trash page so every
//    wave issues the same number of vector-memory instructions per step,
//    which keeps the counted `s_waitcnt vmcnt` exact.
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

namespace seg {

static __device__ uint4 s1_zero[4];
static __device__ uint2 s1_trash[64 * 64];

namespace {

constexpr int S1_TP = 128;       // pixels per tile (8 waves x 16)
constexpr int S1_NST = 6;        // ring stages of S1_TP x 64 channels
constexpr int S1_MAXC = 256;
constexpr int S1_NW = 8;
constexpr int S1_DMA = S1_TP / 8 / S1_NW;   // DMA instructions per wave per step (2)

// wait until at most n younger vector-memory instructions are outstanding
__device__ __forceinline__ void wait_vm_rt(int n) {
    switch (n) {
#define W_(k) case k: wait_vmcnt<k>(); return;
        W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
        W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29) W_(30)
#undef W_
        default: wait_vmcnt<31>(); return;
    }
}

// STAGED: the wave's 16 x 64 output tile (and the BN2 map) leaves through the
// wave's consumed ring rows as 16-byte stores of whole 128-byte rows (2 per
// lane per map) instead of 8-byte stores of 32-byte row pieces (4 per lane)
template <typename T, bool PRO, bool STAGED = false>
__global__ __launch_bounds__(512, 1) void conv1x1_stream(NTParams p, int ntiles, int kt) {
    constexpr int S1_ST = STAGED ? 2 : 4;      // epilogue stores per wave per tile and map
    constexpr int STG = S1_TP * 128;
    __shared__ __attribute__((aligned(16))) char ring[S1_NST * STG];            // 96 KiB
    __shared__ __attribute__((aligned(16))) char wsm[64 * S1_MAXC * 2];          // 32 KiB
    __shared__ __attribute__((aligned(16))) float ptab[2 * S1_MAXC];
    __shared__ __attribute__((aligned(16))) float etab[4][64];   // scale, shift + bias, BN2 scale, BN2 shift

    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, fg = lane >> 4;
    const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ Wt = reinterpret_cast<const T*>(p.w);
    const EpiParams& e = p.epi;
    const int rowb = kt * 128;                       // filter row bytes in LDS

    // ---- resident filter [n][kk][chunk ^ swz(n)], BN table, epilogue table
    for (int i = tid; i < 64 * kt * 8; i += 512) {
        const int c8 = i & 7, kk = (i >> 3) % kt, n = i / (8 * kt);
        const int c = kk * 64 + c8 * 8;
        uint4 v = {0u, 0u, 0u, 0u};
        if (n < p.N && c < p.K) v = *reinterpret_cast<const uint4*>(Wt + (long)n * p.w_col + c);
        *reinterpret_cast<uint4*>(wsm + n * rowb + kk * 128 + 16 * (c8 ^ ((n >> 1) & 7))) = v;
    }
    if constexpr (PRO) {
        for (int k = tid; k < kt * 64; k += 512) {
            const bool v = k < p.pro.cv;
            ptab[2 * k] = v ? p.pro.gamma[k] * p.pro.inv : 0.f;
            ptab[2 * k + 1] = v ? p.pro.beta[k] : 0.f;
        }
    }
    if (tid < 64) {
        const bool cv = tid < e.n_valid;
        etab[0][tid] = (e.scale && cv) ? e.scale[tid] : 1.f;
        etab[1][tid] = ((e.shift && cv) ? e.shift[tid] : 0.f) + ((e.bias && cv) ? e.bias[tid] : 0.f);
        const bool c2 = e.y2 && tid < e.bn2_cv;
        etab[2][tid] = c2 ? e.bn2_gamma[tid] * e.bn2_inv : 0.f;
        etab[3][tid] = c2 ? e.bn2_beta[tid] : 0.f;
    }
    const int stn = e.y2 ? 2 * S1_ST : S1_ST;        // epilogue stores per wave per tile

    // ---- x DMA: every wave stages its own 16 pixel rows (w*16 + q*8 + lr,
    // physical chunk lane & 7, row swizzle (row >> 1) & 7), so the waves never
    // wait for each other: no barrier in the loop, one wave's VALU epilogue /
    // BN prologue overlaps another's load wait
    const int lr = lane >> 3;
    const int nmine = ntiles > (int)blockIdx.x ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
    const int S = nmine * kt;
    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)ring;
    auto issue = [&](int s) {
        const int i = s / kt, kk = s - (s / kt) * kt;
        const int t = (int)blockIdx.x + i * (int)gridDim.x;
        const unsigned sb = lds0 + (s % S1_NST) * STG;
#pragma unroll
        for (int q = 0; q < S1_DMA; ++q) {
            const int row = w * 16 + q * 8 + lr;
            const int c = (lane & 7) ^ ((q * 4 + (lr >> 1)) & 7);
            const int ch = kk * 64 + c * 8;
            const long m = (long)t * S1_TP + row;
            const bool ok = m < p.M && ch < p.K;
            const void* src = ok ? (const void*)(X + m * p.ldx + ch) : (const void*)s1_zero;
            glds16(src, sb + (w * 2 + q) * 1024);   // lane L -> row w*16 + q*8 + L/8, chunk L%8
        }
    };
    // outstanding vector-memory instructions issued after DMA(s) when step s
    // starts: the DMAs of steps s+1 .. s+NST-2 and the epilogue stores of the
    // steps since DMA(s) was issued
    auto younger = [&](int s) {
        int n = S1_DMA * (min(S - 1, s + S1_NST - 2) - s);
        for (int j = max(0, s - S1_NST + 1); j < s; ++j)
            if (j % kt == kt - 1) n += stn;
        return n;
    };
    for (int s = 0; s < S1_NST - 1 && s < S; ++s) issue(s);
    __syncthreads();                                 // filter / tables visible

    f32x4 acc[4];
#pragma unroll
    for (int nf = 0; nf < 4; ++nf) acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int xrow = w * 16 + fr;                    // this lane's B-fragment pixel row
    for (int s = 0; s < S; ++s) {
        wait_vm_rt(younger(s));
        // the wave's own step s - 1 reads of the stage it re-fills are done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (s + S1_NST - 1 < S) issue(s + S1_NST - 1);
        const int kk = s % kt;
        const char* Xs = ring + (s % S1_NST) * STG;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int chunk = ks * 4 + fg;
            uint4 xb = *reinterpret_cast<const uint4*>(Xs + xrow * 128 + 16 * (chunk ^ ((xrow >> 1) & 7)));
            if constexpr (PRO) {
                float ss[16];
                const float4* tp = reinterpret_cast<const float4*>(ptab + 2 * (kk * 64 + chunk * 8));
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t4 = tp[q];
                    ss[4 * q] = t4.x; ss[4 * q + 1] = t4.y; ss[4 * q + 2] = t4.z; ss[4 * q + 3] = t4.w;
                }
                xb = pro_affine8<T>(xb, ss, p.pro.relu);
            }
#pragma unroll
            for (int nf = 0; nf < 4; ++nf) {
                const int n = nf * 16 + fr;
                const uint4 wa = *reinterpret_cast<const uint4*>(wsm + n * rowb + kk * 128 + 16 * (chunk ^ ((n >> 1) & 7)));
                acc[nf] = mfma16x16x32<T>(wa, xb, acc[nf]);     // D^T[n][px]
            }
        }
        if (kk == kt - 1) {
            // lane: channels nf*16 + 4*fg .. +3 of pixel m
            const int t = (int)blockIdx.x + (s / kt) * (int)gridDim.x;
            const long m = (long)t * S1_TP + xrow;
            const uint64_t gidx = (uint64_t)m * e.n_valid;
            uint2 ob[4], ob2[4];
#pragma unroll
            for (int nf = 0; nf < 4; ++nf) {
                const int col0 = nf * 16 + 4 * fg;
                const f32x4 sc4 = *reinterpret_cast<const f32x4*>(&etab[0][col0]);
                const f32x4 ad4 = *reinterpret_cast<const f32x4*>(&etab[1][col0]);
                T o[4];
                const SegDropRun<4> drop(e.seed, gidx + col0, e.keep_prob < 1.f);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = acc[nf][j] * sc4[j] + ad4[j];
                    if (e.relu) v = fmaxf(v, 0.f);
                    if (e.keep_prob < 1.f) v = drop(v, e.keep_prob, j);
                    o[j] = from_f32<T>(col0 + j < e.n_valid ? v : 0.f);
                }
                const bool ok = m < p.M && col0 < p.N;
                ob[nf] = *reinterpret_cast<const uint2*>(o);
                if constexpr (!STAGED) {
                    uint2* dst = ok ? reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.y) + m * p.ldy + col0)
                                    : s1_trash + (tid & 4095);
                    *dst = ob[nf];
                }
                if (e.y2) {      // BN2(+ReLU) of the stored values (seg_bn_relu_fwd's arithmetic)
                    const f32x4 s2 = *reinterpret_cast<const f32x4*>(&etab[2][col0]);
                    const f32x4 t2 = *reinterpret_cast<const f32x4*>(&etab[3][col0]);
                    T o2[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        float v2 = __builtin_fmaf(to_f32(o[j]), s2[j], t2[j]);
                        if (e.bn2_relu) v2 = fmaxf(v2, 0.f);
                        o2[j] = from_f32<T>(v2);
                    }
                    ob2[nf] = *reinterpret_cast<const uint2*>(o2);
                    if constexpr (!STAGED) {
                        uint2* dst2 = ok ? reinterpret_cast<uint2*>(reinterpret_cast<T*>(e.y2) + m * e.ld_y2 + col0)
                                         : s1_trash + (tid & 4095);
                        *dst2 = ob2[nf];
                    }
                }
                acc[nf] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (STAGED) {
                // this step's stage rows of the wave (16 x 128 B) are consumed
                char* Sw = const_cast<char*>(Xs) + w * 2048;
                const int row = lane >> 2;
                const long mr = (long)t * S1_TP + w * 16 + row;
                auto flush = [&](const uint2* v, T* base, int ld) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int nf = 0; nf < 4; ++nf)
                        *reinterpret_cast<uint2*>(Sw + fr * 128 + 16 * ((2 * nf + (fg >> 1)) ^ ((fr >> 1) & 7)) +
                                                  8 * (fg & 1)) = v[nf];
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int c = (lane & 3) * 2 + h;
                        const uint4 q = *reinterpret_cast<const uint4*>(Sw + row * 128 + 16 * (c ^ ((row >> 1) & 7)));
                        const bool ok = mr < p.M && c * 8 < p.N;
                        uint4* dst = ok ? reinterpret_cast<uint4*>(base + mr * ld + c * 8)
                                        : reinterpret_cast<uint4*>(s1_trash) + (tid & 2047);
                        *dst = q;
                    }
                };
                flush(ob, reinterpret_cast<T*>(p.y), p.ldy);
                if (e.y2) flush(ob2, reinterpret_cast<T*>(e.y2), e.ld_y2);
            }
        }
    }
    wait_vmcnt<0>();
}

// ---------------------------------------------------------------------------
// The bottleneck conv's input gradient through the BN(+ReLU) before it
// (seg_conv2d_bwd_data_bn, 1x1 form: FC-DenseNet.py:27 backward into the
// BN of :25-26), streamed: dx[m][c] = BNbwd(sum_k dz[m][k] W[c][k]) over
// k < 64, accumulated into the concat gradient.  Per pixel it reads 64
// dz + C x + C old-dx channels and writes C, at 128 MACs per C -- HBM-bound,
// and the tile-per-block igemm_nt2_bn spent each block in one load latency.
// Here a block owns one 64-channel chunk of the output for a contiguous range
// of 128-pixel tiles (blocks of one tile range and different chunks sit on
// one XCD, so the dz rows they share come from its L2); every wave stages and
// consumes its own 16 pixel rows (dz, x and old dx of its chunk: 6 LDS-DMA
// instructions per step) through a 3-deep ring without barriers; the chunk's
// filter fragments stay in VGPRs; MFMA on D^T = W . dz^T so a lane holds 4
// consecutive channels of one pixel and finishes them from the staged x / old
// dx; the BN column sums stay in VGPRs until the block's last tile.
// ---------------------------------------------------------------------------
constexpr int B1_TP = 128;       // pixels per tile (8 waves x 16)
constexpr int B1_NST = 3;        // ring depth (steps)
constexpr int B1_WST = 3 * 16 * 128;                  // per wave per step: dz, x, old dx rows
template <typename T>
__global__ __launch_bounds__(512, 1) void bn1x1_dgrad_stream(NTParams p, int nch, int G, int ntiles) {
    constexpr int B1_ST = 4;      // 8-byte dx stores per wave per step
    __shared__ __attribute__((aligned(16))) char ring[B1_NST * 8 * B1_WST];   // 144 KiB
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, fg = lane >> 4, lr = lane >> 3;
    const EpiParams& e = p.epi;
    const int b = blockIdx.x;
    const int chunk = (b >> 3) % nch, bx = ((b >> 3) / nch) * 8 + (b & 7);
    const int t0 = (int)((long)bx * ntiles / G), t1 = (int)((long)(bx + 1) * ntiles / G);
    const int S = t1 - t0;
    const int c0 = chunk * 64;
    const bool res = e.residual != nullptr;
    const int ndma = res ? 6 : 4;
    const T* __restrict__ DZ = reinterpret_cast<const T*>(p.x);
    const T* __restrict__ BX = reinterpret_cast<const T*>(e.bn_x);
    const T* __restrict__ RS = reinterpret_cast<const T*>(e.residual);
    const int hw = p.OH * p.OW;

    // the chunk's filter fragments (A operand: row n = ni*16 + fr, k = ks*32 + 8 fg)
    uint4 wf[4][2];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int n = c0 + ni * 16 + fr;
            wf[ni][ks] = n < p.N ? *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(p.w) + (long)n * p.w_col +
                                                                   ks * 32 + fg * 8)
                                 : uint4{0u, 0u, 0u, 0u};
        }
    // BN (scale, shift) of the lane's 16 channels
    float bsc[4][4], bsh[4][4], sgm[4][4], sbt[4][4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = c0 + ni * 16 + 4 * fg + j;
            const bool cv = col < e.bn_cv;
            bsc[ni][j] = cv ? e.bn_gamma[col] * e.bn_inv : 0.f;
            bsh[ni][j] = cv ? e.bn_beta[col] : 0.f;
            sgm[ni][j] = sbt[ni][j] = 0.f;
        }

    const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)ring;
    auto issue = [&](int s) {
        const int t = t0 + s;
        const unsigned sb = lds0 + ((s % B1_NST) * 8 + w) * B1_WST;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int row = q * 8 + lr;                   // wave-local pixel row
            const int c = (lane & 7) ^ ((q * 4 + (lr >> 1)) & 7);
            const int m = t * B1_TP + w * 16 + row;
            const bool mok = m < p.M;
            const int mm = mok ? m : 0;
            const int img = mm / hw, pix = mm - img * hw;
            const bool cok = mok && c0 + c * 8 < p.N;
            const void* zs = (const void*)s1_zero;
            glds16(mok ? (const void*)(DZ + img * p.x_img + (long)pix * p.ldx + c * 8) : zs, sb + q * 1024);
            glds16(cok ? (const void*)(BX + img * e.bn_x_img + (long)pix * e.ld_bn_x + c0 + c * 8) : zs,
                   sb + 2048 + q * 1024);
            if (res)
                glds16(cok ? (const void*)(RS + img * e.res_img + (long)pix * e.ld_res + c0 + c * 8) : zs,
                       sb + 4096 + q * 1024);
        }
    };
    // vector-memory instructions issued after DMA(s) when step s starts: the
    // stores of steps s-2, s-1 and the DMA of step s+1
    auto younger = [&](int s) { return B1_ST * min(2, s) + (s + 1 < S ? ndma : 0); };
    for (int s = 0; s < B1_NST - 1 && s < S; ++s) issue(s);

    const int sw = (fr >> 1) & 7;                        // row swizzle of the lane's pixel row
    for (int s = 0; s < S; ++s) {
        wait_vm_rt(younger(s));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // own reads of the stage refilled next
        if (s + B1_NST - 1 < S) issue(s + B1_NST - 1);
        const char* Ws = ring + ((s % B1_NST) * 8 + w) * B1_WST;
        f32x4 acc[4];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const uint4 zb = *reinterpret_cast<const uint4*>(Ws + fr * 128 + 16 * ((ks * 4 + fg) ^ sw));
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) acc[ni] = mfma16x16x32<T>(wf[ni][ks], zb, acc[ni]);   // D^T[n][px]
        }
        const int m = (t0 + s) * B1_TP + w * 16 + fr;
        const bool mok = m < p.M;
        const int mm = mok ? m : 0;
        const int img = mm / hw, pix = mm - img * hw;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
            const int col0 = c0 + ni * 16 + 4 * fg;
            const int off = fr * 128 + 16 * ((2 * ni + (fg >> 1)) ^ sw) + 8 * (fg & 1);
            const uint2 xr = *reinterpret_cast<const uint2*>(Ws + 2048 + off);
            const T* xh = reinterpret_cast<const T*>(&xr);
            uint2 rr = uint2{0u, 0u};
            if (res) rr = *reinterpret_cast<const uint2*>(Ws + 4096 + off);
            const T* rh = reinterpret_cast<const T*>(&rr);
            T o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = col0 + j;
                const float xv = to_f32(xh[j]);
                const bool on = col < e.bn_cv && (!e.bn_relu || xv * bsc[ni][j] + bsh[ni][j] > 0.f);
                const float dz = on ? acc[ni][j] : 0.f;
                sgm[ni][j] += dz * xv;
                sbt[ni][j] += dz;
                float x = dz * bsc[ni][j];
                if (res) x += to_f32(rh[j]);
                o[j] = from_f32<T>(col < e.n_valid ? x : 0.f);
            }
            const bool ok = mok && col0 < p.N;
            uint2* dst = ok ? reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.y) + img * p.y_img +
                                                       (long)pix * p.ldy + col0)
                            : s1_trash + (tid & 4095);
            *dst = *reinterpret_cast<const uint2*>(o);
        }
    }
    wait_vmcnt<0>();
    // BN column sums: lanes fr share channels -> butterfly, then the 8 waves
    // meet in LDS; one partial row per tile range (block x), this chunk's columns
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                sgm[ni][j] += __shfl_xor(sgm[ni][j], o);
                sbt[ni][j] += __shfl_xor(sbt[ni][j], o);
            }
    __syncthreads();
    float* red = reinterpret_cast<float*>(ring);     // [8 waves][2 kinds][64 columns]
    if (fr == 0) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int lc = ni * 16 + 4 * fg + j;
                red[(w * 2 + 0) * 64 + lc] = sgm[ni][j];
                red[(w * 2 + 1) * 64 + lc] = sbt[ni][j];
            }
    }
    __syncthreads();
    if (tid < 128) {
        const int kind = tid >> 6, lc = tid & 63;
        float sum = 0.f;
        for (int w_ = 0; w_ < 8; ++w_) sum += red[(w_ * 2 + kind) * 64 + lc];
        if (c0 + lc < e.bn_C) e.bn_part[(long)bx * 2 * e.bn_C + kind * e.bn_C + c0 + lc] = sum;
    }
}

}  // namespace

// y = epilogue(W . relu(BN(x))): single-tap 1x1 stride-1, N <= 64, C <= 256,
// dense pixel rows (x_img / y_img are whole images of ldx / ldy rows),
// no residual / mask epilogue
bool s1x1_ok(const NTParams& p, int dtype, int nphases) {
    return g_s1x1 && (dtype == SEG_BF16 || dtype == SEG_F16) && nphases == 1 && !p.phase && p.K == p.C &&
           p.taps_w == 1 && p.ish == 1 && p.isw == 1 && p.ioh == 0 && p.iow == 0 && p.osh == 1 && p.osw == 1 &&
           p.IH == p.Ha && p.IW == p.Wa && p.OH == p.Ha && p.OW == p.Wa && p.x_img == (long)p.IH * p.IW * p.ldx &&
           p.y_img == (long)p.OH * p.OW * p.ldy && p.N <= 64 && p.K <= S1_MAXC && p.K % 8 == 0 && p.ldx % 8 == 0 &&
           p.ldy % 4 == 0 && ((uintptr_t)p.x % 16) == 0 && ((uintptr_t)p.y % 8) == 0 && !p.epi.residual &&
           !p.epi.mask && !p.epi.bn_x && p.M > 0 &&
           (!p.epi.y2 || (p.epi.ld_y2 % 4 == 0 && ((uintptr_t)p.epi.y2 % 8) == 0 && p.epi.y2_img == (long)p.OH * p.OW * p.epi.ld_y2));
}

// The 1x1 input gradient through the BN backward on bn1x1_dgrad_stream: K = 64
// (the bottleneck's 4 * growth filters), dense 1x1 stride-1 geometry, 16-bit.

// geometry (from the descriptor alone: it also fixes the partial-row count)
bool bn1x1s_ok(const NTParams& p, int dtype) {
    return g_bn1x1s && (dtype == SEG_BF16 || dtype == SEG_F16) && !p.phase && p.K == 64 && p.C == 64 &&
           p.taps_w == 1 && p.ish == 1 && p.isw == 1 && p.ioh == 0 && p.iow == 0 && p.osh == 1 && p.osw == 1 &&
           p.ooh == 0 && p.oow == 0 && p.IH == p.Ha && p.IW == p.Wa && p.OH == p.Ha && p.OW == p.Wa &&
           p.N % 8 == 0 && p.M > 0 && p.M % (p.OH * p.OW) == 0 && p.ldx % 8 == 0 && p.ldy % 4 == 0 &&
           p.w_col % 8 == 0 && p.x_img % 8 == 0;
}

// the launch's operands (16-byte DMA rows, 8-byte stores)
static bool bn1x1s_args_ok(const NTParams& p) {
    const EpiParams& e = p.epi;
    return e.bn_x && e.ld_bn_x % 8 == 0 && e.bn_x_img % 8 == 0 && !e.mask && e.keep_prob >= 1.f &&
           (!e.residual || (e.ld_res % 8 == 0 && e.res_img % 8 == 0 && ((uintptr_t)e.residual % 16) == 0)) &&
           ((uintptr_t)p.x % 16) == 0 && ((uintptr_t)e.bn_x % 16) == 0 && ((uintptr_t)p.y % 8) == 0 &&
           ((uintptr_t)p.w % 16) == 0;
}

// blocks per 64-channel chunk (= the BN partial rows): a multiple of 8, one
// block per CU over all chunks
int bn1x1s_rows(const NTParams& p, int cus) {
    const int nch = (p.N + 63) / 64;
    const int ntiles = (p.M + B1_TP - 1) / B1_TP;
    int G = std::max(8, (cus / nch) & ~7);
    return std::min(G, std::max(8, (ntiles + 7) & ~7));
}


int launch_bn1x1s(NTParams& p, int dtype, int cus, hipStream_t s) {
    if (!bn1x1s_args_ok(p)) return SEG_EINVAL;
    const int nch = (p.N + 63) / 64;
    const int ntiles = (p.M + B1_TP - 1) / B1_TP;
    const int G = bn1x1s_rows(p, cus);
    const dim3 grid(nch * G);
    if (dtype == SEG_F16) hipLaunchKernelGGL((bn1x1_dgrad_stream<f16>), grid, dim3(512), 0, s, p, nch, G, ntiles);
    else hipLaunchKernelGGL((bn1x1_dgrad_stream<bf16>), grid, dim3(512), 0, s, p, nch, G, ntiles);
    return SEG_OK;
}

// staged 16-byte output stores: 0 never, 1 for single-k-tile launches (C <= 64:
// write-dominated, 393 vs 475 us at 384x1248x8, C = 48; C3 212 -> 213.5 img/s),
// 2 always (C = 128 / 144: 1-4 % slower)

template <typename T, bool PRO>
static void launch_s1x1_t(NTParams& p, int grid, int ntiles, int kt, bool st, hipStream_t s) {
    if (st) hipLaunchKernelGGL((conv1x1_stream<T, PRO, true>), dim3(grid), dim3(512), 0, s, p, ntiles, kt);
    else hipLaunchKernelGGL((conv1x1_stream<T, PRO, false>), dim3(grid), dim3(512), 0, s, p, ntiles, kt);
}

void launch_s1x1(NTParams& p, int dtype, int cus, hipStream_t s) {
    const int ntiles = (p.M + S1_TP - 1) / S1_TP;
    const int kt = (p.K + 63) / 64;
    const int grid = std::min(ntiles, cus);
    const bool pro = p.pro.gamma != nullptr;
    const bool st = (g_s1x1_st == 2 || (g_s1x1_st == 1 && kt == 1)) && p.N % 8 == 0 && p.ldy % 8 == 0 &&
                    ((uintptr_t)p.y % 16) == 0 &&
                    (!p.epi.y2 || (p.epi.ld_y2 % 8 == 0 && ((uintptr_t)p.epi.y2 % 16) == 0));
    if (dtype == SEG_F16) {
        if (pro) launch_s1x1_t<f16, true>(p, grid, ntiles, kt, st, s);
        else launch_s1x1_t<f16, false>(p, grid, ntiles, kt, st, s);
    } else {
        if (pro) launch_s1x1_t<bf16, true>(p, grid, ntiles, kt, st, s);
        else launch_s1x1_t<bf16, false>(p, grid, ntiles, kt, st, s);
    }
}

}  // namespace seg
