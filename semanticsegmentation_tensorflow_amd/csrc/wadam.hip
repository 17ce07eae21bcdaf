// Conv2DBackpropFilter fused with TF1 Adam for the large fused layers (FCN
// conv6 / conv7: 103 M and 17 M parameters, filter gradient K = 1872 px):
// a persistent, warp-specialized kernel.
//
// The layer is bound by the Adam state stream (p / m / v read + written, the
// bf16 HWIO copy written: 28 B per parameter, 2.9 GB for conv6), not by its
// 385 GFLOP.  igemm_tn3's fused epilogue runs that stream after each tile's
// MFMA loop, so HBM idles during the loop and the MFMA pipes idle during the
// update.  Here every block (one per CU, 8 waves) runs both at once:
//  * waves 0-7 ("MFMA waves", 2 x 4 of 64 x 32, two per SIMD) compute 128 x
//    128 gradient tiles from a 3-stage LDS ring of 64-pixel stages (the
//    gathered x columns and the dy columns, buffer-resource LDS-DMA with
//    32-bit offsets, transposed ds_read_b64_tr_b16 fragment reads, one barrier
//    per stage), then hand the fp32 tile to
//  * waves 8-11 ("update waves") through a 64 KiB LDS staging tile: while the
//    MFMA waves compute tile k+1, the update waves apply Adam to tile k in
//    sixteen half-steps (4 rows x 64 columns per wave) spread over the stage
//    barriers, with the p / m / v loads of the next four steps in flight
//    (branch-free buffer loads / stores: out-of-range lanes carry an offset
//    past num_records).
// Both roles pass every barrier (gfx950 has one workgroup barrier), so a
// period lasts max(MFMA loop, update stream): the update stream, at ~28 B /
// param, is what the kernel is sized to keep busy.
// Tiles: panel-major order (N panel outer, M inner) cut into 8 contiguous
// ranges, one per XCD slot (blockIdx % 8): the 32 CUs of an XCD work on
// neighbouring tiles of the same dy panel, which stays in that XCD's L2.
// The KRSC copy is written afterwards by rows_to_tr_k (conv.hip), as after
// igemm_tn3's fused form.  Arithmetic is igemm_tn3's epilogue expression for
// expression (TF1 ApplyAdam, Network/model/FCN.py:338).
#include "common.h"
#include "igemm.h"
#include "ldsdma.h"

#include <type_traits>

namespace seg {

int g_wadam = 0;   // off until it beats igemm_tn3's fused form
int g_wadam_abl = 0;  // diagnostics (garbage results), bits: 1 update waves idle, 2 MFMA waves idle,
                      // 4 no operand DMA, 8 every tile's operands from tile 0 (L2-hot)
__device__ uint4 g_wadam_zero[4];

__device__ __forceinline__ int wadam_swz(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

// One wave instruction: 64 lanes x 16 B from SGPR buffer base + per-lane 32-bit
// byte offset into 1 KiB of LDS at M0; offsets past num_records land as zeros
// (the padding / tail rows).  Inline asm, as glds16, so the compiler does not
// drain vmcnt before later ds_reads.
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(r), "s"(lds_dst)
                 : "memory");
}

__device__ __forceinline__ void wa_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NST, bool SG, int ABL = 0>
__global__ __launch_bounds__(768) void wgrad_adam_ws(TNParams p, int tiles_m, int tiles_n) {
    static_assert(NST >= 3 && NST <= 6, "ring depth");
    constexpr int MW = 8, BKP = 64;   // MFMA waves (2 x 4 of 64 x 32), pixel rows per stage
    constexpr int BM = 128, BN = 128, ROWB = 256, KS = BKP / 32;
    constexpr int ABUF = BKP * ROWB, STAGE = 2 * ABUF, RING = NST * STAGE;
    constexpr int SROW = BN * 4, STG = BM * SROW;   // rows aligned to the 256-B bank period
    // two MFMA waves per SIMD: one wave's DMA issue and fragment waits overlap
    // the other's MFMAs
    constexpr int NPC = BKP / 4 / MW;               // DMA pieces per operand per MFMA wave per stage
    constexpr int PPW = 2 * NPC;
    constexpr int WTN = 128 / (MW / 2), NI = WTN / 16;
    __shared__ __attribute__((aligned(16))) char smem[RING + STG];
    typedef short s16x8 __attribute__((ext_vector_type(8)));

    const int T = tiles_m * tiles_n;
    const int xs = blockIdx.x & 7, jb = blockIdx.x >> 3, nbx = gridDim.x >> 3;
    const int lo = (int)((long)T * xs / 8), hi = (int)((long)T * (xs + 1) / 8);
    const int first = lo + jb;
    const int nt = first < hi ? (hi - first + nbx - 1) / nbx : 0;
    if (nt == 0) return;
    auto tile_of = [&](int k, int& m0, int& n0) __attribute__((always_inline)) {
        const int q = first + k * nbx;
        const int tn = q / tiles_m;
        m0 = (q - tn * tiles_m) * BM;
        n0 = tn * BN;
    };
    const int nk = (p.P + BKP - 1) / BKP;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* stg = smem + RING;

    if (w < MW) {
        // ================= MFMA waves =================
        const int wm = w / (MW / 2), wn = w % (MW / 2);
        const int nimg = p.P / (p.Ha * p.Wa);
        const __amdgpu_buffer_rsrc_t rx =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.x), (short)0, (int)(2 * nimg * p.x_img), 0x00020000);
        const __amdgpu_buffer_rsrc_t rdy =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.b), (short)0, 2 * p.P * p.ldb, 0x00020000);
        constexpr unsigned OOR = 0x80000000u;
        // DMA: piece i of wave w = stage rows (4 i + w) * 4 .. +3 (1 KiB); a
        // lane's rows in its two pieces differ by 16 -> one swizzled chunk
        const int rsub = lane >> 4, pc = lane & 15;
        const int gc = pc ^ wadam_swz(w * 4 + rsub);
        const unsigned lds0 = (unsigned)(uintptr_t)(SEG_LDS char*)smem;
        const int hw = p.Ha * p.Wa;
        int hoff = 0, woff = 0, ac = 0, bn = 0;
        bool a_mok = false, b_nok = false;
        int pimg[NPC], pa[NPC], pb[NPC], pp[NPC];
        auto setup = [&](int m0, int n0) __attribute__((always_inline)) {
            if (ABL & 8) m0 = n0 = 0;
            const int am = m0 + gc * 8;
            a_mok = am < p.M;
            const int atap = a_mok ? am / p.Cg : 0;
            ac = a_mok ? am - atap * p.Cg : 0;
            const int atj = atap / p.taps_w, ati = atap - atj * p.taps_w;
            hoff = atj * p.tsh + p.ioh;
            woff = ati * p.tsw + p.iow;
            bn = n0 + gc * 8;
            b_nok = bn < p.N;
#pragma unroll
            for (int i = 0; i < NPC; ++i) {
                const int pix = (i * MW + w) * 4 + rsub;
                pp[i] = pix;
                const int q = pix < p.P ? pix : 0;
                pimg[i] = q / hw;
                const int rem = q - pimg[i] * hw;
                pa[i] = rem / p.Wa;
                pb[i] = rem - pa[i] * p.Wa;
            }
        };
        auto issue = [&](int buf) __attribute__((always_inline)) {
            buf = __builtin_amdgcn_readfirstlane(buf);
#pragma unroll
            for (int i = 0; i < NPC; ++i) {
                const int ih = pa[i] * p.ish + hoff, iw = pb[i] * p.isw + woff;
                const bool aok = a_mok && pp[i] < p.P && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
                const unsigned aoffs = aok ? 2u * (unsigned)(pimg[i] * (int)p.x_img + (ih * p.IW + iw) * p.ldx + ac) : OOR;
                blds16(rx, aoffs, lds0 + buf * STAGE + (i * MW + w) * 1024);
                const bool bok = b_nok && pp[i] < p.P;
                blds16(rdy, bok ? 2u * (unsigned)(pp[i] * p.ldb + bn) : OOR, lds0 + buf * STAGE + ABUF + (i * MW + w) * 1024);
                pp[i] += BKP;
                pb[i] += BKP;
                while (pb[i] >= p.Wa) {
                    pb[i] -= p.Wa;
                    if (++pa[i] == p.Ha) { pa[i] = 0; ++pimg[i]; }
                }
            }
        };
        // transposed fragment reads (igemm_tn3's lane offsets at 256-B rows)
        const int fg = lane >> 4, fr = lane & 15;
        const int tq = (lane & 15) >> 2, tpp = lane & 3;
        const int fr1 = 8 * fg + tq, fsw = wadam_swz(fr1);
        auto lane_off = [&](int col0) __attribute__((always_inline)) {
            const int chk = (col0 >> 3) + (tpp >> 1);
            return (unsigned)(fr1 * ROWB + 16 * (chk ^ fsw) + 8 * (tpp & 1));
        };
        unsigned aoff[4], boff[NI];
#pragma unroll
        for (int i = 0; i < 4; ++i) aoff[i] = lane_off(wm * 64 + i * 16);
#pragma unroll
        for (int i = 0; i < NI; ++i) boff[i] = ABUF + lane_off(wn * WTN + i * 16);
        auto frag = [&](SEG_LDS char* a) __attribute__((always_inline)) {
            const s16x4 l4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)a);
            const s16x4 h4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SEG_LDS s16x4*)(a + 4 * ROWB));
            s16x8 v = {l4[0], l4[1], l4[2], l4[3], h4[0], h4[1], h4[2], h4[3]};
            return __builtin_bit_cast(bf16x8, v);
        };

        f32x4 acc[4][NI];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        // Per stage: wait, barrier, fragment reads, the DMA of stage it+NST-1
        // into the slot stage it-1 left (its reads retired at this barrier),
        // MFMAs.  One barrier per stage, shared with the update waves.
        auto wait_stages = [&](int y) __attribute__((always_inline)) {
            if (NST >= 6 && y >= 4) wait_vmcnt<4 * PPW>();
            else if (NST >= 5 && y >= 3) wait_vmcnt<3 * PPW>();
            else if (NST >= 4 && y >= 2) wait_vmcnt<2 * PPW>();
            else if (y >= 1) wait_vmcnt<PPW>();
            else wait_vmcnt<0>();
        };
        int m0, n0;
        auto prologue = [&](int k) __attribute__((always_inline)) {   // stages 0 .. NST-2 of block tile k
            tile_of(k, m0, n0);
            setup(m0, n0);
#pragma unroll
            for (int s = 0; s < NST - 1; ++s)
                if (!(ABL & 6) && s < nk) issue(s);
        };
        prologue(0);
        for (int k = 0; k < nt; ++k) {
            int rbuf = 0, ibuf = NST - 1;
#pragma nounroll
            for (int it = 0; it < nk; ++it) {
                wait_stages(min(NST - 2, nk - 1 - it));   // stage it landed
                wa_bar();   // stage it visible; stage it-1's reads retired; (it == 0) staging published
                if (ABL & 2) continue;
                SEG_LDS char* S = (SEG_LDS char*)smem + rbuf * STAGE;
                bf16x8 af[KS][4], bq[KS][NI];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) af[ks][i] = frag(S + ks * 32 * ROWB + aoff[i]);
#pragma unroll
                    for (int i = 0; i < NI; ++i) bq[ks][i] = frag(S + ks * 32 * ROWB + boff[i]);
                }
                if (!(ABL & 4) && it + NST - 1 < nk) issue(ibuf);
                rbuf = rbuf == NST - 1 ? 0 : rbuf + 1;
                ibuf = ibuf == NST - 1 ? 0 : ibuf + 1;
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                        for (int ni = 0; ni < NI; ++ni)
                            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][mi], bq[ks][ni], acc[mi][ni],
                                                                                  0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
            }
            wa_bar();   // X: ring reads of tile k retired; the update waves are done with the staging
            if (k + 1 < nt) prologue(k + 1);
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int ni = 0; ni < NI; ++ni)
                        *reinterpret_cast<float*>(stg + (wm * 64 + mi * 16 + fg * 4 + r) * SROW +
                                                  (wn * WTN + ni * 16 + fr) * 4) = acc[mi][ni][r];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            // the next tile's first stage barrier publishes the staging
        }
        // the update waves' last period: the nk stage barriers of a tile
        for (int it = 0; it < nk; ++it) wa_bar();
        return;
    }

    // ================= update waves =================
    const auto& A = p.adam;
    const int u = w - MW, rr = lane >> 4, j = lane & 15;
    float pv[4][8], mv[4][8], vv[4][8];
    // Buffer-resource loads / stores (SGPR descriptor + one 32-bit byte offset
    // per slot, the second half an immediate +256 B): out-of-range lanes and
    // prefetches past the last tile carry an offset beyond num_records, so the
    // hardware returns zeros / drops the store -- no branch around any memory
    // instruction, and the compiler's vmcnt waits stay counted (a skipped load
    // or store on one path forces it to vmcnt(0)).
    constexpr unsigned OOR = 0x80000000u;
    constexpr int CP = 0, SP = 0;   // cache policy of the p / m / v stream (nt / sc1 measured no faster)
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(A.p, (short)0, (int)A.state_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(A.m, (short)0, (int)A.state_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(A.v, (short)0, (int)A.state_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rg =
        __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, SG ? (int)A.state_bytes : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(A.rows, (short)0, A.rows ? (int)A.rows_bytes : 0, 0x00020000);
    unsigned eb[4][2], rb[4][2];   // byte offsets per slot and half (OOR: skip)
    auto load = [&](int slot, int k, int c, bool live) __attribute__((always_inline)) {
        int m0, n0;
        tile_of(k, m0, n0);
        const int m = m0 + u * 32 + c * 4 + rr;
        const int tp = m / p.Cg, cc = m - tp * p.Cg;
        const bool okm = live && m < p.M && cc < p.c_valid;
        const int n = n0 + j * 4;
        const unsigned e = 4u * (unsigned)(tp * (int)p.o_tap + cc * (int)p.o_c + n);
        const unsigned r = 2u * (unsigned)((tp * A.rows_ap + cc) * A.rows_bp + n);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool ok = okm && n + 64 * h < p.n_valid;
            eb[slot][h] = ok ? e + 256 * h : OOR;
            rb[slot][h] = ok ? r + 128 * h : OOR;
            *reinterpret_cast<f32x4*>(pv[slot] + 4 * h) = __builtin_amdgcn_raw_buffer_load_b128(rp, eb[slot][h], 0, CP);
            *reinterpret_cast<f32x4*>(mv[slot] + 4 * h) = __builtin_amdgcn_raw_buffer_load_b128(rm, eb[slot][h], 0, CP);
            *reinterpret_cast<f32x4*>(vv[slot] + 4 * h) = __builtin_amdgcn_raw_buffer_load_b128(rv, eb[slot][h], 0, CP);
        }
    };
    // half h of step c of the staged tile (block tile kprev); after the second
    // half, prefetch step c + 4.  Halves, spread over the stage barriers, keep
    // each interval's Adam VALU within the issue slots the MFMA waves leave.
    auto step = [&](int c, int h, int kprev, bool more) __attribute__((always_inline)) {
        const int slot = c & 3;
        const int row = u * 32 + c * 4 + rr;
        const f32x4 g4 = *reinterpret_cast<const f32x4*>(stg + row * SROW + (h * 64 + j * 4) * 4);
        float np[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = 4 * h + e;
            const float gc = g4[e] * A.gs;
            const float mj = A.b1 * mv[slot][q] + (1.f - A.b1) * gc;
            const float vj = A.b2 * vv[slot][q] + (1.f - A.b2) * gc * gc;
            np[e] = pv[slot][q] - A.lr_t * mj / (sqrtf(vj) + A.eps);
            mv[slot][q] = mj;
            vv[slot][q] = vj;
        }
        const unsigned e0 = eb[slot][h];
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{np[0], np[1], np[2], np[3]}, rp, e0, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const f32x4*>(mv[slot] + 4 * h), rm, e0, 0, SP);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const f32x4*>(vv[slot] + 4 * h), rv, e0, 0, SP);
        if constexpr (SG) __builtin_amdgcn_raw_buffer_store_b128(g4, rg, e0, 0, 0);
        const bf16 b0 = (bf16)np[0], b1 = (bf16)np[1], b2 = (bf16)np[2], b3 = (bf16)np[3];
        const unsigned lo2 = (uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16);
        const unsigned hi2 = (uint32_t)__builtin_bit_cast(uint16_t, b2) | ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16);
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo2, hi2}, rw, rb[slot][h], 0, 0);
        if (h == 1) {
            if (c < 4) load(slot, kprev, c + 4, true);
            else load(slot, more ? kprev + 1 : kprev, c - 4, more);
        }
    };

    // period 0: the MFMA waves compute tile 0; prefetch its first four steps
#pragma unroll
    for (int c = 0; c < 4; ++c)
        if (!(ABL & 1)) load(c, 0, c, true);
    for (int it = 0; it < nk; ++it) wa_bar();
    for (int k = 1; k <= nt; ++k) {
        wa_bar();   // X
        wa_bar();   // stage barrier 0: staging of tile k-1 published
        const bool more = k < nt;
        // nk - 1 further stage barriers (the MFMA waves' tile k, or their idle
        // tail after the last tile); half-step q runs before barrier 1 + q * nk / 16
        int bar = 1;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int iq = 1 + (q * nk) / 16;
            while (bar < iq) {
                wa_bar();
                ++bar;
            }
            if (!(ABL & 1)) step(q >> 1, q & 1, k - 1, more);
        }
        while (bar < nk) {
            wa_bar();
            ++bar;
        }
    }
}

// Applies where igemm_tn3's fused form does (tn3_adam_ok) and the KRSC copy is
// left to the rows -> KRSC transpose.
bool wadam_ok(const TNParams& p, int dtype) {
    if (!g_wadam || dtype != SEG_BF16 || p.adam.tr || p.adam.abl || !tn3_adam_ok(p, dtype)) return false;
    // 32-bit byte offsets of the operands, the state and the HWIO copy
    const long nimg = p.P / ((long)p.Ha * p.Wa);
    if (2 * nimg * p.x_img >= (1L << 31) || 2L * p.P * p.ldb >= (1L << 31)) return false;
    const long taps = (p.M + p.Cg - 1) / p.Cg;
    const long last = (taps - 1) * p.o_tap + (long)(p.Cg - 1) * p.o_c + p.N + 128;
    const long rlast = ((taps - 1) * p.adam.rows_ap + p.Cg) * (long)p.adam.rows_bp + p.N + 128;
    return 4 * last < (1L << 31) && 2 * rlast < (1L << 31);
}

void launch_wadam(TNParams& p, hipStream_t s) {
    const int tm = (p.M + 127) / 128, tn = (p.N + 127) / 128;
    const long T = (long)tm * tn;
    int g = (int)std::min<long>(device_cus(), T);
    g = (g + 7) / 8 * 8;
    const bool sg = p.adam.store_grad != 0;
    const long taps = (p.M + p.Cg - 1) / p.Cg;
    p.adam.state_bytes = (unsigned)(4 * ((taps - 1) * p.o_tap + (long)(p.c_valid - 1) * p.o_c + p.n_valid));
    p.adam.rows_bytes = (unsigned)(2 * (((taps - 1) * p.adam.rows_ap + p.c_valid - 1) * (long)p.adam.rows_bp + p.n_valid));
    // 8 MFMA waves (2 per SIMD), 64-pixel stages in a 3-stage ring: the best of
    // the measured forms (4 waves, 32-pixel stages in a 6-stage ring: slower)
#define WADAM(SG, ABL) \
    hipLaunchKernelGGL((wgrad_adam_ws<3, SG, ABL>), dim3(g), dim3(64 * 12), 0, s, p, tm, tn)
    switch (g_wadam_abl) {
        case 1: WADAM(false, 1); return;
        case 2: WADAM(false, 2); return;
        case 5: WADAM(false, 5); return;
        case 9: WADAM(false, 9); return;
    }
    if (sg) WADAM(true, 0);
    else WADAM(false, 0);
#undef WADAM
}

}  // namespace seg
