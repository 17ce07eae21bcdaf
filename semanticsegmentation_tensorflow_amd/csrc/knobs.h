// The library's kernel-selection knobs: its only mutable state.
//
// the library is stateless apart from a mutex-guarded,
// per-device tuned-config cache.  Each HIP device has one KnobSet (the tuned
// defaults below until seg_set_option changes them); seg_set_option writes the
// calling thread's current device's set under a mutex, and a launch reads the
// set of the device it runs on (relaxed atomic loads: a write never tears a
// read, and a change applies to launches issued after it).  No plan or kernel
// choice is cached anywhere else: every entry point re-plans from its
// descriptor and these values.  seg_get_option reads one back.
#pragma once
#include <atomic>

namespace seg {

// X(name, default): g_<name> reads it for the current device
#define SEG_KNOBS(X) \
    X(wpad, 0) \
    X(adam_tr_fused, 0) \
    X(s1x1, 1) \
    X(bn1x1s, 1) \
    X(s1x1_st, 1) \
    X(dropout_flat, 1) \
    X(nt_halo, 1) \
    X(halo_wide, 1) \
    X(res64, 1) \
    X(res16, 1) \
    X(res64_pp, 1) \
    X(wgrad_pxs, 1) \
    X(smallc_tr, 1) \
    X(res16_dma, 1) \
    X(res16c_bh, 4) \
    X(res16c, 1) \
    X(halo_duo, 1) \
    X(halo_min_splits, 1) \
    X(res16c_st, 1) \
    X(halo4, 2) \
    X(nt_nsplit, 1) \
    X(tn_nsplit, 1) \
    X(nt_variant, 2) \
    X(nt3_fill, 1) \
    X(tn_variant, 2) \
    X(tn_fill, 2) \
    X(tn_split_cap, 256) \
    X(tn2_smallm, 0) \
    X(tn_reduce_sl, 16) \
    X(nt2_ablate, 0) \
    X(nt2_short, 8) \
    X(nt3, 1) \
    X(tn3, 1) \
    X(tn3_abl, 0) \
    X(tn3_mfast, 0) \
    X(tn3_half, 0) \
    X(tn3_stagger_us, 40) \
    X(tn3_adam_abl, 0) \
    X(adam_blocks, 0) \
    X(smallc, 1) \
    X(smallk, 1) \
    X(smallk_abl, 0) \
    X(wgrad_halo, 1) \
    X(wgrad_nt, 128) \
    X(wgrad_abl, 0) \
    X(wgrad_nt32, 1) \
    X(wgrad_fill, 88) \
    X(wgrad_nbias, 1)

struct KnobSet {
#define SEG_KNOB_MEMBER(n, d) std::atomic<int> n{d};
    SEG_KNOBS(SEG_KNOB_MEMBER)
#undef SEG_KNOB_MEMBER
};

// the KnobSet of the calling thread's current HIP device
KnobSet& knobs();

}  // namespace seg

#define g_wpad (::seg::knobs().wpad.load(std::memory_order_relaxed))
#define g_adam_tr_fused (::seg::knobs().adam_tr_fused.load(std::memory_order_relaxed))   // 1: the fused epilogue also writes the KRSC copy (transposed 16-byte stores)
#define g_s1x1 (::seg::knobs().s1x1.load(std::memory_order_relaxed))
#define g_bn1x1s (::seg::knobs().bn1x1s.load(std::memory_order_relaxed))
#define g_s1x1_st (::seg::knobs().s1x1_st.load(std::memory_order_relaxed))
#define g_dropout_flat (::seg::knobs().dropout_flat.load(std::memory_order_relaxed))   // dropout re-draw: one chunk per thread (0: the grid-stride loop)
#define g_nt_halo (::seg::knobs().nt_halo.load(std::memory_order_relaxed))
#define g_halo_wide (::seg::knobs().halo_wide.load(std::memory_order_relaxed))
#define g_res64 (::seg::knobs().res64.load(std::memory_order_relaxed))
#define g_res16 (::seg::knobs().res16.load(std::memory_order_relaxed))   // conv_res64 with 16-wide output blocks for N <= 16
#define g_res64_pp (::seg::knobs().res64_pp.load(std::memory_order_relaxed))
#define g_wgrad_pxs (::seg::knobs().wgrad_pxs.load(std::memory_order_relaxed))
#define g_smallc_tr (::seg::knobs().smallc_tr.load(std::memory_order_relaxed))
#define g_res16_dma (::seg::knobs().res16_dma.load(std::memory_order_relaxed))
#define g_res16c_bh (::seg::knobs().res16c_bh.load(std::memory_order_relaxed))   // tile rows of the BN-backward conv_res16c (8 or 4)
#define g_res16c (::seg::knobs().res16c.load(std::memory_order_relaxed))   // conv_res16c: 16 input channels (growth-conv input gradients)
#define g_halo_duo (::seg::knobs().halo_duo.load(std::memory_order_relaxed))   // N <= 128 without split-K: conv_halo_duo (two blocks per CU)
#define g_halo_min_splits (::seg::knobs().halo_min_splits.load(std::memory_order_relaxed))   // at least this many split-K slabs (tests: a split plan on any shape)
#define g_res16c_st (::seg::knobs().res16c_st.load(std::memory_order_relaxed))
#define g_halo4 (::seg::knobs().halo4.load(std::memory_order_relaxed))   // 256 x 256 halo plans on conv_halo4: 2 = 8 waves (default), 1 = 4 waves, 0 = conv_halo2
#define g_nt_nsplit (::seg::knobs().nt_nsplit.load(std::memory_order_relaxed))   // N = 256 k + tail <= 128: igemm_nt3 head + igemm_nt2 tail
#define g_tn_nsplit (::seg::knobs().tn_nsplit.load(std::memory_order_relaxed))   // TN: igemm_tn3 head + igemm_tn2 tail for N = 256 k + <= 128
#define g_nt_variant (::seg::knobs().nt_variant.load(std::memory_order_relaxed))
#define g_nt3_fill (::seg::knobs().nt3_fill.load(std::memory_order_relaxed))
#define g_tn_variant (::seg::knobs().tn_variant.load(std::memory_order_relaxed))
#define g_tn_fill (::seg::knobs().tn_fill.load(std::memory_order_relaxed))   // split-K target: g_tn_fill blocks per CU
#define g_tn_split_cap (::seg::knobs().tn_split_cap.load(std::memory_order_relaxed))   // max split-K slabs
#define g_tn2_smallm (::seg::knobs().tn2_smallm.load(std::memory_order_relaxed))   // 16-bit M < 128: igemm_tn2 (padded 128-row tiles) instead of igemm_tn
#define g_tn_reduce_sl (::seg::knobs().tn_reduce_sl.load(std::memory_order_relaxed))   // max split-lanes of splitk_reduce_tn (1 = one thread per output float4)
#define g_nt2_ablate (::seg::knobs().nt2_ablate.load(std::memory_order_relaxed))
#define g_nt2_short (::seg::knobs().nt2_short.load(std::memory_order_relaxed))
#define g_nt3 (::seg::knobs().nt3.load(std::memory_order_relaxed))
#define g_tn3 (::seg::knobs().tn3.load(std::memory_order_relaxed))
#define g_tn3_abl (::seg::knobs().tn3_abl.load(std::memory_order_relaxed))   // diagnostics (garbage results): 1 no DMA in the loop, 2 no MFMA, 3 no epilogue stores
#define g_tn3_mfast (::seg::knobs().tn3_mfast.load(std::memory_order_relaxed))   // tile order: M fastest when the B (dy) panel is the larger operand
#define g_tn3_half (::seg::knobs().tn3_half.load(std::memory_order_relaxed))   // 256 x 128 two-blocks-per-CU tiles: 1 for the fused Adam (multi-round grids; +4: any grid), 2 for plain single-split; 0 (default since round 6): 256 x 256 everywhere
#define g_tn3_stagger_us (::seg::knobs().tn3_stagger_us.load(std::memory_order_relaxed))   // half-tile fused Adam: start offset of the second block on each CU (multi-round grids)
#define g_tn3_adam_abl (::seg::knobs().tn3_adam_abl.load(std::memory_order_relaxed))   // diagnostics: 1 no p/m/v loads, 2 no p/m/v stores, 4 no HWIO copy, 8 no KRSC copy, 16 no epilogue
#define g_adam_blocks (::seg::knobs().adam_blocks.load(std::memory_order_relaxed))   // seg_set_option("adam_blocks"): grid cap of seg_adam_tf1_pack (0 = one block per tile)
#define g_smallc (::seg::knobs().smallc.load(std::memory_order_relaxed))
#define g_smallk (::seg::knobs().smallk.load(std::memory_order_relaxed))
#define g_smallk_abl (::seg::knobs().smallk_abl.load(std::memory_order_relaxed))   // diagnostics only (see smallk_nt_k)
#define g_wgrad_halo (::seg::knobs().wgrad_halo.load(std::memory_order_relaxed))
#define g_wgrad_nt (::seg::knobs().wgrad_nt.load(std::memory_order_relaxed))
#define g_wgrad_abl (::seg::knobs().wgrad_abl.load(std::memory_order_relaxed))
#define g_wgrad_nt32 (::seg::knobs().wgrad_nt32.load(std::memory_order_relaxed))   // 32-wide dy tiles for N <= 32
#define g_wgrad_fill (::seg::knobs().wgrad_fill.load(std::memory_order_relaxed))   // split-K target: blocks = this percentage of the CUs (round 6: 88 -- in the overlapped step the side-stream filter gradients share the CUs with the input-gradient chain; 596.5 / 596.8 vs 591.5 / 591.9 img/s at 100 on one box)
#define g_wgrad_nbias (::seg::knobs().wgrad_nbias.load(std::memory_order_relaxed))   // max channel blocks sharing the fused BiasAddGrad (1 measured best: the per-wave spread suffices)
