"""The C-ABI library loads and exports every symbol include/segkern.h declares
(no compute calls -- runs without a GPU)."""
import os
import re

from semanticsegmentation_tensorflow_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "segkern.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(seg_[a-z0-9_]+)\s*\(", text))


def test_library_exports_every_declared_symbol():
    _lib.build()
    lib = _lib.load()
    declared = _header_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # and the ctypes binding table covers the header exactly
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_status_strings_and_descriptor_rules():
    import ctypes
    lib = _lib.load()
    assert lib.seg_status_string(0) == b"ok"
    assert b"shape" in lib.seg_status_string(2)
    d = _lib.SegConvDesc()
    # TF SAME, even kernel: pad_total=3 at stride 1 -> top 1, bottom 2
    assert lib.seg_conv_desc_init(ctypes.byref(d), 1, 8, 8, 3, 16, 4, 4, 1, 1, 0, 1) == 0
    assert (d.OH, d.pad_top, d.pad_bottom, d.C, d.c_valid) == (8, 1, 2, 8, 3)
    # conv2d_transpose shape rule: FCN conv_t1 at 375x1242 -> pool5 11x38, pool4 23x77
    assert lib.seg_tconv_desc_init(ctypes.byref(d), 1, 11, 38, 2, 23, 77, 512, 4, 4, 2, 0, 1) == 2
    assert lib.seg_tconv_desc_init(ctypes.byref(d), 1, 12, 39, 2, 24, 78, 512, 4, 4, 2, 0, 1) == 0
    assert (d.pad_top, d.pad_bottom) == (1, 1)
    # k16 s8 conv_t3 at 384 -> pad 4/4
    assert lib.seg_tconv_desc_init(ctypes.byref(d), 1, 48, 156, 256, 384, 1248, 2, 16, 16, 8, 0, 1) == 0
    assert (d.pad_top, d.pad_bottom, d.pad_left, d.pad_right) == (4, 4, 4, 4)


def test_pooled_conv_refuses_a_split_k_plan():
    """a MaxPool-fused conv (p.y null, the pooled map only) must
    never run on split-K slabs or a kernel without the pooled epilogue.  The
    pooled-plan check (seg_conv2d_fwd_pool_ok) and the launch read the same plan
    function, and the launch itself refuses a pooled launch on such a plan
    with SEG_EINVAL -- host-side, before anything reaches the GPU (here: no GPU,
    so the fake pointers are never touched).  Network/model/FCN.py:54-75."""
    import ctypes
    lib = _lib.load()
    d = _lib.SegConvDesc()
    # conv3_3 + pool3 of C2 (conv_halo2, 256-wide tiles) and conv2_2 + pool2
    # (conv_halo_duo): both pooled by default
    for args in ((4, 96, 312, 256, 256), (4, 192, 624, 128, 128)):
        assert lib.seg_conv_desc_init(ctypes.byref(d), *args, 3, 3, 1, 1, 0, 1) == 0
        assert lib.seg_conv2d_fwd_pool_ok(ctypes.byref(d)) == 1
        assert lib.seg_set_option(b"halo_min_splits", 2) == 0
        try:
            name = ctypes.create_string_buffer(64)
            sp = ctypes.c_int(0)
            fl = ctypes.c_double(0)
            assert lib.seg_conv_kernel_info(ctypes.byref(d), 0, name, 64, ctypes.byref(sp), ctypes.byref(fl)) == 0
            assert name.value.startswith(b"conv_halo") and sp.value >= 2, (name.value, sp.value)
            assert lib.seg_conv2d_fwd_pool_ok(ctypes.byref(d)) == 0
            fake = ctypes.c_void_p(1 << 20)
            st = lib.seg_conv2d_fwd_pool(ctypes.byref(d), fake, fake, None, fake, args[4], None, 0, fake,
                                         ctypes.c_size_t(1 << 40), None)
            assert st == 1, st          # SEG_EINVAL, nothing launched
        finally:
            assert lib.seg_set_option(b"halo_min_splits", 1) == 0
        assert lib.seg_conv2d_fwd_pool_ok(ctypes.byref(d)) == 1


def test_product_library_has_no_ablation_knobs():
    """the kernel-ablation modes (garbage results) are not
    reachable through seg_set_option / SEG_OPTIONS in libsegkern.so."""
    lib = _lib.load()
    EINVAL = 1
    for knob in (b"nt2_ablate", b"tn3_abl", b"tn3_adam_abl", b"wgrad_abl", b"wadam_abl", b"wadam"):
        assert lib.seg_set_option(knob, 1) == EINVAL, knob
    assert lib.seg_set_option(b"tn_reduce_sl", 3) == EINVAL
    assert lib.seg_set_option(b"tn_reduce_sl", 16) == 0
    assert lib.seg_set_option(b"wpad", 12) == EINVAL
    # variants measured slower and deleted: no knob selects them
    for knob in (b"bn1x1s_st", b"nt2bn_bm"):
        assert lib.seg_set_option(knob, 1) == EINVAL, knob
    assert lib.seg_set_option(b"nt2bn_bm", 128) == EINVAL
    assert lib.seg_set_option(b"res16c_bh", 2) == EINVAL
    assert lib.seg_set_option(b"res16c_bh", 4) == 0


def test_knobs_are_a_guarded_per_device_set():
    """VERDICT r05 item 7 / SURVEY.md 8b: the kernel-selection knobs are the
    library's only mutable state, one mutex-guarded set per HIP device
    (csrc/knobs.h).  seg_get_option reads back the tuned defaults; a change
    applies to the very next call's plan (seg_conv_kernel_info re-plans from
    the descriptor and the knobs on every call -- nothing else is cached);
    invalid values leave the set untouched; concurrent writers and readers
    from several host threads see only values some writer stored."""
    import ctypes
    import threading
    lib = _lib.load()
    v = ctypes.c_int(-1)
    defaults = {b"halo4": 2, b"nt3": 1, b"tn_reduce_sl": 16, b"wgrad_nt": 128, b"wpad": 0}
    for k, want in defaults.items():
        assert lib.seg_get_option(k, ctypes.byref(v)) == 0 and v.value == want, (k, v.value)
    assert lib.seg_get_option(b"no_such_knob", ctypes.byref(v)) == 1
    d = _lib.SegConvDesc()
    assert lib.seg_conv_desc_init(ctypes.byref(d), 4, 96, 312, 256, 256, 3, 3, 1, 1, 0, 1) == 0
    name = ctypes.create_string_buffer(64)
    sp, fl = ctypes.c_int(0), ctypes.c_double(0)

    def kernel():
        assert lib.seg_conv_kernel_info(ctypes.byref(d), 0, name, 64, ctypes.byref(sp), ctypes.byref(fl)) == 0
        return name.value
    assert kernel().startswith(b"conv_halo4<")
    try:
        assert lib.seg_set_option(b"halo4", 0) == 0
        assert kernel().startswith(b"conv_halo<")        # conv_halo2 (reported under the family name)
        assert lib.seg_set_option(b"halo4", 99) == 1       # rejected: the set keeps 0
        assert lib.seg_get_option(b"halo4", ctypes.byref(v)) == 0 and v.value == 0
    finally:
        assert lib.seg_set_option(b"halo4", 2) == 0
    assert kernel().startswith(b"conv_halo4<")
    seen, errs = set(), []

    def writer(val):
        for _ in range(2000):
            if lib.seg_set_option(b"tn_split_cap", val) != 0:
                errs.append(val)

    def reader():
        r = ctypes.c_int(0)
        for _ in range(2000):
            lib.seg_get_option(b"tn_split_cap", ctypes.byref(r))
            seen.add(r.value)
    ts = [threading.Thread(target=writer, args=(a,)) for a in (64, 128)] + [threading.Thread(target=reader)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and seen <= {64, 128, 256}, (errs, seen)
    assert lib.seg_set_option(b"tn_split_cap", 256) == 0


def test_bn_part_launch_refuses_a_foreign_row_count():
    """seg_conv2d_bwd_data_bn_part writes exactly seg_conv_bwd_data_bn_part_rows
    partial rows -- the count a batched finish plan was made for; any other
    part_rows (a buffer sized under another kernel option) is refused with
    SEG_EWORKSPACE on the host (fake pointers, never touched).  The row count
    follows the launch geometry: bn1x1_stream blocks per 64-channel chunk, or
    igemm_nt2_bn M tiles."""
    import ctypes
    lib = _lib.load()
    d = _lib.SegConvDesc()
    assert lib.seg_conv_desc_init(ctypes.byref(d), 8, 384, 1248, 128, 64, 1, 1, 1, 1, 0, 1) == 0
    rows = lib.seg_conv_bwd_data_bn_part_rows(ctypes.byref(d))
    assert rows > 0
    assert lib.seg_set_option(b"bn1x1s", 0) == 0
    try:
        rows_nt2 = lib.seg_conv_bwd_data_bn_part_rows(ctypes.byref(d))
    finally:
        assert lib.seg_set_option(b"bn1x1s", 1) == 0
    assert rows_nt2 == (8 * 384 * 1248 + 255) // 256 and rows_nt2 != rows
    fake = ctypes.c_void_p(1 << 20)
    bn = _lib.SegBnBwd(1 << 20, 128, 1 << 20, 1 << 20, 1e-3, 1, 1, None, None, 1.0, 0)
    st = lib.seg_conv2d_bwd_data_bn_part(ctypes.byref(d), fake, fake, ctypes.byref(bn), fake, fake, rows_nt2, None)
    assert st == 4, st                  # SEG_EWORKSPACE
