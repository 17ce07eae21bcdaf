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
