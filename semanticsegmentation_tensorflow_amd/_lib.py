"""Build and load `libsegkern.so`, the gfx950 HIP library behind the C-ABI in
`include/segkern.h`.

The library is built in-tree (it travels with the repo snapshot to the GPU
box) by `build()`; `lib()` loads it with ctypes and fails loudly when it is
missing -- there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "build")
LIB_PATH = os.path.join(PKG_DIR, "libsegkern.so")
# diagnostic build (-DSEG_DIAG): the kernel-ablation modes of tools/ (no DMA / no
# MFMA / no stores -- garbage results) exist only in this separate library;
# SEG_DIAG_LIB=1 loads it instead of the product library
DIAG_LIB_PATH = os.path.join(PKG_DIR, "build_diag", "libsegkern_diag.so")
SOURCES = ["igemm.hip", "igemm2.hip", "igemm3.hip", "halo.hip", "halo4.hip", "wgrad.hip", "conv.hip", "eltwise.hip", "optim.hip", "smallc.hip", "augment.hip", "dense1x1.hip"]
HOST_SOURCES = ["pngdec.cpp", "crc32c.cpp"]
HIP_HOST_SOURCES = ["timing.cpp"]   # host code against the HIP runtime API (hipcc, no kernels)
HOST_LIBS = ["-lz"]
# per-source extra compiler flags
EXTRA_FLAGS = {}
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall",
          "-Wno-unused-variable", "-Wno-unused-function", "-munsafe-fp-atomics"]


class SegKernelError(RuntimeError):
    pass


def _newer(a, b):
    return os.path.exists(b) and os.path.getmtime(b) >= os.path.getmtime(a)


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    """Compile every HIP source for gfx950 and link libsegkern.so in-tree
    (diag: the -DSEG_DIAG ablation library build_diag/libsegkern_diag.so)."""
    build_dir = os.path.join(PKG_DIR, "build_diag") if diag else BUILD_DIR
    lib_path = DIAG_LIB_PATH if diag else LIB_PATH
    os.makedirs(build_dir, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(REPO_DIR, "include", "segkern.h"))
    newest_header = max(os.path.getmtime(h) for h in headers)

    def compile_one(src):
        s = os.path.join(CSRC, src)
        o = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
        if (not force and _newer(s, o) and os.path.getmtime(o) >= newest_header):
            return o
        if src in HOST_SOURCES:
            cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-c", s, "-o", o]
        else:
            cmd = [HIPCC, *CFLAGS, *EXTRA_FLAGS.get(src, []), *(["-DSEG_DIAG"] if diag else []), "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise SegKernelError(f"{cmd[0]} failed for {src}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES + HIP_HOST_SOURCES + HOST_SOURCES))
    if force or not os.path.exists(lib_path) or any(
            os.path.getmtime(o) > os.path.getmtime(lib_path) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path, *objs, *HOST_LIBS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise SegKernelError(f"link failed:\n{r.stderr}")
    return lib_path


_LIB = None
_LOCK = threading.Lock()


class SegConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "N", "H", "W", "C", "OH", "OW", "K", "R", "S", "stride_h", "stride_w", "dil_h", "dil_w",
        "pad_top", "pad_bottom", "pad_left", "pad_right", "ldx", "ldy", "c_valid", "k_valid", "dtype")]


class SegEpilogue(ctypes.Structure):
    _fields_ = [("bias", ctypes.c_void_p), ("scale", ctypes.c_void_p), ("shift", ctypes.c_void_p),
                ("residual", ctypes.c_void_p), ("ld_residual", ctypes.c_int), ("relu", ctypes.c_int),
                ("keep_prob", ctypes.c_float), ("seed", ctypes.c_uint64), ("relu_mask", ctypes.c_void_p),
                ("ld_relu_mask", ctypes.c_int), ("mask_scale", ctypes.c_float)]


class SegAugView(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("H0", ctypes.c_int), ("W0", ctypes.c_int), ("x0", ctypes.c_int),
                ("y0", ctypes.c_int), ("w", ctypes.c_int), ("h", ctypes.c_int), ("flip", ctypes.c_int),
                ("bc", ctypes.c_int), ("bright", ctypes.c_int), ("contrast", ctypes.c_double)]


class SegPrologue(ctypes.Structure):
    _fields_ = [("gamma", ctypes.c_void_p), ("beta", ctypes.c_void_p), ("eps", ctypes.c_float),
                ("relu", ctypes.c_int)]


class SegBnBwd(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("ldx", ctypes.c_int), ("gamma", ctypes.c_void_p),
                ("beta", ctypes.c_void_p), ("eps", ctypes.c_float), ("relu", ctypes.c_int),
                ("accumulate", ctypes.c_int), ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
                ("keep_prob", ctypes.c_float), ("seed", ctypes.c_uint64)]


class SegBnFinishSegment(ctypes.Structure):
    _fields_ = [("part", ctypes.c_void_p), ("nrows", ctypes.c_int), ("C", ctypes.c_int), ("cv", ctypes.c_int),
                ("inv", ctypes.c_float), ("dgamma", ctypes.c_void_p), ("dbeta", ctypes.c_void_p),
                ("scratch", ctypes.c_void_p), ("a_blk0", ctypes.c_int), ("a_nblk", ctypes.c_int),
                ("b_blk0", ctypes.c_int), ("b_nblk", ctypes.c_int)]


class SegAdamFused(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("rows_dst", ctypes.c_void_p), ("rows_ap", ctypes.c_int), ("rows_bp", ctypes.c_int),
                ("tr_dst", ctypes.c_void_p), ("tr_ap", ctypes.c_int), ("lr", ctypes.c_float),
                ("beta1", ctypes.c_float), ("beta2", ctypes.c_float), ("eps", ctypes.c_float),
                ("t", ctypes.c_int), ("grad_scale", ctypes.c_float)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float
_Z = ctypes.c_size_t
_DP = ctypes.POINTER(SegConvDesc)
_EP = ctypes.POINTER(SegEpilogue)

# symbol -> (restype, argtypes); must match include/segkern.h exactly
SIGNATURES = {
    "seg_conv_desc_init": (_I, [_DP, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "seg_tconv_desc_init": (_I, [_DP, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "seg_conv2d_fwd": (_I, [_DP, _P, _P, _EP, _P, _P, _Z, _P]),
    "seg_conv2d_fwd_hwio_ok": (_I, [_DP]),
    "seg_conv2d_fwd_hwio": (_I, [_DP, _P, _P, _EP, _P, _P, _Z, _P]),
    "seg_conv2d_fwd_pool_ok": (_I, [_DP]),
    "seg_conv2d_fwd_pool": (_I, [_DP, _P, _P, _EP, _P, _I, _P, _I, _P, _Z, _P]),
    "seg_conv2d_bwd_data": (_I, [_DP, _P, _P, _EP, _P, _P, _Z, _P]),
    "seg_conv2d_fwd_relu_bits_ok": (_I, [_DP]),
    "seg_conv2d_fwd_relu_bits": (_I, [_DP, _P, _P, _EP, _P, _P, _I, _P]),
    "seg_conv2d_bwd_data_bits_ok": (_I, [_DP]),
    "seg_conv2d_bwd_data_bits": (_I, [_DP, _P, _P, _EP, _P, _I, _P, _P, _Z, _P]),
    "seg_conv2d_bwd_data_unpool_ok": (_I, [_DP]),
    "seg_conv2d_bwd_data_unpool": (_I, [_DP, _P, _P, _EP, _P, _I, _I, _P, _I, _P, _Z, _P]),
    "seg_conv2d_fwd_pro": (_I, [_DP, _P, ctypes.POINTER(SegPrologue), _P, _EP, _P, _P, _Z, _P]),
    "seg_conv2d_fwd_bn2": (_I, [_DP, _P, ctypes.POINTER(SegPrologue), _P, _EP, _P, _P, _I, _P, _P, _F, _I, _P, _Z,
                                _P]),
    "seg_conv2d_fwd_bn2_ok": (_I, [_DP, _I]),
    "seg_conv_bwd_data_bn_workspace": (_Z, [_DP]),
    "seg_conv2d_bwd_data_bn": (_I, [_DP, _P, _P, ctypes.POINTER(SegBnBwd), _P, _P, _Z, _P]),
    "seg_conv_bwd_data_bn_part_rows": (_L, [_DP]),
    "seg_conv2d_bwd_data_bn_part": (_I, [_DP, _P, _P, ctypes.POINTER(SegBnBwd), _P, _P, _L, _P]),
    "seg_bn_finish_batch_plan": (_Z, [_P, _I, _P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "seg_bn_grad_finish_batch": (_I, [_P, _I, _I, _I, _P]),
    "seg_conv2d_bwd_filter_pro": (_I, [_DP, _P, ctypes.POINTER(SegPrologue), _P, _P, _P, _P, _Z, _P]),
    "seg_conv2d_bwd_filter": (_I, [_DP, _P, _P, _P, _P, _P, _Z, _P]),
    "seg_tconv2d_fwd": (_I, [_DP, _P, _P, _EP, _P, _P, _Z, _P]),
    "seg_tconv2d_bwd_data": (_I, [_DP, _P, _P, _EP, _P, _P, _Z, _P]),
    "seg_tconv2d_bwd_filter": (_I, [_DP, _P, _P, _P, _P, _P, _Z, _P]),
    "seg_conv_workspace": (_Z, [_DP, _I]),
    "seg_tconv_filter_apad": (_I, [_DP]),
    "seg_conv_wgrad_adam_fusable": (_I, [_DP]),
    "seg_conv2d_bwd_filter_begin": (_I, [_DP, _P, _P, _P, _P, _P, _Z, ctypes.POINTER(_I), _P]),
    "seg_conv2d_bwd_filter_end": (_I, [_DP, _P, _P, _P, ctypes.POINTER(_I), _P]),
    "seg_softmax": (_I, [_P, _I, _I, _L, _P, _I, _I, _P]),
    "seg_conv2d_bwd_filter_adam": (_I, [_DP, _P, _P, _P, _P, ctypes.POINTER(SegAdamFused), _P, _Z, _P]),
    "seg_set_option": (_I, [ctypes.c_char_p, _I]),
    "seg_get_option": (_I, [ctypes.c_char_p, ctypes.POINTER(_I)]),
    "seg_timing_event_create": (_I, [ctypes.POINTER(ctypes.c_void_p)]),
    "seg_timing_event_record": (_I, [_P, _P]),
    "seg_timing_event_elapsed_ms": (_I, [ctypes.POINTER(ctypes.c_float), _P, _P]),
    "seg_timing_event_destroy": (_I, [_P]),
    "seg_conv_kernel_info": (_I, [_DP, _I, ctypes.c_char_p, _I, ctypes.POINTER(_I),
                                  ctypes.POINTER(ctypes.c_double)]),
    "seg_pack_filter": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_bias_relu_bwd": (_I, [_P, _I, _P, _I, _P, _I, _P, _L, _I, _I, _I, _F, _I, _P, _Z, _P]),
    "seg_bias_grad_workspace": (_Z, [_L, _I]),
    "seg_maxpool2x2_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_maxpool2x2_bwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_maxpool2x2_fwd_argmax": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_maxpool2x2_bwd_argmax": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_avgpool2x2_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_avgpool2x2_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_add": (_I, [_P, _P, _P, _L, _I, _P]),
    "seg_dropout_fwd": (_I, [_P, _P, _L, _F, ctypes.c_uint64, _I, _P]),
    "seg_dropout_bwd": (_I, [_P, _P, _L, _F, ctypes.c_uint64, _I, _P]),
    "seg_dropout_bwd_ch": (_I, [_P, _I, _P, _I, _L, _I, _I, _F, ctypes.c_uint64, _I, _P]),
    "seg_bn_relu_fwd": (_I, [_P, _I, _P, _I, _P, _P, _F, _L, _I, _I, _I, _I, _P]),
    "seg_bn_relu_bwd": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _F, _P, _P, _L, _I, _I, _I, _I,
                             _P, _Z, _P]),
    "seg_bn_relu_dropout_bwd": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _P, _P, _F, _P, _P, _L, _I, _I, _I,
                                     _F, ctypes.c_uint64, _I, _I, _P, _Z, _P]),
    "seg_resize_bilinear_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_resize_bilinear_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_copy_channels": (_I, [_P, _I, _P, _I, _L, _I, _I, _P]),
    "seg_spatial_reduce": (_I, [_P, _I, _P, _I, _I, _I, _I, _F, _P, _I, _P]),
    "seg_spatial_broadcast": (_I, [_P, _P, _I, _I, _I, _I, _I, _F, _I, _P]),
    "seg_prepare_input": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_prepare_input_u8": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "seg_png_info": (_I, [_P, _Z, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "seg_png_decode": (_I, [_P, _Z, _P, _Z]),
    "seg_augment": (_I, [ctypes.POINTER(SegAugView), _I, _I, _I, _I, _I, _P, _P]),
    "seg_softmax_xent_fwd_bwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _I, _I, _P,
                                      _Z, _P]),
    "seg_xent_workspace": (_Z, [_I, _I, _I]),
    "seg_softmax_xent_soft_fwd_bwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _I, _I,
                                           _P, _Z, _P]),
    "seg_argmax": (_I, [_P, _I, _I, _L, _P, _I, _P]),
    "seg_confusion": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "seg_adam_tf1_step": (_I, [_P, _P, _P, _P, _L, _F, _F, _F, _F, _I, _F, _P]),
    "seg_adam_segments_plan": (_I, [_P, _I]),
    "seg_concat_fwd": (_I, [_P, _I, _P, _I, _I, _L, _I, _P]),
    "seg_concat_bwd": (_I, [_P, _I, _P, _I, _L, _I, _P]),
    "seg_adam_tf1_pack": (_I, [_P, _P, _P, _P, _P, _I, _I, _F, _F, _F, _F, _I, _F, _I, _P]),
    "seg_pack_segments": (_I, [_P, _P, _I, _I, _I, _P]),
    "seg_fill": (_I, [_P, _L, _F, _I, _P]),
    "seg_cast": (_I, [_P, _I, _P, _I, _L, _P]),
    "seg_axpy": (_I, [_P, _P, _F, _L, _P]),
    "seg_check_finite": (_I, [_P, _L, _P, _P]),
    "seg_crc32c": (ctypes.c_uint32, [_P, _Z, ctypes.c_uint32]),
    "seg_status_string": (ctypes.c_char_p, [_I]),
    "seg_version": (_I, []),
}


def load(path: str = LIB_PATH):
    """Load the library and bind every C-ABI symbol (no GPU work)."""
    if not os.path.exists(path):
        raise SegKernelError(
            f"{path} not found: the HIP kernel library is required (no CPU fallback). "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` first.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                _LIB = load(DIAG_LIB_PATH if os.environ.get("SEG_DIAG_LIB") == "1" else LIB_PATH)
                # kernel-selection overrides for experiments: SEG_OPTIONS="nt3=0,tn3_mfast=1"
                for kv in filter(None, os.environ.get("SEG_OPTIONS", "").split(",")):
                    k, v = kv.split("=")
                    if _LIB.seg_set_option(k.strip().encode(), int(v)) != 0:
                        raise SegKernelError(f"SEG_OPTIONS: bad option {kv!r}")
    return _LIB


def check(status: int, what: str = ""):
    if status != 0:
        msg = lib().seg_status_string(status).decode()
        if status == 2:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: {msg} (status {status})")
