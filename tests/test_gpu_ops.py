"""Op-level parity: every HIP kernel vs the CPU oracle (oracle/tf1_ops.py).

fp32 path: exact-f32 MFMA, compared at ~1e-5 relative (of max |ref|).
bf16 / fp16 paths: the oracle sees the same rounded inputs; tolerance covers
fp32-accumulation order + one output rounding (~2^-8 bf16, ~2^-11 fp16).
"""
import math

import numpy as np
import pytest
import torch

from oracle import tf1_ops as tf
from semanticsegmentation_tensorflow_amd import ops
from tests.gpu_utils import assert_close, from_dev, rnd, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1, 2, 3, 4, 8], ids=["nt1", "nt2", "halo", "halo128", "nt3"])
def ntv(request, dev):
    """Run NT tests on every kernel generation: 1 = register-staged GEMM,
    2 = LDS-DMA GEMM, 3 = 2 + the halo-tiled direct conv where it applies
    (16-bit, stride 1, C % 64 == 0; 256x256 deep-ring tiles for N > 128),
    4 = 3 restricted to the 256x128 halo tiles, 8 = 2 with the 256x256-tile
    GEMM (igemm_nt3) for every N > 128 problem (by default only where its grid
    fills half the CUs; variant 2 keeps it off so igemm_nt2 stays covered for
    wide N).  Variant 8 also turns off the 2-stage short-K igemm_nt2 (K <= 128),
    so the 3-stage ring stays covered for those problems.  N <= 128 halo
    problems without split-K run the two-blocks-per-CU conv_halo_duo except in
    variant 4 (the one-block conv_halo stays covered)."""
    v = request.param
    ops.set_option("igemm_nt_variant", 1 if v == 1 else 2)
    ops.set_option("nt_halo", 1 if v in (3, 4) else 0)
    ops.set_option("nt3", 0 if v == 2 else 1)
    ops.set_option("halo_wide", 0 if v == 4 else 1)
    ops.set_option("halo_duo", 0 if v == 4 else 1)
    ops.set_option("nt3_fill", 0 if v == 8 else 1)   # small test problems: force the 256x256 tiles
    ops.set_option("nt2_short", 0 if v == 8 else 8)
    yield v
    ops.set_option("nt2_short", 8)
    ops.set_option("nt3_fill", 1)
    ops.set_option("igemm_nt_variant", 2)
    ops.set_option("nt_halo", 1)
    ops.set_option("nt3", 1)
    ops.set_option("halo_wide", 1)
    ops.set_option("halo_duo", 1)


DTYPES = [torch.float32, torch.bfloat16, torch.float16]
DT = {torch.float32: ops.F32, torch.bfloat16: ops.BF16, torch.float16: ops.F16}

# (N, H, W, C, K, R, S(=R), stride, dilation, padding)
CONV_CASES = [
    (2, 9, 11, 8, 16, 3, 3, 1, 1, "SAME"),
    (1, 12, 10, 3, 64, 3, 3, 1, 1, "SAME"),     # conv1_1-like: C=3 padded to 8
    (2, 7, 9, 64, 136, 3, 3, 1, 1, "SAME"),     # N tail (136 = 128 + 8)
    (1, 6, 5, 24, 40, 1, 1, 1, 1, "SAME"),      # 1x1
    (1, 5, 7, 16, 32, 7, 7, 1, 1, "SAME"),      # conv6-like 7x7 SAME on tiny map
    (2, 8, 8, 16, 24, 4, 4, 1, 1, "SAME"),      # even kernel: asymmetric SAME pad
    (1, 11, 13, 16, 16, 3, 3, 2, 1, "SAME"),    # strided
    (1, 12, 12, 8, 16, 3, 3, 1, 2, "SAME"),     # atrous (dilation 2)
    (1, 10, 10, 16, 8, 3, 3, 1, 1, "VALID"),
    (3, 20, 20, 128, 256, 3, 3, 1, 1, "SAME"),  # multi-tile M and N, uniform-tap path
    # halo-tiled direct conv: ragged tiles in x and y, BN=64, dilation, split-K
    (2, 37, 70, 64, 64, 3, 3, 1, 1, "SAME"),
    (1, 30, 41, 64, 128, 3, 3, 1, 2, "SAME"),   # atrous halo (hi = 7)
    (1, 9, 21, 512, 128, 3, 3, 1, 1, "SAME"),   # few tiles -> channel-chunk split-K
    (1, 18, 19, 128, 72, 3, 3, 1, 1, "VALID"),
    (2, 33, 45, 64, 328, 3, 3, 1, 1, "SAME"),   # 256-wide halo tiles: 2 N tiles + tail
    (2, 19, 131, 3, 48, 3, 3, 1, 1, "SAME"),    # first-layer kernel (C=3->8): ragged 8x64 tiles, K=48
    (1, 17, 70, 64, 48, 3, 3, 1, 1, "VALID"),   # resident-filter kernel: VALID, N=48 < 64
    (2, 21, 67, 64, 16, 3, 3, 1, 1, "SAME"),    # resident-filter kernel, FC-DenseNet growth conv (K=16)
    (2, 19, 37, 16, 64, 3, 3, 1, 1, "SAME"),    # 16 input channels (conv_res16c; = the growth conv's dgrad)
    (1, 11, 70, 16, 40, 3, 3, 1, 1, "VALID"),   # conv_res16c: VALID, N = 40 < 64
    # 256x256-tile GEMM (N > 128): K tiles straddling taps, N tail, split-K
    (1, 5, 7, 40, 264, 7, 7, 1, 1, "SAME"),     # conv6-like, C=40: a 64-deep K tile spans taps
    (2, 6, 9, 512, 512, 1, 1, 1, 1, "SAME"),    # conv7-like 1x1
    (1, 4, 6, 64, 384, 7, 7, 1, 1, "SAME"),     # M = 24, K = 3136: split-K slabs
]


def _conv_case(case, seed):
    N, H, W, C, K, R, S, st, dil, pad = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    w = torch.randn(R, S, C, K, generator=g, dtype=torch.float64) / math.sqrt(R * S * C)
    b = torch.randn(K, generator=g, dtype=torch.float64) * 0.1
    return x, w, b


def _pack(w64, mode, dtype, dev, a_pad=None):
    R, S, A, B = w64.shape
    src = w64.float().to(dev).contiguous()
    ap = a_pad if a_pad is not None else ops.round8(A)
    dst = torch.empty(ops.packed_shape(R, S, A, B, mode, ap), dtype=dtype, device=dev)
    return ops.pack_filter(src, dst, ap, ops.round8(B), mode)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_fwd_bias_relu(dev, ntv, case, dtype):
    N, H, W, C, K, R, S, st, dil, pad = case
    x, w, b = _conv_case(case, 1)
    xr, wr = rnd(x, dtype), rnd(w, dtype)
    ref = tf.relu(tf.bias_add(tf.conv2d(xr, wr, st, pad, dil), rnd(b.float().double(), torch.float32)))
    d = ops.conv_desc(N, H, W, C, K, R, S, st, dil, pad, DT[dtype])
    xd = to_dev(x, dtype, dev)
    wk = _pack(w, ops.PACK_KRSC, dtype, dev)
    bd = b.float().to(dev)
    y = torch.empty(N, d.OH, d.OW, d.K, dtype=dtype, device=dev)
    ops.conv2d_fwd(d, xd, wk, y, ops.epilogue(bias=bd, relu=True))
    torch.cuda.synchronize()
    assert_close(from_dev(y, K), ref, dtype, f"conv fwd {case}")
    if d.K > K:   # padding channels stay exactly zero
        assert y[..., K:].abs().max().item() == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [(4, 12, 39, 512, 4096, 7, 0.8), (4, 12, 39, 4096, 4096, 1, 0.8),
                                  (2, 6, 10, 512, 520, 7, 1.0), (4, 2, 3, 4096, 4096, 1, 0.5)],
                         ids=["conv6", "conv7", "conv6-ntail-split64", "conv7-small-split10"])
def test_conv2d_fwd_hwio_equals_krsc(dev, case, dtype):
    """igemm_nt3's B-transposed form (ops.conv2d_fwd_hwio: the forward from the
    HWIO copy the input gradient reads, FCN conv6 / conv7 with their bias +
    ReLU + dropout epilogue) equals the KRSC forward bit for bit: the same
    k order into the same MFMAs (full-size conv6 / conv7 of C2, split-K
    plans, an N tail of 8)."""
    N, H, W, C, K, R, kp = case
    cs = (N, H, W, C, K, R, R, 1, 1, "SAME")
    x, w, b = _conv_case(cs, 3)
    d = ops.conv_desc(N, H, W, C, K, R, R, 1, 1, "SAME", DT[dtype])
    assert ops.conv2d_fwd_hwio_ok(d), case
    assert ops.conv_kernel_info(d, ops.OP_FWD)[0].startswith("igemm_nt3")
    xd = to_dev(x, dtype, dev)
    wk = _pack(w, ops.PACK_KRSC, dtype, dev)
    wh = _pack(w, ops.PACK_HWIO, dtype, dev)
    bd = b.float().to(dev)
    epi = ops.epilogue(bias=bd, relu=True, keep_prob=kp, seed=77)
    ref = torch.full((N, H, W, d.K), float("nan"), dtype=dtype, device=dev)
    got = torch.full_like(ref, float("nan"))
    ops.conv2d_fwd(d, xd, wk, ref, epi)
    ops.conv2d_fwd_hwio(d, xd, wh, got, epi)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    assert ref[..., :K].float().abs().max().item() > 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_first_layer_kernels_cover_16bit(dev, dtype):
    """conv1_1 (C = 3 -> 8, 3x3) runs the small-channel kernels in both 16-bit
    storage types (the parity of both is in the CONV_CASES / SPLIT_WGRAD_CASES
    first-layer rows above and below)."""
    d = ops.conv_desc(2, 19, 131, 3, 64, 3, 3, dtype=DT[dtype])
    assert ops.conv_kernel_info(d, ops.OP_FWD)[0].startswith("conv_c8")
    assert ops.conv_kernel_info(d, ops.OP_BWD_FILTER)[0].startswith("wgrad_c8")


@pytest.mark.parametrize("masked", [False, True], ids=["plain", "relu_mask"])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[7] == 1])
def test_conv2d_bwd_data(dev, ntv, case, dtype, masked):
    """Conv2DBackpropInput; relu_mask: the fused ReluGrad x 1/keep_prob of the
    layer that produced x (epilogue mask = that layer's post-ReLU output)."""
    N, H, W, C, K, R, S, st, dil, pad = case
    x, w, _ = _conv_case(case, 2)
    wr = rnd(w, dtype)
    xr = x.clone().requires_grad_(True)
    y = tf.conv2d(xr, wr, st, pad, dil)
    g = torch.Generator().manual_seed(7)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    d = ops.conv_desc(N, H, W, C, K, R, S, st, dil, pad, DT[dtype])
    dyd = to_dev(dy, dtype, dev)
    wh = _pack(w, ops.PACK_HWIO, dtype, dev)
    dx = torch.full((N, H, W, d.C), float("nan"), dtype=dtype, device=dev)
    want = xr.grad
    epi = None
    if masked:
        prev = torch.relu(torch.randn(N, H, W, C, generator=g, dtype=torch.float64))   # ~half zeros
        prev_d = to_dev(prev, dtype, dev)     # epilogue keeps only the pointer: hold the tensor
        epi = ops.epilogue(relu_mask=prev_d, mask_scale=1.25)
        want = torch.where(prev > 0, want * 1.25, torch.zeros_like(want))
    ops.conv2d_bwd_data(d, dyd, wh, dx, epi=epi)
    torch.cuda.synchronize()
    assert_close(from_dev(dx, C), want, dtype, f"conv bwd_data {case}")


@pytest.fixture(params=[1, 2, 3, 4, 5, 6, 7, 8], ids=["tn1", "tn2", "wgrad-halo", "wgrad-halo128", "tn3",
                                                      "wgrad-nbias4", "tn3-half", "wgrad-halo-colsplit"])
def tnv(request, dev):
    """Run filter-gradient tests on every kernel generation: 1 = register-staged
    TN GEMM, 2 = LDS-DMA TN GEMM, 3 = 2 + the halo-tiled 3x3 filter gradient
    where it applies (16-bit, stride 1, C % 64 == 0), 4 = 3 with 128-wide dy
    tiles, 5 = 2 with the 256x256-tile TN GEMM (igemm_tn3; on by default, off
    in 2 so igemm_tn2 stays covered for wide problems), 6 = 4 with the fused
    BiasAddGrad spread over up to 4 channel blocks (extra slab rows), 7 = 5
    with the 256x128 two-blocks-per-CU tiles also for plain single-split
    launches; 3 runs the 64-wide tiles on pixel-split waves (two slabs per
    split, round 6), 8 the same tiles on column-split waves."""
    v = request.param
    ops.set_option("igemm_tn_variant", 1 if v == 1 else 2)
    ops.set_option("wgrad_halo", 1 if v in (3, 4, 6, 8) else 0)
    ops.set_option("wgrad_nt", 128 if v in (4, 6) else 64)
    ops.set_option("wgrad_pxs", 0 if v == 8 else 1)
    ops.set_option("wgrad_nbias", 4 if v == 6 else 1)
    ops.set_option("tn3", 0 if v == 2 else 1)
    ops.set_option("tn3_half", 7 if v == 7 else 0)
    yield v
    ops.set_option("wgrad_pxs", 1)
    ops.set_option("tn3_half", 0)
    ops.set_option("tn3", 1)
    ops.set_option("wgrad_nbias", 1)
    ops.set_option("igemm_tn_variant", 2)
    ops.set_option("wgrad_halo", 1)
    ops.set_option("wgrad_nt", 128)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", CONV_CASES + [(2, 24, 20, 64, 64, 3, 3, 1, 1, "SAME"),
                                               (1, 16, 16, 256, 128, 3, 3, 1, 1, "SAME"),
                                               (1, 9, 10, 128, 264, 3, 3, 1, 1, "SAME")])
def test_conv2d_bwd_filter(dev, tnv, case, dtype):
    N, H, W, C, K, R, S, st, dil, pad = case
    x, w, _ = _conv_case(case, 3)
    xr = rnd(x, dtype)
    wr = w.clone().requires_grad_(True)
    y = tf.conv2d(xr, wr, st, pad, dil)
    g = torch.Generator().manual_seed(8)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    d = ops.conv_desc(N, H, W, C, K, R, S, st, dil, pad, DT[dtype])
    dw = torch.full((R, S, C, K), float("nan"), dtype=torch.float32, device=dev)
    db = torch.full((K,), float("nan"), dtype=torch.float32, device=dev)
    ops.conv2d_bwd_filter(d, to_dev(x, dtype, dev), to_dev(dy, dtype, dev), dw, dbias=db)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-3   # fp32 accumulation of bf16 products
    assert_close(dw.double().cpu(), wr.grad, dtype, f"conv bwd_filter {case}", tol)
    # BiasAddGrad of the same dy (fused into the halo filter gradient)
    assert_close(db.double().cpu(), dy.sum(dim=(0, 1, 2)), dtype, f"bias grad {case}", 2e-5)


# (N, IH, IW, C_in, OH, OW, C_out, k, stride)
TCONV_CASES = [
    (2, 3, 5, 16, 6, 10, 8, 4, 2),       # conv_t1/t2-like k4 s2
    (1, 3, 4, 2, 6, 8, 512, 4, 2),       # conv_t1 exact channel shape (2 -> 512)
    (1, 6, 6, 16, 11, 12, 16, 4, 2),     # odd output: asymmetric tconv pads
    (1, 2, 3, 16, 16, 24, 2, 16, 8),     # conv_t3-like k16 s8 -> 2 classes (tap-dense path)
    (2, 3, 2, 24, 24, 16, 4, 16, 8),     # tap-dense with 4 output channels
    (1, 4, 5, 16, 16, 20, 2, 8, 4),      # tap-dense k8 s4
    (2, 4, 4, 136, 8, 8, 72, 4, 2),      # tails in both channel dims
    (1, 24, 32, 320, 48, 64, 128, 4, 2), # FC-DenseNet transition up 5 (320 -> 128): N = 256 + 64 split GEMMs
]


def _tconv_case(case, seed):
    N, IH, IW, Ci, OH, OW, Co, k, s = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, IH, IW, Ci, generator=g, dtype=torch.float64)
    w = torch.randn(k, k, Co, Ci, generator=g, dtype=torch.float64) / math.sqrt(Ci * 4)
    b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
    return x, w, b


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", TCONV_CASES)
def test_tconv2d_fwd_bias_residual(dev, ntv, case, dtype):
    N, IH, IW, Ci, OH, OW, Co, k, s = case
    x, w, b = _tconv_case(case, 4)
    g = torch.Generator().manual_seed(5)
    res = rnd(torch.randn(N, OH, OW, Co, generator=g, dtype=torch.float64), dtype)
    ref = tf.conv2d_transpose(rnd(x, dtype), rnd(w, dtype), (N, OH, OW, Co), s) + b.float().double() + res
    d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, k, k, s, "SAME", DT[dtype])
    wp = _pack(w, ops.PACK_TCONV_FWD, dtype, dev, ops.tconv_filter_apad(d))
    y = torch.full((N, OH, OW, d.K), float("nan"), dtype=dtype, device=dev)
    resd = to_dev(res, dtype, dev)
    ops.tconv2d_fwd(d, to_dev(x, dtype, dev), wp, y, ops.epilogue(bias=b.float().to(dev), residual=resd))
    torch.cuda.synchronize()
    assert_close(from_dev(y, Co), ref, dtype, f"tconv fwd {case}")


def _tconv_grad_case(case, dtype, dev):
    N, IH, IW, Ci, OH, OW, Co, k, s = case
    x, w, _ = _tconv_case(case, 6)
    xr = rnd(x, dtype).requires_grad_(True)
    wr = rnd(w, dtype).requires_grad_(True)
    y = tf.conv2d_transpose(xr, wr, (N, OH, OW, Co), s)
    g = torch.Generator().manual_seed(9)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, k, k, s, "SAME", DT[dtype])
    return x, w, xr, wr, dy, d


# the input gradient runs the NT kernels, the filter gradient the TN ones:
# each is swept over its own kernel generations (not their cross product)
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", TCONV_CASES)
def test_tconv2d_bwd_data(dev, ntv, case, dtype):
    N, IH, IW, Ci, OH, OW, Co, k, s = case
    x, w, xr, wr, dy, d = _tconv_grad_case(case, dtype, dev)
    wb = _pack(w, ops.PACK_TCONV_BWD, dtype, dev, ops.tconv_filter_apad(d))
    dx = torch.full((N, IH, IW, d.C), float("nan"), dtype=dtype, device=dev)
    ops.tconv2d_bwd_data(d, to_dev(dy, dtype, dev), wb, dx)
    torch.cuda.synchronize()
    assert_close(from_dev(dx, Ci), xr.grad, dtype, f"tconv bwd_data {case}")


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", TCONV_CASES)
def test_tconv2d_bwd_filter(dev, tnv, case, dtype):
    N, IH, IW, Ci, OH, OW, Co, k, s = case
    x, w, xr, wr, dy, d = _tconv_grad_case(case, dtype, dev)
    dw = torch.full((k, k, Co, Ci), float("nan"), dtype=torch.float32, device=dev)
    db = torch.full((Co,), float("nan"), dtype=torch.float32, device=dev)
    ops.tconv2d_bwd_filter(d, to_dev(x, dtype, dev), to_dev(dy, dtype, dev), dw, dbias=db)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-3
    assert_close(dw.double().cpu(), wr.grad, dtype, f"tconv bwd_filter {case}", tol)
    assert_close(db.double().cpu(), dy.sum(dim=(0, 1, 2)), dtype, f"tconv bias grad {case}", 2e-5)


def test_tconv_shape_rule_rejects_375(dev):
    """375x1242 cannot pass FCN's conv_t2 (ceil(375/8)=47 -> pool3 46): TF raises."""
    with pytest.raises(ValueError):
        ops.tconv_desc(1, 11, 38, 512, 23, 77, 256, 4, 4, 2)   # pool5 11x38 -> pool4 23x77


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(2, 6, 8, 16), (1, 7, 9, 24), (1, 5, 5, 8)])
def test_maxpool_fwd_bwd(dev, shape, dtype):
    N, H, W, C = shape
    g = torch.Generator().manual_seed(10)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    x[0, 0, 0, :] = x[0, 0, 1, :]          # exact ties -> first in scan order
    x = rnd(x, dtype).requires_grad_(True)
    y = tf.max_pool2x2(x)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    xd = to_dev(x.detach(), dtype, dev)
    yd = torch.empty(N, H // 2, W // 2, ops.round8(C), dtype=dtype, device=dev)
    ops.maxpool2x2_fwd(xd, yd)
    dxd = torch.full_like(xd, float("nan"))
    ops.maxpool2x2_bwd(xd, yd, to_dev(dy, dtype, dev), dxd)
    torch.cuda.synchronize()
    assert torch.equal(from_dev(yd, C), y.detach())
    assert torch.equal(from_dev(dxd, C), x.grad)
    # fused ReluGrad of a post-ReLU input: relu(x) -> pool; d/dx through both
    xr = torch.relu(x.detach()).requires_grad_(True)
    (tf.max_pool2x2(xr) * dy).sum().backward()
    want = torch.where(xr.detach() > 0, xr.grad, torch.zeros_like(xr.grad))
    xrd = to_dev(xr.detach(), dtype, dev)
    ops.maxpool2x2_fwd(xrd, yd)
    dxd.fill_(float("nan"))
    ops.maxpool2x2_bwd(xrd, yd, to_dev(dy, dtype, dev), dxd, relu_mask=True)
    torch.cuda.synchronize()
    assert torch.equal(from_dev(dxd, C), want)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(2, 6, 8, 16), (1, 7, 9, 24), (1, 5, 5, 8), (4, 96, 312, 64)])
def test_maxpool_argmax_fwd_bwd(dev, shape, dtype):
    """Training form: the forward records its switches, MaxPoolGrad reads them
    (not x); bit-exact with the x-reading pair and the oracle, ties to the
    first max, odd H / W tails zero, fused ReluGrad incl. all-zero windows."""
    N, H, W, C = shape
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    x[0, 0, 0, :] = x[0, 0, 1, :]          # exact ties -> first in scan order
    x[0, 2:4, 2:4, :] = 0.0                # all-equal window (relu: max 0 -> no gradient)
    x = rnd(x, dtype).requires_grad_(True)
    y = tf.max_pool2x2(x)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    xd = to_dev(x.detach(), dtype, dev)
    Cp = ops.round8(C)
    yd = torch.empty(N, H // 2, W // 2, Cp, dtype=dtype, device=dev)
    idx = torch.full((N * (H // 2) * (W // 2) * Cp,), 255, dtype=torch.uint8, device=dev)
    ops.maxpool2x2_fwd_argmax(xd, yd, idx)
    dxd = torch.full_like(xd, float("nan"))
    ops.maxpool2x2_bwd_argmax(idx, to_dev(dy, dtype, dev), dxd)
    torch.cuda.synchronize()
    assert torch.equal(from_dev(yd, C), y.detach())
    assert torch.equal(from_dev(dxd, C), x.grad)
    for relu_in in (False, True):
        xr = (torch.relu(x.detach()) if relu_in else x.detach()).requires_grad_(True)
        (tf.max_pool2x2(xr) * dy).sum().backward()
        want = torch.where(xr.detach() > 0, xr.grad, torch.zeros_like(xr.grad))
        xrd = to_dev(xr.detach(), dtype, dev)
        ops.maxpool2x2_fwd_argmax(xrd, yd, idx)
        dxd.fill_(float("nan"))
        ops.maxpool2x2_bwd_argmax(idx, to_dev(dy, dtype, dev), dxd, relu_mask=True)
        ref = torch.full_like(xrd, float("nan"))
        ops.maxpool2x2_bwd(xrd, yd, to_dev(dy, dtype, dev), ref, relu_mask=True)
        torch.cuda.synchronize()
        assert torch.equal(dxd, ref)
        if relu_in:
            assert torch.equal(from_dev(dxd, C), want)


@pytest.mark.parametrize("dtype", DTYPES)
def test_avgpool_fwd_bwd(dev, dtype):
    N, H, W, C = 2, 7, 6, 16
    g = torch.Generator().manual_seed(11)
    x = rnd(torch.randn(N, H, W, C, generator=g, dtype=torch.float64), dtype).requires_grad_(True)
    y = tf.avg_pool2x2(x)
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    xd = to_dev(x.detach(), dtype, dev)
    yd = torch.empty(N, H // 2, W // 2, C, dtype=dtype, device=dev)
    ops.avgpool2x2_fwd(xd, yd)
    dxd = torch.full_like(xd, float("nan"))
    ops.avgpool2x2_bwd(to_dev(dy, dtype, dev), dxd)
    torch.cuda.synchronize()
    assert_close(from_dev(yd), y.detach(), dtype, "avgpool fwd")
    assert_close(from_dev(dxd), x.grad, dtype, "avgpool bwd")


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("K", [16, 64, 4096, 8])
def test_bias_relu_bwd(dev, dtype, K):
    N, H, W = 2, 9, 13
    g = torch.Generator().manual_seed(12)
    y = rnd(torch.relu(torch.randn(N, H, W, K, generator=g, dtype=torch.float64)), dtype)
    dy = rnd(torch.randn(N, H, W, K, generator=g, dtype=torch.float64), dtype)
    dz = dy * (y > 0)
    kv = K if K != 8 else 2
    db = dz[..., :kv].sum(dim=(0, 1, 2))
    yd, dyd = to_dev(y, dtype, dev), to_dev(dy, dtype, dev)
    dzd = torch.empty_like(dyd)
    dbd = torch.zeros(kv, dtype=torch.float32, device=dev)
    ops.bias_relu_bwd(dyd, yd, dzd, dbd, kv, relu=True)
    torch.cuda.synchronize()
    assert torch.equal(from_dev(dzd), dz)
    assert_close(dbd.double().cpu(), db, torch.float32, "dbias", 1e-5)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("K,P,kv", [(4096, 4 * 12 * 39, 4096), (512, 1000, 500), (1024, 7, 1024), (256, 333, 256)])
def test_bias_grad_wide_colsum(dev, dtype, K, P, kv):
    """BiasAddGrad alone (no ReLU, dz = dy) of a wide dy: col_sum_k + reduce_rows_k
    (C2's conv6 / conv7 bias gradients, P = 4 x 12 x 39), ragged row ranges,
    fewer rows than row lanes, and a partial last chunk group (K = 4096 / 8 = 512
    chunks = 8 groups; fp32: 1024 chunks)."""
    g = torch.Generator().manual_seed(21)
    dy = rnd(torch.randn(1, 1, P, K, generator=g, dtype=torch.float64), dtype)
    dyd = to_dev(dy, dtype, dev)
    dbd = torch.full((kv,), 7.0, dtype=torch.float32, device=dev)
    ops.bias_relu_bwd(dyd, None, dyd, dbd, kv, relu=False)
    torch.cuda.synchronize()
    assert torch.equal(from_dev(dyd), dy)          # dy untouched
    db = dy[..., :kv].sum(dim=(0, 1, 2))
    assert_close(dbd.double().cpu(), db, torch.float32, "dbias", 1e-5)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("labels_kind", ["index", "onehot"])
def test_softmax_xent(dev, dtype, labels_kind):
    N, H, W, C = 2, 12, 16, 2
    g = torch.Generator().manual_seed(13)
    z = rnd(torch.randn(N, H, W, C, generator=g, dtype=torch.float64) * 3, dtype).requires_grad_(True)
    lab = torch.randint(0, C, (N, H, W), generator=g)
    vh, vw = 10, 13
    mask = torch.zeros(N, H, W, dtype=torch.float64)
    mask[:, :vh, :vw] = 1
    y1 = tf.one_hot(lab, C)
    loss = tf.mean_softmax_xent(z, y1, mask)
    loss.backward()
    zd = to_dev(z.detach(), dtype, dev)
    dz = torch.full_like(zd, float("nan"))
    ls = torch.zeros(1, dtype=torch.float32, device=dev)
    cnt = N * vh * vw
    labd = lab.to(torch.uint8).to(dev) if labels_kind == "index" else y1.float().to(dev).contiguous()
    ops.softmax_xent(zd, labd, dz, ls, C, (vh, vw), grad_scale=1.0 / cnt)
    torch.cuda.synchronize()
    assert abs(ls.item() / cnt - loss.item()) <= 1e-5 * max(1.0, abs(loss.item()))
    assert_close(from_dev(dz, C), z.grad, dtype, "dlogits")
    assert dz[..., C:].abs().max().item() == 0


def test_argmax_and_confusion(dev):
    g = torch.Generator().manual_seed(14)
    z = torch.randn(2, 5, 7, 2, generator=g)
    z[0, 0, 0] = torch.tensor([1.0, 1.0])   # tie -> class 0
    zd = to_dev(z.double(), torch.float32, dev)
    pred = torch.empty(2 * 5 * 7, dtype=torch.int64, device=dev)
    ops.argmax(zd, pred, 2)
    torch.cuda.synchronize()
    assert torch.equal(pred.cpu().view(2, 5, 7), tf.argmax(z.double()))
    lab = torch.randint(0, 2, (2, 5, 7), generator=g, dtype=torch.uint8)
    conf = torch.zeros(4, dtype=torch.int64, device=dev)
    ops.confusion(pred, lab.to(dev), conf, 2, (4, 6))
    torch.cuda.synchronize()
    p = pred.cpu().view(2, 5, 7)[:, :4, :6].reshape(-1)
    t = lab[:, :4, :6].reshape(-1).long()
    ref = torch.bincount(t * 2 + p, minlength=4)
    assert torch.equal(conf.cpu(), ref)


def test_adam_tf1(dev):
    n = 1003
    g = torch.Generator().manual_seed(15)
    p0 = torch.randn(n, generator=g, dtype=torch.float64)
    opt = tf.AdamTF1(lr=1e-3)
    params = {"p": p0.clone()}
    pd = p0.float().to(dev)
    m = torch.zeros_like(pd)
    v = torch.zeros_like(pd)
    for t in range(1, 4):
        gr = torch.randn(n, generator=g, dtype=torch.float64) * 1e-3
        params = opt.apply(params, {"p": gr.float().double() * 9.0})
        ops.adam_tf1_step(pd, gr.float().to(dev), m, v, 1e-3, t, grad_scale=9.0)
    torch.cuda.synchronize()
    assert_close(pd.double().cpu(), params["p"], torch.float32, "adam", 1e-6)


def _np_avalanche32(x):
    M = 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    x ^= x >> 16
    return x


def _np_uniform(seed, idx):
    """seg_uniform (csrc/common.h): counters in groups of 8, idx = 8 q + j; the
    group hash of q is a counter finalizer with the avalanched seed key XORed
    in after the first multiply, then one xorshift-multiply-xorshift of
    (group hash + j * golden ratio) per element."""
    M = 0xFFFFFFFF
    key = _np_avalanche32(((seed ^ (seed >> 32)) & M) ^ 0x632BE59B)
    q, j = idx >> 3, idx & 7
    x = ((q & M) ^ (((q >> 32) * 0x85EBCA6B) & M)) & M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= key
    x ^= x >> 15
    x = (x * 0x846CA68B) & M
    x ^= x >> 16
    x = (x + j * 0x9E3779B9) & M
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M
    x ^= x >> 15
    return (x >> 8) / 16777216.0


def test_uniform_grouped_counters_are_independent():
    """Counters in groups of 8 share a group hash: the Bernoulli(0.2) keep
    masks of neighbours within a group, and of the same slot in adjacent
    groups, stay uncorrelated, and every slot keeps its rate."""
    from tests.test_gpu_ops_r2 import _np_uniform_vec
    u = _np_uniform_vec(1234, np.arange(1 << 18, dtype=np.uint64)).reshape(-1, 8)
    k = (u < 0.2).astype(np.float64)
    assert np.all(np.abs(k.mean(0) - 0.2) < 0.01)
    for a, b in ((k[:, :-1], k[:, 1:]), (k[:-1], k[1:]), (k[:, :4], k[:, 4:])):
        c = np.corrcoef(a.ravel(), b.ravel())[0, 1]
        assert abs(c) < 0.01, c


def test_uniform_streams_of_different_seeds_are_not_shifts():
    """with F(idx + key) two seeds' masks were shifted copies of one
    stream; with the key mixed non-additively no small shift aligns them."""
    a = np.array([_np_uniform(1000, i) for i in range(4096)])
    for seed in (1001, 1131, 1000 + 7919):
        b = np.array([_np_uniform(seed, i) for i in range(4096)])
        for shift in range(0, 2048, 7):
            assert np.mean(a[shift:] == b[:4096 - shift]) < 0.01
            assert np.mean(b[shift:] == a[:4096 - shift]) < 0.01
    assert abs(a.mean() - 0.5) < 0.02


@pytest.mark.parametrize("dtype", DTYPES)
def test_dropout_tf1(dev, dtype):
    n, kp, seed = 4096, 0.8, 1234
    x = torch.ones(n, dtype=dtype, device=dev)
    y = torch.empty_like(x)
    ops.dropout_fwd(x, y, kp, seed)
    torch.cuda.synchronize()
    u = np.array([_np_uniform(seed, i) for i in range(n)])
    ref = tf.dropout(torch.ones(n, dtype=torch.float64), kp, torch.from_numpy(u))
    assert_close(y.double().cpu(), ref, dtype, "dropout")
    keep = (y > 0).float().mean().item()
    assert abs(keep - kp) < 0.03


@pytest.mark.parametrize("dtype", DTYPES)
def test_bn_relu(dev, dtype):
    N, H, W, C = 2, 5, 6, 24
    g = torch.Generator().manual_seed(16)
    x = rnd(torch.randn(N, H, W, C, generator=g, dtype=torch.float64), dtype).requires_grad_(True)
    gamma = (1 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)).float().double().requires_grad_(True)
    beta = (0.1 * torch.randn(C, generator=g, dtype=torch.float64)).float().double().requires_grad_(True)
    y = torch.relu(tf.batch_norm_frozen(x, gamma, beta))
    dy = rnd(torch.randn(y.shape, generator=g, dtype=torch.float64), dtype)
    (y * dy).sum().backward()
    xd = to_dev(x.detach(), dtype, dev)
    yd = torch.empty_like(xd)
    gd, bd = gamma.detach().float().to(dev), beta.detach().float().to(dev)
    ops.bn_relu_fwd(xd, yd, gd, bd, C)
    dxd = torch.empty_like(xd)
    dg = torch.zeros(C, device=dev)
    dbt = torch.zeros(C, device=dev)
    ops.bn_relu_bwd(xd, yd, to_dev(dy, dtype, dev), dxd, gd, dg, dbt, C)
    torch.cuda.synchronize()
    assert_close(from_dev(yd), y.detach(), dtype, "bn fwd")
    assert_close(from_dev(dxd), x.grad, dtype, "bn dx")
    assert_close(dg.double().cpu(), gamma.grad, torch.float32, "dgamma", 1e-4)
    assert_close(dbt.double().cpu(), beta.grad, torch.float32, "dbeta", 1e-4)
    # ReLU mask re-derived from x (y not read): bit-identical to the y-masked kernel
    dx2 = torch.full_like(xd, float("nan"))
    dg2, db2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    ops.bn_relu_bwd(xd, None, to_dev(dy, dtype, dev), dx2, gd, dg2, db2, C, beta=bd)
    # accumulate mode into a channel slice of a wider buffer (shared concat gradient)
    wide = rnd(torch.randn(N, H, W, C + 16, generator=g, dtype=torch.float64), dtype)
    wd = to_dev(wide, dtype, dev)
    dg3, db3 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    ops.bn_relu_bwd(xd, None, to_dev(dy, dtype, dev), wd[..., 8:8 + C], gd, dg3, db3, C, beta=bd, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(dx2, dxd) and torch.equal(dg2, dg) and torch.equal(db2, dbt)
    ref = wide.clone()
    ref[..., 8:8 + C] += x.grad
    assert_close(from_dev(wd), ref, dtype, "bn dx accumulate")
    assert torch.equal(dg3, dg)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(2, 5, 7, 3, 8, 8, 8), (1, 4, 4, 8, 4, 6, 8), (1, 3, 5, 11, 4, 5, 16)])
def test_prepare_input(dev, dtype, shape):
    """fp32 NHWC image -> zero-padded compute tensor (bit-exact: a cast)."""
    N, H, W, c, HP, WP, CP = shape
    img = torch.randn(N, H, W, c, generator=torch.Generator().manual_seed(18))
    ref = torch.zeros(N, HP, WP, CP)
    ref[:, :H, :W, :c] = img
    x = torch.full((N, HP, WP, CP), float("nan"), device=dev, dtype=dtype)
    ops.prepare_input(img.to(dev), x)
    torch.cuda.synchronize()
    assert torch.equal(x.cpu(), ref.to(dtype))


RESIZE_CASES = [(1, 5, 7, 3, 9, 15),
                (2, 6, 9, 2, 41, 65),      # x8-style upsample of 2-class logits (DeepLab head)
                (1, 9, 15, 4, 5, 7),       # downsample
                (2, 1, 6, 3, 4, 11),       # single source row
                (1, 4, 5, 2, 1, 1),        # single output pixel
                (1, 3, 3, 8, 128, 96)]     # large factor, C = 8


@pytest.mark.parametrize("case", RESIZE_CASES)
def test_resize_bilinear(dev, case):
    """ResizeBilinear(align_corners=True) forward and its gather-form gradient
    (every source pixel sums the output positions that read it)."""
    N, H, W, C, OH, OW = case
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64).float().double().requires_grad_(True)
    y = tf.resize_bilinear(x, (OH, OW))
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64).float().double()
    (y * dy).sum().backward()
    xd = x.detach().float().to(dev).contiguous()
    yd = torch.empty(N, OH, OW, C, device=dev)
    ops.resize_bilinear_fwd(xd, yd)
    dxd = torch.empty(N, H, W, C, device=dev)
    ops.resize_bilinear_bwd(dy.float().to(dev).contiguous(), dxd)
    torch.cuda.synchronize()
    assert_close(yd.double().cpu(), y.detach(), torch.float32, "resize fwd", 1e-5)
    assert_close(dxd.double().cpu(), x.grad, torch.float32, "resize bwd", 1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", [(2, 48, 156, 8, 384, 1248), (2, 6, 9, 16, 41, 65), (1, 3, 3, 8, 128, 96),
                                  (1, 9, 15, 8, 5, 7)])
def test_resize_bilinear_8wide_equals_scalar(dev, case, dtype):
    """The 8-channel (16-byte) resize kernels (16-bit, C % 8 == 0, aligned
    rows: DeepLab's x8 logits upsampling) against the per-element kernels the
    launcher takes for misaligned storage of the same values: bit-identical
    forward and gradient."""
    N, H, W, C, OH, OW = case
    g = torch.Generator(device=dev).manual_seed(19)

    def misaligned(shape, dt):
        buf = torch.empty(int(np.prod(shape)) + 1, dtype=dt, device=dev)
        return buf[1:].view(shape)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    dy = torch.randn(N, OH, OW, C, device=dev, generator=g).to(dtype)
    y8 = torch.full((N, OH, OW, C), float("nan"), dtype=dtype, device=dev)
    ops.resize_bilinear_fwd(x, y8)
    xs = misaligned(x.shape, dtype)
    xs.copy_(x)
    ys = misaligned(y8.shape, dtype)
    ops.resize_bilinear_fwd(xs, ys)
    dx8 = torch.full((N, H, W, C), float("nan"), device=dev)
    ops.resize_bilinear_bwd(dy, dx8)
    dys = misaligned(dy.shape, dtype)
    dys.copy_(dy)
    dxs = misaligned(dx8.shape, torch.float32)
    ops.resize_bilinear_bwd(dys, dxs)
    torch.cuda.synchronize()
    assert torch.equal(y8.view(torch.int16), ys.view(torch.int16))
    assert torch.equal(dx8.view(torch.int32), dxs.view(torch.int32))


@pytest.mark.parametrize("dtype", DTYPES)
def test_adam_tf1_pack_matches_step_plus_pack(dev, dtype):
    """Fused multi-tensor Adam + packed copies == adam_tf1_step then pack_filter.
    params / m / v: same TF1 expression, FMA contraction may differ between the
    two kernels -> 2e-6 relative; packed copies: bitwise equal to pack_filter
    of the fused kernel's own params (incl. untouched zero padding)."""
    g = torch.Generator().manual_seed(11)
    # (shape, modes): conv1_1-like padded C, ragged 64-tiles, tconv, biases
    spec = [((3, 3, 3, 64), (ops.PACK_KRSC,)),
            ((3, 3, 72, 136), (ops.PACK_KRSC, ops.PACK_HWIO)),
            ((4, 4, 2, 64), (ops.PACK_TCONV_FWD, ops.PACK_TCONV_BWD)),
            ((64,), ()), ((2,), ()), ((1, 1, 40, 2), (ops.PACK_KRSC, ops.PACK_HWIO))]
    offs, off = [], 0
    for shape, _ in spec:
        offs.append(off)
        off += (int(np.prod(shape)) + 3) // 4 * 4
    P = (torch.randn(off, generator=g) * 0.1).to(dev)
    Gr = (torch.randn(off, generator=g) * 0.01).to(dev)
    M = (torch.randn(off, generator=g) * 0.001).to(dev)
    V = (torch.rand(off, generator=g) * 1e-4).to(dev)
    # alignment padding between variables holds zeros in the store (grad / m / v)
    pad = torch.ones(off, dtype=torch.bool)
    for (shape, _), o in zip(spec, offs):
        pad[o:o + int(np.prod(shape))] = False
    for t in (Gr, M, V):
        t[pad.to(dev)] = 0
    ref = [t.clone() for t in (P, Gr, M, V)]
    copies, ref_copies, segs = [], [], []
    for (shape, modes), o in zip(spec, offs):
        rows = tr = None
        if len(shape) == 4:
            R, S, A, B = shape
            for mode in modes:
                t = torch.zeros(ops.packed_shape(R, S, A, B, mode), dtype=dtype, device=dev)
                e = (t, ops.round8(A), ops.round8(B))
                if mode in (ops.PACK_HWIO, ops.PACK_TCONV_FWD):
                    rows = e
                else:
                    tr = e
                copies.append((t, shape, o, mode))
            rs, a, b = R * S, A, B
        else:
            rs, a, b = 1, 1, int(np.prod(shape))
        segs.append((o, rs, a, b, rows, tr))
    plan = ops.AdamPlan(segs, dev)
    kw = dict(beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=9.0)
    for step in (1, 2):
        ops.adam_tf1_pack(P, Gr, M, V, plan, 1e-3, step, dtype=DT[dtype], **kw)
        ops.adam_tf1_step(*ref, 1e-3, step, **kw)
    torch.cuda.synchronize()
    for a_, b_ in zip((P, M, V), (ref[0], ref[2], ref[3])):
        torch.testing.assert_close(a_, b_, rtol=2e-6, atol=1e-9)
    for t, shape, o, mode in copies:
        R, S, A, B = shape
        src = P[o:o + R * S * A * B].view(R, S, A, B).contiguous()
        want = torch.zeros_like(t)
        ops.pack_filter(src, want, ops.round8(A), ops.round8(B), mode)
        torch.cuda.synchronize()
        assert torch.equal(t, want), f"copy mode {mode} of {shape}"


# (N, H, W, C, K, R): filters whose gradient takes the fused wgrad + TF1 Adam launch
ADAM_FUSED_CASES = [
    (1, 5, 7, 40, 264, 7),      # conv6-like 7x7; K tail of the 256-wide tile
    (1, 5, 7, 36, 264, 7),      # c_valid = 36 < Cg = 40: padding rows of the packed copies untouched
    (2, 6, 9, 512, 512, 1),     # conv7-like 1x1
    (2, 11, 13, 256, 392, 1),   # 9 pixel stages of 32, N tail of the 128-wide half tile
    (2, 12, 39, 256, 2048, 7),  # 7x7 over 2048 columns: multi-round half-tile grid, 15 pixel stages
]


# (tn3_half, adam_tr_fused): igemm_tn3's fused epilogue on half / full tiles
# (the KRSC copy by the transpose, or in the epilogue)
@pytest.fixture(params=[(0, 0), (1, 0), (5, 0), (0, 1)],
                ids=["default", "half-tiles-multi-round", "half-tiles", "full-tiles-tr-fused"])
def adam_tiles(request, dev):
    half, trf = request.param
    ops.set_option("tn3_half", half)
    ops.set_option("adam_tr_fused", trf)
    yield request.param
    ops.set_option("tn3_half", 0)
    ops.set_option("adam_tr_fused", 0)


@pytest.mark.parametrize("case", ADAM_FUSED_CASES)
def test_conv2d_bwd_filter_adam_fused(dev, case, adam_tiles):
    """seg_conv2d_bwd_filter_adam == Conv2DBackpropFilter, then TF1 Adam
    (FCN.py:338) on the filter, then repacking of the HWIO / KRSC copies."""
    N, H, W, C, K, R = case
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=ops.BF16)
    assert ops.wgrad_adam_fusable(d)
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    dy = torch.randn(N, H, W, K, generator=g, dtype=torch.float64)
    p0 = torch.randn(R, R, C, K, generator=g) * 0.05
    m0 = torch.randn(R, R, C, K, generator=g) * 1e-3
    v0 = torch.rand(R, R, C, K, generator=g) * 1e-5
    xd, dyd = to_dev(x, torch.bfloat16, dev), to_dev(dy, torch.bfloat16, dev)
    # reference gradient from the plain filter-gradient path
    gref = torch.empty(R, R, C, K, device=dev)
    ops.conv2d_bwd_filter(d, xd, dyd, gref)
    p, m, v = p0.to(dev), m0.to(dev), v0.to(dev)
    cp, kp = ops.round8(C), ops.round8(K)
    rows = torch.full(ops.packed_shape(R, R, C, K, ops.PACK_HWIO), 7.0, dtype=torch.bfloat16, device=dev)
    tr = torch.full(ops.packed_shape(R, R, C, K, ops.PACK_KRSC), 7.0, dtype=torch.bfloat16, device=dev)
    dw = torch.full((R, R, C, K), float("nan"), device=dev)
    lr, t, gs = 1e-3, 3, 0.5
    ops.conv2d_bwd_filter_adam(d, xd, dyd, p, m, v, lr, t, grad_scale=gs, rows=(rows, cp, kp), tr=(tr, cp, kp),
                               dw=dw)
    torch.cuda.synchronize()
    gr = gref.cpu().double()
    assert (dw.cpu().double() - gr).abs().max().item() <= 1e-6 * gr.abs().max().item()
    gc = gr * gs
    me = 0.9 * m0.double() + 0.1 * gc
    ve = 0.999 * v0.double() + 0.001 * gc * gc
    lr_t = lr * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
    pe = p0.double() - lr_t * me / (ve.sqrt() + 1e-8)
    # fp32 arithmetic as TF1's kernel: (1 - beta2) = 1 - 0.999f carries 4.7e-5 relative
    for got, ref, nm, tol in ((p, pe, "p", 1e-5), (m, me, "m", 1e-5), (v, ve, "v", 1e-4)):
        err = (got.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < tol, (nm, err)
    # packed copies: valid entries = bf16(new p), padding entries untouched (7.0)
    pb = p.cpu().to(torch.bfloat16)
    rh = rows.cpu().view(R * R, cp, kp)
    assert torch.equal(rh[:, :C, :K], pb.view(R * R, C, K))
    if cp > C:
        assert (rh[:, C:, :] == 7.0).all()
    tk = tr.cpu().view(kp, R * R, cp)
    assert torch.equal(tk[:K, :, :C], pb.view(R * R, C, K).permute(2, 0, 1))
    if cp > C:
        assert (tk[:, :, C:] == 7.0).all()


# (N, H, W, C, K, R): halo filter gradient (split-K, fused bias), first layer
# (C = 3 -> 8, split-K), generic TN GEMMs (split-K, bias by the fallback)
SPLIT_WGRAD_CASES = [
    (2, 24, 40, 64, 128, 3),
    (2, 19, 131, 3, 48, 3),
    (2, 19, 131, 3, 64, 3),     # wgrad_c8 (K = 64): ragged 4x64 tiles, split-K
    (1, 6, 9, 512, 264, 7),
    (2, 6, 9, 40, 24, 1),
]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("case", SPLIT_WGRAD_CASES)
def test_conv2d_bwd_filter_begin_end(dev, case, dtype):
    """seg_conv2d_bwd_filter_begin + _end (reduction on a second stream) ==
    seg_conv2d_bwd_filter, gradient and BiasAddGrad bit-for-bit."""
    N, H, W, C, K, R = case
    d = ops.conv_desc(N, H, W, C, K, R, R, dtype=DT[dtype])
    g = torch.Generator().manual_seed(31)
    x = to_dev(torch.randn(N, H, W, C, generator=g, dtype=torch.float64), dtype, dev)
    dy = to_dev(torch.randn(N, H, W, K, generator=g, dtype=torch.float64), dtype, dev)
    ref, rdb = torch.empty(R, R, C, K, device=dev), torch.empty(K, device=dev)
    ops.conv2d_bwd_filter(d, x, dy, ref, dbias=rdb)
    out = torch.full((R, R, C, K), float("nan"), device=dev)
    db = torch.full((K,), float("nan"), device=dev)
    wsb = torch.empty(max(256, ops.conv_workspace(d, ops.OP_BWD_FILTER)), dtype=torch.uint8, device=dev)
    tok = ops.conv2d_bwd_filter_begin(d, x, dy, out, wsb, dbias=db)
    side = torch.cuda.Stream(device=dev)
    ev = torch.cuda.Event()
    ev.record()
    side.wait_event(ev)
    ops.conv2d_bwd_filter_end(tok, out, wsb, db, stream=side)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(db, rdb)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("chans", [(16, 48, 8), (24, 40, 12), (5, 11), (64, 16, 16, 16, 430)],
                         ids=["aligned", "aligned-tail", "unaligned", "densenet"])
def test_concat_fwd_bwd(dev, dtype, chans):
    """tf.concat(axis=-1) forward and its gradient split (write and
    accumulate), channel-padded NHWC parts; bit-exact (copies / one add)."""
    N, H, W = 2, 5, 7
    g = torch.Generator().manual_seed(19)
    xs = [torch.randn(N, H, W, c, generator=g) for c in chans]
    parts = [(to_dev(x.double(), dtype, dev), c) for x, c in zip(xs, chans)]
    tot = sum(chans)
    y = torch.full((N, H, W, ops.round8(tot)), float("nan"), dtype=dtype, device=dev)
    ops.concat_fwd(parts, y, tot)
    torch.cuda.synchronize()
    want = torch.cat([x.to(dtype) for x in xs], dim=-1)
    assert torch.equal(y[..., :tot].cpu(), want)
    if y.shape[-1] > tot:
        assert y[..., tot:].abs().max().item() == 0
    dy = to_dev(torch.randn(N, H, W, tot, generator=g, dtype=torch.float64), dtype, dev)
    olds = [to_dev(torch.randn(N, H, W, c, generator=g, dtype=torch.float64), dtype, dev) for c in chans]
    dsts = [o.clone() for o in olds]
    acc = [i % 2 == 1 for i in range(len(chans))]
    ops.concat_bwd(dy, [(d, c, a) for d, c, a in zip(dsts, chans, acc)])
    torch.cuda.synchronize()
    off = 0
    for d, o, c, a in zip(dsts, olds, chans, acc):
        sl = dy[..., off:off + c].float().cpu()
        ref = (o[..., :c].float().cpu() + sl).to(dtype) if a else sl.to(dtype)
        assert torch.equal(d[..., :c].cpu(), ref), (c, a)
        off += c
