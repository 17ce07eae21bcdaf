"""The ReluGrad mask as bits (round 6): conv1_1 of FCN / VGG (3 -> 64,
Network/model/FCN.py:55) writes its ReLU mask at 1 bit per element beside its
map (seg_conv2d_fwd_relu_bits, conv_c8_fwd), and conv1_2's input gradient
(:56, conv_res64pp) reads those bits instead of the 16-bit map
(seg_conv2d_bwd_data_bits).  Every output is compared bit for bit with the
16-bit-mask launches, which the op-level and full-size tests pin to the
oracle; the bits themselves against torch's (y > 0) packed."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import models as M
from semanticsegmentation_tensorflow_amd import ops, tf
from tests.model_inputs import he_weights, synthetic_batch
from tests.test_gpu_fcn import build_fcn

pytestmark = pytest.mark.gpu

SHAPES = [(1, 8, 32), (1, 22, 70), (4, 96, 320), (3, 196, 300), (2, 384, 1248)]
DT = {torch.bfloat16: ops.BF16, torch.float16: ops.F16}


def _i16(t):
    return t.view(torch.int16)


def _pack_bits(y):
    """bit k % 8 of byte k // 8 = y[..., k] > 0."""
    N, H, W, K = y.shape
    pos = (y.float() > 0).view(N, H, W, K // 8, 8).to(torch.int32)
    return (pos << torch.arange(8, device=y.device, dtype=torch.int32)).sum(-1).to(torch.uint8)


@pytest.fixture(params=[1, 0], ids=["tr", "rows"])
def smallc_tr(request, dev):
    """conv_c8_fwd with transposed accumulators (default) and the row form."""
    ops.set_option("smallc_tr", request.param)
    yield request.param
    ops.set_option("smallc_tr", 1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("K", [64, 32, 16])
@pytest.mark.parametrize("shape", SHAPES)
def test_fwd_relu_bits(dev, smallc_tr, shape, K, dtype):
    N, H, W = shape
    d = ops.conv_desc(N, H, W, 3, K, 3, 3, dtype=DT[dtype])
    assert ops.conv_kernel_info(d, ops.OP_FWD)[0].startswith("conv_c8")
    assert ops.conv2d_fwd_relu_bits_ok(d)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.zeros(N, H, W, 8, device=dev, dtype=dtype)
    x[..., :3] = (torch.randn(N, H, W, 3, device=dev, generator=g) * 50).to(dtype)
    w32 = torch.randn(3, 3, 3, K, device=dev, generator=g) / 60.0
    bias = torch.randn(K, device=dev, generator=g) * 0.5
    wk = torch.zeros(ops.packed_shape(3, 3, 3, K, ops.PACK_KRSC, 8), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, 8, K, ops.PACK_KRSC)
    epi = ops.epilogue(bias=bias, relu=True)
    ref = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
    ops.conv2d_fwd(d, x, wk, ref, epi)
    y = torch.full_like(ref, float("nan"))
    bits = torch.full((N, H, W, K // 8), 0xA5, dtype=torch.uint8, device=dev)
    ops.conv2d_fwd_relu_bits(d, x, wk, y, bits, epi)
    torch.cuda.synchronize()
    assert torch.equal(_i16(y), _i16(ref))
    assert torch.equal(bits, _pack_bits(ref))
    frac = (ref > 0).float().mean().item()
    assert 0.2 < frac < 0.8, frac


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("scale", [1.0, 1.25])
@pytest.mark.parametrize("shape", SHAPES)
def test_bwd_data_bits_equals_16bit_mask(dev, shape, scale, dtype):
    N, H, W = shape
    d = ops.conv_desc(N, H, W, 64, 64, 3, 3, dtype=DT[dtype])
    assert ops.conv2d_bwd_data_bits_ok(d)
    g = torch.Generator(device=dev).manual_seed(9)
    dy = torch.randn(N, H, W, 64, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, 64, 64, device=dev, generator=g) / 24.0
    mask = torch.relu(torch.randn(N, H, W, 64, device=dev, generator=g)).to(dtype)    # ~half zeros
    wh = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_HWIO, 64), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, 64, 64, ops.PACK_HWIO)
    ws = ops.Workspace(dev)
    ref = torch.full((N, H, W, 64), float("nan"), dtype=dtype, device=dev)
    ops.conv2d_bwd_data(d, dy, wh, ref, ws, None, ops.epilogue(relu_mask=mask, mask_scale=scale))
    got = torch.full_like(ref, float("nan"))
    ops.conv2d_bwd_data_bits(d, dy, wh, _pack_bits(mask), got, scale, ws)
    torch.cuda.synchronize()
    assert torch.equal(_i16(got), _i16(ref))
    if scale == 1.0:     # the C entry with no epilogue at all: the plain ReluGrad
        bits = _pack_bits(mask)
        raw = torch.full_like(ref, float("nan"))
        dd = ops._with_ld(d, raw, dy)
        wsp, wss = ws.ptr_size(ops.conv_workspace(dd, ops.OP_BWD_DATA))
        assert ops._lib.lib().seg_conv2d_bwd_data_bits(ctypes.byref(dd), ops.ptr(dy), ops.ptr(wh), None, ops.ptr(bits),
                                                         bits.shape[-1], ops.ptr(raw), wsp, wss, None) == 0
        torch.cuda.synchronize()
        assert torch.equal(_i16(raw), _i16(ref))
    zero = mask == 0
    assert bool((got[zero] == 0).all()) and bool((got[~zero] != 0).any())


def test_bits_entry_points_refuse_other_kernels(dev):
    """Only conv_c8_fwd writes and only conv_res64pp reads the bits: the _ok
    queries say no elsewhere and the launches refuse (nothing computed)."""
    wide = ops.conv_desc(1, 16, 64, 128, 128, 3, 3, dtype=ops.BF16)
    assert not ops.conv2d_fwd_relu_bits_ok(wide)
    assert not ops.conv2d_bwd_data_bits_ok(wide)
    assert not ops.conv2d_bwd_data_bits_ok(ops.conv_desc(1, 16, 64, 64, 64, 3, 3, dtype=ops.F32))
    d = ops.conv_desc(1, 16, 64, 64, 64, 3, 3, dtype=ops.BF16)
    dy = torch.zeros(1, 16, 64, 64, dtype=torch.bfloat16, device=dev)
    wh = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_HWIO, 64), dtype=torch.bfloat16, device=dev)
    dx = torch.zeros_like(dy)
    bits = torch.zeros(1, 16, 64, 9, dtype=torch.uint8, device=dev)   # 9-byte rows: not 8-aligned
    with pytest.raises((ValueError, RuntimeError)):
        ops.conv2d_bwd_data_bits(d, dy, wh, bits, dx)


def test_session_step_with_bits_is_bit_identical(dev):
    """Two FCN training steps (bf16) planned with the bits and without: every
    variable after the updates and the loss equal bit for bit."""
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
    img, lab = synthetic_batch(N, H, W, 3)
    feed = {image: img, labels: lab, keep: 1.0}
    sess = []
    for bits in (True, False):
        s = tf.Session(compute_dtype="bf16")
        s.relu_bits = bits
        s.run(tf.global_variables_initializer())
        for k, v in he_weights(M.fcn_param_shapes(3, 2), 2).items():
            s.assign(k, v)
        for _ in range(2):
            s.run(train_step, feed_dict=feed)
        sess.append(s)
    a, b = sess
    (pa,) = [p for p in a.plans.values() if p.train]
    (pb,) = [p for p in b.plans.values() if p.train]
    assert len(pa.mask_bits) == 1 and not pb.mask_bits
    for v in a.store.vars:
        assert np.array_equal(a.variable_value(v.var_name), b.variable_value(v.var_name)), v.var_name
    assert a.run(loss, feed_dict=feed) == b.run(loss, feed_dict=feed)
