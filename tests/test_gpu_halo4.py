"""conv_halo4 (one wave per SIMD, one barrier per (tap, 64-channel) step:
the 3x3 Conv2D forward / Conv2DBackpropInput of conv3_1 ... conv5_3,
Network/model/FCN.py:55-99) against conv_halo2, the 8-wave kernel it replaces
(option halo4=0), in both of its forms: 4 waves of 128 px x 128 ch (one
per SIMD, halo4=1) and 8 waves of 128 px x 64 ch (two per SIMD, halo4=2).
All accumulate every output element over the same (chunk,
tap, k-step) sequence of the same 16x16x32 MFMAs and run the same epilogue
arithmetic, so every output is compared bit for bit; conv_halo2 itself is
pinned to the oracle by the op-level and full-size parity tests, and one case
is also checked against torch's fp32 conv.

Shapes: C2's conv3_2 / conv4_1 / conv4_2 (16 x 16 tiles, two N tiles at 512
channels), an 8 x 32-tile plan, ragged images (partial tiles at the right /
bottom edge), an N tail (320 channels: a half-empty second N tile), 3-way
split-K (conv5_x) and a forced split plan.  Epilogues: bias + ReLU, BN affine,
residual, dropout, the ReluGrad mask of the input gradient, the fused MaxPool
(pooled map + switches) and the fused MaxPoolGrad."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C, K)
FWD_CASES = [
    (4, 96, 312, 256, 256),     # conv3_2: 16 x 16 tiles, 468 blocks
    (4, 48, 156, 256, 512),     # conv4_1: two N tiles
    (9, 40, 96, 256, 256),      # 8 x 32 tiles
    (2, 37, 53, 128, 320),      # ragged tiles, N tail of 64
    (4, 24, 78, 512, 512),      # conv5_x: split-K slabs
]


def _bits(t):
    return t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16) else t


def _both(fn):
    """fn() under conv_halo4 with 4 waves (option halo4=1) and with 8 waves
    (halo4=2) -- checked equal to each other here -- and under conv_halo2
    (halo4=0); returns (conv_halo4 result, conv_halo2 result)."""
    outs = []
    try:
        for v in (1, 2, 0):
            ops.set_option("halo4", v)
            outs.append(fn())
    finally:
        ops.set_option("halo4", 2)      # the default
    torch.cuda.synchronize()
    a4, a8, b = outs
    flat = lambda r: r if isinstance(r, tuple) else (r,)   # noqa: E731
    for x, y in zip(flat(a4), flat(a8)):
        assert torch.equal(_bits(x) if x.dtype != torch.uint8 else x, _bits(y) if y.dtype != torch.uint8 else y)
    return a4, b


def _operands(dev, case, dtype, seed):
    N, H, W, C, K = case
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * C) ** 0.5
    bias = torch.randn(K, device=dev, generator=g) * 0.1
    scale = 1.0 + 0.1 * torch.randn(K, device=dev, generator=g)
    shift = 0.1 * torch.randn(K, device=dev, generator=g)
    other = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    return x, w32, bias, scale, shift, other


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", FWD_CASES, ids=["conv3_2", "conv4_1", "bw32", "ragged", "conv5"])
def test_halo4_forward_equals_halo2(dev, case, dtype):
    N, H, W, C, K = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=dt)
    name = ops.conv_kernel_info(d, ops.OP_FWD)[0]
    assert name.startswith("conv_halo4<"), name
    x, w32, bias, scale, shift, res = _operands(dev, case, dtype, 3)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    for epi in (ops.epilogue(bias=bias, relu=True), ops.epilogue(scale=scale, shift=shift, relu=True),
                ops.epilogue(bias=bias, residual=res), ops.epilogue(bias=bias, relu=True, keep_prob=0.8, seed=77)):
        def run():
            y = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
            ops.conv2d_fwd(d, x, wk, y, epi, ws)
            return y
        a, b = _both(run)
        assert torch.equal(_bits(a), _bits(b))
    if case == FWD_CASES[0] or case == FWD_CASES[3]:
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2),
                                         w32.to(dtype).float().permute(3, 2, 0, 1), padding=1)
        ref = torch.relu(ref + bias.view(1, -1, 1, 1)).permute(0, 2, 3, 1)
        y = torch.empty(N, H, W, K, dtype=dtype, device=dev)
        ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item()
        assert err <= 1.2e-2 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
@pytest.mark.parametrize("case", [(4, 96, 312, 256, 256), (4, 48, 156, 512, 512), (2, 37, 53, 320, 256),
                                  (4, 24, 78, 512, 512)], ids=["conv3_3", "conv4_2", "ragged", "conv5"])
def test_halo4_input_gradient_equals_halo2(dev, case, dtype):
    """dx = Conv2DBackpropInput(dy, W) * (y_prev > 0): N = the conv's input
    channels, the ReluGrad of the producing layer in the epilogue."""
    N, H, W, C, K = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=dt)
    name = ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0]
    assert name.startswith("conv_halo4<"), name
    g = torch.Generator(device=dev).manual_seed(11)
    dy = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * K) ** 0.5
    mask = torch.relu(torch.randn(N, H, W, C, device=dev, generator=g)).to(dtype)
    wh = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_HWIO, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, C, K, ops.PACK_HWIO)
    ws = ops.Workspace(dev)
    for epi in (None, ops.epilogue(relu_mask=mask, mask_scale=1.25)):
        def run():
            dx = torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
            ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, epi)
            return dx
        a, b = _both(run)
        assert torch.equal(_bits(a), _bits(b))


@pytest.mark.parametrize("case", [(4, 96, 312, 256, 256), (9, 40, 96, 256, 256), (4, 48, 156, 512, 512)],
                         ids=["conv3_3", "bw32", "conv4_3"])
def test_halo4_fused_pool_equals_halo2(dev, case):
    N, H, W, C, K = case
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    assert ops.conv2d_fwd_pool_ok(d)
    x, w32, bias, _, _, _ = _operands(dev, case, torch.bfloat16, 5)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC, C), dtype=torch.bfloat16, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    epi = ops.epilogue(bias=bias, relu=True)

    def run():
        out = torch.full((N, H // 2, W // 2, K), float("nan"), dtype=torch.bfloat16, device=dev)
        idx = torch.full((N * (H // 2) * (W // 2) * K,), 255, dtype=torch.uint8, device=dev)
        ops.conv2d_fwd_pool(d, x, wk, out, idx, epi, ws)
        return out, idx
    (a, ai), (b, bi) = _both(run)
    assert torch.equal(_bits(a), _bits(b))
    assert torch.equal(ai, bi)
    y = torch.empty(N, H, W, K, dtype=torch.bfloat16, device=dev)
    ops.conv2d_fwd(d, x, wk, y, epi, ws)
    ref = torch.empty_like(a)
    ref_idx = torch.empty_like(ai)
    ops.maxpool2x2_fwd_argmax(y, ref, ref_idx)
    torch.cuda.synchronize()
    assert torch.equal(_bits(a), _bits(ref))
    assert torch.equal(ai, ref_idx)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16], ids=["bf16", "f16"])
def test_halo4_fused_unpool_equals_halo2(dev, dtype):
    N, H, W, C, K = 2, 96, 312, 256, 256
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=dt)
    assert ops.conv2d_bwd_data_unpool_ok(d)
    g = torch.Generator(device=dev).manual_seed(17)
    xf = torch.relu(torch.randn(N, 2 * H, 2 * W, C, device=dev, generator=g)).to(dtype)
    pooled = torch.empty(N, H, W, C, dtype=dtype, device=dev)
    idx = torch.empty(N * H * W * C, dtype=torch.uint8, device=dev)
    ops.maxpool2x2_fwd_argmax(xf, pooled, idx)
    dy = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * K) ** 0.5
    wh = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_HWIO, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, C, K, ops.PACK_HWIO)
    base = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    ws = ops.Workspace(dev)

    def run():
        out = torch.full((N, 2 * H, 2 * W, C), float("nan"), dtype=dtype, device=dev)
        ops.conv2d_bwd_data_unpool(d, dy, wh, idx, out, relu_mask=True, residual=base, ws=ws)
        return out
    a, b = _both(run)
    assert torch.equal(_bits(a), _bits(b))


def test_halo4_forced_split_equals_halo2(dev):
    """A split-K plan forced on a shape that runs whole (halo_min_splits=4:
    conv4_1's 4 chunks one per slab), through the slab reducer."""
    case = (4, 48, 156, 256, 512)
    N, H, W, C, K = case
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x, w32, bias, _, _, _ = _operands(dev, case, torch.bfloat16, 23)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC, C), dtype=torch.bfloat16, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    ops.set_option("halo_min_splits", 4)
    try:
        assert ops.conv_kernel_info(d, ops.OP_FWD)[1] == 4

        def run():
            y = torch.full((N, H, W, K), float("nan"), dtype=torch.bfloat16, device=dev)
            ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
            return y
        a, b = _both(run)
    finally:
        ops.set_option("halo_min_splits", 1)
    assert torch.equal(_bits(a), _bits(b))
