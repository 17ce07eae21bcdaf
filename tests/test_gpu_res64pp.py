"""conv_res64pp (the two-group ping-pong form of conv_res64: conv1_2 fwd +
pool1 and its input gradient, Network/model/FCN.py:55-57) against the
single-pipeline conv_res64 it replaces.  Both run the same 18 MFMA k-steps in
the same order on the same fragments and the same epilogue arithmetic, so
every output is compared bit for bit; the legacy kernel itself is pinned to
the oracle by the op-level and full-size parity tests.

Shapes vary the tiles per block (grid = min(tiles, CUs)): one tile (group 1
idle all launch), fewer tiles than CUs, and 2-4 tiles per block with odd and
even counts, with ragged 8 x 32 tiles at the bottom / right edges.  Epilogues:
bias + ReLU, the fused MaxPool with switches, the ReluGrad mask of the input
gradient (mask_scale), a residual add, and dropout."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

SHAPES = [(1, 8, 32), (1, 22, 70), (4, 96, 320), (3, 196, 300), (8, 120, 500)]


def _operands(dev, N, H, W, dtype, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(N, H, W, 64, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, 64, 64, device=dev, generator=g) / 24.0
    bias = torch.randn(64, device=dev, generator=g) * 0.1
    other = torch.randn(N, H, W, 64, device=dev, generator=g).to(dtype)
    return x, w32, bias, other


def _both(fn):
    """fn() under the ping-pong kernel (forced for every epilogue) and under
    the legacy one."""
    ops.set_option("res64_pp", 2)
    a = fn()
    ops.set_option("res64_pp", 0)
    try:
        b = fn()
    finally:
        ops.set_option("res64_pp", 1)
    torch.cuda.synchronize()
    return a, b


def _bits(t):
    return t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16) else t


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", SHAPES)
def test_res64pp_forward_epilogues(dev, shape, dtype):
    N, H, W = shape
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, 64, 64, 3, 3, dtype=dt)
    assert ops.conv_kernel_info(d, ops.OP_FWD)[0].startswith("conv_res64")
    x, w32, bias, res = _operands(dev, N, H, W, dtype, 3)
    wk = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_KRSC, 64), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, 64, 64, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    for epi in (ops.epilogue(bias=bias, relu=True), ops.epilogue(bias=bias, relu=True, residual=res),
                ops.epilogue(bias=bias, relu=True, keep_prob=0.8, seed=77)):
        def run():
            y = torch.full((N, H, W, 64), float("nan"), dtype=dtype, device=dev)
            ops.conv2d_fwd(d, x, wk, y, epi, ws)
            return y
        a, b = _both(run)
        assert torch.equal(_bits(a), _bits(b))
    # against torch's fp32 conv on the same rounded operands (sanity of both)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2),
                                     w32.to(dtype).float().permute(3, 2, 0, 1), padding=1)
    ref = torch.relu(ref + bias.view(1, -1, 1, 1)).permute(0, 2, 3, 1)
    y = torch.empty(N, H, W, 64, dtype=dtype, device=dev)
    ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1.2e-2 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] % 2 == 0 and s[2] % 2 == 0])
def test_res64pp_fused_pool(dev, shape):
    N, H, W = shape
    d = ops.conv_desc(N, H, W, 64, 64, 3, 3, dtype=ops.BF16)
    assert ops.conv2d_fwd_pool_ok(d)
    x, w32, bias, _ = _operands(dev, N, H, W, torch.bfloat16, 5)
    wk = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_KRSC, 64), dtype=torch.bfloat16, device=dev)
    ops.pack_filter(w32, wk, 64, 64, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    epi = ops.epilogue(bias=bias, relu=True)

    def run():
        out = torch.full((N, H // 2, W // 2, 64), float("nan"), dtype=torch.bfloat16, device=dev)
        idx = torch.full((N * (H // 2) * (W // 2) * 64,), 255, dtype=torch.uint8, device=dev)
        ops.conv2d_fwd_pool(d, x, wk, out, idx, epi, ws)
        return out, idx
    (a, ai), (b, bi) = _both(run)
    assert torch.equal(_bits(a), _bits(b))
    assert torch.equal(ai, bi)
    # and the pair the fusion replaces
    y = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    ops.conv2d_fwd(d, x, wk, y, epi, ws)
    ref = torch.empty_like(a)
    ref_idx = torch.empty_like(ai)
    ops.maxpool2x2_fwd_argmax(y, ref, ref_idx)
    torch.cuda.synchronize()
    assert torch.equal(_bits(a), _bits(ref))
    assert torch.equal(ai, ref_idx)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", SHAPES)
def test_res64pp_input_gradient_relu_mask(dev, shape, dtype):
    """dx = conv2d_backprop_input(dy, W) * (x > 0): the ReluGrad mask epilogue
    (bits taken after the MFMAs, applied in the next phase)."""
    N, H, W = shape
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, 64, 64, 3, 3, dtype=dt)
    assert ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0].startswith("conv_res64")
    dy, w32, _, xin = _operands(dev, N, H, W, dtype, 9)
    mask = torch.relu(xin)                       # ~half zeros
    wh = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_HWIO, 64), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, 64, 64, ops.PACK_HWIO)
    ws = ops.Workspace(dev)

    def run():
        dx = torch.full((N, H, W, 64), float("nan"), dtype=dtype, device=dev)
        ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, ops.epilogue(relu_mask=mask))
        return dx
    a, b = _both(run)
    assert torch.equal(_bits(a), _bits(b))
    zero = (mask == 0)
    assert bool((a[zero] == 0).all()) and 0.3 < zero.float().mean().item() < 0.7


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("K", [16, 8])
def test_res16_dma_halo_equals_register_halo(dev, shape, dtype, K):
    """The 16-wide conv_res64 (FC-DenseNet's growth conv, 64 -> 16 channels,
    Network/model/FCDenseNet.py:33-34) with its halo landed by LDS DMA (two
    blocks per CU) against the VGPR-staged form: same fragments, same MFMA
    order, same epilogue -> bit-equal, for the forward epilogues and the
    ReluGrad-masked input gradient (64 -> 16 of the transposed filter)."""
    N, H, W = shape
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, 64, K, 3, 3, dtype=dt)
    assert ops.conv_kernel_info(d, ops.OP_FWD)[0].startswith("conv_res64")
    x, w32, bias, other = _operands(dev, N, H, W, dtype, 13)
    w32, bias = w32[..., :K].contiguous(), bias[:K].contiguous()
    res = other[..., :K].contiguous()
    wk = torch.zeros(ops.packed_shape(3, 3, 64, K, ops.PACK_KRSC, 64), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, 64, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)

    def both(fn):
        a = fn()
        ops.set_option("res16_dma", 0)
        try:
            b = fn()
        finally:
            ops.set_option("res16_dma", 1)
        torch.cuda.synchronize()
        return a, b
    for epi in (ops.epilogue(bias=bias, relu=True), ops.epilogue(residual=res),
                ops.epilogue(bias=bias, keep_prob=0.8, seed=5)):
        def run():
            y = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
            ops.conv2d_fwd(d, x, wk, y, epi, ws)
            return y
        a, b = both(run)
        assert torch.equal(_bits(a), _bits(b))
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2),
                                     w32.to(dtype).float().permute(3, 2, 0, 1), padding=1)
    ref = torch.relu(ref + bias.view(1, -1, 1, 1)).permute(0, 2, 3, 1)
    y = torch.empty(N, H, W, K, dtype=dtype, device=dev)
    ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    assert err <= 1.2e-2 * ref.abs().max().item() + 1e-3, err
