"""conv_halo2s (option halo2_1p: conv_halo2's 256 x 256 tiles with one MFMA
phase per (chunk, tap) iteration and wave group, two barriers per iteration
instead of four) against conv_halo2.  Both run the same MFMAs on the same
fragments in the same per-accumulator order and share the epilogue, so every
output is compared bit for bit; conv_halo2 itself is pinned to the oracle by
the op-level and full-size parity tests (tests/test_gpu_ops.py,
tests/test_gpu_fullsize.py).

Shapes: FCN's conv3_x / conv4_x / conv5_x (Network/model/FCN.py:60-75) at
the bench's batch 4 (384 x 1248 input) and at batch 1 / 2, ragged tiles on both edges, 16- and 32-px tile rows (the
planner's choice by width), one 64-channel chunk (9 iterations) up to eight,
and split-K slabs (forced with halo_min_splits).  Epilogues: bias + ReLU,
residual add, dropout, the fused MaxPool with switches, and the ReluGrad
mask of the input gradient."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C, K)
SHAPES = [(4, 96, 312, 256, 256), (4, 48, 156, 256, 512), (4, 48, 156, 512, 512), (4, 24, 78, 512, 512),
          (1, 24, 78, 512, 512), (2, 40, 88, 256, 256), (1, 20, 36, 64, 256), (1, 17, 45, 128, 384)]


def _bits(t):
    return t.view(torch.int16) if t.dtype in (torch.bfloat16, torch.float16) else t


def _both(fn):
    ops.set_option("halo2_1p", 1)
    try:
        a = fn()
    finally:
        ops.set_option("halo2_1p", 0)
    b = fn()
    torch.cuda.synchronize()
    return a, b


def _operands(dev, N, H, W, C, K, dtype, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (3.0 * C ** 0.5)
    bias = torch.randn(K, device=dev, generator=g) * 0.1
    other = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    return x, w32, bias, other


def _dt(dtype):
    return ops.BF16 if dtype == torch.bfloat16 else ops.F16


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", SHAPES)
def test_halo2s_forward_epilogues(dev, shape, dtype):
    N, H, W, C, K = shape
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=_dt(dtype))
    name = ops.conv_kernel_info(d, ops.OP_FWD)[0]
    if not name.endswith(",256,256>"):
        assert shape not in SHAPES[:4], name      # FCN's conv3_x .. conv5_x shapes run on it
        pytest.skip(f"planner chose {name}")
    x, w32, bias, res = _operands(dev, N, H, W, C, K, dtype, 3)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    for epi in (ops.epilogue(bias=bias, relu=True), ops.epilogue(bias=bias, relu=True, residual=res),
                ops.epilogue(bias=bias, relu=True, keep_prob=0.8, seed=77)):
        def run():
            y = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
            ops.conv2d_fwd(d, x, wk, y, epi, ws)
            return y
        a, b = _both(run)
        assert torch.equal(_bits(a), _bits(b))
    # sanity of both against torch's fp32 conv on the same rounded operands
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w32.to(dtype).float().permute(3, 2, 0, 1),
                                     padding=1)
    ref = torch.relu(ref + bias.view(1, -1, 1, 1)).permute(0, 2, 3, 1)
    ops.set_option("halo2_1p", 1)
    try:
        y = torch.empty(N, H, W, K, dtype=dtype, device=dev)
        ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
        torch.cuda.synchronize()
    finally:
        ops.set_option("halo2_1p", 0)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1.2e-2 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] % 2 == 0 and s[2] % 2 == 0])
def test_halo2s_fused_pool(dev, shape):
    N, H, W, C, K = shape
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    if not ops.conv2d_fwd_pool_ok(d):
        pytest.skip("split-K plan: no pooled epilogue")
    x, w32, bias, _ = _operands(dev, N, H, W, C, K, torch.bfloat16, 5)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC), dtype=torch.bfloat16, device=dev)
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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", SHAPES)
def test_halo2s_input_gradient_relu_mask(dev, shape, dtype):
    """Conv2DBackpropInput (the transposed filter, K -> C; conv_halo2 when C >
    128) with the ReluGrad mask of the layer below."""
    N, H, W, C, K = shape
    if C <= 128:
        pytest.skip("input gradient with <= 128 channels runs on conv_halo_duo")
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=_dt(dtype))
    name = ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0]
    if not name.endswith(",256,256>"):
        pytest.skip(f"planner chose {name}")
    g = torch.Generator(device=dev).manual_seed(9)
    dy = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (3.0 * K ** 0.5)
    mask = torch.relu(torch.randn(N, H, W, C, device=dev, generator=g)).to(dtype)
    wh = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_HWIO), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, C, K, ops.PACK_HWIO)
    ws = ops.Workspace(dev)

    def run():
        dx = torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
        ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, ops.epilogue(relu_mask=mask, mask_scale=1.25))
        return dx
    a, b = _both(run)
    assert torch.equal(_bits(a), _bits(b))


@pytest.mark.parametrize("splits", [2, 3])
def test_halo2s_split_k_slabs(dev, splits):
    """Split-K over channel chunks (fp32 slabs + the NT reducer): each split's
    iterations start at its own chunk."""
    N, H, W, C, K = 1, 24, 78, 512, 512
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    x, w32, bias, _ = _operands(dev, N, H, W, C, K, torch.bfloat16, 11)
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC), dtype=torch.bfloat16, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    ws = ops.Workspace(dev)
    ops.set_option("halo_min_splits", splits)
    try:
        assert ops.conv_kernel_info(d, ops.OP_FWD)[1] >= splits

        def run():
            y = torch.full((N, H, W, K), float("nan"), dtype=torch.bfloat16, device=dev)
            ops.conv2d_fwd(d, x, wk, y, ops.epilogue(bias=bias, relu=True), ws)
            return y
        a, b = _both(run)
    finally:
        ops.set_option("halo_min_splits", 1)
    assert torch.equal(_bits(a), _bits(b))
