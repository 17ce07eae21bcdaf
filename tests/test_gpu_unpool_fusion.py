"""Conv2DBackpropInput + MaxPoolGrad in one launch (seg_conv2d_bwd_data_unpool:
the backward of max_pool -> conv_layer, Network/model/FCN.py:57-63 / :63-69
with :158-160) against the unfused pair the oracle-tested path runs
(seg_conv2d_bwd_data, then seg_maxpool2x2_bwd_argmax): the full-resolution
gradient must be equal bit for bit -- the fused epilogue rounds each pooled
value to the 16-bit type before routing it, as the stored pooled gradient is.

Shapes pick each kernel with the MaxPoolGrad epilogue (the launch chooser
decides; the test asserts the family): conv_halo_duo (N = 64 and N = 128, C2's
conv2_1 / conv3_1 input gradients) and conv_halo2 (N = 256, 16-px rows), each
without split-K; with the ReluGrad of the post-ReLU pool input on and off, and
with a residual (the pooled gradient of the pool's other consumers: FCN's
score_pool3 / score_pool4 skip branches)."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C = the dgrad's output channels, K) at the pooled resolution
CASES = [
    (4, 192, 624, 64, 128),    # conv_halo_duo<16, 6, 64>: C2 conv2_1 after pool1
    (4, 96, 312, 128, 256),    # conv_halo_duo<16, 6, 128>: C2 conv3_1 after pool2
    (2, 96, 312, 256, 256),    # conv_halo2<16>
]


def _setup(dev, case, dtype, seed):
    N, H, W, C, K = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=dt)
    g = torch.Generator(device=dev).manual_seed(seed)
    # the pool's switches from a post-ReLU full-resolution map (ties and zeros present)
    xf = torch.relu(torch.randn(N, 2 * H, 2 * W, C, device=dev, generator=g)).to(dtype)
    xf[:, ::7] = 0
    pooled = torch.empty(N, H, W, C, dtype=dtype, device=dev)
    idx = torch.empty(N * H * W * C, dtype=torch.uint8, device=dev)
    ops.maxpool2x2_fwd_argmax(xf, pooled, idx)
    dy = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * K) ** 0.5
    wh = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_HWIO, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, C, K, ops.PACK_HWIO)
    base = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    return d, idx, dy, wh, base


@pytest.mark.parametrize("residual", [False, True], ids=["plain", "residual"])
@pytest.mark.parametrize("relu", [True, False], ids=["relu", "norelu"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES, ids=["duo64", "duo128", "halo2"])
def test_dgrad_unpool_fused_equals_unfused(dev, case, dtype, relu, residual):
    N, H, W, C, K = case
    d, idx, dy, wh, base = _setup(dev, case, dtype, 17)
    assert ops.conv2d_bwd_data_unpool_ok(d), case
    name, splits, _ = ops.conv_kernel_info(d, ops.OP_BWD_DATA)
    assert name.startswith("conv_halo") and splits == 1, (name, splits)
    ws = ops.Workspace(dev)
    # unfused: the pooled input gradient (+ the other consumers' sum in place), then MaxPoolGrad
    dxp = base.clone() if residual else torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
    ops.conv2d_bwd_data(d, dy, wh, dxp, ws, epi=ops.epilogue(residual=dxp) if residual else None)
    ref = torch.full((N, 2 * H, 2 * W, C), float("nan"), dtype=dtype, device=dev)
    ops.maxpool2x2_bwd_argmax(idx, dxp, ref, relu_mask=relu)
    # fused
    out = torch.full_like(ref, float("nan"))
    ops.conv2d_bwd_data_unpool(d, dy, wh, idx, out, relu_mask=relu, residual=base if residual else None, ws=ws)
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    assert (out != 0).float().mean().item() < 0.26          # one window element in four at most


def test_dgrad_unpool_rejects_split_plans(dev):
    """A split-K plan (conv5_x's input gradient: 3-way slabs) has no
    MaxPoolGrad epilogue: the fused launch is refused on the host (SEG_EINVAL,
    nothing written) and the Session keeps the unfused pair."""
    d = ops.conv_desc(4, 12, 39, 512, 512, 3, 3, dtype=ops.BF16)
    assert ops.conv_kernel_info(d, ops.OP_BWD_DATA)[1] > 1
    assert not ops.conv2d_bwd_data_unpool_ok(d)
    dy = torch.zeros(4, 12, 39, 512, dtype=torch.bfloat16, device=dev)
    wh = torch.zeros(ops.packed_shape(3, 3, 512, 512, ops.PACK_HWIO, 512), dtype=torch.bfloat16, device=dev)
    idx = torch.zeros(4 * 12 * 39 * 512, dtype=torch.uint8, device=dev)
    out = torch.full((4, 24, 78, 512), 7.0, dtype=torch.bfloat16, device=dev)
    with pytest.raises(RuntimeError):
        ops.conv2d_bwd_data_unpool(d, dy, wh, idx, out, relu_mask=True)
    torch.cuda.synchronize()
    assert bool((out == 7.0).all())
