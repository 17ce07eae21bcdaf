"""Conv2D + bias + ReLU + MaxPool 2x2/2 in one launch (seg_conv2d_fwd_pool:
conv_layer -> max_pool, Network/model/FCN.py:56-57, :158-160) against the
unfused pair the oracle-tested path runs (seg_conv2d_fwd, then
seg_maxpool2x2_fwd_argmax): the pooled map and the switches must be equal bit
for bit -- the fused epilogue rounds every value to the 16-bit type before
comparing, exactly as the pool kernel sees the stored conv output.

Shapes pick each kernel with the pooled epilogue (the launch chooser decides;
the test asserts the family): conv_res64 (C = K = 64, ragged 8 x 32 tiles),
conv_halo_duo (N = 128, 16-px tile rows, incl. an N tail), conv_halo2
(N = 256, BW = 16 and BW = 32 tiles), each without split-K."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C, K, kernel family)
CASES = [
    (2, 40, 70, 64, 64, "conv_res64"),
    (1, 22, 70, 64, 64, "conv_res64"),           # last tile row half outside the image
    (4, 96, 128, 128, 128, "conv_halo<"),        # conv_halo_duo 256 x 128 tiles
    (4, 96, 128, 128, 120, "conv_halo<"),        # N tail (padded columns stay 0)
    (2, 96, 312, 256, 256, "conv_halo4<"),       # conv_halo4, 16 x 16 tiles
    (9, 40, 96, 256, 256, "conv_halo4<"),        # conv_halo4, 8 x 32 tiles
]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_conv_pool_fused_equals_unfused(dev, case, dtype):
    N, H, W, C, K, fam = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=dt)
    assert ops.conv2d_fwd_pool_ok(d), case
    name, splits, _ = ops.conv_kernel_info(d, ops.OP_FWD)
    assert name.startswith(fam) and splits == 1, (name, splits)
    g = torch.Generator(device=dev).manual_seed(11)
    Kp = ops.round8(K)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * C) ** 0.5
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, C, Kp, ops.PACK_KRSC)
    bias = torch.randn(K, device=dev, generator=g) * 0.1
    epi = ops.epilogue(bias=bias, relu=True)
    ws = ops.Workspace(dev)
    # unfused: conv output, then the switch-recording pool
    y = torch.full((N, H, W, Kp), float("nan"), dtype=dtype, device=dev)
    ops.conv2d_fwd(d, x, wk, y, epi, ws)
    ref = torch.empty(N, H // 2, W // 2, Kp, dtype=dtype, device=dev)
    ref_idx = torch.empty(N * (H // 2) * (W // 2) * Kp, dtype=torch.uint8, device=dev)
    ops.maxpool2x2_fwd_argmax(y, ref, ref_idx)
    # fused
    out = torch.full_like(ref, float("nan"))
    idx = torch.full_like(ref_idx, 255)
    ops.conv2d_fwd_pool(d, x, wk, out, idx, epi, ws)
    out2 = torch.full_like(ref, float("nan"))
    ops.conv2d_fwd_pool(d, x, wk, out2, None, epi, ws)       # switches optional
    torch.cuda.synchronize()
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    assert torch.equal(out2.view(torch.int16), ref.view(torch.int16))
    assert torch.equal(idx, ref_idx)
    # the max > 0 bit is set somewhere and clear somewhere (ReLU zeros present)
    b = (idx >> 2) & 1
    assert 0 < b.float().mean().item() < 1


def test_conv_pool_rejects_unsupported(dev):
    """Odd output sizes, dropout / residual epilogues and split-K convs return
    SEG_EINVAL (the Session then runs the unfused pair)."""
    d = ops.conv_desc(4, 24, 78, 512, 512, 3, 3, dtype=ops.BF16)        # conv5_x: 3-way split-K
    assert not ops.conv2d_fwd_pool_ok(d)
    x = torch.zeros(4, 24, 78, 512, dtype=torch.bfloat16, device=dev)
    wk = torch.zeros(ops.packed_shape(3, 3, 512, 512, ops.PACK_KRSC, 512), dtype=torch.bfloat16, device=dev)
    out = torch.empty(4, 12, 39, 512, dtype=torch.bfloat16, device=dev)
    with pytest.raises(Exception):
        ops.conv2d_fwd_pool(d, x, wk, out, None, ops.epilogue(relu=True))
    d2 = ops.conv_desc(2, 40, 70, 64, 64, 3, 3, dtype=ops.BF16)
    x2 = torch.zeros(2, 40, 70, 64, dtype=torch.bfloat16, device=dev)
    w2 = torch.zeros(ops.packed_shape(3, 3, 64, 64, ops.PACK_KRSC, 64), dtype=torch.bfloat16, device=dev)
    out2 = torch.empty(2, 20, 35, 64, dtype=torch.bfloat16, device=dev)
    with pytest.raises(Exception):
        ops.conv2d_fwd_pool(d2, x2, w2, out2, None, ops.epilogue(relu=True, keep_prob=0.5))


@pytest.mark.parametrize("case", [(2, 96, 312, 256, 256), (4, 96, 128, 128, 128)],
                         ids=["conv_halo2", "conv_halo_duo"])
def test_forced_split_plan_refuses_pool_and_stays_exact(dev, case):
    """VERDICT r03 (the halo_cus hang): force a split-K halo plan on a conv the
    default plan pools.  The pooled launch is refused on the host (SEG_EINVAL,
    no kernel runs); the same conv unpooled on the split plan (conv_halo +
    splitk_reduce_nt) equals the default single-pass kernel's output within
    bf16 rounding of the fp32 slab sums."""
    N, H, W, C, K = case
    d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
    assert ops.conv2d_fwd_pool_ok(d)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
    w32 = torch.randn(3, 3, C, K, device=dev, generator=g) / (9 * C) ** 0.5
    wk = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_KRSC, C), dtype=torch.bfloat16, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    epi = ops.epilogue(bias=torch.randn(K, device=dev, generator=g) * 0.1, relu=True)
    ws = ops.Workspace(dev)
    ref = torch.empty(N, H, W, K, dtype=torch.bfloat16, device=dev)
    ops.conv2d_fwd(d, x, wk, ref, epi, ws)
    ops.set_option("halo_min_splits", 2)
    try:
        assert ops.conv_kernel_info(d, ops.OP_FWD)[1] >= 2
        assert not ops.conv2d_fwd_pool_ok(d)
        pooled = torch.full((N, H // 2, W // 2, K), 7.0, dtype=torch.bfloat16, device=dev)
        with pytest.raises(RuntimeError):
            ops.conv2d_fwd_pool(d, x, wk, pooled, None, epi, ws)
        torch.cuda.synchronize()
        assert bool((pooled == 7.0).all())          # nothing was written
        y = torch.full_like(ref, float("nan"))
        ops.conv2d_fwd(d, x, wk, y, epi, ws)
        torch.cuda.synchronize()
    finally:
        ops.set_option("halo_min_splits", 1)
    err = (y.float() - ref.float()).abs().max().item()
    assert err <= 1e-2 * ref.float().abs().max().item(), err
