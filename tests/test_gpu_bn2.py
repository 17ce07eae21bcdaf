"""seg_conv2d_fwd_bn2: a conv whose output also feeds a frozen BatchNorm +
ReLU writes both maps in one launch (FC-DenseNet's bottleneck conv1 ->
dropout -> BN -> ReLU, Network/model/FCDenseNet.py:28-31).  Against the pair
the oracle-tested path runs (conv2d_fwd[_pro], then bn_relu_fwd on the stored
output): the conv output and the BN(+ReLU) map must be equal bit for bit, on
each kernel that carries the second output -- conv1x1_stream (BN prologue,
C <= 256), igemm_nt2 with the BN prologue (C > 256) and plain igemm_nt2
(an unfolded conv, channel count not a multiple of 8)."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C, K, with BN1 prologue, kernel family, keep_prob)
CASES = [
    (2, 96, 312, 96, 64, True, "conv1x1_stream", 0.2),
    (1, 48, 156, 320, 64, True, "igemm_nt2_pro", 0.2),
    (2, 24, 78, 174, 64, False, "igemm_nt2", 0.2),
    (2, 96, 312, 96, 64, True, "conv1x1_stream", 1.0),
]


@pytest.mark.parametrize("st", [0, 2], ids=["st8", "st16"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
def test_conv_bn2_equals_conv_then_bn_relu(dev, case, dtype, st):
    N, H, W, C, K, with_pro, fam, kp = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 1, 1, dtype=dt)
    assert ops.conv2d_fwd_bn2_ok(d, with_pro), case
    name = ops.conv_kernel_info(d, ops.OP_FWD_PRO if with_pro else ops.OP_FWD)[0]
    assert name.startswith(fam), (name, fam)
    g = torch.Generator(device=dev).manual_seed(21)
    Cp = ops.round8(C)
    x = torch.zeros(N, H, W, Cp, dtype=dtype, device=dev)
    x[..., :C] = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    w32 = torch.randn(1, 1, C, K, device=dev, generator=g) / C ** 0.5
    wk = torch.zeros(ops.packed_shape(1, 1, C, K, ops.PACK_KRSC, Cp), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, Cp, K, ops.PACK_KRSC)
    g1 = 1.0 + 0.1 * torch.randn(C, device=dev, generator=g)
    b1 = 0.1 * torch.randn(C, device=dev, generator=g)
    g2 = 1.0 + 0.1 * torch.randn(K, device=dev, generator=g)
    b2 = 0.1 * torch.randn(K, device=dev, generator=g)
    pro = ops.prologue(g1, b1) if with_pro else None
    epi = ops.epilogue(keep_prob=kp, seed=99)
    ws = ops.Workspace(dev)
    ops.set_option("s1x1_st", st)       # conv1x1_stream's staged 16-byte stores (both launches)
    # the pair
    y_ref = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
    if with_pro:
        ops.conv2d_fwd_pro(d, x, pro, wk, y_ref, epi, ws)
    else:
        ops.conv2d_fwd(d, x, wk, y_ref, epi, ws)
    a_ref = torch.full_like(y_ref, float("nan"))
    ops.bn_relu_fwd(y_ref, a_ref, g2, b2, K, True)
    # one launch
    y = torch.full_like(y_ref, float("nan"))
    a = torch.full_like(y_ref, float("nan"))
    ops.conv2d_fwd_bn2(d, x, pro, wk, y, a, g2, b2, True, 1e-3, epi, ws)
    torch.cuda.synchronize()
    ops.set_option("s1x1_st", 1)
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
    assert torch.equal(a.view(torch.int16), a_ref.view(torch.int16))
    zero = (a == 0).float().mean().item()
    assert 0.2 < zero < 0.95, zero            # the ReLU (and the dropout) bite


def test_conv_bn2_refused_on_split_k(dev):
    """A plan without the second output (here: a 3x3 conv on the halo kernel)
    is refused on the host -- SEG_EINVAL, nothing launched."""
    d = ops.conv_desc(2, 48, 156, 256, 256, 3, 3, dtype=ops.BF16)
    assert not ops.conv2d_fwd_bn2_ok(d, False)
    x = torch.zeros(2, 48, 156, 256, dtype=torch.bfloat16, device=dev)
    wk = torch.zeros(ops.packed_shape(3, 3, 256, 256, ops.PACK_KRSC, 256), dtype=torch.bfloat16, device=dev)
    y = torch.full((2, 48, 156, 256), 7.0, dtype=torch.bfloat16, device=dev)
    a = torch.full_like(y, 7.0)
    one = torch.ones(256, device=dev)
    with pytest.raises(RuntimeError):
        ops.conv2d_fwd_bn2(d, x, None, wk, y, a, one, one)
    torch.cuda.synchronize()
    assert bool((y == 7.0).all()) and bool((a == 7.0).all())


# igemm_nt3 with split-K carries the second output too, written by its
# splitk_reduce_nt: DeepLab's ASPP convs -> BN -> ReLU (Network/utils/utils.py
# :186-229) on the 1/8-resolution map of a 384x1248 input (48x156, where the
# plan splits K) -- the rate-6 / rate-18 3x3 convs and the 1280 -> 256
# concat_projection
# concat_projection.  Round 6: unsplit igemm_nt3 writes it in its own
# epilogue -- the same convs on the 128 x 256 map of C5's 1024 x 2048 input
# (the ASPP 1x1 branch too), where the five separate bn_relu_fwd passes ran.
NT3_CASES = [(2, 48, 156, 512, 256, 3, 6), (2, 48, 156, 512, 256, 3, 18), (2, 48, 156, 1280, 256, 1, 1),
             (2, 128, 256, 512, 256, 3, 6), (2, 128, 256, 512, 256, 3, 18), (2, 128, 256, 1280, 256, 1, 1),
             (2, 128, 256, 512, 256, 1, 1)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", NT3_CASES, ids=["aspp1_rate6", "aspp3_rate18", "projection_1x1", "c5_aspp1_rate6",
                                                 "c5_aspp3_rate18", "c5_projection_1x1", "c5_aspp0_1x1"])
def test_nt3_bn2_equals_conv_then_bn_relu(dev, case, dtype):
    N, H, W, C, K, R, dil = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, R, R, dilation=dil, dtype=dt)
    name, splits, _ = ops.conv_kernel_info(d, ops.OP_FWD)
    assert name.startswith("igemm_nt3") and (splits > 1) == (H == 48), (name, splits)
    assert ops.conv2d_fwd_bn2_ok(d, False)
    g = torch.Generator(device=dev).manual_seed(23)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    w32 = torch.randn(R, R, C, K, device=dev, generator=g) / (R * R * C) ** 0.5
    wk = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_KRSC, C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wk, C, K, ops.PACK_KRSC)
    g2 = 1.0 + 0.1 * torch.randn(K, device=dev, generator=g)
    b2 = 0.1 * torch.randn(K, device=dev, generator=g)
    bias = 0.1 * torch.randn(K, device=dev, generator=g)
    epi = ops.epilogue(bias=bias)
    ws = ops.Workspace(dev)
    y_ref = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
    ops.conv2d_fwd(d, x, wk, y_ref, epi, ws)
    a_ref = torch.full_like(y_ref, float("nan"))
    ops.bn_relu_fwd(y_ref, a_ref, g2, b2, K, True)
    y = torch.full_like(y_ref, float("nan"))
    a = torch.full_like(y_ref, float("nan"))
    ops.conv2d_fwd_bn2(d, x, None, wk, y, a, g2, b2, True, 1e-3, epi, ws)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
    assert torch.equal(a.view(torch.int16), a_ref.view(torch.int16))
    zero = (a == 0).float().mean().item()
    assert 0.2 < zero < 0.8, zero
