"""smallk_nt: single-tap NT problems with a reduction of K <= 16 -- the input
gradient of FC-DenseNet's final_conv (256 -> 2 classes, Network/model/
FCDenseNet.py:160) -- as a streaming kernel, against torch's fp32 conv on the
same rounded operands and against the tile kernel it replaces (option
smallk=0).  The k-sum runs in fp32 in k order, so the two kernels agree to
fp32 rounding before the 16-bit store (at most one unit in the last place)."""
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu

# (N, H, W, C = dgrad output channels, K = classes)
CASES = [(2, 96, 312, 256, 2), (1, 40, 70, 64, 2), (3, 24, 78, 128, 16)]


def _ulp_close(a, b):
    d = (a.view(torch.int16).int() - b.view(torch.int16).int()).abs()
    return int(d.max())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("epi_kind", ["plain", "mask", "residual"])
def test_smallk_input_gradient(dev, case, dtype, epi_kind):
    N, H, W, C, K = case
    dt = ops.BF16 if dtype == torch.bfloat16 else ops.F16
    d = ops.conv_desc(N, H, W, C, K, 1, 1, dtype=dt)
    assert ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0].startswith("smallk_nt")
    g = torch.Generator(device=dev).manual_seed(3)
    Kp = ops.round8(K)
    dy = torch.zeros(N, H, W, Kp, dtype=dtype, device=dev)
    dy[..., :K] = torch.randn(N, H, W, K, device=dev, generator=g).to(dtype)
    w32 = torch.randn(1, 1, C, K, device=dev, generator=g) / C ** 0.5
    wh = torch.zeros(ops.packed_shape(1, 1, C, K, ops.PACK_HWIO, d.C), dtype=dtype, device=dev)
    ops.pack_filter(w32, wh, d.C, d.K, ops.PACK_HWIO)
    other = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    epi = {"plain": None, "mask": ops.epilogue(relu_mask=torch.relu(other)),
           "residual": ops.epilogue(residual=other)}[epi_kind]
    ws = ops.Workspace(dev)

    def run():
        dx = torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
        ops.conv2d_bwd_data(d, dy, wh, dx, ws, None, epi)
        return dx
    a = run()
    ops.set_option("smallk", 0)
    try:
        assert not ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0].startswith("smallk_nt")
        b = run()
    finally:
        ops.set_option("smallk", 1)
    torch.cuda.synchronize()
    assert _ulp_close(a, b) <= 1
    ref = dy[..., :K].float() @ w32.to(dtype).float().view(C, K).t()
    if epi_kind == "mask":
        ref = ref * (other.float() > 0)
    elif epi_kind == "residual":
        ref = ref + other.float()
    err = (a.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
