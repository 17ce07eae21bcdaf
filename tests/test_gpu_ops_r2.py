"""Op-level parity of the round-2 C-ABI entry points against plain torch
fp32 references: seg_spatial_reduce / seg_spatial_broadcast (global average
pooling and the 1x1 -> HxW align_corners resize of DeepLab's image-pooling
branch, Network/model/DeepLabv3Plus.py:215-225) and seg_axpy (the
accumulate template's assign_add, Network/main.py:92-95).
Tolerances: fp32 sums 1e-5 relative; bf16 outputs one bf16 rounding (4e-3)."""
import numpy as np
import pytest
import torch

from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 7, 9, 8), (1, 128, 256, 512), (3, 1, 1, 24), (2, 33, 5, 2048)])
def test_spatial_reduce_mean_and_sum(dev, dtype, shape):
    if dtype == torch.float32 and shape[3] > 1024:
        pytest.skip("fp32 chunks: C <= 1024")
    N, H, W, C = shape
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    y = torch.empty(N, 1, 1, C, device=dev, dtype=dtype)
    ws = ops.Workspace(dev)
    for scale in (1.0 / (H * W), 1.0):
        ops.spatial_reduce(x, y, scale, ws)
        ref = x.float().sum(dim=(1, 2), keepdim=True) * scale
        tol = 1e-5 if dtype == torch.float32 else 4e-3
        err = (y.float() - ref).abs().max().item()
        assert err <= tol * ref.abs().max().item() + 1e-6, err
    # the oracle's align_corners resize from 1x1 is a broadcast; its gradient a spatial sum
    xo = torch.randn(N, 1, 1, C, dtype=torch.float64, requires_grad=True)
    yo = T.resize_bilinear(xo, (H, W))
    assert torch.equal(yo, xo.expand(N, H, W, C))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_spatial_broadcast(dev, dtype):
    N, H, W, C = 2, 17, 30, 256
    x = torch.randn(N, 1, 1, C, device=dev).to(dtype)
    full = torch.zeros(N, H, W, C + 16, device=dev, dtype=dtype)
    y = full[..., :C]                                  # strided destination (pixel stride C + 16)
    ops.spatial_broadcast(x, y, 0.25)
    ref = (x.float() * 0.25).expand(N, H, W, C)
    assert (y.float() - ref).abs().max().item() <= 4e-3 * ref.abs().max().item()
    assert full[..., C:].abs().max().item() == 0.0


def test_axpy(dev):
    n = 1_000_003
    y = torch.randn(n, device=dev)
    x = torch.randn(n, device=dev)
    ref = y + 1.5 * x
    ops.axpy(y, x, 1.5)
    np.testing.assert_allclose(y.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6, atol=1e-6)
