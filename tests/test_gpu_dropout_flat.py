"""seg_dropout_bwd_ch (the dropout gradient re-drawn from the counter RNG:
FC-DenseNet's growth-conv Dropout, Network/model/FCDenseNet.py:33-35): the
one-chunk-per-thread kernel against the grid-stride kernel it replaces
(option dropout_flat = 0) -- the same per-element formula, so bit for bit --
and the drawn mask against the numpy restatement of the counter hash."""
import numpy as np
import pytest
import torch

from semanticsegmentation_tensorflow_amd import ops
from tests.test_gpu_ops_r2 import _np_uniform_vec

pytestmark = pytest.mark.gpu

# (pixels, channels in the buffer, valid channels, row strides of dy / dz)
CASES = [(2 * 96 * 312, 16, 16, 16, 16), (3 * 17 * 29, 24, 20, 40, 24), (1000, 64, 64, 64, 72), (7, 8, 3, 8, 8)]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("case", CASES)
def test_dropout_grad_flat_equals_loop(dev, case, dtype):
    P, C, cv, ldy, ldz = case
    kp, seed = 0.2, 987654321
    g = torch.Generator(device=dev).manual_seed(5)
    dy = torch.randn(P, ldy, device=dev, generator=g).to(dtype)

    def run():
        dz = torch.full((P, ldz), float("nan"), dtype=dtype, device=dev)
        ops.dropout_bwd_ch(dy[:, :C], dz[:, :C], cv, kp, seed)
        return dz
    a = run()
    ops.set_option("dropout_flat", 0)
    try:
        b = run()
    finally:
        ops.set_option("dropout_flat", 1)
    torch.cuda.synchronize()
    assert torch.equal(a[:, :C].view(torch.uint8), b[:, :C].view(torch.uint8))
    assert bool(torch.isnan(a[:, C:]).all())           # nothing past the channel range written
    u = _np_uniform_vec(seed, (np.arange(P, dtype=np.uint64)[:, None] * np.uint64(cv) +
                               np.arange(cv, dtype=np.uint64)[None, :]).reshape(-1)).reshape(P, cv)
    keep = torch.from_numpy(np.floor(np.float32(kp) + u) > 0).to(dev)
    got = a[:, :cv].float()
    assert bool((got[~keep] == 0).all())
    ref = dy[:, :cv].float() / kp
    assert torch.allclose(got[keep], ref[keep], rtol=1e-2 if dtype != torch.float32 else 1e-6, atol=0)
    assert bool((a[:, cv:C].float() == 0).all())
