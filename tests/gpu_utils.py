"""Helpers shared by the GPU parity tests (device tensors <-> oracle tensors)."""
import torch

from semanticsegmentation_tensorflow_amd import ops

TOL = {torch.float32: 2e-5, torch.bfloat16: 1.2e-2, torch.float16: 2e-3}


def to_dev(x, dtype, dev, cpad=None):
    """float64 NHWC -> padded device tensor [N,H,W,round8(C)] (zeros in padding)."""
    N, H, W, C = x.shape
    cp = cpad or ops.round8(C)
    t = torch.zeros(N, H, W, cp, dtype=dtype, device=dev)
    t[..., :C] = x.to(dtype).to(dev)
    return t


def from_dev(t, C=None):
    C = t.shape[-1] if C is None else C
    return t[..., :C].double().cpu()


def rnd(x, dtype):
    """Round a float64 tensor through `dtype` (what the device sees)."""
    return x.to(dtype).double()


def rel_err(a, b):
    a = a.double()
    b = b.double()
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


def assert_close(got, ref, dtype, what="", tol=None):
    tol = TOL[dtype] if tol is None else tol
    e = rel_err(got, ref)
    assert e <= tol, f"{what}: rel err {e:.3e} > {tol:.1e}"
    return e
