"""wgrad_img (csrc/wgrad_img.hip): Conv2DBackpropFilter for large filters on
small feature maps -- FCN conv6's 7x7 over 12x39 (Network/model/FCN.py:78)
-- with the whole padded input image of a 16-channel chunk staged in LDS,
plain and fused with TF1 Adam (Network/model/FCN.py:338-340).

* filter gradient vs the float64 oracle (Conv2DBackpropFilter of the same
  bf16 operands; fp32 accumulation over up to 1,872 pixels: 2e-3 of max) and
  vs igemm_tn3, the kernel it replaces (1e-5 of max: fp32 summation order);
* fused TF1 Adam: p / m / v against float64 Adam on the oracle's gradient
  (m 1e-5, p 1e-5, v 1e-4 relative to max: fp32 (1 - beta2) as TF's kernel),
  the packed HWIO / KRSC bf16 copies bit-equal to bf16(p_new) with padding
  untouched;
* the launch chooser picks it exactly for conv6-like shapes (5x5 / 7x7,
  C % 16 == 0, K % 32 == 0, padded image within 28 KiB, >= 8 k-steps per
  image when there are several)."""
import math

import pytest
import torch

from oracle import tf1_ops as tf
from semanticsegmentation_tensorflow_amd import ops
from tests.gpu_utils import to_dev

pytestmark = pytest.mark.gpu

# (N, H, W, C, K, R, dilation): conv6 at the C2 shape (4 images of 12 x 39),
# one image with a single partial k-step, 5x5 over 3 images, a dilated 5x5
CASES = [
    (4, 12, 39, 512, 4096, 7, 1),
    (1, 5, 7, 32, 64, 7, 1),
    (3, 12, 30, 32, 96, 5, 1),
    (2, 14, 17, 48, 32, 5, 2),
]


def _case(case, seed):
    N, H, W, C, K, R, dil = case
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    d = ops.conv_desc(N, H, W, C, K, R, R, 1, dil, "SAME", ops.BF16)
    dy = torch.randn(N, d.OH, d.OW, K, generator=g, dtype=torch.float64)
    return x, dy, d


def _oracle_wgrad(x, dy, R, dil):
    xr = x.to(torch.bfloat16).double()
    w = torch.zeros(R, R, x.shape[3], dy.shape[3], dtype=torch.float64, requires_grad=True)
    y = tf.conv2d(xr, w, 1, "SAME", dil)
    (y * dy.to(torch.bfloat16).double()).sum().backward()
    return w.grad


@pytest.mark.parametrize("case", CASES)
def test_wgrad_img_filter_gradient(dev, case):
    N, H, W, C, K, R, dil = case
    x, dy, d = _case(case, 31)
    assert ops.conv_kernel_info(d, ops.OP_BWD_FILTER)[0].startswith("wgrad_img")
    xd, dyd = to_dev(x, torch.bfloat16, dev), to_dev(dy, torch.bfloat16, dev)
    ws = ops.Workspace(dev)
    dw = torch.full((R, R, C, K), float("nan"), device=dev)
    db = torch.full((K,), float("nan"), device=dev)
    ops.conv2d_bwd_filter(d, xd, dyd, dw, ws, None, db)
    ops.set_option("wgrad_img", 0)
    try:
        ws.get(ops.conv_workspace(d, ops.OP_BWD_FILTER))
        dw3 = torch.full((R, R, C, K), float("nan"), device=dev)
        ops.conv2d_bwd_filter(d, xd, dyd, dw3, ws)
    finally:
        ops.set_option("wgrad_img", 1)
    torch.cuda.synchronize()
    ref = _oracle_wgrad(x, dy, R, dil)
    got = dw.cpu().double()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, err
    e3 = (got - dw3.cpu().double()).abs().max().item() / ref.abs().max().item()
    assert e3 < 1e-5, e3
    dbr = dy.to(torch.bfloat16).double().sum(dim=(0, 1, 2))
    assert (db.cpu().double() - dbr).abs().max().item() <= 2e-5 * dbr.abs().max().item() + 1e-6


@pytest.mark.parametrize("case", CASES)
def test_wgrad_img_fused_adam(dev, case):
    N, H, W, C, K, R, dil = case
    x, dy, d = _case(case, 32)
    assert ops.wgrad_adam_fusable(d)
    g = torch.Generator().manual_seed(33)
    p0 = torch.randn(R, R, C, K, generator=g) * 0.05
    m0 = torch.randn(R, R, C, K, generator=g) * 1e-3
    v0 = torch.rand(R, R, C, K, generator=g) * 1e-5
    xd, dyd = to_dev(x, torch.bfloat16, dev), to_dev(dy, torch.bfloat16, dev)
    p, m, v = p0.to(dev), m0.to(dev), v0.to(dev)
    cp, kp = ops.round8(C), ops.round8(K)
    rows = torch.full(ops.packed_shape(R, R, C, K, ops.PACK_HWIO), 7.0, dtype=torch.bfloat16, device=dev)
    tr = torch.full(ops.packed_shape(R, R, C, K, ops.PACK_KRSC), 7.0, dtype=torch.bfloat16, device=dev)
    lr, t, gs = 1e-3, 3, 0.5
    # the gradient the fused launch applies: the plain launch's (same kernel,
    # same summation order), itself checked against the oracle above
    gref = torch.empty(R, R, C, K, device=dev)
    ops.conv2d_bwd_filter(d, xd, dyd, gref)
    ops.conv2d_bwd_filter_adam(d, xd, dyd, p, m, v, lr, t, grad_scale=gs, rows=(rows, cp, kp), tr=(tr, cp, kp))
    torch.cuda.synchronize()
    gc = gref.cpu().double() * gs
    me = 0.9 * m0.double() + 0.1 * gc
    ve = 0.999 * v0.double() + 0.001 * gc * gc
    lr_t = lr * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
    pe = p0.double() - lr_t * me / (ve.sqrt() + 1e-8)
    # fp32 arithmetic as TF1's kernel: (1 - beta2) = 1 - 0.999f carries 4.7e-5 relative
    for got, ref, nm, tol in ((p, pe, "p", 1e-5), (m, me, "m", 1e-5), (v, ve, "v", 1e-4)):
        err = (got.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < tol, (nm, err)
    # the oracle's gradient, through m: 2e-3 of max as the plain test
    go = _oracle_wgrad(x, dy, R, dil) * gs
    mo = 0.9 * m0.double() + 0.1 * go
    assert (m.cpu().double() - mo).abs().max().item() < 2e-3 * mo.abs().max().item()
    pb = p.cpu().to(torch.bfloat16)
    rh = rows.cpu().view(R * R, cp, kp)
    assert torch.equal(rh[:, :C, :K], pb.view(R * R, C, K))
    tk = tr.cpu().view(kp, R * R, cp)
    assert torch.equal(tk[:K, :, :C], pb.view(R * R, C, K).permute(2, 0, 1))
