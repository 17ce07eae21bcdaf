"""Pinning the CPU oracle (no GPU).

The reference has no tests/fixtures and TF is absent, so the oracle is pinned
by (1) an independent numpy-loop restatement, (2) hand-derived known answers
for every TF-specific rule the hot path relies on, and (3) the committed
golden vectors (tests/golden/make_golden.py) -- which also guard the oracle
against silent drift."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import naive
from oracle import tf1_ops as T
from tests.golden import make_golden as MG
from tests.model_inputs import he_weights, reference_init_weights, synthetic_batch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ---------------------------------------------------------------- (1) naive loops
@pytest.mark.parametrize("case", [(1, 5, 6, 3, 2, 4, 1, 1, "SAME"), (2, 7, 5, 4, 3, 3, 2, 1, "SAME"),
                                  (1, 9, 9, 2, 3, 3, 1, 2, "SAME"), (1, 6, 7, 3, 2, 3, 1, 1, "VALID"),
                                  (1, 4, 5, 2, 2, 7, 1, 1, "SAME")])
def test_conv2d_matches_naive_loops(case):
    N, H, W, C, K, R, s, d, pad = case
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    w = torch.randn(R, R, C, K, generator=g, dtype=torch.float64)
    np.testing.assert_allclose(T.conv2d(x, w, s, pad, d).numpy(),
                               naive.conv2d(x.numpy(), w.numpy(), s, pad, d), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("case", [((1, 3, 4, 5), (4, 4, 6, 5), (1, 6, 8, 6), 2),
                                  ((1, 3, 4, 5), (4, 4, 6, 5), (1, 5, 7, 6), 2),
                                  ((2, 2, 3, 4), (16, 16, 2, 4), (2, 16, 24, 2), 8)])
def test_conv2d_transpose_matches_naive_loops(case):
    xs, ws, os_, s = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(*xs, generator=g, dtype=torch.float64)
    w = torch.randn(*ws, generator=g, dtype=torch.float64)
    np.testing.assert_allclose(T.conv2d_transpose(x, w, os_, s).numpy(),
                               naive.conv2d_transpose(x.numpy(), w.numpy(), os_, s), rtol=1e-12, atol=1e-12)


def test_conv2d_transpose_is_adjoint_of_conv2d():
    """<conv(u), v> == <u, conv_T(v)>: Conv2DBackpropInput is the exact adjoint."""
    g = torch.Generator().manual_seed(2)
    u = torch.randn(1, 12, 10, 3, generator=g, dtype=torch.float64)
    w = torch.randn(4, 4, 3, 5, generator=g, dtype=torch.float64)
    y = T.conv2d(u, w, stride=2)
    v = torch.randn(y.shape, generator=g, dtype=torch.float64)
    lhs = (y * v).sum()
    rhs = (u * T.conv2d_transpose(v, w, tuple(u.shape), 2)).sum()
    assert abs(lhs - rhs) < 1e-10 * abs(lhs)


def test_maxpool_grad_matches_naive():
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 5, 7, 3, generator=g, dtype=torch.float64)
    x[0, 0, 0, :] = x[0, 0, 1, :]
    x[1, 2, 2, :] = x[1, 3, 3, :]
    xr = x.clone().requires_grad_(True)
    y = T.max_pool2x2(xr)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    (y * dy).sum().backward()
    y_n, dx_n = naive.max_pool2x2_with_grad(x.numpy(), dy.numpy())
    np.testing.assert_array_equal(y.detach().numpy(), y_n)
    np.testing.assert_array_equal(xr.grad.numpy(), dx_n)


# ---------------------------------------------------------------- (2) known answers
def test_same_padding_even_kernel_known_answer():
    """TF SAME with k=4, s=1: total pad 3 -> 1 before, 2 after (extra goes bottom/right)."""
    assert T.same_pads(4, 4, 1) == (4, 1, 2)
    assert T.same_pads(375, 2, 2) == (188, 0, 1)
    x = torch.tensor([1.0, 2, 3, 4], dtype=torch.float64).view(1, 1, 4, 1)
    w = torch.tensor([1.0, 10, 100, 1000], dtype=torch.float64).view(1, 4, 1, 1)
    y = T.conv2d(x, w).view(-1).tolist()
    assert y == [3210.0, 4321.0, 432.0, 43.0]


def test_conv2d_transpose_shape_rule_known_answer():
    """375x1242 cannot go through FCN's conv_t1 (pool5 11x38, pool4 23x77), SURVEY.md 0-3."""
    with pytest.raises(T.TFShapeError):
        T.conv2d_transpose_pads(11, 23, 4, 2, "SAME")
    assert T.conv2d_transpose_pads(12, 24, 4, 2, "SAME") == (1, 1)
    assert T.conv2d_transpose_pads(48, 384, 16, 8, "SAME") == (4, 4)


def test_adam_tf1_epsilon_placement_known_answer():
    """Step 1: theta -= lr*sqrt(1-b2)/(1-b1) * m/(sqrt(v)+eps)  (TF1), not torch's form."""
    lr, gv = 1e-4, 1e-7
    opt = T.AdamTF1(lr)
    out = opt.apply({"p": torch.zeros(1, dtype=torch.float64)}, {"p": torch.full((1,), gv, dtype=torch.float64)})
    m, v = 0.1 * gv, 0.001 * gv * gv
    expect = -lr * math.sqrt(1 - 0.999) / (1 - 0.9) * m / (math.sqrt(v) + 1e-8)
    assert abs(out["p"].item() - expect) < 1e-12 * abs(expect)
    torch_form = -lr * (m / 0.1) / (math.sqrt(v / 0.001) + 1e-8)
    assert abs(expect - torch_form) > 0.1 * abs(expect)     # the two forms really differ here


def test_dropout_tf1_formula_known_answer():
    x = torch.tensor([2.0, 2.0, 2.0], dtype=torch.float64)
    u = torch.tensor([0.19, 0.2, 0.99], dtype=torch.float64)
    assert T.dropout(x, 0.8, u).tolist() == [0.0, 2.5, 2.5]


def test_softmax_xent_and_argmax_known_answers():
    z = torch.tensor([[0.0, 0.0], [3.0, 1.0]], dtype=torch.float64).view(1, 1, 2, 2)
    y = torch.tensor([[1.0, 0.0], [0.0, 1.0]], dtype=torch.float64).view(1, 1, 2, 2)
    per = T.softmax_cross_entropy_with_logits(z, y).view(-1)
    assert abs(per[0] - math.log(2)) < 1e-15
    assert abs(per[1] - (math.log(math.exp(3) + math.exp(1)) - 1)) < 1e-14
    assert T.argmax(z).view(-1).tolist() == [0, 0]          # tie -> lowest index


def test_bilinear_align_corners_and_frozen_bn_known_answers():
    x = torch.tensor([0.0, 10.0], dtype=torch.float64).view(1, 1, 2, 1)
    assert T.resize_bilinear(x, (1, 3)).view(-1).tolist() == [0.0, 5.0, 10.0]
    y = T.batch_norm_frozen(torch.tensor([2.0], dtype=torch.float64), torch.tensor([1.0], dtype=torch.float64),
                            torch.tensor([0.5], dtype=torch.float64))
    assert abs(y.item() - (2.0 / math.sqrt(1.001) + 0.5)) < 1e-15


# ---------------------------------------------------------------- (3) golden vectors
def test_ops_golden_vectors():
    gold = np.load(os.path.join(GOLD, "ops.npz"))
    now = MG.ops_cases()
    assert set(gold.files) == set(now)
    for k in gold.files:
        np.testing.assert_allclose(now[k], gold[k], rtol=1e-12, atol=1e-14, err_msg=k)


@pytest.mark.parametrize("which", ["he", "ref"])
def test_fcn_golden_vectors(which):
    shapes = M.fcn_param_shapes(3, 2)
    w = he_weights(shapes, 1) if which == "he" else reference_init_weights(shapes, 0)
    img, lab = synthetic_batch(MG.N, MG.H, MG.W, 2)
    now = MG.fcn_case(w, img, lab)
    gold = np.load(os.path.join(GOLD, f"fcn_{which}_init.npz"))
    for k in gold.files:
        np.testing.assert_allclose(now[k], gold[k], rtol=1e-9, atol=1e-30, err_msg=k)
    if which == "ref":
        # reference init: activations vanish, loss ~ ln 2
        assert abs(float(gold["loss"]) - math.log(2)) < 1e-3


def test_fcdensenet_golden_vectors():
    """FC-DenseNet oracle (FCDenseNet.py:23-163) pinned to its committed fixture."""
    from tests.model_inputs import densenet_weights
    w = densenet_weights(M.fcdensenet_param_shapes(3, 2), 7)
    img, lab = synthetic_batch(MG.DN_N, MG.H, MG.W, 8)
    now = MG.densenet_case(w, img, lab)
    gold = np.load(os.path.join(GOLD, "fcdensenet_he.npz"))
    assert set(gold.files) == set(now)
    for k in gold.files:
        np.testing.assert_allclose(now[k], gold[k], rtol=1e-9, atol=1e-30, err_msg=k)
