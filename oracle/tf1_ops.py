"""TF 1.x op semantics restated on torch-CPU (TEST INFRASTRUCTURE ONLY).

Every function is differentiable through torch.autograd where the TF op is,
except where TF's gradient routing is not the plain mathematical derivative
(max-pool ties), which gets an explicit autograd.Function.

Layouts follow the reference: activations NHWC, conv filters HWIO
`[kh, kw, in, out]` (`Network/model/FCN.py:125`), transposed-conv filters
`[kh, kw, out, in]` (`Network/model/FCN.py:143`, `:102`).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


class TFShapeError(ValueError):
    """Mirror of TF's InvalidArgumentError for shape-rule violations."""


# ---------------------------------------------------------------------------
# padding rules
# ---------------------------------------------------------------------------
def same_pads(in_size: int, k: int, s: int, d: int = 1):
    """TF SAME: out = ceil(in/s); extra pad row/col goes bottom/right."""
    k_eff = k + (k - 1) * (d - 1)
    out = -(-in_size // s)
    total = max((out - 1) * s + k_eff - in_size, 0)
    return out, total // 2, total - total // 2


def valid_out(in_size: int, k: int, s: int, d: int = 1):
    k_eff = k + (k - 1) * (d - 1)
    return (in_size - k_eff) // s + 1


def conv_pads(in_size, k, s, d, padding):
    if padding == "SAME":
        return same_pads(in_size, k, s, d)
    if padding == "VALID":
        return valid_out(in_size, k, s, d), 0, 0
    raise ValueError(padding)


# ---------------------------------------------------------------------------
# Conv2D  (Network/model/FCN.py:130, Network/utils/utils.py:182)
# ---------------------------------------------------------------------------
def conv2d(x, w, stride=1, padding="SAME", dilation=1):
    """tf.nn.conv2d(x, w, strides=[1,s,s,1], padding, dilations) -- NHWC / HWIO.

    Cross-correlation (no kernel flip), asymmetric SAME padding."""
    N, H, W, C = x.shape
    R, S, Ci, Co = w.shape
    if Ci != C:
        raise TFShapeError(f"conv2d: input depth {C} != filter depth {Ci}")
    OH, pt, pb = conv_pads(H, R, stride, dilation, padding)
    OW, pl, pr = conv_pads(W, S, stride, dilation, padding)
    xn = x.permute(0, 3, 1, 2)
    xn = F.pad(xn, (pl, pr, pt, pb))
    y = F.conv2d(xn, w.permute(3, 2, 0, 1), stride=stride, dilation=dilation)
    y = y.permute(0, 2, 3, 1)
    assert y.shape[1] == OH and y.shape[2] == OW, (y.shape, OH, OW)
    return y


def atrous_conv2d(x, w, rate, padding="SAME"):
    """tf.nn.atrous_conv2d == conv2d with dilation=rate (Network/utils/utils.py:227)."""
    return conv2d(x, w, 1, padding, rate)


# ---------------------------------------------------------------------------
# conv2d_transpose (Network/model/FCN.py:155, :106; Network/utils/utils.py:272)
# ---------------------------------------------------------------------------
def conv2d_transpose_pads(in_size, out_size, k, s, padding):
    """Padding of Conv2DBackpropInput: treat output->input as a forward conv.

    Raises TFShapeError unless the forward conv of `out_size` yields `in_size`
    (SURVEY.md Appendix A.3 -- the rule that makes 375x1242 invalid for FCN)."""
    if padding == "SAME":
        exp, pt, pb = same_pads(out_size, k, s)
    else:
        exp, pt, pb = valid_out(out_size, k, s), 0, 0
    if exp != in_size:
        raise TFShapeError(
            f"conv2d_transpose: output size {out_size} with k={k} s={s} {padding} "
            f"implies input {exp}, got {in_size}")
    return pt, pb


def conv2d_transpose(x, w, output_shape, stride, padding="SAME"):
    """y = Conv2DBackpropInput(input_sizes=output_shape, filter=w, out_backprop=x).

    w is `[kh, kw, out_channels, in_channels]`; output channels = w.shape[2].
    y[n, ih*s + r - pt, iw*s + c - pl, co] += x[n, ih, iw, ci] * w[r, c, co, ci]
    Restated as an explicit per-tap scatter (independent of torch's
    conv_transpose)."""
    N, IH, IW, Ci = x.shape
    R, S, Co, Ci_w = w.shape
    if Ci_w != Ci:
        raise TFShapeError(f"conv2d_transpose: filter in-depth {Ci_w} != input depth {Ci}")
    ON, OH, OW, OC = output_shape
    if OC != Co or ON != N:
        raise TFShapeError("conv2d_transpose: output_shape mismatch with filter/input")
    pt, _ = conv2d_transpose_pads(IH, OH, R, stride, padding)
    pl, _ = conv2d_transpose_pads(IW, OW, S, stride, padding)
    BH = (IH - 1) * stride + R
    BW = (IW - 1) * stride + S
    big = x.new_zeros((N, BH, BW, Co))
    for r in range(R):
        for c in range(S):
            contrib = torch.einsum("nhwi,oi->nhwo", x, w[r, c])
            big[:, r:r + (IH - 1) * stride + 1:stride, c:c + (IW - 1) * stride + 1:stride, :] = (
                big[:, r:r + (IH - 1) * stride + 1:stride, c:c + (IW - 1) * stride + 1:stride, :] + contrib)
    return big[:, pt:pt + OH, pl:pl + OW, :]


# ---------------------------------------------------------------------------
# BiasAdd / ReLU / Add  (Network/model/FCN.py:132-134, :157, :171)
# ---------------------------------------------------------------------------
def bias_add(x, b):
    return x + b


def relu(x):
    # TF ReluGrad: dy * (y > 0) -- zero at 0, same as torch.relu's derivative.
    return torch.relu(x)


def add(a, b):
    return a + b


# ---------------------------------------------------------------------------
# MaxPool 2x2/2 VALID (Network/model/FCN.py:161-163) with TF1 CPU tie routing
# ---------------------------------------------------------------------------
class _MaxPool2x2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        OH, OW = H // 2, W // 2
        xs = x[:, :2 * OH, :2 * OW, :].reshape(N, OH, 2, OW, 2, C)
        cands = [xs[:, :, 0, :, 0], xs[:, :, 0, :, 1], xs[:, :, 1, :, 0], xs[:, :, 1, :, 1]]
        best = cands[0].clone()
        arg = torch.zeros_like(best, dtype=torch.int64)
        for i in range(1, 4):           # strict '>' keeps the first max in scan order
            upd = cands[i] > best
            best = torch.where(upd, cands[i], best)
            arg = torch.where(upd, torch.full_like(arg, i), arg)
        ctx.save_for_backward(arg)
        ctx.shape = x.shape
        return best

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, H, W, C = ctx.shape
        OH, OW = H // 2, W // 2
        dx = dy.new_zeros((N, OH, 2, OW, 2, C))
        for i in range(4):
            m = (arg == i).to(dy.dtype)
            dx[:, :, i // 2, :, i % 2] = dy * m
        out = dy.new_zeros((N, H, W, C))
        out[:, :2 * OH, :2 * OW, :] = dx.reshape(N, 2 * OH, 2 * OW, C)
        return out


def max_pool2x2(x):
    return _MaxPool2x2.apply(x)


def avg_pool2x2(x):
    """tf.nn.avg_pool 2x2/2 VALID (Network/utils/utils.py:309-310)."""
    N, H, W, C = x.shape
    OH, OW = H // 2, W // 2
    return x[:, :2 * OH, :2 * OW, :].reshape(N, OH, 2, OW, 2, C).mean(dim=(2, 4))


# ---------------------------------------------------------------------------
# Dropout (Network/model/FCN.py:165-167): x / kp * floor(kp + U[0,1))
# ---------------------------------------------------------------------------
def dropout(x, keep_prob, uniform=None):
    if keep_prob >= 1.0 and uniform is None:
        return x
    binary = torch.floor(keep_prob + uniform)
    return x / keep_prob * binary


# ---------------------------------------------------------------------------
# softmax_cross_entropy_with_logits + reduce_mean (Network/model/FCN.py:334)
# ---------------------------------------------------------------------------
def softmax_cross_entropy_with_logits(logits, labels):
    """Per-pixel loss = sum_c y_c * (logsumexp(z) - z_c)."""
    lse = torch.logsumexp(logits, dim=-1, keepdim=True)
    return (labels * (lse - logits)).sum(-1)


def mean_softmax_xent(logits, labels, mask=None):
    per = softmax_cross_entropy_with_logits(logits, labels)
    if mask is None:
        return per.mean()
    return (per * mask).sum() / mask.sum()


def one_hot(labels_idx, num_classes, dtype=torch.float64):
    return F.one_hot(labels_idx.long(), num_classes).to(dtype)


# ---------------------------------------------------------------------------
# ArgMax (Network/model/FCN.py:111): ties -> lowest index
# ---------------------------------------------------------------------------
def argmax(logits):
    C = logits.shape[-1]
    best = logits[..., 0]
    idx = torch.zeros(best.shape, dtype=torch.int64)
    for c in range(1, C):
        upd = logits[..., c] > best
        best = torch.where(upd, logits[..., c], best)
        idx = torch.where(upd, torch.full_like(idx, c), idx)
    return idx


# ---------------------------------------------------------------------------
# Frozen-statistics BatchNorm (Network/utils/utils.py:300-301; training=False)
# ---------------------------------------------------------------------------
BN_EPS = 1e-3


def batch_norm_frozen(x, gamma, beta, eps=BN_EPS):
    """moving_mean=0, moving_var=1 never updated: y = gamma*x/sqrt(1+eps) + beta."""
    return x * (gamma / math.sqrt(1.0 + eps)) + beta


# ---------------------------------------------------------------------------
# resize_bilinear(align_corners=True) (Network/utils/utils.py:329-330)
# ---------------------------------------------------------------------------
def _lerp_index(in_size, out_size):
    scale = (in_size - 1) / (out_size - 1) if out_size > 1 else 0.0
    src = torch.arange(out_size, dtype=torch.float64) * scale
    lo = torch.floor(src).long()
    hi = torch.clamp(lo + 1, max=in_size - 1)
    frac = src - lo.to(torch.float64)
    return lo, hi, frac


def resize_bilinear(x, size):
    OH, OW = size
    N, H, W, C = x.shape
    y0, y1, fy = _lerp_index(H, OH)
    x0, x1, fx = _lerp_index(W, OW)
    fy = fy.to(x.dtype).view(1, OH, 1, 1)
    fx = fx.to(x.dtype).view(1, 1, OW, 1)
    tl = x[:, y0][:, :, x0]
    tr = x[:, y0][:, :, x1]
    bl = x[:, y1][:, :, x0]
    br = x[:, y1][:, :, x1]
    top = tl + (tr - tl) * fx
    bot = bl + (br - bl) * fx
    return top + (bot - top) * fy


def concat(xs, axis=-1):
    """tf.concat (Network/utils/utils.py:332-333)."""
    return torch.cat(xs, dim=axis)


# ---------------------------------------------------------------------------
# AdamOptimizer (Network/model/FCN.py:338-340) -- TF1 epsilon placement
# ---------------------------------------------------------------------------
class AdamTF1:
    """lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m=b1 m+(1-b1)g; v=b2 v+(1-b2)g^2;
    theta -= lr_t * m / (sqrt(v) + eps)   (SURVEY.md Appendix A.8)."""

    def __init__(self, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.t = 0
        self.m = {}
        self.v = {}

    def apply(self, params: dict, grads: dict):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - self.b2 ** self.t) / (1 - self.b1 ** self.t)
        out = {}
        for k, p in params.items():
            g = grads[k]
            m = self.m.get(k, torch.zeros_like(p))
            v = self.v.get(k, torch.zeros_like(p))
            m = self.b1 * m + (1 - self.b1) * g
            v = self.b2 * v + (1 - self.b2) * g * g
            self.m[k], self.v[k] = m, v
            out[k] = p - lr_t * m / (torch.sqrt(v) + self.eps)
        return out
