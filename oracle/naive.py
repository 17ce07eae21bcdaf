"""Independent pure-numpy loop restatements (TEST INFRASTRUCTURE ONLY).

Used to pin `oracle/tf1_ops.py` on tiny shapes: these loops follow the TF1
definitions directly with no torch involved.
"""
import numpy as np

from .tf1_ops import conv_pads, conv2d_transpose_pads


def conv2d(x, w, stride=1, padding="SAME", dilation=1):
    N, H, W, C = x.shape
    R, S, _, K = w.shape
    OH, pt, _ = conv_pads(H, R, stride, dilation, padding)
    OW, pl, _ = conv_pads(W, S, stride, dilation, padding)
    y = np.zeros((N, OH, OW, K), dtype=np.float64)
    for n in range(N):
        for oh in range(OH):
            for ow in range(OW):
                acc = np.zeros(K)
                for r in range(R):
                    ih = oh * stride + r * dilation - pt
                    if ih < 0 or ih >= H:
                        continue
                    for s in range(S):
                        iw = ow * stride + s * dilation - pl
                        if iw < 0 or iw >= W:
                            continue
                        acc += x[n, ih, iw, :] @ w[r, s]
                y[n, oh, ow] = acc
    return y


def conv2d_transpose(x, w, output_shape, stride, padding="SAME"):
    N, IH, IW, Ci = x.shape
    R, S, Co, _ = w.shape
    _, OH, OW, _ = output_shape
    pt, _ = conv2d_transpose_pads(IH, OH, R, stride, padding)
    pl, _ = conv2d_transpose_pads(IW, OW, S, stride, padding)
    y = np.zeros((N, OH, OW, Co))
    for n in range(N):
        for ih in range(IH):
            for iw in range(IW):
                for r in range(R):
                    oh = ih * stride + r - pt
                    if oh < 0 or oh >= OH:
                        continue
                    for s in range(S):
                        ow = iw * stride + s - pl
                        if ow < 0 or ow >= OW:
                            continue
                        y[n, oh, ow] += w[r, s] @ x[n, ih, iw]
    return y


def max_pool2x2_with_grad(x, dy):
    N, H, W, C = x.shape
    OH, OW = H // 2, W // 2
    y = np.zeros((N, OH, OW, C))
    dx = np.zeros_like(x)
    for n in range(N):
        for i in range(OH):
            for j in range(OW):
                for c in range(C):
                    best, bi, bj = -np.inf, 0, 0
                    for a in range(2):
                        for b in range(2):
                            v = x[n, 2 * i + a, 2 * j + b, c]
                            if v > best:
                                best, bi, bj = v, a, b
                    y[n, i, j, c] = best
                    dx[n, 2 * i + bi, 2 * j + bj, c] += dy[n, i, j, c]
    return y, dx
