"""Generate the committed golden vectors from the CPU oracle (float64).

    python tests/golden/make_golden.py

The reference ships no tests or fixtures and TensorFlow is not installed, so
these vectors come from the oracle's restatement of TF1 semantics (parity is
unpinned by the reference itself; see oracle/__init__.py).  Only inputs that
are cheap to regenerate are implied (seeds), outputs are stored.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import models as M          # noqa: E402
from oracle import tf1_ops as T         # noqa: E402
from tests.model_inputs import densenet_weights, he_weights, reference_init_weights, synthetic_batch  # noqa: E402

N, H, W = 2, 64, 96
SLICE = 512


def fcn_case(weights, img, lab):
    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in weights.items()}
    pred, logits = M.fcn_forward(p, torch.from_numpy(img).double())
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(lab), 2))
    loss.backward()
    out = {"logits": logits.detach().numpy(), "loss": np.array(loss.item()),
           "pred": pred.numpy().astype(np.int8)}
    opt = T.AdamTF1(1e-4)
    upd = opt.apply({k: v.detach() for k, v in p.items()}, {k: v.grad for k, v in p.items()})
    for k, v in p.items():
        g = v.grad.numpy().reshape(-1)
        out[f"gnorm/{k}"] = np.array(np.linalg.norm(g))
        out[f"gslice/{k}"] = g[:SLICE].copy()
        out[f"adam1/{k}"] = upd[k].numpy().reshape(-1)[:SLICE].copy()
    return out


DN_N, DN_SLICE = 1, 64


def densenet_case(weights, img, lab):
    """FC-DenseNet (FCDenseNet.py:83-163) 1x64x96x3: logits, loss, per-variable
    gradient norms, 64-element gradient / Adam slices (SURVEY.md 8c item iii)."""
    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in weights.items()}
    pred, logits = M.fcdensenet_forward(p, torch.from_numpy(img).double())
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(lab), 2))
    loss.backward()
    out = {"logits": logits.detach().numpy(), "loss": np.array(loss.item()),
           "pred": pred.numpy().astype(np.int8)}
    opt = T.AdamTF1(1e-4)
    upd = opt.apply({k: v.detach() for k, v in p.items()}, {k: v.grad for k, v in p.items()})
    for k, v in p.items():
        g = v.grad.numpy().reshape(-1)
        out[f"gnorm/{k}"] = np.array(np.linalg.norm(g))
        out[f"gslice/{k}"] = g[:DN_SLICE].copy()
        out[f"adam1/{k}"] = upd[k].numpy().reshape(-1)[:DN_SLICE].copy()
    return out


def ops_cases():
    g = torch.Generator().manual_seed(123)
    o = {}
    x = torch.randn(1, 5, 6, 3, generator=g, dtype=torch.float64)
    w = torch.randn(4, 4, 3, 2, generator=g, dtype=torch.float64)
    o["conv_even_x"], o["conv_even_w"] = x.numpy(), w.numpy()
    o["conv_even_y"] = T.conv2d(x, w).numpy()                      # SAME, pads (1,2)x(1,2)
    o["conv_s2_y"] = T.conv2d(x, w, stride=2).numpy()
    xt = torch.randn(1, 3, 4, 5, generator=g, dtype=torch.float64)
    wt = torch.randn(4, 4, 6, 5, generator=g, dtype=torch.float64)
    o["tconv_x"], o["tconv_w"] = xt.numpy(), wt.numpy()
    o["tconv_y"] = T.conv2d_transpose(xt, wt, (1, 6, 8, 6), 2).numpy()
    o["tconv_odd_y"] = T.conv2d_transpose(xt, wt, (1, 5, 7, 6), 2).numpy()   # asymmetric pads
    x3 = torch.randn(1, 2, 3, 4, generator=g, dtype=torch.float64)
    w3 = torch.randn(16, 16, 2, 4, generator=g, dtype=torch.float64)
    o["tconv8_x"], o["tconv8_w"] = x3.numpy(), w3.numpy()
    o["tconv8_y"] = T.conv2d_transpose(x3, w3, (1, 16, 24, 2), 8).numpy()
    xp = torch.randn(2, 5, 7, 3, generator=g, dtype=torch.float64)
    xp[0, 0, 0] = xp[0, 0, 1]
    xp = xp.requires_grad_(True)
    yp = T.max_pool2x2(xp)
    dyp = torch.randn(yp.shape, generator=g, dtype=torch.float64)
    (yp * dyp).sum().backward()
    o["pool_x"], o["pool_dy"], o["pool_y"], o["pool_dx"] = (xp.detach().numpy(), dyp.numpy(),
                                                            yp.detach().numpy(), xp.grad.numpy())
    z = (torch.randn(1, 4, 5, 2, generator=g, dtype=torch.float64) * 3).requires_grad_(True)
    lab = torch.randint(0, 2, (1, 4, 5), generator=g)
    loss = T.mean_softmax_xent(z, T.one_hot(lab, 2))
    loss.backward()
    o["xent_z"], o["xent_lab"], o["xent_loss"], o["xent_dz"] = (z.detach().numpy(), lab.numpy(),
                                                                np.array(loss.item()), z.grad.numpy())
    pa = torch.randn(10, generator=g, dtype=torch.float64)
    opt = T.AdamTF1(1e-3)
    params = {"p": pa}
    gs = []
    for _ in range(3):
        gr = torch.randn(10, generator=g, dtype=torch.float64) * 1e-2
        gs.append(gr.numpy())
        params = opt.apply(params, {"p": gr})
    o["adam_p0"], o["adam_g"], o["adam_p3"] = pa.numpy(), np.stack(gs), params["p"].numpy()
    xb = torch.randn(1, 3, 4, 2, generator=g, dtype=torch.float64)
    o["bilinear_x"], o["bilinear_y"] = xb.numpy(), T.resize_bilinear(xb, (5, 7)).numpy()
    return o


def main():
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **ops_cases())
    shapes = M.fcn_param_shapes(3, 2)
    img, lab = synthetic_batch(N, H, W, 2)
    np.savez_compressed(os.path.join(HERE, "fcn_ref_init.npz"),
                        **fcn_case(reference_init_weights(shapes, 0), img, lab))
    np.savez_compressed(os.path.join(HERE, "fcn_he_init.npz"), **fcn_case(he_weights(shapes, 1), img, lab))
    dimg, dlab = synthetic_batch(DN_N, H, W, 8)
    np.savez_compressed(os.path.join(HERE, "fcdensenet_he.npz"),
                        **densenet_case(densenet_weights(M.fcdensenet_param_shapes(3, 2), 7), dimg, dlab))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
