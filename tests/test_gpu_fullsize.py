"""Parity at the benchmarked configurations: the exact
composed kernel set `bench.py` times, checked against the oracle.

C2 -- FCN bf16, 4 x 384 x 1248 (375 x 1242 zero-padded, loss masked), ONE
train step through `Session` exactly as `bench.py` builds it (keep_prob = 1:
TF's dropout mask is not reproducible; the fused dropout has its own test).
At this size the launch chooser picks the paths small tests only reach when
forced: 256x256 `conv_halo2` tiles, the resident-filter `conv_res64`, deferred
side-stream split-K filter-gradient reductions, the 256x128 half-tile fused
conv6 filter-gradient + Adam.  Three checks:

* layer-local, tight (every conv): the device's own bf16 input x, the
  gradient dz its filter-gradient launch consumed and the bf16-rounded filter
  go through the oracle's conv in fp32; forward output and input gradient
  (bf16) within 4e-3 relative + 1e-3 of max (one bf16 rounding), filter and
  bias gradients (fp32) within 1e-3 of max (fp32 summation order over up to
  1.9 M pixels);
* end-to-end against the oracle with bf16 rounding points (fp32 CPU): logits
  within 3e-2 of max, loss 1e-2, per-variable gradient cosine >= 0.95 and
  median relative L2 <= 0.1 (ReLU-flip amplification, tests/test_gpu_fcn.py);
* the TF1 Adam update: conv6 (fused filter-gradient + Adam, half tiles),
  conv7 (fused, full tiles) and conv3_2 (multi-tensor adam_pack) against
  float64 Adam on the device gradient (1e-6 + 1e-5 max|p|), and their packed
  bf16 compute copies (KRSC / HWIO) bit-equal to bf16(p_new).

C3 -- FC-DenseNet bf16 at 1 x 384 x 1248 with the dense-block concat views:
end-to-end vs the oracle with bf16 rounding points and layer-local checks of a
sample of its convs.  C5 -- DeepLab bf16 at a small size, end-to-end.
"""
import math

import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import ops, tf
from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.model_inputs import densenet_weights, he_weights

pytestmark = pytest.mark.gpu
LR = 1e-4


def bf16r(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _cpu_threads():
    torch.set_num_threads(16)


def _kitti_batch(N, H, W, HP, WP, seed):
    rng = np.random.default_rng(seed)
    img = np.zeros((N, HP, WP, 3), np.float32)
    img[:, :H, :W] = rng.integers(0, 256, size=(N, H, W, 3))
    lab = np.zeros((N, HP, WP), np.uint8)
    lab[:, H // 2:H, W // 4:3 * W // 4] = 1
    flip = rng.random((N, H, W)) < 0.05
    lab[:, :H, :W] = np.where(flip, 1 - lab[:, :H, :W], lab[:, :H, :W])
    return img, lab


def _run_step(builder, weights, img, lab, H, W):
    G.reset_default_graph()
    N, HP, WP, _ = img.shape
    image = tf.placeholder(tf.float32, [None, HP, WP, 3], name="input_image")
    labels = tf.placeholder(tf.uint8, [None, HP, WP], name="annotation")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    pred, logits = builder(image, keep)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels, valid_hw=(H, W)))
    train = tf.train.AdamOptimizer(LR).minimize(loss)
    sess = tf.Session(compute_dtype="bf16", seed=0)
    sess.store_fused_grads = True
    sess.run(tf.global_variables_initializer())
    for k, v in weights.items():
        sess.assign(k, v)
    sess.capture = []
    out_logits, out_loss, _ = sess.run([logits, loss, train], feed_dict={image: img, labels: lab, keep: 1.0})
    torch.cuda.synchronize()
    return sess, out_logits, float(out_loss)


def _host(t, c):
    return t[..., :c].float().cpu()


def _layer_local(rec, w, b, sess, weights=None):
    """Oracle fwd / dgrad / wgrad of one conv from the device's own operands
    (`weights`: the pre-step values of a folded BatchNorm's gamma / beta --
    the store holds the post-Adam ones)."""
    C, K = w.shape[2], w.shape[3]
    x = _host(rec["x"], C)
    if rec.get("pro"):          # BatchNorm + ReLU folded into this conv's operand prologue
        gname, bname, eps, relu = rec["pro"]
        gamma, beta = (torch.from_numpy(weights[gname]), torch.from_numpy(weights[bname]))
        x = x * (gamma / np.sqrt(1.0 + eps)) + beta
        x = bf16r(torch.relu(x) if relu else x)
    x = x.requires_grad_(True)
    wt = bf16r(torch.from_numpy(w)).requires_grad_(True)
    z = T.conv2d(x, wt, rec["stride"], rec["padding"], rec["dilation"])
    y = z + torch.from_numpy(b) if b is not None else z
    if rec["relu"]:
        y = torch.relu(y)
    dz = _host(rec["dz"], K)
    z.backward(dz)
    res = {}
    yd = _host(rec["y"], K)
    res["fwd"] = (yd - y.detach()).abs() - (4e-3 * y.detach().abs() + 1e-3 * y.detach().abs().max())
    if rec["dx"] is not None:
        dx = x.grad
        if rec["dx_masked"]:
            dx = dx * (x.detach() > 0)
        dxd = _host(rec["dx"], C)
        res["dgrad"] = (dxd - dx).abs() - (4e-3 * dx.abs() + 1e-3 * dx.abs().max())
    gw = sess.store.grad(rec["name"]).cpu()
    res["wgrad"] = (gw - wt.grad).abs() - 1e-3 * wt.grad.abs().max()
    if rec["bias"] is not None:
        db = dz.sum(dim=(0, 1, 2))
        res["bgrad"] = (sess.store.grad(rec["bias"]).cpu() - db).abs() - 1e-3 * db.abs().max()
    return {k: float(v.max()) for k, v in res.items()}


def _grad_stats(sess, ref_grads):
    worst = []
    for k, gref in ref_grads.items():
        gg = sess.store.grad(k).cpu().numpy().reshape(-1).astype(np.float64)
        gr = gref.reshape(-1).astype(np.float64)
        cos = gg @ gr / max(np.linalg.norm(gg) * np.linalg.norm(gr), 1e-300)
        l2 = np.linalg.norm(gg - gr) / max(np.linalg.norm(gr), 1e-300)
        worst.append((cos, l2, k))
    return worst


# --------------------------------------------------------------------- C2
FCN_H, FCN_W, FCN_HP, FCN_WP, FCN_N = 375, 1242, 384, 1248, 4


@pytest.fixture(scope="module")
def c2(dev):
    weights = he_weights(M.fcn_param_shapes(3, 2), 61)
    img, lab = _kitti_batch(FCN_N, FCN_H, FCN_W, FCN_HP, FCN_WP, 62)
    sess, lg, lo = _run_step(lambda im, kp: FCN(im, kp, 2).create(), weights, img, lab, FCN_H, FCN_W)
    return {"sess": sess, "weights": weights, "img": img, "lab": lab, "logits": lg, "loss": lo}


def test_c2_kernel_set_is_the_benchmarked_one(c2):
    """The composed paths the bench times are the ones under test."""
    names = set()
    for rec in c2["sess"].capture:
        for op in (ops.OP_FWD, ops.OP_BWD_DATA, ops.OP_BWD_FILTER):
            names.add(ops.conv_kernel_info(rec["desc"], op)[0])
    print(sorted(names))
    assert any("halo2" in n or "conv_halo<bf16,256,256>" in n for n in names), names
    assert any("res64" in n for n in names), names
    assert len(c2["sess"].capture) == 17


def test_c2_layer_local_parity(c2):
    _cpu_threads()
    sess, weights = c2["sess"], c2["weights"]
    bad = []
    for rec in sess.capture:
        b = weights.get(rec["bias"]) if rec["bias"] else None
        r = _layer_local(rec, weights[rec["name"]], b, sess)
        print(rec["name"], {k: f"{v:+.2e}" for k, v in r.items()})
        bad += [(rec["name"], k, v) for k, v in r.items() if v > 0]
    assert not bad, bad


def test_c2_end_to_end_vs_oracle(c2):
    _cpu_threads()
    weights = c2["weights"]
    wr = {k: (bf16r(torch.from_numpy(v)) if v.ndim == 4 else torch.from_numpy(v)).requires_grad_(True)
          for k, v in weights.items()}
    x = torch.from_numpy(c2["img"])
    _, logits = M.fcn_forward(wr, x, quant=bf16r)
    mask = torch.zeros(FCN_N, FCN_HP, FCN_WP)
    mask[:, :FCN_H, :FCN_W] = 1
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(c2["lab"]).long(), 2, torch.float32), mask)
    loss.backward()
    rl = logits.detach().numpy()
    e = np.abs(c2["logits"] - rl).max() / np.abs(rl).max()
    assert e < 3e-2, e
    assert abs(c2["loss"] - loss.item()) <= 1e-2 * max(1.0, abs(loss.item())), (c2["loss"], loss.item())
    agree = (np.argmax(c2["logits"], -1) == np.argmax(rl, -1))[:, :FCN_H, :FCN_W].mean()
    assert agree > 0.99, agree
    stats = _grad_stats(c2["sess"], {k: v.grad.numpy() for k, v in wr.items()})
    for cos, l2, k in sorted(stats):
        print(f"GRAD {k:20s} cos={cos:.5f} relL2={l2:.3e}")
    assert min(s[0] for s in stats) >= 0.95
    assert np.median([s[1] for s in stats]) <= 0.1


def test_c2_adam_update_and_packed_copies(c2):
    sess, weights = c2["sess"], c2["weights"]
    st = sess.store
    t = 1
    lr_t = LR * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
    for k in ("conv6/weights", "conv7/weights", "conv3_2/weights", "conv6/biases", "conv_t2/weights"):
        g = st.grad(k).cpu().double()
        p0 = torch.from_numpy(weights[k]).double()
        m = 0.1 * g
        v = 0.001 * g * g
        ref = (p0 - lr_t * m / (v.sqrt() + 1e-8)).numpy()
        got = sess.variable_value(k)
        assert np.abs(got - ref).max() <= 1e-6 + 1e-5 * np.abs(ref).max(), k
        np.testing.assert_allclose(st.adam_m(k).cpu().numpy(), m.numpy(), rtol=1e-5, atol=1e-12)
    for k in ("conv6/weights", "conv7/weights", "conv3_2/weights"):
        p = torch.from_numpy(sess.variable_value(k)).to(torch.bfloat16)         # R S C K
        R, S, C, K = p.shape
        krsc = st.packed[(k, ops.PACK_KRSC)][0].cpu()[:K, :, :, :C]
        assert torch.equal(krsc, p.permute(3, 0, 1, 2)), k
        hwio = st.packed[(k, ops.PACK_HWIO)][0].cpu()[:, :, :C, :K]
        assert torch.equal(hwio, p), k


# --------------------------------------------------------------------- C3
@pytest.fixture(scope="module")
def c3(dev):
    H, W = 384, 1248
    weights = densenet_weights(M.fcdensenet_param_shapes(3, 2), 71)
    img, lab = _kitti_batch(1, H, W, H, W, 72)
    sess, lg, lo = _run_step(lambda im, kp: FCDenseNet(im, kp, 2), weights, img, lab, H, W)
    return {"sess": sess, "weights": weights, "img": img, "lab": lab, "logits": lg, "loss": lo}


def test_c3_concat_views_active(c3):
    plan = next(iter(c3["sess"].plans.values()))
    assert len(plan.alias_nodes) >= 20, len(plan.alias_nodes)


def test_c3_layer_local_parity(c3):
    _cpu_threads()
    sess, weights = c3["sess"], c3["weights"]
    recs = sess.capture
    sample = recs[:6] + recs[len(recs) // 2:len(recs) // 2 + 4] + recs[-6:]
    bad = []
    for rec in sample:
        r = _layer_local(rec, weights[rec["name"]], None, sess, weights)
        if "dgrad" in r:
            del r["dgrad"]      # dense-block input gradients accumulate in place (concat views)
        print(rec["name"], {k: f"{v:+.2e}" for k, v in r.items()})
        bad += [(rec["name"], k, v) for k, v in r.items() if v > 0]
    assert not bad, bad


def test_c3_end_to_end_vs_oracle(c3):
    _cpu_threads()
    weights = c3["weights"]
    wr = {k: (bf16r(torch.from_numpy(v)) if v.ndim == 4 else torch.from_numpy(v)).requires_grad_(True)
          for k, v in weights.items()}
    _, logits = M.fcdensenet_forward(wr, torch.from_numpy(c3["img"]), quant=bf16r)
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(c3["lab"]).long(), 2, torch.float32))
    loss.backward()
    rl = logits.detach().numpy()
    e = np.abs(c3["logits"] - rl).max() / np.abs(rl).max()
    assert e < 3e-2, e
    assert abs(c3["loss"] - loss.item()) <= 1e-2 * max(1.0, abs(loss.item()))
    stats = _grad_stats(c3["sess"], {k: v.grad.numpy() for k, v in wr.items()})
    for cos, l2, k in sorted(stats)[:10]:
        print(f"GRAD {k:40s} cos={cos:.5f} relL2={l2:.3e}")
    assert min(s[0] for s in stats) >= 0.95
    assert np.median([s[1] for s in stats]) <= 0.1


# --------------------------------------------------------------------- C5
def test_c5_deeplab_bf16_vs_oracle(dev):
    from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
    _cpu_threads()
    H, W = 128, 192
    weights = he_weights(M.deeplab_param_shapes(3, 2), 81)
    for k in weights:
        if k.endswith("gamma"):
            weights[k] = (1.0 + 0.1 * np.random.default_rng(82).standard_normal(weights[k].shape)).astype(np.float32)
    img, lab = _kitti_batch(2, H, W, H, W, 83)
    sess, lg, lo = _run_step(lambda im, kp: DeepLabASPP(im, kp, 2), weights, img, lab, H, W)
    wr = {k: (bf16r(torch.from_numpy(v)) if v.ndim == 4 else torch.from_numpy(v)).requires_grad_(True)
          for k, v in weights.items()}
    _, logits = M.deeplab_forward(wr, torch.from_numpy(img), quant=bf16r)
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(lab).long(), 2, torch.float32))
    loss.backward()
    rl = logits.detach().numpy()
    assert np.abs(lg - rl).max() / np.abs(rl).max() < 3e-2
    assert abs(lo - loss.item()) <= 1e-2 * max(1.0, abs(loss.item()))
    stats = _grad_stats(sess, {k: v.grad.numpy() for k, v in wr.items()})
    assert min(s[0] for s in stats) >= 0.95, sorted(stats)[:3]
    assert np.median([s[1] for s in stats]) <= 0.1
