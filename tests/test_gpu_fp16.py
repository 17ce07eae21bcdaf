"""fp16 compute path (BASELINE.json config C5: "fp16 with fp32 accum"):
IEEE-half activations and filter copies, v_mfma_f32_16x16x32_f16 with fp32
accumulation, fp32 master weights / Adam state, dynamic loss scaling.

* DeepLab-style C5 model (semanticsegmentation_tensorflow_amd/deeplab.py, incl.
  the ASPP image-pooling branch) and the FCN: one train step vs the oracle
  with fp16 rounding points (fp32 CPU).  The device's stored gradients carry
  the loss scale S; they are compared after dividing by S.  Tolerances:
  logits 1e-2 of max, loss 5e-3, gradient cosine >= 0.98 per variable and
  median relative L2 <= 0.05 (fp16 keeps 3 more mantissa bits than bf16;
  the residual spread is ReLU-flip amplification, as tests/test_gpu_fcn.py).
* dynamic loss scaling (TF DynamicLossScale semantics): an overflowing step
  is skipped (parameters, Adam slots and step count unchanged) and the scale
  halved; after `scale_increment_period` finite steps it doubles."""
import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.model_inputs import he_weights, synthetic_batch

pytestmark = pytest.mark.gpu


def f16r(t):
    return t.to(torch.float16).to(t.dtype)


def _graph(builder, H, W):
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = builder(image, keep)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    return image, labels, keep, logits, loss, train


def _weights(shapes, seed):
    w = he_weights(shapes, seed)
    rng = np.random.default_rng(seed + 1)
    for k in w:
        if k.endswith("gamma"):
            w[k] = (1.0 + 0.1 * rng.standard_normal(w[k].shape)).astype(np.float32)
    return w


@pytest.mark.parametrize("model", ["deeplab", "fcn"])
def test_f16_train_step_vs_oracle(dev, model):
    torch.set_num_threads(16)
    H, W, N = 64, 96, 2
    if model == "deeplab":
        builder, shapes, fwd = (lambda im, kp: DeepLabASPP(im, kp, 2)), M.deeplab_param_shapes(3, 2), M.deeplab_forward
    else:
        builder, shapes, fwd = (lambda im, kp: FCN(im, kp, 2).create()), M.fcn_param_shapes(3, 2), M.fcn_forward
    image, labels, keep, logits, loss, train = _graph(builder, H, W)
    weights = _weights(shapes, 91)
    img, lab = synthetic_batch(N, H, W, 92)
    sess = tf.Session(compute_dtype="f16")
    assert sess.dynamic_scale and sess.loss_scale == 2.0 ** 15
    sess.run(tf.global_variables_initializer())
    for k, v in weights.items():
        sess.assign(k, v)
    S = sess.loss_scale
    lg, lo, _ = sess.run([logits, loss, train], feed_dict={image: img, labels: lab, keep: 1.0})
    assert sess.skipped_steps == 0 and sess.store.step == 1
    wr = {k: (f16r(torch.from_numpy(v)) if v.ndim == 4 else torch.from_numpy(v)).requires_grad_(True)
          for k, v in weights.items()}
    _, rl = fwd(wr, torch.from_numpy(img), quant=f16r)
    rloss = T.mean_softmax_xent(rl, T.one_hot(torch.from_numpy(lab).long(), 2, torch.float32))
    rloss.backward()
    rl = rl.detach().numpy()
    assert np.abs(lg - rl).max() / np.abs(rl).max() < 1e-2
    assert abs(float(lo) - rloss.item()) <= 5e-3 * max(1.0, abs(rloss.item()))
    stats = []
    for k, v in wr.items():
        g = sess.store.grad(k).cpu().numpy().reshape(-1).astype(np.float64) / S
        r = v.grad.numpy().reshape(-1).astype(np.float64)
        cos = g @ r / max(np.linalg.norm(g) * np.linalg.norm(r), 1e-300)
        stats.append((cos, np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-300), k))
    print(sorted(stats)[:4])
    assert min(s[0] for s in stats) >= 0.98, sorted(stats)[:3]
    assert np.median([s[1] for s in stats]) <= 0.05


def test_dynamic_loss_scale_skips_overflow_and_grows(dev):
    H, W, N = 64, 96, 2
    image, labels, keep, logits, loss, train = _graph(lambda im, kp: DeepLabASPP(im, kp, 2), H, W)
    weights = _weights(M.deeplab_param_shapes(3, 2), 93)
    img, lab = synthetic_batch(N, H, W, 94)
    feed = {image: img, labels: lab, keep: 1.0}
    sess = tf.Session(compute_dtype="f16")
    sess.run(tf.global_variables_initializer())
    for k, v in weights.items():
        sess.assign(k, v)
    sess.loss_scale = 2.0 ** 40            # the scaled loss gradient overflows fp16
    p0 = sess.store.params.clone()
    sess.run(train, feed_dict=feed)
    assert sess.skipped_steps == 1 and sess.store.step == 0
    assert sess.loss_scale == 2.0 ** 39
    assert torch.equal(sess.store.params, p0)
    assert float(sess.store.m.abs().max()) == 0.0
    # back to a representable scale: steps apply, and the scale doubles every period
    sess.loss_scale = 2.0 ** 12
    sess.scale_increment_period = 2
    for _ in range(2):
        sess.run(train, feed_dict=feed)
    assert sess.store.step == 2 and sess.skipped_steps == 1
    assert sess.loss_scale == 2.0 ** 13
    assert not torch.equal(sess.store.params, p0)
    assert torch.isfinite(sess.store.params).all()
