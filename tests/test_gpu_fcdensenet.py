"""FC-DenseNet ("U-Net", config C3) parity: Session (HIP path) vs the CPU
oracle restatement of Network/model/FCDenseNet.py:23-163 on identical inputs
and weights.

Tolerances: fp32 compute path -- logits / loss within 1e-4 relative; every
one of the 250 gradients within 5e-3 relative of its max |value| (fp32
accumulation order vs the fp64 oracle through ~60 pre-activation layers and 64
concats).  bf16 path: runs, finite, loss decreases with dropout on.
"""
import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import tf1_ops as tf_ref
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
from tests.model_inputs import densenet_weights, synthetic_batch

pytestmark = pytest.mark.gpu


def build(H, W):
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, shape=[None, H, W, 3], name="input_image")
    labels = tf.placeholder(tf.uint8, shape=[None, H, W], name="annotation")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    pred, logits = FCDenseNet(image, keep, 2)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train_step = tf.train.AdamOptimizer(1e-4).minimize(loss)
    return image, labels, keep, pred, logits, loss, train_step


@pytest.mark.parametrize("alias", [True, False], ids=["concat-views", "concat-copies"])
def test_fcdensenet_logits_grads_adam_f32(dev, alias):
    """alias: DenseBlock concats as channel views of one buffer (default) or
    as copies."""
    N, H, W = 1, 64, 96
    image, labels, keep, pred, logits, loss, train_step = build(H, W)
    shapes = M.fcdensenet_param_shapes(3, 2)
    assert {v.var_name for v in tf.trainable_variables()} == set(shapes)
    weights = densenet_weights(shapes, 7)
    img, lab = synthetic_batch(N, H, W, 8)

    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in weights.items()}
    r_pred, r_logits = M.fcdensenet_forward(p, torch.from_numpy(img).double())
    r_loss = tf_ref.mean_softmax_xent(r_logits, tf_ref.one_hot(torch.from_numpy(lab), 2))
    r_loss.backward()
    r_logits = r_logits.detach().numpy()

    sess = tf.Session(compute_dtype="f32")
    sess.alias_concat = alias
    sess.run(tf.global_variables_initializer())
    for k, v in weights.items():
        sess.assign(k, v)
    out_pred, out_logits, out_loss, _ = sess.run(
        [pred, logits, loss, train_step], feed_dict={image: img, labels: lab, keep: 1.0})
    torch.cuda.synchronize()

    e_log = np.abs(out_logits - r_logits).max() / np.abs(r_logits).max()
    assert e_log < 1e-4, f"logits rel err {e_log:.3e}"
    assert abs(out_loss - r_loss.item()) <= 1e-4 * max(1.0, abs(r_loss.item()))
    assert (out_pred == r_pred.numpy()).mean() > 0.999
    worst = []
    for k, t in p.items():
        gref = t.grad.numpy()
        gg = sess.store.grad(k).cpu().numpy()
        e = np.abs(gg - gref).max() / max(np.abs(gref).max(), 1e-30)
        worst.append((e, k))
        assert e < 5e-3, f"grad {k} max-rel err {e:.3e}"
    print("worst grads", sorted(worst)[-3:])
    # one TF1 Adam step on every variable (conv, tconv and BN)
    opt = tf_ref.AdamTF1(lr=1e-4)
    upd = opt.apply({k: torch.from_numpy(v).double() for k, v in weights.items()},
                    {k: torch.from_numpy(sess.store.grad(k).cpu().numpy()).double() for k in weights})
    for k in ["dense_init/weights", "transition_up1/weights", "batch_normalization/gamma", "final_conv/weights"]:
        got = sess.variable_value(k)
        ref = upd[k].numpy()
        assert np.abs(got - ref).max() <= 1e-6 + 1e-5 * np.abs(ref).max(), k


def test_fcdensenet_bf16_dropout_trains(dev):
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss, train_step = build(H, W)
    sess = tf.Session(compute_dtype="bf16", seed=5)
    sess.run(tf.global_variables_initializer())
    for k, v in densenet_weights(M.fcdensenet_param_shapes(3, 2), 9).items():
        sess.assign(k, v)
    img, lab = synthetic_batch(N, H, W, 10)
    losses = []
    for _ in range(6):
        _, l = sess.run([train_step, loss], feed_dict={image: img, labels: lab, keep: 0.8})
        losses.append(float(l))
    assert all(np.isfinite(losses))
    assert losses[-1] < losses[0], losses


def test_fcdensenet_bf16_deferred_bn_finish_bit_identical(dev):
    """The step's dgamma / dbeta finished together at the end of backward
    (Session.defer_bn_finish: one segment table, two launches) equal the
    per-launch finishes bit for bit -- every gradient and the Adam step, at
    keep_prob 0.2 (the folded BN backwards of both the 1x1 and the growth
    convs)."""
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss, train_step = build(H, W)
    weights = densenet_weights(M.fcdensenet_param_shapes(3, 2), 11, keep_prob=0.2)
    img, lab = synthetic_batch(N, H, W, 12)
    out = []
    for defer in (True, False):
        sess = tf.Session(compute_dtype="bf16", seed=3)
        sess.defer_bn_finish = defer
        sess.run(tf.global_variables_initializer())
        for k, v in weights.items():
            sess.assign(k, v)
        sess.run(train_step, feed_dict={image: img, labels: lab, keep: 0.2})
        torch.cuda.synchronize()
        out.append({k: (sess.store.grad(k).cpu().clone(), torch.from_numpy(sess.variable_value(k)))
                    for k in weights})
    a, b = out
    gammas = [k for k in a if k.endswith("gamma")]
    assert len(gammas) >= 100
    for k in a:
        assert torch.equal(a[k][0], b[k][0]), k
        assert torch.equal(a[k][1], b[k][1]), k
