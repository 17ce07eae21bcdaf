"""Train-step surfaces on the MI355X vs the CPU oracle (fp32 compute path):

* the accumulate-then-apply template (Network/main.py:66-101, :158-184;
  Network/model/FCDenseNet.py:195-216, :266-277): zero_ops, 3B runs of
  `accum += (3/B) * g`, one apply_gradients -> TF1 Adam on 9*g; equal to
  `minimize(loss, grad_scale=9)` and to the oracle's Adam on 9*g;
* K = 3 TF1-Adam train steps at keep_prob = 1 (tier 3): loss
  curve and parameter slices against the oracle's own 3-step trajectory;
* `minimize(var_list=...)` leaves a frozen mid-network layer bit-identical;
* the FCN driver's own 4-channel `merge` input (Network/model/FCN.py:225,
  :312) at its default training shape 160x576 (Network/model/FCN.py:24).

Tolerances: logits 1e-4 relative, gradients 2e-3 of each variable's max
|value| (fp32 accumulation order vs the float64 oracle, as
tests/test_gpu_fcn.py).  Parameters after Adam on the SAME gradient: 1e-6 +
1e-5 * max|p|.  Parameters after Adam on gradients from a different summation
order (another plan, or the float64 oracle): all but 1 % of the elements
within 2 % of lr per step, and none off by more than a full Adam step -- TF1
Adam moves an element whose gradient g is a near-cancelling sum by
lr_t * (1 - b1) * g / (sqrt(v) + eps), so a rounding difference in g that is
tiny against max|g| but comparable to eps = 1e-8 (or flips g's sign) changes
that element's update by up to a whole step while the rest agree to ~1e-6."""
import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.model_inputs import he_weights, synthetic_batch

pytestmark = pytest.mark.gpu
LR = 1e-4


def _fcn(H, W, cin=3):
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, shape=[None, H, W, cin], name="input_image")
    labels = tf.placeholder(tf.uint8, shape=[None, H, W], name="annotation")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    pred, logits = FCN(image, keep, 2).create()
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    return image, labels, keep, pred, logits, loss


def _session(weights):
    sess = tf.Session(compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    for k, v in weights.items():
        sess.assign(k, v)
    return sess


def _oracle_grads(weights, img, lab):
    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in weights.items()}
    _, logits = M.fcn_forward(p, torch.from_numpy(img).double())
    loss = T.mean_softmax_xent(logits, T.one_hot(torch.from_numpy(lab), 2))
    loss.backward()
    return logits.detach().numpy(), loss.item(), {k: v.grad for k, v in p.items()}


def _close_params(got, ref, what):
    err = np.abs(got - ref).max()
    assert err <= 1e-6 + 1e-5 * np.abs(ref).max(), f"{what}: {err:.3e}"


def _close_updates(got, ref, what, steps):
    d = np.abs(got - ref)
    frac = float((d > 2e-2 * LR * steps).mean())
    assert frac <= 1e-2, f"{what}: {frac:.2e} of the elements off by > 2% of lr per step"
    assert d.max() <= 3.5 * LR * steps, f"{what}: {d.max():.3e}"


def test_accumulate_template_is_adam_on_9g(dev):
    N, H, W, B = 2, 64, 96, 2
    image, labels, keep, pred, logits, loss = _fcn(H, W)
    opt = tf.train.AdamOptimizer(LR)
    const = tf.constant(1 / B * 3)                                   # Network/main.py:71
    t_vars = tf.trainable_variables()
    accum = [tf.Variable(tf.zeros_like(t.initialized_value()), trainable=False) for t in t_vars]
    zero_ops = [a.assign(tf.zeros_like(a)) for a in accum]
    gvs = opt.compute_gradients(loss, t_vars)
    accum_ops = [accum[i].assign_add(tf.scalar_mul(const, gv[0])) for i, gv in enumerate(gvs)]
    train_step = opt.apply_gradients([(accum[i], gv[1]) for i, gv in enumerate(gvs)])
    weights = he_weights(M.fcn_param_shapes(3, 2), 11)
    img, lab = synthetic_batch(N, H, W, 12)
    feed = {image: img, labels: lab, keep: 1.0}

    sess = _session(weights)
    for step in range(2):                                           # two batches, zeroed in between
        sess.run(zero_ops)
        for _ in range(3 * B):                                      # Network/main.py:168-170
            sess.run(accum_ops, feed_dict=feed)
        if step == 0:
            acc0 = [sess.store.aux[a.var_name].cpu().numpy() for a in accum]
        sess.run(train_step, feed_dict=feed)
        if step == 0:   # the parameters batch 2 accumulates its gradient at
            w1 = {k: sess.variable_value(k) for k in weights}
    assert sess.store.step == 2

    # the same two steps computed once per batch with grad_scale = 9: the
    # batch-2 accumulators hold 9x that plan's gradient (fp32 sums of six
    # 1.5 g terms vs one 9 g scale), and its parameters track
    step9 = tf.train.AdamOptimizer(LR).minimize(loss, grad_scale=9.0)
    ref = _session(weights)
    ref.store_fused_grads = True
    for step in range(2):
        ref.run(step9, feed_dict={image: img, labels: lab, keep: 1.0})
        if step == 0:    # same parameters as the first accumulation: 9 g vs sum of 6 x 1.5 g, tight
            for i, v in enumerate(t_vars):
                g9 = 9.0 * ref.store.grad(v.var_name).cpu().numpy()
                assert np.abs(acc0[i] - g9).max() <= 1e-5 * max(np.abs(g9).max(), 1e-30), v.var_name
    for i, v in enumerate(t_vars):
        _close_updates(sess.variable_value(v.var_name), ref.variable_value(v.var_name), v.var_name, 2)

    # the oracle: the batch-2 accumulators hold 9 * g at the device's step-1
    # parameters (its own trajectory drifts by TF1 Adam's 1/eps rounding gain).
    # fp32 vs float64: a pre-activation within rounding of 0 flips its ReLU
    # and moves a few gradient entries by ~1e-3 of the max -> L2 + tail bound
    _, _, g1 = _oracle_grads(w1, img, lab)
    for i, v in enumerate(t_vars):
        a = sess.store.aux[accum[i].var_name].cpu().numpy().astype(np.float64)
        gr = 9.0 * g1[v.var_name].numpy()
        rel = np.linalg.norm(a - gr) / max(np.linalg.norm(gr), 1e-300)
        tail = np.mean(np.abs(a - gr) > 2e-3 * max(np.abs(gr).max(), 1e-30))
        assert rel <= 2e-3 and tail <= 1e-3, (v.var_name, rel, tail)
    # and TF1 Adam on 9 * g for two steps, along the oracle's own trajectory
    adam = T.AdamTF1(lr=LR)
    w = {k: torch.from_numpy(v).double() for k, v in weights.items()}
    for step in range(2):
        _, _, g = _oracle_grads({k: v.numpy().astype(np.float32) for k, v in w.items()}, img, lab)
        w = adam.apply(w, {k: 9.0 * g[k] for k in w})
    for k in ["conv1_1/weights", "conv4_2/weights", "conv6/weights", "conv8/biases", "conv_t3/bias"]:
        _close_updates(sess.variable_value(k), w[k].numpy(), k, 2)


def test_three_adam_steps_track_the_oracle(dev):
    """SURVEY.md 4 tier 3: K = 3 train steps at keep_prob = 1, loss curve and
    parameter slices vs the oracle's own trajectory (each oracle step starts
    from the oracle's parameters, not the device's)."""
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss = _fcn(H, W)
    gstep = tf.Variable(0, trainable=False, name="global_step")
    train = tf.train.AdamOptimizer(LR).minimize(loss, global_step=gstep)
    weights = he_weights(M.fcn_param_shapes(3, 2), 21)
    img, lab = synthetic_batch(N, H, W, 22)
    sess = _session(weights)
    losses = [float(sess.run([train, loss], feed_dict={image: img, labels: lab, keep: 1.0})[1]) for _ in range(3)]
    assert float(sess.store.aux["global_step"]) == 3.0

    adam = T.AdamTF1(lr=LR)
    w = {k: torch.from_numpy(v).double() for k, v in weights.items()}
    ref_losses = []
    for _ in range(3):
        _, lo, g = _oracle_grads({k: v.numpy().astype(np.float32) for k, v in w.items()}, img, lab)
        ref_losses.append(lo)
        w = adam.apply(w, {k: g[k] for k in w})
    print("loss curve", losses, ref_losses)
    np.testing.assert_allclose(losses, ref_losses, rtol=1e-4)
    assert ref_losses[2] < ref_losses[0]
    for k in ["conv1_1/weights", "conv3_3/weights", "conv5_3/biases", "conv6/weights", "conv7/weights",
              "conv_t1/weights", "conv_t3/weights"]:
        got, ref = sess.variable_value(k), w[k].numpy()
        _close_updates(got, ref, k, 3)


def test_var_list_freezes_a_mid_network_layer(dev):
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss = _fcn(H, W)
    frozen = {"conv3_2/weights", "conv3_2/biases", "conv6/weights"}
    var_list = [v for v in tf.trainable_variables() if v.var_name not in frozen]
    train = tf.train.AdamOptimizer(LR).minimize(loss, var_list=var_list)
    weights = he_weights(M.fcn_param_shapes(3, 2), 31)
    img, lab = synthetic_batch(N, H, W, 32)
    for dtype in ("f32", "bf16"):
        sess = tf.Session(compute_dtype=dtype)
        sess.run(tf.global_variables_initializer())
        for k, v in weights.items():
            sess.assign(k, v)
        for _ in range(2):
            sess.run(train, feed_dict={image: img, labels: lab, keep: 1.0})
        for k in frozen:
            assert np.array_equal(sess.variable_value(k), weights[k]), (dtype, k)
        for k in ("conv3_1/weights", "conv3_3/weights", "conv6/biases", "conv7/weights"):
            assert not np.array_equal(sess.variable_value(k), weights[k]), (dtype, k)
    # fp32: the updated variables take TF1 Adam on their gradient (tight: the
    # same gradient), and that gradient is the oracle's
    _, _, g = _oracle_grads(weights, img, lab)
    sess = _session(weights)
    sess.store_fused_grads = True
    sess.run(train, feed_dict={image: img, labels: lab, keep: 1.0})
    dg = {k: sess.store.grad(k).cpu().numpy() for k in weights if k not in frozen}
    w = T.AdamTF1(lr=LR).apply({k: torch.from_numpy(weights[k]).double() for k in dg},
                               {k: torch.from_numpy(v).double() for k, v in dg.items()})
    for k in ("conv3_1/weights", "conv3_3/weights", "conv6/biases", "conv7/weights", "conv_t2/weights"):
        _close_params(sess.variable_value(k), w[k].numpy(), k)
        gr = g[k].numpy()
        assert np.abs(dg[k] - gr).max() <= 2e-3 * np.abs(gr).max(), k


def test_fcn_merge_rgba_input_at_160x576(dev):
    """FCN.py's own driver feeds 4-channel `merge` images (FCN.py:225, :312) at
    IMAGE_SHAPE_KITTI = (160, 576) (FCN.py:24)."""
    N, H, W = 1, 160, 576
    image, labels, keep, pred, logits, loss = _fcn(H, W, cin=4)
    train = tf.train.AdamOptimizer(LR).minimize(loss)
    shapes = M.fcn_param_shapes(4, 2)
    assert {v.var_name: tuple(v.shape) for v in tf.trainable_variables()} == {k: tuple(s) for k, s in shapes.items()}
    weights = he_weights(shapes, 41)
    rng = np.random.default_rng(42)
    img = rng.integers(0, 256, size=(N, H, W, 4)).astype(np.float32)
    _, lab = synthetic_batch(N, H, W, 43)
    sess = _session(weights)
    out_logits, out_loss, _ = sess.run([logits, loss, train], feed_dict={image: img, labels: lab, keep: 1.0})
    r_logits, r_loss, g = _oracle_grads(weights, img, lab)
    e = np.abs(out_logits - r_logits).max() / np.abs(r_logits).max()
    assert e < 1e-4, e
    assert abs(float(out_loss) - r_loss) < 1e-4 * max(1.0, abs(r_loss))
    for k, gr in g.items():
        gr = gr.numpy()
        got = sess.store.grad(k).cpu().numpy()
        assert np.abs(got - gr).max() < 2e-3 * max(np.abs(gr).max(), 1e-30), k
