"""Host-logic tests (no GPU, recording C-ABI stub) of the train-step surfaces
beyond `minimize`:

* the accumulate-then-apply template of Network/main.py:66-101 and
  Network/model/FCDenseNet.py:195-216 (`tf.Variable(tf.zeros_like(...),
  trainable=False)` accumulators, `zero_ops`, `assign_add(scalar_mul(const,
  g))` from `compute_gradients`, `apply_gradients` on the accumulators);
* `minimize(var_list=...)`: variables outside var_list get no filter gradient
  launch and no Adam update;
* `tf.Variable(0, trainable=False, name='global_step')` incremented by
  `minimize(global_step=...)`.
Numerics of the same flows: tests/test_gpu_train_api.py."""
import numpy as np
import torch

from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import session as S
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.test_session_dryrun import dry  # noqa: F401  (fixture)

H, W = 64, 96


def _fcn():
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = FCN(image, keep, 2).create()
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    feed = {image: np.zeros((2, H, W, 3), np.float32), labels: np.zeros((2, H, W), np.uint8), keep: 1.0}
    return loss, feed


def test_accumulate_template_plan(dry):  # noqa: F811
    loss, feed = _fcn()
    opt = tf.train.AdamOptimizer(1e-4)
    const = tf.constant(1 / 8 * 3)
    t_vars = tf.trainable_variables()
    accum = [tf.Variable(tf.zeros_like(t.initialized_value()), trainable=False) for t in t_vars]
    zero_ops = [a.assign(tf.zeros_like(a)) for a in accum]
    gvs = opt.compute_gradients(loss, t_vars)
    accum_ops = [accum[i].assign_add(tf.scalar_mul(const, gv[0])) for i, gv in enumerate(gvs)]
    train_step = opt.apply_gradients([(accum[i], gv[1]) for i, gv in enumerate(gvs)])
    assert len(tf.global_variables()) == 2 * len(t_vars)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    st = sess.store
    assert len(st.vars) == 40 and len(st.aux) == 40          # accumulators stay out of the flat buffers
    dry.calls.clear()
    sess.run(zero_ops)
    assert dry.calls == ["seg_fill"] * 40
    dry.calls.clear()
    sess.run(accum_ops, feed_dict=feed)
    c = dry.calls
    assert (c.count("seg_conv2d_fwd") + c.count("seg_conv2d_fwd_pool") + c.count("seg_conv2d_fwd_hwio")
            + c.count("seg_conv2d_fwd_relu_bits") == 17)
    # no optimizer in this run: every filter gradient is a plain launch
    assert c.count("seg_conv2d_bwd_filter") == 17 and "seg_conv2d_bwd_filter_adam" not in c
    assert "seg_adam_tf1_pack" not in c
    assert c.count("seg_axpy") == 40
    assert st.step == 0
    dry.calls.clear()
    sess.run(train_step, feed_dict=feed)
    c = dry.calls
    assert "seg_conv2d_fwd" not in c and "seg_conv2d_fwd_pool" not in c   # apply_gradients: no forward pass
    assert "seg_conv2d_fwd_hwio" not in c and "seg_conv2d_fwd_relu_bits" not in c
    assert c.count("seg_axpy") == 40 and c.count("seg_adam_tf1_pack") == 1
    assert st.step == 1


def test_apply_gradients_of_compute_gradients_is_minimize(dry):  # noqa: F811
    loss, feed = _fcn()
    opt = tf.train.AdamOptimizer(1e-4)
    gvs = opt.compute_gradients(loss)
    step = opt.apply_gradients([(tf.scalar_mul(9.0, g), v) for g, v in gvs])
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run(step, feed_dict=feed)
    c = dry.calls
    assert c.count("seg_conv2d_bwd_filter_adam") == 2 and c.count("seg_adam_tf1_pack") == 1
    plan = next(iter(sess.plans.values()))
    assert plan.train.attrs["grad_scale"] == 9.0


def test_minimize_var_list_skips_frozen_layer(dry):  # noqa: F811
    loss, feed = _fcn()
    frozen = {"conv3_2/weights", "conv3_2/biases", "conv6/weights"}
    var_list = [v for v in tf.trainable_variables() if v.var_name not in frozen]
    gstep = tf.Variable(0, trainable=False, name="global_step")
    train = tf.train.AdamOptimizer(1e-4).minimize(loss, global_step=gstep, var_list=var_list)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run(train, feed_dict=feed)
    c = dry.calls
    # conv3_2 gets no filter gradient; conv6's filter is frozen but its bias is
    # not, so it leaves the fused wgrad+Adam launch for a plain one (filter
    # gradient into a scratch sink, bias gradient summed by the same launch);
    # input gradients still flow to the trainable layers below
    assert c.count("seg_conv2d_bwd_filter") == 17 - 1 - 1
    assert c.count("seg_conv2d_bwd_filter_adam") == 1
    assert c.count("seg_conv2d_bwd_data") + c.count("seg_conv2d_bwd_data_bits") == 16
    (gk, plan), = sess._adam_groups.items()
    assert not (set(gk[1]) & frozen)
    assert plan.nsegs == len(var_list) - 1                 # conv7 filter updated in its fused launch
    assert float(sess.store.aux["global_step"]) == 1.0
    sess.run(train, feed_dict=feed)
    assert float(sess.store.aux["global_step"]) == 2.0


def test_deeplab_image_pooling_plan(dry):  # noqa: F811
    """C5's image-pooling ASPP branch (DeepLabv3Plus.py:215-225): one global
    average pool, its 1x1 -> HxW align_corners resize as a broadcast, and in
    backward the matching broadcast / spatial-sum pair (no scatter-add resize)."""
    from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
    G.reset_default_graph()
    Hh, Ww = 64, 96
    image = tf.placeholder(tf.float32, [None, Hh, Ww, 3])
    labels = tf.placeholder(tf.uint8, [None, Hh, Ww])
    pred, logits = DeepLabASPP(image, 1.0, 2)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run([train, loss], feed_dict={image: np.zeros((2, Hh, Ww, 3), np.float32),
                                       labels: np.zeros((2, Hh, Ww), np.uint8)})
    c = dry.calls
    assert c.count("seg_spatial_reduce") == 2          # GAP forward, resize-from-1x1 backward
    assert c.count("seg_spatial_broadcast") == 2       # resize-from-1x1 forward, GAP backward
    assert c.count("seg_resize_bilinear_fwd") == 1 and c.count("seg_resize_bilinear_bwd") == 1
    plan = next(iter(sess.plans.values()))
    gap = next(n for n in plan.nodes if n.kind == "GlobalAvgPool")
    assert plan.shapes[id(gap.output)] == (2, 1, 1, 512)
