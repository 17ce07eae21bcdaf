"""Eval path (softmax > 0.5 road mask, Network/utils/utils.py:43-89), the GPU
mIoU evaluator, and ResizeBilinear inside a trained graph (forward + gradient)
-- all through the HIP C-ABI, against the CPU oracle.

Tolerances: fp32 path; softmax 1e-5 absolute; mIoU bit-exact vs a confusion
matrix counted on the host from the same class map; ResizeBilinear graph
logits 1e-4 relative, gradients 2e-3 relative (of max |grad|)."""
import numpy as np
import pytest
import torch

from oracle import models as M
from oracle import tf1_ops as tf_ref
from semanticsegmentation_tensorflow_amd import evaluate as E
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.model_inputs import he_weights, synthetic_batch

pytestmark = pytest.mark.gpu


def test_softmax_mask_and_miou(dev):
    N, H, W = 3, 64, 96
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, H, W, 3], name="input_image")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    pred, logits = FCN(image, keep, 2).create()
    sm = tf.nn.softmax(logits)
    sess = tf.Session(compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    weights = he_weights(M.fcn_param_shapes(3, 2), 3)
    for k, v in weights.items():
        sess.assign(k, v)
    img, lab = synthetic_batch(N, H, W, 7)
    lg, prob, pr = sess.run([logits, sm, pred], feed_dict={image: img, keep: 1.0})
    ref = torch.softmax(torch.from_numpy(lg).double(), dim=-1).numpy()
    assert np.abs(prob - ref).max() < 1e-5
    # road mask exactly where p(road) > 0.5, same class map as argmax (2 classes)
    outs = list(E.gen_test_output(sess, sm, keep, image, img, (H, W)))
    assert len(outs) == N
    mask = outs[0][1]
    assert mask.shape == (H, W, 4)
    assert np.array_equal(mask[..., 1] == 255, prob[0, ..., 1] > 0.5)
    # mIoU on the device == host confusion of the same prediction
    miou, iou, conf = E.mean_iou(sess, pred, image, keep, img, lab, 2, batch=2)
    host = np.zeros((2, 2), np.int64)
    np.add.at(host, (lab.reshape(-1).astype(np.int64), pr.reshape(-1)), 1)
    assert np.array_equal(conf, host)
    assert abs(miou - E.confusion_to_iou(host)[0]) < 1e-12
    # masked to a valid region (375x1242-style padding)
    m = E.MeanIoU(2, dev, valid_hw=(50, 80))
    m.update(torch.as_tensor(pr).to(dev), torch.as_tensor(lab).to(dev))
    host_v = np.zeros((2, 2), np.int64)
    np.add.at(host_v, (lab[:, :50, :80].reshape(-1).astype(np.int64), pr[:, :50, :80, 0].reshape(-1)), 1)
    assert np.array_equal(m.confusion(), host_v)


def test_resize_bilinear_in_training_graph(dev):
    """conv -> Resize_Bilinear (align_corners, utils.py:329) x2 -> conv -> xent:
    logits and all gradients vs the oracle."""
    N, H, W, C = 2, 12, 20, 16
    G.reset_default_graph()
    x = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, 2 * H, 2 * W])
    with tf.variable_scope("a"):
        wa = tf.get_variable("w", [3, 3, 3, C], initializer=tf.random_normal_initializer(0.0, 0.2))
        ba = tf.get_variable("b", [C], initializer=tf.constant_initializer(0.1))
    with tf.variable_scope("b"):
        wb = tf.get_variable("w", [3, 3, C, 2], initializer=tf.random_normal_initializer(0.0, 0.2))
    h = tf.nn.relu(tf.nn.bias_add(tf.nn.conv2d(x, wa, [1, 1, 1, 1], "SAME"), ba))
    up = tf.image.resize_bilinear(h, [2 * H, 2 * W], align_corners=True)
    logits = tf.nn.conv2d(up, wb, [1, 1, 1, 1], "SAME")
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = tf.Session(compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    g = np.random.default_rng(3)
    xi = g.standard_normal((N, H, W, 3)).astype(np.float32)
    li = (g.random((N, 2 * H, 2 * W)) < 0.4).astype(np.uint8)
    p = {k: torch.from_numpy(sess.variable_value(k)).double().requires_grad_(True) for k in ("a/w", "a/b", "b/w")}
    lg, ls, _ = sess.run([logits, loss, train], feed_dict={x: xi, labels: li})
    hr = tf_ref.relu(tf_ref.bias_add(tf_ref.conv2d(torch.from_numpy(xi).double(), p["a/w"]), p["a/b"]))
    lr_ = tf_ref.conv2d(tf_ref.resize_bilinear(hr, (2 * H, 2 * W)), p["b/w"])
    l_ref = tf_ref.mean_softmax_xent(lr_, tf_ref.one_hot(torch.from_numpy(li), 2))
    l_ref.backward()
    assert np.abs(lg - lr_.detach().numpy()).max() <= 1e-4 * np.abs(lr_.detach().numpy()).max()
    assert abs(float(ls) - l_ref.item()) < 1e-5
    for k, v in p.items():
        gg = sess.store.grad(k).cpu().numpy()
        ref = v.grad.numpy()
        assert np.abs(gg - ref).max() <= 2e-3 * np.abs(ref).max(), k


def test_gen_test_output_files_and_uint8_feed(dev, tmp_path):
    """FCN.py:213-233 from a data folder: PNG -> GPU imresize (PIL-exact) ->
    softmax mask; the uint8 device batch feeds the float32 image placeholder
    exactly like the same values fed as float32."""
    from PIL import Image
    from oracle import augment as A
    H, W = 64, 96
    rng = np.random.default_rng(12)
    (tmp_path / "merge").mkdir()
    srcs = []
    for i in range(2):
        a = rng.integers(0, 256, (75, 124, 3), dtype=np.uint8)
        Image.fromarray(a, "RGB").save(tmp_path / "merge" / f"um_00000{i}.png")
        srcs.append(a)
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, H, W, 3], name="input_image")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    pred, logits = FCN(image, keep, 2).create()
    sm = tf.nn.softmax(logits)
    sess = tf.Session(compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    outs = list(E.gen_test_output_files(sess, sm, keep, image, str(tmp_path), (H, W)))
    assert [o[0] for o in outs] == ["um_000000.png", "um_000001.png"]
    for (name, mask, resized, _), a in zip(outs, srcs):
        want = A.imresize(a, (H, W))
        assert np.array_equal(resized, want)
        p32 = sess.run(sm, feed_dict={image: want[None].astype(np.float32), keep: 1.0})
        assert np.array_equal(mask[..., 1] == 255, p32[0, ..., 1] > 0.5)
        p8 = sess.run(sm, feed_dict={image: torch.from_numpy(want[None].copy()).to(dev), keep: 1.0})
        assert np.array_equal(p8, p32)
