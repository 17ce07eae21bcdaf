"""Save / resume (Network/model/FCN.py:370-378): a session restored from a
checkpoint continues training bit-for-bit like the one that saved it."""
import numpy as np
import pytest

from oracle import models as M
from semanticsegmentation_tensorflow_amd import tf
from tests.model_inputs import he_weights, synthetic_batch
from tests.test_gpu_fcn import build_fcn

pytestmark = pytest.mark.gpu


def test_resume_is_bit_exact(dev, tmp_path):
    N, H, W = 2, 64, 96
    image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
    img, lab = synthetic_batch(N, H, W, 3)
    feed = {image: img, labels: lab, keep: 1.0}
    a = tf.Session(compute_dtype="bf16")
    a.run(tf.global_variables_initializer())
    for k, v in he_weights(M.fcn_param_shapes(3, 2), 2).items():
        a.assign(k, v)
    for _ in range(2):
        a.run(train_step, feed_dict=feed)
    saver = tf.train.Saver()
    path = saver.save(a, str(tmp_path / "model.ckpt"), global_step=2)
    a.run(train_step, feed_dict=feed)
    b = tf.Session(compute_dtype="bf16")
    b.run(tf.global_variables_initializer())
    saver.restore(b, tf.train.get_checkpoint_state(str(tmp_path)).model_checkpoint_path)
    assert b.store.step == 2
    b.run(train_step, feed_dict=feed)
    for v in a.store.vars:
        assert np.array_equal(a.variable_value(v.var_name), b.variable_value(v.var_name)), v.var_name
    la, lb = a.run(loss, feed_dict=feed), b.run(loss, feed_dict=feed)
    assert la == lb
