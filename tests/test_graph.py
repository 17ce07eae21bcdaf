"""Host-side graph logic (no GPU): variable creation / AUTO_REUSE / shapes
match the reference FCN and FC-DenseNet exactly."""
import numpy as np
import pytest

from oracle import models as M
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcn import FCN
from semanticsegmentation_tensorflow_amd.variables import init_value


def test_fcn_variables_match_reference():
    G.reset_default_graph()
    x = tf.placeholder(tf.float32, [None, 160, 576, 3])
    kp = tf.placeholder(tf.float32)
    fcn = FCN(x, kp, 2)             # __init__ builds once ...
    pred, logits = fcn.create()     # ... and main() builds again (FCN.py:47, :319)
    vs = {v.var_name: tuple(v.shape) for v in tf.global_variables()}
    ref = M.fcn_param_shapes(3, 2)
    assert vs == {k: tuple(s) for k, s in ref.items()}
    assert len(vs) == 40
    assert sum(int(np.prod(s)) for s in vs.values()) == 138_873_924
    assert logits.shape[1:] == (160, 576, 2)
    assert pred.shape[-1] == 1


def test_auto_reuse_shape_mismatch_raises():
    G.reset_default_graph()
    with tf.variable_scope("a", reuse=tf.AUTO_REUSE):
        v1 = tf.get_variable("w", [3, 3])
    with tf.variable_scope("a", reuse=tf.AUTO_REUSE):
        v2 = tf.get_variable("w", [3, 3])
        with pytest.raises(ValueError):
            tf.get_variable("w", [4, 3])
    assert v1 is v2


def test_initializers_deterministic_and_scaled():
    G.reset_default_graph()
    with tf.variable_scope("conv6"):
        w = tf.get_variable("weights", [7, 7, 512, 64], initializer=tf.random_normal_initializer(0.0, 0.01))
        b = tf.get_variable("biases", [64], initializer=tf.constant_initializer(0.0))
    a1, a2 = init_value(w, 0), init_value(w, 0)
    assert np.array_equal(a1, a2)
    assert not np.array_equal(a1, init_value(w, 1))
    assert abs(a1.std() - 0.01) < 2e-4 and abs(a1.mean()) < 2e-4
    assert not init_value(b, 0).any()


def test_shape_helpers_resolve_tf_shape_stack():
    G.reset_default_graph()
    x = tf.placeholder(tf.float32, [None, 64, 96, 3])
    s = tf.shape(x)
    st = tf.stack([s[0], s[1], s[2], 2])
    assert G.resolve_shape(st, lambda t: (5, 64, 96, 3)) == (5, 64, 96, 2)
    assert G.resolve_shape(tf.shape(x), lambda t: (5, 64, 96, 3)) == (5, 64, 96, 3)


def test_fcdensenet_variables_match_reference():
    """FCDenseNet.py:83-163 builds 250 variables (125 bias-free convs incl. 5
    transposed, 123 BN gamma/beta pairs counted separately) with the
    reference's auto-generated batch_normalization names."""
    from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
    G.reset_default_graph()
    x = tf.placeholder(tf.float32, [None, 64, 96, 3])
    kp = tf.placeholder(tf.float32)
    pred, logits = FCDenseNet(x, kp, 2)
    vs = {v.var_name: tuple(v.shape) for v in tf.trainable_variables()}
    ref = {k: tuple(s) for k, s in M.fcdensenet_param_shapes(3, 2).items()}
    assert vs == ref
    assert logits.shape[1:] == (64, 96, 2)
    assert pred.shape[-1] == 1
    # channel widths of the encoder skips (128/160/208/280/348/430)
    assert ref["transition_up1/weights"] == (4, 4, 348, 430)
    assert ref["transition_up5/weights"] == (4, 4, 128, 320)
    assert ref["final_conv/weights"] == (1, 1, 256, 2)


def test_deeplab_variables_match_oracle():
    """C5 DeepLab-style model: graph variables == the oracle's parameter table
    (VGG16 stack with biases, ASPP / projection BN gammas+betas, bias-free heads)."""
    from oracle import models as M
    from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 64, 96, 3])
    pred, logits = DeepLabASPP(image, 1.0, 2)
    got = {v.var_name: tuple(v.shape) for v in tf.trainable_variables()}
    assert got == {k: tuple(s) for k, s in M.deeplab_param_shapes(3, 2).items()}
    assert tuple(logits.shape) == (None, 64, 96, 2) or list(logits.shape)[1:] == [64, 96, 2]
