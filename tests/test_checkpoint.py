"""tf.train.Saver round trip with TF1 names (host logic; the Session runs
against the recording stub of tests/test_session_dryrun.py, so no GPU)."""
import os

import numpy as np

from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import session as S
from semanticsegmentation_tensorflow_amd import tf, tf_bundle
from semanticsegmentation_tensorflow_amd.fcn import FCN
from tests.test_session_dryrun import dry  # noqa: F401  (fixture)

import torch


def test_saver_round_trip_tf_names(dry, tmp_path):  # noqa: F811
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 64, 96, 3])
    FCN(image, 1.0, 2).create()
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    st = sess.store
    st.step = 7
    st.adam_m("conv6/weights").fill_(0.25)
    st.adam_v("conv_t3/bias").fill_(0.5)
    saver = tf.train.Saver()
    path = saver.save(sess, str(tmp_path / "model" / "model.ckpt"), global_step=7)
    assert path.endswith("model.ckpt-7")
    state = tf.train.get_checkpoint_state(str(tmp_path / "model"))
    assert state.model_checkpoint_path == path
    assert tf.train.latest_checkpoint(str(tmp_path / "model")) == path
    # TF's V2 format: <prefix>.index (SSTable) + <prefix>.data-00000-of-00001
    assert os.path.exists(path + ".index") and os.path.exists(path + ".data-00000-of-00001")
    index = tf_bundle.read_index(path)
    assert {"conv1_1/weights", "conv1_1/weights/Adam", "conv1_1/weights/Adam_1", "beta1_power",
            "beta2_power"} <= set(index)
    assert index["conv6/weights"]["shape"] == (7, 7, 512, 4096)            # HWIO, as TF
    assert index["conv6/weights"]["dtype"] == 1                            # DT_FLOAT
    assert index["conv_t3/weights"]["shape"] == (16, 16, 2, 256)           # [kh, kw, out, in]
    z = tf_bundle.read_bundle(path, ["beta1_power", "conv_t3/bias/Adam_1"])
    # TF1 Adam: beta1_power starts at beta1 and is multiplied after every
    # update, so after 7 steps it holds 0.9^8
    assert abs(float(z["beta1_power"]) - 0.9 ** 8) < 1e-7
    assert float(z["conv_t3/bias/Adam_1"][0]) == 0.5
    ref = {v.var_name: st.read(v.var_name) for v in st.vars}
    # clobber and restore
    sess.run(tf.global_variables_initializer())
    st.params.add_(1.0)
    st.m.zero_()
    st.step = 0
    saver.restore(sess, state.model_checkpoint_path)
    assert st.step == 7
    for k, v in ref.items():
        assert np.array_equal(st.read(k), v), k
    assert float(st.adam_m("conv6/weights")[0, 0, 0, 0]) == 0.25
    assert float(st.adam_v("conv_t3/bias")[0]) == 0.5
    # max_to_keep prunes the oldest files and the index lists the kept ones
    s2 = tf.train.Saver(max_to_keep=2)
    for step in (1, 2, 3):
        s2.save(sess, str(tmp_path / "k" / "m"), global_step=step)
    assert sorted(os.listdir(tmp_path / "k")) == ["checkpoint", "m-2.data-00000-of-00001", "m-2.index",
                                                  "m-3.data-00000-of-00001", "m-3.index"]
    assert len(tf.train.get_checkpoint_state(str(tmp_path / "k")).all_model_checkpoint_paths) == 2


def test_saver_global_step_variable_and_bn_stats(dry, tmp_path):  # noqa: F811
    """FCDenseNet.py:247, :285: `global_step = tf.Variable(0, trainable=False,
    name='global_step')` passed to save(); tf.global_variables() includes the
    BN moving statistics, saved under TF's names."""
    from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 64, 96, 3])
    FCDenseNet(image, 1.0, 2)
    gstep = tf.Variable(0, trainable=False, name="global_step")
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    sess.assign("global_step", 12)
    saver = tf.train.Saver(tf.global_variables())
    path = saver.save(sess, str(tmp_path / "FCHarDNet.ckpt"), global_step=gstep)
    assert path.endswith("FCHarDNet.ckpt-12")
    index = tf_bundle.read_index(path)
    assert index["global_step"]["dtype"] == 9 and index["global_step"]["shape"] == ()      # DT_INT64 scalar
    assert "batch_normalization/moving_mean" in index and "batch_normalization_122/moving_variance" in index
    z = tf_bundle.read_bundle(path, ["global_step", "batch_normalization/moving_variance"])
    assert int(z["global_step"]) == 12
    assert np.all(z["batch_normalization/moving_variance"] == 1.0)
    sess.assign("global_step", 0)
    saver.restore(sess, path)
    assert float(sess.variable_value("global_step")) == 12.0


def test_saver_beta_powers_at_step0_and_large_steps(dry, tmp_path):  # noqa: F811
    """a save before the first update writes TF's initial
    beta1_power = 0.9 (not 1.0, which makes TF's lr_t 0/0); the step is
    recovered from beta2_power where 0.9^(t+1) has gone denormal; global_step
    round-trips as an int64 beyond float32's 2^24."""
    from semanticsegmentation_tensorflow_amd import checkpoint as C
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 32, 32, 3])
    FCN(image, 1.0, 2).create()
    gstep = tf.Variable(0, trainable=False, name="global_step")
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    saver = tf.train.Saver(tf.global_variables())
    p0 = saver.save(sess, str(tmp_path / "a" / "m"))
    z = tf_bundle.read_bundle(p0, ["beta1_power", "beta2_power"])
    assert float(z["beta1_power"]) == np.float32(0.9) and float(z["beta2_power"]) == np.float32(0.999)
    sess.store.step = 5
    saver.restore(sess, p0)
    assert sess.store.step == 0
    big = 2 ** 24 + 3
    sess.assign("global_step", big)
    sess.store.step = 2000
    p1 = saver.save(sess, str(tmp_path / "b" / "m"), global_step=gstep)
    assert p1.endswith(f"m-{big}")
    sess.assign("global_step", 0)
    sess.store.step = 0
    saver.restore(sess, p1)
    assert sess.store.step == 2000
    assert int(sess.variable_value("global_step")) == big
    # TF-written powers: 0.9^(t+1) denormal / zero, 0.999^(t+1) still normal
    assert C._adam_step({"beta1_power": np.float32(0.0), "beta2_power": np.float32(0.999 ** 5001)}) == 5000
    assert C._adam_step({}) == 0


def test_adam_step_past_float32_range(dry, tmp_path):  # noqa: F811
    """a run of the reference's length (MAX_ITERATION = 100001)
    leaves beta2_power = 0.999^(t+1) denormal (t ~ 87k-103k) or 0 (beyond);
    restore still recovers the step (denormal: an estimate, bias correction
    is 1 to float32 precision there), falling back to global_step or the
    underflow step instead of refusing the checkpoint."""
    from semanticsegmentation_tensorflow_amd import checkpoint as C
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 32, 32, 3])
    FCN(image, 1.0, 2).create()
    gstep = tf.Variable(0, trainable=False, name="global_step")
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    saver = tf.train.Saver(tf.global_variables())
    for t, gs in ((100000, 100000), (250000, 250000), (250000, 0)):
        sess.store.step = t
        sess.assign("global_step", gs)
        p = saver.save(sess, str(tmp_path / f"m{t}_{gs}" / "m"))
        z = tf_bundle.read_bundle(p, ["beta2_power"])
        assert float(z["beta2_power"]) == np.float32(0.999 ** (t + 1))
        sess.store.step = 0
        saver.restore(sess, p)
        if t == 100000:                 # denormal beta2_power: within its resolution
            assert abs(sess.store.step - t) <= 50, sess.store.step
        elif gs:
            assert sess.store.step == gs
        else:
            assert sess.store.step == C._UNDERFLOW_STEP
    assert np.float32(0.999 ** C._UNDERFLOW_STEP) == 0 and np.float32(0.999 ** (C._UNDERFLOW_STEP - 900)) > 0
    # legacy .npz convention (beta^t): no off-by-one
    assert C._adam_step({"beta2_power": np.float32(0.999 ** 7)}, offset=0) == 7
