"""tf.train.Saver round trip with TF1 names (host logic; the Session runs
against the recording stub of tests/test_session_dryrun.py, so no GPU)."""
import os

import numpy as np

from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import session as S
from semanticsegmentation_tensorflow_amd import tf
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
    with np.load(path + ".npz") as z:
        names = set(z.files)
        assert {"conv1_1/weights", "conv1_1/weights/Adam", "conv1_1/weights/Adam_1", "beta1_power",
                "beta2_power"} <= names
        assert z["conv6/weights"].shape == (7, 7, 512, 4096)            # HWIO, as TF
        assert z["conv_t3/weights"].shape == (16, 16, 2, 256)           # [kh, kw, out, in]
        assert abs(float(z["beta1_power"]) - 0.9 ** 7) < 1e-7
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
    assert sorted(os.listdir(tmp_path / "k")) == ["checkpoint", "m-2.npz", "m-3.npz"]
    assert len(tf.train.get_checkpoint_state(str(tmp_path / "k")).all_model_checkpoint_paths) == 2
