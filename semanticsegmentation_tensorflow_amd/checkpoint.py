"""tf.train.Saver / get_checkpoint_state / latest_checkpoint for the
reference's save-and-resume flow (Network/model/FCN.py:370-378,
Network/main.py:143-153 and :190).

Checkpoints carry TF1 Saver names: every variable under its graph name
(`conv1_1/weights`, `batch_normalization_3/gamma`, ...), the Adam slots as
`<name>/Adam` and `<name>/Adam_1`, and the optimizer's `beta1_power` /
`beta2_power` (beta^t, as TF keeps them).  Filters keep TF's layouts (HWIO;
conv2d_transpose [kh, kw, out, in]); the packed compute copies are rebuilt on
the next step.  Storage is a NumPy .npz (no pickle) per checkpoint plus TF's
`checkpoint` index file, so `get_checkpoint_state(dir).model_checkpoint_path`
works as in the reference.  Reading TF's own tensor-bundle files needs
TensorFlow, which is not part of this path.
"""
from __future__ import annotations

import os
import re

import numpy as np

BETA1, BETA2 = 0.9, 0.999


def _npz(path):
    return path if path.endswith(".npz") else path + ".npz"


class Saver:
    def __init__(self, var_list=None, max_to_keep=5):
        self.var_list = var_list
        self.max_to_keep = max_to_keep
        self._kept = []

    def _names(self, sess):
        store = sess._ensure_store()
        if self.var_list is None:
            return [v.var_name for v in store.vars]
        return [v.var_name for v in self.var_list]

    def save(self, sess, save_path, global_step=None):
        store = sess._ensure_store()
        path = save_path if global_step is None else f"{save_path}-{int(global_step)}"
        sd = store.state_dict()
        names = set(self._names(sess))
        out = {}
        for k, v in sd.items():
            base = re.sub(r"/Adam(_1)?$", "", k)
            if k == "beta_step":
                continue
            if base in names:
                out[k] = np.ascontiguousarray(v)
        t = int(sd["beta_step"])
        out["beta1_power"] = np.float32(BETA1 ** t)
        out["beta2_power"] = np.float32(BETA2 ** t)
        out["global_step"] = np.int64(t)
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        np.savez(_npz(path), **out)
        self._kept.append(path)
        while self.max_to_keep and len(self._kept) > self.max_to_keep:
            old = self._kept.pop(0)
            if os.path.exists(_npz(old)):
                os.remove(_npz(old))
        with open(os.path.join(d, "checkpoint"), "w") as f:
            f.write(f'model_checkpoint_path: "{os.path.basename(path)}"\n')
            for p in self._kept:
                f.write(f'all_model_checkpoint_paths: "{os.path.basename(p)}"\n')
        return path

    def restore(self, sess, save_path):
        store = sess._ensure_store()
        with np.load(_npz(save_path), allow_pickle=False) as z:
            d = {k: z[k] for k in z.files}
        missing = [n for n in self._names(sess) if n not in d]
        if missing:
            raise ValueError(f"checkpoint {save_path} lacks variables {missing[:5]}")
        if "global_step" in d:
            d["beta_step"] = int(d["global_step"])
        elif "beta1_power" in d:
            d["beta_step"] = int(round(np.log(float(d["beta1_power"])) / np.log(BETA1)))
        store.load_state_dict(d)


class CheckpointState:
    def __init__(self, model_checkpoint_path, all_model_checkpoint_paths):
        self.model_checkpoint_path = model_checkpoint_path
        self.all_model_checkpoint_paths = all_model_checkpoint_paths


def get_checkpoint_state(checkpoint_dir):
    """Parse TF's `checkpoint` index file; None when absent (as TF)."""
    f = os.path.join(checkpoint_dir, "checkpoint")
    if not os.path.exists(f):
        return None
    last, allp = None, []
    for line in open(f):
        m = re.match(r'\s*(model_checkpoint_path|all_model_checkpoint_paths):\s*"(.*)"', line)
        if not m:
            continue
        p = m.group(2)
        p = p if os.path.isabs(p) else os.path.join(checkpoint_dir, p)
        if m.group(1) == "model_checkpoint_path":
            last = p
        else:
            allp.append(p)
    return CheckpointState(last, allp) if last else None


def latest_checkpoint(checkpoint_dir):
    st = get_checkpoint_state(checkpoint_dir)
    return st.model_checkpoint_path if st else None
