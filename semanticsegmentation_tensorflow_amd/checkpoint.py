"""tf.train.Saver / get_checkpoint_state / latest_checkpoint for the
reference's save-and-resume flow (Network/model/FCN.py:370-378,
Network/main.py:143-153 and :190, Network/model/FCDenseNet.py:247-263, :285).

`Saver.save` writes TensorFlow's own V2 checkpoint format (tensor bundle:
`<prefix>.index` + `<prefix>.data-00000-of-00001`, tf_bundle.py) under TF1
Saver names:

* every graph variable under its name (`conv1_1/weights` HWIO,
  `conv_t1/weights` [kh, kw, out, in], `batch_normalization_3/gamma`,
  the BN `moving_mean` / `moving_variance`, non-trainable `tf.Variable`s such
  as the accumulate template's accumulators and `global_step`, int64);
* the Adam slots as `<name>/Adam` and `<name>/Adam_1`;
* the optimizer's `beta1_power` / `beta2_power` (beta^(t+1) after t updates,
  float32, as TF1's AdamOptimizer keeps them: created at beta, multiplied by
  beta after every update) -- the Adam step t is restored from these.

plus TF's `checkpoint` state file, so `get_checkpoint_state(dir)
.model_checkpoint_path` works as in the reference.  `restore` reads bundles
(ours or TensorFlow's: sliced / multi-shard / compressed ones are refused)
and the `.npz` checkpoints of earlier versions of this package.
"""
from __future__ import annotations

import math
import os
import re

import numpy as np
import torch.distributed as dist

from . import tf_bundle

BETA1, BETA2 = 0.9, 0.999


def _npz(path):
    return path if path.endswith(".npz") else path + ".npz"


def _adam_step(d, offset=1):
    """Adam t from TF's beta powers.  TF1's AdamOptimizer creates beta1_power =
    beta1 and multiplies it by beta1 after every update (_finish), so after t
    updates it holds beta1^(t+1) (float32; `offset` 1, or 0 for the beta^t
    convention of this package's legacy .npz checkpoints).  beta2_power =
    0.999^(t+1) is a normal float32 up to t ~ 87k and a denormal (fewer
    significant bits, still an estimate of t) up to t ~ 103k, so it decides
    while it is > 0; beta1_power is the fallback.  Both 0 (a run longer than
    ~103k steps, e.g. the reference's MAX_ITERATION = 100001 loops past their
    end): float32 underflow, so the bias correction sqrt(1-b2^t)/(1-b1^t) is 1
    to float32 precision -- `global_step` when the checkpoint holds one, else
    the first step at which beta2^t underflows.  No beta powers: step 0.
    Known limit: tensor-bundle checkpoints this package wrote before round 4
    (it stored beta^t there too, until the bundle writer switched to TF's
    beta^(t+1)) restore one Adam step low; resave them, or set the step from
    their `global_step` after restore."""
    b1 = float(d.get("beta1_power", BETA1))
    b2 = float(d.get("beta2_power", BETA2))
    if 0.0 < b2 < 1.0:
        return max(0, int(round(math.log(b2) / math.log(BETA2))) - offset)
    if 0.0 < b1 < 1.0:
        return max(0, int(round(math.log(b1) / math.log(BETA1))) - offset)
    if b1 == 0.0 and b2 == 0.0:
        if "global_step" in d and int(np.asarray(d["global_step"]).reshape(-1)[0]) > 0:
            return int(np.asarray(d["global_step"]).reshape(-1)[0])
        return _UNDERFLOW_STEP
    raise ValueError(f"checkpoint beta powers ({b1!r}, {b2!r}) do not encode an Adam step")


# first t with float32(0.999^t) == 0 (below half the smallest denormal, 2^-150)
_UNDERFLOW_STEP = int(math.ceil(-150 * math.log(2) / math.log(BETA2)))


class Saver:
    def __init__(self, var_list=None, max_to_keep=5):
        self.var_list = var_list
        self.max_to_keep = max_to_keep
        self._kept = []

    def _vars(self, sess):
        store = sess._ensure_store()
        if self.var_list is None:
            return list(store.all_vars)
        return list(self.var_list)

    def _global_step_value(self, sess, global_step):
        if global_step is None:
            return None
        if hasattr(global_step, "var_name"):          # tf.Variable(0, trainable=False, name='global_step')
            return int(round(float(sess.variable_value(global_step.var_name).reshape(-1)[0])))
        return int(global_step)

    def save(self, sess, save_path, global_step=None, write=None):
        """Write `save_path[-global_step]` and TF's `checkpoint` state file.

        Under data parallelism EVERY rank calls save: gathering the ZeRO-1
        Adam slots is a collective (`Session.sync_optimizer_slots`), so a
        rank-0-only call would hang the job.  Only one rank writes and prunes
        the files: `write=None` means rank 0 of the Session's data-parallel
        group (every process when there is none).  Every rank returns only
        once the bundle, the pruning and the `checkpoint` state file are on
        disk (a barrier on the data-parallel group after the write), so a
        rank may restore or call latest_checkpoint right after save."""
        store = sess._ensure_store()
        sess.sync_optimizer_slots()        # ZeRO-1 data parallelism: Adam slots gathered first (collective)
        gs = self._global_step_value(sess, global_step)
        path = save_path if gs is None else f"{save_path}-{gs}"
        dp = getattr(sess, "dp", None)
        if write is None:
            write = dp is None or getattr(dp, "rank", 0) == 0
        try:
            if write:
                self._write(sess, store, path)
        finally:
            if dp is not None and dist.is_available() and dist.is_initialized():
                dist.barrier(group=getattr(dp, "group", None))
        return path

    def _write(self, sess, store, path):
        out = {}
        for v in self._vars(sess):
            name = v.var_name
            val = store.read(name)
            if getattr(v, "dtype", None) == "int64":
                val = np.rint(val).astype(np.int64)
            out[name] = val
            if name in store.by_name:                 # trainable: Adam slots
                out[name + "/Adam"] = store.adam_m(name).cpu().numpy()
                out[name + "/Adam_1"] = store.adam_v(name).cpu().numpy()
        t = store.step
        out["beta1_power"] = np.float32(BETA1 ** (t + 1))
        out["beta2_power"] = np.float32(BETA2 ** (t + 1))
        tf_bundle.write_bundle(path, out)
        d = os.path.dirname(os.path.abspath(path))
        self._kept.append(path)
        while self.max_to_keep and len(self._kept) > self.max_to_keep:
            old = self._kept.pop(0)
            for f in (f"{old}.index", tf_bundle.data_path(old), _npz(old)):
                if os.path.exists(f):
                    os.remove(f)
        with open(os.path.join(d, "checkpoint"), "w") as f:
            f.write(f'model_checkpoint_path: "{os.path.basename(path)}"\n')
            for p in self._kept:
                f.write(f'all_model_checkpoint_paths: "{os.path.basename(p)}"\n')
        return path

    def restore(self, sess, save_path):
        store = sess._ensure_store()
        names = [v.var_name for v in self._vars(sess)]
        if tf_bundle.is_bundle(save_path):
            index = tf_bundle.read_index(save_path)
            want = [n for n in names if n in index]
            want += [n + s for n in names if n in store.by_name for s in ("/Adam", "/Adam_1") if n + s in index]
            want += [k for k in ("beta1_power", "beta2_power") if k in index]
            d = tf_bundle.read_bundle(save_path, want)
        elif os.path.exists(_npz(save_path)):
            with np.load(_npz(save_path), allow_pickle=False) as z:
                d = {k: z[k] for k in z.files}
        else:
            raise FileNotFoundError(f"no checkpoint at {save_path}")
        missing = [n for n in names if n not in d]
        if missing:
            raise ValueError(f"checkpoint {save_path} lacks variables {missing[:5]}")
        for n in names:
            want = tuple(store.by_name[n].shape) if n in store.by_name else tuple(store.aux[n].shape)
            if tuple(np.shape(d[n])) != want:
                raise ValueError(f"{n}: checkpoint shape {np.shape(d[n])} != variable shape {want}")
        # int64 values (global_step) keep their integer width
        d = {k: (v if np.asarray(v).dtype.kind in "iu" else np.asarray(v, np.float32)) for k, v in d.items()}
        legacy = not tf_bundle.is_bundle(save_path)      # .npz of earlier versions: beta^t
        d["beta_step"] = (_adam_step(d, offset=0 if legacy else 1)
                          if ("beta1_power" in d or "beta2_power" in d) else store.step)
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
