"""One rank of tests/test_gpu_dp.py: the real Session data-parallel path
(dp.DataParallel buckets + all-reduce hooks, 1/world Adam scale, per-rank
shard) on a shared cuda:0 over the gloo backend (RCCL refuses two ranks on one
device).  Writes its gradients and updated parameters to OUT/rank{R}_{case}.npz.

usage: python -m tests.workers.dp_session_worker RANK WORLD PORT OUT"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import models as M  # noqa: E402
from semanticsegmentation_tensorflow_amd.dp import DataParallel  # noqa: E402
from tests.model_inputs import he_weights, synthetic_batch  # noqa: E402
from tests.test_gpu_fcn import build_fcn  # noqa: E402

N_GLOBAL, H, W = 4, 64, 96
CASES = [("f32", False), ("f32", True), ("bf16", False)]


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from semanticsegmentation_tensorflow_amd import tf
    try:
        weights = he_weights(M.fcn_param_shapes(3, 2), 51)
        img, lab = synthetic_batch(N_GLOBAL, H, W, 52)
        per = N_GLOBAL // world
        shard = slice(rank * per, rank * per + per)
        for dtype, overlap in CASES:
            image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
            # small buckets: several all-reduces, conv6's filter gradient chunked
            dp = DataParallel(bucket_mb=16.0)
            sess = tf.Session(compute_dtype=dtype, data_parallel=dp, overlap_optimizer=overlap, seed=5)
            sess.run(tf.global_variables_initializer())
            for k, v in weights.items():
                sess.assign(k, v)
            l, _ = sess.run([loss, train_step], feed_dict={image: img[shard], labels: lab[shard], keep: 1.0})
            torch.cuda.synchronize()
            assert any(len(b) > 1 for b in dp.var_buckets.values()), "no chunked variable"
            res = {"loss": np.float64(l), "buckets": np.int64(len(dp.buckets))}
            for k in weights:
                res["g:" + k] = sess.store.grad(k).cpu().numpy()
                res["p:" + k] = sess.variable_value(k)
            np.savez(os.path.join(out, f"rank{rank}_{dtype}_{int(overlap)}.npz"), **res)
            dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
