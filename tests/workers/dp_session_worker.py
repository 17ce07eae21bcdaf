"""One rank of tests/test_gpu_dp.py: the real Session data-parallel path
(dp.DataParallel buckets + collective hooks, 1/world Adam scale, per-rank
shard) on a shared cuda:0 over the gloo backend (RCCL refuses two ranks on one
device).  Cases: (dtype, overlapped per-layer optimizer, ZeRO-1 sharded
Adam).  Writes its gradients (the reduced slices all-gathered for a sharded
step), updated parameters and Adam slots to OUT/rank{R}_{case}.npz.

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
CASES = [("f32", False, True), ("f32", False, False), ("f32", True, False), ("bf16", False, True)]


def case_tag(dtype, overlap, shard):
    return f"{dtype}_{int(overlap)}_{int(shard)}"


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
        part = slice(rank * per, rank * per + per)
        for dtype, overlap, shard in CASES:
            image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
            # small buckets: several collectives, conv6's filter gradient chunked
            dp = DataParallel(bucket_mb=16.0, shard_optimizer=shard)
            sess = tf.Session(compute_dtype=dtype, data_parallel=dp, overlap_optimizer=overlap, seed=5)
            sess.run(tf.global_variables_initializer())
            for k, v in weights.items():
                sess.assign(k, v)
            l, _ = sess.run([loss, train_step], feed_dict={image: img[part], labels: lab[part], keep: 1.0})
            torch.cuda.synchronize()
            assert any(len(b) > 1 for b in dp.var_buckets.values()), "no chunked variable"
            assert dp.mode == ("zero" if shard and not overlap else "allreduce"), dp.mode
            if dp.mode == "zero":
                dp._gather(sess.store.grads)          # test only: every rank's reduced slices
                assert dp.slots_stale
            sess.sync_optimizer_slots()
            torch.cuda.synchronize()
            res = {"loss": np.float64(l), "buckets": np.int64(len(dp.buckets))}
            for k in weights:
                res["g:" + k] = sess.store.grad(k).cpu().numpy()
                res["p:" + k] = sess.variable_value(k)
                res["m:" + k] = sess.store.adam_m(k).cpu().numpy()
                res["v:" + k] = sess.store.adam_v(k).cpu().numpy()
            np.savez(os.path.join(out, f"rank{rank}_{case_tag(dtype, overlap, shard)}.npz"), **res)
            dist.barrier()
        # a ZeRO-1 step (m / v current on this rank's slices only),
        # then an all-reduce-mode step (the overlapped per-layer optimizer reads
        # whole variables) with no explicit sync between them: the Session
        # gathers the stale slices first, so the ranks stay bit-identical
        image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
        dp = DataParallel(bucket_mb=16.0, shard_optimizer=True)
        sess = tf.Session(compute_dtype="f32", data_parallel=dp, seed=5)
        sess.run(tf.global_variables_initializer())
        for k, v in weights.items():
            sess.assign(k, v)
        feed = {image: img[part], labels: lab[part], keep: 1.0}
        sess.run(train_step, feed_dict=feed)
        assert dp.mode == "zero" and dp.slots_stale
        sess.overlap_optimizer = True
        sess.run(train_step, feed_dict=feed)
        torch.cuda.synchronize()
        assert dp.mode == "allreduce" and not dp.slots_stale, (dp.mode, dp.slots_stale)
        res = {}
        for k in weights:
            res["p:" + k] = sess.variable_value(k)
            res["m:" + k] = sess.store.adam_m(k).cpu().numpy()
            res["v:" + k] = sess.store.adam_v(k).cpu().numpy()
        np.savez(os.path.join(out, f"rank{rank}_mixed.npz"), **res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
