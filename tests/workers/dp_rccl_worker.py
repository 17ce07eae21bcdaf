"""World-1 RCCL ('nccl') data-parallel Session step on the GPU box's one card
(tests/test_gpu_dp_rccl.py): the collectives are forced on at world 1
(DataParallel(force_collectives=True)), so the ZeRO-1 reduce-scatter /
all-gather and the all-reduce path run through RCCL exactly as a world > 1 rank
issues them -- on the Session's side stream, beside the side-stream filter
gradients and their deferred split-K reductions -- under every schedule
attribute value.  Also the single-process Session under the same schedules.
Writes OUT/<case>.npz (gradients, parameters, Adam m / v).

usage: python -m tests.workers.dp_rccl_worker PORT OUT"""
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

N, H, W = 4, 64, 96
# (tag, dtype, data parallel: None | "zero" | "allreduce", schedule attributes)
CASES = [
    ("ref_f32", "f32", None, {}),
    ("sp_f32_serial", "f32", None, {"side_wgrad": 0, "main_wgrad": 0}),
    ("sp_f32_side1", "f32", None, {"side_wgrad": 1, "main_wgrad": 0, "fused_delay": 0}),
    ("sp_f32_nofuse", "f32", None, {"fuse_pool": False, "fuse_grad_sum": False}),
    ("dp_f32_zero", "f32", "zero", {}),
    ("dp_f32_zero_serial", "f32", "zero", {"side_wgrad": 0, "main_wgrad": 0}),
    ("dp_f32_zero_side1", "f32", "zero", {"side_wgrad": 1, "main_wgrad": 0}),
    ("dp_f32_allreduce", "f32", "allreduce", {"main_wgrad": 3}),
    ("ref_bf16", "bf16", None, {}),
    ("sp_bf16_serial", "bf16", None, {"side_wgrad": 0, "main_wgrad": 0, "fused_delay": 0}),
    ("sp_bf16_side1", "bf16", None, {"side_wgrad": 1, "main_wgrad": 1}),
    ("sp_bf16_mw2", "bf16", None, {"main_wgrad": 2}),
    ("sp_bf16_nofuse", "bf16", None, {"fuse_pool": False, "fuse_grad_sum": False}),
    ("dp_bf16_zero", "bf16", "zero", {}),
    ("dp_bf16_zero_serial", "bf16", "zero", {"side_wgrad": 0, "main_wgrad": 0}),
    ("dp_bf16_allreduce", "bf16", "allreduce", {"side_wgrad": 1}),
    ("dp_bf16_allreduce_big", "bf16", "allreduce", {"overlap_big_mb": 4}),
    ("dp_f32_allreduce_big", "f32", "allreduce", {"overlap_big_mb": 1}),
    ("dp_bf16_allreduce_end", "bf16", "allreduce", {"overlap_big_mb": 0}),
]


def main():
    port, out = sys.argv[1], sys.argv[2]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from semanticsegmentation_tensorflow_amd import tf
    try:
        weights = he_weights(M.fcn_param_shapes(3, 2), 91)
        img, lab = synthetic_batch(N, H, W, 92)
        for tag, dtype, mode, sched in CASES:
            image, labels, keep, pred, logits, loss, train_step = build_fcn(H, W)
            dp = None
            if mode is not None:
                dp = DataParallel(bucket_mb=16.0, shard_optimizer=mode == "zero", force_collectives=True)
                assert dp.active and dist.get_backend() == "nccl"
            sess = tf.Session(compute_dtype=dtype, data_parallel=dp, seed=5)
            sess.store_fused_grads = True
            for k, v in sched.items():
                assert hasattr(sess, k), k
                setattr(sess, k, v)
            sess.run(tf.global_variables_initializer())
            for k, v in weights.items():
                sess.assign(k, v)
            sess.run(train_step, feed_dict={image: img, labels: lab, keep: 1.0})
            torch.cuda.synchronize()
            if dp is not None:
                assert dp.mode == mode, (dp.mode, mode)
                assert len(dp.buckets) >= 3
            sess.sync_optimizer_slots()
            torch.cuda.synchronize()
            res = {}
            for k in weights:
                res["g:" + k] = sess.store.grad(k).cpu().numpy()
                res["p:" + k] = sess.variable_value(k)
                res["m:" + k] = sess.store.adam_m(k).cpu().numpy()
                res["v:" + k] = sess.store.adam_v(k).cpu().numpy()
            np.savez(os.path.join(out, tag + ".npz"), **res)
            del sess
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
