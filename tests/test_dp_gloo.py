"""Data-parallel path on CPU: world size 2 over gloo (127.0.0.1).

Checks dp.DataParallel's bucketing / in-order async all-reduce on a store
shaped like the Session's, and the DP identity the bench relies on: the
mean of per-shard mean-loss gradients equals the full-batch gradient."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd.dp import DataParallel


class _V:
    def __init__(self, name, shape):
        self.var_name, self.shape = name, shape


class FakeStore:
    """Same attributes DataParallel uses on VariableStore."""

    def __init__(self, shapes):
        self.vars = [_V(k, s) for k, s in shapes.items()]
        self.order = list(reversed(self.vars))
        self.offset = {}
        off = 0
        for v in self.order:
            self.offset[v.var_name] = off
            off += (int(np.prod(v.shape)) + 3) // 4 * 4
        self.numel = off
        self.grads = torch.zeros(off, dtype=torch.float32)

    def grad(self, name):
        v = next(x for x in self.vars if x.var_name == name)
        n = int(np.prod(v.shape))
        return self.grads[self.offset[name]:self.offset[name] + n].view(*v.shape)


SHAPES = {"c1/weights": (3, 3, 3, 8), "c1/biases": (8,), "c2/weights": (3, 3, 8, 8), "c2/biases": (8,),
          "t1/weights": (4, 4, 2, 8), "t1/biases": (2,)}


def tiny_net(p, x):
    h = T.relu(T.bias_add(T.conv2d(x, p["c1/weights"]), p["c1/biases"]))
    h = T.max_pool2x2(h)
    h = T.relu(T.bias_add(T.conv2d(h, p["c2/weights"]), p["c2/biases"]))
    N, H, W, _ = x.shape
    return T.bias_add(T.conv2d_transpose(h, p["t1/weights"], (N, H, W, 2), 2), p["t1/biases"])


def grads_of(weights, x, lab):
    p = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in weights.items()}
    loss = T.mean_softmax_xent(tiny_net(p, torch.from_numpy(x).double()), T.one_hot(torch.from_numpy(lab), 2))
    loss.backward()
    return {k: v.grad.float() for k, v in p.items()}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0)
        weights = {k: (rng.standard_normal(s) * 0.3).astype(np.float32) for k, s in SHAPES.items()}
        x = rng.standard_normal((4, 8, 12, 3))
        lab = rng.integers(0, 2, (4, 8, 12))
        shard = slice(rank * 2, rank * 2 + 2)
        g = grads_of(weights, x[shard], lab[shard])
        store = FakeStore(SHAPES)
        dp = DataParallel(bucket_mb=0.002)          # tiny buckets: several, c2/weights chunked
        dp.prepare(store)
        assert len(dp.buckets) >= 3
        assert len(dp.var_buckets["c2/weights"]) >= 2             # chunked across buckets
        # contiguous, disjoint, cover the whole buffer
        spans = sorted((s, e) for s, e, _ in dp.buckets)
        assert spans[0][0] == 0 and spans[-1][1] == store.numel
        assert all(spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
        for v in store.order:                        # backward order, as the Session does
            store.grad(v.var_name).copy_(g[v.var_name])
            dp.ready([v.var_name])
        dp.finish()
        out = {k: (store.grad(k) / world).numpy().copy() for k in SHAPES}
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_world2_mean_of_shard_means():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(0)
    weights = {k: (rng.standard_normal(s) * 0.3).astype(np.float32) for k, s in SHAPES.items()}
    x = rng.standard_normal((4, 8, 12, 3))
    lab = rng.integers(0, 2, (4, 8, 12))
    full = grads_of(weights, x, lab)
    for k in SHAPES:
        np.testing.assert_allclose(res[0][k], res[1][k], rtol=0, atol=0)   # ranks agree bitwise
        np.testing.assert_allclose(res[0][k], full[k].numpy(), rtol=1e-5, atol=1e-7)
