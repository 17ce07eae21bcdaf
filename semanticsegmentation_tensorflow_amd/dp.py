"""Data-parallel gradient exchange: one process per GPU, RCCL all-reduce over
xGMI through torch.distributed (backend "nccl" is RCCL on ROCm).

The reference has no multi-device code; this is new.  The
VariableStore keeps every gradient in one flat fp32 buffer laid out in the
order backward produces them, so a bucket is a contiguous slice.  The Session
calls `ready(var_names)` right after enqueueing each layer's filter-gradient
kernel; when a bucket's last variable is in, its all-reduce is issued at once
-- ProcessGroupNCCL makes its stream wait on the compute stream up to that
point, so the collective overlaps the remaining backward kernels.  `finish()`
makes the compute stream wait for every bucket before Adam.  Gradients are
summed; the Session folds 1/world into Adam's grad_scale (mean of per-shard
means == the global-batch mean for equal shards).
"""
from __future__ import annotations

import torch.distributed as dist


class DataParallel:
    def __init__(self, bucket_mb: float = 64.0, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised (one process per GPU)")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.buckets = []
        self.var_bucket = {}
        self.store = None
        # optional hook (work_or_None, var_names) called as each bucket's
        # all-reduce is issued: the Session runs that bucket's Adam update on a
        # side stream once the collective completes
        self.on_launch = None

    def prepare(self, store):
        """Cut the flat gradient buffer into contiguous buckets (backward order)."""
        if self.store is store and self.buckets:
            return
        self.store = store
        self.buckets = []
        self.var_bucket = {}
        cur, start, nbytes = [], None, 0
        for v in store.order:
            name = v.var_name
            off = store.offset[name]
            n = 1
            for s in v.shape:
                n *= int(s)
            if cur and nbytes + 4 * n > self.bucket_bytes:
                self.buckets.append((start, off, cur))
                cur, start, nbytes = [], None, 0
            if start is None:
                start = off
            cur.append(name)
            nbytes += 4 * n
        if cur:
            self.buckets.append((start, store.numel, cur))
        for i, (_, _, names) in enumerate(self.buckets):
            for nm in names:
                self.var_bucket[nm] = i
        self._reset()

    def _reset(self):
        self.remaining = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []

    def _launch(self, i):
        s, e, names = self.buckets[i]
        w = None
        if e > s:
            w = dist.all_reduce(self.store.grads[s:e], op=dist.ReduceOp.SUM, group=self.group,
                                async_op=True)
            self.works.append(w)
        self.launched[i] = True
        if self.on_launch is not None:
            self.on_launch(w, names)

    def ready(self, names):
        for nm in names:
            i = self.var_bucket.get(nm)
            if i is None:
                continue
            self.remaining[i] -= 1
            # launch strictly in bucket order so every rank issues the same sequence
            if self.remaining[i] == 0:
                j = 0
                while j < len(self.buckets) and self.launched[j]:
                    j += 1
                while j < len(self.buckets) and self.remaining[j] <= 0 and not self.launched[j]:
                    self._launch(j)
                    j += 1

    def finish(self):
        for i in range(len(self.buckets)):
            if not self.launched[i]:
                self._launch(i)
        for w in self.works:
            w.wait()
        self._reset()
