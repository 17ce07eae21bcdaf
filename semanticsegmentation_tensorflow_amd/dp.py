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
        self.var_buckets = {}
        self.store = None
        # optional hook (works, var_names) called as each bucket's all-reduce
        # is issued, with the variables whose last piece it carries and the
        # collectives covering them: the Session runs their Adam update on a
        # side stream once those complete
        self.on_launch = None
        # (side, compute) streams while the Session defers split-K filter-
        # gradient reductions to the side stream: a bucket's all-reduce is
        # then issued from the side stream after it has caught up with the
        # compute stream, so it waits for both the kernels enqueued on the
        # compute stream and the deferred reductions -- without the compute
        # stream ever waiting on the side stream
        self.launch_streams = None

    def prepare(self, store):
        """Cut the flat gradient buffer into contiguous buckets of at most
        bucket_bytes (backward order).  A variable larger than a bucket is
        chunked (conv6's 411 MB filter gradient -> 64 MB all-reduces), so its
        first bytes leave while the rest are still queued; a bucket is ready
        once every variable with a piece in it is."""
        if self.store is store and self.buckets:
            return
        self.store = store
        cap = max(1, self.bucket_bytes // 4)              # fp32 elements per bucket
        spans = []                                        # (name, start, end) in backward order
        order = list(store.order)
        for i, v in enumerate(order):
            s0 = store.offset[v.var_name]
            e0 = store.offset[order[i + 1].var_name] if i + 1 < len(order) else store.numel
            spans.append((v.var_name, s0, e0))
        self.buckets = []                                 # (start, end, [names with a piece here])
        cur, start, fill = [], None, 0
        for name, s0, e0 in spans:
            pos = s0
            while pos < e0:
                if start is None:
                    start = pos
                take = min(e0 - pos, cap - fill)
                if not cur or cur[-1] != name:
                    cur.append(name)
                pos += take
                fill += take
                if fill >= cap:
                    self.buckets.append((start, pos, cur))
                    cur, start, fill = [], None, 0
        if cur:
            self.buckets.append((start, store.numel, cur))
        self.var_buckets = {}
        for i, (_, _, names) in enumerate(self.buckets):
            for nm in names:
                self.var_buckets.setdefault(nm, []).append(i)
        self.var_bucket = {nm: b[-1] for nm, b in self.var_buckets.items()}   # bucket holding its last piece
        self._reset()

    def _reset(self):
        self.remaining = [len(b[2]) for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.bucket_work = [None] * len(self.buckets)

    def _launch(self, i):
        s, e, names = self.buckets[i]
        w = None
        if e > s:
            if self.launch_streams is not None:
                import torch
                side, main = self.launch_streams
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    w = dist.all_reduce(self.store.grads[s:e], op=dist.ReduceOp.SUM, group=self.group,
                                        async_op=True)
            else:
                w = dist.all_reduce(self.store.grads[s:e], op=dist.ReduceOp.SUM, group=self.group,
                                    async_op=True)
            self.works.append(w)
        self.bucket_work[i] = w
        self.launched[i] = True
        if self.on_launch is not None:
            done = [nm for nm in names if self.var_bucket[nm] == i]     # variables complete with this bucket
            if done:
                works = [self.bucket_work[j] for nm in done for j in self.var_buckets[nm]]
                self.on_launch([x for x in works if x is not None], done)

    def ready(self, names):
        for nm in names:
            for i in self.var_buckets.get(nm, ()):
                self.remaining[i] -= 1
        # launch strictly in bucket order so every rank issues the same sequence
        j = 0
        while j < len(self.buckets) and self.launched[j]:
            j += 1
        while j < len(self.buckets) and self.remaining[j] <= 0 and not self.launched[j]:
            self._launch(j)
            j += 1

    def abort_step(self):
        """A step that raised mid-backward: forget its bucket state (the
        collectives already issued complete on their own streams)."""
        self._reset()

    def finish(self):
        for i in range(len(self.buckets)):
            if not self.launched[i]:
                self._launch(i)
        for w in self.works:
            w.wait()
        self._reset()
