"""Stream scheduling of a Session step (mixin): the side stream that runs the
filter gradients and their split-K reductions beside the input-gradient chain,
the deferred fused filter-gradient + Adam launches, per-launch HIP-event
timing, and the overlapped per-layer optimizer.  Split out of session.py;
`Session` inherits these methods unchanged."""
from __future__ import annotations

import contextlib
import math

import torch

from . import ops


class _AdamOverlap:
    """Per-step driver of the overlapped optimizer: each variable group's fused
    Adam + pack launch runs on a side stream after an event on the compute
    stream (or, with data parallelism, after the bucket's all-reduce), so the
    HBM-bound update of layer L hides under the MFMA-bound backward of layers
    < L.  Nothing later in the step reads L's parameters or packed copies
    (its input gradient is enqueued before its filter gradient).  finish()
    updates the remaining variables and makes the compute stream wait."""

    def __init__(self, sess, opt, gs, var_set, big_only=False):
        self.s = sess
        self.opt = opt
        self.gs = gs
        self.var_set = var_set
        self.side = sess.side_stream()
        self.main = torch.cuda.current_stream(sess.device)
        self.done = set()
        # big_only (data-parallel all-reduce steps, Session.overlap_big_mb):
        # only variables of >= overlap_big_mb MB overlap (FCN: conv6, conv7 --
        # the 2.9 GB of Adam traffic the single-process step fuses into their
        # filter gradients); finish() updates the rest in one launch on the
        # compute stream
        self.big = None
        if big_only:
            st = sess.store
            lim = sess.overlap_big_mb * (1 << 20) / 4
            self.big = {nm for nm in var_set if nm in st.by_name and math.prod(st.by_name[nm].shape) >= lim}

    def _adam(self, names, stream=None):
        st = self.s.store
        o = self.opt
        names = [nm for nm in names if nm in self.var_set]
        if not names:
            return
        ops.adam_tf1_pack(st.params, st.grads, st.m, st.v, self.s._adam_plan(names), o.lr, st.step, o.beta1,
                          o.beta2, o.epsilon, grad_scale=self.gs, dtype=self.s._pack_dtype(),
                          stream=self.side if stream is None else stream)
        self.done.update(names)

    def launch(self, names):
        ev = torch.cuda.Event()
        ev.record(self.main)
        self.side.wait_event(ev)
        self._adam(names)

    def after_work(self, works, names):
        if self.big is not None:
            names = [nm for nm in names if nm in self.big]
            if not names:
                return
        if works:
            with torch.cuda.stream(self.side):
                for w in works:
                    w.wait()
        else:
            ev = torch.cuda.Event()
            ev.record(self.main)
            self.side.wait_event(ev)
        self._adam(names)

    def finish(self):
        rest = [v.var_name for v in self.s.store.order if v.var_name in self.var_set and v.var_name not in self.done]
        if self.big is not None:           # the small variables: one launch on the compute stream
            self.main.wait_stream(self.side)
            if rest:
                self._adam(rest, stream=self.main)
            return
        if rest:
            self.launch(rest)
        self.main.wait_stream(self.side)


class StreamMixin:
    @contextlib.contextmanager
    def _beside(self, side):
        """Run the enclosed launches on `side` (the filter-gradient stream),
        ordered after everything enqueued so far on the compute stream; a no-op
        context when side is None (no side stream: CPU plans, disabled)."""
        if side is None:
            yield None
            return
        ev = torch.cuda.Event()
        ev.record(self._red[1])
        side.wait_event(ev)
        with torch.cuda.stream(side):
            yield side

    def _wgrad_side(self, p, n, level=1):
        """The side stream for node n's filter gradient, or None."""
        return self._red[0] if (self._red is not None and self.side_wgrad >= level) else None

    def _tick_fused(self, flush=False):
        keep = []
        for item in self._pending_fused:
            item[0] -= 1
            if flush or item[0] <= 0:
                item[1]()
            else:
                keep.append(item)
        self._pending_fused = keep

    def _node_ws(self, p, n):
        """The conv's own filter-gradient workspace (p.wg_ws) as an ops.Workspace,
        for launches on the side stream (the shared one belongs to the compute stream)."""
        w = ops.Workspace(self.device)
        w.buf = p.wg_ws[id(n)]
        return w

    def _timed(self, desc, op, fn, *args):
        """fn(*args), bracketed by HIP events on the launch stream when
        self.timer is a list (and self.timer_match, if set, accepts the
        launch: bench.py times only the dominant kernel's launches)."""
        if self.timer is None or (self.timer_match is not None and not self.timer_match(desc, op)):
            return fn(*args)
        s, e = ops.TimingEvent(), ops.TimingEvent()    # no cache flush in the interval
        stream = torch.cuda.current_stream(self.device)
        s.record(stream)
        r = fn(*args)
        e.record(stream)
        self.timer.append((desc, op, s, e))
        return r
