"""Device storage for the graph's variables.

All trainable variables live in ONE flat fp32 buffer (plus flat grad / Adam m
/ Adam v buffers of the same layout), ordered in *reverse creation order* --
the order backward produces their gradients -- so that data-parallel
all-reduce buckets are contiguous slices that become ready one after another.
Each variable keeps its TF name and TF layout (`conv1_1/weights` HWIO,
`conv_t1/weights` [kh,kw,out,in]) so checkpoints map 1:1.

Initial values come from a counter-based generator (numpy Philox keyed by
(seed, crc32(name))), so any host -- including the CPU oracle in the tests --
can regenerate exactly the same weights.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch

from . import graph as G

ALIGN = 4   # floats: every variable starts 16-byte aligned


def init_value(var: G.Variable, seed: int = 0) -> np.ndarray:
    """Deterministic initial value of a variable (float32 numpy)."""
    ini = var.initializer
    shape = tuple(var.shape)
    if isinstance(ini, G.constant_initializer):
        return np.full(shape, ini.value, dtype=np.float32)
    if isinstance(ini, G.random_normal_initializer):
        key = zlib.crc32(var.var_name.encode()) & 0xFFFFFFFF
        rng = np.random.Generator(np.random.Philox(key=[seed & 0xFFFFFFFFFFFFFFFF, key]))
        return (rng.standard_normal(shape, dtype=np.float32) * np.float32(ini.stddev)
                + np.float32(ini.mean)).astype(np.float32)
    if callable(ini):
        return np.asarray(ini(shape), dtype=np.float32)
    raise TypeError(f"unsupported initializer {ini!r}")


def _aux_dtype(var):
    return torch.int64 if getattr(var, "dtype", None) == G.int64 else torch.float32


TAIL_SLACK = 1024


class VariableStore:
    """Trainable variables in the flat buffers (`vars`, backward order);
    non-trainable ones (the accumulate template's gradient accumulators,
    `global_step`, BatchNorm moving statistics) as separate fp32 tensors in
    `aux` -- they never enter Adam or the gradient all-reduce."""

    def __init__(self, variables, device, seed=0):
        variables = list(variables)
        self.vars = [v for v in variables if getattr(v, "trainable", True)]
        self.aux_vars = [v for v in variables if not getattr(v, "trainable", True)]
        self.device = device
        self.seed = seed
        order = list(reversed(self.vars))
        self.offset = {}
        off = 0
        for v in order:
            self.offset[v.var_name] = off
            n = int(np.prod(v.shape))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        # zero tail slack: data-parallel buckets are padded to multiples of
        # 4 * world elements (dp.py), world <= TAIL_SLACK / 4
        self.alloc = off + TAIL_SLACK
        self.params = torch.zeros(self.alloc, dtype=torch.float32, device=device)
        self.grads = torch.zeros(self.alloc, dtype=torch.float32, device=device)
        self.m = torch.zeros(self.alloc, dtype=torch.float32, device=device)
        self.v = torch.zeros(self.alloc, dtype=torch.float32, device=device)
        self.by_name = {v.var_name: v for v in self.vars}
        self.aux_by_name = {v.var_name: v for v in self.aux_vars}
        # int64 non-trainables (global_step) stay int64, as TF keeps them: an
        # fp32 counter stops advancing at 2^24
        self.aux = {v.var_name: torch.zeros(tuple(v.shape), dtype=_aux_dtype(v), device=device)
                    for v in self.aux_vars}
        self.aux_version = 0    # bumped when a non-trainable value is written from the host
        self.order = order
        self.step = 0           # Adam t (TF beta powers)
        self.packed = {}        # (var_name, mode) -> (tensor, a_pad, b_pad)
        self.hwio_only = set()  # filters whose forward reads the HWIO copy (no KRSC copy; planner.py)
        self.version = 0        # bumped on every update -> repack

    def _view(self, buf, name):
        v = self.by_name[name]
        n = int(np.prod(v.shape))
        o = self.offset[name]
        return buf[o:o + n].view(*v.shape)

    @property
    def all_vars(self):
        return self.vars + self.aux_vars

    def param(self, name):
        if name in self.aux:
            return self.aux[name]
        return self._view(self.params, name)

    def grad(self, name):
        return self._view(self.grads, name)

    def adam_m(self, name):
        return self._view(self.m, name)

    def adam_v(self, name):
        return self._view(self.v, name)

    def initialize(self):
        host = np.zeros(self.alloc, dtype=np.float32)
        for v in self.vars:
            n = int(np.prod(v.shape))
            o = self.offset[v.var_name]
            host[o:o + n] = init_value(v, self.seed).reshape(-1)
        self.params.copy_(torch.from_numpy(host).to(self.device))
        for v in self.aux_vars:
            t = self.aux[v.var_name]
            if t.dtype == torch.int64:
                ini = v.initializer
                val = np.full(tuple(v.shape), int(ini.value), np.int64) if isinstance(ini, G.constant_initializer) \
                    else np.rint(np.asarray(ini(tuple(v.shape)), np.float64)).astype(np.int64)
                t.copy_(torch.from_numpy(np.asarray(val, np.int64).reshape(tuple(v.shape))).to(self.device))
            else:
                t.copy_(torch.from_numpy(init_value(v, self.seed)).to(self.device))
        self.aux_version += 1
        self.m.zero_()
        self.v.zero_()
        self.step = 0
        self.version += 1

    def assign(self, name, value):
        if name in self.aux and self.aux[name].dtype == torch.int64:
            a = np.asarray(value)
            a = a.astype(np.int64) if a.dtype.kind in "iu" else np.rint(a).astype(np.int64)
            self.aux[name].copy_(torch.from_numpy(a).to(self.device).view(self.aux[name].shape))
            self.aux_version += 1
            return
        t = torch.as_tensor(np.asarray(value, dtype=np.float32)).to(self.device)
        if name in self.aux:
            self.aux[name].copy_(t.view(self.aux[name].shape))
            self.aux_version += 1
            return
        self.param(name).copy_(t.view(self.by_name[name].shape))
        self.version += 1

    def read(self, name):
        return self.param(name).detach().cpu().numpy().copy()

    def state_dict(self):
        """TF-Saver-compatible names -> numpy arrays (plus Adam slots)."""
        out = {}
        for v in self.vars:
            out[v.var_name] = self.read(v.var_name)
            out[v.var_name + "/Adam"] = self._view(self.m, v.var_name).cpu().numpy().copy()
            out[v.var_name + "/Adam_1"] = self._view(self.v, v.var_name).cpu().numpy().copy()
        for v in self.aux_vars:
            out[v.var_name] = self.aux[v.var_name].cpu().numpy().copy()
        out["beta_step"] = np.array(self.step)
        return out

    def load_state_dict(self, d):
        for v in self.vars:
            if v.var_name in d:
                self.assign(v.var_name, d[v.var_name])
            if v.var_name + "/Adam" in d:
                self._view(self.m, v.var_name).copy_(torch.from_numpy(np.asarray(d[v.var_name + "/Adam"], np.float32)).to(self.device))
                self._view(self.v, v.var_name).copy_(torch.from_numpy(np.asarray(d[v.var_name + "/Adam_1"], np.float32)).to(self.device))
        for v in self.aux_vars:
            if v.var_name in d:
                self.assign(v.var_name, d[v.var_name])
        if "beta_step" in d:
            self.step = int(d["beta_step"])
        self.version += 1
