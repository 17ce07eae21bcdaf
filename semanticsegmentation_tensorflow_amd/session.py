"""Session: compiles the symbolic graph into a static launch plan over the HIP
C-ABI and runs it -- the stand-in for the reference's
`sess.run(train_step, feed_dict)` (Network/model/FCN.py:395-398).

Compilation (per fetch set and fed shapes):
  * shape resolution with TF's rules (conv2d_transpose shape check included);
  * fusion of single-consumer chains into one kernel launch each:
      Conv2D [+BiasAdd] [+Relu] [+Dropout]      -> conv (fused epilogue)
      Conv2DTranspose [+BiasAdd] [+Add]         -> tconv (bias + skip fusion)
      FusedBatchNorm [+Relu]                    -> bn
      SoftmaxXent + Mean                        -> xent (loss and dlogits)
  * static device buffers (NHWC, channels padded to 8) for every activation,
    gradient and workspace -- nothing is allocated while a step runs;
  * backward in reverse order with gradients written straight into the flat
    fp32 gradient buffer of the VariableStore; data-parallel buckets are
    all-reduced (RCCL) as soon as their gradients are complete, overlapping the
    rest of backward;
  * TF1 Adam over the flat buffer, then re-packing of the bf16/fp32 filter
    copies the convolution kernels read.
"""
from __future__ import annotations

import collections

import numpy as np
import torch

from . import graph as G
from . import ops
from .ops import round8
from .planner import PlanMixin
from .streams import StreamMixin, _AdamOverlap
from .variables import VariableStore

_SEED_MIX = 0x9E3779B1


class _Node:
    """One fused kernel in the forward plan."""

    def __init__(self, kind, ops_, inputs, output, **kw):
        self.kind = kind
        self.ops = ops_
        self.inputs = inputs
        self.output = output
        self.__dict__.update(kw)


class Plan:
    pass


def _is_op(f, type_):
    return isinstance(f, G.Op) and f.type == type_


def _accumulator_pairs(op):
    """apply_gradients whose gradient sources are all variables (accumulators)."""
    return all(isinstance(g, G.Variable) for g, _ in op.attrs["pairs"])


def _gradient_source(t):
    """(loss, var, scale) of a compute_gradients output, optionally wrapped in
    tf.scalar_mul."""
    scale = 1.0
    if isinstance(t, G.Tensor) and t.op.type == "ScalarMul":
        scale = G.const_value(t.op.attrs["scalar"])
        t = t.op.attrs["x"]
    if not (isinstance(t, G.Tensor) and t.op.type == "Gradient"):
        raise NotImplementedError("expected an optimizer.compute_gradients output")
    return t.op.attrs["loss"], t.op.attrs["var"], scale


class _TrainSpec:
    """What a run call's gradient-consuming fetches ask for: the loss, the
    variables whose gradients are needed, and what consumes them (Adam with
    `optimizer`, or `accum` = [(accumulator, variable, scale)])."""

    def __init__(self, loss, optimizer, var_list, grad_scale, global_step, accum, ops_):
        self.inputs = [loss]
        self.attrs = {"optimizer": optimizer, "var_list": list(var_list), "grad_scale": float(grad_scale),
                      "global_step": global_step}
        self.accum = accum
        self.ops = ops_


def _np(x):
    if isinstance(x, torch.Tensor):
        return x
    return torch.from_numpy(np.ascontiguousarray(x))


_SIDE_STREAMS = {}


def side_stream_for(device):
    """The process-wide side stream of a device (filter gradients, their
    split-K reductions, the fused conv6 / conv7 update, bucket collectives),
    shared by every Session on it.  HIP maps streams onto a fixed pool of
    hardware queues (GPU_MAX_HW_QUEUES, 4 on the box), and a stream created
    after an RCCL communicator took some of them can land on the compute
    stream's queue: every launch of the step then runs serialised on one queue
    (round 6: the world-1 data-parallel step at 7.6 ms instead of 6.8,
    tools/queue_probe.py).  Created before init_process_group -- bench.py
    calls this first; a data-parallel program should too -- it keeps a queue
    of its own."""
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
        with torch.cuda.stream(s):      # a first launch binds the stream to its queue now
            torch.zeros(1, device=device)
    return s


class Session(PlanMixin, StreamMixin):
    def __init__(self, graph=None, compute_dtype="bf16", device=None, seed=0, data_parallel=None,
                 overlap_optimizer=False, fuse_adam=True, loss_scale=None):
        """compute_dtype: "bf16" (default), "f16" (IEEE half activations and
        filter copies, fp32 accumulation -- config C5) or "f32" (parity path).
        loss_scale (f16): "dynamic" (default for f16: TF's DynamicLossScale,
        2^15 initial, x2 after 2000 finite steps, /2 and skip the update on
        overflow), a fixed number, or None/1 (no scaling)."""
        self.graph = graph or G.get_default_graph()
        if not torch.cuda.is_available():
            raise RuntimeError("Session needs an MI355X (HIP device); there is no CPU fallback")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.cdt = {"bf16": ops.BF16, "bfloat16": ops.BF16, "f16": ops.F16, "fp16": ops.F16,
                    "float16": ops.F16, "f32": ops.F32, "fp32": ops.F32, "float32": ops.F32}[compute_dtype]
        self.tdt = ops.torch_dtype(self.cdt)
        if loss_scale is None and self.cdt == ops.F16:
            loss_scale = "dynamic"
        self.dynamic_scale = loss_scale == "dynamic"
        self.loss_scale = 2.0 ** 15 if self.dynamic_scale else float(loss_scale or 1.0)
        self.scale_increment_period = 2000
        self.good_steps = 0
        self.skipped_steps = 0
        self._finite_flag = None
        self.seed = seed
        self.store = None
        self.plans = {}
        self.ws = ops.Workspace(self.device)
        self.dp = data_parallel
        self.run_count = 0
        self._packed_version = -1
        self._adam_key = None
        self._adam = None
        self._adam_groups = {}
        self.overlap_optimizer = overlap_optimizer
        # Adam fused into the filter-gradient epilogue where the library supports
        # it (single process: nothing sits between gradient and update)
        self.fuse_adam = fuse_adam
        self.store_fused_grads = False   # tests: also write the fused layers' gradients
        self._fused = None               # names updated inside backward this step
        # split-K reductions of filter gradients on a side stream, overlapping
        # the next layer's input gradient (with data parallelism each bucket's
        # all-reduce is issued from that side stream, after it has caught up
        # with the compute stream)
        self.defer_wgrad_reduce = True
        # Dropout right after a bias-free / ReLU-free conv (FC-DenseNet's
        # Conv2D_Block + dropout) applied in the conv epilogue
        self.fuse_dropout = True
        # DenseBlock concatenations as channel views of one block buffer
        self.alias_concat = True
        # BatchNorm(+ReLU) feeding a single 1x1 conv folded into its operand prologue
        self.fold_bn = True
        self.fold_dropout_grad = True   # Conv -> Dropout -> BN: the dropout gradient inside the BN backward
        # Schedule attributes (measured defaults; every value is exercised by
        # tests/test_gpu_dp_rccl.py against the default schedule -- bench.py
        # --schedule NAME=VALUE sets them for A/B runs):
        # a tensor's later input-gradient contributions accumulate in the epilogue
        self.fuse_grad_sum = True
        self.fuse_bn_bwd = True         # folded BN: its backward in the consuming 1x1 conv's dgrad epilogue
        # conv (+bias +ReLU) -> 2x2 MaxPool as one launch (pooled epilogue)
        self.fuse_pool = True
        # 2x2 MaxPool -> conv: the MaxPoolGrad in the conv's input-gradient
        # epilogue (the pooled gradient never written)
        self.fuse_unpool = True
        # filters of >= 8 M elements: one packed copy (HWIO), read by the
        # forward too (igemm_nt3's B-transposed form) -- set before the first run
        self.fwd_hwio = True
        # conv1_1's ReLU mask written as bits for conv1_2's input gradient
        # (planner._plan_relu_bits)
        self.relu_bits = True
        # conv -> BatchNorm(+ReLU): the BN output written by the conv epilogue
        self.fuse_bn_out = True
        # the dgamma / dbeta sums of the BN backwards fused into input-gradient
        # launches finished together at the end of backward (two launches per
        # step instead of one or two per BatchNorm; single-process steps)
        self.defer_bn_finish = True
        self._red = None                 # (side stream, compute stream) during a step
        # deferred filter gradients: the kernel too (not only its reduction) on
        # the side stream (1), and the fused filter-gradient + Adam launches (2)
        self.side_wgrad = 2
        # the fused conv6 / conv7 filter-gradient + Adam launches go to the side
        # stream after the next `fused_delay` filter gradients there (the
        # HBM-bound update then overlaps the smaller conv4_x / conv3_x layers
        # instead of starving conv5_x's input gradients: 547 -> 554 img/s at 5-7
        # in round 3; round 6, with conv_halo4 and the update on 256 x 256
        # tiles: 2 -- 592.1 / 590.8 vs 583.6 / 582.8 img/s at 6 on the same box)
        self.fused_delay = 2
        self._pending_fused = []
        # the filter gradients of the first `main_wgrad` convs (the last in the
        # backward: conv1_1 / conv1_2 / conv2_1 in FCN) stay on the compute
        # stream, which has no input gradient left to run then, beside the side
        # stream's remaining filter gradients instead of after them (round 5:
        # 3 over 2 by 0.3 % in five A/B pairs)
        self.main_wgrad = 3
        # data-parallel all-reduce steps: the Adam update of every variable of
        # >= overlap_big_mb MB (FCN conv6 / conv7) as soon as its buckets'
        # collectives complete, on the side stream beside the rest of backward
        # (0: all at the end).  Default since round 6: the world-1 RCCL probe
        # 558.0 vs 555.7 img/s with the side stream on a queue of its own
        self.overlap_big_mb = 64

        self._side = None
        self._adam_ctx = None
        self._ready_filter = None
        self.capture = None    # tests: list -> per-conv buffer records of the last backward
        self.timer = None      # list -> (desc, op, start_event, end_event) per conv launch
        self.timer_match = None   # (desc, op) -> bool: which launches self.timer records (None: all)

    # ------------------------------------------------------------------ vars
    def _ensure_store(self):
        if self.store is None or len(self.store.all_vars) != len(self.graph.variables):
            old = self.store
            self.store = VariableStore(list(self.graph.variables.values()), self.device, self.seed)
            self.store.initialize()
            if old is not None:
                for v in old.all_vars:
                    self.store.assign(v.var_name, old.read(v.var_name))
            self.plans = {}
        return self.store

    def variable_value(self, name):
        return self._ensure_store().read(name)

    def assign(self, name, value):
        self._ensure_store().assign(name, value)

    # ------------------------------------------------------------------- run
    def run(self, fetches, feed_dict=None, as_numpy=True):
        feed_dict = feed_dict or {}
        single = not isinstance(fetches, (list, tuple))
        flist = [fetches] if single else list(fetches)
        if any(_is_op(f, "InitAll") for f in flist):
            self._ensure_store().initialize()
        self._ensure_store()
        out = {}
        rest, post = [], []
        for f in flist:
            if _is_op(f, "InitAll"):
                out[id(f)] = None
            elif _is_op(f, "Assign"):              # zero_ops (Network/main.py:84-85)
                self._run_assign(f)
                out[id(f)] = None
            elif _is_op(f, "ApplyGradients") and _accumulator_pairs(f):
                post.append(f)                      # Adam on accumulated gradients, after the fetches
            else:
                rest.append(f)
        if rest:
            key = (tuple(id(f) for f in rest),
                   tuple(sorted((id(k), tuple(np.shape(v))) for k, v in feed_dict.items())))
            plan = self.plans.get(key)
            if plan is None:
                plan = self._compile(rest, feed_dict)
                self.plans[key] = plan
            out.update(self._execute(plan, feed_dict))
        for f in post:
            self._apply_accumulated(f)
            out[id(f)] = None
        res = []
        for f in flist:
            r = out.get(id(f))
            if as_numpy and isinstance(r, torch.Tensor):
                r = r.cpu().numpy()
            res.append(r)
        return res[0] if single else res

    # ------------------------------------------- accumulate-then-apply template
    def _run_assign(self, op):
        """`var.assign(tf.zeros_like(var))` / `var.assign(constant)` on device."""
        store = self.store
        var, val = op.attrs["var"], op.attrs["value"]
        if isinstance(val, G.Tensor) and val.op.type == "ZerosLike":
            value = 0.0
        else:
            value = G.const_value(val)
        if var.var_name in store.aux:
            t = store.aux[var.var_name]
            if t.dtype == torch.int64:
                t.fill_(int(round(value)))
            else:
                ops.fill(t, value)
            store.aux_version += 1
        else:
            ops.fill(store.param(var.var_name), value)
            store.version += 1

    def _apply_accumulated(self, op):
        """optimizer.apply_gradients([(accum_i, var_i)]) (Network/main.py:98-101):
        TF1 Adam on each var_i with the accumulated gradient accum_i; nothing
        else in the graph runs."""
        store = self.store
        opt = op.attrs["optimizer"]
        names = []
        for acc, var in op.attrs["pairs"]:
            g = store.grad(var.var_name)
            ops.fill(g, 0.0)
            ops.axpy(g.view(-1), store.aux[acc.var_name].view(-1), 1.0)
            names.append(var.var_name)
        self._repack(None)
        self.sync_optimizer_slots()      # after ZeRO-1 steps: whole m / v before a whole-variable Adam
        store.step += 1
        ops.adam_tf1_pack(store.params, store.grads, store.m, store.v, self._adam_plan(names), opt.lr,
                          store.step, opt.beta1, opt.beta2, opt.epsilon, grad_scale=1.0,
                          dtype=self._pack_dtype())
        store.version += 1
        self._packed_version = store.version     # adam_tf1_pack rewrote the packed copies it owns
        self._bump_global_step(op.attrs.get("global_step"))

    def _bump_global_step(self, gs):
        if gs is not None:
            t = self.store.aux.get(gs.var_name)
            if t is None:
                raise ValueError(f"global_step {gs.var_name} must be a non-trainable tf.Variable")
            t.add_(1)

    def _train_spec(self, fetches):
        """The gradient-consuming fetches of one run call as one spec:
        TrainStep (minimize), ApplyGradients over compute_gradients outputs, or
        AssignAdd(accum, [scalar_mul(c,] gradient[)]) accumulation ops."""
        trains = [f for f in fetches if _is_op(f, "TrainStep")]
        applies = [f for f in fetches if _is_op(f, "ApplyGradients")]
        accs = [f for f in fetches if _is_op(f, "AssignAdd")]
        if len(trains) + len(applies) + (1 if accs else 0) > 1:
            raise NotImplementedError("one train / apply_gradients / accumulate group per run call")
        if trains:
            a = trains[0].attrs
            return _TrainSpec(trains[0].inputs[0], a["optimizer"], a["var_list"], a["grad_scale"],
                              a.get("global_step"), [], [trains[0]])
        if applies:
            op = applies[0]
            loss, scales, vars_ = None, set(), []
            for g, v in op.attrs["pairs"]:
                lss, var, sc = _gradient_source(g)
                if var is not v:
                    raise NotImplementedError("apply_gradients: gradient paired with a different variable")
                if loss is not None and lss is not loss:
                    raise NotImplementedError("apply_gradients: gradients of different losses")
                loss = lss
                scales.add(sc)
                vars_.append(v)
            if len(scales) != 1:
                raise NotImplementedError("apply_gradients: one gradient scale for all variables")
            return _TrainSpec(loss, op.attrs["optimizer"], vars_, scales.pop(), op.attrs.get("global_step"),
                              [], [op])
        if accs:
            loss, vars_, acc = None, [], []
            for op in accs:
                lss, var, sc = _gradient_source(op.attrs["value"])
                if loss is not None and lss is not loss:
                    raise NotImplementedError("assign_add: gradients of different losses")
                loss = lss
                if op.attrs["var"].trainable:
                    raise NotImplementedError("assign_add target must be a non-trainable accumulator")
                if tuple(op.attrs["var"].shape) != tuple(var.shape):
                    raise ValueError(f"{op.attrs['var'].var_name}: accumulator shape != {var.var_name}")
                vars_.append(var)
                acc.append((op.attrs["var"].var_name, var.var_name, sc))
            return _TrainSpec(loss, None, vars_, 1.0, None, acc, accs)
        return None

    # --------------------------------------------------------------- compile
    def _compile(self, fetches, feed_dict):
        g = self.graph
        store = self.store
        p = Plan()
        p.fetches = fetches
        p.train = self._train_spec(fetches)
        train_ops = {id(o) for o in p.train.ops} if p.train else set()
        stray = [f for f in fetches if isinstance(f, G.Op) and id(f) not in train_ops]
        if stray:
            raise NotImplementedError(f"cannot fetch {stray[0]!r} here")
        roots = [f for f in fetches if not isinstance(f, G.Op)]
        if p.train:
            roots.append(p.train.inputs[0])

        # ---- needed ops (ancestors of the fetches), topological = creation order
        needed = set()
        stack = [t.op for t in roots]
        while stack:
            op = stack.pop()
            if op.id in needed:
                continue
            needed.add(op.id)
            stack.extend(t.op for t in op.inputs)
        order = [op for op in g.ops if op.id in needed]
        consumers = {}
        for op in order:
            for t in op.inputs:
                consumers.setdefault(id(t), []).append(op)
        fetched = {id(t) for t in roots}

        # ---- concrete shapes
        shp = {}
        feeds = {id(k): v for k, v in feed_dict.items()}
        for op in order:
            y = op.outputs[0]
            if op.type == "Placeholder":
                if id(y) not in feeds:
                    raise ValueError(f"placeholder {op.name} must be fed")
                shp[id(y)] = tuple(np.shape(feeds[id(y)]))
            elif op.type == "VariableV2":
                shp[id(y)] = tuple(y.shape)
            else:
                shp[id(y)] = self._infer(op, shp)
        p.shapes = shp

        # ---- which tensors need gradients (depend on a trainable variable)
        needs_grad = set()
        if p.train:
            var_ids = {id(v) for v in p.train.attrs["var_list"]}
            for op in order:
                if op.type == "VariableV2" and id(op.outputs[0]) in var_ids:
                    needs_grad.add(id(op.outputs[0]))
                elif any(id(t) in needs_grad for t in op.inputs):
                    needs_grad.add(id(op.outputs[0]))
        p.needs_grad = needs_grad

        # ---- fusion into nodes
        def single_consumer(t, type_):
            cs = consumers.get(id(t), [])
            if len(cs) == 1 and cs[0].type == type_ and id(t) not in fetched:
                return cs[0]
            return None

        absorbed = set()
        nodes = []
        for op in order:
            if op.id in absorbed or op.type in ("VariableV2",):
                continue
            t = op.type
            y = op.outputs[0]
            if t == "Conv2D":
                x, w = op.inputs
                chain = [op]
                bias = relu = None
                kp = None
                cur = y
                nxt = single_consumer(cur, "BiasAdd")
                if nxt is not None and nxt.inputs[0] is cur:
                    bias = nxt.inputs[1]
                    chain.append(nxt)
                    cur = nxt.outputs[0]
                nxt = single_consumer(cur, "Relu")
                if nxt is not None:
                    relu = True
                    chain.append(nxt)
                    cur = nxt.outputs[0]
                if relu or self.fuse_dropout:
                    # Conv [+BiasAdd] [+Relu] + Dropout: applied in the epilogue (without
                    # a ReLU the gradient re-draws the mask: seg_dropout_bwd_ch)
                    nxt = single_consumer(cur, "Dropout")
                    if nxt is not None:
                        kp = nxt.attrs["keep_prob"]
                        chain.append(nxt)
                        cur = nxt.outputs[0]
                for c in chain[1:]:
                    absorbed.add(c.id)
                nodes.append(_Node("conv", chain, [x], cur, w=w, bias=bias, relu=bool(relu), kp=kp,
                                   stride=op.attrs["stride"], dilation=op.attrs["dilation"],
                                   padding=op.attrs["padding"]))
            elif t == "Conv2DTranspose":
                x, w = op.inputs
                chain = [op]
                bias = res = None
                cur = y
                nxt = single_consumer(cur, "BiasAdd")
                if nxt is not None and nxt.inputs[0] is cur:
                    bias = nxt.inputs[1]
                    chain.append(nxt)
                    cur = nxt.outputs[0]
                nxt = single_consumer(cur, "Add")
                if nxt is not None:
                    a, b = nxt.inputs
                    other = b if a is cur else a
                    if shp[id(other)] == shp[id(nxt.outputs[0])] and other is not cur:
                        res = other
                        chain.append(nxt)
                        cur = nxt.outputs[0]
                for c in chain[1:]:
                    absorbed.add(c.id)
                nodes.append(_Node("tconv", chain, [x], cur, w=w, bias=bias, residual=res,
                                   stride=op.attrs["stride"], padding=op.attrs["padding"],
                                   output_shape=op.attrs["output_shape"]))
            elif t == "FusedBatchNorm":
                x, gamma, beta = op.inputs
                chain = [op]
                cur = y
                relu = False
                nxt = single_consumer(cur, "Relu")
                if nxt is not None:
                    relu = True
                    chain.append(nxt)
                    cur = nxt.outputs[0]
                    absorbed.add(nxt.id)
                nodes.append(_Node("bn", chain, [x], cur, gamma=gamma, beta=beta, relu=relu,
                                   eps=op.attrs["epsilon"]))
            elif t == "SoftmaxXent":
                logits, labels = op.inputs
                mean = single_consumer(y, "Mean")
                if mean is None:
                    raise NotImplementedError("softmax_cross_entropy_with_logits must feed reduce_mean")
                absorbed.add(mean.id)
                nodes.append(_Node("xent", [op, mean], [logits], mean.outputs[0], labels=labels,
                                   valid_hw=op.attrs["valid_hw"]))
            elif t == "Placeholder":
                nodes.append(_Node("input", [op], [], y))
            elif t in ("MaxPool", "AvgPool", "Add", "Relu", "Dropout", "BiasAdd", "ConcatV2",
                       "ResizeBilinear", "ArgMax", "ExpandDims", "Softmax", "GlobalAvgPool"):
                nodes.append(_Node(t, [op], list(op.inputs), y))
            elif t == "Mean":
                raise NotImplementedError("reduce_mean is only supported on the xent loss")
            else:
                raise NotImplementedError(f"op {t} is not on the hot path")
        p.nodes = nodes
        p.fetched = fetched
        self._fold_bn_prologues(p, fetched)
        self._fold_dropout_grads(p, fetched)
        self._allocate(p, consumers, feeds)
        return p

    @property
    def _dpa(self):
        """The DataParallel whose collectives run (None: single process, or
        world 1 where every collective is the identity)."""
        return self.dp if (self.dp is not None and self.dp.active) else None

    def side_stream(self):
        """The side stream of this Session's device (side_stream_for)."""
        if self._side is None:
            self._side = side_stream_for(self.device)
        return self._side

    def sync_optimizer_slots(self):
        """After ZeRO-1 steps each rank's Adam m / v are current on its own
        slices only: gather them (checkpoints, tests)."""
        if self._dpa is not None and self.store is not None and self.dp.store is self.store:
            self.dp.gather_slots()

    def _zero_update(self, p, opt, gs):
        """ZeRO-1 (dp.py): TF1 Adam on this rank's reduce-scattered slices of
        the variables being trained, the updated fp32 slices all-gathered in
        place, then every packed compute copy rewritten from the full
        parameters in one launch (seg_pack_segments)."""
        store = self.store
        key = ("zero", tuple(p.adam_names), len(store.packed))
        ranges = self._adam_groups.get(key)
        if ranges is None:
            spans = sorted((store.offset[nm], store.offset[nm] + int(np.prod(store.by_name[nm].shape)))
                           for nm in p.adam_names)
            starts = sorted(store.offset.values())
            ranges = []
            for a, b in self.dp.owned_ranges():
                for s0, e0 in spans:
                    lo, hi = max(a, s0), min(b, e0)
                    if lo >= hi:
                        continue
                    # merge over a gap that is only 16-byte alignment padding
                    # (zeros, which Adam leaves zero) -- never over a variable
                    # outside var_list
                    if ranges and lo - ranges[-1][1] <= 3 and not any(ranges[-1][1] <= o < lo for o in starts):
                        ranges[-1] = (ranges[-1][0], hi)
                    else:
                        ranges.append((lo, hi))
            self._adam_groups[key] = ranges
        for a, b in ranges:
            ops.adam_tf1_step(store.params[a:b], store.grads[a:b], store.m[a:b], store.v[a:b], opt.lr, store.step,
                              opt.beta1, opt.beta2, opt.epsilon, grad_scale=gs)
        self.dp.gather_params()
        ops.pack_segments(store.params, self._adam_plan(p.adam_names), dtype=self._pack_dtype())

    # -------------------------------------------------------------- execute
    def _repack(self, p):
        store = self.store
        if self._packed_version == store.version:
            return
        for (name, mode), (t, ap, bp) in store.packed.items():
            ops.pack_filter(store.param(name), t, ap, bp, mode)
        self._packed_version = store.version

    def _adam_plan(self, names=None):
        """Segment table of the fused Adam + pack launch: every variable of the
        store (or the subset `names`), with the packed copies that exist
        (rebuilt when packs are added)."""
        store = self.store
        key = (len(store.packed), store.numel)
        if names is not None:
            gk = (key, tuple(names))
            plan = self._adam_groups.get(gk)
            if plan is None:
                plan = ops.AdamPlan(self._adam_segments(set(names)), self.device)
                self._adam_groups[gk] = plan
            return plan
        if self._adam_key == key:
            return self._adam
        self._adam = ops.AdamPlan(self._adam_segments(None), self.device)
        self._adam_key = key
        return self._adam

    def _adam_segments(self, subset):
        store = self.store
        segs = []
        for v in store.order:
            if subset is not None and v.var_name not in subset:
                continue
            shape = tuple(v.shape)
            n = int(np.prod(shape))
            if len(shape) == 4:
                rs, a, b = shape[0] * shape[1], shape[2], shape[3]
            else:
                rs, a, b = 1, 1, n
            rows = tr = None
            for mode in (ops.PACK_KRSC, ops.PACK_HWIO, ops.PACK_TCONV_FWD, ops.PACK_TCONV_BWD):
                e = store.packed.get((v.var_name, mode))
                if e is None:
                    continue
                if mode in (ops.PACK_HWIO, ops.PACK_TCONV_FWD):
                    rows = e
                else:
                    tr = e
            segs.append((store.offset[v.var_name], rs, a, b, rows, tr))
        return segs

    def _feed(self, p, feed_dict):
        feeds = {id(k): v for k, v in feed_dict.items()}
        # scalars (keep_probability) are read at launch time, not staged
        scal = {id(k): float(v) for k, v in feed_dict.items() if np.ndim(v) == 0}
        for tid, (kind, stage) in p.feed_slots.items():
            v = feeds[tid]
            if kind == "scalar":
                scal[tid] = float(v)
                continue
            src = _np(v)
            if kind == "image" and src.is_cuda and src.dtype == torch.uint8 and src.is_contiguous() \
                    and src.shape == stage.shape:
                ops.prepare_input(src, p.buf[tid])   # augmented uint8 batch resident in HBM
                continue
            if src.is_cuda and src.dtype == stage.dtype and src.is_contiguous() and src.shape == stage.shape:
                src_dev = src                      # resident in HBM: no copy
            else:
                stage.copy_(src.to(stage.dtype) if src.dtype != stage.dtype else src, non_blocking=True)
                src_dev = stage
            if kind == "image":
                ops.prepare_input(src_dev, p.buf[tid])
            else:
                p.buf[tid] = src_dev
        return scal

    def _kp(self, kp, scal):
        if kp is None:
            return 1.0
        if isinstance(kp, G.Tensor):
            return scal[id(kp)]
        return float(kp)

    def _execute(self, p, feed_dict):
        self.run_count += 1
        # packed filter copies are current from here on; every update below
        # (fused filter-gradient + Adam, adam_tf1_pack) rewrites the copies of
        # the variables it changes, so they stay current after the step
        self._repack(p)
        self._check_bn_stats(p)
        scal = self._feed(p, feed_dict)
        buf = p.buf
        store = self.store
        step_seed = (self.seed * 1000003 + self.run_count * 7919) & 0xFFFFFFFF
        if self.dp is not None:
            step_seed ^= (self.dp.rank + 1) * _SEED_MIX
        out = {}
        # ---------------- forward
        for i, n in enumerate(p.nodes):
            k = n.kind
            if k == "input":
                continue
            y = buf[id(n.output)]
            if k == "conv":
                x = buf[id(n.inputs[0])]
                kp = self._kp(n.kp, scal)
                n.kp_val = kp
                n.seed_val = (step_seed + i * 131) & 0xFFFFFFFF
                epi = ops.epilogue(bias=store.param(n.bias.var_name) if n.bias is not None else None,
                                   relu=n.relu, keep_prob=kp, seed=n.seed_val)
                if id(n) in p.bn_out2:
                    b2 = p.bn_out2[id(n)]
                    b = getattr(n, "pro", None)
                    self._timed(n.desc, ops.OP_FWD_PRO if b is not None else ops.OP_FWD, ops.conv2d_fwd_bn2, n.desc,
                                x if b is None else buf[id(b.inputs[0])], None if b is None else self._prologue(b),
                                store.packed[(n.w.var_name, ops.PACK_KRSC)][0], y, buf[id(b2.output)],
                                store.param(b2.gamma.var_name), store.param(b2.beta.var_name), b2.relu, b2.eps,
                                epi, self.ws)
                elif getattr(n, "pro", None) is not None:
                    b = n.pro
                    self._timed(n.desc, ops.OP_FWD_PRO, ops.conv2d_fwd_pro, n.desc, buf[id(b.inputs[0])],
                                self._prologue(b), store.packed[(n.w.var_name, ops.PACK_KRSC)][0], y, epi, self.ws)
                elif id(n) in p.pool_fuse:
                    m = p.pool_fuse[id(n)]
                    self._timed(n.desc, ops.OP_FWD, ops.conv2d_fwd_pool, n.desc, x,
                                store.packed[(n.w.var_name, ops.PACK_KRSC)][0], buf[id(m.output)],
                                p.pool_idx.get(id(m)), epi, self.ws)
                elif getattr(n, "fwd_hwio", False):
                    self._timed(n.desc, ops.OP_FWD, ops.conv2d_fwd_hwio, n.desc, x,
                                store.packed[(n.w.var_name, ops.PACK_HWIO)][0], y, epi, self.ws)
                elif id(n) in getattr(p, "mask_bits", {}):
                    self._timed(n.desc, ops.OP_FWD, ops.conv2d_fwd_relu_bits, n.desc, x,
                                store.packed[(n.w.var_name, ops.PACK_KRSC)][0], y, p.mask_bits[id(n)], epi)
                else:
                    self._timed(n.desc, ops.OP_FWD, ops.conv2d_fwd, n.desc, x,
                                store.packed[(n.w.var_name, ops.PACK_KRSC)][0], y, epi, self.ws)
            elif k == "tconv":
                x = buf[id(n.inputs[0])]
                res = buf[id(n.residual)] if n.residual is not None else None
                epi = ops.epilogue(bias=store.param(n.bias.var_name) if n.bias is not None else None,
                                   residual=res)
                self._timed(n.desc, ops.OP_TFWD, ops.tconv2d_fwd, n.desc, x,
                            store.packed[(n.w.var_name, ops.PACK_TCONV_FWD)][0], y, epi, self.ws)
            elif k == "MaxPool":
                idx = p.pool_idx.get(id(n))
                if id(n) in p.pool_fused:
                    pass                       # written by the producing conv's pooled epilogue
                elif idx is not None:
                    ops.maxpool2x2_fwd_argmax(buf[id(n.inputs[0])], y, idx)
                else:
                    ops.maxpool2x2_fwd(buf[id(n.inputs[0])], y)
            elif k == "AvgPool":
                ops.avgpool2x2_fwd(buf[id(n.inputs[0])], y)
            elif k == "Add":
                ops.add(buf[id(n.inputs[0])], buf[id(n.inputs[1])], y)
            elif k == "bn":
                if id(n) in p.folded or id(n) in p.bn_out2_done:
                    continue                        # applied by its conv's operand prologue / written by its conv
                C = p.shapes[id(n.inputs[0])][3]
                ops.bn_relu_fwd(buf[id(n.inputs[0])], y, store.param(n.gamma.var_name),
                                store.param(n.beta.var_name), C, n.relu, n.eps)
            elif k == "Relu":
                self._relu_fwd(buf[id(n.inputs[0])], y)
            elif k == "Dropout":
                kp = self._kp(n.ops[0].attrs["keep_prob"], scal)
                n.kp_val = kp
                n.seed_val = (step_seed + i * 131) & 0xFFFFFFFF
                if kp < 1.0:
                    ops.dropout_fwd(buf[id(n.inputs[0])], y, kp, n.seed_val)
                else:
                    ops.copy_channels(buf[id(n.inputs[0])], y)
            elif k == "xent":
                lg = buf[id(n.inputs[0])]
                labels = buf[id(n.labels)]
                ops.softmax_xent(lg, labels, n.dlogits, n.loss_sum, n.num_classes, n.valid_hw,
                                 grad_scale=(self.loss_scale if p.train else 1.0) / n.count, ws=self.ws)
            elif k == "ConcatV2":
                if id(n) not in p.alias_nodes:      # aliased: the parts already sit in place
                    ops.concat_fwd([(buf[id(t)], p.shapes[id(t)][3]) for t in n.inputs], y,
                                   p.shapes[id(n.output)][3])
            elif k == "ArgMax":
                x = buf[id(n.inputs[0])]
                C = p.shapes[id(n.inputs[0])][3]
                ops.argmax(x, y.view(-1), C)
            elif k == "Softmax":
                ops.softmax(buf[id(n.inputs[0])], y, p.shapes[id(n.inputs[0])][3])
            elif k == "ResizeBilinear":
                x = buf[id(n.inputs[0])]
                if x.shape[1] == 1 and x.shape[2] == 1:      # align_corners from 1x1: a broadcast
                    ops.spatial_broadcast(x, y, 1.0)
                else:
                    ops.resize_bilinear_fwd(x, y)
            elif k == "GlobalAvgPool":
                x = buf[id(n.inputs[0])]
                ops.spatial_reduce(x, y, 1.0 / (x.shape[1] * x.shape[2]), self.ws)
            elif k == "ExpandDims":
                pass
            else:
                raise NotImplementedError(k)
        # ---------------- backward + optimizer
        if p.train:
            ts = p.train.attrs
            opt = ts["optimizer"]
            dpa = self._dpa
            world = dpa.world if dpa is not None else 1
            S = self.loss_scale                     # the scale this step's loss gradient carries
            scaled = S != 1.0
            gs = ts["grad_scale"] / world / S
            if scaled and self.overlap_optimizer:
                raise NotImplementedError("loss scaling needs the whole gradient checked before any update")
            if opt is not None:
                store.step += 1
            self._fused = None
            if opt is not None and self.fuse_adam and dpa is None and not self.overlap_optimizer \
                    and not scaled and p.adam_fusable:
                self._fused = (opt, gs, set())
            # ZeRO-1 exchange for an Adam step (dp.py); the accumulate template
            # and the overlapped per-layer optimizer read whole gradients
            zero = (dpa is not None and dpa.shard and opt is not None and not self.overlap_optimizer
                    and not p.train.accum)
            if dpa is not None:
                dpa.mode = "zero" if zero else "allreduce"
                if opt is not None and not zero and dpa.slots_stale:
                    # a whole-variable Adam after ZeRO-1 steps: gather the m / v
                    # slices of the other ranks first, or the replicas diverge
                    self.sync_optimizer_slots()
            self._red = None
            if self.defer_wgrad_reduce and self.device.type == "cuda":
                # (with the overlapped optimizer the reductions and each layer's
                # Adam share the side stream: a layer's reduction precedes its update)
                self._red = (self.side_stream(), torch.cuda.current_stream(self.device))
                if dpa is not None:
                    dpa.launch_streams = self._red
            if opt is not None and self.overlap_optimizer and self.device.type == "cuda":
                # per-layer Adam on a side stream as soon as the layer's gradient is final
                self._adam_ctx = _AdamOverlap(self, opt, gs, p.var_set)
                if dpa is not None:
                    dpa.on_launch = self._adam_ctx.after_work
            elif (opt is not None and dpa is not None and not zero and self.overlap_big_mb and not scaled
                  and not p.train.accum and self.device.type == "cuda"):
                self._adam_ctx = _AdamOverlap(self, opt, gs, p.var_set, big_only=True)
                dpa.on_launch = self._adam_ctx.after_work
            if dpa is not None and p.never_ready:
                dpa.ready(p.never_ready)
            self._ready_filter = p.var_set
            ok = False
            try:
                self._backward(p, scal)
                self._tick_fused(flush=True)
                ok = True
            finally:
                # on an exception: no stale fused conv6 / conv7 update is left
                # for the next step, and the compute stream does not run ahead
                # of side-stream kernels still reading this step's buffers
                self._ready_filter = None
                if not ok:
                    self._pending_fused = []
                    self._fused = None
                    self._adam_ctx = None
                if self._red is not None:        # pending filter-gradient reductions done before Adam
                    self._red[1].wait_stream(self._red[0])
                    self._red = None
                if dpa is not None:
                    if ok:
                        dpa.finish()
                    else:
                        dpa.abort_step()
                    dpa.on_launch = None
                    dpa.launch_streams = None
            if scaled and not self._grads_finite():
                # overflow in the scaled fp16 gradients: no update this step
                # (TF LossScaleOptimizer), halve the scale
                self.skipped_steps += 1
                if opt is not None:
                    store.step -= 1
                self.loss_scale = max(self.loss_scale / 2.0, 1.0)
                self.good_steps = 0
                opt = None
                p_accum = []
            else:
                p_accum = p.train.accum
                if scaled and self.dynamic_scale:
                    self.good_steps += 1
                    if self.good_steps >= self.scale_increment_period:
                        self.loss_scale *= 2.0
                        self.good_steps = 0
            if opt is None:
                # accumulate template: accum += const * grad (Network/main.py:92-95)
                for acc, var, sc in p_accum:
                    ops.axpy(store.aux[acc].view(-1), store.grad(var).view(-1), sc / world / S)
                store.aux_version += 1
            elif self._adam_ctx is not None:
                self._adam_ctx.finish()
                self._adam_ctx = None
            elif zero:
                self._zero_update(p, opt, gs)
            else:
                done = self._fused[2] if self._fused is not None else set()
                rest = [nm for nm in p.adam_names if nm not in done]
                if rest:
                    ops.adam_tf1_pack(store.params, store.grads, store.m, store.v, self._adam_plan(rest), opt.lr,
                                      store.step, opt.beta1, opt.beta2, opt.epsilon, grad_scale=gs,
                                      dtype=self._pack_dtype())
            self._fused = None
            if opt is not None:
                store.version += 1
                self._packed_version = store.version
                self._bump_global_step(ts.get("global_step"))
        # ---------------- fetch values
        for f in p.fetches:
            if isinstance(f, G.Op):
                out[id(f)] = None
                continue
            t = buf.get(id(f))
            node = next((n for n in p.nodes if n.output is f), None)
            if node is not None and node.kind == "xent":
                out[id(f)] = (t / node.count).reshape(())
            elif f.dtype == G.int64:
                out[id(f)] = t
            else:
                C = p.shapes[id(f)][3]
                out[id(f)] = t[..., :C].float()
        return out

    def _relu_fwd(self, x, y):
        C = x.shape[-1]
        one = torch.ones(C, dtype=torch.float32, device=self.device)
        zero = torch.zeros(C, dtype=torch.float32, device=self.device)
        ops.bn_relu_fwd(x, y, one, zero, C, True, eps=0.0)

    def _pack_dtype(self):
        return self.cdt

    def _grad_ready(self, names):
        """The gradients of `names` are final once the kernels enqueued so far
        run: hand them to the all-reduce (DP) or straight to the overlapped
        optimizer."""
        if self._ready_filter is not None:
            names = [nm for nm in names if nm in self._ready_filter]
        if self._dpa is not None:
            self.dp.ready(names)
        elif self._adam_ctx is not None:
            self._adam_ctx.launch(names)

    def _mask_epi(self, p, x):
        """Epilogue fusing the ReluGrad (x 1/keep_prob) of x's producer into the
        input-gradient kernel of x's (only) consumer, or None."""
        prod = p.producer.get(id(x))
        if prod is None or id(prod) not in p.mask_fuse:
            return None
        kp = prod.kp_val
        scale = 1.0 / kp if (kp is not None and kp < 1.0) else 1.0
        return ops.epilogue(relu_mask=p.buf[id(x)], mask_scale=scale)

    # ------------------------------------------------------------- backward
    def _backward(self, p, scal):
        buf = p.buf
        store = self.store
        grad = {}
        ws = self.ws
        ng = p.needs_grad

        def zeros_for(t):
            # (a pool-fused conv's output has no buffer: only its shape)
            return torch.zeros_like(buf[id(t)]) if buf[id(t)] is not None else self._act(p.shapes[id(t)])

        def dest(t):
            """(buffer to write t's gradient into, accumulate-after flag)."""
            if id(t) not in grad:
                gbuf = p.tmp.get(("g", id(t)))
                if gbuf is None:
                    gbuf = zeros_for(t)
                    p.tmp[("g", id(t))] = gbuf
                grad[id(t)] = gbuf
                return gbuf, None
            tmp = p.tmp.get(("acc", id(t)))
            if tmp is None:
                tmp = zeros_for(t)
                p.tmp[("acc", id(t))] = tmp
            return tmp, grad[id(t)]

        def done(dst, acc):
            if acc is not None:
                ops.add(acc, dst, acc)

        def gdst(name):
            """Where a variable's gradient is written: its slice of the flat
            buffer when it is in var_list; otherwise a scratch sink, so the
            slices the data-parallel buckets release up front (never_ready) are
            not written while their all-reduce may be reading them."""
            if name in p.var_set:
                return store.grad(name)
            t = p.tmp.get(("gscratch", name))
            if t is None:
                t = torch.zeros_like(store.grad(name))
                p.tmp[("gscratch", name)] = t
            return t

        ginit = set()      # aliased-concat roots whose gradient buffer holds data this step

        # deferred BN-backward finishes: (segment, variable names) per fused launch
        bn_defer = ([] if (self.defer_bn_finish and self._dpa is None and self._adam_ctx is None
                           and self.device.type == "cuda") else None)

        def bn_part(n):
            """Persistent partial-row buffer of node n's fused BN backward."""
            t = p.tmp.get(("bnpart", id(n)))
            if t is None:
                t = torch.empty(max(1, ops.conv_bwd_data_bn_part_rows(n.desc)) * 2 * n.desc.C,
                                dtype=torch.float32, device=self.device)
                p.tmp[("bnpart", id(n))] = t
            return t

        def adest(t):
            """Slice of the root's gradient buffer for aliased t, and whether the
            kernel must accumulate into it (False only for the first write
            when it covers the whole root)."""
            r, off = p.alias[id(t)]
            dB = p.tmp.get(("ga", r))
            if dB is None:
                dB = torch.zeros_like(buf[r])
                p.tmp[("ga", r)] = dB
            C = p.shapes[id(t)][3]
            view = dB[..., off:off + C]
            grad[id(t)] = view
            if r not in ginit:
                ginit.add(r)
                if off == 0 and C == p.shapes[r][3]:
                    return view, False
                dB.zero_()
            return view, True

        if not hasattr(p, "ncons"):
            p.ncons = collections.Counter(id(i) for m in p.nodes
                                          for i in list(m.inputs) + [getattr(m, "residual", None)] if i is not None)

        def contribute_alias(t, g):
            if id(t) not in ng:
                return
            if id(t) not in grad:
                # share the buffer only when no later contribution will add into
                # it (side-stream filter gradients may still be reading g)
                grad[id(t)] = g if p.ncons[id(t)] <= 1 else g.clone()
            else:
                ops.add(grad[id(t)], g, grad[id(t)])

        main_wg = set()
        if self._red is not None and self.main_wgrad > 0:
            convs = [m for m in p.nodes if m.kind == "conv" and m.w.var_name in p.var_set
                     and getattr(m, "pro", None) is None and id(m) not in p.adam_fusable]
            main_wg = {id(m) for m in convs[:self.main_wgrad]}

        for n in reversed(p.nodes):
            k = n.kind
            if k == "input" or id(n.output) not in ng:
                continue
            if id(n) in p.alias_nodes:
                # concat as a view: its parts' gradients are slices of the
                # root's buffer, which the consumers accumulated into
                r = p.alias[id(n.output)][0]
                if r in ginit:
                    dB = p.tmp[("ga", r)]
                    for t in n.inputs:
                        if id(t) in ng and id(t) not in grad:
                            off = p.alias[id(t)][1]
                            grad[id(t)] = dB[..., off:off + p.shapes[id(t)][3]]
                continue
            if k == "xent":
                contribute_alias(n.inputs[0], n.dlogits)
                continue
            dy = grad.get(id(n.output))
            if dy is None:
                continue          # output does not reach the loss
            if k == "conv":
                x = n.inputs[0]
                yb = buf[id(n.output)]
                dz = dy
                fused_db = None
                if not n.relu and n.kp_val is not None and n.kp_val < 1.0 and id(n) not in p.drop_folded:
                    # dropout applied in the forward epilogue, no ReLU: re-draw its mask
                    dz = p.tmp.get(("dz", id(n.output)))
                    if dz is None:
                        dz = torch.zeros_like(yb)
                        p.tmp[("dz", id(n.output))] = dz
                    ops.dropout_bwd_ch(dy, dz, n.desc.k_valid, n.kp_val, n.seed_val)
                    if n.bias is not None:
                        fused_db = gdst(n.bias.var_name)
                elif id(n) in p.mask_fuse or (n.bias is not None and not n.relu):
                    # gradient arrives masked (or there is no ReLU): BiasAddGrad is
                    # summed by the filter-gradient launch below
                    if n.bias is not None:
                        fused_db = gdst(n.bias.var_name)
                elif n.relu or n.bias is not None:
                    scale = 1.0 / n.kp_val if (n.kp_val is not None and n.kp_val < 1.0) else 1.0
                    dz = p.tmp.get(("dz", id(n.output)))
                    if dz is None:
                        dz = torch.zeros_like(yb)
                        p.tmp[("dz", id(n.output))] = dz
                    db = gdst(n.bias.var_name) if n.bias is not None else None
                    K = n.desc.k_valid
                    self._bias_relu_bwd(dy, yb if n.relu else None, dz, db, K, n.relu, scale)
                dx = None
                dx_base = None
                unpool = None       # tests: (full-res gradient, switches, relu) of a fused MaxPoolGrad
                bnb = None          # tests: record of a BatchNorm backward run in this conv's dgrad epilogue
                pro = getattr(n, "pro", None)
                if (id(x) in ng and pro is not None and self.fuse_bn_bwd and id(pro.inputs[0]) in ng
                        and ops.conv_bwd_data_bn_workspace(n.desc) > 0):
                    # input gradient carried through the folded BatchNorm(+ReLU)
                    # backward in the same launch: the BN node's own backward is
                    # skipped (its output gradient is never materialised)
                    xb = pro.inputs[0]
                    if id(xb) in p.alias:
                        dxb, accf = adest(xb)
                        acc = None
                    else:
                        (dxb, acc), accf = dest(xb), False
                    gn, bn_ = pro.gamma.var_name, pro.beta.var_name
                    if self.capture is not None:
                        bnb = {"xb": buf[id(xb)], "gamma": gn, "beta": bn_, "eps": pro.eps, "relu": pro.relu,
                               "base": dxb.clone() if accf else None, "drop": None, "folded": True}
                    if bn_defer is not None:
                        part = bn_part(n)
                        self._timed(n.desc, ops.OP_BWD_DATA_BN, ops.conv2d_bwd_data_bn_part, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], buf[id(xb)], store.param(gn),
                                    store.param(bn_), dxb, part, pro.eps, pro.relu, accf)
                        bn_defer.append(((part, ops.conv_bwd_data_bn_part_rows(n.desc), n.desc.C, n.desc.c_valid,
                                          pro.eps, gdst(gn), gdst(bn_)), [gn, bn_]))
                    else:
                        self._timed(n.desc, ops.OP_BWD_DATA_BN, ops.conv2d_bwd_data_bn, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], buf[id(xb)], store.param(gn),
                                    store.param(bn_), dxb, gdst(gn), gdst(bn_), pro.eps, pro.relu, accf, ws)
                    if bnb is not None:
                        bnb["dxb"] = dxb.clone()
                        bnb["kernel"] = ops.conv_kernel_info(n.desc, ops.OP_BWD_DATA_BN)[0]
                    done(dxb, acc)
                    if bn_defer is None:
                        self._grad_ready([gn, bn_])
                elif (id(x) in ng and id(n) in p.bn_before and self.fuse_bn_bwd
                      and id(p.bn_before[id(n)].inputs[0]) in ng and id(p.bn_before[id(n)].inputs[0]) not in p.alias
                      and id(p.bn_before[id(n)].inputs[0]) not in grad
                      and ops.conv_bwd_data_bn_workspace(n.desc) > 0):
                    # growth conv: its input gradient continues through the BN
                    # (+ the dropout before it) that produced its input
                    b = p.bn_before[id(n)]
                    xb = b.inputs[0]
                    dxb, acc = dest(xb)
                    c1 = p.drop_fold.get(id(b))
                    drop = (c1.kp_val, c1.seed_val) if (c1 is not None and c1.kp_val is not None
                                                         and c1.kp_val < 1.0) else None
                    gn, bn_ = b.gamma.var_name, b.beta.var_name
                    if bn_defer is not None:
                        part = bn_part(n)
                        self._timed(n.desc, ops.OP_BWD_DATA_BN, ops.conv2d_bwd_data_bn_part, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], buf[id(xb)], store.param(gn),
                                    store.param(bn_), dxb, part, b.eps, b.relu, False, None, drop)
                        bn_defer.append(((part, ops.conv_bwd_data_bn_part_rows(n.desc), n.desc.C, n.desc.c_valid,
                                          b.eps, gdst(gn), gdst(bn_)), [gn, bn_]))
                    else:
                        self._timed(n.desc, ops.OP_BWD_DATA_BN, ops.conv2d_bwd_data_bn, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], buf[id(xb)], store.param(gn),
                                    store.param(bn_), dxb, gdst(gn), gdst(bn_), b.eps, b.relu, False, ws,
                                    None, drop)
                    if self.capture is not None:
                        bnb = {"xb": buf[id(xb)], "gamma": gn, "beta": bn_, "eps": b.eps, "relu": b.relu,
                               "base": None, "drop": drop, "folded": False, "dxb": dxb.clone(),
                               "kernel": ops.conv_kernel_info(n.desc, ops.OP_BWD_DATA_BN)[0]}
                    done(dxb, acc)
                    if bn_defer is None:
                        self._grad_ready([gn, bn_])
                elif id(n) in p.unpool_fuse:
                    # input gradient continued through the MaxPoolGrad of the pool
                    # before this conv (and its input's ReluGrad): written at the
                    # pool input's resolution; the pooled gradient of the pool's
                    # other consumers (done earlier in backward) is the residual
                    m = p.unpool_fuse[id(n)]
                    xf = m.inputs[0]
                    dxf, accf = dest(xf)
                    prod = p.producer.get(id(xf))
                    res = grad.get(id(x))
                    if res is not None and self.capture is not None:
                        dx_base = res.clone()
                    self._timed(n.desc, ops.OP_BWD_DATA, ops.conv2d_bwd_data_unpool, n.desc, dz,
                                store.packed[(n.w.var_name, ops.PACK_HWIO)][0], p.pool_idx[id(m)], dxf,
                                prod is not None and id(prod) in p.mask_fuse, res, ws)
                    if self.capture is not None:
                        unpool = (dxf.clone(), p.pool_idx[id(m)], prod is not None and id(prod) in p.mask_fuse)
                    done(dxf, accf)
                elif id(x) in ng and id(x) in p.alias:
                    # the input is an aliased concat root (FC-DenseNet decoder
                    # concat views): the input gradient lands in the shared
                    # gradient buffer -- whole (first write) or accumulated
                    # in the epilogue
                    dx, accf = adest(x)
                    if accf and self.capture is not None:
                        dx_base = dx.clone()
                    self._timed(n.desc, ops.OP_BWD_DATA, ops.conv2d_bwd_data, n.desc, dz,
                                store.packed[(n.w.var_name, ops.PACK_HWIO)][0], dx, ws, None,
                                ops.epilogue(residual=dx) if accf else None)
                elif id(x) in ng:
                    dx, acc = dest(x)
                    mepi = self._mask_epi(p, x)
                    if acc is not None and mepi is None and self.fuse_grad_sum:
                        # a further consumer's contribution: accumulated in the
                        # epilogue, in place (residual = the gradient so far)
                        if self.capture is not None:
                            # tests: the sum before this launch (an extra copy on
                            # the stream; the launch plan is unchanged)
                            dx_base = acc.clone()
                        self._timed(n.desc, ops.OP_BWD_DATA, ops.conv2d_bwd_data, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], acc, ws, None,
                                    ops.epilogue(residual=acc))
                        dx = acc
                    elif mepi is not None and acc is None and id(n) in p.bits_dgrad:
                        # the ReluGrad mask from the producer's bits (planner._plan_relu_bits)
                        self._timed(n.desc, ops.OP_BWD_DATA, ops.conv2d_bwd_data_bits, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0],
                                    p.mask_bits[id(p.producer[id(x)])], dx, mepi.mask_scale, ws)
                        done(dx, acc)
                    else:
                        self._timed(n.desc, ops.OP_BWD_DATA, ops.conv2d_bwd_data, n.desc, dz,
                                    store.packed[(n.w.var_name, ops.PACK_HWIO)][0], dx, ws, None, mepi)
                        done(dx, acc)
                if self.capture is not None:
                    # tests: the buffers of this layer's three kernels (they persist
                    # after the step; dx before any accumulation of later consumers,
                    # or -- accumulated in the epilogue -- with dx_base, the sum it
                    # was added to; None when it went straight through a folded BN
                    # backward)
                    mask = self._mask_epi(p, x) if dx is not None else None
                    self.capture.append({"kind": "conv", "name": n.w.var_name, "bias": getattr(n.bias, "var_name", None),
                                         "x": buf[id(x)] if pro is None else buf[id(pro.inputs[0])],
                                         "pro": None if pro is None else (pro.gamma.var_name, pro.beta.var_name,
                                                                          pro.eps, pro.relu),
                                         "y": buf[id(n.output)], "dz": dz,
                                         # MaxPool fused into the forward: (pooled map, switches)
                                         "pool": ((buf[id(p.pool_fuse[id(n)].output)],
                                                   p.pool_idx.get(id(p.pool_fuse[id(n)])))
                                                  if id(n) in p.pool_fuse else None),
                                         # a copy: later consumers may accumulate into the buffer
                                         "dx": None if dx is None else dx.clone(), "dx_base": dx_base,
                                         "unpool": unpool,
                                         "dx_masked": mask is not None,
                                         "mask_scale": (mask.mask_scale if mask is not None else 1.0),
                                         "relu": n.relu, "keep_prob": n.kp_val, "seed": n.seed_val,
                                         # input gradient through a BatchNorm(+ReLU) backward in
                                         # the dgrad epilogue (igemm_nt2_bn / conv_res16c_bn)
                                         "bn_bwd": bnb,
                                         "fused_adam": False, "desc": n.desc,
                                         "stride": n.stride, "dilation": n.dilation, "padding": n.padding})
                want_w = n.w.var_name in p.var_set
                want_b = n.bias is not None and n.bias.var_name in p.var_set
                gw = store.grad(n.w.var_name) if want_w else self._scratch_grad(p, n.w)
                if not (want_w or want_b):
                    pass          # frozen layer (outside var_list): no filter gradient
                elif getattr(n, "pro", None) is not None:
                    # input relu(BN(x)) recomputed from x while staging (folded BatchNorm);
                    # on the side stream beside the input-gradient chain, as below
                    b = n.pro
                    side = self._wgrad_side(p, n)
                    with self._beside(side):
                        self._timed(n.desc, ops.OP_BWD_FILTER_PRO, ops.conv2d_bwd_filter_pro, n.desc,
                                    buf[id(b.inputs[0])], self._prologue(b), dz, gw,
                                    self._node_ws(p, n) if side is not None else ws, None, fused_db)
                elif self._fused is not None and id(n) in p.adam_fusable and want_w:
                    # Conv2DBackpropFilter + AdamOptimizer on the filter in one launch
                    opt, gs, fdone = self._fused
                    wn = n.w.var_name
                    side = self._wgrad_side(p, n, level=2)

                    def launch_fused(n=n, x=x, dz=dz, wn=wn, fused_db=fused_db, side=side, opt=opt, gs=gs):
                        # on the side stream too: its input gradient (the only reader of the
                        # packed copies it rewrites) is already enqueued on the compute stream
                        with self._beside(side):
                            self._timed(n.desc, ops.OP_BWD_FILTER, ops.conv2d_bwd_filter_adam, n.desc, buf[id(x)],
                                        dz, store.param(wn), store.adam_m(wn), store.adam_v(wn), opt.lr, store.step,
                                        opt.beta1, opt.beta2, opt.epsilon, gs, store.packed.get((wn, ops.PACK_HWIO)),
                                        store.packed.get((wn, ops.PACK_KRSC)),
                                        store.grad(wn) if self.store_fused_grads else None, fused_db,
                                        self._node_ws(p, n) if side is not None else ws)
                    if side is not None and self.fused_delay > 0:
                        # issued after the next `fused_delay` side-stream filter gradients, so
                        # the HBM-bound update does not starve the input-gradient chain early on
                        self._pending_fused.append([self.fused_delay, launch_fused])
                    else:
                        launch_fused()
                    fdone.add(wn)
                    if self.capture is not None:
                        self.capture[-1]["fused_adam"] = True
                elif self._red is not None and self.side_wgrad >= 1 and id(n) not in main_wg:
                    # the whole filter gradient (kernel + split-K reduction) on the
                    # side stream, beside the input-gradient chain: every operand
                    # (x, dz, the per-node workspace) stays untouched until the
                    # join before Adam
                    wsb = p.wg_ws[id(n)]
                    with self._beside(self._red[0]):
                        tok = self._timed(n.desc, ops.OP_BWD_FILTER, ops.conv2d_bwd_filter_begin, n.desc, buf[id(x)],
                                          dz, gw, wsb, fused_db)
                        ops.conv2d_bwd_filter_end(tok, gw, wsb, fused_db)
                    self._tick_fused()
                elif self._red is not None and id(n) not in main_wg:
                    # kernel now, its split-K reduction on the side stream
                    side, main = self._red
                    wsb = p.wg_ws[id(n)]
                    tok = self._timed(n.desc, ops.OP_BWD_FILTER, ops.conv2d_bwd_filter_begin, n.desc, buf[id(x)],
                                      dz, gw, wsb, fused_db)
                    if tok[1][0] > 1:
                        ev = torch.cuda.Event()
                        ev.record(main)
                        side.wait_event(ev)
                        ops.conv2d_bwd_filter_end(tok, gw, wsb, fused_db, stream=side)
                else:
                    self._timed(n.desc, ops.OP_BWD_FILTER, ops.conv2d_bwd_filter, n.desc, buf[id(x)], dz,
                                gw, ws, None, fused_db)
                self._grad_ready([n.w.var_name] + ([n.bias.var_name] if n.bias is not None else []))
            elif k == "tconv":
                x = n.inputs[0]
                if n.residual is not None:
                    contribute_alias(n.residual, dy)
                if id(x) in ng and id(x) in p.alias:
                    # the input is an aliased concat root (decoder concat views)
                    dx, accf = adest(x)
                    self._timed(n.desc, ops.OP_TBWD_DATA, ops.tconv2d_bwd_data, n.desc, dy,
                                store.packed[(n.w.var_name, ops.PACK_TCONV_BWD)][0], dx, ws, None,
                                ops.epilogue(residual=dx) if accf else None)
                elif id(x) in ng:
                    dx, acc = dest(x)
                    self._timed(n.desc, ops.OP_TBWD_DATA, ops.tconv2d_bwd_data, n.desc, dy,
                                store.packed[(n.w.var_name, ops.PACK_TCONV_BWD)][0], dx, ws, None,
                                self._mask_epi(p, x))
                    done(dx, acc)
                want_w = n.w.var_name in p.var_set
                want_b = n.bias is not None and n.bias.var_name in p.var_set
                if want_w or want_b:
                    # on the side stream beside the input-gradient chain (as the conv filter gradients)
                    side = self._wgrad_side(p, n)
                    with self._beside(side):
                        self._timed(n.desc, ops.OP_TBWD_FILTER, ops.tconv2d_bwd_filter, n.desc, buf[id(x)], dy,
                                    store.grad(n.w.var_name) if want_w else self._scratch_grad(p, n.w),
                                    self._node_ws(p, n) if side is not None else ws, None,
                                    gdst(n.bias.var_name) if n.bias is not None else None)
                self._grad_ready([n.w.var_name] + ([n.bias.var_name] if n.bias is not None else []))
            elif k == "MaxPool":
                x = n.inputs[0]
                if id(n) in p.unpool_pools:
                    continue          # done in the consuming conv's input-gradient epilogue
                if id(x) in ng:
                    dx, acc = dest(x)
                    prod = p.producer.get(id(x))
                    relu = prod is not None and id(prod) in p.mask_fuse
                    idx = p.pool_idx.get(id(n))
                    if idx is not None:
                        ops.maxpool2x2_bwd_argmax(idx, dy, dx, relu_mask=relu)
                    else:
                        ops.maxpool2x2_bwd(buf[id(x)], buf[id(n.output)], dy, dx, relu_mask=relu)
                    done(dx, acc)
            elif k == "AvgPool":
                x = n.inputs[0]
                if id(x) in ng:
                    dx, acc = dest(x)
                    ops.avgpool2x2_bwd(dy, dx)
                    done(dx, acc)
            elif k == "Add":
                for t in n.inputs:
                    contribute_alias(t, dy)
            elif k == "ConcatV2":
                parts = []
                for t in n.inputs:
                    if id(t) not in ng:
                        # still consume its channel range: a zero-width part is not allowed,
                        # so write into a scratch gradient that nobody reads
                        g = p.tmp.get(("cz", id(t)))
                        if g is None:
                            g = torch.zeros_like(buf[id(t)])
                            p.tmp[("cz", id(t))] = g
                        parts.append((g, p.shapes[id(t)][3], False))
                        continue
                    if id(t) in p.alias:
                        v, accf = adest(t)
                        parts.append((v, p.shapes[id(t)][3], accf))
                    elif id(t) in grad:
                        parts.append((grad[id(t)], p.shapes[id(t)][3], True))
                    else:
                        g = p.tmp.get(("g", id(t)))
                        if g is None:
                            g = torch.zeros_like(buf[id(t)])
                            p.tmp[("g", id(t))] = g
                        grad[id(t)] = g
                        parts.append((g, p.shapes[id(t)][3], False))
                ops.concat_bwd(dy, parts)
            elif k == "bn":
                x = n.inputs[0]
                C = p.shapes[id(x)][3]
                if id(x) in p.alias:
                    dx, accf = adest(x)
                    acc = None
                else:
                    (dx, acc), accf = dest(x), False
                drop = None
                c = p.drop_fold.get(id(n))
                if c is not None and c.kp_val is not None and c.kp_val < 1.0:
                    if accf or acc is not None:
                        raise RuntimeError(f"{n.ops[0].name}: folded dropout gradient needs a sole reader")
                    drop = (c.kp_val, c.seed_val, c.desc.k_valid)
                ops.bn_relu_bwd(buf[id(x)], buf[id(n.output)], dy, dx, store.param(n.gamma.var_name),
                                gdst(n.gamma.var_name), gdst(n.beta.var_name), C, n.relu,
                                n.eps, ws, accumulate=accf, beta=store.param(n.beta.var_name), dropout=drop)
                done(dx, acc)
                self._grad_ready([n.gamma.var_name, n.beta.var_name])
            elif k == "Relu":
                x = n.inputs[0]
                dx, acc = dest(x)
                self._bias_relu_bwd(dy, buf[id(n.output)], dx, None, p.shapes[id(x)][3], True, 1.0)
                done(dx, acc)
            elif k == "Dropout":
                x = n.inputs[0]
                dx, acc = dest(x)
                if n.kp_val < 1.0:
                    ops.dropout_fwd(dy, dx, n.kp_val, n.seed_val)
                else:
                    ops.copy_channels(dy, dx)
                done(dx, acc)
            elif k == "GlobalAvgPool":
                x = n.inputs[0]
                if id(x) in ng:
                    dx, acc = dest(x)
                    xs = buf[id(x)]
                    ops.spatial_broadcast(dy, dx, 1.0 / (xs.shape[1] * xs.shape[2]))
                    done(dx, acc)
            elif k == "ExpandDims" and len(p.shapes[id(n.output)]) == 4 and len(p.shapes[id(n.inputs[0])]) == 4:
                contribute_alias(n.inputs[0], dy)          # global-average-pool chain: same buffer
            elif k == "ResizeBilinear" and buf[id(n.inputs[0])].shape[1] == 1 and buf[id(n.inputs[0])].shape[2] == 1:
                x = n.inputs[0]
                if id(x) in ng:                            # 1x1 -> HxW broadcast: gradient = spatial sum
                    dx, acc = dest(x)
                    ops.spatial_reduce(dy, dx, 1.0, self.ws)
                    done(dx, acc)
            elif k == "ResizeBilinear":
                # align_corners bilinear: fp32 scatter-add, then cast to the compute dtype
                x = n.inputs[0]
                if id(x) in ng:
                    dx, acc = dest(x)
                    g32 = p.tmp.get(("rb32", id(x)))
                    if g32 is None:
                        g32 = torch.zeros(dx.shape, dtype=torch.float32, device=self.device)
                        p.tmp[("rb32", id(x))] = g32
                    ops.resize_bilinear_bwd(dy, g32)
                    ops.cast(g32, dx)
                    done(dx, acc)
            elif k == "Softmax":
                raise NotImplementedError("gradient of tf.nn.softmax: the reference uses it for evaluation only "
                                          "(Network/utils/utils.py:54); train on softmax_cross_entropy_with_logits")
            elif k in ("ArgMax", "ExpandDims"):
                continue
            else:
                raise NotImplementedError(f"backward of {k}")
        if bn_defer:
            # every deferred dgamma / dbeta in two launches (the same sums as
            # each launch's own finish); the segment table is built once per plan
            segs = [s for s, _ in bn_defer]
            key = tuple((s[0].data_ptr(), int(s[1]), s[5].data_ptr()) for s in segs)
            batch = getattr(p, "bn_batch", None)
            if batch is None or batch.key != key:
                batch = ops.BnFinishBatch(segs, self.device)
                p.bn_batch = batch
            batch.run()
            self._grad_ready([nm for _, names in bn_defer for nm in names])

    def _grads_finite(self):
        """All gradients finite (every rank's, under data parallelism)?  One
        device-to-host read per step on the loss-scaled path."""
        if self._finite_flag is None:
            self._finite_flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        ops.check_finite(self.store.grads, self._finite_flag)
        if self._dpa is not None:
            import torch.distributed as dist
            dist.all_reduce(self._finite_flag, op=dist.ReduceOp.MAX, group=self.dp.group)
        return int(self._finite_flag.item()) == 0

    def _prologue(self, b):
        st = self.store
        return ops.prologue(st.param(b.gamma.var_name), st.param(b.beta.var_name), b.eps, b.relu)

    def _scratch_grad(self, p, var):
        """fp32 gradient sink for a filter outside var_list whose layer still
        needs its bias gradient (the filter-gradient launch sums it)."""
        t = p.tmp.get(("wscratch", var.var_name))
        if t is None:
            t = torch.zeros(tuple(var.shape), dtype=torch.float32, device=self.device)
            p.tmp[("wscratch", var.var_name)] = t
        return t

    def _check_bn_stats(self, p):
        """The kernels fold BatchNorm's frozen statistics as mean 0 / variance
        1 (tf.layers.batch_normalization with training=False and never-updated
        moving averages, Network/utils/utils.py:300-301).  Refuse to run if a
        restore or assign changed them."""
        store = self.store
        if not store.aux_vars or getattr(self, "_bn_checked", None) == store.aux_version:
            return
        for v in store.aux_vars:
            kind = getattr(v, "bn_stat", None)
            if kind is None:
                continue
            t = store.aux[v.var_name]
            want = 0.0 if kind == "mean" else 1.0
            if not bool((t == want).all()):
                raise NotImplementedError(f"{v.var_name}: BatchNormalization moving statistics other than "
                                          f"the frozen (0, 1) of the reference are not on the hot path")
        self._bn_checked = store.aux_version

    def _bias_relu_bwd(self, dy, y, dz, dbias, k_valid, relu, scale):
        # with TF1 dropout fused after the relu: dz = dy * (y > 0) / keep_prob
        ops.bias_relu_bwd(dy, y, dz, dbias, k_valid, relu, self.ws, scale=scale)

    def close(self):
        self.plans = {}

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
