"""Symbolic graph mirroring the TF 1.x graph-construction surface the
reference builds its models with (`tf.placeholder`, `tf.get_variable` under
`tf.variable_scope(..., reuse=AUTO_REUSE)`, `tf.nn.*`, `tf.train.AdamOptimizer`).

Nothing here computes; `session.Session` compiles the graph into a static
launch plan over the HIP C-ABI.  Only the ops on the reference's hot path
 exist.
"""
from __future__ import annotations

import contextlib
import itertools

AUTO_REUSE = "AUTO_REUSE"
float32, uint8, int64, bfloat16 = "float32", "uint8", "int64", "bfloat16"


class Dimension:
    __slots__ = ("value",)

    def __init__(self, v):
        self.value = v

    def __int__(self):
        return int(self.value)

    def __index__(self):
        return int(self.value)

    def __eq__(self, o):
        return self.value == (o.value if isinstance(o, Dimension) else o)

    def __hash__(self):
        return hash(self.value)

    def __repr__(self):
        return f"Dimension({self.value})"


class TensorShape(tuple):
    """tuple of Dimension, so `shape[3].value` works as in FCN.py:95."""

    def __new__(cls, dims):
        return super().__new__(cls, [d if isinstance(d, Dimension) else Dimension(d) for d in dims])

    def as_list(self):
        return [d.value for d in self]

    def __repr__(self):
        return f"TensorShape({self.as_list()})"


class Graph:
    def __init__(self):
        self.ops = []
        self.variables = {}            # name -> Variable, creation order
        self._scope = []
        self._ids = itertools.count()
        self._names = {}
        self.bn_count = 0

    def unique(self, base):
        n = self._names.get(base, 0)
        self._names[base] = n + 1
        return base if n == 0 else f"{base}_{n}"

    def scoped(self, name):
        return "/".join(self._scope + [name]) if self._scope else name


_GRAPH = Graph()


def get_default_graph() -> Graph:
    return _GRAPH


def reset_default_graph():
    global _GRAPH
    _GRAPH = Graph()
    return _GRAPH


class Op:
    def __init__(self, type_, inputs, attrs=None, name=None, n_out=1):
        g = get_default_graph()
        self.graph = g
        self.id = next(g._ids)
        self.type = type_
        self.inputs = list(inputs)
        self.attrs = attrs or {}
        self.name = g.unique(name or type_)
        self.outputs = [Tensor(self, i) for i in range(n_out)]
        for t in self.inputs:
            t.consumers.append(self)
        g.ops.append(self)

    def __repr__(self):
        return f"<Op {self.name}:{self.type}>"


class Tensor:
    def __init__(self, op, index=0):
        self.op = op
        self.index = index
        self.consumers = []
        self.shape = None     # static shape (tuple, None = batch) set by builders
        self.dtype = float32

    @property
    def name(self):
        return f"{self.op.name}:{self.index}"

    @property
    def graph(self):
        return self.op.graph

    def get_shape(self):
        return TensorShape(self.shape)

    def __add__(self, other):
        return add(self, other)

    def __repr__(self):
        return f"<Tensor {self.name} shape={self.shape} {self.dtype}>"


class Variable(Tensor):
    def __init__(self, name, shape, initializer, trainable=True):
        op = Op("VariableV2", [], {"var_name": name}, name=name)
        super().__init__(op, 0)
        op.outputs[0] = self
        self.var_name = name
        self.shape = tuple(shape)
        self.initializer = initializer
        self.trainable = trainable

    def __repr__(self):
        return f"<Variable {self.var_name} {self.shape}>"

    # --- the tf.Variable methods the accumulate-then-apply template uses
    # (Network/main.py:78-95, Network/model/FCDenseNet.py:204-213)
    def initialized_value(self):
        return self

    def value(self):
        return self

    def assign(self, value, name=None):
        """`var.assign(value)`: value a tf.zeros_like / tf.constant / number."""
        ins = [self] + ([value] if isinstance(value, Tensor) else [])
        return Op("Assign", ins, {"var": self, "value": value}, name or "Assign")

    def assign_add(self, value, name=None):
        """`var.assign_add(value)`: value a gradient from compute_gradients,
        optionally through tf.scalar_mul."""
        return Op("AssignAdd", [self, value], {"var": self, "value": value}, name or "AssignAdd")


# ---------------------------------------------------------------------------
# initializers (Network/model/FCN.py:125-127)
# ---------------------------------------------------------------------------
class random_normal_initializer:
    def __init__(self, mean=0.0, stddev=1.0):
        self.mean, self.stddev = mean, stddev

    def __repr__(self):
        return f"N({self.mean},{self.stddev})"


class constant_initializer:
    def __init__(self, value=0.0):
        self.value = value


ones_initializer = lambda: constant_initializer(1.0)  # noqa: E731
zeros_initializer = lambda: constant_initializer(0.0)  # noqa: E731


# ---------------------------------------------------------------------------
# scopes / variables
# ---------------------------------------------------------------------------
class _VarScope:
    def __init__(self, name):
        self.name = name
        self.original_name_scope = name


@contextlib.contextmanager
def variable_scope(name, reuse=None):
    g = get_default_graph()
    g._scope.append(name)
    try:
        yield _VarScope("/".join(g._scope))
    finally:
        g._scope.pop()


@contextlib.contextmanager
def name_scope(name):
    # tf.name_scope does not prefix get_variable names (FCDenseNet.py:24)
    yield name


def get_variable(name, shape, initializer=None, trainable=True):
    g = get_default_graph()
    full = g.scoped(name)
    if full in g.variables:                       # AUTO_REUSE semantics
        v = g.variables[full]
        if tuple(v.shape) != tuple(int(s) for s in shape):
            raise ValueError(f"variable {full} reused with shape {shape} != {v.shape}")
        return v
    v = Variable(full, [int(s) for s in shape], initializer or random_normal_initializer(0.0, 1.0),
                 trainable)
    g.variables[full] = v
    return v


def Variable_(initial_value=0, trainable=True, name=None, dtype=None):
    """tf.Variable(initial_value, trainable=..., name=...): the reference's
    gradient accumulators `tf.Variable(tf.zeros_like(v.initialized_value()),
    trainable=False)` (Network/main.py:78-81) and `global_step =
    tf.Variable(0, trainable=False, name='global_step')`
    (Network/model/FCDenseNet.py:247).  Created at the root scope."""
    g = get_default_graph()
    if isinstance(initial_value, Tensor):
        if initial_value.op.type not in ("ZerosLike", "Const"):
            raise NotImplementedError("tf.Variable initial_value must be tf.zeros_like(...), a "
                                      "tf.constant or a number")
        shape = tuple(initial_value.shape or ())
        if initial_value.op.type == "ZerosLike":
            init = constant_initializer(0.0)
        else:
            val = initial_value.op.attrs["value"]
            init = lambda s, _v=val: _np_full(s, _v)  # noqa: E731
    else:
        import numpy as _np
        arr = _np.asarray(initial_value, dtype=_np.float64)
        shape = arr.shape
        init = lambda s, _v=arr: _np_full(s, _v)  # noqa: E731
    full = g.unique(name or "Variable")
    v = Variable(full, shape, init, trainable)
    v.dtype = dtype or (int64 if (not isinstance(initial_value, Tensor) and isinstance(initial_value, int))
                        else float32)
    g.variables[full] = v
    return v


def _np_full(shape, v):
    import numpy as _np
    return _np.broadcast_to(_np.asarray(v, dtype=_np.float32), shape).copy()


def zeros_like(t, name=None):
    op = Op("ZerosLike", [t], {}, name)
    op.outputs[0].shape = t.shape
    return op.outputs[0]


def constant(value, dtype=None, shape=None, name=None):
    import numpy as _np
    arr = _np.asarray(value, dtype=_np.float32)
    op = Op("Const", [], {"value": arr}, name or "Const")
    op.outputs[0].shape = arr.shape
    return op.outputs[0]


def scalar_mul(scalar, x, name=None):
    """tf.scalar_mul(scalar, x) with scalar a tf.constant or a number."""
    ins = [x] + ([scalar] if isinstance(scalar, Tensor) else [])
    op = Op("ScalarMul", ins, {"scalar": scalar, "x": x}, name)
    op.outputs[0].shape = x.shape
    return op.outputs[0]


def const_value(t):
    """Python float of a number or a scalar tf.constant."""
    if isinstance(t, Tensor):
        if t.op.type != "Const":
            raise NotImplementedError(f"expected a tf.constant, got {t.op.type}")
        return float(t.op.attrs["value"])
    return float(t)


def trainable_variables():
    return [v for v in get_default_graph().variables.values() if v.trainable]


def global_variables():
    return list(get_default_graph().variables.values())


# ---------------------------------------------------------------------------
# placeholders and dynamic shapes
# ---------------------------------------------------------------------------
def placeholder(dtype, shape=None, name=None):
    op = Op("Placeholder", [], {"dtype": dtype}, name=name or "Placeholder")
    t = op.outputs[0]
    t.dtype = dtype
    t.shape = None if shape is None else tuple(shape)
    return t


class ShapeOf:
    """tf.shape(x): resolved when the session knows the fed shapes."""

    def __init__(self, t):
        self.t = t

    def __getitem__(self, i):
        if isinstance(i, slice):                    # size_before[1:3] (DeepLabv3Plus.py:222)
            return [ShapeElem(self.t, j) for j in range(*i.indices(4))]
        return ShapeElem(self.t, i)


class ShapeElem:
    def __init__(self, t, i):
        self.t, self.i = t, i


def shape(t):
    return ShapeOf(t)


def stack(values):
    return list(values)


def _static(t, i):
    return None if t.shape is None else t.shape[i]


# ---------------------------------------------------------------------------
# ops (shape-propagating builders)
# ---------------------------------------------------------------------------
def _pads(in_size, k, s, d, padding):
    if in_size is None:
        return None
    k_eff = k + (k - 1) * (d - 1)
    if padding == "SAME":
        return -(-in_size // s)
    return (in_size - k_eff) // s + 1


def _strides(s):
    if isinstance(s, int):
        return s, s
    s = list(s)
    if len(s) == 4:
        return s[1], s[2]
    return s[0], s[1]


def conv2d(input, filter, strides=(1, 1, 1, 1), padding="SAME", dilations=1, name=None):
    sh, sw = _strides(strides)
    dh, dw = _strides(dilations) if not isinstance(dilations, int) else (dilations, dilations)
    if sh != sw or dh != dw:
        raise NotImplementedError("anisotropic stride/dilation")
    R, S, C, K = filter.shape
    op = Op("Conv2D", [input, filter], {"stride": sh, "dilation": dh, "padding": padding}, name)
    y = op.outputs[0]
    N, H, W, _ = input.shape
    y.shape = (N, _pads(H, R, sh, dh, padding), _pads(W, S, sw, dw, padding), K)
    return y


def atrous_conv2d(value, filters, rate, padding="SAME", name=None):
    return conv2d(value, filters, 1, padding, rate, name)


def conv2d_transpose(value, filter, output_shape, strides, padding="SAME", name=None):
    sh, sw = _strides(strides)
    if sh != sw:
        raise NotImplementedError("anisotropic stride")
    op = Op("Conv2DTranspose", [value, filter], {"stride": sh, "padding": padding,
                                                  "output_shape": output_shape}, name)
    y = op.outputs[0]
    os_ = resolve_shape(output_shape)
    y.shape = (value.shape[0], os_[1], os_[2], filter.shape[2])
    return y


def resolve_shape(s, lookup=None):
    """Resolve an output_shape argument (ints, Dimensions, tf.shape(t), or a
    tf.stack of tf.shape elements) to a 4-tuple; `lookup(t)` gives concrete
    shapes at compile time, otherwise static shapes (None = unknown)."""
    get = lookup or (lambda t: t.shape if t.shape is not None else (None,) * 4)
    if isinstance(s, ShapeOf):
        return tuple(get(s.t))
    out = []
    for v in s:
        if isinstance(v, ShapeElem):
            out.append(get(v.t)[v.i])
        else:
            out.append(getattr(v, "value", v))
    return tuple(out)


def bias_add(value, bias, name=None):
    op = Op("BiasAdd", [value, bias], {}, name)
    op.outputs[0].shape = value.shape
    return op.outputs[0]


def relu(features, name=None):
    op = Op("Relu", [features], {}, name)
    op.outputs[0].shape = features.shape
    return op.outputs[0]


def _pool(kind, value, ksize, strides, padding, name):
    k = _strides(ksize)
    s = _strides(strides)
    if k != (2, 2) or s != (2, 2) or padding != "VALID":
        raise NotImplementedError(f"{kind}: only 2x2 stride-2 VALID pooling is on the hot path")
    op = Op(kind, [value], {}, name)
    N, H, W, C = value.shape
    op.outputs[0].shape = (N, None if H is None else H // 2, None if W is None else W // 2, C)
    return op.outputs[0]


def max_pool(value, ksize, strides, padding, name=None):
    return _pool("MaxPool", value, ksize, strides, padding, name)


def avg_pool(value, ksize, strides, padding, name=None):
    return _pool("AvgPool", value, ksize, strides, padding, name)


def dropout(x, keep_prob, name=None):
    """tf.nn.dropout (TF1): x / kp * floor(kp + U).  keep_prob: float or a fed scalar."""
    op = Op("Dropout", [x], {"keep_prob": keep_prob}, name)
    op.outputs[0].shape = x.shape
    return op.outputs[0]


def add(x, y, name=None):
    op = Op("Add", [x, y], {}, name)
    op.outputs[0].shape = x.shape
    return op.outputs[0]


def concat(values, axis, name=None):
    if axis not in (-1, 3):
        raise NotImplementedError("concat only along channels")
    op = Op("ConcatV2", list(values), {}, name)
    c = [v.shape[3] for v in values]
    op.outputs[0].shape = tuple(values[0].shape[:3]) + (None if None in c else sum(c),)
    return op.outputs[0]


def batch_normalization(inputs, epsilon=1e-3, name=None):
    """tf.layers.batch_normalization(x) with training=False (utils.py:300-301):
    frozen moving stats (0, 1) -> y = gamma*x/sqrt(1+eps) + beta."""
    g = get_default_graph()
    base = name or ("batch_normalization" if g.bn_count == 0 else f"batch_normalization_{g.bn_count}")
    g.bn_count += 1
    C = inputs.shape[3]
    with _root_scope():
        gamma = get_variable(f"{base}/gamma", [C], constant_initializer(1.0))
        beta = get_variable(f"{base}/beta", [C], constant_initializer(0.0))
        # TF's non-trainable moving statistics (saved by tf.train.Saver; frozen
        # at their initial values since training=False never updates them)
        mean = get_variable(f"{base}/moving_mean", [C], constant_initializer(0.0), trainable=False)
        var = get_variable(f"{base}/moving_variance", [C], constant_initializer(1.0), trainable=False)
        mean.bn_stat, var.bn_stat = "mean", "variance"
    op = Op("FusedBatchNorm", [inputs, gamma, beta], {"epsilon": epsilon}, base)
    op.outputs[0].shape = inputs.shape
    return op.outputs[0]


@contextlib.contextmanager
def _root_scope():
    g = get_default_graph()
    saved, g._scope = g._scope, []
    try:
        yield
    finally:
        g._scope = saved


def resize_bilinear(images, size, align_corners=True, name=None):
    """size: two ints, Dimensions or tf.shape(t) elements (resolved at compile time)."""
    if not align_corners:
        raise NotImplementedError("only align_corners=True (utils.py:330)")
    size = tuple(size)
    op = Op("ResizeBilinear", [images], {"size": size}, name)
    st = [v if not isinstance(v, ShapeElem) else _static(v.t, v.i) for v in size]
    op.outputs[0].shape = (images.shape[0], getattr(st[0], "value", st[0]), getattr(st[1], "value", st[1]),
                           images.shape[3])
    return op.outputs[0]


def global_avg_pool(x, name=None):
    """tflearn global_avg_pool (Network/utils/utils.py:312): tf.reduce_mean(x,
    [1, 2]) -> [N, C]."""
    op = Op("GlobalAvgPool", [x], {}, name or "global_avg_pooling")
    op.outputs[0].shape = (x.shape[0], x.shape[3])
    return op.outputs[0]


def softmax_cross_entropy_with_logits(logits=None, labels=None, name=None, valid_hw=None):
    """Per-pixel loss.  labels: one-hot float [N,H,W,C] (FCN.py:334) or a uint8
    class-index map [N,H,W].  valid_hw crops the loss region (375x1242 KITTI
    images zero-padded to 384x1248)."""
    op = Op("SoftmaxXent", [logits, labels], {"valid_hw": valid_hw}, name)
    op.outputs[0].shape = tuple(logits.shape[:3])
    return op.outputs[0]


def reduce_mean(x, name=None):
    op = Op("Mean", [x], {}, name)
    op.outputs[0].shape = ()
    return op.outputs[0]


def argmax(x, dimension=3, axis=None, name=None):
    op = Op("ArgMax", [x], {"axis": axis if axis is not None else dimension}, name)
    op.outputs[0].shape = tuple(x.shape[:3])
    op.outputs[0].dtype = int64
    return op.outputs[0]


def expand_dims(x, dim=-1, axis=None, name=None):
    d = axis if axis is not None else dim
    shp = list(x.shape)
    d = d if d >= 0 else len(shp) + 1 + d
    op = Op("ExpandDims", [x], {"dim": d}, name)
    op.outputs[0].shape = tuple(shp[:d] + [1] + shp[d:])
    op.outputs[0].dtype = x.dtype
    return op.outputs[0]


def softmax(logits, name=None):
    op = Op("Softmax", [logits], {}, name)
    op.outputs[0].shape = logits.shape
    return op.outputs[0]


# ---------------------------------------------------------------------------
# training (Network/model/FCN.py:338-340; Network/main.py:66-101)
# ---------------------------------------------------------------------------
class AdamOptimizer:
    """TF1 AdamOptimizer: epsilon outside the bias correction."""

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8):
        self.lr, self.beta1, self.beta2, self.epsilon = learning_rate, beta1, beta2, epsilon

    def minimize(self, loss, global_step=None, var_list=None, grad_scale=1.0, name=None):
        """grad_scale=1 gives FCN.py's `minimize` semantics; grad_scale=9 the
        effective gradient of the accumulate-then-apply template
        (Network/main.py:71, :168-175: 3B accumulations of (3/B)*g) computed
        once.  Only `var_list` (default: all trainables) is updated;
        `global_step`, if given, is incremented per step as in TF."""
        var_list = var_list or trainable_variables()
        op = Op("TrainStep", [loss], {"optimizer": self, "var_list": list(var_list),
                                      "grad_scale": float(grad_scale), "global_step": global_step},
                name or "train_step")
        return op

    def compute_gradients(self, loss, var_list=None):
        """[(gradient, variable)] (Network/main.py:88-89): each gradient is a
        symbolic d loss / d var the Session computes in one backward pass."""
        var_list = var_list or trainable_variables()
        out = []
        for v in var_list:
            op = Op("Gradient", [loss, v], {"loss": loss, "var": v}, "gradients")
            op.outputs[0].shape = tuple(v.shape)
            out.append((op.outputs[0], v))
        return out

    def apply_gradients(self, grads_and_vars, global_step=None, name=None):
        """One TF1 Adam step on each variable with the paired gradient source:
        a compute_gradients gradient (optionally scalar_mul-scaled) or an
        accumulator variable (Network/main.py:98-101)."""
        pairs = list(grads_and_vars)
        ins = [g for g, _ in pairs if isinstance(g, Tensor)]
        return Op("ApplyGradients", ins, {"optimizer": self, "pairs": pairs, "global_step": global_step},
                  name or "Adam")


def global_variables_initializer():
    return Op("InitAll", [], {}, "init")
