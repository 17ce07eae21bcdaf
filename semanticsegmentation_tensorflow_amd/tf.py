"""`import semanticsegmentation_tensorflow_amd.tf as tf` -- the TF 1.x names the
reference's hot path uses (Network/model/FCN.py, Network/utils/utils.py,
Network/model/FCDenseNet.py), backed by the graph in `graph.py` and executed
by `session.Session` on the MI355X kernels.  Only hot-path ops exist; anything
else raises NotImplementedError instead of silently running elsewhere.
"""
from types import SimpleNamespace

from . import checkpoint as _ckpt
from . import graph as _g
from .session import Session  # noqa: F401

float32, uint8, int64 = _g.float32, _g.uint8, _g.int64
AUTO_REUSE = _g.AUTO_REUSE

placeholder = _g.placeholder
get_variable = _g.get_variable
variable_scope = _g.variable_scope
name_scope = _g.name_scope
random_normal_initializer = _g.random_normal_initializer
constant_initializer = _g.constant_initializer
trainable_variables = _g.trainable_variables
global_variables = _g.global_variables
global_variables_initializer = _g.global_variables_initializer
get_default_graph = _g.get_default_graph
reset_default_graph = _g.reset_default_graph
shape = _g.shape
stack = _g.stack
add = _g.add
concat = _g.concat
argmax = _g.argmax
expand_dims = _g.expand_dims
reduce_mean = _g.reduce_mean
Variable = _g.Variable_
zeros_like = _g.zeros_like
constant = _g.constant
scalar_mul = _g.scalar_mul

nn = SimpleNamespace(
    conv2d=_g.conv2d,
    atrous_conv2d=_g.atrous_conv2d,
    conv2d_transpose=_g.conv2d_transpose,
    bias_add=_g.bias_add,
    relu=_g.relu,
    max_pool=_g.max_pool,
    avg_pool=_g.avg_pool,
    dropout=_g.dropout,
    softmax=_g.softmax,
    global_avg_pool=_g.global_avg_pool,
    softmax_cross_entropy_with_logits=_g.softmax_cross_entropy_with_logits,
)
layers = SimpleNamespace(batch_normalization=_g.batch_normalization)
image = SimpleNamespace(resize_bilinear=_g.resize_bilinear)
train = SimpleNamespace(AdamOptimizer=_g.AdamOptimizer, Saver=_ckpt.Saver,
                        get_checkpoint_state=_ckpt.get_checkpoint_state,
                        latest_checkpoint=_ckpt.latest_checkpoint)
compat = SimpleNamespace(v1=SimpleNamespace(
    train=train, placeholder=placeholder, Variable=Variable, zeros_like=zeros_like, constant=constant,
    trainable_variables=trainable_variables, global_variables=global_variables,
    global_variables_initializer=global_variables_initializer, Session=Session))
