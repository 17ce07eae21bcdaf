"""The reference's layer builders (L1 of SURVEY.md 1), same names, arguments
and semantics, building graph ops that the Session runs on MI355X kernels.

FCN helpers: Network/model/FCN.py:117-171.
Generic builders: Network/utils/utils.py:164-333.
"""
from __future__ import annotations

from . import tf

STDDEV = 1e-2


# ---------------------------------------------------------------------------
# Network/model/FCN.py:117-171
# ---------------------------------------------------------------------------
def conv_layer(x, num_filters, name, filter_height=3, filter_width=3, stride=1, padding="SAME"):
    """relu(conv2d(x, W, SAME) + b), W ~ N(0, 0.01), b = 0 (FCN.py:117-136)."""
    input_channels = int(x.get_shape()[-1].value)
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, input_channels, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        b = tf.get_variable("biases", shape=[num_filters], initializer=tf.constant_initializer(0.0))
        conv = tf.nn.conv2d(x, W, strides=[1, stride, stride, 1], padding=padding)
        z = tf.nn.bias_add(conv, b)
        return tf.nn.relu(z)


def deconv_layer(x, shape, num_filters, name, output_shape, filter_height=4, filter_width=4, stride=2,
                 padding="SAME"):
    """conv2d_transpose(x, W[kh,kw,shape[3],num_filters]) + b (FCN.py:138-159).
    Note: `num_filters` is the INPUT depth, output depth comes from shape[3]."""
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, shape[3].value, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        b = tf.get_variable("biases", shape=[shape[3].value], initializer=tf.constant_initializer(0.0))
        if output_shape is None:
            output_shape = x.get_shape().as_list()
            output_shape[1] *= 2
            output_shape[2] *= 2
            output_shape[3] = W.shape[2]
        deconv = tf.nn.conv2d_transpose(x, W, output_shape, strides=[1, stride, stride, 1], padding=padding)
        return tf.nn.bias_add(deconv, b)


def max_pool(x, name, filter_height=2, filter_width=2, stride=2, padding="VALID"):
    return tf.nn.max_pool(x, ksize=[1, filter_height, filter_width, 1], strides=[1, stride, stride, 1],
                          padding=padding, name=name)


def dropout(x, keep_prob):
    return tf.nn.dropout(x, keep_prob=keep_prob)


def fuse(x1, x2, name):
    return tf.add(x1, x2, name=name)


# ---------------------------------------------------------------------------
# Network/utils/utils.py:164-333
# ---------------------------------------------------------------------------
def Conv2D_Layer(x, num_filters, filter_height=3, filter_width=3, stride=1, padding="SAME", dilation=1,
                 name=None):
    """Bias-free conv with optional dilation (utils.py:164-184)."""
    input_channels = int(x.get_shape()[-1].value)
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, input_channels, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        return tf.nn.conv2d(x, W, strides=[1, stride, stride, 1], dilations=dilation, padding=padding)


def Conv2D_Block(x, num_filters, filter_height=3, filter_width=3, stride=1, padding="SAME", dilation=1,
                 batch_normalization=False, relu=False, name=None):
    """utils.py:186-208 -- defaults: no BN, no ReLU."""
    conv = Conv2D_Layer(x, num_filters, filter_height=filter_height, filter_width=filter_width, stride=stride,
                        padding=padding, dilation=dilation, name=name)
    if batch_normalization is True:
        conv = Batch_Normalization(conv)
    if relu is True:
        conv = tf.nn.relu(conv)
    return conv


def Atrous_Conv2D_Layer(x, num_filters, filter_height=3, filter_width=3, dilation=1, padding="SAME",
                        name=None):
    """tf.nn.atrous_conv2d == dilated conv2d (utils.py:210-229)."""
    input_channels = int(x.get_shape()[-1].value)
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, input_channels, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        return tf.nn.atrous_conv2d(x, W, dilation, padding=padding)


def Atrous_Conv2D_Block(x, num_filters, filter_height=3, filter_width=3, dilation=1, padding="SAME",
                        batch_normalization=False, relu=False, name=None):
    conv = Atrous_Conv2D_Layer(x, num_filters, filter_height=filter_height, filter_width=filter_width,
                               dilation=dilation, padding=padding, name=name)
    if batch_normalization is True:
        conv = Batch_Normalization(conv)
    if relu is True:
        conv = tf.nn.relu(conv)
    return conv


def Deconv2D_Layer(x, shape, num_filters, output_shape, filter_height=4, filter_width=4, stride=2,
                   padding="SAME", name=None):
    """Bias-free conv2d_transpose, W [kh,kw,shape[3],num_filters] (utils.py:255-274)."""
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, shape[3].value, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        if output_shape is None:
            output_shape = x.get_shape().as_list()
            output_shape[1] *= 2
            output_shape[2] *= 2
            output_shape[3] = W.shape[2]
        return tf.nn.conv2d_transpose(x, W, output_shape, strides=[1, stride, stride, 1], padding=padding)


def Deconv2D_Block(x, shape, num_filters, output_shape, filter_height=4, filter_width=4, stride=2,
                   padding="SAME", batch_normalization=False, relu=False, name=None):
    deconv = Deconv2D_Layer(x, shape, num_filters, output_shape, filter_height=filter_height,
                            filter_width=filter_width, stride=stride, padding=padding, name=name)
    if batch_normalization is True:
        deconv = Batch_Normalization(deconv)
    if relu is True:
        deconv = tf.nn.relu(deconv)
    return deconv


def Batch_Normalization(x):
    """tf.layers.batch_normalization(x): training=False, frozen stats (utils.py:300-301)."""
    return tf.layers.batch_normalization(x)


def ReLU(x):
    return tf.nn.relu(x)


def Max_Pooling(x, name, filter_height=2, filter_width=2, stride=2, padding="VALID"):
    return tf.nn.max_pool(x, ksize=[1, filter_height, filter_width, 1], strides=[1, stride, stride, 1],
                          padding=padding, name=name)


def Avg_Pooling(x, name, filter_height=2, filter_width=2, stride_height=2, stride_width=2, padding="VALID"):
    return tf.nn.avg_pool(x, ksize=[1, filter_height, filter_width, 1],
                          strides=[1, stride_height, stride_width, 1], padding=padding, name=name)


def Global_Avg_Pool(x, stride=1):
    """utils.py:312-313: tflearn global_avg_pool -> [N, C]."""
    return tf.nn.global_avg_pool(x, name="global_avg_pooling")


def Dropout(x, keep_prob):
    return tf.nn.dropout(x, keep_prob=keep_prob)


def Softmax(x):
    return tf.nn.softmax(x)


def Resize_Bilinear(x, size, name):
    return tf.image.resize_bilinear(x, size=size, align_corners=True, name=name)


def Concat(x, axis, name):
    return tf.concat(x, axis=axis, name=name)
