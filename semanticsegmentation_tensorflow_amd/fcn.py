"""The reference FCN (Network/model/FCN.py:31-114), same class, constructor and
`create()` contract: returns (pred [N,H,W,1] int64, logits [N,H,W,C]).

Topology reproduced exactly, including the reference's quirks:
14-conv encoder (block 4 has four convs, conv5_4 commented out), 7x7 SAME
conv6, ReLU on conv8, feature-width skip fusion (conv_t1 C->512 + pool4,
conv_t2 512->256 + pool3), 16x16 stride-8 conv_t3 with variable `conv_t3/bias`.

Difference by design: the reference's __init__ calls create() and main()
calls it again (the first graph is dead, FCN.py:47/:319); building a graph
here is free, so we keep that behaviour -- both builds share variables via
AUTO_REUSE and only the one reachable from the fetched loss is compiled.
"""
from __future__ import annotations

from . import tf
from .layers import conv_layer, deconv_layer, dropout, fuse, max_pool


class FCN(object):
    """Implementation of the reference's VGG16-style FCN."""

    def __init__(self, x, keep_prob, num_classess):
        self.X = x
        self.NUM_CLASSESS = num_classess
        self.KEEP_PROB = keep_prob
        self.create()

    def create(self):
        conv1_1 = conv_layer(self.X, 64, "conv1_1")
        conv1_2 = conv_layer(conv1_1, 64, "conv1_2")
        pool1 = max_pool(conv1_2, "pool1")

        conv2_1 = conv_layer(pool1, 128, "conv2_1")
        conv2_2 = conv_layer(conv2_1, 128, "conv2_2")
        pool2 = max_pool(conv2_2, "pool2")

        conv3_1 = conv_layer(pool2, 256, "conv3_1")
        conv3_2 = conv_layer(conv3_1, 256, "conv3_2")
        conv3_3 = conv_layer(conv3_2, 256, "conv3_3")
        pool3 = max_pool(conv3_3, "pool3")

        conv4_1 = conv_layer(pool3, 512, "conv4_1")
        conv4_2 = conv_layer(conv4_1, 512, "conv4_2")
        conv4_3 = conv_layer(conv4_2, 512, "conv4_3")
        conv4_4 = conv_layer(conv4_3, 512, "conv4_4")
        pool4 = max_pool(conv4_4, "pool4")

        conv5_1 = conv_layer(pool4, 512, "conv5_1")
        conv5_2 = conv_layer(conv5_1, 512, "conv5_2")
        conv5_3 = conv_layer(conv5_2, 512, "conv5_3")
        pool5 = max_pool(conv5_3, "pool5")

        conv6 = conv_layer(pool5, 4096, "conv6", filter_height=7, filter_width=7)
        dropout6 = dropout(conv6, self.KEEP_PROB)
        conv7 = conv_layer(dropout6, 4096, "conv7", filter_height=1, filter_width=1)
        dropout7 = dropout(conv7, self.KEEP_PROB)
        conv8 = conv_layer(dropout7, self.NUM_CLASSESS, "conv8", filter_height=1, filter_width=1)

        deconv_shape1 = pool4.get_shape()
        conv_t1 = deconv_layer(conv8, deconv_shape1, self.NUM_CLASSESS, "conv_t1", tf.shape(pool4))
        fuse_1 = fuse(conv_t1, pool4, "fuse_1")

        deconv_shape2 = pool3.get_shape()
        conv_t2 = deconv_layer(fuse_1, deconv_shape2, deconv_shape1[3].value, "conv_t2", tf.shape(pool3))
        fuse_2 = fuse(conv_t2, pool3, "fuse_2")

        shape = tf.shape(self.X)
        deconv_shape3 = tf.stack([shape[0], shape[1], shape[2], self.NUM_CLASSESS])
        with tf.variable_scope("conv_t3", reuse=tf.AUTO_REUSE):
            W_t3 = tf.get_variable("weights", shape=[16, 16, self.NUM_CLASSESS, deconv_shape2[3].value],
                                   initializer=tf.random_normal_initializer(mean=0.0, stddev=0.01))
            b_t3 = tf.get_variable("bias", shape=[self.NUM_CLASSESS], initializer=tf.constant_initializer(0.0))
        conv_t3 = tf.nn.conv2d_transpose(fuse_2, W_t3, deconv_shape3, strides=[1, 8, 8, 1], padding="SAME")
        conv_t3 = tf.nn.bias_add(conv_t3, b_t3)

        annotation_pred = tf.argmax(conv_t3, dimension=3, name="prediction")
        return tf.expand_dims(annotation_pred, dim=3), conv_t3
