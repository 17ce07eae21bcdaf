"""DeepLab-style atrous segmentation model (BASELINE config C5) built from
the reference's own layer builders.

The reference's DeepLabV3Plus (Network/model/DeepLabv3Plus.py:129-271) cannot
run as written (it imports a missing utils module and its Xception /
MobileNetV2 backbones need depthwise convolutions, which no hot-path builder
of the reference provides), so SURVEY.md 8f-4 leaves the variant to the build.
This one keeps the parts of that file that ARE the DeepLab method and maps
them onto the hot-path builders:

* backbone: the FCN's VGG16 conv stack (Network/model/FCN.py:55-83, same
  conv_layer names), pool1..pool3 only (output stride 8), conv5_x as atrous
  3x3 convs with rate 2 -- DeepLab's removal of the last poolings;
* ASPP head (DeepLabv3Plus.py:227-243): 1x1 branch `aspp0` and three atrous
  3x3 branches `aspp1..3` (rates 6 / 12 / 18, the out_stride=16 rates of
  :150), each Conv2D_Block / Atrous_Conv2D_Block with frozen-stat BN + ReLU
  (utils.py:186-229), concatenated (Concat, utils.py:332) and projected by a
  1x1 `concat_projection` block + Dropout (:246-247); first in the concat,
  the image-pooling branch b4 (:213-225): Global_Avg_Pool (utils.py:312),
  two expand_dims, a 1x1 `image_pooling` Conv2D_Block with BN + ReLU and
  Resize_Bilinear back to the feature map size (tf.shape(feat)[1:3]);
* classifier `Last_layer` (1x1, :262) and Resize_Bilinear (align_corners,
  utils.py:329) back to the input size (:264-266).

Returns (expand_dims(argmax(logits)), logits) like FCN.create().
"""
from . import tf
from .layers import (STDDEV, Atrous_Conv2D_Block, Concat, Conv2D_Block, Dropout, Global_Avg_Pool, Resize_Bilinear,
                     conv_layer, max_pool)

ASPP_RATES = (6, 12, 18)
ASPP_DEPTH = 256
KEEP_PROB = 0.9


def atrous_conv_layer(x, num_filters, name, rate, filter_height=3, filter_width=3):
    """relu(atrous_conv2d(x, W, rate, SAME) + b): FCN.py:117-136 with a rate."""
    input_channels = int(x.get_shape()[-1].value)
    with tf.variable_scope(name, reuse=tf.AUTO_REUSE):
        W = tf.get_variable("weights", shape=[filter_height, filter_width, input_channels, num_filters],
                            initializer=tf.random_normal_initializer(mean=0.0, stddev=STDDEV))
        b = tf.get_variable("biases", shape=[num_filters], initializer=tf.constant_initializer(0.0))
        return tf.nn.relu(tf.nn.bias_add(tf.nn.atrous_conv2d(x, W, rate, padding="SAME"), b))


def DeepLabASPP(x, keep_prob, num_classes):
    H, W = int(x.get_shape()[1].value), int(x.get_shape()[2].value)
    h = conv_layer(x, 64, "conv1_1")
    h = conv_layer(h, 64, "conv1_2")
    h = max_pool(h, "pool1")
    h = conv_layer(h, 128, "conv2_1")
    h = conv_layer(h, 128, "conv2_2")
    h = max_pool(h, "pool2")
    h = conv_layer(h, 256, "conv3_1")
    h = conv_layer(h, 256, "conv3_2")
    h = conv_layer(h, 256, "conv3_3")
    h = max_pool(h, "pool3")
    h = conv_layer(h, 512, "conv4_1")
    h = conv_layer(h, 512, "conv4_2")
    h = conv_layer(h, 512, "conv4_3")
    h = atrous_conv_layer(h, 512, "conv5_1", 2)
    h = atrous_conv_layer(h, 512, "conv5_2", 2)
    feat = atrous_conv_layer(h, 512, "conv5_3", 2)

    # image feature branch (DeepLabv3Plus.py:215-223)
    b4 = Global_Avg_Pool(feat)
    b4 = tf.expand_dims(b4, dim=1)
    b4 = tf.expand_dims(b4, dim=1)
    b4 = Conv2D_Block(b4, ASPP_DEPTH, filter_height=1, filter_width=1, stride=1, padding="SAME",
                      batch_normalization=True, relu=True, name="image_pooling")
    size_before = tf.shape(feat)
    b4 = Resize_Bilinear(b4, size_before[1:3], name="Upsampling")
    b0 = Conv2D_Block(feat, ASPP_DEPTH, filter_height=1, filter_width=1, batch_normalization=True, relu=True,
                      name="aspp0")
    branches = [b4, b0]
    for i, r in enumerate(ASPP_RATES):
        branches.append(Atrous_Conv2D_Block(feat, ASPP_DEPTH, dilation=r, batch_normalization=True, relu=True,
                                            name=f"aspp{i + 1}"))
    cat = Concat(branches, axis=-1, name="concatenation")
    proj = Conv2D_Block(cat, ASPP_DEPTH, filter_height=1, filter_width=1, batch_normalization=True, relu=True,
                        name="concat_projection")
    proj = Dropout(proj, keep_prob=keep_prob)
    last = Conv2D_Block(proj, num_classes, filter_height=1, filter_width=1, name="Last_layer")
    logits = Resize_Bilinear(last, [H, W], name="Upsampling3")
    pred = tf.argmax(logits, dimension=3, name="prediction")
    return tf.expand_dims(pred, dim=3), logits
