"""FC-DenseNet ("U-Net" config C3) -- same builder functions, names and
quirks as the reference (Network/model/FCDenseNet.py:23-163), on this
package's TF1-style graph (`semanticsegmentation_tensorflow_amd.tf`).

* bottleneck_layer  = BN -> ReLU -> 1x1 conv (4*growth) -> dropout ->
                      BN -> ReLU -> 3x3 conv (growth) -> dropout   (:23-35)
* Transition_Layer  = BN -> ReLU -> 1x1 conv (theta*C) -> 2x2 avg pool (:37-46)
* DenseBlock        = bottleneck_0 + n more, each on the concat of all
                      previous features; returns the final concat (:48-61)
* FCDenseNet        = 48-ch stem, blocks [4,5,7,10,12,15], five
                      transition-ups (k4 s2 tconv, widths hard-coded as in
                      the reference: 430/696/560/416/320) concatenated with
                      the encoder skips, 1x1 head; returns
                      (expand_dims(argmax), logits)                        (:83-163)

All convolutions are bias-free (utils.py:180 has the bias commented out) and
batch normalization is tf.layers.batch_normalization's inference form
(training=False: gamma * x / sqrt(1 + 1e-3) + beta, utils.py:300-301).
"""
from . import tf
from .layers import (Avg_Pooling, Batch_Normalization, Concat, Conv2D_Block, Deconv2D_Block, Dropout, ReLU)

N_FILTERS_FIRST_CONV = 48
GROWTH_RATE = 16
THETA = 0.5
N_LAYERS_PER_BLOCKS = [4, 5, 7, 10, 12, 15]
KEEP_PROB = 0.2            # Network/model/FCDenseNet.py:13


def bottleneck_layer(x, growth_rate, keep_prob, name):
    """Network/model/FCDenseNet.py:23-35."""
    with tf.name_scope(name):
        x = Batch_Normalization(x)
        x = ReLU(x)
        x = Conv2D_Block(x, 4 * growth_rate, filter_height=1, filter_width=1, stride=1, name=name + "_conv1")
        x = Dropout(x, keep_prob=keep_prob)

        x = Batch_Normalization(x)
        x = ReLU(x)
        x = Conv2D_Block(x, growth_rate, stride=1, name=name + "_conv2")
        x = Dropout(x, keep_prob=keep_prob)
        return x


def Transition_Layer(x, theta, name):
    """Network/model/FCDenseNet.py:37-46 (avg pool, despite the comment above
    the reference model that says max pool)."""
    with tf.name_scope(name):
        x = Batch_Normalization(x)
        x = ReLU(x)
        in_channel = int(x.shape[-1])
        x = Conv2D_Block(x, int(in_channel * theta), filter_height=1, filter_width=1, stride=1, name=name + "_conv")
        x = Avg_Pooling(x, name=name + "avg_pool")
        return x


def DenseBlock(x, num_bottleneck_layers, growth_rate, keep_prob, name):
    """Network/model/FCDenseNet.py:48-61."""
    layers_concat = [x]
    x = bottleneck_layer(x, growth_rate=growth_rate, keep_prob=keep_prob, name=name + "bottleneck_layer_0")
    layers_concat.append(x)
    for i in range(num_bottleneck_layers):
        x = Concat(layers_concat, axis=-1, name=name + "bottleneck_layer_concatenate_" + str(i + 1))
        x = bottleneck_layer(x, growth_rate=growth_rate, keep_prob=keep_prob,
                             name=name + "bottleneck_layer_" + str(i + 1))
        layers_concat.append(x)
    return Concat(layers_concat, axis=-1, name=name + "bottleneck_layer_concatenate_final")


def FCDenseNet(x, keep_prob, num_classes):
    """Network/model/FCDenseNet.py:83-163 -> (prediction [N,H,W,1], logits)."""
    n_layers = N_LAYERS_PER_BLOCKS
    dense_init = Conv2D_Block(x, N_FILTERS_FIRST_CONV, name="dense_init")

    dense_block1 = DenseBlock(dense_init, n_layers[0], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock1")
    transition_down1 = Transition_Layer(dense_block1, theta=THETA, name="transition_layer1")
    dense_block2 = DenseBlock(transition_down1, n_layers[1], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock2")
    transition_down2 = Transition_Layer(dense_block2, theta=THETA, name="transition_layer2")
    dense_block3 = DenseBlock(transition_down2, n_layers[2], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock3")
    transition_down3 = Transition_Layer(dense_block3, theta=THETA, name="transition_layer3")
    dense_block4 = DenseBlock(transition_down3, n_layers[3], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock4")
    transition_down4 = Transition_Layer(dense_block4, theta=THETA, name="transition_layer4")
    dense_block5 = DenseBlock(transition_down4, n_layers[4], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock5")
    transition_down5 = Transition_Layer(dense_block5, theta=THETA, name="transition_layer5")
    dense_block6 = DenseBlock(transition_down5, n_layers[5], growth_rate=GROWTH_RATE, keep_prob=keep_prob,
                              name="denseblock6")

    # decoder: the reference hard-codes the transposed-conv input widths
    transition_up1 = Deconv2D_Block(dense_block6, dense_block5.get_shape(), 430, tf.shape(dense_block5),
                                    name="transition_up1")
    tu_db_concat1 = Concat([transition_up1, dense_block5], axis=-1, name="tu_db_concat1")
    transition_up2 = Deconv2D_Block(tu_db_concat1, dense_block4.get_shape(), 696, tf.shape(dense_block4),
                                    name="transition_up2")
    tu_db_concat2 = Concat([transition_up2, dense_block4], axis=-1, name="tu_db_concat2")
    transition_up3 = Deconv2D_Block(tu_db_concat2, dense_block3.get_shape(), 560, tf.shape(dense_block3),
                                    name="transition_up3")
    tu_db_concat3 = Concat([transition_up3, dense_block3], axis=-1, name="tu_db_concat3")
    transition_up4 = Deconv2D_Block(tu_db_concat3, dense_block2.get_shape(), 416, tf.shape(dense_block2),
                                    name="transition_up4")
    tu_db_concat4 = Concat([transition_up4, dense_block2], axis=-1, name="tu_db_concat4")
    transition_up5 = Deconv2D_Block(tu_db_concat4, dense_block1.get_shape(), 320, tf.shape(dense_block1),
                                    name="transition_up5")
    tu_db_concat5 = Concat([transition_up5, dense_block1], axis=-1, name="tu_db_concat5")

    final_conv = Conv2D_Block(tu_db_concat5, num_classes, filter_height=1, filter_width=1, name="final_conv")
    prediction = tf.argmax(final_conv, dimension=3, name="prediction")
    return tf.expand_dims(prediction, dim=3), final_conv
