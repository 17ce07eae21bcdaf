"""CPU restatements of the reference models (TEST INFRASTRUCTURE ONLY).

`fcn_forward` follows `Network/model/FCN.py:49-114` exactly, including the
reference's quirks: 14-conv encoder with a
4-conv block 4, 7x7 SAME conv6, ReLU on conv8, feature-width skip fusion
(conv_t1 2->512 + pool4, conv_t2 512->256 + pool3) and a 16x16 stride-8
conv_t3 with variable name `conv_t3/bias` (`:103`).

`fcdensenet_forward` follows `Network/model/FCDenseNet.py:23-163` with the
layer builders of `Network/utils/utils.py:164-333` (bias-free convs,
frozen-statistics BN, avg-pool transitions, skip-concat decoder).
"""
from __future__ import annotations

import torch

from . import tf1_ops as tf

# (name, out_channels, kernel) in build order, FCN.py:52-86
FCN_CONVS = [
    ("conv1_1", 64, 3), ("conv1_2", 64, 3),
    ("conv2_1", 128, 3), ("conv2_2", 128, 3),
    ("conv3_1", 256, 3), ("conv3_2", 256, 3), ("conv3_3", 256, 3),
    ("conv4_1", 512, 3), ("conv4_2", 512, 3), ("conv4_3", 512, 3), ("conv4_4", 512, 3),
    ("conv5_1", 512, 3), ("conv5_2", 512, 3), ("conv5_3", 512, 3),
    ("conv6", 4096, 7), ("conv7", 4096, 1),
]
POOL_AFTER = {"conv1_2": "pool1", "conv2_2": "pool2", "conv3_3": "pool3",
              "conv4_4": "pool4", "conv5_3": "pool5"}


def fcn_param_shapes(in_channels=3, num_classes=2):
    """TF variable name -> shape, in creation order (FCN.py:117-159, :101-103)."""
    shapes = {}
    c = in_channels
    for name, k, r in FCN_CONVS:
        shapes[f"{name}/weights"] = (r, r, c, k)
        shapes[f"{name}/biases"] = (k,)
        c = k
    shapes["conv8/weights"] = (1, 1, 4096, num_classes)
    shapes["conv8/biases"] = (num_classes,)
    # deconv_layer: W [4,4, shape[3], num_filters]; num_filters = INPUT depth (FCN.py:143)
    shapes["conv_t1/weights"] = (4, 4, 512, num_classes)
    shapes["conv_t1/biases"] = (512,)
    shapes["conv_t2/weights"] = (4, 4, 256, 512)
    shapes["conv_t2/biases"] = (256,)
    shapes["conv_t3/weights"] = (16, 16, num_classes, 256)
    shapes["conv_t3/bias"] = (num_classes,)
    return shapes


def conv_layer(x, p, name):
    """FCN.py:117-136: relu(conv2d(x, W, SAME) + b)."""
    return tf.relu(tf.bias_add(tf.conv2d(x, p[f"{name}/weights"]), p[f"{name}/biases"]))


def deconv_layer(x, p, name, out_shape, stride=2):
    """FCN.py:138-159: conv2d_transpose(x, W, output_shape, s, SAME) + b."""
    return tf.bias_add(tf.conv2d_transpose(x, p[f"{name}/weights"], out_shape, stride),
                       p[f"{name}/biases"])


def fcn_forward(p, x, keep_prob=1.0, dropout_u=None, num_classes=2, return_acts=False, quant=None):
    """Returns (pred [N,H,W,1] int64, logits [N,H,W,C]) like FCN.create() (FCN.py:114).

    `quant` (optional) is applied wherever a device implementation stores an
    activation (each conv/tconv layer output and the logits) -- e.g. rounding
    to bf16 -- so a reduced-precision device path can be compared at matched
    rounding points.  Gradients pass through it unchanged."""
    q = quant or (lambda t: t)
    acts = {}
    h = x
    for name, _, _ in FCN_CONVS[:14]:
        h = q(conv_layer(h, p, name))
        acts[name] = h
        if name in POOL_AFTER:
            h = tf.max_pool2x2(h)
            acts[POOL_AFTER[name]] = h
    du = dropout_u or {}
    h = q(tf.dropout(conv_layer(h, p, "conv6"), keep_prob, du.get("dropout6")))
    h = q(tf.dropout(conv_layer(h, p, "conv7"), keep_prob, du.get("dropout7")))
    conv8 = q(conv_layer(h, p, "conv8"))
    pool4, pool3 = acts["pool4"], acts["pool3"]
    t1 = deconv_layer(conv8, p, "conv_t1", tuple(pool4.shape))
    fuse1 = q(tf.add(t1, pool4))
    t2 = deconv_layer(fuse1, p, "conv_t2", tuple(pool3.shape))
    fuse2 = q(tf.add(t2, pool3))
    N, H, W, _ = x.shape
    t3 = tf.conv2d_transpose(fuse2, p["conv_t3/weights"], (N, H, W, num_classes), 8)
    logits = q(tf.bias_add(t3, p["conv_t3/bias"]))
    pred = tf.argmax(logits).unsqueeze(-1)
    if return_acts:
        acts.update(conv8=conv8, fuse_1=fuse1, fuse_2=fuse2)
        return pred, logits, acts
    return pred, logits


# ---------------------------------------------------------------------------
# FC-DenseNet ("U-Net" config), FCDenseNet.py:83-163
# ---------------------------------------------------------------------------
DENSENET_LAYERS = [4, 5, 7, 10, 12, 15]
DENSENET_GROWTH = 16
DENSENET_FIRST = 48
DENSENET_THETA = 0.5


class _BNCounter:
    """tf.layers.batch_normalization auto-names 'batch_normalization', '_1', ..."""

    def __init__(self):
        self.i = 0

    def next(self):
        name = "batch_normalization" if self.i == 0 else f"batch_normalization_{self.i}"
        self.i += 1
        return name


def fcdensenet_param_shapes(in_channels=3, num_classes=2):
    shapes = {}
    bn = _BNCounter()

    def conv(name, r, cin, cout):
        shapes[f"{name}/weights"] = (r, r, cin, cout)

    def bnv(c):
        n = bn.next()
        shapes[f"{n}/gamma"] = (c,)
        shapes[f"{n}/beta"] = (c,)

    conv("dense_init", 3, in_channels, DENSENET_FIRST)
    c = DENSENET_FIRST
    skips = []
    for b, nl in enumerate(DENSENET_LAYERS):
        name = f"denseblock{b + 1}"
        cin = c
        for i in range(nl + 1):
            ln = f"{name}bottleneck_layer_{i}"
            bnv(cin)
            conv(f"{ln}_conv1", 1, cin, 4 * DENSENET_GROWTH)
            bnv(4 * DENSENET_GROWTH)
            conv(f"{ln}_conv2", 3, 4 * DENSENET_GROWTH, DENSENET_GROWTH)
            cin += DENSENET_GROWTH
        c = cin
        if b < 5:
            skips.append(c)
            bnv(c)
            conv(f"transition_layer{b + 1}_conv", 1, c, int(c * DENSENET_THETA))
            c = int(c * DENSENET_THETA)
    for u in range(5):
        skip_c = skips[4 - u]
        shapes[f"transition_up{u + 1}/weights"] = (4, 4, skip_c, c)
        c = skip_c + skip_c
    shapes["final_conv/weights"] = (1, 1, c, num_classes)
    return shapes


def fcdensenet_forward(p, x, keep_prob=1.0, num_classes=2, quant=None, dropout_u=None):
    """`quant` as in fcn_forward: applied where the device stores an activation
    (conv / BN+ReLU / avg-pool / transposed-conv outputs; concats copy).
    `dropout_u`: {conv name: U[0,1) tensor} for the dropout after that conv
    (FCDenseNet.py:30, :34); absent entries use keep_prob with a fresh draw."""
    q = quant or (lambda t: t)
    du = dropout_u or {}

    def conv_drop(h, name):
        """Conv2D_Block + Dropout: the device applies the dropout in the conv
        epilogue and rounds once."""
        z = tf.conv2d(h, p[f"{name}/weights"])
        u = du.get(name)
        if u is None and keep_prob < 1.0:
            u = torch.rand(z.shape, dtype=torch.float32)
        return q(tf.dropout(z, keep_prob, u) if u is not None else z)
    bn = _BNCounter()

    def BN(h):
        n = bn.next()
        return tf.batch_norm_frozen(h, p[f"{n}/gamma"], p[f"{n}/beta"])

    def conv(h, name):
        return q(tf.conv2d(h, p[f"{name}/weights"]))

    def bottleneck(h, name):                       # FCDenseNet.py:23-35
        h = conv_drop(q(tf.relu(BN(h))), f"{name}_conv1")
        return conv_drop(q(tf.relu(BN(h))), f"{name}_conv2")

    def dense_block(h, nl, name):                  # FCDenseNet.py:48-61
        feats = [h]
        h = bottleneck(h, f"{name}bottleneck_layer_0")
        feats.append(h)
        for i in range(nl):
            h = tf.concat(feats)
            h = bottleneck(h, f"{name}bottleneck_layer_{i + 1}")
            feats.append(h)
        return tf.concat(feats)

    def transition(h, name):                       # FCDenseNet.py:37-46
        h = q(tf.relu(BN(h)))
        h = conv(h, f"{name}_conv")
        return q(tf.avg_pool2x2(h))

    h = conv(x, "dense_init")
    dbs = []
    for b, nl in enumerate(DENSENET_LAYERS):
        h = dense_block(h, nl, f"denseblock{b + 1}")
        if b < 5:
            dbs.append(h)
            h = transition(h, f"transition_layer{b + 1}")
    for u in range(5):                              # FCDenseNet.py:141-154
        skip = dbs[4 - u]
        t = q(tf.conv2d_transpose(h, p[f"transition_up{u + 1}/weights"], tuple(skip.shape), 2))
        h = tf.concat([t, skip])
    logits = conv(h, "final_conv")
    pred = tf.argmax(logits).unsqueeze(-1)
    return pred, logits


# ---------------------------------------------------------------------------
# DeepLab-style atrous model (config C5), semanticsegmentation_tensorflow_amd/
# deeplab.py: VGG16 backbone at output stride 8 (conv5 rate 2), ASPP (image
# pooling + 1x1 + rates 6/12/18, frozen BN + ReLU), 1x1 projection,
# classifier, bilinear x8.
# ---------------------------------------------------------------------------
DEEPLAB_ASPP_RATES = (6, 12, 18)


def deeplab_param_shapes(in_channels=3, num_classes=2, depth=256):
    shapes = {}
    chans = [("conv1_1", in_channels, 64), ("conv1_2", 64, 64), ("conv2_1", 64, 128), ("conv2_2", 128, 128),
             ("conv3_1", 128, 256), ("conv3_2", 256, 256), ("conv3_3", 256, 256), ("conv4_1", 256, 512),
             ("conv4_2", 512, 512), ("conv4_3", 512, 512), ("conv5_1", 512, 512), ("conv5_2", 512, 512),
             ("conv5_3", 512, 512)]
    for n, ci, co in chans:
        shapes[f"{n}/weights"] = (3, 3, ci, co)
        shapes[f"{n}/biases"] = (co,)
    bn = _BNCounter()

    def bnv(c):
        n = bn.next()
        shapes[f"{n}/gamma"] = (c,)
        shapes[f"{n}/beta"] = (c,)

    shapes["image_pooling/weights"] = (1, 1, 512, depth)      # DeepLabv3Plus.py:215-223
    bnv(depth)
    shapes["aspp0/weights"] = (1, 1, 512, depth)
    bnv(depth)
    for i in range(3):
        shapes[f"aspp{i + 1}/weights"] = (3, 3, 512, depth)
        bnv(depth)
    shapes["concat_projection/weights"] = (1, 1, 5 * depth, depth)
    bnv(depth)
    shapes["Last_layer/weights"] = (1, 1, depth, num_classes)
    return shapes


def deeplab_forward(p, x, keep_prob=1.0, num_classes=2, quant=None, dropout_u=None):
    """`dropout_u`: U[0,1) tensor of the projection's Dropout (deeplab.py:82)."""
    q = quant or (lambda t: t)
    bn = _BNCounter()

    def BN(h):
        n = bn.next()
        return tf.batch_norm_frozen(h, p[f"{n}/gamma"], p[f"{n}/beta"])

    def cl(h, name, rate=1):
        return q(tf.relu(tf.bias_add(tf.conv2d(h, p[f"{name}/weights"], dilation=rate), p[f"{name}/biases"])))

    h = cl(cl(x, "conv1_1"), "conv1_2")
    h = tf.max_pool2x2(h)
    h = cl(cl(h, "conv2_1"), "conv2_2")
    h = tf.max_pool2x2(h)
    h = cl(cl(cl(h, "conv3_1"), "conv3_2"), "conv3_3")
    h = tf.max_pool2x2(h)
    h = cl(cl(cl(h, "conv4_1"), "conv4_2"), "conv4_3")
    feat = cl(cl(cl(h, "conv5_1", 2), "conv5_2", 2), "conv5_3", 2)
    # image pooling: reduce_mean over H, W -> 1x1 conv -> BN -> ReLU -> align_corners resize
    gap = q(feat.mean(dim=(1, 2), keepdim=True))
    b4 = q(tf.relu(BN(q(tf.conv2d(gap, p["image_pooling/weights"])))))
    br = [q(tf.resize_bilinear(b4, (feat.shape[1], feat.shape[2])))]
    br.append(q(tf.relu(BN(q(tf.conv2d(feat, p["aspp0/weights"]))))))
    for i, r in enumerate(DEEPLAB_ASPP_RATES):
        br.append(q(tf.relu(BN(q(tf.conv2d(feat, p[f"aspp{i + 1}/weights"], dilation=r))))))
    h = tf.concat(br)
    h = q(tf.relu(BN(q(tf.conv2d(h, p["concat_projection/weights"])))))
    if dropout_u is not None or keep_prob < 1.0:
        h = q(tf.dropout(h, keep_prob, dropout_u if dropout_u is not None else torch.rand(h.shape, dtype=h.dtype)))
    last = q(tf.conv2d(h, p["Last_layer/weights"]))
    logits = q(tf.resize_bilinear(last, (x.shape[1], x.shape[2])))
    pred = tf.argmax(logits).unsqueeze(-1)
    return pred, logits
