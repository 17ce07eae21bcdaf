"""Host-logic test of the Session compiler (no GPU): the C-ABI is replaced by a
recording stub so plan construction, fusion decisions, buffer allocation and
launch order can be checked on CPU.  Nothing is computed -- numerics are
covered by the -m gpu tests."""
import numpy as np
import pytest
import torch

from semanticsegmentation_tensorflow_amd import _lib, ops
from semanticsegmentation_tensorflow_amd import graph as G
from semanticsegmentation_tensorflow_amd import session as S
from semanticsegmentation_tensorflow_amd import tf
from semanticsegmentation_tensorflow_amd.fcn import FCN


class _Rec:
    def __init__(self, real):
        self.real = real
        self.calls = []

    def __getattr__(self, name):
        real_fn = getattr(self.real, name)
        host_only = name in ("seg_conv_desc_init", "seg_tconv_desc_init", "seg_conv_workspace",
                             "seg_bias_grad_workspace", "seg_xent_workspace", "seg_status_string",
                             "seg_adam_segments_plan", "seg_tconv_filter_apad",
                             "seg_conv_wgrad_adam_fusable", "seg_conv_bwd_data_bn_workspace",
                             "seg_conv2d_fwd_pool_ok", "seg_conv2d_fwd_bn2_ok", "seg_conv2d_fwd_hwio_ok",
                             "seg_conv2d_fwd_relu_bits_ok", "seg_conv2d_bwd_data_bits_ok")

        def fn(*a):
            if host_only:
                return real_fn(*a)
            self.calls.append(name)
            return 0
        return fn


@pytest.fixture
def dry(monkeypatch):
    real = _lib.load()
    rec = _Rec(real)
    monkeypatch.setattr(_lib, "lib", lambda: rec)
    monkeypatch.setattr(ops, "stream_ptr", lambda s=None: None)
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    return rec


def test_fcn_train_plan(dry):
    G.reset_default_graph()
    H, W = 64, 96
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = FCN(image, keep, 2).create()
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    img = np.zeros((2, H, W, 3), np.float32)
    lab = np.zeros((2, H, W), np.uint8)
    dry.calls.clear()
    sess.run([train, loss], feed_dict={image: img, labels: lab, keep: 0.8})
    c = dry.calls
    # forward: 17 fused conv launches, 3 tconv, 5 pools, 1 loss; a pool whose
    # conv's kernel has the pooled epilogue runs inside that conv's launch
    fused = c.count("seg_conv2d_fwd_pool")
    # conv6 / conv7 read their one (HWIO) packed copy
    assert c.count("seg_conv2d_fwd_hwio") == 2
    # conv1_1 (first-layer kernel) also writes its ReLU mask as bits, read by
    # conv1_2's input gradient instead of the 16-bit map
    assert c.count("seg_conv2d_fwd_relu_bits") == 1
    assert c.count("seg_conv2d_bwd_data_bits") == 1
    assert (c.count("seg_conv2d_fwd") + c.count("seg_conv2d_fwd_hwio") + c.count("seg_conv2d_fwd_relu_bits")
            + fused == 17)
    assert c.count("seg_tconv2d_fwd") == 3
    # train plans record the pool switches; MaxPoolGrad reads them instead of x
    assert c.count("seg_maxpool2x2_fwd_argmax") + fused == 5
    assert fused >= 1                                  # conv1_2 (conv_res64) at least
    assert c.count("seg_softmax_xent_fwd_bwd") == 1
    # backward: conv1_1 needs no input gradient (image is a placeholder)
    assert c.count("seg_conv2d_bwd_data") + c.count("seg_conv2d_bwd_data_bits") == 16
    # conv6 / conv7 filters (bf16, 256x256 TN tiles without split-K) take the
    # wgrad+Adam fused launch; the other 15 the plain filter gradient
    assert c.count("seg_conv2d_bwd_filter") == 15
    assert c.count("seg_conv2d_bwd_filter_adam") == 2
    assert c.count("seg_tconv2d_bwd_data") == 3
    assert c.count("seg_tconv2d_bwd_filter") == 3
    assert c.count("seg_maxpool2x2_bwd_argmax") == 5
    assert c.count("seg_adam_tf1_pack") == 1          # one fused multi-tensor launch
    # skip fusion: pool3/pool4 gradients = sum of two consumers, the second
    # accumulated in its input-gradient epilogue (no separate add)
    assert c.count("seg_add") == 0
    # filter copies are packed once per update (first run) -- KRSC for the 15 convs
    # below 8 M elements, HWIO for the 16 with input grads (conv6 / conv7 HWIO
    # only), 2 layouts x 3 tconvs
    assert c.count("seg_pack_filter") == 15 + 16 + 6
    assert c.index("seg_adam_tf1_pack") > c.index("seg_conv2d_bwd_filter")
    dry.calls.clear()
    sess.run(train, feed_dict={image: img, labels: lab, keep: 1.0})
    # the fused Adam launch rewrote every packed copy: no repack pass
    assert dry.calls.count("seg_pack_filter") == 0
    assert dry.calls.count("seg_adam_tf1_pack") == 1
    # the segment table covers every variable once (except the two filters
    # updated by the fused wgrad+Adam launches), with both copies of each conv
    assert dry.calls.count("seg_conv2d_bwd_filter_adam") == 2
    (gk, plan), = sess._adam_groups.items()
    assert plan.nsegs == len(sess.store.vars) - 2
    assert "conv6/weights" not in gk[1] and "conv7/weights" not in gk[1]
    assert (dry.calls.count("seg_conv2d_fwd") + dry.calls.count("seg_conv2d_fwd_pool")
            + dry.calls.count("seg_conv2d_fwd_hwio") + dry.calls.count("seg_conv2d_fwd_relu_bits")) == 17


def test_adam_segment_plan_host():
    """seg_adam_segments_plan: tile prefix over 32x128 [a][b] tiles per rs slice."""
    lib = _lib.load()
    arr = (ops.AdamSegment * 3)()
    for e, (rs, a, b) in zip(arr, [(9, 3, 64), (1, 1, 130), (49, 512, 4096)]):
        e.rs, e.a, e.b = rs, a, b
    import ctypes
    total = lib.seg_adam_segments_plan(ctypes.byref(arr), 3)
    assert [e.tile_begin for e in arr] == [0, 9, 9 + 2]
    assert total == 9 + 2 + 49 * 16 * 32
    assert ctypes.sizeof(ops.AdamSegment) == 56
    bad = (ops.AdamSegment * 1)()
    assert lib.seg_adam_segments_plan(ctypes.byref(bad), 1) < 0      # rs = 0


def test_inference_plan_has_no_backward(dry):
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 64, 96, 3])
    pred, logits = FCN(image, 1.0, 2).create()
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f32")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run(pred, feed_dict={image: np.zeros((1, 64, 96, 3), np.float32)})
    assert "seg_conv2d_bwd_data" not in dry.calls
    assert dry.calls.count("seg_argmax") == 1


def test_hwio_only_filter_stays_single_copy(dry):
    """FCN conv6 / conv7 (>= 8 M elements) keep ONE packed bf16 copy: the
    training plan reads their HWIO copy in the forward (seg_conv2d_fwd_hwio).
    A second plan at another batch size and an inference plan of the same
    Session reuse that choice, so the store never gains a KRSC copy that every
    later training step's update would rewrite (planner.py)."""
    G.reset_default_graph()
    H, W = 64, 96
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = FCN(image, keep, 2).create()
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    big = {n for n, v in sess.store.by_name.items() if len(v.shape) == 4 and int(np.prod(v.shape)) >= (1 << 23)}
    assert len(big) == 2, big           # conv6, conv7

    def packs():
        return {k for k in sess.store.packed if k[0] in big}
    sess.run(train, feed_dict={image: np.zeros((4, H, W, 3), np.float32),
                               labels: np.zeros((4, H, W), np.uint8), keep: 0.8})
    first = packs()
    assert first == {(n, ops.PACK_HWIO) for n in big}, first
    assert sess.store.hwio_only == big
    dry.calls.clear()
    sess.run(train, feed_dict={image: np.zeros((1, H, W, 3), np.float32),
                               labels: np.zeros((1, H, W), np.uint8), keep: 0.8})
    sess.run(pred, feed_dict={image: np.zeros((1, H, W, 3), np.float32), keep: 1.0})
    assert packs() == first
    assert dry.calls.count("seg_conv2d_fwd_hwio") >= 4


def test_tconv_shape_rule_at_375x1242(dry):
    """The reference cannot run 375x1242 through FCN: same here."""
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, 375, 1242, 3])
    pred, logits = FCN(image, 1.0, 2).create()
    sess = S.Session(device=torch.device("cpu"))
    with pytest.raises(ValueError):
        sess.run(logits, feed_dict={image: np.zeros((1, 375, 1242, 3), np.float32)})


def test_fcdensenet_train_plan(dry):
    """C3 model plans: 125 convs + 5 transposed, pre-activation BN+ReLU fused,
    dropout in the conv epilogues; the concats of dense blocks 1-4 are channel
    views of one buffer per block, and those block buffers are themselves
    channel slices of the decoder concats [transition_up_k, dense_block]
    (k = 2..5, nested views: the transposed conv writes its slice, its input
    gradient is the first write into the decoder concat's gradient buffer).
    Blocks 5 and 6 start from 140 / 174 channels and decoder concat 1 joins
    348-channel parts (slices would not start on 16-byte chunks): their
    13 + 16 + 1 concats run (fwd) and split (bwd)."""
    from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
    G.reset_default_graph()
    H, W = 64, 96
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = FCDenseNet(image, keep, 2)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run([train, loss], feed_dict={image: np.zeros((1, H, W, 3), np.float32),
                                       labels: np.zeros((1, H, W), np.uint8), keep: 0.8})
    c = dry.calls
    # stem + 118 bottleneck + 5 transition + head = 125 convs; the 1x1 convs
    # whose input has a multiple of 8 channels read BN+ReLU through their
    # operand prologue (the BatchNorm is folded, its output never written):
    # dense blocks 1-4 (5 + 6 + 8 + 11 bottlenecks) and 4 transitions -- blocks
    # 5 and 6 start from 140 / 174 channels (140 + 16 i, 174 + 16 i)
    fwd = ("seg_conv2d_fwd", "seg_conv2d_fwd_pro", "seg_conv2d_fwd_bn2")
    assert sum(c.count(f) for f in fwd) == 125
    n_fold = 5 + 6 + 8 + 11 + 4
    assert c.count("seg_tconv2d_fwd") == 5
    assert c.count("seg_concat_fwd") == 1 + (12 + 1) + (15 + 1)
    assert c.count("seg_concat_bwd") == c.count("seg_concat_fwd")
    # every bottleneck conv1 also writes the BN2 + ReLU map feeding its growth
    # conv (seg_conv2d_fwd_bn2: the BN's forward pass never re-reads the conv
    # output); the n_fold - 4 of them with a folded BN1 prologue among them
    assert c.count("seg_conv2d_fwd_bn2") == 59
    assert c.count("seg_conv2d_fwd_pro") == 4
    assert c.count("seg_bn_relu_fwd") == 123 - n_fold - 59
    # the 59 bottleneck conv1 -> Dropout -> BN chains: the dropout gradient
    # rides in the BN backward; only the growth convs' dropouts keep a pass
    # BN backward inside the consuming conv's input-gradient launch: the n_fold
    # folded 1x1 convs, the 59 growth convs (3x3 over BN -> ReLU, with the
    # bottleneck conv1's dropout gradient) and the 27 decoder-block 1x1 convs
    # whose BN stays materialised in the forward (input is a copying concat)
    assert c.count("seg_conv2d_bwd_data_bn") == n_fold + 59 + 27
    assert c.count("seg_bn_relu_bwd") + c.count("seg_bn_relu_dropout_bwd") == 123 - (n_fold + 59 + 27)
    assert c.count("seg_bn_relu_dropout_bwd") == 0
    assert c.count("seg_dropout_bwd_ch") == 59
    assert c.count("seg_avgpool2x2_fwd") == 5
    assert c.count("seg_conv2d_bwd_filter") + c.count("seg_conv2d_bwd_filter_pro") == 125
    assert c.count("seg_conv2d_bwd_filter_pro") == n_fold
    assert c.count("seg_adam_tf1_pack") == 1


def test_dropout_before_folded_bn_keeps_its_own_gradient(dry):
    """Conv -> Dropout -> BN -> ReLU -> 1x1 conv.  The BN is folded
    into the 1x1 conv's operand prologue (its backward rides in that conv's
    input-gradient epilogue, which has no dropout stage), so the first conv's
    dropout gradient must stay a separate mask re-draw, not be handed to the BN."""
    from semanticsegmentation_tensorflow_amd import layers as L
    G.reset_default_graph()
    H, W = 32, 48
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    h = L.Conv2D_Block(image, 16, 3, 3, name="c1")
    h = tf.nn.dropout(h, keep)
    h = L.Batch_Normalization(h)
    h = tf.nn.relu(h)
    logits = L.Conv2D_Block(h, 2, 1, 1, name="c2")
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="bf16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run([train, loss], feed_dict={image: np.zeros((1, H, W, 3), np.float32),
                                       labels: np.zeros((1, H, W), np.uint8), keep: 0.5})
    plan = next(iter(sess.plans.values()))
    assert plan.folded and not plan.drop_fold
    c = dry.calls
    assert c.count("seg_conv2d_fwd_pro") == 1
    assert c.count("seg_conv2d_bwd_data_bn") == 1
    assert c.count("seg_dropout_bwd_ch") == 1



def test_pool_fusion_choice_at_c2_shapes():
    """(host) conv -> MaxPool fusion at the benchmarked 4 x 384 x 1248 FCN:
    conv1_2 (conv_res64), conv2_2 (conv_halo_duo), conv3_3 / conv4_4
    (conv_halo2 256x256) carry the pooled epilogue; conv5_3 splits K (3 fp32
    slabs + a reducer) and keeps the separate pool; fp32 never fuses."""
    take = [(4, 384, 1248, 64, 64), (4, 192, 624, 128, 128), (4, 96, 312, 256, 256), (4, 48, 156, 512, 512)]
    for N, H, W, C, K in take:
        d = ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.BF16)
        assert ops.conv2d_fwd_pool_ok(d), (H, W, C, K)
        assert ops.conv2d_fwd_pool_ok(ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.F16)), (H, W, C, K)
        assert not ops.conv2d_fwd_pool_ok(ops.conv_desc(N, H, W, C, K, 3, 3, dtype=ops.F32))
    assert not ops.conv2d_fwd_pool_ok(ops.conv_desc(4, 24, 78, 512, 512, 3, 3, dtype=ops.BF16))
    # odd output size (375 x 1242 unpadded is even; 375 x 1241 is not): no whole windows
    assert not ops.conv2d_fwd_pool_ok(ops.conv_desc(1, 375, 1241, 64, 64, 3, 3, dtype=ops.BF16))


def test_deeplab_aspp_concat_is_a_view(dry):
    """C5: the ASPP concat [image pooling, aspp0..3] (Network/utils/utils.py
    :186-229, 332) is a channel view: the branches' BatchNorm+ReLU and the
    image-pooling branch's 1x1 -> HxW broadcast write their slices of one
    buffer, the concat_projection conv's input gradient is the first write into
    its gradient buffer and the branches read theirs from it -- no concat copy
    in either direction."""
    from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
    G.reset_default_graph()
    H, W = 64, 96
    image = tf.placeholder(tf.float32, [None, H, W, 3])
    labels = tf.placeholder(tf.uint8, [None, H, W])
    keep = tf.placeholder(tf.float32)
    pred, logits = DeepLabASPP(image, keep, 2)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels))
    train = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = S.Session(device=torch.device("cpu"), compute_dtype="f16")
    sess.run(tf.global_variables_initializer())
    dry.calls.clear()
    sess.run([train, loss], feed_dict={image: np.zeros((1, H, W, 3), np.float32),
                                       labels: np.zeros((1, H, W), np.uint8), keep: 0.8})
    c = dry.calls
    assert c.count("seg_concat_fwd") == 0
    assert c.count("seg_concat_bwd") == 0
    assert c.count("seg_spatial_broadcast") >= 1        # the image-pooling resize, into its slice
    (p,) = [q for q in sess.plans.values() if q.train]
    assert len(p.alias_nodes) == 1
