"""Compile-time planners of the Session (mixin): BatchNorm / dropout folding,
DenseBlock concatenations as views of one buffer, static buffer allocation,
MaxPool and BN-output epilogue fusion, and the backward plan.  Split out of
session.py; `Session` inherits these methods unchanged."""
from __future__ import annotations

import torch

from . import graph as G
from . import ops
from .ops import round8


class PlanMixin:
    def _fold_bn_prologues(self, p, fetched):
        """FC-DenseNet's pre-activation BN -> ReLU -> 1x1 conv
        (Network/model/FCDenseNet.py:25-28, :39-41): a BatchNorm(+ReLU) node
        whose output feeds exactly one 1x1 conv becomes that conv's operand
        prologue -- the BN output is never written (forward) and the filter
        gradient recomputes it from x while staging.  Its backward is
        unchanged (the BN gradient re-derives the mask from x)."""
        p.folded = set()
        if not self.fold_bn:
            return
        users = {}
        for n in p.nodes:
            for t in list(n.inputs) + [getattr(n, "residual", None)]:
                if t is not None:
                    users.setdefault(id(t), []).append(n)
        for b in p.nodes:
            if b.kind != "bn" or id(b.output) in fetched:
                continue
            us = users.get(id(b.output), [])
            if len(us) != 1 or us[0].kind != "conv" or us[0].inputs[0] is not b.output:
                continue
            c = us[0]
            R, S_, C, _ = c.w.shape
            if (R, S_) != (1, 1) or c.stride != 1 or C % 8:
                continue
            c.pro = b
            p.folded.add(id(b))

    def _fold_dropout_grads(self, p, fetched):
        """Conv2D_Block -> Dropout -> Batch_Normalization (FC-DenseNet's
        bottleneck conv1, Network/model/FCDenseNet.py:28-30): the dropout sits
        in the conv's forward epilogue with no ReLU, so its gradient is a
        re-draw of the mask; when the BN is the conv output's only reader, the
        BN backward applies it (seg_bn_relu_dropout_bwd) and the conv's own
        dropout-gradient pass is skipped.  p.drop_fold: bn node id -> conv."""
        p.drop_fold = {}
        p.drop_folded = set()
        p.bn_before = {}
        if not self.fold_dropout_grad:
            return
        users = {}
        for n in p.nodes:
            for t in list(n.inputs) + [getattr(n, "residual", None)]:
                if t is not None:
                    users.setdefault(id(t), []).append(n)
        for c in p.nodes:
            if c.kind != "conv" or c.relu or getattr(c, "kp", None) is None:
                continue
            out = c.output
            if id(out) in fetched:
                continue
            us = users.get(id(out), [])
            if len(us) != 1 or us[0].kind != "bn" or us[0].inputs[0] is not out:
                continue
            if id(us[0]) in p.folded:
                # that BN runs inside a 1x1 conv's operand prologue and its
                # backward inside that conv's input-gradient epilogue, which has
                # no dropout stage: the conv keeps its own mask re-draw
                continue
            p.drop_fold[id(us[0])] = c
            p.drop_folded.add(id(c))
        # BN(+ReLU) -> 3x3 conv (FC-DenseNet's growth conv): the conv's input
        # gradient kernel can continue through that BN's backward when the BN
        # output has no other reader and its input gradient is not shared
        p.bn_before = {}
        for c in p.nodes:
            if c.kind != "conv" or getattr(c, "pro", None) is not None:
                continue
            t = c.inputs[0]
            us = users.get(id(t), [])
            b = next((n for n in p.nodes if n.kind == "bn" and n.output is t), None)
            if b is None or len(us) != 1 or id(t) in fetched:
                continue
            xb = b.inputs[0]
            if len(users.get(id(xb), [])) == 1 and id(xb) not in fetched:
                p.bn_before[id(c)] = b

    def _infer(self, op, shp):
        t = op.type
        ins = [shp.get(id(i)) for i in op.inputs]
        if t == "Conv2D":
            N, H, W, C = ins[0]
            R, S, Ci, K = ins[1]
            if Ci != C:
                raise ValueError(f"{op.name}: input depth {C} != filter depth {Ci}")
            d = ops.conv_desc(N, H, W, C, K, R, S, op.attrs["stride"], op.attrs["dilation"],
                              op.attrs["padding"], self.cdt)
            return (N, d.OH, d.OW, K)
        if t == "Conv2DTranspose":
            N, H, W, C = ins[0]
            R, S, Co, Ci = ins[1]
            os_ = G.resolve_shape(op.attrs["output_shape"], lambda tt: shp[id(tt)])
            if os_[3] != Co or Ci != C:
                raise ValueError(f"{op.name}: output/filter channel mismatch {os_} {ins[1]}")
            ops.tconv_desc(N, H, W, C, os_[1], os_[2], Co, R, S, op.attrs["stride"],
                           op.attrs["padding"], self.cdt)  # raises on TF shape-rule violation
            return (N, os_[1], os_[2], Co)
        if t in ("BiasAdd", "Relu", "Dropout", "FusedBatchNorm", "Softmax"):
            return ins[0]
        if t == "Add":
            if ins[0] != ins[1]:
                raise ValueError(f"{op.name}: incompatible shapes {ins[0]} vs {ins[1]}")
            return ins[0]
        if t in ("MaxPool", "AvgPool"):
            N, H, W, C = ins[0]
            return (N, H // 2, W // 2, C)
        if t == "ConcatV2":
            return tuple(ins[0][:3]) + (sum(s[3] for s in ins),)
        if t == "ResizeBilinear":
            N, H, W, C = ins[0]
            OH, OW = G.resolve_shape(op.attrs["size"], lambda tt: shp[id(tt)])
            return (N, int(OH), int(OW), C)
        if t == "GlobalAvgPool":          # kept 4-D on the device: [N, 1, 1, C]
            N, H, W, C = ins[0]
            return (N, 1, 1, C)
        if t == "SoftmaxXent":
            return tuple(ins[0][:3])
        if t == "Mean":
            return ()
        if t == "ArgMax":
            return tuple(ins[0][:3])
        if t == "ExpandDims":
            if len(ins[0]) == 4:          # global-average-pool chain: already [N, 1, 1, C]
                return tuple(ins[0])
            return tuple(ins[0]) + (1,)
        raise NotImplementedError(t)

    # -------------------------------------------------------------- buffers
    def _act(self, shape):
        N, H, W, C = shape
        return torch.zeros(N, H, W, round8(C), dtype=self.tdt, device=self.device)

    def _plan_concat_alias(self, p):
        """Zero-copy concatenation for FC-DenseNet's DenseBlock
        (Network/model/FCDenseNet.py:48-61), where concat i is
        [x0, h0, ..., h_i]: every concat of the block is a channel prefix of the
        last one.  That last concat (the root) gets one buffer; its parts are
        channel slices of it (their producers write there through the row
        stride) and the earlier concats are prefix views, so no concat copies
        data.  Gradients mirror this: one buffer per root, the consumers' input
        gradients accumulate into their slice (BatchNorm backward in
        accumulate mode, or a copying concat's split) and the parts' producers
        read theirs from it.

        A root qualifies when every part has a multiple of 8 channels (slices
        start on 16-byte chunks and carry no padding), is produced by a node
        that writes through a row stride (conv, pooling, BatchNorm, transposed
        conv) or is itself a concat root (nested), and is not already a slice,
        and every other reader of the group is a BatchNorm or a concat -- the
        consumers whose input gradient can land in a shared buffer in place --
        except that the root itself may have ONE conv / transposed-conv
        reader: its input gradient is the first write into the root's gradient
        buffer (it runs first in backward) and covers it whole.

        DeepLab's ASPP concat [image pooling, aspp0..3] (Network/utils/utils.py
        :186-229, 332) qualifies too: its parts are BatchNorm+ReLU outputs and
        the image-pooling branch's 1x1 -> HxW resize (a broadcast through the
        row stride), its one reader the concat_projection conv.

        Nested roots: FC-DenseNet's decoder concat [transition_up, dense_block]
        (Network/model/FCDenseNet.py:141-154) has the dense block's own root as
        a part, so that block buffer becomes a channel slice of the decoder
        buffer (offsets compose): the transposed conv writes its slice, the
        block's layers theirs, and neither concat copies."""
        p.alias = {}          # tensor id -> (root tensor id, channel offset)
        p.alias_nodes = set()  # ConcatV2 node ids that became views
        if not self.alias_concat:
            return
        nested = {}           # concat output id -> (outer root id, offset): a part of an accepted outer root
        shp = p.shapes
        producer = {id(n.output): n for n in p.nodes}
        users = {}
        for n in p.nodes:
            for t in list(n.inputs) + [getattr(n, "residual", None)]:
                if t is not None:
                    users.setdefault(id(t), []).append(n)
        fetched = {id(f) for f in p.fetches if isinstance(f, G.Tensor)}
        concats = [n for n in p.nodes if n.kind == "ConcatV2"]
        def part_ok(i):
            prod = producer.get(i)
            if prod is None or shp[i][3] % 8 or i in fetched:
                return False
            if i in p.alias:
                return False
            if prod.kind == "ResizeBilinear":
                # the 1x1 -> HxW align_corners resize is a broadcast written
                # (and its gradient, a spatial sum, read) through the row
                # stride: DeepLab's image-pooling ASPP branch
                xs = shp[id(prod.inputs[0])]
                return len(xs) == 4 and xs[1] == 1 and xs[2] == 1
            return prod.kind in ("conv", "AvgPool", "MaxPool", "bn", "tconv") or (
                prod.kind == "ConcatV2" and i not in nested)

        for root in reversed(concats):
            rid = id(root.output)
            if rid in p.alias and rid not in nested:
                continue            # a prefix view of an accepted root
            ids = [id(t) for t in root.inputs]
            if len(set(ids)) != len(ids):
                continue
            prefixes = [c for c in concats if c is not root and id(c.output) not in p.alias and
                        len(c.inputs) < len(ids) and [id(t) for t in c.inputs] == ids[:len(c.inputs)]]
            ok = all(part_ok(i) for i in ids) and (rid in nested or shp[rid][3] % 8 == 0)
            views = {root} | set(prefixes)
            group = {id(c.output) for c in views} | set(ids)
            if ok:
                root_users = users.get(rid, [])
                for g in group:
                    for u in users.get(g, []):
                        if u in views or u.kind in ("bn", "ConcatV2"):
                            continue
                        if (g == rid and len(root_users) == 1 and u.kind in ("conv", "tconv")
                                and u.inputs[0] is root.output and getattr(u, "residual", None) is not root.output):
                            continue
                        ok = False
            if not ok:
                continue
            r, base = nested.get(rid, (rid, 0))
            off = base
            for t in root.inputs:
                p.alias[id(t)] = (r, off)
                if producer[id(t)].kind == "ConcatV2":
                    nested[id(t)] = (r, off)
                off += shp[id(t)][3]
            for c in views:
                p.alias[id(c.output)] = (r, base)
                p.alias_nodes.add(id(c))

    def _allocate(self, p, consumers, feeds):
        dev = self.device
        shp = p.shapes
        buf = {}            # tensor id -> device tensor (padded)
        p.buf = buf
        self._plan_concat_alias(p)
        roots = {r: self._act(shp[r]) for r, _ in set(p.alias.values())}
        p.feed_slots = {}   # tensor id -> (kind, staging)
        store = self.store
        ws_need = 0
        p.packs = set()
        p.pack_apad = {}
        p.pool_idx = {}     # MaxPool node id -> recorded switches (train plans)
        for n in p.nodes:
            y = n.output
            if n.kind == "input":
                s = shp[id(y)]
                dt = n.ops[0].attrs["dtype"]
                if dt in (G.float32, "float32") and len(s) == 4:
                    # image placeholder: fp32 feed -> padded compute tensor
                    stage = torch.zeros(s, dtype=torch.float32, device=dev)
                    buf[id(y)] = self._act(s)
                    p.feed_slots[id(y)] = ("image", stage)
                elif dt in (G.uint8, "uint8"):
                    stage = torch.zeros(s, dtype=torch.uint8, device=dev)
                    buf[id(y)] = stage
                    p.feed_slots[id(y)] = ("raw", stage)
                elif len(s) == 0:
                    p.feed_slots[id(y)] = ("scalar", None)
                else:
                    stage = torch.zeros(s, dtype=torch.float32, device=dev)
                    buf[id(y)] = stage
                    p.feed_slots[id(y)] = ("raw", stage)
                continue
            if n.kind == "xent":
                n.loss_sum = torch.zeros(1, dtype=torch.float32, device=dev)
                lg = n.inputs[0]
                n.dlogits = torch.zeros_like(buf[id(lg)])
                N, H, W = shp[id(lg)][:3]
                vh, vw = n.valid_hw or (H, W)
                n.count = N * vh * vw
                n.num_classes = shp[id(lg)][3]
                buf[id(y)] = n.loss_sum
                continue
            if n.kind in ("ArgMax",):
                s = shp[id(y)]
                buf[id(y)] = torch.zeros(s, dtype=torch.int64, device=dev)
                continue
            if n.kind == "ExpandDims":
                src = buf[id(n.inputs[0])]
                buf[id(y)] = src if len(shp[id(y)]) == 4 and src.dim() == 4 else src.unsqueeze(-1)
                continue
            s = shp[id(y)]
            if id(n) in p.folded:
                buf[id(y)] = buf[id(n.inputs[0])]    # never written: its consumer reads x through the prologue
            elif id(y) in p.alias:
                r, off = p.alias[id(y)]
                buf[id(y)] = roots[r][..., off:off + s[3]]
            else:
                buf[id(y)] = self._act(s)
            if n.kind == "conv":
                x = n.inputs[0]
                N, H, W, C = shp[id(x)]
                R, S, _, K = n.w.shape
                n.desc = ops.conv_desc(N, H, W, C, K, R, S, n.stride, n.dilation, n.padding, self.cdt)
                ws_need = max(ws_need, ops.conv_workspace(n.desc, ops.OP_FWD))
                # a large filter (FCN conv6 / conv7) keeps ONE packed copy: its
                # forward reads the HWIO copy the input gradient reads
                # (ops.conv2d_fwd_hwio), and its fused filter-gradient + Adam
                # launch has no KRSC copy to rewrite
                # The choice is sticky per filter: once a plan made it HWIO-only,
                # every later plan (another batch size, an inference plan) that
                # can read the HWIO copy does, so no KRSC copy appears that
                # each training step's update would then rewrite.  A later
                # plan whose shape igemm_nt3 does not take
                # (conv2d_fwd_hwio_ok false) still adds the KRSC copy, and
                # the filter leaves the HWIO-only set
                # (tests/test_session_dryrun.py::test_hwio_only_filter_stays_single_copy).
                hwio_only = store.hwio_only
                name = n.w.var_name
                n.fwd_hwio = (getattr(n, "pro", None) is None and ops.conv2d_fwd_hwio_ok(n.desc)
                              and (name in hwio_only or (self.fwd_hwio and R * S * C * K >= (1 << 23)
                                                         and (name, ops.PACK_KRSC) not in store.packed)))
                if n.fwd_hwio:
                    hwio_only.add(name)
                else:
                    hwio_only.discard(name)
                if not n.fwd_hwio:
                    p.packs.add((n.w.var_name, ops.PACK_KRSC))
                if id(x) in p.needs_grad or n.fwd_hwio:
                    p.packs.add((n.w.var_name, ops.PACK_HWIO))
                if p.train:
                    ws_need = max(ws_need, ops.conv_workspace(n.desc, ops.OP_BWD_DATA),
                                  ops.conv_workspace(n.desc, ops.OP_BWD_FILTER),
                                  4 * 1024 * 2 * round8(K))
            elif n.kind == "tconv":
                x = n.inputs[0]
                N, H, W, C = shp[id(x)]
                R, S, Co, _ = n.w.shape
                _, OH, OW, _ = s
                n.desc = ops.tconv_desc(N, H, W, C, OH, OW, Co, R, S, n.stride, n.padding, self.cdt)
                ws_need = max(ws_need, ops.conv_workspace(n.desc, ops.OP_TFWD))
                ap = ops.tconv_filter_apad(n.desc)
                p.packs.add((n.w.var_name, ops.PACK_TCONV_FWD))
                p.pack_apad[(n.w.var_name, ops.PACK_TCONV_FWD)] = ap
                if id(x) in p.needs_grad:
                    p.packs.add((n.w.var_name, ops.PACK_TCONV_BWD))
                    p.pack_apad[(n.w.var_name, ops.PACK_TCONV_BWD)] = ap
                if p.train:
                    ws_need = max(ws_need, ops.conv_workspace(n.desc, ops.OP_TBWD_DATA),
                                  ops.conv_workspace(n.desc, ops.OP_TBWD_FILTER),
                                  4 * 1024 * 2 * round8(Co))
            elif n.kind == "bn":
                ws_need = max(ws_need, 4 * 1024 * 2 * round8(s[3]))
            elif n.kind == "MaxPool" and p.train and id(n.inputs[0]) in p.needs_grad:
                # the forward records its switches; MaxPoolGrad reads them, not x
                xb = buf[id(n.inputs[0])]
                if ops.maxpool_argmax_fits(xb):
                    N, H, W, C = xb.shape
                    p.pool_idx[id(n)] = torch.empty(N * (H // 2) * (W // 2) * C, dtype=torch.uint8, device=dev)
        self._plan_pool_fusion(p, consumers)
        self._plan_bn_outputs(p, consumers)
        ws_need = max(ws_need, 8192)
        self.ws.get(ws_need)
        # packed filter copies
        for name, mode in sorted(p.packs):
            ap = p.pack_apad.get((name, mode))
            old = store.packed.get((name, mode))
            if old is None or (ap is not None and old[1] != ap):
                R, S, A, B = store.by_name[name].shape
                ap = ap if ap is not None else round8(A)
                t = torch.zeros(ops.packed_shape(R, S, A, B, mode, ap), dtype=self.tdt, device=dev)
                store.packed[(name, mode)] = (t, ap, round8(B))
                self._packed_version = -1          # new copies must be filled
        # gradient buffers / plan for backward
        if p.train:
            self._plan_backward(p)

    def _plan_pool_fusion(self, p, consumers):
        """conv_layer -> max_pool (Network/model/FCN.py:56-57, :158-160): a
        ReLU conv whose only consumer is a 2x2 / 2 MaxPool runs as one launch
        (ops.conv2d_fwd_pool) that writes the pooled map and the switches; the
        conv output itself is never materialised (its gradient comes from the
        switches: MaxPoolGrad's fused ReluGrad)."""
        p.pool_fuse = {}
        p.pool_fused = set()
        if not self.fuse_pool or self.cdt == ops.F32:
            return
        for n in p.nodes:
            if (n.kind != "conv" or getattr(n, "pro", None) is not None or n.kp is not None
                    or getattr(n, "fwd_hwio", False)):
                continue
            y = n.output
            cs = consumers.get(id(y), [])
            if len(cs) != 1 or cs[0].type != "MaxPool" or id(y) in p.fetched or id(y) in p.alias:
                continue
            m = next((c for c in p.nodes if c.kind == "MaxPool" and c.ops[0] is cs[0]), None)
            if m is None or m.inputs[0] is not y:
                continue
            if p.train and id(y) in p.needs_grad and id(m) not in p.pool_idx:
                continue                       # MaxPoolGrad would read the conv output
            if not ops.conv2d_fwd_pool_ok(n.desc):
                continue
            p.pool_fuse[id(n)] = m
            p.buf[id(y)] = None                # never written
        p.pool_fused = {id(m) for m in p.pool_fuse.values()}

    def _plan_unpool_fusion(self, p, consumers):
        """max_pool -> conv_layer (Network/model/FCN.py:57-63, :63-69): the
        MaxPoolGrad (+ the ReluGrad of the post-ReLU pool input) runs in the
        epilogue of the input gradient of the pool output's first consumer in
        forward order -- the last contribution in backward, so the pooled
        gradient of any other consumer (FCN's score_pool3 / 4) is complete
        and comes in as the epilogue residual (ops.conv2d_bwd_data_unpool).
        The pooled gradient is never written and the MaxPool node's backward
        is skipped.  The pool input has no other consumer, even dims and
        recorded switches.  p.unpool_fuse: conv node id -> MaxPool node."""
        p.unpool_fuse = {}
        p.unpool_pools = set()
        if not self.fuse_unpool or self.cdt == ops.F32:
            return
        pos = {id(n): i for i, n in enumerate(p.nodes)}
        for m in p.nodes:
            if m.kind != "MaxPool" or id(m) not in p.pool_idx or id(m.output) not in p.needs_grad:
                continue
            xf, y = m.inputs[0], m.output
            if len(consumers.get(id(xf), [])) != 1 or id(xf) in p.alias or id(y) in p.alias:
                continue
            cs = consumers.get(id(y), [])
            if not cs:
                continue
            c = min(cs, key=lambda q: pos[id(q)])
            if c.kind != "conv" or c.inputs[0] is not y or getattr(c, "pro", None) is not None:
                continue
            if getattr(c, "residual", None) is y or sum(1 for q in cs if q is c) != 1:
                continue
            N, H, W = p.shapes[id(y)][:3]
            if tuple(p.shapes[id(xf)][:3]) != (N, 2 * H, 2 * W):
                continue
            if not ops.conv2d_bwd_data_unpool_ok(c.desc):
                continue
            p.unpool_fuse[id(c)] = m
        p.unpool_pools = {id(m) for m in p.unpool_fuse.values()}

    def _plan_relu_bits(self, p, consumers):
        """The ReluGrad mask as bits: a mask-fused ReLU conv whose forward runs
        on the first-layer kernel (FCN / VGG conv1_1, Network/model/FCN.py:55)
        also writes its ReLU mask at 1 bit per element, and its consumer conv's
        input gradient (conv1_2's, on conv_res64pp) reads those instead of the
        16-bit map: 8 instead of 128 bytes per pixel.  p.mask_bits: producer
        conv id -> uint8 [N, OH, OW, K/8]; p.bits_dgrad: the consumer conv ids."""
        p.mask_bits = {}
        p.bits_dgrad = set()
        if not self.relu_bits or self.cdt == ops.F32:
            return
        for n in p.nodes:
            if n.kind != "conv" or id(n) not in p.mask_fuse:
                continue
            if (id(n) in p.pool_fuse or id(n) in p.bn_out2 or getattr(n, "pro", None) is not None
                    or getattr(n, "fwd_hwio", False) or p.buf.get(id(n.output)) is None):
                continue
            c = consumers[id(n.output)][0]
            if (c.kind != "conv" or getattr(c, "pro", None) is not None or id(c) in p.bn_before
                    or id(c) in p.unpool_fuse or id(n.output) in p.alias):
                continue
            if not (ops.conv2d_fwd_relu_bits_ok(n.desc) and ops.conv2d_bwd_data_bits_ok(c.desc)):
                continue
            N, H, W = p.shapes[id(n.output)][:3]
            p.mask_bits[id(n)] = ops.relu_bits_buffer(N, H, W, n.desc.K, self.device)   # padded channels
            p.bits_dgrad.add(id(c))

    def _plan_bn_outputs(self, p, consumers):
        """Conv -> (its epilogue's dropout) -> BatchNorm(+ReLU): FC-DenseNet's
        bottleneck conv1 -> BN -> ReLU before the growth conv
        (Network/model/FCDenseNet.py:28-31).  When the BN node is the conv
        output's only forward reader, the conv launch also writes the BN(+ReLU)
        map (ops.conv2d_fwd_bn2, bit-identical to bn_relu_fwd) and the BN's own
        forward pass -- a full re-read of the conv output -- is skipped.  The
        conv output is still written: the BN backward re-derives its ReLU mask
        and dgamma from it.  p.bn_out2: conv node id -> BN node."""
        p.bn_out2 = {}
        p.bn_out2_done = set()
        if not self.fuse_bn_out or self.cdt == ops.F32:
            return
        producer = {id(n.output): n for n in p.nodes if n.kind == "conv"}
        for b in p.nodes:
            if b.kind != "bn" or id(b) in p.folded or id(b.output) in p.fetched:
                continue
            c = producer.get(id(b.inputs[0]))
            if (c is None or id(c) in p.pool_fuse or id(c) in p.bn_out2 or id(c.output) in p.fetched
                    or getattr(c, "fwd_hwio", False)):
                continue
            cs = consumers.get(id(c.output), [])
            if len(cs) != 1 or cs[0] is not b.ops[0]:
                continue
            if p.buf.get(id(c.output)) is None or p.buf.get(id(b.output)) is None:
                continue
            if not ops.conv2d_fwd_bn2_ok(c.desc, getattr(c, "pro", None) is not None):
                continue
            p.bn_out2[id(c)] = b
            p.bn_out2_done.add(id(b))

    def _plan_backward(self, p):
        dev = self.device
        grad = {}
        p.grad = grad
        p.tmp = {}
        # grads of variables go to the flat buffer; activations get their own
        covered = set()
        for n in p.nodes:
            if n.kind == "conv":
                covered.add(n.w.var_name)
                if n.bias is not None:
                    covered.add(n.bias.var_name)
            elif n.kind == "tconv":
                covered.add(n.w.var_name)
                if n.bias is not None:
                    covered.add(n.bias.var_name)
            elif n.kind == "bn":
                covered.update([n.gamma.var_name, n.beta.var_name])
            elif n.kind == "BiasAdd":
                covered.add(n.inputs[1].var_name)
        # ReluGrad fusion: a ReLU conv whose output has exactly one consumer that
        # is a conv / tconv (input gradient via the NT epilogue mask) or a
        # dropout-free max-pool (MaxPoolGrad relu flag) gets its gradient
        # already masked; it then only needs the bias column sum.
        p.producer = {id(n.output): n for n in p.nodes}
        consumers = {}
        for n in p.nodes:
            ins = list(n.inputs) + ([n.residual] if getattr(n, "residual", None) is not None else []) \
                + ([n.labels] if getattr(n, "labels", None) is not None else [])
            for t in ins:
                consumers.setdefault(id(t), []).append(n)
        p.mask_fuse = set()
        for n in p.nodes:
            if n.kind != "conv" or not n.relu or id(n.output) not in p.needs_grad:
                continue
            cs = consumers.get(id(n.output), [])
            if len(cs) != 1 or cs[0].inputs[0] is not n.output:
                continue
            c = cs[0]
            if c.kind in ("conv", "tconv") or (c.kind == "MaxPool" and n.kp is None):
                p.mask_fuse.add(id(n))
        self._plan_unpool_fusion(p, consumers)
        self._plan_relu_bits(p, consumers)
        p.adam_fusable = set()
        p.wg_ws = {}                     # per-conv filter-gradient workspace (pending split-K slabs)
        for n in p.nodes:
            if n.kind == "conv" and ops.wgrad_adam_fusable(n.desc):
                p.adam_fusable.add(id(n))
            if n.kind in ("conv", "tconv"):
                op = ops.OP_BWD_FILTER if n.kind == "conv" else ops.OP_TBWD_FILTER
                p.wg_ws[id(n)] = torch.empty(max(256, ops.conv_workspace(n.desc, op)),
                                             dtype=torch.uint8, device=self.device)
        p.var_names = [v.var_name for v in p.train.attrs["var_list"]]
        p.var_set = set(p.var_names)
        # Adam / accumulation touch var_list only (TF: minimize(var_list=...)),
        # in store (= backward) order
        p.adam_names = [v.var_name for v in self.store.order if v.var_name in p.var_set]
        p.uncovered = [v for v in p.var_names if v not in covered]
        for v in p.uncovered:            # no gradient path: keep the grad slice at 0
            self.store.grad(v).zero_()
        # variables whose gradient is never reported ready during backward
        # (outside var_list, or no gradient path): released to the
        # data-parallel buckets up front so they do not hold later buckets back
        p.never_ready = [v.var_name for v in self.store.order
                         if v.var_name not in p.var_set or v.var_name not in covered]
        # data parallel bucket schedule (var readiness in backward order)
        if self._dpa is not None:
            self.dp.prepare(self.store)
