"""Evaluation path: the reference's test-time helpers (softmax > 0.5 road
mask, Network/utils/utils.py:43-92) plus the mIoU evaluator the reference
lacks, computed on the GPU from the model's class map.

The reference reads PNGs from data_road/ and resizes them on the host
(scipy.misc, Network/model/FCN.py:213-233, Network/utils/utils.py:71-83);
`gen_test_output_files` does the same from a data folder with the native
PNG decoder and the PIL-exact GPU resize (data.py); `gen_test_output` takes
decoded arrays already shaped like the graph's image placeholder."""
from __future__ import annotations

import time

import numpy as np
import torch

from . import graph as G
from . import ops


def _feed(image_pl, x, keep_prob):
    d = {image_pl: x}
    if isinstance(keep_prob, G.Tensor):
        d[keep_prob] = 1.0
    return d


def paste_mask(im_soft_max, image_shape, color=1, obj_color_schema=((0, 255, 0, 127),)):
    """RGBA overlay of pixels whose class-`color` softmax exceeds 0.5
    (Network/utils/utils.py:43-61, without the PIL paste)."""
    prob = np.asarray(im_soft_max)[..., color].reshape(image_shape[0], image_shape[1])
    seg = (prob > 0.5).reshape(image_shape[0], image_shape[1], 1)
    return np.dot(seg, np.asarray(obj_color_schema, dtype=np.float64)).astype(np.uint8)


def gen_test_output(sess, softmax, keep_prob, image_pl, images, image_shape):
    """Per image: (index, RGBA road mask, softmax map, processing seconds) --
    the generator of Network/utils/utils.py:63-89 over in-memory images.
    `softmax` is tf.nn.softmax(logits) built in the same graph."""
    for i, img in enumerate(images):
        start = time.time()
        sm = sess.run(softmax, feed_dict=_feed(image_pl, np.asarray(img, np.float32)[None], keep_prob))
        processing_time = time.time() - start
        yield i, paste_mask(sm[0], image_shape), sm[0], processing_time


def gen_test_output_files(sess, softmax, keep_prob, image_pl, data_folder, image_shape):
    """Network/model/FCN.py:213-233: for each `merge/*.png` of data_folder,
    imread + imresize(image, image_shape) (on the GPU, bit-exact with
    scipy.misc/PIL), softmax, road mask; yields (basename, RGBA mask,
    resized image uint8 [h,w,C], processing seconds)."""
    import glob
    import os

    from . import data
    oh, ow = image_shape
    for path in sorted(glob.glob(os.path.join(data_folder, "merge", "*.png"))):
        start = time.time()
        img = data.imread(path)
        src = torch.from_numpy(np.ascontiguousarray(img)).cuda()
        C = img.shape[2]
        out = torch.empty((1, oh, ow, C), dtype=torch.uint8, device=src.device)
        ops.augment([(src, (0, 0, img.shape[0], img.shape[1]), False, False, 1.0, 0)], C, oh, ow, out)
        sm = sess.run(softmax, feed_dict=_feed(image_pl, out, keep_prob))
        processing_time = time.time() - start
        yield os.path.basename(path), paste_mask(sm[0], image_shape), out[0].cpu().numpy(), processing_time


def confusion_to_iou(conf):
    """Per-class IoU = TP / (TP + FP + FN) from conf[true][pred]; classes that
    never occur (zero denominator) are excluded from the mean."""
    conf = np.asarray(conf, dtype=np.float64)
    tp = np.diag(conf)
    denom = conf.sum(0) + conf.sum(1) - tp
    iou = np.where(denom > 0, tp / np.maximum(denom, 1), np.nan)
    return float(np.nanmean(iou)), iou


class MeanIoU:
    """Streaming confusion matrix on the device (seg_confusion, atomic
    per-pixel counts), masked to the valid (unpadded) image region."""

    def __init__(self, num_classes, device, valid_hw=None):
        self.C = int(num_classes)
        self.valid_hw = valid_hw
        self.conf = torch.zeros(self.C * self.C, dtype=torch.int64, device=device)

    def update(self, pred, labels):
        """pred: int64 class map [N,H,W] or [N,H,W,1] (device); labels: uint8 [N,H,W] (device)."""
        pred = pred.reshape(labels.shape).contiguous()
        ops.confusion(pred, labels.contiguous(), self.conf, self.C, self.valid_hw)
        return self

    def confusion(self):
        return self.conf.view(self.C, self.C).cpu().numpy()

    def result(self):
        return confusion_to_iou(self.confusion())


def mean_iou(sess, pred, image_pl, keep_prob, images, labels, num_classes=2, valid_hw=None, batch=4):
    """mIoU of the model's prediction (FCN(...).create()[0]) over (images,
    labels) in batches; images float32 [N,H,W,C], labels uint8 class indices."""
    dev = sess.device
    m = MeanIoU(num_classes, dev, valid_hw)
    for s in range(0, len(images), batch):
        x = np.asarray(images[s:s + batch], np.float32)
        y = torch.as_tensor(np.asarray(labels[s:s + batch], np.uint8)).to(dev)
        p = sess.run(pred, feed_dict=_feed(image_pl, x, keep_prob), as_numpy=False)
        m.update(p, y)
    miou, iou = m.result()
    return miou, iou, m.confusion()
