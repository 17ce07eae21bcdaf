"""KITTI road training data: `gen_batch_function` (Network/model/FCN.py:235-307,
Network/utils/utils.py:94-162) with the augmentation on the GPU.

Per file the reference decodes the `merge/*.png` image and its
`gt_image_2/*_road_*.png` label, makes three samples -- resized original with
bc_img brightness/contrast, resized random crop_image window, resized
flip_image -- and one-hot labels from process_gt_image.  Here:

  * decoding stays on the host (PIL, as scipy.misc.imread; zlib inflate is
    serial work), on a thread pool, one batch ahead of the consumer;
  * decoded images go to HBM once per file (pinned staging, async copy);
  * the three samples and their labels are made by two `seg_augment`
    launches per batch (bit-exact PIL bilinear resample, crop, flip, bc_img,
    process_gt_image), into uint8 device tensors that feed the image /
    annotation placeholders directly (`seg_prepare_input_u8` pads them into
    the compute layout inside the train step).

Random draws use Python's `random` in the reference's order -- shuffle of
the file list, then per file crop_image's three randint, uniform contrast,
randint brightness -- so a seeded `random.Random` reproduces the reference's
augmentation parameters for the same file list.
"""
from __future__ import annotations

import ctypes
import os
import random
import re
import threading
from concurrent.futures import ThreadPoolExecutor
from glob import glob
from queue import Queue

import numpy as np
import torch

from . import ops


def img_size(image):
    return image.shape[0], image.shape[1]


def crop_window(h, w, rng=random):
    """crop_image's draws (Network/model/FCN.py:176-182): (y1, x1, nh, nw)."""
    nw = rng.randint(1150, w - 5)
    nh = int(nw / 3.3)
    x1 = rng.randint(0, w - nw)
    y1 = rng.randint(0, h - nh)
    return y1, x1, nh, nw


def png_decode(data):
    """Decode PNG bytes with seg_png_decode (native, releases the GIL); None
    for PNG variants it does not take (palette, 16-bit, interlaced)."""
    from ._lib import lib
    L = lib()
    h, w, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if L.seg_png_info(data, len(data), ctypes.byref(h), ctypes.byref(w), ctypes.byref(c)) != 0:
        return None
    out = np.empty((h.value, w.value, c.value), np.uint8)
    if L.seg_png_decode(data, len(data), out.ctypes.data, out.nbytes) != 0:
        return None
    return out


def imread(path):
    """scipy.misc.imread: uint8 HxWxC array (RGB / RGBA as stored; grey
    images come back HxW like scipy's).  8-bit non-interlaced PNGs go through
    the native decoder, anything else through PIL."""
    with open(path, "rb") as f:
        raw = f.read()
    a = png_decode(raw)
    if a is None:
        import io
        from PIL import Image
        with Image.open(io.BytesIO(raw)) as im:
            if im.mode == "P":
                im = im.convert("RGBA" if "transparency" in im.info else "RGB")
            a = np.array(im)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[..., 0]
    return a


def file_pairs(data_folder):
    """(image, label) paths as the reference pairs them: `merge/*.png` with
    the `gt_image_2/*_road_*.png` of the same name minus `_road`/`_lane`."""
    image_paths = sorted(glob(os.path.join(data_folder, "merge", "*.png")))
    label_paths = {re.sub(r"_(lane|road)_", "_", os.path.basename(p)): p
                   for p in glob(os.path.join(data_folder, "gt_image_2", "*_road_*.png"))}
    return image_paths, label_paths


def file_views(image, gt, rng=random):
    """The three samples of one file (reference order) as augment views:
    [(window, flip, bc, contrast, bright)] -- original (+bc), crop, flip.
    Draw order matches the reference: crop_image first, then contrast and
    brightness (Network/model/FCN.py:273, :291-293)."""
    h, w = img_size(image)
    if gt.shape[:2] != (h, w):
        raise ValueError("image and ground truth sizes differ")
    y1, x1, nh, nw = crop_window(h, w, rng)
    contrast = rng.uniform(0.85, 1.15)
    bright = rng.randint(-45, 30)
    full = (0, 0, h, w)
    return [(full, False, True, contrast, bright), ((y1, x1, nh, nw), False, False, 1.0, 0),
            (full, True, False, 1.0, 0)]


class Batch:
    """One augmented batch in HBM: images uint8 [3B,H,W,C], labels uint8 [3B,H,W]
    (0 = background, 1 = road: channel 1 of process_gt_image's one-hot)."""

    def __init__(self, images, labels, names):
        self.images, self.labels, self.names = images, labels, names

    def one_hot(self):
        """process_gt_image's bool [3B,H,W,2] (background, not background)."""
        return torch.stack((self.labels == 0, self.labels != 0), dim=-1)


def augment_batch(decoded, image_shape, rng=random, device=None, stream=None):
    """decoded: [(image uint8 HxWxC, gt uint8 HxWx3)] host arrays or device
    tensors -> Batch on `device` (the reference's batch of 3 x len(decoded))."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    oh, ow = image_shape
    C = decoded[0][0].shape[2]
    views, gviews, keep = [], [], []
    for image, gt in decoded:
        if image.shape[2] != C:
            raise ValueError("all images of a batch must have the same channel count")
        im_d = _to_device(image, device)
        gt_d = _to_device(gt[..., :3] if gt.shape[2] > 3 else gt, device)
        keep += [im_d, gt_d]
        for win, flip, bc, contrast, bright in file_views(image, gt, rng):
            views.append((im_d, win, flip, bc, contrast, bright))
            gviews.append((gt_d, win, flip, False, 1.0, 0))
    n = len(views)
    images = torch.empty((n, oh, ow, C), dtype=torch.uint8, device=device)
    labels = torch.empty((n, oh, ow), dtype=torch.uint8, device=device)
    ops.augment(views, C, oh, ow, images, labels=False, stream=stream)
    ops.augment(gviews, 3, oh, ow, labels, labels=True, stream=stream)
    b = Batch(images, labels, None)
    b._keep = keep      # sources stay alive until the launches are done
    return b


def _to_device(a, device):
    if isinstance(a, torch.Tensor):
        return a.to(device).contiguous()
    t = torch.from_numpy(np.ascontiguousarray(a))
    if device.type == "cuda":
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


def gen_batch_function(data_folder, image_shape, rng=None, workers=8, device=None):
    """Network/model/FCN.py:235 `gen_batch_function(data_folder, image_shape)`:
    returns get_batches_fn(batch_size) yielding (images, gt_images) per
    batch -- here uint8 device tensors [3B,H,W,C] and class-index labels
    [3B,H,W] (feed them to a uint8 [N,H,W] annotation placeholder; pass
    one_hot=True for the reference's bool [3B,H,W,2]).  PNG decoding runs
    `workers` threads one batch ahead."""
    rng = rng or random

    def get_batches_fn(batch_size, one_hot=False):
        image_paths, label_paths = file_pairs(data_folder)
        rng.shuffle(image_paths)
        batches = [image_paths[i:i + batch_size] for i in range(0, len(image_paths), batch_size)]
        pool = ThreadPoolExecutor(max_workers=workers)

        def decode(paths):
            futs = [(pool.submit(imread, p), pool.submit(imread, label_paths[os.path.basename(p)])) for p in paths]
            return [(a.result(), b.result()) for a, b in futs]

        q: Queue = Queue(maxsize=2)

        def producer():
            try:
                for paths in batches:
                    q.put((paths, decode(paths)))
            except BaseException as e:     # surfaced in the consumer
                q.put(e)
                return
            q.put(None)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                paths, dec = item
                b = augment_batch(dec, image_shape, rng, device)
                b.names = [os.path.basename(p) for p in paths]
                yield b.images, (b.one_hot() if one_hot else b.labels)
        finally:
            th.join(timeout=0.1)
            pool.shutdown(wait=False)

    return get_batches_fn
