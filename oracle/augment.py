"""KITTI training-data augmentation restated in numpy (TEST INFRASTRUCTURE ONLY).

Follows `gen_batch_function` (Network/model/FCN.py:235-307, identical in
Network/utils/utils.py:94-162) and its helpers:
  crop_image        Network/model/FCN.py:176-182
  flip_image        Network/model/FCN.py:184-185
  bc_img            Network/model/FCN.py:187-193
  process_gt_image  Network/model/FCN.py:195-201
  scipy.misc.imresize(arr, image_shape)  (interp='bilinear')

`scipy.misc.imresize` hands the uint8 array to PIL (toimage: 3 channels ->
'RGB', 4 -> 'RGBA'; uint8 data is not rescaled) and calls
`Image.resize((w, h), BILINEAR)`.  That is Pillow's ImagingResample
(libImaging/Resample.c): per axis, a triangle filter widened by the
downscale factor (antialiasing), coefficients normalised in float64 and
rounded to 22-bit fixed point, a horizontal pass with 8-bit clipping, then a
vertical pass; an unchanged size returns a copy.  'RGBA' images are resampled
premultiplied ('RGBa', libImaging/Convert.c rgba2rgbA / rgbA2rgba).  PIL is
third-party (the reference pins no version); this restatement is pinned
against the PIL in this image by tests/golden/make_augment_golden.py.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def _c_int(x: float) -> int:
    """C (int) cast of a double: truncation toward zero."""
    return int(math.trunc(x))


def resample_coeffs(in_size: int, out_size: int):
    """precompute_coeffs + normalize_coeffs_8bpc for BILINEAR (support 1) on
    box (0, in_size): returns (xmin[out], count[out], k[out, ksize] int64)."""
    scale = float(np.float32(in_size) - np.float32(0.0)) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = _c_int(math.ceil(support)) * 2 + 1
    xmins = np.zeros(out_size, np.int64)
    counts = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        xmin = _c_int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = _c_int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs(((x + xmin) - center + 0.5) * ss)
            wx = 1.0 - t if t < 1.0 else 0.0
            w.append(wx)
            ww += wx
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = _c_int(-0.5 + k * (1 << PRECISION_BITS)) if k < 0 else _c_int(0.5 + k * (1 << PRECISION_BITS))
        xmins[xx], counts[xx] = xmin, xmax
    return xmins, counts, kk


def _clip8(acc):
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img, axis, out_size):
    """One separable pass along `axis` (1 = x, 0 = y) of a uint8 HxWxC image."""
    in_size = img.shape[axis]
    xmin, cnt, kk = resample_coeffs(in_size, out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    out = np.empty((out_size,) + src.shape[1:], np.uint8)
    for o in range(out_size):
        acc = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(cnt[o]):
            acc += src[xmin[o] + t] * kk[o, t]
        out[o] = _clip8(acc)
    return np.moveaxis(out, 0, axis)


def premultiply(img):
    """rgba2rgbA: MULDIV255(c, alpha) on the colour channels."""
    a = img[..., 3:4].astype(np.int64)
    tmp = img[..., :3].astype(np.int64) * a + 128
    rgb = ((tmp >> 8) + tmp) >> 8
    return np.concatenate([rgb, a], axis=-1).astype(np.uint8)


def unpremultiply(img):
    """rgbA2rgba: 255 * c / alpha (integer division, clipped) unless alpha is 0 or 255."""
    a = img[..., 3:4].astype(np.int64)
    c = img[..., :3].astype(np.int64)
    div = np.clip((255 * c) // np.maximum(a, 1), 0, 255)
    rgb = np.where((a == 0) | (a == 255), c, div)
    return np.concatenate([rgb, a], axis=-1).astype(np.uint8)


def imresize(img, image_shape):
    """scipy.misc.imresize(img, image_shape) with interp='bilinear' (uint8 HxWx3|4)."""
    oh, ow = image_shape
    h, w = img.shape[:2]
    if (h, w) == (oh, ow):
        return img.copy()
    rgba = img.shape[2] == 4
    x = premultiply(img) if rgba else img
    # Pillow crops the source rows to those the vertical pass reads before
    # the horizontal pass; the values are the same as resampling every row.
    if ow != w:
        x = _pass(x, 1, ow)
    if oh != h:
        x = _pass(x, 0, oh)
    return unpremultiply(x) if rgba else x


def crop_window(h, w, rng):
    """crop_image's random draws (Network/model/FCN.py:178-181) from a
    `random.Random`-like rng: (y1, x1, nh, nw)."""
    nw = rng.randint(1150, w - 5)
    nh = int(nw / 3.3)
    x1 = rng.randint(0, w - nw)
    y1 = rng.randint(0, h - nh)
    return y1, x1, nh, nw


def bc_img(img, s=1.0, m=0.0):
    """Network/model/FCN.py:187-193 (np.int -> int64)."""
    x = img.astype(np.int64) * s + m
    x[x > 255] = 255
    x[x < 0] = 0
    return x.astype(np.uint8)


def process_gt_image(gt):
    """Network/model/FCN.py:195-201: one-hot [bg, not bg] (bool)."""
    bg = np.all(gt == np.array([255, 0, 0]), axis=2)[..., None]
    return np.concatenate((bg, np.invert(bg)), axis=2)


def augment_file(image, gt_image, image_shape, rng):
    """One file's three training samples in the reference's order: resized
    original with brightness/contrast, resized random crop, resized flip.
    Returns (images [3,h,w,C] uint8, gt one-hot [3,h,w,2] bool)."""
    y1, x1, nh, nw = crop_window(image.shape[0], image.shape[1], rng)
    image2, gt2 = image[y1:y1 + nh, x1:x1 + nw], gt_image[y1:y1 + nh, x1:x1 + nw]
    image3, gt3 = image[:, ::-1], gt_image[:, ::-1]
    ims = [imresize(image, image_shape), imresize(image2, image_shape), imresize(image3, image_shape)]
    gts = [imresize(gt_image, image_shape), imresize(gt2, image_shape), imresize(gt3, image_shape)]
    contrast = rng.uniform(0.85, 1.15)
    bright = rng.randint(-45, 30)
    ims[0] = bc_img(ims[0], contrast, bright)
    return np.stack(ims), np.stack([process_gt_image(g) for g in gts])
