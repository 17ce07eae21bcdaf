"""Generate tests/golden/augment.npz: the KITTI augmentation arithmetic
(`gen_batch_function`, Network/model/FCN.py:235-307) evaluated by the
libraries the reference calls, not by our restatement:

  * resizes by PIL `Image.resize(size, BILINEAR)` -- what
    `scipy.misc.imresize(arr, image_shape)` runs (toimage keeps uint8 data;
    3 channels -> 'RGB', 4 -> 'RGBA'); scipy.misc is gone from this image's
    scipy, PIL (12.2) is present;
  * bc_img / process_gt_image written out with numpy exactly as the reference
    lines (Network/model/FCN.py:187-201; np.int is int64).

    python tests/golden/make_augment_golden.py

The crop windows are fixed here (crop_image draws nw >= 1150, which needs
full-size images); the draw order is tested on the host separately.
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def imresize(arr, shape):
    mode = {3: "RGB", 4: "RGBA"}[arr.shape[2]]
    return np.asarray(Image.fromarray(np.ascontiguousarray(arr), mode).resize((shape[1], shape[0]), Image.BILINEAR))


def bc_img(img, s, m):
    img = img.astype(np.int64)
    img = img * s + m
    img[img > 255] = 255
    img[img < 0] = 0
    return img.astype(np.uint8)


def process_gt_image(gt):
    bg = np.all(gt == np.array([255, 0, 0]), axis=2).reshape(gt.shape[0], gt.shape[1], 1)
    return np.concatenate((bg, np.invert(bg)), axis=2)


def gt_colour(rng, h, w):
    """KITTI road GT style: red background, magenta road region, a few black pixels."""
    g = np.zeros((h, w, 3), np.uint8)
    g[:] = (255, 0, 0)
    yy, xx = np.mgrid[0:h, 0:w]
    road = (yy > h * 0.55) & (np.abs(xx - w / 2) < (yy - h * 0.4) * w / h * 1.2)
    g[road] = (255, 0, 255)
    g[rng.random((h, w)) < 0.02] = (0, 0, 0)
    return g


def main():
    rng = np.random.default_rng(2024)
    out = {}
    H0, W0 = 45, 150
    shape = (20, 64)
    win = (3, 10, 30, 100)   # y1, x1, nh, nw
    for c in (3, 4):
        img = rng.integers(0, 256, (H0, W0, c), dtype=np.uint8)
        if c == 4:
            img[..., 3] = rng.choice(np.array([0, 1, 9, 128, 200, 255, 255, 255], np.uint8), (H0, W0))
        y1, x1, nh, nw = win
        crop = img[y1:y1 + nh, x1:x1 + nw]
        flip = np.flip(img, axis=1)
        out[f"c{c}_src"] = img
        out[f"c{c}_full"] = imresize(img, shape)                 # downscale
        out[f"c{c}_crop_full"] = imresize(crop, (H0, W0))        # crop -> upscale
        out[f"c{c}_crop"] = imresize(crop, shape)
        out[f"c{c}_flip"] = imresize(flip, shape)
        out[f"c{c}_same"] = imresize(img, (H0, W0))              # unchanged size: a copy
        out[f"c{c}_wide"] = imresize(img, (H0, 2 * W0 + 3))      # horizontal pass only
        out[f"c{c}_tall"] = imresize(img, (2 * H0 - 7, W0))      # vertical pass only
        out[f"c{c}_bc"] = bc_img(out[f"c{c}_full"], 0.93, -17)
        out[f"c{c}_bc_hi"] = bc_img(out[f"c{c}_full"], 1.15, 30)
    out["window"] = np.array(win, np.int64)
    out["shape"] = np.array(shape, np.int64)
    gt = gt_colour(rng, H0, W0)
    y1, x1, nh, nw = win
    out["gt_src"] = gt
    out["gt_full"] = process_gt_image(imresize(gt, shape))
    out["gt_crop"] = process_gt_image(imresize(gt[y1:y1 + nh, x1:x1 + nw], shape))
    out["gt_flip"] = process_gt_image(imresize(np.flip(gt, axis=1), shape))
    out["gt_same"] = process_gt_image(imresize(gt, (H0, W0)))
    np.savez_compressed(os.path.join(HERE, "augment.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
