"""The augmentation oracle (oracle/augment.py) against the golden vectors made
by PIL + the reference's numpy lines (tests/golden/make_augment_golden.py),
and the crop draw order of crop_image (Network/model/FCN.py:176-182)."""
import os
import random

import numpy as np
import pytest

from oracle import augment as A

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "augment.npz"))


@pytest.mark.parametrize("c", [3, 4])
def test_resize_matches_pil_golden(c):
    src = G[f"c{c}_src"]
    shape = tuple(G["shape"])
    H0, W0 = src.shape[:2]
    y1, x1, nh, nw = G["window"]
    crop = src[y1:y1 + nh, x1:x1 + nw]
    assert np.array_equal(A.imresize(src, shape), G[f"c{c}_full"])
    assert np.array_equal(A.imresize(crop, (H0, W0)), G[f"c{c}_crop_full"])
    assert np.array_equal(A.imresize(crop, shape), G[f"c{c}_crop"])
    assert np.array_equal(A.imresize(src[:, ::-1], shape), G[f"c{c}_flip"])
    assert np.array_equal(A.imresize(src, (H0, W0)), G[f"c{c}_same"])
    assert np.array_equal(A.imresize(src, (H0, 2 * W0 + 3)), G[f"c{c}_wide"])
    assert np.array_equal(A.imresize(src, (2 * H0 - 7, W0)), G[f"c{c}_tall"])
    assert np.array_equal(A.bc_img(G[f"c{c}_full"], 0.93, -17), G[f"c{c}_bc"])
    assert np.array_equal(A.bc_img(G[f"c{c}_full"], 1.15, 30), G[f"c{c}_bc_hi"])


def test_gt_labels_golden():
    gt = G["gt_src"]
    shape = tuple(G["shape"])
    y1, x1, nh, nw = G["window"]
    assert np.array_equal(A.process_gt_image(A.imresize(gt, shape)), G["gt_full"])
    assert np.array_equal(A.process_gt_image(A.imresize(gt[y1:y1 + nh, x1:x1 + nw], shape)), G["gt_crop"])
    assert np.array_equal(A.process_gt_image(A.imresize(gt[:, ::-1], shape)), G["gt_flip"])
    assert np.array_equal(A.process_gt_image(A.imresize(gt, gt.shape[:2])), G["gt_same"])


def test_crop_window_draw_order():
    """randint(1150, w-5), int(nw/3.3), randint(0, w-nw), randint(0, h-nh)."""
    a, b = random.Random(7), random.Random(7)
    for _ in range(20):
        y1, x1, nh, nw = A.crop_window(375, 1242, a)
        enw = b.randint(1150, 1242 - 5)
        enh = int(enw / 3.3)
        ex1 = b.randint(0, 1242 - enw)
        ey1 = b.randint(0, 375 - enh)
        assert (y1, x1, nh, nw) == (ey1, ex1, enh, enw)


def test_full_size_against_pil():
    """KITTI sizes (375x1242 RGBA 'merge' image) -> image_shape (160, 576) and a
    crop -> 375x1242 upscale, directly against PIL when it is importable."""
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (375, 1242, 4), dtype=np.uint8)
    img[..., 3] = rng.choice(np.array([255, 255, 120, 0], np.uint8), (375, 1242))
    for arr, shape in ((img, (160, 576)), (img[20:20 + 360, 30:30 + 1190], (375, 1242))):
        want = np.asarray(Image.fromarray(np.ascontiguousarray(arr), "RGBA").resize((shape[1], shape[0]),
                                                                                   Image.BILINEAR))
        assert np.array_equal(A.imresize(arr, shape), want)
