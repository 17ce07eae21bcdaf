"""seg_augment (the GPU half of gen_batch_function, Network/model/FCN.py:235-307)
bit-exact against the PIL golden vectors and the numpy oracle
(oracle/augment.py), from fixture sizes to KITTI's 375x1242."""
import os
import random

import numpy as np
import pytest
import torch

from oracle import augment as A
from semanticsegmentation_tensorflow_amd import data, ops

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "augment.npz"))


def _aug(src, views, shape, labels=False):
    s = torch.from_numpy(np.ascontiguousarray(src)).cuda()
    C = src.shape[2]
    out = torch.empty((len(views),) + tuple(shape) + (() if labels else (C,)), dtype=torch.uint8, device="cuda")
    ops.augment([(s,) + v for v in views], C, shape[0], shape[1], out, labels=labels)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("c", [3, 4])
def test_augment_golden(dev, c):
    src = G[f"c{c}_src"]
    H0, W0 = src.shape[:2]
    shape = tuple(G["shape"])
    win = tuple(int(v) for v in G["window"])
    full = (0, 0, H0, W0)
    got = _aug(src, [(full, False, False, 1.0, 0), (win, False, False, 1.0, 0), (full, True, False, 1.0, 0),
                     (full, False, True, 0.93, -17), (full, False, True, 1.15, 30)], shape)
    for i, key in enumerate(("full", "crop", "flip", "bc", "bc_hi")):
        assert np.array_equal(got[i], G[f"c{c}_{key}"]), key
    assert np.array_equal(_aug(src, [(win, False, False, 1.0, 0)], (H0, W0))[0], G[f"c{c}_crop_full"])
    assert np.array_equal(_aug(src, [(full, False, False, 1.0, 0)], (H0, W0))[0], G[f"c{c}_same"])
    assert np.array_equal(_aug(src, [(full, False, False, 1.0, 0)], (H0, 2 * W0 + 3))[0], G[f"c{c}_wide"])
    assert np.array_equal(_aug(src, [(full, False, False, 1.0, 0)], (2 * H0 - 7, W0))[0], G[f"c{c}_tall"])


def test_augment_labels_golden(dev):
    gt = G["gt_src"]
    H0, W0 = gt.shape[:2]
    shape = tuple(G["shape"])
    win = tuple(int(v) for v in G["window"])
    full = (0, 0, H0, W0)
    got = _aug(gt, [(full, False, False, 1.0, 0), (win, False, False, 1.0, 0), (full, True, False, 1.0, 0)],
               shape, labels=True)
    for i, key in enumerate(("full", "crop", "flip")):
        assert np.array_equal(got[i], G[f"gt_{key}"][..., 1].astype(np.uint8)), key
    same = _aug(gt, [(full, False, False, 1.0, 0)], (H0, W0), labels=True)[0]
    assert np.array_equal(same, G["gt_same"][..., 1].astype(np.uint8))


@pytest.mark.parametrize("c", [3, 4])
def test_augment_kitti_size(dev, c):
    """375x1242 image: the reference's three samples at image_shape (160, 576)
    (FCN.py's training size) and the crop upscaled back to 375x1242."""
    rng = np.random.default_rng(11 + c)
    img = rng.integers(0, 256, (375, 1242, c), dtype=np.uint8)
    if c == 4:
        img[..., 3] = rng.choice(np.array([255, 255, 255, 90, 0, 1], np.uint8), (375, 1242))
    y1, x1, nh, nw = A.crop_window(375, 1242, random.Random(5))
    full = (0, 0, 375, 1242)
    views = [(full, False, True, 1.07, -31), ((y1, x1, nh, nw), False, False, 1.0, 0), (full, True, False, 1.0, 0)]
    got = _aug(img, views, (160, 576))
    want = [A.bc_img(A.imresize(img, (160, 576)), 1.07, -31), A.imresize(img[y1:y1 + nh, x1:x1 + nw], (160, 576)),
            A.imresize(img[:, ::-1], (160, 576))]
    for i in range(3):
        assert np.array_equal(got[i], want[i]), i
    up = _aug(img, [((y1, x1, nh, nw), False, False, 1.0, 0)], (375, 1242))[0]
    assert np.array_equal(up, A.imresize(img[y1:y1 + nh, x1:x1 + nw], (375, 1242)))


def test_augment_many_views(dev):
    """More views than one launch carries (kernel-argument block of 24)."""
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (30, 50, 3), dtype=np.uint8)
    views = [((i % 5, i % 7, 20 + i % 3, 30 + i % 11), bool(i % 2), bool(i % 3 == 0), 0.9 + 0.01 * i, i - 20)
             for i in range(53)]
    got = _aug(img, views, (17, 23))
    for i, ((y0, x0, h, w), flip, bc, s, m) in enumerate(views):
        win = img[y0:y0 + h, x0:x0 + w]
        want = A.imresize(win[:, ::-1] if flip else win, (17, 23))
        if bc:
            want = A.bc_img(want, s, m)
        assert np.array_equal(got[i], want), i


def test_augment_rejects_bad_views(dev):
    img = torch.zeros((10, 12, 3), dtype=torch.uint8, device="cuda")
    out = torch.empty((1, 5, 5, 3), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        ops.augment([(img, (0, 3, 10, 10), False, False, 1.0, 0)], 3, 5, 5, out)   # window past the edge
    with pytest.raises(ValueError):
        ops.augment([(img, (0, 0, 10, 12), False, False, 1.0, 0)], 3, 1, 1, torch.empty(
            (1, 1, 1, 3), dtype=torch.uint8, device="cuda"))   # 12x downscale: beyond the supported 8x


def test_gen_batch_function_end_to_end(dev, tmp_path):
    """PNG files on disk -> get_batches_fn -> device batch, against the oracle
    run with the same seeded draws (shuffle, crop, contrast, brightness)."""
    from PIL import Image
    rng = np.random.default_rng(9)
    (tmp_path / "merge").mkdir()
    (tmp_path / "gt_image_2").mkdir()
    names = ["um_000000.png", "um_000001.png", "uu_000007.png"]
    for i, nm in enumerate(names):
        img = rng.integers(0, 256, (375, 1242, 4), dtype=np.uint8)
        gt = np.zeros((375, 1242, 3), np.uint8)
        gt[:] = (255, 0, 0)
        gt[200 + 10 * i:, 300:900] = (255, 0, 255)
        Image.fromarray(img, "RGBA").save(tmp_path / "merge" / nm)
        Image.fromarray(gt, "RGB").save(tmp_path / "gt_image_2" / nm.replace("_0", "_road_0"))
    shape = (160, 576)
    fn = data.gen_batch_function(str(tmp_path), shape, rng=random.Random(3), workers=2)
    got = list(fn(2, one_hot=True))
    assert [g[0].shape[0] for g in got] == [6, 3]
    # oracle with the same draw sequence
    orng = random.Random(3)
    paths = sorted(str(tmp_path / "merge" / n) for n in names)
    orng.shuffle(paths)
    k = 0
    for b, (ims, gts) in enumerate(got):
        for j in range(ims.shape[0] // 3):
            p = paths[k]
            k += 1
            img = np.asarray(Image.open(p))
            gt = np.asarray(Image.open(tmp_path / "gt_image_2" / os.path.basename(p).replace("_0", "_road_0")))
            wi, wg = A.augment_file(img, gt, shape, orng)
            assert np.array_equal(ims[3 * j:3 * j + 3].cpu().numpy(), wi), (b, j)
            assert np.array_equal(gts[3 * j:3 * j + 3].cpu().numpy(), wg), (b, j)


def test_prepare_input_u8(dev):
    img = torch.randint(0, 256, (2, 5, 7, 3), dtype=torch.uint8)
    x = torch.full((2, 8, 8, 8), float("nan"), dtype=torch.bfloat16, device="cuda")
    ops.prepare_input(img.cuda(), x)
    ref = torch.zeros(2, 8, 8, 8)
    ref[:, :5, :7, :3] = img.float()
    torch.cuda.synchronize()
    assert torch.equal(x.cpu(), ref.to(torch.bfloat16))
