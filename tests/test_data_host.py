"""Host half of the KITTI pipeline (no GPU): file pairing and the random draw
order of gen_batch_function (Network/model/FCN.py:250-293)."""
import random

import numpy as np

from oracle import augment as A
from semanticsegmentation_tensorflow_amd import data


def test_file_pairs(tmp_path):
    (tmp_path / "merge").mkdir()
    (tmp_path / "gt_image_2").mkdir()
    for n in ("um_000003.png", "umm_000010.png"):
        (tmp_path / "merge" / n).write_bytes(b"")
    for n in ("um_road_000003.png", "um_lane_000003.png", "umm_road_000010.png"):
        (tmp_path / "gt_image_2" / n).write_bytes(b"")
    images, labels = data.file_pairs(str(tmp_path))
    assert [p.split("/")[-1] for p in images] == ["um_000003.png", "umm_000010.png"]
    assert labels["um_000003.png"].endswith("um_road_000003.png")
    assert labels["umm_000010.png"].endswith("umm_road_000010.png")


def test_file_views_draw_order():
    """crop_image's three randint, then uniform contrast, randint brightness."""
    img = np.zeros((375, 1242, 3), np.uint8)
    a, b = random.Random(17), random.Random(17)
    for _ in range(10):
        v = data.file_views(img, img, a)
        y1, x1, nh, nw = A.crop_window(375, 1242, b)
        contrast = b.uniform(0.85, 1.15)
        bright = b.randint(-45, 30)
        assert v[0] == ((0, 0, 375, 1242), False, True, contrast, bright)
        assert v[1] == ((y1, x1, nh, nw), False, False, 1.0, 0)
        assert v[2] == ((0, 0, 375, 1242), True, False, 1.0, 0)
