"""Host logic of the evaluator (no GPU): IoU from a confusion matrix and the
reference's RGBA road-mask overlay rule (softmax > 0.5, utils.py:43-61)."""
import numpy as np

from semanticsegmentation_tensorflow_amd import evaluate as E


def test_confusion_to_iou():
    conf = np.array([[50, 10], [5, 35]])
    miou, iou = E.confusion_to_iou(conf)
    assert np.allclose(iou, [50 / 65, 35 / 50])
    assert abs(miou - (50 / 65 + 35 / 50) / 2) < 1e-12
    # a class that never occurs is left out of the mean
    miou1, iou1 = E.confusion_to_iou(np.array([[10, 0], [0, 0]]))
    assert miou1 == 1.0 and np.isnan(iou1[1])


def test_paste_mask():
    sm = np.zeros((2, 3, 2))
    sm[..., 1] = [[0.2, 0.5, 0.51], [0.9, 0.0, 1.0]]
    m = E.paste_mask(sm, (2, 3))
    assert m.shape == (2, 3, 4) and m.dtype == np.uint8
    assert np.array_equal(m[..., 1] == 255, sm[..., 1] > 0.5)
    assert (m[sm[..., 1] > 0.5] == [0, 255, 0, 127]).all()
