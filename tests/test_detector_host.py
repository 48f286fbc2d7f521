"""Host-side pieces of the MI355X detector (mqhip/detector.py) vs the oracle (oracle/swin_det.py):
the cv2 INTER_LINEAR coefficient tables, the keep-ratio rescale size and the base anchors."""
import numpy as np
import torch

from mqhip import detector as det
from oracle import swin_det as sd


def test_resize_tables_equal_oracle():
    for dst, src in ((800, 2048), (600, 1536), (256, 320), (192, 240), (333, 97)):
        o1, a1 = det.linear_coeffs(dst, src)
        o2, a2 = sd._linear_coeffs(dst, src)
        assert np.array_equal(o1, o2) and np.array_equal(a1, a2)
        assert np.all(a1.sum(axis=1) == 2048)


def test_rescale_size_equals_oracle():
    for w, h in ((2048, 1536), (320, 240), (1920, 1080), (640, 640)):
        nw, nh = det.rescale_size(w, h)
        onw, onh, _ = sd.rescale_size(w, h)
        assert (nw, nh) == (onw, onh)
    assert det.rescale_size(2048, 1536) == (800, 600)


def test_base_anchors_equal_oracle():
    for s in det.STRIDES:
        assert torch.equal(det.base_anchors(s), sd.base_anchors(s))


def test_oracle_resize_keeps_constant_image():
    img = np.full((97, 131, 3), 77, dtype=np.uint8)
    out = sd.resize_linear_u8(img, 50, 40)
    assert out.shape == (40, 50, 3) and np.all(out == 77)
