"""Host side of the MI355X ID classifier (mqhip/resnet_id.py) vs the oracle (oracle/resnet_id.py):
the patch slice semantics of classify_patches (step1_proc2d.py:301-302), the eval-mode BatchNorm
folding the GEMM weights carry, and the preprocessing restatement's fixed points."""
import numpy as np
import torch
import torch.nn.functional as F

from mqhip import resnet_id as rid
from oracle import resnet_id as orid
from oracle.swin_det import resize_linear_u8


def test_patch_bounds_follow_numpy_slicing():
    img = np.zeros((40, 60, 3), np.uint8)
    boxes = [(5, 6, 20, 30), (-5, 3, 10, 12), (50, 30, 80, 90), (10, 10, 10, 20), (20, 5, 10, 9), (-70, -50, -1, -2),
             (0, 0, 60, 40)]
    for b in boxes:
        x1, y1, x2, y2 = b
        ref = img[y1:y2, x1:x2]
        pb = rid.patch_bounds(img.shape, b)
        assert pb == orid.numpy_slice(img, b)
        if ref.size == 0:
            assert pb is None
        else:
            y0, y1_, x0, x1_ = pb
            assert (y1_ - y0, x1_ - x0) == ref.shape[:2]


def test_bn_folding_equals_conv_then_bn():
    sd = rid.make_random_weights(50, seed=1)
    g = torch.Generator().manual_seed(0)
    for conv, bn, stride, pad in (("backbone.conv1.weight", "backbone.bn1", 2, 3),
                                  ("backbone.layer2.0.conv2.weight", "backbone.layer2.0.bn2", 2, 1),
                                  ("backbone.layer1.0.downsample.0.weight", "backbone.layer1.0.downsample.1", 1, 0)):
        co, ci, kh, kw = sd[conv].shape
        x = torch.randn(2, ci, 13, 11, generator=g)
        ref = orid._bn(F.conv2d(x, sd[conv], stride=stride, padding=pad), sd, bn)
        wm, b = rid.fold_conv_bn(sd, conv, bn)
        assert wm.shape[1] % 32 == 0 and torch.all(wm[:, kh * kw * ci:] == 0)
        cols = F.unfold(x, (kh, kw), padding=pad, stride=stride)          # (n, ci*kh*kw, L), k = c*kh*kw + tap
        cols = cols.view(2, ci, kh * kw, -1).permute(0, 3, 2, 1).reshape(2, -1, kh * kw * ci)  # k = tap*ci + c
        y = cols @ wm[:, :kh * kw * ci].t() + b
        torch.testing.assert_close(y.permute(0, 2, 1).reshape(ref.shape), ref, rtol=1e-4, atol=1e-4)


def test_preprocess_fixed_points():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    assert np.array_equal(resize_linear_u8(img, 224, 224), img)           # identity resize
    big = rng.integers(0, 256, (448, 448, 3), dtype=np.uint8)
    area = resize_linear_u8(big, 224, 224)                                # exact 2x: INTER_AREA
    ref = (big[0::2, 0::2].astype(int) + big[0::2, 1::2] + big[1::2, 0::2] + big[1::2, 1::2] + 2) >> 2
    assert np.array_equal(area, ref)
    assert orid.resize_edge(img, 256).shape == (256, 256, 3)
    assert orid.resize_edge(img[:100], 256).shape == (256, 573, 3)
    assert orid.center_crop(np.zeros((256, 256, 3)), 224).shape == (224, 224, 3)
    x = orid.preprocess(np.full((50, 30, 3), (10, 20, 30), np.uint8))
    assert x.shape == (3, 224, 224)
    torch.testing.assert_close(x[:, 0, 0], torch.tensor([(30 - 123.675) / 58.395, (20 - 116.28) / 57.12,
                                                         (10 - 103.53) / 57.375]))


def test_oracle_classifier_output_format():
    sd = rid.make_random_weights(50, seed=2)
    rng = np.random.default_rng(1)
    patches = [rng.integers(0, 256, (37, 25, 3), dtype=np.uint8), np.zeros((0, 5, 3), np.uint8)]
    out = orid.classify_patches(sd, patches, depth=50)
    assert out[1] == {"pred_label": -1, "pred_score": 0.0}
    assert 0 <= out[0]["pred_label"] < 6 and 1 / 6 <= out[0]["pred_score"] <= 1
