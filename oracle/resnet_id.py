"""CPU restatement of the step-1 collar-ID classifier (TEST INFRASTRUCTURE ONLY: imported by tests/,
smoke() and bench.py's cpu_baseline leg, never by the product path).

Reference: ``classify_patches`` (src/pipeline/step1_proc2d.py:140-163) feeds each tracked box's
patch ``img[y1:y2, x1:x2]`` (:301-302) through ``cv2.resize(patch, (224, 224), INTER_LINEAR)`` and
mmpretrain's ``ImageClassificationInferencer`` built from
model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py:

* test pipeline (:93-99 ``test_dataloader.dataset.pipeline``): ResizeEdge(scale=256, edge='short')
  (cv2 bilinear), CenterCrop(224), PackInputs;
* data_preprocessor (:9-22): to_rgb, mean (123.675, 116.28, 103.53), std (58.395, 57.12, 57.375);
* model (:40-73): ResNet depth 152, style 'pytorch' (stride on the 3x3 conv), out_indices (3,),
  BatchNorm in eval mode -> GlobalAveragePooling -> LinearClsHead(2048 -> 6);
* prediction: softmax, ``pred_label`` = argmax, ``pred_score`` = max probability.

mmpretrain 1.2.0 and cv2 are third-party and absent here: the ResNet and pipeline
semantics are restated from their published definitions (torchvision-equivalent ResNet v1.5
Bottleneck; mmpretrain ResizeEdge / CenterCrop rounding), so parity with mmpretrain itself is
unpinned; the resize follows oracle/swin_det.resize_linear_u8 (OpenCV fixed point).
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle.swin_det import resize_linear_u8

ID_CLASSES = ["b", "d", "g", "r", "unknown", "w"]
MEAN = (123.675, 116.28, 103.53)
STD = (58.395, 57.12, 57.375)
BN_EPS = 1e-5
DEPTH_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}
STAGE_WIDTHS = (64, 128, 256, 512)


def numpy_slice(img, box):
    """img[y1:y2, x1:x2] with Python slice semantics (negative starts wrap) -> (y0, y1, x0, x1) bounds."""
    x1, y1, x2, y2 = (int(v) for v in box)
    H, W = img.shape[:2]
    ys = range(H)[slice(y1, y2)]
    xs = range(W)[slice(x1, x2)]
    if len(ys) == 0 or len(xs) == 0:
        return None
    return ys.start, ys.stop, xs.start, xs.stop


def resize_edge(img, scale=256, edge="short"):
    """mmpretrain ResizeEdge: the short edge to ``scale``, the other int(scale * other / short)."""
    h, w = img.shape[:2]
    if (edge == "short" and w < h) or (edge == "long" and w > h):
        width, height = scale, int(scale * h / w)
    else:
        height, width = scale, int(scale * w / h)
    return resize_linear_u8(img, width, height)


def center_crop(img, crop=224):
    """mmpretrain CenterCrop: y1 = max(0, int(round((h - crop) / 2.))), same for x."""
    h, w = img.shape[:2]
    y1 = max(0, int(round((h - crop) / 2.0)))
    x1 = max(0, int(round((w - crop) / 2.0)))
    return img[y1:y1 + crop, x1:x1 + crop]


def preprocess(patch_bgr, input_size=224, edge=256, crop=224):
    """classify_patches' resize + the inferencer pipeline + data_preprocessor -> (3, crop, crop) f32."""
    r = resize_linear_u8(np.ascontiguousarray(patch_bgr), input_size, input_size)
    r = center_crop(resize_edge(r, edge), crop)
    x = torch.from_numpy(np.ascontiguousarray(r[..., ::-1])).float().permute(2, 0, 1)
    return (x - torch.tensor(MEAN).view(3, 1, 1)) / torch.tensor(STD).view(3, 1, 1)


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, BN_EPS)


def forward(sd, x, depth=152):
    """ImageClassifier.forward(mode='tensor') + softmax on (N, 3, 224, 224) f32 -> (logits, probs)."""
    x = F.relu(_bn(F.conv2d(x, sd["backbone.conv1.weight"], stride=2, padding=3), sd, "backbone.bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for si, nb in enumerate(DEPTH_BLOCKS[depth]):
        for bi in range(nb):
            p = f"backbone.layer{si + 1}.{bi}"
            stride = 2 if (bi == 0 and si > 0) else 1
            idn = x
            h = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"]), sd, p + ".bn1"))
            h = F.relu(_bn(F.conv2d(h, sd[p + ".conv2.weight"], stride=stride, padding=1), sd, p + ".bn2"))
            h = _bn(F.conv2d(h, sd[p + ".conv3.weight"]), sd, p + ".bn3")
            if bi == 0:
                idn = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], stride=stride), sd, p + ".downsample.1")
            x = F.relu(h + idn)
    feat = x.mean(dim=(2, 3))
    logits = feat @ sd["head.fc.weight"].t() + sd["head.fc.bias"]
    return logits, torch.softmax(logits, dim=1)


def classify_patches(sd, patches, input_size=224, depth=152):
    """classify_patches (step1_proc2d.py:140-163) with the restated model: list of {pred_label, pred_score}."""
    out = [{"pred_label": -1, "pred_score": 0.0} for _ in patches]
    valid = [(i, p) for i, p in enumerate(patches) if p.shape[0] > 0 and p.shape[1] > 0]
    if not valid:
        return out
    x = torch.stack([preprocess(p, input_size) for _, p in valid])
    with torch.no_grad():
        _, probs = forward(sd, x, depth)
    for (i, _), pr in zip(valid, probs):
        out[i] = {"pred_label": int(pr.argmax()), "pred_score": float(pr.max())}
    return out
