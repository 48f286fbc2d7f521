"""mmpose-compatible pose API on MI355X: ``init_model`` + ``inference_topdown``.

Drop-in for the two calls the reference makes (``src/pipeline/step1_proc2d.py``:40
import, :100-101 ``init_pose_model(POSE_CONFIG, POSE_CHECKPOINT, device)`` and
``pose_model.test_cfg = ...``, :294-298 ``inference_topdown(pose_model, img,
bboxes=np.float32 (N,4), bbox_format="xyxy")``).  Results expose
``pred_instances.keypoints`` (1, J, 2) float64 image pixels and
``pred_instances.keypoint_scores`` (1, J) float32, as read at step1_proc2d.py:308-312.

The mmengine config file is read as data (``ast``; nothing in it is executed) to
pick the backbone arch; the checkpoint is loaded with ``torch.load(weights_only=True)``.
Without a checkpoint the model gets seeded random weights (the reference's weights
are not distributed with it, README.md:86).

MI355X-first extension: ``inference_topdown_batch`` runs every box of every view of
a frame (or of many frames) in ONE batched crop -> ViT -> decode launch sequence.
"""
from __future__ import annotations

import ast
import os
import warnings
from types import SimpleNamespace

import numpy as np
import torch

from .pose import VitPoseHip
from .weights import CONFIGS, VIT_H, load_mmpose_checkpoint, make_random_weights

_ARCH = {"huge": "huge", "h": "huge", "base": "base", "b": "base", "tiny": "tiny"}


def _literal_config(path):
    """Top-level ``name = <literal>`` assignments of an mmengine config file."""
    out = {}
    if not path or not os.path.exists(path):
        return out
    tree = ast.parse(open(path).read(), filename=path)
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            try:
                out[node.targets[0].id] = _eval_node(node.value)
            except ValueError:
                pass
    return out


def _eval_node(node):
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id == "dict" and not node.args:
        return {kw.arg: _eval_node(kw.value) for kw in node.keywords}
    if isinstance(node, ast.Dict):
        return {_eval_node(k): _eval_node(v) for k, v in zip(node.keys, node.values)}
    if isinstance(node, (ast.List, ast.Tuple)):
        vals = [_eval_node(e) for e in node.elts]
        return vals if isinstance(node, ast.List) else tuple(vals)
    return ast.literal_eval(node)


class PoseModelHip:
    """Stands in for mmpose's TopdownPoseEstimator at the step-1 call sites."""

    def __init__(self, cfg, weights, device_index, flip_indices=None):
        self.cfg = cfg
        self.device_index = device_index
        self.net = VitPoseHip(cfg, weights, device=device_index, graph=True)
        self.test_cfg = dict(flip_test=True, flip_mode="heatmap", shift_heatmap=False)
        self.dataset_meta = {"flip_indices": flip_indices}

    @property
    def flip_test(self):
        tc = self.test_cfg or {}
        if tc.get("flip_test", False) and tc.get("flip_mode", "heatmap") != "heatmap":
            raise NotImplementedError("only flip_mode='heatmap' is implemented (the reference's setting)")
        if tc.get("shift_heatmap", False):
            raise NotImplementedError("shift_heatmap=True is not on the reference's path")
        return bool(tc.get("flip_test", False))


def init_model(config, checkpoint=None, device="cuda:0", cfg_options=None, seed: int = 0):
    """mmpose.apis.init_model equivalent (step1_proc2d.py:100)."""
    conf = _literal_config(config) if isinstance(config, str) else (config or {})
    arch = "huge"
    try:
        arch = _ARCH.get(str(conf["model"]["backbone"]["arch"]).lower(), "huge")
    except (KeyError, TypeError):
        pass
    cfg = CONFIGS.get(arch, VIT_H)
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else 0
    if checkpoint and os.path.exists(checkpoint):
        weights = load_mmpose_checkpoint(checkpoint)
    else:
        if checkpoint:
            warnings.warn(f"checkpoint {checkpoint} not found: using seeded random ViTPose-{cfg.name} weights")
        weights = make_random_weights(cfg, seed=seed, device=torch.device("cuda", idx))
    return PoseModelHip(cfg, weights, idx)


def _sample(kp, sc, bbox):
    inst = SimpleNamespace(keypoints=kp[None], keypoint_scores=sc[None], bboxes=bbox[None],
                           bbox_scores=np.ones(1, dtype=np.float32))
    return SimpleNamespace(pred_instances=inst)


def inference_topdown_batch(model: PoseModelHip, imgs, bboxes_per_img):
    """Every box of every image in one batch.  imgs: list of HxWx3 uint8 BGR (same size)
    or a uint8 tensor (V,H,W,3) already on the GPU; bboxes_per_img: list of (Ni,4) xyxy."""
    dev = torch.device("cuda", model.device_index)
    if isinstance(imgs, torch.Tensor):
        frames = imgs.to(dev)
    else:
        frames = torch.from_numpy(np.ascontiguousarray(np.stack(imgs))).to(dev)
    boxes, owner = [], []
    for i, b in enumerate(bboxes_per_img):
        b = np.asarray(b, dtype=np.float32).reshape(-1, 4)
        boxes.append(b)
        owner += [i] * len(b)
    if not owner:
        return [[] for _ in bboxes_per_img]
    allb = np.concatenate(boxes)
    kp, score, _ = model.net.topdown(frames, torch.from_numpy(allb).to(dev),
                                     torch.tensor(owner, dtype=torch.int32, device=dev), flip_test=model.flip_test)
    kp, score = kp.cpu().numpy(), score.cpu().numpy()
    out = [[] for _ in bboxes_per_img]
    for k, i in enumerate(owner):
        out[i].append(_sample(kp[k], score[k], allb[k]))
    return out


def inference_topdown(model: PoseModelHip, img, bboxes=None, bbox_format="xyxy"):
    """mmpose.apis.inference_topdown equivalent for an ndarray image (step1_proc2d.py:294-298)."""
    if isinstance(img, str):
        raise NotImplementedError("image paths need an image decoder; pass the decoded BGR ndarray")
    img = np.asarray(img)
    h, w = img.shape[:2]
    if bboxes is None or len(bboxes) == 0:
        bboxes = np.array([[0, 0, w, h]], dtype=np.float32)
    bboxes = np.asarray(bboxes, dtype=np.float32).reshape(-1, 4)
    assert bbox_format in {"xyxy", "xywh"}
    if bbox_format == "xywh":
        bboxes = np.concatenate([bboxes[:, :2], bboxes[:, :2] + bboxes[:, 2:]], axis=1)
    return inference_topdown_batch(model, [img], [bboxes])[0]
