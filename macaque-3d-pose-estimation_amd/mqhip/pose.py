"""ViTPose top-down pose on MI355X through libmq_hip.

``VitPoseHip`` owns one native ``mq_vitpose`` (bf16 weights in HBM, workspace,
hipGraph cache).  All tensors passed in are torch CUDA tensors; nothing here
computes on the CPU.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .weights import VIT_H, VitPoseConfig

HM_H, HM_W = 64, 48
INPUT_W, INPUT_H = 192, 256


class VitPoseHip:
    def __init__(self, cfg: VitPoseConfig = VIT_H, weights: dict | None = None, device: int = 0,
                 graph: bool = True):
        self.cfg = cfg
        self.device = device
        self.ctx = _lib.Context.get(device)
        self.lib = self.ctx.lib
        h = C.c_void_p()
        _lib.check(self.lib.mq_vitpose_create(self.ctx.handle, cfg.embed_dims, cfg.num_layers, cfg.num_heads,
                                              cfg.ffn, cfg.n_joints, C.byref(h)), "mq_vitpose_create")
        self.handle = h
        self.dev = torch.device("cuda", device)
        if weights is not None:
            self.load_state_dict(weights)
        _lib.check(self.lib.mq_vitpose_set_graph(self.handle, 1 if graph else 0), "mq_vitpose_set_graph")

    def load_state_dict(self, weights: dict):
        for name, t in weights.items():
            if not (name.startswith("backbone.") or name.startswith("head.")):
                continue
            if name.endswith("num_batches_tracked"):
                continue
            src = t.detach().to(device=self.dev, dtype=torch.float32).contiguous()
            _lib.check(self.lib.mq_vitpose_set_param(self.handle, name.encode(), _lib.ptr(src), src.numel(), 1),
                       f"mq_vitpose_set_param({name})")
        _lib.check(self.lib.mq_vitpose_finalize(self.handle), "mq_vitpose_finalize")

    def __del__(self):
        try:
            if getattr(self, "handle", None) is not None:
                self.lib.mq_vitpose_destroy(self.handle)
        except Exception:
            pass

    # ------------------------------------------------------------------ stages
    def crop(self, frames: torch.Tensor, boxes: torch.Tensor, box_frame: torch.Tensor):
        """frames uint8 (V,H,W,3) BGR; boxes f32 (n,4) xyxy; box_frame int32 (n,)."""
        assert frames.dtype == torch.uint8 and frames.dim() == 4 and frames.shape[-1] == 3
        n = boxes.shape[0]
        V, H, W, _ = frames.shape
        frames = frames.contiguous()
        boxes = boxes.to(self.dev, torch.float32).contiguous()
        box_frame = box_frame.to(self.dev, torch.int32).contiguous()
        crops = torch.empty((n, 3, INPUT_H, INPUT_W), device=self.dev, dtype=torch.float32)
        center = torch.empty((n, 2), device=self.dev, dtype=torch.float32)
        scale = torch.empty((n, 2), device=self.dev, dtype=torch.float32)
        _lib.check(self.lib.mq_crop_udp(self.ctx.handle, _lib.ptr(frames), H * W * 3, H, W, _lib.ptr(boxes),
                                        _lib.ptr(box_frame), n, _lib.ptr(crops), _lib.ptr(center), _lib.ptr(scale),
                                        _lib.stream_ptr(self.dev)), "mq_crop_udp")
        return crops, center, scale

    def forward(self, crops: torch.Tensor, flip_test: bool = True, out: torch.Tensor | None = None):
        n = crops.shape[0]
        assert crops.shape[1:] == (3, INPUT_H, INPUT_W) and crops.dtype == torch.float32
        crops = crops.contiguous()
        if out is None:
            out = torch.empty((n, self.cfg.n_joints, HM_H, HM_W), device=self.dev, dtype=torch.float32)
        _lib.check(self.lib.mq_vitpose_forward(self.handle, _lib.ptr(crops), n, 1 if flip_test else 0, _lib.ptr(out),
                                               _lib.stream_ptr(self.dev)), "mq_vitpose_forward")
        return out

    def decode(self, heatmaps: torch.Tensor, center: torch.Tensor, scale: torch.Tensor):
        n, J, hh, ww = heatmaps.shape
        heatmaps = heatmaps.contiguous()
        kp = torch.empty((n, J, 2), device=self.dev, dtype=torch.float64)
        score = torch.empty((n, J), device=self.dev, dtype=torch.float32)
        am = torch.empty((n, J), device=self.dev, dtype=torch.int32)
        kp_hm = torch.empty((n, J, 2), device=self.dev, dtype=torch.float32)
        center, scale = center.contiguous(), scale.contiguous()
        _lib.check(self.lib.mq_decode_udp(self.ctx.handle, _lib.ptr(heatmaps), n, J, hh, ww,
                                          _lib.ptr(center), _lib.ptr(scale), _lib.ptr(kp),
                                          _lib.ptr(score), _lib.ptr(am), _lib.ptr(kp_hm), _lib.stream_ptr(self.dev)),
                   "mq_decode_udp")
        return kp, score, am, kp_hm

    def topdown(self, frames, boxes, box_frame, flip_test=True):
        """inference_topdown over every box of every view in one batch."""
        crops, center, scale = self.crop(frames, boxes, box_frame)
        hm = self.forward(crops, flip_test)
        kp, score, am, _ = self.decode(hm, center, scale)
        return kp, score, am


def decode_heatmaps(heatmaps: torch.Tensor, center: torch.Tensor, scale: torch.Tensor, device: int = 0):
    """Stand-alone mq_decode_udp (no model needed)."""
    ctx = _lib.Context.get(device)
    dev = torch.device("cuda", device)
    n, J, hh, ww = heatmaps.shape
    kp = torch.empty((n, J, 2), device=dev, dtype=torch.float64)
    score = torch.empty((n, J), device=dev, dtype=torch.float32)
    am = torch.empty((n, J), device=dev, dtype=torch.int32)
    kp_hm = torch.empty((n, J, 2), device=dev, dtype=torch.float32)
    heatmaps, center, scale = heatmaps.contiguous(), center.contiguous(), scale.contiguous()
    _lib.check(ctx.lib.mq_decode_udp(ctx.handle, _lib.ptr(heatmaps), n, J, hh, ww,
                                     _lib.ptr(center), _lib.ptr(scale), _lib.ptr(kp),
                                     _lib.ptr(score), _lib.ptr(am), _lib.ptr(kp_hm), _lib.stream_ptr(dev)),
               "mq_decode_udp")
    return kp, score, am, kp_hm


def crop_boxes(frames: torch.Tensor, boxes: torch.Tensor, box_frame: torch.Tensor, device: int = 0):
    """Stand-alone mq_crop_udp."""
    ctx = _lib.Context.get(device)
    dev = torch.device("cuda", device)
    n = boxes.shape[0]
    V, H, W, _ = frames.shape
    crops = torch.empty((n, 3, INPUT_H, INPUT_W), device=dev, dtype=torch.float32)
    center = torch.empty((n, 2), device=dev, dtype=torch.float32)
    scale = torch.empty((n, 2), device=dev, dtype=torch.float32)
    frames = frames.contiguous()
    boxes = boxes.to(dev, torch.float32).contiguous()
    box_frame = box_frame.to(dev, torch.int32).contiguous()
    _lib.check(ctx.lib.mq_crop_udp(ctx.handle, _lib.ptr(frames), H * W * 3, H, W,
                                   _lib.ptr(boxes),
                                   _lib.ptr(box_frame), n, _lib.ptr(crops),
                                   _lib.ptr(center), _lib.ptr(scale), _lib.stream_ptr(dev)), "mq_crop_udp")
    return crops, center, scale
