"""BASELINE config 5 as one hipGraph per frame: detector -> boxes -> top-down pose -> triangulation.

The reference's per-frame step-1 path (src/pipeline/step1_proc2d.py:226-298) is detector ->
BoT-SORT -> box expansion -> ``inference_topdown``; step 4 then triangulates.  Everything of it that
is per-frame arithmetic runs here in ONE captured graph over the 8 synchronized views:

  Swin-S Mask R-CNN on all views (mqhip.detector, every stage a libmq_hip launch)
  -> mq_det_topk_boxes: per view the first k detections above the score threshold whose truncated
     box is non-degenerate, expanded like step 1 (the capturable stand-in for the tracker's box list:
     the data-dependent box count becomes k static slots with a valid flag)
  -> mq_crop_udp -> mq_vitpose_forward (flip test) -> mq_decode_udp
  -> keypoints of empty slots / below the score threshold -> NaN -> mq_triangulate_dlt (omnidir
     undistort + SVD DLT) of slot a of every view as individual a (association is out of scope,
     SURVEY 8(d)).

The graph is captured with torch's hipGraph capture on the caller's device (every launch of the
sequence goes to torch's current stream; allocations come from the graph's private pool).  A frame
is fed by copying it into the static input buffer (``run(frames)``) or by writing ``self.frames``
directly (the H2D upload of the next frame can target it); ``replay()`` launches the whole frame.
BoT-SORT and the ID classifier stay on the host after the graph (mqhip.tracker, mqhip.resnet_id).
"""
from __future__ import annotations

import torch

from . import _lib

MIN_MARGIN, MAX_MARGIN, DESIRED_AR = 0.20, 0.50, 192.0 / 256.0   # step1_proc2d.py:71-73


class FramePoseGraph:
    def __init__(self, detector, pose_model, cams_dev, n_views=8, height=1536, width=2048, k=4, det_score_thr=0.85,
                 tri_score_thr=0.5, flip_test=True):
        assert getattr(pose_model, "handle", None) is not None, "pose_model: a mqhip.pose.VitPoseHip"
        self.det, self.pose = detector, pose_model
        self.ctx, self.lib = pose_model.ctx, pose_model.lib
        self.dev = torch.device("cuda", pose_model.device)
        self.V, self.H, self.W, self.k = n_views, height, width, k
        self.det_thr, self.tri_thr, self.flip = float(det_score_thr), float(tri_score_thr), flip_test
        self.cams = cams_dev
        J = pose_model.cfg.n_joints
        n = n_views * k
        d = self.dev
        self.n, self.J = n, J
        self.frames = torch.zeros((n_views, height, width, 3), dtype=torch.uint8, device=d)
        self.boxes = torch.empty((n, 4), dtype=torch.float32, device=d)
        self.tight = torch.empty((n, 4), dtype=torch.float32, device=d)
        self.box_img = torch.empty((n,), dtype=torch.int32, device=d)
        self.valid = torch.empty((n,), dtype=torch.int32, device=d)
        self.crops = torch.empty((n, 3, 256, 192), dtype=torch.float32, device=d)
        self.center = torch.empty((n, 2), dtype=torch.float32, device=d)
        self.scale = torch.empty((n, 2), dtype=torch.float32, device=d)
        self.heatmaps = torch.empty((n, J, 64, 48), dtype=torch.float32, device=d)
        self.kp = torch.empty((n, J, 2), dtype=torch.float64, device=d)
        self.score = torch.empty((n, J), dtype=torch.float32, device=d)
        self.argmax = torch.empty((n, J), dtype=torch.int32, device=d)
        self.kp_masked = torch.empty((n, J, 2), dtype=torch.float64, device=d)
        self.pts = torch.empty((n_views, k * J, 2), dtype=torch.float64, device=d)
        self.p3d = torch.empty((k * J, 3), dtype=torch.float64, device=d)
        self.graph = None
        self.det_out = None

    # ------------------------------------------------------------------ the frame's launch sequence
    def _sequence(self):
        s = _lib.stream_ptr(self.dev)
        lib, h = self.lib, self.ctx.handle
        dboxes, dscores, dcount = self.det.forward(self.frames)
        self.det_out = (dboxes, dscores, dcount)
        _lib.check(lib.mq_det_topk_boxes(h, _lib.ptr(dboxes), _lib.ptr(dscores), _lib.ptr(dcount), self.V,
                                         dboxes.shape[1], self.k, self.det_thr, MIN_MARGIN, MAX_MARGIN, DESIRED_AR,
                                         _lib.ptr(self.boxes), _lib.ptr(self.tight), _lib.ptr(self.box_img),
                                         _lib.ptr(self.valid), s), "mq_det_topk_boxes")
        _lib.check(lib.mq_crop_udp(h, _lib.ptr(self.frames), self.H * self.W * 3, self.H, self.W,
                                   _lib.ptr(self.boxes), _lib.ptr(self.box_img), self.n, _lib.ptr(self.crops),
                                   _lib.ptr(self.center), _lib.ptr(self.scale), s), "mq_crop_udp")
        _lib.check(lib.mq_vitpose_forward(self.pose.handle, _lib.ptr(self.crops), self.n, 1 if self.flip else 0,
                                          _lib.ptr(self.heatmaps), s), "mq_vitpose_forward")
        _lib.check(lib.mq_decode_udp(h, _lib.ptr(self.heatmaps), self.n, self.J, 64, 48, _lib.ptr(self.center),
                                     _lib.ptr(self.scale), _lib.ptr(self.kp), _lib.ptr(self.score),
                                     _lib.ptr(self.argmax), None, s), "mq_decode_udp")
        bad = ((self.score < self.tri_thr) | (self.valid == 0).unsqueeze(1)).unsqueeze(-1)
        torch.where(bad, torch.full_like(self.kp, float("nan")), self.kp, out=self.kp_masked)
        self.pts.copy_(self.kp_masked.view(self.V, self.k * self.J, 2))
        _lib.check(lib.mq_triangulate_dlt(h, _lib.ptr(self.cams), self.V, _lib.ptr(self.pts), self.k * self.J, 1,
                                          _lib.ptr(self.p3d), s), "mq_triangulate_dlt")

    def eager(self, frames=None):
        """Run the frame's sequence without the graph (also the warm-up that sizes every workspace)."""
        if frames is not None:
            self.frames.copy_(frames)
        self._sequence()

    def capture(self, warmup=2):
        """Warm up eagerly (workspaces reach their final sizes, tables are cached) and capture the
        sequence into one graph on a side stream."""
        if self.pose.lib.mq_vitpose_set_graph(self.pose.handle, 0) != 0:
            raise _lib.MqError("mq_vitpose_set_graph failed")
        for _ in range(warmup):
            self.eager()
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._sequence()
        torch.cuda.synchronize(self.dev)
        self.graph = g
        return self

    def replay(self):
        assert self.graph is not None, "capture() first"
        self.graph.replay()

    def run(self, frames=None):
        """One frame through the captured graph: (boxes (V k, 4), valid (V k), kp (V k, J, 2) image px,
        score (V k, J), p3d (k J, 3)) as device tensors (the static buffers: copy before the next replay)."""
        if frames is not None:
            self.frames.copy_(frames)
        self.replay()
        return self.boxes, self.valid, self.kp, self.score, self.p3d
