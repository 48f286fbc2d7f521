"""Step-2 cross-view geometry affinity on MI355X (first piece).

``geometry_affinity_batch`` runs ``geometry_affinity2``
(``src/pipeline/step2_crossviewmatching.py``:373-432) for many frames in one call through
``mq_geometry_affinity``: rays through every keypoint at depth 0 and 1000 (``deproject`` :327-355),
the mean ray-to-ray distance (``calc_dist_btw_lines`` :359-369) over the keypoints both detections
score above ``THR_KP``, the frame's z-score and logistic.  The reference calls it once per frame in
a Python double loop over detection pairs; here a frame is one row of a batch and every pair is one
GPU thread.  No CPU fallback: without a HIP device the call raises.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .geometry import CameraGroup, OmnidirCamera

THR_KP = 0.1  # step2_crossviewmatching.py:21


def group_from_camparam(camparam, device: int = 0) -> CameraGroup:
    """Cameras with R from ``pmat[:, :3]`` and t from ``tvecs`` (what ``deproject`` reads)."""
    cams = []
    for i, cid in enumerate(camparam["camera_id"]):
        P = np.asarray(camparam["pmat"][i], dtype=np.float64).copy()
        P[:, 3] = np.asarray(camparam["tvecs"][i], dtype=np.float64).ravel()
        cams.append(OmnidirCamera.from_projection(P, name=str(cid)))
    return CameraGroup(cams, device=device)


def geometry_affinity_batch(cams: CameraGroup, points, cam_of_det, thr_kp: float = THR_KP):
    """points (B, M, J, 3) undistorted x, y, score; cam_of_det (B, M) int (-1 = padding).
    Returns affinity (B, M, M) float64 (0 on padding rows and columns)."""
    pts = np.ascontiguousarray(points, dtype=np.float64)
    cod = np.ascontiguousarray(cam_of_det, dtype=np.int32)
    assert pts.ndim == 4 and pts.shape[-1] == 3, "points must be (B, M, J, 3)"
    B, M, J, _ = pts.shape
    assert cod.shape == (B, M), "cam_of_det must be (B, M)"
    assert np.all(cod < len(cams.cameras)), "camera index out of range"
    dev = cams._dev()
    out = torch.empty((B, M, M), dtype=torch.float64, device=dev)
    if B * M == 0:
        return out.cpu().numpy()
    ctx = cams._ctx()
    p_d = cams._to_dev(pts)
    c_d = torch.from_numpy(cod).to(dev)
    _lib.check(ctx.lib.mq_geometry_affinity(ctx.handle, _lib.ptr(cams.cams_tensor()), len(cams.cameras), _lib.ptr(p_d),
                                            _lib.ptr(c_d), B, M, J, float(thr_kp), _lib.ptr(out),
                                            _lib.stream_ptr(dev)), "mq_geometry_affinity")
    return out.cpu().numpy()


def dimgroup_to_cams(dimGroup, M):
    """Camera index of each detection: np.searchsorted(dimGroup, i, side='right') - 1 (step2:395-397)."""
    return (np.searchsorted(np.asarray(dimGroup), np.arange(M), side="right") - 1).astype(np.int32)
