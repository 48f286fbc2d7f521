"""Step-2 cross-view matching on MI355X.

``geometry_affinity_batch`` runs ``geometry_affinity2``
(``src/pipeline/step2_crossviewmatching.py``:373-432) for many frames in one call through
``mq_geometry_affinity``: rays through every keypoint at depth 0 and 1000 (``deproject`` :327-355),
the mean ray-to-ray distance (``calc_dist_btw_lines`` :359-369) over the keypoints both detections
score above ``THR_KP``, the frame's z-score and logistic.  The reference calls it once per frame in
a Python double loop over detection pairs; here a frame is one row of a batch and every pair is one
GPU thread.  ``match_svt_batch`` runs ``matchSVT`` (:130-216) for many keyframes in one launch
(``mq_match_svt``: one workgroup per keyframe, eigen-thresholding by parallel Jacobi in LDS), and
``calc_3dpose_batch`` / ``_combo_rmse`` evaluate ``calc_3dpose`` (:436-461) and ``get_best_comb``'s
reprojection RMSE (:610-646) for every candidate combination of every keyframe in one batch of
undistort / pinv-DLT / projection launches.  No CPU fallback: without a HIP device the calls raise.
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


# ----------------------------------------------------------------------------- matchSVT

def match_svt_batch(W, n_det, cam_of_det, alpha=0.5, _lambda=50.0, mu=64.0, tol=5e-4, maxIter=500, pselect=1,
                    device: int = 0, return_x=False):
    """matchSVT (step2:130-216) for B keyframes at once through ``mq_match_svt``.
    W (B, Nmax, Nmax) affinities, n_det (B,) detections per keyframe, cam_of_det (B, Nmax) camera of
    each detection.  Returns match uint8 (B, Nmax, Nmax), iters (B,) [, X (B, Nmax, Nmax)]."""
    Wn = np.ascontiguousarray(W, dtype=np.float64)
    assert Wn.ndim == 3 and Wn.shape[1] == Wn.shape[2], "W must be (B, Nmax, Nmax)"
    B, Nmax, _ = Wn.shape
    nd = np.ascontiguousarray(n_det, dtype=np.int32).reshape(B)
    cod = np.ascontiguousarray(cam_of_det, dtype=np.int32).reshape(B, Nmax)
    assert np.all((nd >= 0) & (nd <= Nmax)), "n_det out of range"
    dev = torch.device("cuda", device)
    match = torch.zeros((B, Nmax, Nmax), dtype=torch.uint8, device=dev)
    iters = torch.zeros((B,), dtype=torch.int32, device=dev)
    xo = torch.zeros((B, Nmax, Nmax), dtype=torch.float64, device=dev) if return_x else None
    if B * Nmax > 0:
        ctx = _lib.Context.get(device)
        w_d = torch.from_numpy(Wn).to(dev)
        n_d = torch.from_numpy(nd).to(dev)
        c_d = torch.from_numpy(cod).to(dev)
        _lib.check(ctx.lib.mq_match_svt(ctx.handle, _lib.ptr(w_d), _lib.ptr(n_d), _lib.ptr(c_d), B, Nmax,
                                        float(alpha), float(_lambda), float(mu), float(tol), int(maxIter),
                                        int(pselect), _lib.ptr(match), _lib.ptr(xo) if return_x else None,
                                        _lib.ptr(iters), _lib.stream_ptr(dev)), "mq_match_svt")
    out = (match.cpu().numpy(), iters.cpu().numpy())
    return out + (xo.cpu().numpy(),) if return_x else out


# ----------------------------------------------------------------------------- calc_3dpose / reproject

class StepTwoCameras:
    """The two camera views step 2 takes of one ``camparam`` dict (step2:35-75): ``proj`` (K, D, xi,
    rvec, tvec) for cv2.omnidir undistortPoints / projectPoints, and ``pmat`` ([R|t] rows) for
    multicam_toolbox.triangulatePoints and the affinity rays."""

    def __init__(self, camparam, device: int = 0):
        self.camparam = camparam
        cams = []
        for i, cid in enumerate(camparam["camera_id"]):
            cams.append(OmnidirCamera(K=camparam["K"][i], D=np.ravel(camparam["D"][i])[:4], xi=camparam["xi"][i],
                                      rvec=camparam["rvecs"][i], tvec=camparam["tvecs"][i], name=str(cid)))
        self.proj = CameraGroup(cams, device=device)
        self.pmat = CameraGroup([OmnidirCamera.from_projection(camparam["pmat"][i], name=str(cid))
                                 for i, cid in enumerate(camparam["camera_id"])], device=device)
        self.rays = group_from_camparam(camparam, device=device)
        self.n_cam = len(cams)


def calc_3dpose_batch(cams: StepTwoCameras, kp2d, thr_kp: float = THR_KP):
    """calc_3dpose (step2:436-461) for n poses at once: kp2d (n, C, J, 3) raw x, y, score ->
    (n, J, 3).  Undistortion, the pinv DLT and its frame_use mask (finite x, score >= THR_KP)."""
    from .geometry import triangulate_pinv
    kp = np.asarray(kp2d, dtype=np.float64)
    n, C, J, _ = kp.shape
    if n == 0:
        return np.zeros((0, J, 3))
    pts = np.ascontiguousarray(kp[..., :2].transpose(1, 0, 2, 3).reshape(C, n * J, 2))
    und = cams.proj.undistort_points(pts)
    sc = kp[..., 2].transpose(0, 2, 1).reshape(n * J, C)
    x = kp[..., 0].transpose(0, 2, 1).reshape(n * J, C)
    use = ~(np.isnan(x) | (sc < thr_kp))
    return triangulate_pinv(cams.pmat, und, use).reshape(n, J, 3)


def _combo_rmse(cams: StepTwoCameras, kp2d, present, thr_kp: float = THR_KP):
    """get_best_comb's score (step2:621-642) for n combos: kp2d (n, C, J, 3), present (n, C) bool.
    RMSE over every (camera, keypoint, axis) with score > THR_KP of the reprojected DLT pose; NaN when
    nothing qualifies or a qualifying keypoint has no 3D point (np.argmin then picks it, as there)."""
    p3d = calc_3dpose_batch(cams, kp2d, thr_kp)
    n, C, J, _ = kp2d.shape
    rp = cams.proj.project(p3d.reshape(-1, 3)).reshape(C, n, J, 2).transpose(1, 0, 2, 3)
    ok = present[:, :, None] & (kp2d[..., 2] > thr_kp)
    d2 = np.where(ok[..., None], (kp2d[..., :2] - rp) ** 2, 0.0)
    cnt = ok.sum(axis=(1, 2)) * 2
    with np.errstate(invalid="ignore", divide="ignore"):
        return np.sqrt(d2.sum(axis=(1, 2, 3)) / cnt)
