"""multicam_toolbox point functions used by steps 2-3 (row a17), backed by libmq_hip.

``undistortPoints(config_path, pos_2d, omnidir, camparam)`` and
``triangulatePoints(config_path, pos_2d_undist, frame_use, use_optim_extrin, camparam)``
keep the reference signatures (multicam_toolbox.py:393-486).  The ``camparam``
dict path is supported (``camera_id``, ``K``, ``xi``, ``D`` and ``pmat`` = [R|t]
per camera); the h5 path needs h5py, which this image lacks, and raises.
Only omnidir undistortion is on the path (step2/3 call it with omnidir=True).
"""
import numpy as np

from mqhip.geometry import CameraGroup, OmnidirCamera, triangulate_pinv


def _group_from_camparam(camparam, with_extrinsics=False, device: int = 0):
    cams = []
    for i, cid in enumerate(camparam['camera_id']):
        rvec = np.zeros(3)
        tvec = np.zeros(3)
        cams.append(OmnidirCamera(K=np.asarray(camparam['K'][i], dtype=np.float64),
                                  xi=float(np.ravel(camparam['xi'][i])[0]),
                                  D=np.asarray(camparam['D'][i], dtype=np.float64).ravel(),
                                  rvec=rvec, tvec=tvec, name=str(cid), size=[2048, 1536]))
    return CameraGroup(cams, device=device)


def _require_camparam(camparam):
    if camparam is None:
        raise NotImplementedError("the h5 calibration path needs h5py (absent); pass camparam")


def undistortPoints(config_path, pos_2d, omnidir=False, camparam=None, device: int = 0):
    """list/array of per-camera (N,2) pixels -> list of per-camera (N,2) normalized points."""
    _require_camparam(camparam)
    if not omnidir:
        raise NotImplementedError("pinhole cv2.undistortPoints is not on the omnidir pipeline's path")
    g = _group_from_camparam(camparam, device=device)
    pts = np.stack([np.asarray(p, dtype=np.float64).reshape(-1, 2) for p in pos_2d])
    und = g.undistort_points(pts)
    return [np.squeeze(u) for u in und]


def triangulatePoints(config_path, pos_2d_undist, frame_use, use_optim_extrin=True, camparam=None,
                      device: int = 0):
    """(C, N, 2) undistorted + frame_use (N, C) -> (N, 3), NaN where < 2 cameras are used."""
    _require_camparam(camparam)
    C = len(camparam['camera_id'])
    cams = []
    for i, cid in enumerate(camparam['camera_id']):
        P = np.asarray(camparam['pmat'][i], dtype=np.float64)
        cams.append(OmnidirCamera.from_projection(P, name=str(cid)))
    g = CameraGroup(cams, device=device)
    und = np.stack([np.asarray(u, dtype=np.float64).reshape(-1, 2) for u in pos_2d_undist[:C]])
    return triangulate_pinv(g, und, np.asarray(frame_use, dtype=bool))
