"""Step 2 (cross-view matching) -- the geometry affinity, on MI355X.

Mirrors ``geometry_affinity2(points_set, dimGroup, config_path, camparam=None)`` of
``src/pipeline/step2_crossviewmatching.py``:373-432 (same arguments, same M x M result), backed by
``mq_geometry_affinity``.  ``camparam`` is the reference's dict (``camera_id``, ``pmat`` = [R|t],
``tvecs``); the h5 calibration path needs h5py, which this image lacks, and raises.  Matching
(``matchSVT``), ``get_best_comb`` and the rest of step 2 are not on the hot path.
"""
from __future__ import annotations

import numpy as np

from mqhip.association import THR_KP, dimgroup_to_cams, geometry_affinity_batch, group_from_camparam


def geometry_affinity2(points_set, dimGroup, config_path, camparam=None, device: int = 0):
    """points_set (M, N_kp, 3) undistorted keypoints + scores; dimGroup (n_cam + 1,) cumulative counts."""
    if camparam is None:
        raise NotImplementedError("the h5 calibration path needs h5py (absent); pass camparam")
    points_set = np.asarray(points_set, dtype=np.float64)
    M = points_set.shape[0]
    g = group_from_camparam(camparam, device=device)
    aff = geometry_affinity_batch(g, points_set[None], dimgroup_to_cams(dimGroup, M)[None], thr_kp=THR_KP)
    return aff[0]
