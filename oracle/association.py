"""ORACLE (test infrastructure only): float64 restatement of the step-2 cross-view geometry affinity.

Follows ``/root/reference/src/pipeline/step2_crossviewmatching.py``:
* ``deproject`` :327-355 -- undistorted (x, y) at depth d -> world point ``inv(R) @ (d [x, y, 1] - t)``,
* ``calc_dist_btw_lines`` :359-369 -- distance between two rays given as (near, far) point pairs,
* ``geometry_affinity2`` :373-432 -- per detection pair on different cameras, the mean ray distance
  over keypoints scored above ``THR_KP`` (:21, 0.1) by both, when at least 3 qualify (else 2*Dth2,
  Dth2 = 150); diagonal 0; z-score over the entries below 2*Dth2, logistic(-5 z), 0 where > Dth2.

Camera inputs are the reference ``camparam`` dict entries it uses: ``pmat`` (3x4 [R|t]) and ``tvecs``.
Never imported by the product path.
"""
from __future__ import annotations

import numpy as np

THR_KP = 0.1
DTH2 = 150.0


def deproject(pmat, tvec, p2d, depth):
    """step2:327-355 (loop over points kept as a matrix product of the same terms)."""
    p2d = p2d if p2d.ndim == 2 else p2d[np.newaxis, :]
    pts3d = np.hstack([p2d, np.ones((p2d.shape[0], 1), float)]) * depth
    R_inv = np.linalg.inv(np.asarray(pmat, dtype=np.float64)[:, :3])
    t = np.asarray(tvec, dtype=np.float64).ravel()
    return np.vstack([R_inv @ (p - t) for p in pts3d])


def calc_dist_btw_lines(v1, v2):
    """step2:359-369."""
    p1, p2 = v1[:3], v2[:3]
    d1 = (v1[3:6] - p1) / np.linalg.norm(v1[3:6] - p1)
    d2 = (v2[3:6] - p2) / np.linalg.norm(v2[3:6] - p2)
    c = np.cross(d1, d2)
    return abs(np.dot(p2 - p1, c)) / np.linalg.norm(c)


def geometry_affinity2(points_set, dimGroup, pmats, tvecs, thr_kp=THR_KP):
    """step2:373-432.  points_set (M, J, 3): undistorted x, y and score; dimGroup (n_cam + 1,)."""
    M, n_kp, _ = points_set.shape
    dist_mat = np.full((M, M), DTH2 * 2, dtype=np.float64)
    np.fill_diagonal(dist_mat, 0)
    cam_for_det = [np.searchsorted(dimGroup, i, side="right") - 1 for i in range(M)]
    V = []
    for i in range(M):
        c = cam_for_det[i]
        xy = points_set[i, :, :2]
        V.append(np.hstack([deproject(pmats[c], tvecs[c], xy, 0.0), deproject(pmats[c], tvecs[c], xy, 1000.0)]))
    S = [points_set[i, :, 2] for i in range(M)]
    for i in range(M):
        for j in range(i + 1, M):
            if cam_for_det[i] == cam_for_det[j]:
                continue
            dists = [calc_dist_btw_lines(V[i][k], V[j][k]) for k in range(n_kp)
                     if S[i][k] > thr_kp and S[j][k] > thr_kp]
            if len(dists) >= 3:
                dist_mat[i, j] = dist_mat[j, i] = np.mean(dists)
    valid = dist_mat < DTH2 * 2
    dm_mean = dist_mat[valid].mean()
    dm_std = dist_mat[valid].std()
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        affinity = -(dist_mat - dm_mean) / dm_std
        affinity = 1 / (1 + np.exp(-5 * affinity))
    affinity[dist_mat > DTH2] = 0
    return affinity
