"""ORACLE (test infrastructure only): restatement of the anipose Viterbi 2D filter.

Follows ``/root/reference/src/third_party/anipose/filter_pose.py``:26-46 (remove_dups),
48-120 (viterbi_path), 151-186 (filter_pose_viterbi, run serially here instead of a
spawn pool -- results are per joint and independent), 332-343 (wrap_points); driven
as ``src/pipeline/step4_aniposefiltering.py``:140-170 drives it.  scipy's
``norm.logcdf``, ``logsumexp`` and ``cdist`` are called exactly as the reference does.
"""
from __future__ import annotations

import numpy as np
from scipy import stats
from scipy.spatial import cKDTree
from scipy.spatial.distance import cdist
from scipy.special import logsumexp


def remove_dups(pts, thres=7):
    """filter_pose.py:26-46 (NaN/Inf-safe variant of the reference)."""
    tindex = np.repeat(np.arange(pts.shape[0])[:, None], pts.shape[1], axis=1) * 100
    pts_ix = np.dstack([pts, tindex])
    pts_ix = np.where(np.isfinite(pts_ix), pts_ix, 1e9)
    tree = cKDTree(pts_ix.reshape(-1, 3))
    shape = (pts.shape[0], pts.shape[1])
    pairs = tree.query_pairs(thres)
    indices = [b for a, b in pairs]
    if len(pairs) == 0:
        return pts
    i0, i1 = np.unravel_index(indices, shape)
    pts_out = np.copy(pts)
    pts_out[i0, i1] = np.nan
    return pts_out


def viterbi_path(points, scores, n_back=3, thres_dist=30, return_indices=False):
    """filter_pose.py:48-120."""
    n_frames = points.shape[0]
    points_nans = remove_dups(points, thres=5)
    num_points = np.sum(~np.isnan(points_nans[:, :, 0]), axis=1)
    num_max = np.max(num_points)
    particles = np.zeros((n_frames, num_max * n_back + 1, 3), dtype='float64')
    valid = np.zeros(n_frames, dtype='int64')
    for i in range(n_frames):
        s = 0
        for j in range(n_back):
            if i - j < 0:
                break
            ixs = np.where(~np.isnan(points_nans[i - j, :, 0]))[0]
            n_valid = len(ixs)
            particles[i, s:s + n_valid, :2] = points[i - j, ixs]
            particles[i, s:s + n_valid, 2] = scores[i - j, ixs] * np.power(2.0, -j)
            s += n_valid
        if s == 0:
            particles[i, 0] = [-1, -1, 0.001]
            s = 1
        valid[i] = s
    n_particles = np.max(valid)
    T_logprob = np.full((n_frames, n_particles), -np.inf)
    T_back = np.zeros((n_frames, n_particles), dtype='int64')
    T_logprob[0, :valid[0]] = np.log(particles[0, :valid[0], 2])
    T_back[0, :] = -1
    for i in range(1, n_frames):
        va, vb = valid[i - 1], valid[i]
        pa = particles[i - 1, :va, :2]
        pb = particles[i, :vb, :2]
        dists = cdist(pa, pb)
        cdf_high = stats.norm.logcdf(dists + 2, scale=thres_dist)
        cdf_low = stats.norm.logcdf(dists - 2, scale=thres_dist)
        cdfs = np.array([cdf_high, cdf_low])
        P_trans = logsumexp(cdfs.T, b=[1, -1], axis=2)
        P_trans[P_trans < -100] = -100
        P_trans[pb[:, 0] == -1, :] = np.log(0.001)
        P_trans[:, pa[:, 0] == -1] = np.log(0.001)
        pflat = particles[i, :vb, 2]
        possible = T_logprob[i - 1, :va] + P_trans
        T_logprob[i, :vb] = np.max(possible, axis=1) + np.log(pflat)
        T_back[i, :vb] = np.argmax(possible, axis=1)
    out = np.zeros(n_frames, dtype='int')
    out[-1] = np.argmax(T_logprob[-1])
    for i in range(n_frames - 1, 0, -1):
        out[i - 1] = T_back[i, out[i]]
    trace = np.array([particles[i, out[i]] for i in range(n_frames)])
    if return_indices:
        return trace[:, :2], trace[:, 2], out
    return trace[:, :2], trace[:, 2]


def filter_pose_viterbi(config, all_points, bodyparts=()):
    """filter_pose.py:151-186 (serial).  NOTE: mutates ``all_points`` like the reference."""
    n_frames, n_joints, n_possible, _ = all_points.shape
    points_full = all_points[:, :, :, :2]
    scores_full = all_points[:, :, :, 2]
    points_full[scores_full < config['filter']['score_threshold']] = np.nan
    points = np.full((n_frames, n_joints, 2), np.nan, dtype='float64')
    scores = np.empty((n_frames, n_joints), dtype='float64')
    for jix in range(n_joints):
        pts_new, scs_new = viterbi_path(points_full[:, jix, :], scores_full[:, jix],
                                        config['filter']['n_back'],
                                        config['filter']['offset_threshold'])
        points[:, jix] = pts_new
        scores[:, jix] = scs_new
    return points, scores


def wrap_points(points, scores):
    """filter_pose.py:332-343."""
    if len(points.shape) == 3:
        points = points[:, :, None]
        scores = scores[:, :, None]
    n_frames, n_joints, n_possible, _ = points.shape
    all_points = np.full((n_frames, n_joints, n_possible, 3), np.nan, dtype='float64')
    all_points[:, :, :, :2] = points
    all_points[:, :, :, 2] = scores
    return all_points


STEP4_FILTER_CONFIG = {"filter": {"score_threshold": 0.3, "n_back": 3,
                                  "offset_threshold": 25, "multiprocessing": False}}


def step4_filter(kp2d):
    """step4_aniposefiltering.py:142-167: (A,F,C,J,3) -> kp2d_f (F,J,A,3,C)."""
    kp2d = np.array(kp2d, dtype=np.float64, copy=True)
    n_animal, n_frame, n_cam = kp2d.shape[:3]
    kp2d = kp2d.transpose((1, 3, 0, 4, 2))
    kp2d_f = np.zeros(kp2d.shape, dtype=float)
    for a in range(n_animal):
        for c in range(n_cam):
            points = np.expand_dims(kp2d[:, :, a, :, c], 2)
            pf, sf = filter_pose_viterbi(STEP4_FILTER_CONFIG, points, [])
            pf = wrap_points(pf, sf)
            kp2d_f[:, :, a, :, c] = np.squeeze(pf)
    return kp2d_f


def viterbi_paths_batched(points, scores, n_back=3, thres_dist=30):
    """``viterbi_path`` (filter_pose.py:48-120) for N independent single-candidate chains at once.

    points (N, F, 2) with NaN for missing (already score-thresholded), scores (N, F).  With one
    candidate per frame ``remove_dups`` never pairs two points (candidates of different frames sit
    >= 100 apart in its time coordinate), so it is the identity here.  Every chain runs the loop
    version's arithmetic on the same values: the same particles (frames i, i-1, ..., score * 2^-j,
    or the (-1, -1, 0.001) placeholder), the same scipy ``norm.logcdf`` / ``logsumexp`` calls on the
    same distances, the same clamps, and first-index max / argmax rules; padding slots of chains
    with fewer particles are masked to -inf so they never win.  tests/test_oracle_kat.py checks it
    against the loop version (``step4_filter``) value for value."""
    N, F, _ = points.shape
    K = n_back
    good = ~np.isnan(points[:, :, 0])
    part = np.zeros((N, F, K, 3))
    valid = np.zeros((N, F), dtype=np.int64)
    for i in range(F):
        s = np.zeros(N, dtype=np.int64)
        for j in range(n_back):
            if i - j < 0:
                break
            g = good[:, i - j]
            idx = np.flatnonzero(g)
            part[idx, i, s[idx], :2] = points[idx, i - j]
            part[idx, i, s[idx], 2] = scores[idx, i - j] * np.power(2.0, -j)
            s += g
        none = s == 0
        part[none, i, 0] = [-1, -1, 0.001]
        s[none] = 1
        valid[:, i] = s
    slot = np.arange(K)
    T = np.full((N, F, K), -np.inf)
    back = np.zeros((N, F, K), dtype=np.int64)
    ok0 = slot[None, :] < valid[:, 0:1]
    with np.errstate(divide="ignore", invalid="ignore"):
        T[:, 0] = np.where(ok0, np.log(np.where(ok0, part[:, 0, :, 2], 1.0)), -np.inf)
    for i in range(1, F):
        pa = part[:, i - 1, :, :2]                                   # (N, K, 2)
        pb = part[:, i, :, :2]
        diff = pb[:, :, None, :] - pa[:, None, :, :]                 # (N, Kb, Ka, 2): cdist(pa, pb).T
        d = np.sqrt(diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1])
        cdf_high = stats.norm.logcdf(d + 2, scale=thres_dist)
        cdf_low = stats.norm.logcdf(d - 2, scale=thres_dist)
        with np.errstate(invalid="ignore", divide="ignore"):
            P = logsumexp(np.stack([cdf_high, cdf_low], axis=-1), b=[1, -1], axis=-1)
        P[P < -100] = -100
        P = np.where((pb[:, :, 0] == -1)[:, :, None], np.log(0.001), P)
        P = np.where((pa[:, :, 0] == -1)[:, None, :], np.log(0.001), P)
        va = slot[None, :] < valid[:, i - 1:i]                       # (N, Ka)
        vb = slot[None, :] < valid[:, i:i + 1]                       # (N, Kb)
        possible = np.where(va[:, None, :], T[:, i - 1][:, None, :] + P, -np.inf)
        m = np.max(possible, axis=2)
        with np.errstate(divide="ignore", invalid="ignore"):
            T[:, i] = np.where(vb, m + np.log(np.where(vb, part[:, i, :, 2], 1.0)), -np.inf)
        back[:, i] = np.where(vb, np.argmax(possible, axis=2), 0)
    out = np.zeros((N, F), dtype=np.int64)
    out[:, -1] = np.argmax(T[:, -1], axis=1)
    for i in range(F - 1, 0, -1):
        out[:, i - 1] = back[np.arange(N), i, out[:, i]]
    trace = part[np.arange(N)[:, None], np.arange(F)[None, :], out]  # (N, F, 3)
    return trace[..., :2], trace[..., 2]


def step4_filter_batched(kp2d, config=STEP4_FILTER_CONFIG):
    """``step4_filter`` with every (animal, camera, joint) chain in one batched Viterbi: the
    clip-sized (config 4: 544 chains x 300 frames) form used by the parity tests."""
    kp = np.array(kp2d, dtype=np.float64, copy=True)                 # (A, F, C, J, 3)
    A, F, C, J, _ = kp.shape
    ch = kp.transpose(0, 2, 3, 1, 4).reshape(-1, F, 3)              # (A*C*J, F, 3)
    pts = ch[..., :2].copy()
    sc = ch[..., 2].copy()
    pts[sc < config['filter']['score_threshold']] = np.nan
    p, s = viterbi_paths_batched(pts, sc, config['filter']['n_back'], config['filter']['offset_threshold'])
    out = np.concatenate([p, s[..., None]], axis=-1).reshape(A, C, J, F, 3)
    return np.ascontiguousarray(out.transpose(3, 2, 0, 4, 1))       # (F, J, A, 3, C)
