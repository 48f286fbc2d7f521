"""ORACLE (test infrastructure only): float64 restatement of the step-2 cross-view geometry affinity.

Follows ``/root/reference/src/pipeline/step2_crossviewmatching.py``:
* ``deproject`` :327-355 -- undistorted (x, y) at depth d -> world point ``inv(R) @ (d [x, y, 1] - t)``,
* ``calc_dist_btw_lines`` :359-369 -- distance between two rays given as (near, far) point pairs,
* ``geometry_affinity2`` :373-432 -- per detection pair on different cameras, the mean ray distance
  over keypoints scored above ``THR_KP`` (:21, 0.1) by both, when at least 3 qualify (else 2*Dth2,
  Dth2 = 150); diagonal 0; z-score over the entries below 2*Dth2, logistic(-5 z), 0 where > Dth2.

Camera inputs are the reference ``camparam`` dict entries it uses: ``pmat`` (3x4 [R|t]) and ``tvecs``
(plus ``K``, ``D``, ``xi``, ``rvecs`` for the undistortion / reprojection of ``calc_3dpose``).

The rest of step 2 is restated below it: ``matchSVT`` :130-216 (with ``proj2pav`` / ``myproj2dpam``
:79-126), ``calc_3dpose`` :436-461, ``reproject`` :465-489, ``MultiEstimator.predict_data``
:502-713 (incl. ``get_best_comb`` :610-646), and the 2D-tracklet ID voting
``set_id_for_each_frame_of_2dtracklets`` :717-800 / ``get_id_of_2dtrack`` :802-850.
Never imported by the product path.
"""
from __future__ import annotations

import itertools

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


# ----------------------------------------------------------------------------- matching (matchSVT)

ALPHA_ID = 0.2   # step2:22
CID_THR = 0.8    # step2:23
P_THR_2DT = 0.8  # step2:24
MODEL_CFG = {"joint_num": 17, "spectral": True, "alpha_SVT": 0.5, "lambda_SVT": 50,
             "dual_stochastic_SVT": False}  # step2:25-31


def proj2pav(y):
    """step2:79-94 -- Euclidean projection onto the simplex (sort + cumulative sum)."""
    y = y.copy()
    y[y < 0] = 0
    if y.sum() < 1:
        return y
    u = np.sort(y)[::-1]
    sv = np.cumsum(u)
    rho = np.nonzero(u > (sv - 1) / np.arange(1, len(u) + 1))[0][-1]
    theta = max(0, (sv[rho] - 1) / (rho + 1))
    return np.maximum(y - theta, 0)


def myproj2dpam(Y, tol=1e-4):
    """step2:97-126 -- alternating row / column simplex projections (at most 10 rounds)."""
    X = Y.copy()
    I2 = np.zeros_like(X)
    for _ in range(10):
        Z = X + I2
        X1 = np.stack([proj2pav(Z[i, :]) for i in range(Z.shape[0])])
        I1 = X1 - Z
        Z = X + I1
        X2 = np.stack([proj2pav(Z[:, j]) for j in range(Z.shape[1])], axis=1)
        I2 = X2 - Z
        if np.abs(X2 - X).sum() / X.size < tol:
            break
        X = X2
    return X


def matchSVT(S, dimGroup, alpha=0.1, pselect=1, tol=5e-4, maxIter=500, _lambda=50, mu=64,
             dual_stochastic_SVT=True, return_info=False):
    """step2:130-216.  Returns the uint8 match matrix (and, with return_info, the final X and the
    last iteration index)."""
    S = np.array(S, dtype=np.float64)
    N = S.shape[0]
    S[np.arange(N), np.arange(N)] = 0
    S = (S + S.T) / 2
    X = S.copy()
    Y = np.zeros_like(S)
    W = alpha - S
    it = 0
    for it in range(maxIter):
        X0 = X.copy()
        U, s, Vh = np.linalg.svd((Y / mu) + X, full_matrices=False)
        Q = U @ np.diag(np.maximum(s - (_lambda / mu), 0)) @ Vh
        X = Q - (W + Y) / mu
        for g in range(len(dimGroup) - 1):
            i0, i1 = int(dimGroup[g]), int(dimGroup[g + 1])
            X[i0:i1, i0:i1] = 0
        if pselect == 1:
            X[np.arange(N), np.arange(N)] = 1
        X = np.clip(X, 0, 1)
        if dual_stochastic_SVT:
            for gi in range(len(dimGroup) - 1):
                r0, r1 = int(dimGroup[gi]), int(dimGroup[gi + 1])
                for gj in range(len(dimGroup) - 1):
                    c0, c1 = int(dimGroup[gj]), int(dimGroup[gj + 1])
                    if r1 > r0 and c1 > c0:
                        X[r0:r1, c0:c1] = myproj2dpam(X[r0:r1, c0:c1], tol=1e-2)
        X = (X + X.T) / 2
        Y = Y + mu * (X - Q)
        pRes = np.linalg.norm(X - Q) / N
        dRes = mu * np.linalg.norm(X - X0) / N
        if pRes < tol and dRes < tol:
            break
        if pRes > 10 * dRes:
            mu *= 2
        elif dRes > 10 * pRes:
            mu /= 2
    X = (X + X.T) / 2
    match = (X > 0.5).astype(np.uint8)
    if return_info:
        return match, X, it
    return match


# ----------------------------------------------------------------------------- 3D pose helpers

def camparam_cams(camparam):
    """Oracle cameras (K, D, xi, rvec, tvec) of a reference ``camparam`` dict (step2:35-75)."""
    from .geometry import OmnidirCam
    return [OmnidirCam({"name": str(cid), "K": camparam["K"][i], "D": camparam["D"][i], "xi": camparam["xi"][i],
                        "rvec": camparam["rvecs"][i], "tvec": camparam["tvecs"][i]})
            for i, cid in enumerate(camparam["camera_id"])]


def calc_3dpose(kp_2d, camparam, thr_kp=THR_KP):
    """step2:436-461 -- omnidir undistortion per camera, frame_use = finite x and score >= THR_KP,
    multicam_toolbox.triangulatePoints (pinv DLT on pmat)."""
    from .geometry import mct_triangulate_points
    cams = camparam_cams(camparam)
    n_cam, n_kp, _ = kp_2d.shape
    pos2d = [kp_2d[i, :, :2] for i in range(n_cam)]
    und = [cams[i].undistort_points(pos2d[i] + 0.0) for i in range(n_cam)]
    frame_use = np.ones((n_kp, n_cam), dtype=bool)
    for k in range(n_kp):
        for c in range(n_cam):
            if np.isnan(pos2d[c][k, 0]) or kp_2d[c, k, 2] < thr_kp:
                frame_use[k, c] = False
    return mct_triangulate_points(und, frame_use, camparam["pmat"])


def reproject(i_cam, p3d, camparam):
    """step2:465-489 -- cv2.omnidir.projectPoints through camera i_cam."""
    return camparam_cams(camparam)[i_cam].project(np.asarray(p3d, dtype=np.float64).reshape(-1, 3))


def predict_data(info_dict, camparam, thr_kp=THR_KP):
    """MultiEstimator.predict_data (step2:502-713) without the drawing branch.  The spectral
    initialisation (:577-586) only fills X0, which matchSVT never receives; it is skipped (its
    np.random.rand call only advances numpy's global generator).  Returns (matched_list, P3d_list,
    bcomb_list)."""
    n_cam = len(info_dict)
    dimGroup = [0]
    for c in range(n_cam):
        dimGroup.append(dimGroup[-1] + len(info_dict[c][0]))
    dimGroup = np.array(dimGroup)
    info_list = []
    for c in range(n_cam):
        info_list.extend(info_dict[c][0])
    if not info_list:
        return [], [], []
    M = len(info_list)
    n_kp = MODEL_CFG["joint_num"]
    pose2d = np.array([d["pose2d"] for d in info_list]).reshape(M, n_kp, 2)
    pose_score = np.array([d["pose2d_raw"] for d in info_list]).reshape(M, n_kp, 3)[..., 2]
    kp_mat = np.concatenate([pose2d, pose_score[..., None]], axis=2)
    sub2cam = np.zeros(M, dtype=int)
    for g in range(len(dimGroup) - 1):
        sub2cam[dimGroup[g]:dimGroup[g + 1]] = g
    cid_list = [d["cid"] for d in info_list]
    geo = geometry_affinity2(kp_mat.copy(), dimGroup, camparam["pmat"], camparam["tvecs"], thr_kp=thr_kp)
    cid_mat = np.zeros_like(geo)
    for i in range(M):
        for j in range(M):
            if sub2cam[i] != sub2cam[j] and cid_list[i] >= 0 and cid_list[i] == cid_list[j]:
                cid_mat[i, j] = 1.0
    W = ALPHA_ID * cid_mat + (1 - ALPHA_ID) * geo
    W *= (geo > 0)
    W = np.nan_to_num(W)
    match = matchSVT(W, dimGroup, alpha=MODEL_CFG["alpha_SVT"], _lambda=MODEL_CFG["lambda_SVT"],
                     dual_stochastic_SVT=MODEL_CFG["dual_stochastic_SVT"])
    cols = np.nonzero(match.sum(axis=0) > 1.9)[0]
    bin_match = match[:, cols] > 0.9
    matched = [[] for _ in range(bin_match.shape[1])]
    for sub, row in enumerate(bin_match):
        if row.sum() != 0:
            matched[row.argmax()].append(sub)
    matched = [np.array(m) for m in matched]

    def get_best_comb(person):
        person = np.asarray(person, dtype=int)
        cams_of = sub2cam[person]
        groups = [person[np.where(cams_of == c)].tolist() or [None] for c in range(n_cam)]
        combos = list(itertools.product(*groups))
        if len(combos) == 1:
            return person
        errors = []
        for combo in combos:
            kp2d = np.zeros((n_cam, n_kp, 3))
            for c, sub in enumerate(combo):
                if sub is not None:
                    kp2d[c] = info_list[sub]["pose2d_raw"]
            p3d = calc_3dpose(kp2d, camparam, thr_kp)
            derrs = []
            for c, sub in enumerate(combo):
                if sub is None:
                    continue
                rp = reproject(c, p3d, camparam)
                raw = info_list[sub]["pose2d_raw"]
                ok = raw[:, 2] > thr_kp
                derrs.append(raw[:, :2][ok] - rp[ok])
            if derrs:
                d = np.vstack(derrs)
                with np.errstate(invalid="ignore"):
                    errors.append(np.sqrt((d ** 2).mean()) if d.size else np.nan)
            else:
                errors.append(np.inf)
        best = combos[int(np.argmin(errors))]
        return np.array([i for i in best if i is not None], dtype=int)

    refined = []
    for person in matched:
        best = get_best_comb(person)
        refined.append(best)
        leftover = set(person.tolist()) - set(best.tolist())
        if len(leftover) > 1:
            refined.append(get_best_comb(np.array(list(leftover), dtype=int)))
    P3d, matched2, bcombs = [], [], []
    for person in refined:
        if person.shape[0] < 2:
            continue
        kp2d = np.zeros((n_cam, n_kp, 3))
        for sub in person:
            kp2d[sub2cam[sub]] = info_list[sub]["pose2d_raw"]
        P3d.append(calc_3dpose(kp2d, camparam, thr_kp))
        bc = -np.ones(n_cam, dtype=int)
        for sub in person:
            bc[sub2cam[sub]] = info_list[sub]["bbox_id"][1]
        matched2.append(person)
        bcombs.append(bc)
    return matched2, P3d, bcombs


# ----------------------------------------------------------------------------- 2D tracklet IDs

VALID_IDS = [0, 2, 3, 5]  # step2:734


def set_id_for_each_frame_of_2dtracklets(Cid, n_frame, wsize):
    """step2:717-800 -- per tracklet: windowed majority labels (columns of VALID_IDS), then one
    label, a global label, or midpoint splits between consecutive labels."""
    out = {k: v.copy() for k, v in Cid.items()}
    for k, arr in Cid.items():
        valid = np.argwhere(arr >= -1)
        start_f, end_f = valid.min(), valid.max()
        onehot = np.zeros((n_frame, len(VALID_IDS)), int)
        for f in range(n_frame):
            if arr[f] in VALID_IDS:
                onehot[f, VALID_IDS.index(arr[f])] = 1
        labels = np.full(n_frame, -1, dtype=int)
        h = wsize // 2
        for f in range(max(start_f, h), min(end_f, n_frame - h)):
            cnts = onehot[f - h:f + h].sum(axis=0)
            if cnts.sum() > 0 and cnts.max() / cnts.sum() > P_THR_2DT and cnts.max() >= 12:
                labels[f] = np.argmax(cnts)
        uniq = np.unique(labels[start_f:end_f + 1])
        uniq = uniq[uniq >= 0]
        if uniq.size == 0:
            g = onehot.sum(axis=0)
            if g.sum() > 0 and g.max() / g.sum() > P_THR_2DT and g.max() >= 12:
                labels[:] = np.argmax(g)
        elif uniq.size == 1:
            labels[:] = uniq[0]
        else:
            prev_id, prev_frame = -1, 0
            for f in range(n_frame):
                cur = labels[f]
                if cur >= 0 and cur != prev_id:
                    if prev_id == -1:
                        labels[:f] = cur
                    else:
                        b0, b1 = max(1, prev_frame - h), f
                        ip = np.argwhere(onehot[:, prev_id] > 0).flatten()
                        ip = ip[(ip >= b0) & (ip <= b1)]
                        i_prev = ip.max() if ip.size > 0 else prev_frame
                        c0, c1 = prev_frame, min(f + h, n_frame)
                        ic = np.argwhere(onehot[:, cur] > 0).flatten()
                        ic = ic[(ic >= c0) & (ic <= c1)]
                        i_curr = ic.min() if ic.size > 0 else f
                        mid = (i_prev + i_curr) // 2
                        labels[prev_frame:mid] = prev_id
                        labels[mid:f] = cur
                    prev_id, prev_frame = cur, f
            if prev_id >= 0:
                labels[prev_frame:] = prev_id
        out[k] = labels
    return out


def get_id_of_2dtrack(data_per_cam, wsize=24 * 5):
    """step2:802-850 on already-loaded alldata rows (data_per_cam[cam][frame] = rows); the rows'
    id scores are zeroed in place for duplicated confident IDs, as in the reference."""
    n_cam = len(data_per_cam)
    n_frame = len(data_per_cam[0])
    for c in range(n_cam):
        for f in range(n_frame):
            dets = data_per_cam[c][f]
            cnts = np.zeros(20, int)
            for det in dets:
                if det[6] in {0, 2, 3, 5} and det[7] > CID_THR:
                    cnts[det[6]] += 1
            for dup in np.where(cnts > 1)[0]:
                for det in dets:
                    if det[6] == int(dup):
                        det[7] = 0.0
    out = []
    for c in range(n_cam):
        ids = {}
        for f in range(n_frame):
            for det in data_per_cam[c][f]:
                if det[0] not in ids:
                    ids[det[0]] = -2 * np.ones(n_frame, dtype=int)
                ids[det[0]][f] = det[6] if det[6] in {0, 2, 3, 5} and det[7] > CID_THR else -1
        out.append(set_id_for_each_frame_of_2dtracklets(ids, n_frame, wsize))
    return out
