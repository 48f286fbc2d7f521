"""Step 2 (cross-view matching at keyframes) on MI355X.

Mirrors ``src/pipeline/step2_crossviewmatching.py`` (same names, arguments and results):

* ``geometry_affinity2`` :373-432 -> ``mq_geometry_affinity`` (one thread per detection pair);
* ``matchSVT`` :130-216 -> ``mq_match_svt`` (one workgroup per keyframe, the whole ADMM loop on the GPU);
* ``calc_3dpose`` :436-461 / ``reproject`` :465-489 -> the omnidir undistort / pinv-DLT / projection
  kernels of step 4;
* ``MultiEstimator.predict_data`` :502-713 -> ``predict_batch``: every keyframe of a clip at once --
  one affinity launch, one matchSVT launch and two batched rounds of ``get_best_comb`` candidate
  evaluation.  The reference's keyframes are independent (its ``bcomb_prev`` only fills
  ``cont_mat``, which never enters W, :563-575), so batching does not change any result;
* ``set_id_for_each_frame_of_2dtracklets`` :717-800 / ``get_id_of_2dtrack`` :802-850 (host integer
  bookkeeping, vectorised windows);
* ``proc`` :854-959 -> ``match_keyframe.pickle`` with the same records (frame, bcomb, pose3d).

Drawing (``show`` / ``show_result``) and the imgstore frame reads it needs are out of scope and
raise.  ``get_camparam`` reads the reference's h5 calibration when h5py is importable (it is not in
this image) and otherwise the anipose ``calibration.toml`` (same cameras, the file step 4 reads).
The spectral initialisation in predict_data (:577-586) builds an X0 that matchSVT never receives; it
is not computed.
"""
from __future__ import annotations

import itertools
import json
import os

import numpy as np
import yaml

from mqhip import io as mqio
from mqhip.association import (THR_KP, StepTwoCameras, _combo_rmse, calc_3dpose_batch, dimgroup_to_cams,
                               geometry_affinity_batch, group_from_camparam, match_svt_batch)
from mqhip.geometry import rodrigues

ALPHA_ID = 0.2          # step2:22
CID_THR = 0.8           # step2:23
P_THR_2DT = 0.8         # step2:24
MODEL_CFG = {           # step2:25-31
    "joint_num": 17,
    "spectral": True,
    "alpha_SVT": 0.5,
    "lambda_SVT": 50,
    "dual_stochastic_SVT": False,
}
VALID_IDS = (0, 2, 3, 5)  # step2:734
KEYFRAME_STEP = 12        # step2:899


# ----------------------------------------------------------------------------- calibration

def get_camparam(config_path, calibration_path=None):
    """step2:35-75: {camera_id, K, xi, D, rvecs, tvecs, pmat}.  From cam_intrinsic.h5 /
    cam_extrinsic_optim.h5 next to config.yaml (needs h5py), else from an anipose calibration.toml
    (``calibration_path``, default next to config.yaml) whose cameras are named by camera_id or
    listed in camera_id order."""
    with open(config_path, "r") as f:
        cam_ids = yaml.safe_load(f)["camera_id"]
    base = os.path.dirname(config_path)
    if os.path.exists(os.path.join(base, "cam_intrinsic.h5")):
        import h5py  # absent in this image; reached only when the reference's h5 files exist
        out = {k: [] for k in ("K", "xi", "D", "rvecs", "tvecs", "pmat")}
        with h5py.File(os.path.join(base, "cam_intrinsic.h5"), "r") as fi, \
                h5py.File(os.path.join(base, "cam_extrinsic_optim.h5"), "r") as fe:
            for cid in cam_ids:
                out["K"].append(fi[f"/{cid}/K"][()])
                out["xi"].append(fi[f"/{cid}/xi"][()])
                out["D"].append(fi[f"/{cid}/D"][()])
                rv, tv = fe[f"/{cid}/rvec"][()], fe[f"/{cid}/tvec"][()]
                out["rvecs"].append(rv)
                out["tvecs"].append(tv)
                out["pmat"].append(np.hstack([rodrigues(rv), np.asarray(tv, dtype=np.float64).reshape(3, 1)]))
        out["camera_id"] = cam_ids
        return out
    path = calibration_path or os.path.join(base, "calibration.toml")
    calib = mqio.load_toml(path)
    cams = {str(v.get("name", k)): v for k, v in calib.items() if k != "metadata"}
    keys = [k for k in sorted(calib.keys()) if k != "metadata"]
    out = {"camera_id": cam_ids, "K": [], "xi": [], "D": [], "rvecs": [], "tvecs": [], "pmat": []}
    for i, cid in enumerate(cam_ids):
        d = cams.get(str(cid)) or calib[keys[i]]
        K = np.asarray(d.get("K", d.get("matrix")), dtype=np.float64)
        rv = np.asarray(d.get("rotation", d.get("rvec")), dtype=np.float64).reshape(3, 1)
        tv = np.asarray(d.get("translation", d.get("tvec")), dtype=np.float64).reshape(3, 1)
        out["K"].append(K)
        out["xi"].append(np.asarray(d["xi"], dtype=np.float64).reshape(1, 1))
        out["D"].append(np.asarray(d.get("D", d.get("distortions")), dtype=np.float64).reshape(1, -1)[:, :4])
        out["rvecs"].append(rv)
        out["tvecs"].append(tv)
        out["pmat"].append(np.hstack([rodrigues(rv), tv]))
    return out


def _load_json(path):
    with open(path, "r") as f:
        return json.load(f)


def _cams(camparam, device):
    if isinstance(camparam, StepTwoCameras):
        return camparam
    return StepTwoCameras(camparam, device=device)


# ----------------------------------------------------------------------------- reference surface

def undistort_points(config_path, i_cam, pos_2d, camparam=None, device: int = 0):
    """step2:306-325: cv2.omnidir.undistortPoints of (N_kp, 2) points of camera i_cam."""
    cams = _cams(camparam if camparam is not None else get_camparam(config_path), device)
    pts = np.zeros((cams.n_cam,) + np.asarray(pos_2d).reshape(-1, 2).shape)
    pts[i_cam] = np.asarray(pos_2d, dtype=np.float64).reshape(-1, 2)
    return cams.proj.undistort_points(pts)[i_cam]


def geometry_affinity2(points_set, dimGroup, config_path, camparam=None, device: int = 0):
    """step2:373-432: points_set (M, N_kp, 3) undistorted keypoints + scores; dimGroup (n_cam + 1,)."""
    if camparam is None:
        camparam = get_camparam(config_path)
    points_set = np.asarray(points_set, dtype=np.float64)
    M = points_set.shape[0]
    g = camparam.rays if isinstance(camparam, StepTwoCameras) else group_from_camparam(camparam, device=device)
    aff = geometry_affinity_batch(g, points_set[None], dimgroup_to_cams(dimGroup, M)[None], thr_kp=THR_KP)
    return aff[0]


def matchSVT(S, dimGroup, *, alpha=0.1, pselect=1, tol=5e-4, maxIter=500, verbose=False, eigenvalues=False,
             _lambda=50, mu=64, dual_stochastic_SVT=True, device: int = 0):
    """step2:130-216 -> uint8 match matrix.  Like the reference, S's diagonal is zeroed in place.  The dual-stochastic projection is not implemented (step 2 runs with
    dual_stochastic_SVT=False, MODEL_CFG :30)."""
    if dual_stochastic_SVT:
        raise NotImplementedError("matchSVT(dual_stochastic_SVT=True): step 2 runs with MODEL_CFG "
                                  "dual_stochastic_SVT=False; the myproj2dpam projection is not on MI355X")
    if verbose or eigenvalues:
        raise NotImplementedError("matchSVT verbose / eigenvalues diagnostics are not kept")
    N = S.shape[0]
    S[np.arange(N), np.arange(N)] = 0
    dg = np.asarray(dimGroup)
    match, _ = match_svt_batch(S[None], [N], dimgroup_to_cams(dg, N)[None], alpha=alpha, _lambda=_lambda, mu=mu,
                               tol=tol, maxIter=maxIter, pselect=pselect, device=device)
    return match[0]


def calc_3dpose(kp_2d, config_path, camparam=None, device: int = 0):
    """step2:436-461: kp_2d (n_cam, n_kp, 3) raw x, y, score -> (n_kp, 3)."""
    cams = _cams(camparam if camparam is not None else get_camparam(config_path), device)
    return calc_3dpose_batch(cams, np.asarray(kp_2d, dtype=np.float64)[None])[0]


def reproject(i_cam, p3d, camparam=None, config_path="", device: int = 0):
    """step2:465-489: (N_pts, 3) -> (N_pts, 2) through camera i_cam."""
    cams = _cams(camparam if camparam is not None else get_camparam(config_path), device)
    return cams.proj.project(np.asarray(p3d, dtype=np.float64).reshape(-1, 3))[i_cam]


# ----------------------------------------------------------------------------- MultiEstimator

class _Keyframe:
    """predict_data's per-keyframe state (step2:521-551)."""

    def __init__(self, info_dict, n_kp):
        self.n_cam = len(info_dict)
        counts = [len(info_dict[c][0]) for c in range(self.n_cam)]
        self.dimGroup = np.concatenate([[0], np.cumsum(counts)]).astype(int)
        self.info = [d for c in range(self.n_cam) for d in info_dict[c][0]]
        self.M = len(self.info)
        self.sub2cam = np.repeat(np.arange(self.n_cam), counts)
        if self.M:
            self.raw = np.array([d["pose2d_raw"] for d in self.info], dtype=np.float64).reshape(self.M, n_kp, 3)
            pose2d = np.array([d["pose2d"] for d in self.info], dtype=np.float64).reshape(self.M, n_kp, 2)
            self.kp_mat = np.concatenate([pose2d, self.raw[..., 2:3]], axis=2)
            self.cid = np.array([d["cid"] for d in self.info])
        self.matched = []


class MultiEstimator:
    """step2:493-713 on MI355X.  ``predict_data`` keeps the reference signature for one keyframe;
    ``predict_batch`` runs many keyframes together."""

    def __init__(self, cfg, debug=False, device: int = 0):
        self.cfg = cfg
        self.debug = debug
        self.device = device

    def predict_data(self, info_dict, show=False, plt_id=0, camparam=None, bcomb_prev=None):
        """step2:502-713 -> (matched_list, P3d_list, bcomb_list)."""
        return self.predict_batch([info_dict], show=show, camparam=camparam)[0]

    def predict_batch(self, info_dicts, show=False, camparam=None):
        if show:
            raise NotImplementedError("predict_data(show=True): drawing is out of scope on MI355X")
        if camparam is None:
            camparam = get_camparam(self.cfg)
        cams = _cams(camparam, self.device)
        n_kp = MODEL_CFG["joint_num"]
        kfs = [_Keyframe(d, n_kp) for d in info_dicts]
        live = [k for k in kfs if k.M > 0]
        if live:
            self._match(live, cams, n_kp)
            self._refine(live, cams, n_kp)
        return [self._finish(k, cams, n_kp) if k.M > 0 else ([], [], []) for k in kfs]

    # -- affinity + matchSVT for every keyframe (step2:553-607)
    def _match(self, kfs, cams, n_kp):
        B, Mmax = len(kfs), max(k.M for k in kfs)
        pts = np.zeros((B, Mmax, n_kp, 3))
        cod = np.full((B, Mmax), -1, dtype=np.int32)
        for b, k in enumerate(kfs):
            pts[b, :k.M] = k.kp_mat
            cod[b, :k.M] = k.sub2cam
        geo_all = geometry_affinity_batch(cams.rays, pts, cod, thr_kp=THR_KP)
        W_all = np.zeros((B, Mmax, Mmax))
        for b, k in enumerate(kfs):
            geo = geo_all[b, :k.M, :k.M]
            cid_mat = ((k.sub2cam[:, None] != k.sub2cam[None, :]) & (k.cid[:, None] >= 0)
                       & (k.cid[:, None] == k.cid[None, :])).astype(np.float64)
            W = ALPHA_ID * cid_mat + (1 - ALPHA_ID) * geo
            W *= (geo > 0)
            W_all[b, :k.M, :k.M] = np.nan_to_num(W)
        match, _ = match_svt_batch(W_all, [k.M for k in kfs], cod, alpha=MODEL_CFG["alpha_SVT"],
                                   _lambda=MODEL_CFG["lambda_SVT"], device=self.device)
        for b, k in enumerate(kfs):
            mm = match[b, :k.M, :k.M]
            cols = np.nonzero(mm.sum(axis=0) > 1.9)[0]
            bin_match = mm[:, cols] > 0.9
            lists = [[] for _ in range(bin_match.shape[1])]
            for sub, row in enumerate(bin_match):
                if row.sum() != 0:
                    lists[row.argmax()].append(sub)
            k.matched = [np.array(lst) for lst in lists]

    # -- get_best_comb (step2:610-658), two batched rounds: every cluster, then the leftovers
    def _best_combs(self, reqs, cams, n_kp):
        """reqs: list of (keyframe, person index array) -> list of best index arrays."""
        out = [None] * len(reqs)
        kp_rows, present_rows, owners = [], [], []
        spans = {}
        for r, (k, person) in enumerate(reqs):
            person = np.asarray(person, dtype=int)
            cam_ids = k.sub2cam[person]
            groups = [person[np.where(cam_ids == c)].tolist() or [None] for c in range(k.n_cam)]
            combos = list(itertools.product(*groups))
            if len(combos) == 1:
                out[r] = person
                continue
            start = len(kp_rows)
            for combo in combos:
                kp = np.zeros((k.n_cam, n_kp, 3))
                pres = np.zeros(k.n_cam, dtype=bool)
                for c, sub in enumerate(combo):
                    if sub is not None:
                        kp[c] = k.raw[sub]
                        pres[c] = True
                kp_rows.append(kp)
                present_rows.append(pres)
            spans[r] = (start, combos)
        if kp_rows:
            err = _combo_rmse(cams, np.stack(kp_rows), np.stack(present_rows))
            for r, (start, combos) in spans.items():
                best = combos[int(np.argmin(err[start:start + len(combos)]))]
                out[r] = np.array([i for i in best if i is not None], dtype=int)
        return out

    def _refine(self, kfs, cams, n_kp):
        reqs = [(k, person) for k in kfs for person in k.matched]
        best = self._best_combs(reqs, cams, n_kp)
        second = []
        for (k, person), bst in zip(reqs, best):
            k._refined = getattr(k, "_refined", [])
            k._refined.append([bst, None])
            leftover = set(person.tolist()) - set(bst.tolist())
            if len(leftover) > 1:
                second.append((k, np.array(list(leftover), dtype=int), k._refined[-1]))
        best2 = self._best_combs([(k, p) for k, p, _ in second], cams, n_kp)
        for (_, _, slot), b2 in zip(second, best2):
            slot[1] = b2
        for k in kfs:
            k.matched = [p for pair in getattr(k, "_refined", []) for p in pair if p is not None]

    # -- final 3D poses and bcomb arrays (step2:694-713)
    def _finish(self, k, cams, n_kp):
        people = [p for p in k.matched if p.shape[0] >= 2]
        kp = np.zeros((len(people), k.n_cam, n_kp, 3))
        for i, person in enumerate(people):
            for sub in person:
                kp[i, k.sub2cam[sub]] = k.raw[sub]
        p3d = calc_3dpose_batch(cams, kp)
        bcombs = []
        for person in people:
            bc = -np.ones(k.n_cam, dtype=int)
            for sub in person:
                bc[k.sub2cam[sub]] = k.info[sub]["bbox_id"][1]
            bcombs.append(bc)
        return people, [p3d[i] for i in range(len(people))], bcombs


# ----------------------------------------------------------------------------- 2D tracklet IDs

def set_id_for_each_frame_of_2dtracklets(Cid, n_frame, wsize):
    """step2:717-800 with the window counts from prefix sums."""
    out = {k: v.copy() for k, v in Cid.items()}
    h = wsize // 2
    for k, arr in Cid.items():
        arr = np.asarray(arr)
        valid = np.flatnonzero(arr >= -1)
        start_f, end_f = int(valid.min()), int(valid.max())
        onehot = np.stack([arr == v for v in VALID_IDS], axis=1).astype(np.int64)
        csum = np.concatenate([np.zeros((1, len(VALID_IDS)), np.int64), np.cumsum(onehot, axis=0)])
        labels = np.full(n_frame, -1, dtype=int)
        f = np.arange(max(start_f, h), min(end_f, n_frame - h))
        if f.size:
            cnts = csum[f + h] - csum[f - h]
            tot = cnts.sum(axis=1)
            mx = cnts.max(axis=1)
            with np.errstate(invalid="ignore", divide="ignore"):
                ok = (tot > 0) & (mx / np.where(tot > 0, tot, 1) > P_THR_2DT) & (mx >= 12)
            labels[f[ok]] = np.argmax(cnts[ok], axis=1)
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
            for fi in np.flatnonzero(labels >= 0):
                cur = labels[fi]
                if cur == prev_id:
                    continue
                if prev_id == -1:
                    labels[:fi] = cur
                else:
                    ip = np.flatnonzero(onehot[max(1, prev_frame - h):fi + 1, prev_id]) + max(1, prev_frame - h)
                    i_prev = ip.max() if ip.size else prev_frame
                    c1 = min(fi + h, n_frame)
                    ic = np.flatnonzero(onehot[prev_frame:c1 + 1, cur]) + prev_frame
                    i_curr = ic.min() if ic.size else fi
                    mid = (i_prev + i_curr) // 2
                    labels[prev_frame:mid] = prev_id
                    labels[mid:fi] = cur
                prev_id, prev_frame = cur, fi
            if prev_id >= 0:
                labels[prev_frame:] = prev_id
        out[k] = labels
    return out


def _id_sequences(data_per_cam, wsize=24 * 5):
    """get_id_of_2dtrack's body on loaded alldata rows (zeroes duplicated confident ID scores in place)."""
    n_frame = len(data_per_cam[0])
    for rows_cam in data_per_cam:
        for dets in rows_cam:
            cnts = np.zeros(20, int)
            for det in dets:
                if det[6] in VALID_IDS and det[7] > CID_THR:
                    cnts[det[6]] += 1
            for dup in np.flatnonzero(cnts > 1):
                for det in dets:
                    if det[6] == int(dup):
                        det[7] = 0.0
    out = []
    for rows_cam in data_per_cam:
        ids = {}
        for f, dets in enumerate(rows_cam):
            for det in dets:
                if det[0] not in ids:
                    ids[det[0]] = -2 * np.ones(n_frame, dtype=int)
                ids[det[0]][f] = det[6] if det[6] in VALID_IDS and det[7] > CID_THR else -1
        out.append(set_id_for_each_frame_of_2dtracklets(ids, n_frame, wsize))
    return out


def get_id_of_2dtrack(config_path, result_dir):
    """step2:802-850: per camera {track id: per-frame ID label} from alldata.json."""
    with open(config_path, "r") as f:
        cam_ids = yaml.safe_load(f)["camera_id"]
    data = [_load_json(os.path.join(result_dir, str(c), "alldata.json")) for c in cam_ids]
    return _id_sequences(data)


# ----------------------------------------------------------------------------- main entry point

def build_info_dicts(T, Cid2d, cams: StepTwoCameras, frames, n_kp=17):
    """step2:900-926 for the given frames: per camera {0: [detections], 'image_data': []} with the
    undistorted pose2d (one batched undistortion for every detection of every frame)."""
    raw, where = [], []
    for fi, f in enumerate(frames):
        for c in range(cams.n_cam):
            for di, det in enumerate(T[c][f]):
                raw.append(np.asarray(det[5], dtype=np.float64).reshape(n_kp, 3))
                where.append((fi, c, di))
    und = None
    if raw:
        pts = np.zeros((cams.n_cam, len(raw), n_kp, 2))
        for r, (fi, c, di) in enumerate(where):
            pts[c, r] = raw[r][:, :2]
        und = cams.proj.undistort_points(pts.reshape(cams.n_cam, -1, 2)).reshape(cams.n_cam, len(raw), n_kp, 2)
    infos = [{c: {0: [], "image_data": []} for c in range(cams.n_cam)} for _ in frames]
    for r, (fi, c, di) in enumerate(where):
        det = T[c][frames[fi]][di]
        infos[fi][c][0].append({"pose2d": und[c, r], "pose2d_raw": raw[r], "bbox": det[1:5],
                                "bbox_id": [c, det[0]], "cid": Cid2d[c][det[0]][frames[fi]]})
    return infos


def proc(data_name, result_dir_root, raw_data_dir, config_path, show_result=False, camparam=None,
         device: int = 0):
    """step2:854-959: keyframes 1, 13, 25, ... (< n_frame - 12) -> <result_dir>/match_keyframe.pickle
    = [{frame, bcomb, pose3d}]."""
    if show_result:
        raise NotImplementedError("show_result: drawing is out of scope on MI355X")
    result_dir = os.path.join(result_dir_root, data_name)
    if camparam is None:
        calib = os.path.join(os.path.dirname(config_path), "calibration.toml")
        if not os.path.exists(calib):
            calib = os.path.join(result_dir, "calibration.toml")
        camparam = get_camparam(config_path, calibration_path=calib)
    cams = _cams(camparam, device)
    with open(config_path, "r") as f:
        cam_ids = yaml.safe_load(f)["camera_id"]
    T = [_load_json(os.path.join(result_dir, str(c), "alldata.json")) for c in cam_ids]
    Cid2d = _id_sequences([[[list(det) for det in rows] for rows in Tc] for Tc in T])
    frames = list(range(1, len(T[0]) - KEYFRAME_STEP, KEYFRAME_STEP))
    infos = build_info_dicts(T, Cid2d, cams, frames, MODEL_CFG["joint_num"])
    results = MultiEstimator(config_path, device=device).predict_batch(infos, camparam=cams)
    match_keyframes = [{"frame": f, "bcomb": bc, "pose3d": p3}
                       for f, (_, p3, bc) in zip(frames, results)]
    mqio.dump_pickle(match_keyframes, os.path.join(result_dir, "match_keyframe.pickle"))
    return match_keyframes
