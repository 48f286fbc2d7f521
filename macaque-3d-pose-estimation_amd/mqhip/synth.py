"""Seeded synthetic inputs for the 2D->3D pose hot path.

Nothing here is the reference's code; it fabricates data of the reference's
shapes so that parity tests and bench.py can run offline:

* 8 omnidirectional (Mei unified model) cameras with the ids and order of
  ``calib/config.yaml:2-9`` and the real intrinsics printed in
  ``notebooks/bbox_optimisation_algorithm.ipynb:57-212`` (K with skew; the
  pinhole ``mtx`` focal gives xi = K.fx / mtx.fx - 1).  D ~ N(0, (.05,.05,1e-3,1e-3)).
* A ring of cameras at radius ~1.7 m around a 2.2 m cage (``calib/config.yaml:25-49``).
* A macaques x 17 joints, limb lengths in the 30-350 mm range
  (``notebooks/validation_track3_for_siddharth.ipynb:506-511``), random-walk roots.
* 2D observations: omnidir projection + N(0, 2 px), scores U(0.3, 1), 10 %
  dropped as zero rows (the ``create_kp2dfile`` zero-fill, ``step3...py:872-915``).
* Frames: uint8 1536x2048x3 BGR per view with blobs at the projected joints.
"""
from __future__ import annotations

import numpy as np

IMG_W, IMG_H = 2048, 1536

CAMERA_IDS = ["22983524", "23131347", "23131353", "23131363",
              "22983528", "22972495", "22983529", "23131354"]

# id -> (K fx, fy, skew, cx, cy, pinhole mtx fx)  (bbox_optimisation_algorithm.ipynb:57-212)
_INTRINSICS = {
    "22972495": (4958.07188, 4965.82504, 16.1050747, 1029.77310, 731.464908, 1189.91588),
    "22983524": (4992.86218, 5023.12633, -2.24000231, 1025.33048, 773.132847, 1290.93735),
    "22983528": (2521.43831, 2530.23506, 9.94888978, 1019.43873, 741.916251, 1223.11326),
    "22983529": (2413.32291, 2417.52222, -0.563821763, 1017.97898, 782.730777, 1197.64330),
    "23131347": (2922.99826, 2934.67217, -1.28646670, 1032.03937, 746.760561, 1202.61222),
    "23131353": (2288.16094, 2295.40601, -4.76453302, 1092.74441, 759.836352, 1240.72627),
    "23131354": (3424.88996, 3445.88210, -7.84068910, 1073.74580, 765.745380, 1225.80138),
    "23131363": (6817.84868, 6867.29933, 3.41498858, 1029.48494, 702.140629, 1255.70287),
}

BODYPARTS = ['nose', 'left_eye', 'right_eye', 'left_ear', 'right_ear',
             'left_shoulder', 'right_shoulder', 'left_elbow', 'right_elbow',
             'left_wrist', 'right_wrist', 'left_hip', 'right_hip',
             'left_knee', 'right_knee', 'left_ankle', 'right_ankle']

# model/pose/macaque.py:15-130 swap pairs
FLIP_INDICES = [0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15]

# configs/config_tmpl.toml:66-97
CONSTRAINTS = [
    ["nose", "left_eye"], ["nose", "right_eye"], ["left_eye", "right_eye"],
    ["nose", "left_ear"], ["nose", "right_ear"],
    ["left_eye", "left_ear"], ["right_eye", "right_ear"],
    ["left_ear", "right_ear"],
    ["left_shoulder", "left_ear"], ["right_shoulder", "right_ear"],
    ["left_shoulder", "right_shoulder"], ["left_shoulder", "left_elbow"],
    ["left_elbow", "left_wrist"], ["right_shoulder", "right_elbow"],
    ["right_elbow", "right_wrist"], ["left_hip", "right_hip"],
    ["left_hip", "left_knee"], ["left_knee", "left_ankle"],
    ["right_hip", "right_knee"], ["right_knee", "right_ankle"]]
CONSTRAINTS_WEAK = [
    ["left_shoulder", "left_hip"], ["right_shoulder", "right_hip"],
    ["left_shoulder", "right_hip"], ["right_shoulder", "left_hip"],
    ["left_shoulder", "right_shoulder"], ["left_hip", "right_hip"],
    ["left_eye", "nose"], ["right_eye", "nose"], ["left_eye", "left_ear"],
    ["right_eye", "right_ear"], ["left_ear", "right_ear"]]


def constraint_indices(names):
    ix = {b: i for i, b in enumerate(BODYPARTS)}
    return [[ix[a], ix[b]] for a, b in names]


def rodrigues_to_mat(rvec):
    r = np.asarray(rvec, dtype=np.float64).ravel()
    th = np.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2])
    if th < np.finfo(np.float64).eps:
        return np.eye(3)
    c, s = np.cos(th), np.sin(th)
    c1 = 1.0 - c
    u = r * (1.0 / th)
    rrt = np.outer(u, u)
    rx = np.array([[0, -u[2], u[1]], [u[2], 0, -u[0]], [-u[1], u[0], 0]])
    return c * np.eye(3) + c1 * rrt + s * rx


def mat_to_rodrigues(R):
    R = np.asarray(R, dtype=np.float64)
    c = (np.trace(R) - 1.0) * 0.5
    c = min(1.0, max(-1.0, c))
    th = np.arccos(c)
    if th < 1e-12:
        return np.zeros(3)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return w * (th / (2.0 * np.sin(th)))


def make_cameras(n_cams: int = 8, seed_dist: int = 0, seed_ext: int = 1):
    """Return a list of camera dicts with keys name,size,K,xi,D,rvec,tvec (float64)."""
    rng_d = np.random.default_rng(seed_dist)
    rng_e = np.random.default_rng(seed_ext)
    cams = []
    for i in range(n_cams):
        cid = CAMERA_IDS[i % len(CAMERA_IDS)]
        fx, fy, sk, cx, cy, mfx = _INTRINSICS[cid]
        K = np.array([[fx, sk, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]])
        xi = fx / mfx - 1.0
        D = rng_d.normal(0.0, 1.0, 4) * np.array([0.05, 0.05, 1e-3, 1e-3])
        ang = 2.0 * np.pi * i / n_cams + rng_e.normal(0, 0.05)
        radius = 1700.0 + rng_e.normal(0, 60.0)
        height = 700.0 if i % 2 == 0 else -500.0
        C = np.array([radius * np.cos(ang), radius * np.sin(ang), height + rng_e.normal(0, 40)])
        target = rng_e.normal(0, 80.0, 3)
        z = target - C
        z /= np.linalg.norm(z)
        up = np.array([0.0, 0.0, 1.0])
        x = np.cross(z, up)
        x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R = np.stack([x, y, z])
        # small roll jitter
        roll = rng_e.normal(0, 0.03)
        Rz = np.array([[np.cos(roll), -np.sin(roll), 0], [np.sin(roll), np.cos(roll), 0], [0, 0, 1]])
        R = Rz @ R
        rvec = mat_to_rodrigues(R)
        R = rodrigues_to_mat(rvec)
        tvec = -R @ C
        mtx = np.array([[mfx, 0.0, cx], [0.0, mfx, cy], [0.0, 0.0, 1.0]])
        cams.append(dict(name=cid, size=[IMG_W, IMG_H], K=K, xi=np.array([xi]), D=D,
                         rvec=rvec, tvec=tvec, matrix=mtx, distortions=np.zeros(5), fisheye=False,
                         omnidir=True))
    return cams


def camera_array(cams):
    """Pack cameras into the (C, 24) float64 parameter rows of the C ABI (include/mq_hip.h).

    Row layout: fx, fy, skew, cx, cy, xi, k1, k2, p1, p2, r00..r22 (9), t0, t1, t2.
    """
    out = np.zeros((len(cams), 24), dtype=np.float64)
    for i, c in enumerate(cams):
        K = np.asarray(c["K"], dtype=np.float64)
        D = np.asarray(c["D"], dtype=np.float64).ravel()
        R = rodrigues_to_mat(c["rvec"])
        out[i, 0:6] = [K[0, 0], K[1, 1], K[0, 1], K[0, 2], K[1, 2], float(np.ravel(c["xi"])[0])]
        out[i, 6:10] = D[:4]
        out[i, 10:19] = R.ravel()
        out[i, 19:22] = np.asarray(c["tvec"], dtype=np.float64).ravel()
    return out


def _template_skeleton():
    """17-joint macaque template (mm, body frame: x forward, z up)."""
    P = np.zeros((17, 3))
    P[5] = [60, 70, 0]      # left shoulder
    P[6] = [60, -70, 0]     # right shoulder
    P[11] = [-220, 60, 0]   # left hip
    P[12] = [-220, -60, 0]  # right hip
    P[0] = [190, 0, 60]     # nose
    P[1] = [160, 25, 80]
    P[2] = [160, -25, 80]
    P[3] = [120, 45, 80]
    P[4] = [120, -45, 80]
    P[7] = [80, 85, -150]
    P[8] = [80, -85, -150]
    P[9] = [90, 85, -300]
    P[10] = [90, -85, -300]
    P[13] = [-200, 70, -170]
    P[14] = [-200, -70, -170]
    P[15] = [-230, 70, -330]
    P[16] = [-230, -70, -330]
    return P


def make_skeletons(n_animals: int = 4, n_frames: int = 300, seed: int = 2):
    """Return (A, F, J, 3) float64 3D joints in mm inside a 2.2 m cage."""
    rng = np.random.default_rng(seed)
    T = _template_skeleton()
    out = np.zeros((n_animals, n_frames, 17, 3))
    for a in range(n_animals):
        scale = rng.uniform(0.85, 1.15)
        root = rng.uniform(-600, 600, 3) * np.array([1, 1, 0.3])
        yaw = rng.uniform(0, 2 * np.pi)
        vel = np.zeros(3)
        for f in range(n_frames):
            vel = 0.9 * vel + rng.normal(0, 4.0, 3) * np.array([1, 1, 0.3])
            root = np.clip(root + vel, -800, 800)
            yaw += rng.normal(0, 0.02)
            Rz = np.array([[np.cos(yaw), -np.sin(yaw), 0], [np.sin(yaw), np.cos(yaw), 0], [0, 0, 1]])
            jit = rng.normal(0, 3.0, (17, 3))
            out[a, f] = (T * scale + jit) @ Rz.T + root
    return out


def project_numpy(cam, X):
    """Projection (float64) used only to fabricate observations: the dict's camera model
    (pinhole / fisheye dicts from make_cameras_model, otherwise omnidir)."""
    if cam.get("fisheye", False) or not cam.get("omnidir", True):
        return _project_plain(cam, X)
    R = rodrigues_to_mat(cam["rvec"])
    Xc = X @ R.T + np.asarray(cam["tvec"]).ravel()
    nrm = np.sqrt(np.sum(Xc * Xc, axis=-1, keepdims=True))
    Xs = Xc / nrm
    xi = float(np.ravel(cam["xi"])[0])
    xu = Xs[..., 0] / (Xs[..., 2] + xi)
    yu = Xs[..., 1] / (Xs[..., 2] + xi)
    k1, k2, p1, p2 = np.asarray(cam["D"]).ravel()[:4]
    r2 = xu * xu + yu * yu
    r4 = r2 * r2
    rad = 1 + k1 * r2 + k2 * r4
    xd = xu * rad + 2 * p1 * xu * yu + p2 * (r2 + 2 * xu * xu)
    yd = yu * rad + p1 * (r2 + 2 * yu * yu) + 2 * p2 * xu * yu
    K = np.asarray(cam["K"])
    u = K[0, 0] * xd + K[0, 1] * yd + K[0, 2]
    v = K[1, 1] * yd + K[1, 2]
    return np.stack([u, v], axis=-1)


def _project_plain(cam, X):
    R = rodrigues_to_mat(cam["rvec"])
    Xc = X @ R.T + np.asarray(cam["tvec"]).ravel()
    x, y = Xc[..., 0] / Xc[..., 2], Xc[..., 1] / Xc[..., 2]
    d = np.asarray(cam["distortions"], dtype=np.float64).ravel()
    r2 = x * x + y * y
    if cam.get("fisheye", False):
        r = np.sqrt(r2)
        th = np.arctan(r)
        td = th * (1 + d[0] * th ** 2 + d[1] * th ** 4 + d[2] * th ** 6 + d[3] * th ** 8)
        g = np.where(r > 1e-8, td / np.maximum(r, 1e-300), 1.0)
        xd, yd = x * g, y * g
    else:
        k = np.zeros(5)
        k[:d.size] = d[:5]
        rad = 1 + k[0] * r2 + k[1] * r2 ** 2 + k[4] * r2 ** 3
        xd = x * rad + 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
        yd = y * rad + k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
    m = np.asarray(cam["matrix"], dtype=np.float64)
    return np.stack([m[0, 0] * xd + m[0, 2], m[1, 1] * yd + m[1, 2]], axis=-1)


def make_cameras_model(n_cams: int = 8, model: str = "pinhole", seed: int = 5):
    """Camera dicts of aniposelib's pinhole ``Camera`` or ``FisheyeCamera`` (cameras.py:173-426) in the
    calibration.toml key layout (name, size, matrix, distortions, rotation, translation, fisheye), on the
    extrinsics of make_cameras.  The matrix is each camera's omnidir "matrix" (its effective focal
    length) with a non-zero skew entry, which OpenCV's pinhole and fisheye functions ignore."""
    assert model in ("pinhole", "fisheye")
    rng = np.random.default_rng(seed)
    out = []
    for c in make_cameras(n_cams):
        m = np.asarray(c["matrix"], dtype=np.float64).copy()
        m[0, 1] = 3.0
        if model == "pinhole":
            dist = rng.normal(0.0, 1.0, 5) * np.array([0.05, 0.02, 1e-3, 1e-3, 0.005])
        else:
            dist = rng.normal(0.0, 1.0, 4) * np.array([0.02, 0.005, 1e-3, 5e-4])
        out.append(dict(name=c["name"], size=list(c["size"]), matrix=m, distortions=dist,
                        rotation=np.ravel(c["rvec"]).copy(), translation=np.ravel(c["tvec"]).copy(),
                        rvec=np.ravel(c["rvec"]).copy(), tvec=np.ravel(c["tvec"]).copy(),
                        fisheye=model == "fisheye", omnidir=False))
    return out


def make_kp2d(cams, skel, noise_px: float = 2.0, drop: float = 0.1, seed: int = 3):
    """Return kp2d (A, F, C, J, 3) float64 like step 3's kp2d.pickle (zero rows = missing)."""
    rng = np.random.default_rng(seed)
    A, F, J, _ = skel.shape
    C = len(cams)
    out = np.zeros((A, F, C, J, 3))
    for c, cam in enumerate(cams):
        uv = project_numpy(cam, skel.reshape(-1, 3)).reshape(A, F, J, 2)
        uv = uv + rng.normal(0, noise_px, uv.shape)
        sc = rng.uniform(0.3, 1.0, (A, F, J))
        dropped = rng.uniform(0, 1, (A, F, J)) < drop
        inimg = (uv[..., 0] >= 0) & (uv[..., 0] < IMG_W) & (uv[..., 1] >= 0) & (uv[..., 1] < IMG_H)
        keep = (~dropped) & inimg
        out[:, :, c, :, :2] = np.where(keep[..., None], uv, 0.0)
        out[:, :, c, :, 2] = np.where(keep, sc, 0.0)
    return out


def expand_boxes(boxes_xyxy_int, min_margin=0.20, max_margin=0.50, desired_ar=192.0 / 256.0):
    """Box expansion + aspect fix of step1_proc2d.py:270-292 (consts :71-73).

    ``boxes_xyxy_int``: (N,4) int tracker boxes.  Returns float32 (N,4) xyxy.
    """
    out = []
    for (x1, y1, x2, y2) in np.asarray(boxes_xyxy_int):
        w, h = float(x2 - x1), float(y2 - y1)
        cx, cy = x1 + 0.5 * w, y1 + 0.5 * h
        frac = np.clip((h - 50.0) / (200.0 - 50.0), 0.0, 1.0)
        margin = max_margin - (max_margin - min_margin) * frac
        wn, hn = w * (1 + margin), h * (1 + margin)
        ar = wn / hn
        if abs(ar - desired_ar) > 0.20:
            if ar < desired_ar:
                wn = hn * desired_ar
            else:
                hn = wn / desired_ar
        out.append([cx, cy, wn, hn])
    xywh = np.array(out, dtype=np.float32).reshape(-1, 4)
    res = []
    for cx, cy, w, h in xywh:
        res.append([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h])
    return np.array(res, dtype=np.float32).reshape(-1, 4)


def boxes_from_kp2d(kp2d_frame):
    """(C, A, J, 3) -> int32 tight boxes (C, A, 4) around visible joints (+ small pad)."""
    C, A, J, _ = kp2d_frame.shape
    out = np.zeros((C, A, 4), dtype=np.int32)
    for c in range(C):
        for a in range(A):
            v = kp2d_frame[c, a, :, 2] > 0
            if v.sum() < 2:
                out[c, a] = [900, 600, 1100, 860]
                continue
            p = kp2d_frame[c, a, v, :2]
            x1, y1 = np.floor(p.min(0) - 10)
            x2, y2 = np.ceil(p.max(0) + 10)
            x1, y1 = max(0, x1), max(0, y1)
            x2, y2 = min(IMG_W - 1, x2), min(IMG_H - 1, y2)
            if x2 <= x1 + 4:
                x2 = x1 + 5
            if y2 <= y1 + 4:
                y2 = y1 + 5
            out[c, a] = [x1, y1, x2, y2]
    return out


def make_frames(n_views: int, kp2d_frame=None, seed: int = 4, height: int = IMG_H, width: int = IMG_W):
    """Seeded uint8 BGR frames (V, H, W, 3): low-amplitude noise + bright blobs at joints."""
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 48, size=(n_views, height, width, 3), dtype=np.uint8)
    if kp2d_frame is not None:
        yy, xx = np.mgrid[-6:7, -6:7]
        disk = (xx * xx + yy * yy) <= 36
        for v in range(n_views):
            pts = kp2d_frame[v].reshape(-1, 3)
            for (u, w, s) in pts:
                if s <= 0:
                    continue
                x0, y0 = int(u), int(w)
                if 6 <= x0 < width - 7 and 6 <= y0 < height - 7:
                    col = rng.integers(120, 256, 3)
                    patch = frames[v, y0 - 6:y0 + 7, x0 - 6:x0 + 7]
                    patch[disk] = col
    return frames


def write_calibration_toml(cams, path):
    """calibration.toml in the layout step4 writes (step4:101-138) for synthetic cameras; pinhole / fisheye
    dicts of make_cameras_model in aniposelib's Camera.get_dict layout (cameras.py:191-199, 361-364)."""
    from .io import dump_toml
    calib = {}
    for i, c in enumerate(cams):
        if not c.get("omnidir", True):
            calib[f"cam_{i}"] = {
                "name": str(c["name"]), "size": list(c["size"]), "matrix": np.asarray(c["matrix"]).tolist(),
                "distortions": np.ravel(c["distortions"]).tolist(), "rotation": np.ravel(c["rotation"]).tolist(),
                "translation": np.ravel(c["translation"]).tolist(), "fisheye": bool(c["fisheye"])}
            continue
        calib[f"cam_{i}"] = {
            "name": str(c["name"]), "size": list(c["size"]), "matrix": np.asarray(c["matrix"]).tolist(),
            "distortions": np.ravel(c["distortions"]).tolist(), "rotation": np.ravel(c["rvec"]).tolist(),
            "translation": np.ravel(c["tvec"]).tolist(), "fisheye": False, "omnidir": True,
            "xi": np.ravel(c["xi"]).tolist(), "K": np.asarray(c["K"]).tolist(), "D": np.ravel(c["D"]).tolist()}
    dump_toml(calib, path)


# ----------------------------------------------------------------------------- step-2 scenes

def camparam_from_cams(cams):
    """The reference's step-2 ``camparam`` dict (step2:35-75) of synthetic cameras."""
    out = {"camera_id": [c["name"] for c in cams], "K": [], "xi": [], "D": [], "rvecs": [], "tvecs": [], "pmat": []}
    for c in cams:
        R = rodrigues_to_mat(c["rvec"])
        t = np.asarray(c["tvec"], dtype=np.float64).reshape(3, 1)
        out["K"].append(np.asarray(c["K"], dtype=np.float64))
        out["xi"].append(np.asarray(c["xi"], dtype=np.float64).reshape(1, 1))
        out["D"].append(np.asarray(c["D"], dtype=np.float64).reshape(1, 4))
        out["rvecs"].append(np.asarray(c["rvec"], dtype=np.float64).reshape(3, 1))
        out["tvecs"].append(t)
        out["pmat"].append(np.hstack([R, t]))
    return out


ID_LABELS = (0, 2, 3, 5)  # the ID classifier's individual classes (step2:734)


def make_alldata(cams, skel, noise_px=2.0, p_seen=0.9, p_dup=0.1, id_score=0.95, seed=5):
    """Per-camera step-1 rows T[c][f] = [track id, x1, y1, x2, y2, [[x, y, s] x J], id, id score] of
    skeletons (A, F, J, 3): each individual is seen by a camera with probability p_seen and gets a
    spurious second (shifted) detection with probability p_dup; track id = individual index
    (duplicates 10 + index); low-score keypoints are NaN as step 1 writes them."""
    rng = np.random.default_rng(seed)
    A, F, J, _ = skel.shape
    T = []
    for cam in cams:
        uv_all = project_numpy(cam, skel.reshape(-1, 3)).reshape(A, F, J, 2)
        rows_cam = []
        for f in range(F):
            rows = []
            for a in range(A):
                if rng.random() > p_seen:
                    continue
                for dup in ((False, True) if rng.random() < p_dup else (False,)):
                    uv = uv_all[a, f] + rng.normal(0, noise_px, (J, 2)) + (rng.normal(0, 25.0, 2) if dup else 0.0)
                    sc = rng.uniform(0.2, 1.0, J)
                    sc[rng.random(J) < 0.08] = 0.05
                    kp = np.concatenate([uv, sc[:, None]], axis=1)
                    kp[sc < 0.1, :2] = np.nan
                    x1, y1 = np.nanmin(uv, axis=0)
                    x2, y2 = np.nanmax(uv, axis=0)
                    cls = ID_LABELS[a % len(ID_LABELS)]
                    rows.append([10 + a if dup else a, float(x1), float(y1), float(x2), float(y2), kp.tolist(),
                                 cls, float(id_score * (0.5 if dup else 1.0))])
            rows_cam.append(rows)
        T.append(rows_cam)
    return T


# ----------------------------------------------------------------------------- clips on disk

def write_clip(root, data_name="clip", n_frames=300, n_views=8, n_animals=4, pool=4, height=IMG_H, width=IMG_W,
               fps=24.0, seed=2):
    """A synchronized multi-view clip on disk in the layout ``run_demo.proc`` reads (BASELINE config 3):
    per camera a FrameStore ``<root>/videos/<data_name>.<cam>`` (frames of ``pool`` rendered images reused
    through ``frame_index``, tracker rows = the tight boxes of the projected skeletons with track id =
    individual), ``<root>/results3D/<data_name>/calibration.toml`` and ``<root>/calib/config.yaml``.
    Camera 0's frame times are exactly 1/fps apart and the others jitter by +-2 ms, so step 1's time grid
    has ``n_frames`` steps.  Returns (cams, raw_dir, results_root, config_path, kp2d truth)."""
    import os

    import yaml

    from . import io as mqio
    cams = make_cameras(n_views)
    skel = make_skeletons(n_animals, n_frames + 1, seed=seed)
    truth = make_kp2d(cams, skel, noise_px=0.0, drop=0.0, seed=seed + 1)          # (A, F+1, C, J, 3)
    raw = os.path.join(root, "videos")
    rng = np.random.default_rng(seed + 2)
    t0 = 1000.0
    boxes = [boxes_from_kp2d(truth[:, f].transpose(1, 0, 2, 3)) for f in range(n_frames + 1)]  # (C, A, 4) each
    for c, cam in enumerate(cams):
        imgs = np.stack([make_frames(1, truth[:, j, c][None], seed=100 * c + j, height=height, width=width)[0]
                         for j in range(pool)])
        tracks = []
        for f in range(n_frames + 1):
            b = boxes[f][c]
            rows = [[float(x1), float(y1), float(x2), float(y2), float(a), 0.95]
                    for a, (x1, y1, x2, y2) in enumerate(b) if x2 > x1 and y2 > y1]
            tracks.append(rows)
        times = t0 + np.arange(n_frames + 1) / fps
        if c:
            times = times + rng.uniform(-2e-3, 2e-3, n_frames + 1)
        mqio.write_frame_store(os.path.join(raw, f"{data_name}.{cam['name']}"), imgs, times,
                               np.arange(n_frames + 1), tracks, cam["name"], frame_index=np.arange(n_frames + 1) % pool)
    res = os.path.join(root, "results3D")
    os.makedirs(os.path.join(res, data_name), exist_ok=True)
    write_calibration_toml(cams, os.path.join(res, data_name, "calibration.toml"))
    os.makedirs(os.path.join(root, "calib"), exist_ok=True)
    cfg = os.path.join(root, "calib", "config.yaml")
    with open(cfg, "w") as f:
        yaml.safe_dump({"camera_id": [int(c["name"]) for c in cams]}, f)
    return cams, raw, res, cfg, truth[:, :n_frames]


def confident_head(weights, gain=20.0, shift=0.5):
    """Random ViTPose weights with the 1x1 head scaled and shifted so that heatmap peaks score above
    step 1's KP_THR / step 4's score threshold (seeded random weights otherwise give scores near 0 and
    an empty 3D stage).  In place; returns ``weights``."""
    weights["head.final_layer.weight"] = weights["head.final_layer.weight"] * gain
    weights["head.final_layer.bias"] = weights["head.final_layer.bias"] + shift
    return weights
