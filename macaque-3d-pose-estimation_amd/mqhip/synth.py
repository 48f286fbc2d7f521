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


# ----------------------------------------------------------------------------- marker scenes
#
# Seeded random ViTPose weights give noise-like heatmaps: flat tops, peaks nowhere near the joints, and a
# DARK Newton step that is ill-conditioned.  A parity test of 3D joints needs realistic heatmaps: one
# smooth peak per joint at the joint.  No trained checkpoint is distributable, so the scene and the
# weights are built together: every joint is painted into the frames as a two-tone Gaussian marker, and
# ``marker_weights`` is a ViTPose whose patch embedding is a matched filter for those markers, whose
# encoder layers are the seeded random layers with their residual branches scaled down (they still run,
# and still perturb every token), and whose deconvolution head is a pixel shuffle of the filter outputs.
#
# Flip test (step1_proc2d.py:101; the second forward sees x.flip(-1), its heatmap is flipped back and
# re-indexed by FLIP_INDICES): a marker is colour A_j left of its centre line and B_j right of it, and a
# mirror pair (j, FLIP_INDICES[j]) swaps the two, so the flipped image of joint j's marker is exactly joint
# FLIP_INDICES[j]'s marker -- the flip-equivariance a trained network learns.  Joint 0 (nose) is one
# colour.  Heatmap column h matches the marker whose centre line lies between crop columns 4h+1 and 4h+2,
# which is mirror-symmetric (4h + 1.5 + 4(47 - h) + 1.5 = 191), so both forwards peak at the same pixel.

_MEAN_RGB = np.array([123.675, 116.28, 103.53])
_STD_RGB = np.array([58.395, 57.12, 57.375])
MARKER_AMP = 1.5           # marker colour deviation from the background, in normalised units
MARKER_SIGMA_CROP = 4.0    # marker Gaussian sigma in crop pixels (~1 heatmap pixel)
# Colours (unit directions in normalised RGB): mirror pair k = (joints 2k+1, 2k+2) is (A_k | B_k) and
# (B_k | A_k) with A_k orthogonal to B_k; the nose is one colour.  Numerically packed so that no joint's
# template reads another joint's marker -- whole, or a uniform region of either half -- above 1/2 of its own
# perfect match (the floor: a template inside the half of its mirror partner's marker that has its own
# colour reads exactly 1/2).
_NOSE_DIR = np.array([-0.9318, 0.1957, 0.3057])
_PAIR_A = np.array([[0.7961, 0.3362, -0.5031], [-0.3831, -0.4358, -0.8145], [0.2773, 0.4808, 0.8318],
                    [-0.4393, 0.841, -0.3159], [-0.7377, -0.6037, -0.3021], [-0.6996, -0.6919, -0.1783],
                    [0.5245, -0.1587, -0.8365], [0.4829, -0.831, 0.2763]])
_PAIR_B = np.array([[0.2756, 0.5387, 0.7961], [0.4328, -0.8636, 0.2585], [0.4666, -0.8242, 0.3209],
                    [-0.1284, 0.2893, 0.9486], [-0.4753, 0.7823, -0.4026], [-0.2094, -0.04, 0.977],
                    [-0.4093, 0.8145, -0.4112], [0.8065, 0.299, -0.5101]])
MARKER_CH_PER_JOINT = 20   # 4 row groups x (3 in-token column templates + the two halves of the 4th)


def marker_colours():
    """(J, 2, 3) unit colour directions (left half A, right half B) in normalised RGB per joint."""
    unit = lambda v: v / np.linalg.norm(v, axis=-1, keepdims=True)
    A = unit(_PAIR_A)
    B = unit(_PAIR_B - np.sum(_PAIR_B * A, axis=-1, keepdims=True) * A)
    out = np.zeros((17, 2, 3))
    out[0] = [unit(_NOSE_DIR), unit(_NOSE_DIR)]
    for j in range(1, 17):
        k = (j - 1) // 2
        out[j] = [A[k], B[k]] if FLIP_INDICES[j] > j else [B[k], A[k]]
    return out


def marker_weights(cfg, seed: int = 11, device="cpu", branch_scale: float = 1.0 / 32, gain: float = 0.6):
    """ViTPose weights (mmpose naming, bf16-representable) that detect the markers of ``render_markers``.

    * patch embedding: for joint j, row group sy (crop rows 4sy..4sy+3 of the token's 16) and heatmap column
      sx of the token, a template reading colour A_j on four crop columns and B_j on the next four (weights
      1/32, so a perfect match reads MARKER_AMP; eight columns, so a marker half-way between two heatmap
      columns still reads 3/4 of a match while a uniform half of the mirror partner's marker reads 1/2); the
      4th column's template straddles two tokens, so its A half is a channel of this token and its B half a
      channel of the next one.  340 channels; the rest keep
      the seeded random weights with biases of +-1 (they set the LayerNorm scale, as real features would);
    * encoder layers: the seeded random layers with the attention and FFN output projections scaled by
      ``branch_scale`` (a power of two, so still bf16-exact);
    * head: deconvolution 1 adds the two halves of the 4th template (tap kx = 0 of the next token) and
      shuffles each token's 4x4 templates into 2x2 parity channels, deconvolution 2 shuffles those into the
      64x48 map, the 1x1 layer scales joint j's channel by ``gain``.
    """
    import torch
    from .weights import make_random_weights
    w = make_random_weights(cfg, seed=seed, device="cpu")
    D, J, c = cfg.embed_dims, cfg.n_joints, cfg.deconv_ch
    nsig = MARKER_CH_PER_JOINT * J
    assert D >= nsig + 64 and c >= 4 * J and cfg.patch == 16 and cfg.patch_pad == 2, "marker weights need ViT-B/H"
    col = marker_colours()
    pe = torch.zeros(nsig, 3, 16, 16)
    for j in range(J):
        A, B = (torch.tensor(v, dtype=torch.float32) / 32.0 for v in col[j])
        for sy in range(4):
            base = MARKER_CH_PER_JOINT * j + 5 * sy
            rows = slice(4 * sy, 4 * sy + 4)
            for sx in range(3):
                pe[base + sx, :, rows, 4 * sx:4 * sx + 4] = A[:, None, None]
                pe[base + sx, :, rows, 4 * sx + 4:4 * sx + 8] = B[:, None, None]
            pe[base + 3, :, rows, 12:16] = A[:, None, None]
            pe[base + 4, :, rows, 0:4] = B[:, None, None]
    bf = lambda t: t.to(torch.bfloat16).to(torch.float32)
    w["backbone.patch_embed.projection.weight"][:nsig] = bf(pe)
    bias = w["backbone.patch_embed.projection.bias"]
    bias[:nsig] = 0.0
    bias[nsig:] = torch.tensor([1.0, -1.0]).repeat((D - nsig + 1) // 2)[:D - nsig]
    # top-down prior: a token centred outside the middle of the crop (where step 1's tight box sits after
    # the margin and the x1.25 scale) pushes its templates below zero, so the same joint of a neighbouring
    # individual inside the crop does not out-score the centred one (pos_embed is not flipped, and the prior
    # is symmetric about the crop centre)
    gh, gw = cfg.grid
    xi_t = np.abs((16.0 * np.arange(gw) + 5.5 - 95.5) / 96.0)
    eta_t = np.abs((16.0 * np.arange(gh) + 5.5 - 127.5) / 128.0)
    pen = np.minimum(2.0, 10.0 * (np.maximum(0.0, eta_t[:, None] - 0.66) + np.maximum(0.0, xi_t[None, :] - 0.66)))
    w["backbone.pos_embed"][..., :nsig] = bf(-torch.tensor(pen, dtype=torch.float32).reshape(1, gh * gw, 1))
    for i in range(cfg.num_layers):
        p = f"backbone.layers.{i}."
        for k in ("attn.proj.weight", "attn.proj.bias", "ffn.layers.1.weight", "ffn.layers.1.bias"):
            w[p + k] = w[p + k] * branch_scale
    w["backbone.ln1.weight"][:nsig] = 1.0
    w["backbone.ln1.bias"][:nsig] = 0.0
    d1 = torch.zeros(D, c, 4, 4)
    for j in range(J):
        for sy in range(4):
            base = MARKER_CH_PER_JOINT * j + 5 * sy
            py, qy = sy // 2, sy % 2
            for sx in range(3):
                d1[base + sx, 4 * j + 2 * qy + sx % 2, 1 + py, 1 + sx // 2] = 1.0
            d1[base + 3, 4 * j + 2 * qy + 1, 1 + py, 2] = 1.0      # 4th column, A half: this token (b = 1)
            d1[base + 4, 4 * j + 2 * qy + 1, 1 + py, 0] = 1.0      # B half: the previous token's column (b = 0)
    w["head.deconv_layers.0.weight"] = d1
    d2 = torch.zeros(c, c, 4, 4)
    for j in range(J):
        for qy in range(2):
            for qx in range(2):
                d2[4 * j + 2 * qy + qx, j, 1 + qy, 1 + qx] = 1.0
    w["head.deconv_layers.3.weight"] = d2
    for bn in (1, 4):
        w[f"head.deconv_layers.{bn}.weight"][:] = 1.0
        w[f"head.deconv_layers.{bn}.bias"][:] = 0.0
        w[f"head.deconv_layers.{bn}.running_mean"][:] = 0.0
        w[f"head.deconv_layers.{bn}.running_var"][:] = 1.0
    fin = torch.zeros(J, c, 1, 1)
    fin[torch.arange(J), torch.arange(J)] = gain
    w["head.final_layer.weight"] = bf(fin)
    w["head.final_layer.bias"] = torch.zeros(J)
    return {k: v.to(device) for k, v in w.items()}


def render_markers(kp2d_frame, boxes, seed: int = 4, height: int = IMG_H, width: int = IMG_W, noise: int = 12):
    """uint8 BGR frames (C, H, W, 3) for ``marker_weights``: background = the normalisation mean +-``noise``,
    every visible joint of kp2d_frame (C, A, J, 3) a two-tone Gaussian marker (``marker_colours``, amplitude
    MARKER_AMP) whose frame-pixel sigma maps to MARKER_SIGMA_CROP crop pixels through its individual's box
    (boxes (C, A, 4) xyxy; expanded and aspect-fixed like step 1, x1.25 like mmpose's TopdownAffine)."""
    rng = np.random.default_rng(seed)
    C, A, J, _ = kp2d_frame.shape
    col = marker_colours() * MARKER_AMP * _STD_RGB              # (J, 2, 3) RGB deviations
    frames = np.empty((C, height, width, 3), np.uint8)
    for c in range(C):
        img = _MEAN_RGB[None, None, :] + rng.uniform(-noise, noise, (height, width, 3))
        bb = expand_boxes(np.asarray(boxes[c], np.float64).reshape(-1, 4))
        for a in range(A):
            w_, h_ = bb[a, 2] - bb[a, 0], bb[a, 3] - bb[a, 1]
            h_fix = max(h_, w_ / 0.75) * 1.25
            sig = MARKER_SIGMA_CROP * h_fix / 256.0
            R = int(np.ceil(3.0 * sig))
            for j in range(J):
                u, v, s = kp2d_frame[c, a, j]
                if s <= 0 or not (R <= u < width - R - 1 and R <= v < height - R - 1):
                    continue
                x0, y0 = int(np.floor(u)) - R, int(np.floor(v)) - R
                xs = np.arange(x0, x0 + 2 * R + 2) - u                 # pixel centres (integer coordinates) relative to the marker
                ys = np.arange(y0, y0 + 2 * R + 2) - v
                al = np.exp(-(ys[:, None] ** 2 + xs[None, :] ** 2) / (2.0 * sig * sig))[..., None]
                dev = np.where((xs < 0.0)[None, :, None], col[j, 0], col[j, 1])
                patch = img[y0:y0 + 2 * R + 2, x0:x0 + 2 * R + 2]
                patch[:] = patch * (1.0 - al) + (_MEAN_RGB + dev) * al
        frames[c] = np.clip(np.rint(img), 0, 255).astype(np.uint8)[..., ::-1]
    return frames


def confident_head(weights, gain=20.0, shift=0.5):
    """Random ViTPose weights with the 1x1 head scaled and shifted so that heatmap peaks score above
    step 1's KP_THR / step 4's score threshold (seeded random weights otherwise give scores near 0 and
    an empty 3D stage).  In place; returns ``weights``."""
    weights["head.final_layer.weight"] = weights["head.final_layer.weight"] * gain
    weights["head.final_layer.bias"] = weights["head.final_layer.bias"] + shift
    return weights
