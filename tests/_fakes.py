"""Deterministic CPU stand-ins used by the host-logic tests (no GPU): a pose 'model' whose
keypoints depend on the image and the box, so batching and ordering mistakes show up."""
from types import SimpleNamespace

import numpy as np


def fake_pose_batch(model, imgs, bboxes_per_img):
    out = []
    for img, bb in zip(imgs, bboxes_per_img):
        res = []
        for b in np.asarray(bb, dtype=np.float32).reshape(-1, 4):
            c = 0.5 * (b[:2] + b[2:])
            kp = c[None, :].astype(np.float64) + np.arange(17)[:, None] * float(img[0, 0, 0] + 1) / 7.0
            sc = (0.2 + 0.05 * np.arange(17) + 0.001 * float(img[0, 0, 0])).astype(np.float32)
            res.append(SimpleNamespace(pred_instances=SimpleNamespace(keypoints=kp[None], keypoint_scores=sc[None])))
        out.append(res)
    return out


def make_stores(root, n_cams=3, n_frames=9, seed=0):
    from mqhip import io as mqio
    rng = np.random.default_rng(seed)
    for c in range(n_cams):
        frames = np.zeros((n_frames, 8, 8, 3), np.uint8)
        frames[:, 0, 0, 0] = rng.integers(0, 200, n_frames)
        times = np.cumsum(rng.uniform(0.03, 0.06, n_frames)) + 10.0
        tracks = []
        for f in range(n_frames):
            rows = []
            for tid in range(2):
                if rng.uniform() < 0.2:
                    continue
                x, y = rng.uniform(100, 900, 2)
                rows.append([x, y, x + rng.uniform(40, 200), y + rng.uniform(60, 300), tid, 0.9])
            if f == 3 and c == 1:
                rows.append([50.7, 60.2, 50.9, 80.0, 7, 0.9])   # degenerate after int() truncation
            tracks.append(rows)
        mqio.write_frame_store(f"{root}/demo.{1000 + c}", frames, times, np.arange(n_frames) * 2 + 5, tracks,
                               1000 + c)
    return open_stores(root)


def open_stores(root):
    import glob
    from mqhip import io as mqio
    return [mqio.FrameStore(d) for d in sorted(glob.glob(f"{root}/demo.*"))]


# ----------------------------------------------------------------------------- h5py stand-in
class _H5Dataset:
    """``f[cam][key][()]`` returns a fresh copy, as h5py reads a dataset into a new array."""

    def __init__(self, a):
        self._a = np.asarray(a)

    def __getitem__(self, key):
        assert key == (), "the reference reads whole datasets only (step4:118-135)"
        return self._a.copy()


class _H5File:
    def __init__(self, store, path, mode="r"):
        assert mode == "r"
        self._groups = {k: {kk: _H5Dataset(vv) for kk, vv in v.items()} for k, v in store[str(path)].items()}

    def __getitem__(self, k):
        return self._groups[k]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def install_fake_h5py(monkeypatch, store):
    """Put a module named h5py into sys.modules whose File(path) serves ``store[path]`` =
    {camera id: {dataset name: array}}; h5py itself is absent in this image."""
    import sys
    import types
    mod = types.ModuleType("h5py")
    mod.File = lambda path, mode="r": _H5File(store, path, mode)
    monkeypatch.setitem(sys.modules, "h5py", mod)
    return mod


def calibration_h5_store(cams, base):
    """The two h5 files step 4 reads (step4:107-108) for synthetic omnidir cameras, in the shapes
    OpenCV's omnidir calibration stores: mtx at twice the image resolution (the first two rows are
    halved on read), dist (1, 4), xi (1, 1), K (3, 3), D (1, 4), rvec / tvec (3, 1)."""
    import os
    intr, extr = {}, {}
    for c in cams:
        k = str(c["name"])
        mtx = np.asarray(c["matrix"], dtype=np.float64).copy()
        mtx[:2, :] *= 2
        intr[k] = {"mtx": mtx, "dist": np.ravel(c["distortions"])[:4].reshape(1, 4),
                   "xi": np.ravel(c["xi"]).reshape(1, 1), "K": np.asarray(c["K"], dtype=np.float64),
                   "D": np.ravel(c["D"]).reshape(1, 4)}
        extr[k] = {"rvec": np.ravel(c["rvec"]).reshape(3, 1), "tvec": np.ravel(c["tvec"]).reshape(3, 1)}
    return {os.path.join(base, "cam_intrinsic.h5"): intr, os.path.join(base, "cam_extrinsic_optim.h5"): extr}
