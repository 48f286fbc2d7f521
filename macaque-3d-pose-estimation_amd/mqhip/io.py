"""On-disk formats around the hot path.

* ``kp2d.pickle`` / ``kp2d_f.pickle`` / ``kp3d.pickle``: the reference pickles plain
  numpy arrays and dicts of them (step4:151-170, :332-339).  ``load_array_pickle``
  reads them with an allow-list unpickler that can only rebuild numpy arrays,
  dtypes and builtin containers -- nothing else in the file can execute.
* ``calibration.toml`` / ``config.toml``: read with tomli; ``dump_toml`` writes the
  subset of TOML the reference's ``toml.dump`` produces for these files (tables of
  strings, numbers, booleans and nested lists).
* ``alldata.json`` / ``frame_num.npy`` (step1_proc2d.py:364-375): plain JSON / npy.
* ``FrameStore``: the per-camera frame source of step 1 (stands in for imgstore).
"""
from __future__ import annotations

import io
import json
import os
import pickle

import numpy as np

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
    ("builtins", "list"),
    ("builtins", "dict"),
    ("builtins", "tuple"),
    ("collections", "OrderedDict"),
}


class _ArrayUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a keypoint pickle")


def load_array_pickle(path):
    """Load a pickle holding numpy arrays / dicts / lists only."""
    with open(path, "rb") as f:
        return _ArrayUnpickler(io.BytesIO(f.read())).load()


def dump_pickle(obj, path):
    with open(path, "wb") as f:
        pickle.dump(obj, f)


def load_toml(path):
    try:
        import tomllib as _toml  # py >= 3.11
    except ImportError:  # pragma: no cover - py3.10 image
        import tomli as _toml
    with open(path, "rb") as f:
        return _toml.load(f)


def _val(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    if isinstance(v, (float, np.floating)):
        v = float(v)
        if v != v:
            return "nan"
        if v in (float("inf"), float("-inf")):
            return "inf" if v > 0 else "-inf"
        return repr(v)
    if isinstance(v, str):
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"') + '"'
    if isinstance(v, np.ndarray):
        v = v.tolist()
    if isinstance(v, (list, tuple)):
        return "[ " + ", ".join(_val(x) for x in v) + ",]" if len(v) else "[]"
    raise TypeError(f"cannot write {type(v)} to TOML")


def dump_toml(data: dict, path):
    """Top-level scalars first, then one [table] per dict value (one nesting level)."""
    lines = []
    for k, v in data.items():
        if not isinstance(v, dict):
            lines.append(f"{k} = {_val(v)}")
    for k, v in data.items():
        if isinstance(v, dict):
            lines.append("")
            lines.append(f"[{k}]")
            for kk, vv in v.items():
                if isinstance(vv, dict):
                    raise TypeError("nested tables are not used by these files")
                lines.append(f"{kk} = {_val(vv)}")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


# ----------------------------------------------------------------------------- frame stores
class FrameStore:
    """One camera's synchronized frames plus the detector/tracker output for them.

    Stands in for the reference's imgstore (``imgstore.new_for_filename(<raw>/<data>.<cam>/
    metadata.yaml)``, step1_proc2d.py:403-408), which is not installable here and decodes video
    this build does not handle.  Directory layout (``write_frame_store`` makes one):

      metadata.yaml     imgstore-style metadata (camera id, image size); its presence is what
                        step 1 globs for, exactly like the reference
      frames.npy        uint8 (N, H, W, 3) BGR, memory-mapped (never loaded whole)
      frame_time.npy    float64 (N,)  -- get_frame_metadata()["frame_time"]
      frame_number.npy  int64 (N,)    -- get_frame_metadata()["frame_number"]
      tracks.json       per stored frame, the tracker rows [x1, y1, x2, y2, track_id, ...] that the
                        out-of-scope Swin detector + BoT-SORT produce (step1_proc2d.py:226-252)
      id_preds.json     optional: per stored frame, per row {"pred_label", "pred_score"} of the
                        ResNet-152 ID classifier (step1_proc2d.py:140-163)
      frame_index.npy   optional int64 (N,): frame i is frames.npy[frame_index[i]] -- synthetic clips
                        reuse a small pool of rendered images so a 300-frame x 8-view clip at the
                        cameras' 2048x1536 stays a few hundred MB on disk
    """

    def __init__(self, directory):
        self.filename = str(directory)
        meta = os.path.join(directory, "metadata.yaml")
        if not os.path.exists(meta):
            raise FileNotFoundError(meta)
        self.frames = np.load(os.path.join(directory, "frames.npy"), mmap_mode="r")
        self.frame_time = np.load(os.path.join(directory, "frame_time.npy"))
        self.frame_number = np.load(os.path.join(directory, "frame_number.npy"))
        with open(os.path.join(directory, "tracks.json")) as f:
            self.tracks = json.load(f)
        idp = os.path.join(directory, "id_preds.json")
        self.id_preds = None
        if os.path.exists(idp):
            with open(idp) as f:
                self.id_preds = json.load(f)
        fi = os.path.join(directory, "frame_index.npy")
        self.frame_index = np.load(fi) if os.path.exists(fi) else np.arange(len(self.frames))
        if len(self.frame_index) and (self.frame_index.min() < 0 or self.frame_index.max() >= len(self.frames)):
            raise ValueError(f"{directory}: frame_index out of range")
        if not (len(self.frame_index) == len(self.frame_time) == len(self.frame_number) == len(self.tracks)):
            raise ValueError(f"{directory}: frames, times, numbers and tracks differ in length")
        self._pos = {int(n): i for i, n in enumerate(self.frame_number)}

    def get_frame_metadata(self):
        return {"frame_time": self.frame_time, "frame_number": self.frame_number}

    def index_of(self, frame_number):
        return self._pos[int(frame_number)]

    def image(self, frame_number):
        return np.asarray(self.frames[self.frame_index[self.index_of(frame_number)]])

    def tracks_of(self, frame_number):
        return self.tracks[self.index_of(frame_number)]

    def id_preds_of(self, frame_number):
        return None if self.id_preds is None else self.id_preds[self.index_of(frame_number)]


def write_frame_store(directory, frames, frame_time, frame_number, tracks, camera_id, id_preds=None,
                      frame_index=None):
    """Write a FrameStore directory (used by tests and synthetic runs).  With ``frame_index`` the
    ``frames`` are a pool of images and frame i shows ``frames[frame_index[i]]``."""
    import yaml
    os.makedirs(directory, exist_ok=True)
    frames = np.asarray(frames, dtype=np.uint8)
    with open(os.path.join(directory, "metadata.yaml"), "w") as f:
        yaml.safe_dump({"__store": {"camera_id": str(camera_id), "imgshape": list(frames.shape[1:]),
                                    "format": "npy"}}, f)
    np.save(os.path.join(directory, "frames.npy"), frames)
    np.save(os.path.join(directory, "frame_time.npy"), np.asarray(frame_time, dtype=np.float64))
    np.save(os.path.join(directory, "frame_number.npy"), np.asarray(frame_number, dtype=np.int64))
    with open(os.path.join(directory, "tracks.json"), "w") as f:
        json.dump([[list(map(float, r)) for r in t] for t in tracks], f)
    if id_preds is not None:
        with open(os.path.join(directory, "id_preds.json"), "w") as f:
            json.dump(id_preds, f)
    if frame_index is not None:
        np.save(os.path.join(directory, "frame_index.npy"), np.asarray(frame_index, dtype=np.int64))
