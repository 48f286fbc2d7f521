"""On-disk formats around the hot path.

* ``kp2d.pickle`` / ``kp2d_f.pickle`` / ``kp3d.pickle``: the reference pickles plain
  numpy arrays and dicts of them (step4:151-170, :332-339).  ``load_array_pickle``
  reads them with an allow-list unpickler that can only rebuild numpy arrays,
  dtypes and builtin containers -- nothing else in the file can execute.
* ``calibration.toml`` / ``config.toml``: read with tomli; ``dump_toml`` writes the
  subset of TOML the reference's ``toml.dump`` produces for these files (tables of
  strings, numbers, booleans and nested lists).
"""
from __future__ import annotations

import io
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
