"""Drop-in mirror of the reference's ``src`` package for the hot path.

Same module paths and entry points as the reference (``src.pipeline.step4_aniposefiltering``,
``src.pipeline.step1_proc2d``, ``src.third_party.aniposelib.cameras``,
``src.third_party.anipose.filter_pose``, ``src.utils.multicam_toolbox``); every
computation underneath runs in libmq_hip (``mqhip``).
"""
import os as _os
import sys as _sys

_PKG_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _PKG_ROOT not in _sys.path:
    _sys.path.insert(0, _PKG_ROOT)
