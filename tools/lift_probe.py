"""bench.py's config-4 lift leg (lift_gpu: Viterbi, RANSAC, batched optim_points, reprojection on the
bench's own synthetic clip) run alone, optionally against another libmq_hip.so (A/B).  One JSON line.

python tools/lift_probe.py [--lib path/to/libmq_hip.so] [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from mqhip import _lib
    if args.lib:  # after torch: torch's HIP runtime must be the one the library binds to
        import ctypes
        probe = ctypes.CDLL(os.path.abspath(args.lib))
        for name in list(_lib._SIGS):  # an older build may lack newer entry points
            if not hasattr(probe, name):
                del _lib._SIGS[name]
        _lib.ABI_VERSION = probe.mq_abi_version()  # an A/B build may predate the current ABI
        _lib.load(os.path.abspath(args.lib))
    _lib.apply_tuning_env(_lib.load())
    import bench
    print(json.dumps(bench.lift_gpu(0, reps=args.reps)), flush=True)


if __name__ == "__main__":
    main()
