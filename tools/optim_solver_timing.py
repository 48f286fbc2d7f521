"""Wall time of optim_points per solver ("trf": scipy's algorithm restated, the default; "lm"): BASELINE config 4's
300-frame clip (4 individuals, the bench's lift inputs after Viterbi + RANSAC) and the marker-scene problems of
tests/golden/optim_problems.npz (4 individuals per scene), median of --reps after a warm-up, with the solver stats.
python tools/optim_solver_timing.py [--reps 3] [--solvers trf,lm] [--chunk 16] [--fb 4]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"), os.path.join(ROOT, "tests")]


def config4_problem():
    import bench
    from mqhip import synth
    from mqhip.geometry import CameraGroup, viterbi_filter
    cams, kp2d = bench.lift_inputs()
    A, F, C, J, _ = kp2d.shape
    g = CameraGroup.from_dicts(cams)
    kf = viterbi_filter(kp2d)
    pts = kf[..., :2].copy()
    pts[kf[..., 2] < 0.5] = np.nan
    flat = np.ascontiguousarray(pts.transpose(2, 0, 1, 3, 4).reshape(C, -1, 2))
    p3 = g.triangulate_ransac(flat, min_cams=2)[0].reshape(A, F, J, 3)
    P2 = np.ascontiguousarray(pts.transpose(0, 2, 1, 3, 4))
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    return g, P2, p3, cons, weak, bench.LIFT_ARGS


def marker_problems(key):
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    z = np.load(os.path.join(ROOT, "tests", "golden", "optim_problems.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in z.files if k.startswith(key)})
    ss, sl, slw, rp, nd = z["tri"]
    args = dict(scale_smooth=ss, scale_length=sl, scale_length_weak=slw, reproj_error_threshold=rp,
                n_deriv_smooth=int(nd))
    return (CameraGroup.from_dicts(synth.make_cameras(8)), np.stack([z[k + "_p2"] for k in keys]),
            np.stack([z[k + "_init"] for k in keys]), z["cons"], z["weak"], args)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--solvers", default="trf,lm")
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--fb", type=int, default=0, help="most frames per workgroup (MQ_TUNE_OPTIM_TRF_FB)")
    ap.add_argument("--cases", default="config4,s7f24,s8f24,s9f24")
    ap.add_argument("--lib", default="", help="another build of libmq_hip.so (e.g. the -DTRF_PROFILE one in lib_prof/)")
    a = ap.parse_args()
    import torch
    from mqhip import _lib
    if a.lib:
        _lib.load(os.path.join(ROOT, a.lib))
    from mqhip.optim import optim_points_batch
    if a.chunk:
        _lib.check(_lib.Context.get(0).lib.mq_set_tuning(22, a.chunk), "chunk")
    if a.fb:
        _lib.check(_lib.Context.get(0).lib.mq_set_tuning(25, a.fb), "fb")
    for case in a.cases.split(","):
        g, P2, I3, cons, weak, args = config4_problem() if case == "config4" else marker_problems(case)
        for solver in a.solvers.split(","):
            ts = []
            for _ in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                p3, jl, st, _ = optim_points_batch(g, P2, I3, cons, weak, solver=solver, return_stats=True, **args)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            print(json.dumps({"case": case, "solver": solver, "B": int(P2.shape[0]), "F": int(P2.shape[2]),
                              "ms_median": round(float(np.median(ts[1:])) * 1e3, 2),
                              "ms_all": [round(t * 1e3, 2) for t in ts],
                              "iterations": st[:, 2].astype(int).tolist(), "status": st[:, 3].astype(int).tolist(),
                              "nfev": st[:, 4].astype(int).tolist(), "lsmr_total": st[:, 6].astype(int).tolist(),
                              "lsmr_longest": st[:, 7].astype(int).tolist()}), flush=True)


if __name__ == "__main__":
    main()
