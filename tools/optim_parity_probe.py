"""GPU optim_points vs scipy on the 2D keypoints of the marker-scene oracle chain (tests/parity3d.py): per
individual the cost of the GPU solution under the oracle's objective / scipy's cost at ftol 1e-3, the distance
to scipy's converged (ftol 1e-10) solution, and the solver's iterations / stop status, for several conjugate-
gradient caps (MQ_TUNE_OPTIM_PCG_ITERS), stop rules and GPU ftol values, on one or more marker scenes.
python tools/optim_parity_probe.py [--frames 24] [--seeds 7,8,9] [--pcg 40] [--stop 2] [--ftol 1e-3,5e-4]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--pcg", default="20,40")
    ap.add_argument("--ftol", default="1e-3")
    ap.add_argument("--stop", default="0,2", help="MQ_TUNE_OPTIM_STOP values (key 21)")
    ap.add_argument("--seeds", default="7", help="marker-scene seeds (tests/parity3d.make_scene)")
    a = ap.parse_args()
    import parity3d
    config = parity3d.load_config()
    weights = parity3d.make_weights()
    for seed in [int(x) for x in a.seeds.split(",")]:
        scene = parity3d.make_scene(n_frames=a.frames, seed=seed)
        ora = parity3d.oracle_chain(scene, weights, config)
        probe_scene(a, parity3d, config, scene, ora, seed)


def probe_scene(a, parity3d, config, scene, ora, seed):
    from mqhip import _lib
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch
    from src.pipeline.step4_aniposefiltering import BODYPARTS, load_constraints
    tri = config["triangulation"]
    cons, weak = load_constraints(config, BODYPARTS), load_constraints(config, BODYPARTS, "constraints_weak")
    cg = CameraGroup.from_dicts(scene["cams"])
    kp = ora["kp2d_f"].transpose((2, 4, 0, 1, 3))
    A, C, F, J, _ = kp.shape
    run = sorted(ora["problems"])
    pts = np.stack([ora["problems"][i][0] for i in run])                  # (B, C, F, J, 2) oracle inputs
    init = np.stack([np.asarray(cg.triangulate(pts[b].reshape(C, -1, 2))).reshape(F, J, 3) for b in range(len(run))])
    lib = _lib.Context.get(0).lib
    import time
    for pcg, stop, ftol in [(int(p), int(st), float(f)) for p in a.pcg.split(",") for st in a.stop.split(",")
                            for f in a.ftol.split(",")]:
        _lib.check(lib.mq_set_tuning(4, pcg), "pcg")
        _lib.check(lib.mq_set_tuning(21, stop), "stop")
        t0 = time.perf_counter()
        p3, jl, stats, _ = optim_points_batch(
            cg, pts, init, cons, weak, scale_smooth=tri["scale_smooth"], scale_length=tri["scale_length"],
            scale_length_weak=tri["scale_length_weak"], reproj_error_threshold=tri["reproj_error_threshold"],
            n_deriv_smooth=tri["n_deriv_smooth"], ftol=ftol, return_stats=True)
        ms = (time.perf_counter() - t0) * 1e3
        rows = []
        for b, i in enumerate(run):
            p2, targs, cost, _ = ora["problems"][i]
            r = ora["cgroup"]._error_fun_triangulation(np.hstack([p3[b].ravel(), jl[b]]), p2, *targs)
            d = np.linalg.norm(p3[b] - ora["kp3d_tight"][i], axis=-1)
            d = d[np.isfinite(d)]
            st = np.asarray(stats).reshape(len(run), -1)[b]
            rows.append({"ind": i, "cost_ratio": round(0.5 * float(r @ r) / cost, 5),
                         "to_converged_mm_p50_p99": [round(float(np.median(d)), 3), round(float(np.percentile(d, 99)), 2)],
                         "iters": int(st[2]), "status": int(st[3])})
        allp = np.concatenate([np.linalg.norm(p3[b] - ora["kp3d_tight"][i], axis=-1).ravel() for b, i in enumerate(run)])
        allp = allp[np.isfinite(allp)]
        print(json.dumps({"seed": seed, "pcg": pcg, "stop": stop, "ftol": ftol, "ms": round(ms, 1),
                          "cost_ratio_max": max(r["cost_ratio"] for r in rows),
                          "to_converged_mm_p50_p99": [round(float(np.median(allp)), 3),
                                                      round(float(np.percentile(allp, 99)), 2)],
                          "rows": rows}), flush=True)
    _lib.check(lib.mq_set_tuning(4, 40), "pcg")      # the ABI-6 defaults
    _lib.check(lib.mq_set_tuning(21, 6), "stop")
    band = np.linalg.norm(ora["kp3d"] - ora["kp3d_tight"], axis=-1)
    print(json.dumps({"seed": seed, "scipy_1e-3_to_converged_mm_p50_p99": [round(float(np.nanmedian(band)), 3),
                                                                          round(float(np.nanpercentile(band, 99)), 2)]}))


if __name__ == "__main__":
    main()
