"""BASELINE config 4: the step-4 lift of a 300-frame clip (8 views x 4 individuals x 17 joints)
on one MI355X, stage by stage, with the oracle (CPU port of the reference path) timed beside it.

Stages: a15 Viterbi over all 544 chains, a12 initial DLT, a13 RANSAC
(min_cams 2), a16 optim_points for all 4 animals (batched LM), a14 mean reprojection error.
CPU timings run the oracle on a bounded sample and scale to the full clip (the sample is named
in the output).  Writes one JSON object to stdout.

python tools/bench_lift.py [--frames 300] [--cpu-optim-frames 300] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--animals", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-optim-frames", type=int, default=300)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--lib", default=None, help="libmq_hip.so to load instead of the in-tree build (A/B runs)")
    args = ap.parse_args()
    import numpy as np
    import torch
    if args.lib:  # after torch: torch's HIP runtime must be the one the library binds to
        from mqhip import _lib
        _lib.load(args.lib)
    from mqhip import synth
    from mqhip.geometry import CameraGroup, viterbi_filter
    from mqhip.optim import optim_points_batch

    A, F, C, J = args.animals, args.frames, 8, 17
    cams = synth.make_cameras(C)
    skel = synth.make_skeletons(A, F)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=0.1)         # (A,F,C,J,3)
    g = CameraGroup.from_dicts(cams)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    tri = dict(scale_smooth=3, scale_length=5, scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3)

    def timed(fn, reps=args.reps):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3, out

    res = {"config": f"BASELINE config 4: {F} frames x {C} views x {A} individuals x {J} joints", "gpu_ms": {},
           "note": "GPU times include host<->device copies of the stage inputs/outputs (numpy in, numpy out)"}
    ms, kp_f = timed(lambda: viterbi_filter(kp2d))
    res["gpu_ms"]["viterbi_a15"] = ms
    pts = kp_f[..., :2].copy()                                           # (A,F,C,J,2)
    pts[kp_f[..., 2] < 0.5] = np.nan
    flat = np.ascontiguousarray(pts.transpose(2, 0, 1, 3, 4).reshape(C, -1, 2))
    ms, init = timed(lambda: g.triangulate(flat))
    res["gpu_ms"]["dlt_a12"] = ms
    ms, rr = timed(lambda: g.triangulate_ransac(flat, min_cams=2))
    res["gpu_ms"]["ransac_a13"] = ms
    P2 = np.ascontiguousarray(pts.transpose(0, 2, 1, 3, 4))              # (A,C,F,J,2)
    I3 = init.reshape(A, F, J, 3)
    ms, (p3, jl, stats, ssf) = timed(lambda: optim_points_batch(g, P2, I3, cons, weak, return_stats=True, **tri))
    res["gpu_ms"]["optim_points_a16"] = ms
    res["optim_stats"] = {"cost0": stats[:, 0].tolist(), "cost": stats[:, 1].tolist(),
                          "lm_iters": stats[:, 2].tolist(), "status": stats[:, 3].tolist()}
    ms, err = timed(lambda: g.reprojection_error(np.ascontiguousarray(p3.reshape(-1, 3)), flat, mean=True))
    res["gpu_ms"]["reproj_a14"] = ms
    res["gpu_ms"]["total"] = sum(res["gpu_ms"].values())
    res["individuals_frames_per_s_lift"] = A * F / (res["gpu_ms"]["total"] * 1e-3)

    if not args.no_cpu:
        from oracle.geometry import CameraGroupOracle, optim_points
        from oracle.viterbi import STEP4_FILTER_CONFIG, filter_pose_viterbi
        o = CameraGroupOracle(cams)
        cpu = {}
        # Viterbi: 8 of the 544 chains (full length), scaled
        t0 = time.perf_counter()
        for a in range(1):
            for c in range(8):
                x = np.ascontiguousarray(kp2d[a, :, c][:, :, None, :]).copy()
                filter_pose_viterbi(STEP4_FILTER_CONFIG, x[:, :1].copy(), [])
        cpu["viterbi_a15"] = (time.perf_counter() - t0) * (A * C * J) / 8
        sample = 200
        t0 = time.perf_counter()
        o.triangulate(flat[:, :sample])
        cpu["dlt_a12"] = (time.perf_counter() - t0) * flat.shape[1] / sample
        t0 = time.perf_counter()
        o.triangulate_ransac(flat[:, :sample], min_cams=2)
        cpu["ransac_a13"] = (time.perf_counter() - t0) * flat.shape[1] / sample
        Fo = min(args.cpu_optim_frames, F)
        t0 = time.perf_counter()
        ro = optim_points(o, P2[0][:, :Fo], I3[0][:Fo], cons, weak, return_result=True, **tri)
        cpu["optim_points_a16"] = (time.perf_counter() - t0) * A * F / Fo
        t0 = time.perf_counter()
        o.reprojection_error(p3.reshape(-1, 3)[:2000], flat[:, :2000], mean=True)
        cpu["reproj_a14"] = (time.perf_counter() - t0) * flat.shape[1] / 2000
        cpu["total"] = sum(cpu.values())
        res["cpu_s"] = cpu
        res["cpu_baseline"] = {"value": A * F / cpu["total"], "unit": "individuals×frames/s", "cores": 1,
                               "kind": "port",
                               "sample": f"oracle (numpy/scipy, 1 thread): Viterbi 8/{A*C*J} chains, DLT/RANSAC "
                                         f"{sample} of {flat.shape[1]} points, reprojection 2000 points, "
                                         f"optim_points animal 0 over {Fo} frames; each scaled to the clip"}
        res["speedup_vs_cpu_port"] = cpu["total"] / (res["gpu_ms"]["total"] * 1e-3)
        if Fo == F:
            d = np.linalg.norm(p3[0] - ro[0], axis=-1)
            res["optim_vs_scipy_mm"] = {"median": float(np.median(d)), "p99": float(np.percentile(d, 99)),
                                        "gpu_cost": float(stats[0, 1]), "scipy_cost": float(ro[2].cost)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
