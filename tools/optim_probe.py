"""optim_points on the BASELINE config-4 clip (300 frames x 8 views x 4 animals) for several caps on
the PCG iterations per LM step (MQ_TUNE_OPTIM_PCG_ITERS): wall time, LM steps, final cost against
scipy's TRF cost on the same problem, and the distance to scipy's solution (the parity criteria of
tests/test_gpu_optim.py: median <= 1 mm, p99 <= 5 mm, cost <= scipy + 0.1 %)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd")]


def main():
    import numpy as np
    import torch
    import bench
    from mqhip import _lib, synth
    from mqhip.geometry import CameraGroup
    from mqhip.optim import optim_points_batch
    from oracle.geometry import CameraGroupOracle, optim_points
    cams, kp2d = bench.lift_inputs()
    A, F, C, J, _ = kp2d.shape
    pts = kp2d[..., :2].copy()
    pts[kp2d[..., 2] < 0.5] = np.nan
    P2 = np.ascontiguousarray(pts.transpose(0, 2, 1, 3, 4))
    o = CameraGroupOracle(cams)
    init = o.triangulate(np.ascontiguousarray(pts.transpose(2, 0, 1, 3, 4).reshape(C, -1, 2))).reshape(A, F, J, 3)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    ref = [optim_points(o, P2[a], init[a], cons, weak, return_result=True, **bench.LIFT_ARGS) for a in range(2)]
    print("scipy costs", [r[2].cost for r in ref], flush=True)
    g = CameraGroup.from_dicts(cams)
    ctx = _lib.Context.get(0)
    out = {}
    for cap in (6, 10, 15, 20, 30, 40):
        _lib.check(ctx.lib.mq_set_tuning(4, cap), "tuning")
        optim_points_batch(g, P2, init, cons, weak, **bench.LIFT_ARGS)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p3, jl, stats, ssf = optim_points_batch(g, P2, init, cons, weak, return_stats=True, **bench.LIFT_ARGS)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        dev = [np.linalg.norm(p3[a] - ref[a][0], axis=-1) for a in range(2)]
        costs = []
        for a in range(2):
            r = o._error_fun_triangulation(np.hstack([p3[a].ravel(), jl[a]]), P2[a], np.array(cons), np.array(weak),
                                           ref[a][3], 5, 2, 3, "soft_l1", 2)
            costs.append(0.5 * float(np.sum(r ** 2)))
        out[cap] = {"ms": round(ms, 2), "lm": stats[:, 2].tolist(), "cost_ratio": [c / r[2].cost for c, r in zip(costs, ref)],
                    "median_mm": [float(np.median(d)) for d in dev], "p99_mm": [float(np.percentile(d, 99)) for d in dev]}
        print(cap, out[cap], flush=True)
    _lib.check(ctx.lib.mq_set_tuning(4, 20), "tuning")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
