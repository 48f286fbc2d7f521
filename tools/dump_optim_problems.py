"""Dump the optim_points problems of the marker-scene oracle chain (tests/parity3d.py) to an npz, so the
scipy-TRF restatement can be studied and pinned on the CPU: per (scene, individual) the oracle chain's
score-thresholded 2D (C, F, J, 2), its DLT initialisation (F, J, 3), scipy's ftol-1e-3 answer with its
nfev / njev, and the converged (ftol 1e-10) answer.  Needs a GPU (the fp32 ViT-H of the oracle chain).

python tools/dump_optim_problems.py OUT.npz [--scenes 7:24,8:24,9:24,7:8]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--scenes", default="7:24,8:24,9:24,7:8", help="seed:frames,...")
    a = ap.parse_args()
    import parity3d
    from oracle.geometry import CameraGroupOracle, optim_points
    config = parity3d.load_config()
    tri = config["triangulation"]
    weights = parity3d.make_weights()
    out = {}
    for item in a.scenes.split(","):
        seed, nf = (int(v) for v in item.split(":"))
        t0 = time.time()
        scene = parity3d.make_scene(n_frames=nf, seed=seed)
        ora = parity3d.oracle_chain(scene, weights, config)
        o = CameraGroupOracle(scene["cams"])
        from src.pipeline.step4_aniposefiltering import BODYPARTS, load_constraints
        cons = np.array(load_constraints(config, BODYPARTS))
        weak = np.array(load_constraints(config, BODYPARTS, "constraints_weak"))
        for ind, (p2, targs, cost, _) in sorted(ora["problems"].items()):
            C, F, J, _ = p2.shape
            init = o.triangulate(p2.reshape(C, -1, 2)).reshape(F, J, 3)
            args = dict(scale_smooth=tri["scale_smooth"], scale_length=tri["scale_length"],
                        scale_length_weak=tri["scale_length_weak"],
                        reproj_error_threshold=tri["reproj_error_threshold"], n_deriv_smooth=tri["n_deriv_smooth"])
            p3, jl, res, ssf, x0 = optim_points(o, p2, init, cons, weak, ftol=1e-3, return_result=True, **args)
            key = f"s{seed}f{nf}a{ind}"
            out[key + "_p2"] = p2
            out[key + "_init"] = init
            out[key + "_x"] = res.x
            out[key + "_stats"] = np.array([res.nfev, res.njev, res.cost, res.status, ssf])
            out[key + "_tight"] = ora["kp3d_tight"][ind]
            print(key, "nfev", res.nfev, "njev", res.njev, "cost", res.cost, flush=True)
        print(f"scene {seed}:{nf} done in {time.time() - t0:.1f} s", flush=True)
    out["cons"] = cons
    out["weak"] = weak
    out["tri"] = np.array([tri["scale_smooth"], tri["scale_length"], tri["scale_length_weak"],
                           tri["reproj_error_threshold"], tri["n_deriv_smooth"]], dtype=np.float64)
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
