#!/usr/bin/env python3
"""Headline benchmark: individuals x frames / s of 3D pose (8-view ViTPose-H + triangulate).

Workload (BASELINE.json configs[1]), per GPU per step:
one synchronized frame = 8 views (uint8 BGR 1536x2048) x 4 individuals
-> 32 top-down crops (UDP warp, bf16 ViTPose-H 256x192, flip test = 64 forwards)
-> UDP/DARK decode -> score-threshold -> omnidir undistort + DLT of 4 x 17 joints.
Everything in the step runs on the GPU from inputs already resident in HBM.

Multi-GPU (torch.distributed over RCCL, one process per GPU): frames are sharded
across ranks (weak scaling, per-GPU work fixed).  Per-frame triangulation needs
only that frame's 8 views, so the step has no collective; the one real exchange,
the all-gather of every rank's per-view 2D keypoints that feeds the clip-level
Viterbi / optim_points stage, runs once inside the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "macaque-3d-pose-estimation_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "individuals×frames/sec 3D pose (8-view ViTPose-h + triangulate), 1/2/4/8 GPU"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
N_VIEWS, N_ANIMALS, N_JOINTS = 8, 4, 17
IMG_H, IMG_W = 1536, 2048
KP_THR, TRI_THR = 0.30, 0.5   # step1_proc2d.py:68 (KP_THR), config_tmpl.toml:96 (score_threshold)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-step", type=int, default=1)
    ap.add_argument("--model", default="huge", choices=["huge", "base", "tiny"])
    ap.add_argument("--resident-frames", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-lift", action="store_true", help="skip the config-4 lift timing (extra keys)")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 detector + pose timing (extra keys)")
    ap.add_argument("--graph", action="store_true", help="replay the forward as a hipGraph (disables live timing)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the multi-frame-batch and overlapped-H2D measurements (extra keys)")
    return ap.parse_args()


def log(msg):
    """Progress to stderr (the harness takes a silent run for a hung one)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_share():
    """Threads for the CPU baseline: the CPU share this process is given.  On the GPU pool nproc and
    os.cpu_count() report the whole machine while the job's share is OMP_NUM_THREADS (16 per GPU);
    oversubscribing a CPU quota would time the scheduler, not the restatement."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_info():
    """Host cores this process may use (what `nproc` reports) and the CPU model (`lscpu`)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(), "model": model}


def _median_time(fn, reps):
    """Median wall time of `reps` calls after a warm-up, and the last call's result."""
    import numpy as np
    fn()  # warm-up
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def cpu_baseline(cams_np, n_crops_sample=8, reps=5):
    """The build's CPU restatement of the reference path (oracle/, "port"), timed on this host per
    BASELINE.md's plan: torch fp32 with one thread per available core, median of `reps` runs after
    a warm-up.  Config 2 (the headline): ViT-H flip-test forward + UDP decode of `n_crops_sample` of
    the frame's 32 crops (scaled by 32 / sample) + the frame's omnidir DLT.  Config 1: ViT-B on its
    4 crops + decode + DLT, whole.  Config 4: the step-4 lift of the 300-frame clip (batched
    Viterbi and RANSAC restatements, scipy optim_points on one animal scaled x4, reprojection)."""
    import numpy as np
    import torch
    from mqhip import synth
    from mqhip.weights import CONFIGS, make_random_weights
    from oracle.decode import decode_batch
    from oracle.geometry import CameraGroupOracle
    from oracle.vitpose import forward_flip_test
    info = cpu_info()
    threads = cpu_share()
    torch.set_num_threads(threads)
    log(f"cpu baseline: {threads} threads (nproc {info['nproc']}, os.cpu_count {info['os_cpu_count']})")
    g = CameraGroupOracle(cams_np)

    def frame_pass(cfg, n_crops, n_views):
        w = make_random_weights(cfg, seed=0, device="cpu")
        x = torch.randn((n_crops, 3, 256, 192), generator=torch.Generator().manual_seed(0))
        c = np.tile(np.array([[800, 600]], np.float32), (n_crops, 1))
        s = np.tile(np.array([[300, 400]], np.float32), (n_crops, 1))
        skel = synth.make_skeletons(N_ANIMALS, 1)
        kp2d = synth.make_kp2d(cams_np, skel)
        pts = kp2d[:, 0].transpose(1, 0, 2, 3)[:n_views].reshape(n_views, -1, 3)
        p = pts[..., :2].copy()
        p[pts[..., 2] < TRI_THR] = np.nan
        gv = g.subset(range(n_views))

        def run():
            with torch.no_grad():
                hm, _, _ = forward_flip_test(x, w, cfg)
            decode_batch(hm.numpy(), c, s)
            return hm

        t_vit, hm = _median_time(run, reps)
        t_tri, _ = _median_time(lambda: gv.triangulate(p), reps)
        log(f"cpu baseline: ViT-{cfg.name} {n_crops} crops {t_vit:.3f} s (median of {reps})")
        sample[cfg.name] = (w, x, hm)
        return t_vit, t_tri

    sample = {}
    crops = N_VIEWS * N_ANIMALS
    t2, tri2 = frame_pass(CONFIGS["huge"], n_crops_sample, N_VIEWS)
    t_frame2 = t2 * crops / n_crops_sample + tri2
    t1, tri1 = frame_pass(CONFIGS["base"], 4, 4)
    parity = parity_check(*sample["huge"], CONFIGS["huge"], crops)
    lift = lift_cpu(cams_np)
    log(f"cpu baseline: config-4 lift {lift['total_s']:.1f} s")
    det = detector_cpu(reps=min(reps, 3))
    idc = id_cpu(reps=min(reps, 3))
    return {"value": round(N_ANIMALS / t_frame2, 5), "unit": "individuals×frames/s", "cores": threads,
            "kind": "port", "nproc": info["nproc"], "os_cpu_count": info["os_cpu_count"], "cpu_model": info["model"],
            "statistic": f"median of {reps} after 1 warm-up",
            "sample": f"config 2: oracle ViT-H fp32 flip-test forward + UDP decode of {n_crops_sample} of the frame's "
                      f"{crops} crops (x{crops / n_crops_sample:g}) + omnidir DLT of the frame's "
                      f"{N_ANIMALS}x{N_JOINTS} joints; torch CPU {threads} threads",
            "seconds_per_frame": round(t_frame2, 4),
            "config1": {"seconds_per_frame": round(t1 + tri1, 4), "individuals_frames_per_s": round(1.0 / (t1 + tri1), 4),
                        "sample": "ViT-B fp32 flip-test forward + decode of 4 crops (4 views x 1 individual) + DLT"},
            "config4_lift": lift,
            "config5_detector": det, "config5_id": idc, "parity_check": parity}


def parity_check(w, x, hm_cpu, cfg, batch):
    """The CPU sample's fp32 oracle heatmaps against the GPU path at the bench's batch size: a
    `batch`-crop forward (bf16 MFMA, flip test) whose first crops are the CPU sample's crops, with the
    same weights.  Tolerance per crop: max|dH| <= 2e-2 * max|H| (tests/test_gpu_pose.py)."""
    import torch
    from mqhip.pose import VitPoseHip
    dev = torch.device("cuda", 0)
    model = VitPoseHip(cfg, {k: v.to(dev) for k, v in w.items()}, device=0, graph=False)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    xb = torch.randn((batch, 3, 256, 192), generator=g, device=dev)
    xb[:x.shape[0]] = x.to(dev)
    got = model.forward(xb, flip_test=True)[:x.shape[0]].float().cpu()
    del model
    torch.cuda.empty_cache()
    ref = hm_cpu.float()
    rel = [float((got[i] - ref[i]).abs().max() / ref[i].abs().max()) for i in range(ref.shape[0])]
    am_equal = float((got.flatten(2).argmax(-1) == ref.flatten(2).argmax(-1)).float().mean())
    return {"crops_checked": ref.shape[0], "gpu_batch": batch, "max_rel_err": round(max(rel), 5), "tol": 2e-2,
            "pass": max(rel) <= 2e-2, "argmax_agreement": round(am_equal, 4),
            "what": "fp32 CPU oracle heatmaps (the cpu_baseline sample) vs the GPU flip-test forward of a "
                    f"{batch}-crop batch holding those crops, same weights"}


def parity_3d(device, slice_frames=8):
    """End-to-end 2D -> 3D parity of the headline path (tests/parity3d.py, the same
    harness as tests/test_gpu_parity3d.py): the HIP chain (step 1 crop -> ViTPose-H bf16 -> decode -> KP_THR
    / EMA, step 3 kp2d, step 4 Viterbi -> DLT [-> optim_points]) against the oracle chain (oracle crop -> fp32
    ViT-H on the GPU, TF32 off -> oracle decode / smoother / Viterbi / DLT -> scipy optim_points) from the same
    frames and weights: config 2 (one 8-view x 4-individual frame) and a ``slice_frames``-frame clip slice.
    The scene is a marker scene (mqhip/synth.py: two-tone joint markers and matched-filter ViTPose-H weights,
    so every joint has one smooth, flip-consistent heatmap peak as with a trained checkpoint).
    Figures per case: clear fraction, argmax agreement on clear joints, max keypoint deviation on clear
    Taylor-regime joints, kp3d deviation (mm) on all-clear points and on every point."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import parity3d
    out = {"scene": "marker scene (mqhip/synth.py): two-tone joint markers in the synthetic frames and matched-"
                    "filter ViTPose-H weights (one flip-consistent heatmap peak per joint); identical frames and "
                    "weights in both chains",
           "tolerances": {"argmax": "bit-exact on clear joints (top-2 margin > 5e-2 max|H|)",
                          "keypoint_px": parity3d.KP_TOL_PX,
                          "kp3d_dlt_mm_all_clear": {"median": parity3d.KP3D_DLT_MM_MEDIAN,
                                                    "p99": parity3d.KP3D_DLT_MM_P99},
                          "kp3d_optim_mm_all_clear": f"within max(scipy ftol 1e-3 vs 1e-10 band, "
                                                     f"{parity3d.KP3D_OPTIM_MM_MEDIAN} mm median / "
                                                     f"{parity3d.KP3D_OPTIM_MM_P99} mm p99)"}}
    w = parity3d.make_weights(device=torch_device(device))
    seed = 7
    for name, nf in (("config2_frame", 1), ("clip_slice", slice_frames)):
        t0 = time.perf_counter()
        fig, _, _ = parity3d.run(n_frames=nf, seed=seed, weights=w)
        fig = {k: (round(v, 6) if isinstance(v, float) else v) for k, v in fig.items()}
        fig["frames"] = nf
        fig["seed"] = seed
        # the stated absolute bounds of this scene (tests/parity3d.py) and whether the figures meet them
        dlt_p99, final_p99 = parity3d.every_point_p99_bounds(nf, seed)
        bounds = {"kp3d_dlt_mm_every_point_p99": dlt_p99, "kp3d_mm_every_point_p99": final_p99}
        if fig.get("optim_points"):
            bounds["kp3d_optim_mm_all_clear_p99"] = parity3d.optim_e2e_p99_bound(nf, seed)
        fig["bounds_mm"] = bounds
        fig["bounds_met"] = all(isinstance(fig.get(k), (int, float)) and fig[k] <= v for k, v in bounds.items())
        fig["seconds"] = round(time.perf_counter() - t0, 1)
        out[name] = fig
        log(f"parity 3D {name}: {fig}")
    del w
    return out


def torch_device(i):
    import torch
    return torch.device("cuda", i)


def detector_cpu(reps=3):
    """Config-5 detection stage on the CPU port (oracle/swin_det.py, torch fp32): resize +
    normalise + Swin-S + FPN + RPN head convolutions of ONE 1536x2048 view, x8 views.  The RPN
    selection, RoIAlign and box head are excluded from the sample (the oracle's RoIAlign is a
    Python loop that would dominate and say nothing about the reference)."""
    import numpy as np
    import torch
    import torch.nn.functional as F
    from oracle import swin_det as sd
    w = sd.make_weights(sd.SWIN_S, seed=0)
    img = np.random.default_rng(0).integers(0, 256, (IMG_H, IMG_W, 3), dtype=np.uint8)

    def run():
        with torch.no_grad():
            x, _, _ = sd.preprocess(img)
            p = sd.fpn_forward(sd.swin_forward(x, w), w)
            for f in p:
                h = F.relu(F.conv2d(f, w["rpn_head.rpn_conv.weight"], w["rpn_head.rpn_conv.bias"], padding=1))
                F.conv2d(h, w["rpn_head.rpn_cls.weight"], w["rpn_head.rpn_cls.bias"])
                F.conv2d(h, w["rpn_head.rpn_reg.weight"], w["rpn_head.rpn_reg.bias"])

    t, _ = _median_time(run, reps)
    log(f"cpu baseline: detector backbone + FPN + RPN head, 1 view {t:.2f} s (median of {reps})")
    return {"seconds_per_frame": round(t * N_VIEWS, 3), "seconds_per_view": round(t, 3),
            "sample": "oracle Swin-S + FPN + RPN head convolutions of 1 of the frame's 8 views (x8); RPN selection, "
                      "RoIAlign and the box head excluded", "statistic": f"median of {reps} after 1 warm-up"}


def id_cpu(reps=3):
    """Config-5 ID stage on the CPU port (oracle/resnet_id.py, torch fp32): preprocessing + ResNet-152 of 4 of
    the frame's 32 tracked boxes, x8."""
    import numpy as np
    import torch
    from mqhip.resnet_id import make_random_weights
    from oracle import resnet_id as orid
    sd = make_random_weights(152, seed=0)
    img = np.random.default_rng(1).integers(0, 256, (IMG_H, IMG_W, 3), dtype=np.uint8)
    patches = [img[200:700, 100 + 300 * a:400 + 300 * a] for a in range(4)]

    def run():
        with torch.no_grad():
            orid.forward(sd, torch.stack([orid.preprocess(p) for p in patches]))

    t, _ = _median_time(run, reps)
    log(f"cpu baseline: ID classifier, 4 boxes {t:.2f} s (median of {reps})")
    return {"seconds_per_frame": round(t * 8, 3), "sample": "oracle preprocessing + ResNet-152 of 4 of the frame's "
            "32 tracked boxes (x8)", "statistic": f"median of {reps} after 1 warm-up"}


def lift_inputs(A=4, F=300, C=8, seed=2):
    import numpy as np
    from mqhip import synth
    cams = synth.make_cameras(C)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(A, F, seed=seed), noise_px=2.0, drop=0.1)
    return cams, kp2d


LIFT_ARGS = dict(scale_smooth=3, scale_length=5, scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3)


def _viterbi_joint(args):
    """one joint series of filter_pose_viterbi (filter_pose.py:171-176): the pool task of the reference"""
    from oracle.viterbi import viterbi_path
    jix, pts, scs, n_back, thres = args
    p, sc = viterbi_path(pts, scs, n_back, thres)
    return jix, p, sc


def lift_cpu(cams_np):
    """Config-4 step-4 lift on the CPU restatement (oracle/), shaped like the reference's own CPU path
    (VERDICT r4 item 7): the Viterbi filter per individual x camera through a spawn pool of
    max(min(cores // 2, joints), 1) workers over the 17 joint series (filter_pose.py:151-186, called per
    individual x camera by step4:142-167), RANSAC batched in numpy on one core, scipy least_squares
    optim_points on every individual in turn (step4:219-331), reprojection.  Wall seconds per stage and the
    cores each used."""
    import multiprocessing as mproc
    import numpy as np
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle, optim_points
    from oracle.viterbi import STEP4_FILTER_CONFIG, wrap_points
    cams, kp2d = lift_inputs()
    A, F, C, J, _ = kp2d.shape
    o = CameraGroupOracle(cams)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    fc = STEP4_FILTER_CONFIG["filter"]
    n_proc = max(min(cpu_share() // 2, J), 1)
    t = {}
    t0 = time.perf_counter()
    kt = np.array(kp2d, dtype=np.float64, copy=True).transpose((1, 3, 0, 4, 2))   # (F, J, A, 3, C) as step 4
    kf = np.zeros(kt.shape)
    ctx = mproc.get_context("spawn")
    for a in range(A):
        for c in range(C):
            pts = kt[:, :, a, :2, c].copy()
            scs = kt[:, :, a, 2, c].copy()
            pts[scs < fc["score_threshold"]] = np.nan
            # closed and joined, not terminated (a `with` block SIGTERMs the workers, which profilers log as aborts)
            pool = ctx.Pool(n_proc)
            try:
                res = list(pool.imap_unordered(_viterbi_joint, [(j, pts[:, j, None], scs[:, j, None], fc["n_back"],
                                                                 fc["offset_threshold"]) for j in range(J)]))
            finally:
                pool.close()
                pool.join()
            pf = np.full((F, J, 2), np.nan)
            sf = np.empty((F, J))
            for j, p, sc in res:
                pf[:, j], sf[:, j] = p, sc
            kf[:, :, a, :, c] = np.squeeze(wrap_points(pf, sf))
    t["viterbi_a15"] = time.perf_counter() - t0
    log(f"cpu lift: viterbi {t['viterbi_a15']:.2f} s ({A * C} pools of {n_proc} spawn workers)")
    kf = kf.transpose((2, 4, 0, 1, 3))                                        # (A, C, F, J, 3)
    pts = kf[..., :2].copy()
    pts[kf[..., 2] < 0.5] = np.nan
    flat = np.ascontiguousarray(pts.transpose(1, 0, 2, 3, 4).reshape(C, -1, 2))
    t0 = time.perf_counter()
    p3, _, _, _ = o.triangulate_ransac_batched(flat, min_cams=2)
    t["ransac_a13"] = time.perf_counter() - t0
    log(f"cpu lift: ransac {t['ransac_a13']:.2f} s")
    init = p3.reshape(A, F, J, 3)
    t0 = time.perf_counter()
    res = [optim_points(o, pts[a], init[a], cons, weak, **LIFT_ARGS) for a in range(A)]
    t["optim_points_a16"] = time.perf_counter() - t0
    log(f"cpu lift: optim_points {t['optim_points_a16']:.2f} s for {A} individuals")
    t0 = time.perf_counter()
    o.reprojection_error(np.ascontiguousarray(np.stack([r[0] for r in res]).reshape(-1, 3)), flat, mean=True)
    t["reproj_a14"] = time.perf_counter() - t0
    tot = sum(t.values())
    return {"seconds": {k: round(v, 4) for k, v in t.items()}, "total_s": round(tot, 4),
            "individuals_frames_per_s": round(A * F / tot, 3),
            "cores": {"viterbi_a15": n_proc, "ransac_a13": 1, "optim_points_a16": 1, "reproj_a14": 1},
            "kind": "port",
            "sample": f"{F} frames x {C} views x {A} individuals x {J} joints, whole: the Viterbi filter per "
                      f"individual x camera through a spawn pool of {n_proc} workers over the joint series "
                      f"(the reference's filter_pose_viterbi shape), batched numpy RANSAC, scipy least_squares "
                      f"optim_points on every individual in turn, reprojection"}


def lift_gpu(device, reps=3, solver="trf"):
    """Config-4 step-4 lift on the GPU (HIP kernels through the drop-in API, numpy in / out):
    Viterbi over the 544 chains, RANSAC (min_cams 2) over 20,400 points, batched optim_points over
    the 4 animals (``solver``: "trf", scipy's algorithm and the default, or "lm"), mean reprojection error.
    Median wall ms per stage over `reps` runs."""
    import numpy as np
    import torch
    from mqhip import synth
    from mqhip.geometry import CameraGroup, viterbi_filter
    from mqhip.optim import optim_points_batch
    cams, kp2d = lift_inputs()
    A, F, C, J, _ = kp2d.shape
    g = CameraGroup.from_dicts(cams, device=device)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    times = {k: [] for k in ("viterbi_a15", "ransac_a13", "optim_points_a16", "reproj_a14")}
    stats = None
    for _ in range(reps + 1):
        def tick():
            torch.cuda.synchronize(device)
            return time.perf_counter()
        t0 = tick()
        kf = viterbi_filter(kp2d, device=device)
        t1 = tick()
        pts = kf[..., :2].copy()
        pts[kf[..., 2] < 0.5] = np.nan
        flat = np.ascontiguousarray(pts.transpose(2, 0, 1, 3, 4).reshape(C, -1, 2))
        t2 = tick()
        p3 = g.triangulate_ransac(flat, min_cams=2)[0]
        t3 = tick()
        P2 = np.ascontiguousarray(pts.transpose(0, 2, 1, 3, 4))
        t4 = tick()
        res, jl, stats, _ = optim_points_batch(g, P2, p3.reshape(A, F, J, 3), cons, weak, return_stats=True,
                                               solver=solver, **LIFT_ARGS)
        t5 = tick()
        g.reprojection_error(np.ascontiguousarray(res.reshape(-1, 3)), flat, mean=True)
        t6 = tick()
        for k, v in (("viterbi_a15", t1 - t0), ("ransac_a13", t3 - t2), ("optim_points_a16", t5 - t4),
                     ("reproj_a14", t6 - t5)):
            times[k].append(v)
        log(f"gpu lift ({solver}): viterbi {1e3 * (t1 - t0):.1f} ms, ransac {1e3 * (t3 - t2):.1f} ms, "
            f"optim {1e3 * (t5 - t4):.1f} ms, reproj {1e3 * (t6 - t5):.1f} ms")
    med = {k: float(np.median(v[1:])) * 1e3 for k, v in times.items()}
    tot = sum(med.values())
    import hashlib
    digest = hashlib.sha256(np.ascontiguousarray(res).tobytes() + np.ascontiguousarray(jl).tobytes()).hexdigest()[:16]
    return {"gpu_ms": {k: round(v, 3) for k, v in med.items()}, "total_ms": round(tot, 3),
            "optim_result_sha256_16": digest,
            "individuals_frames_per_s": round(A * F / (tot * 1e-3), 2),
            "optim_solver": solver, "optim_iterations": stats[:, 2].astype(int).tolist(),
            "optim_status": stats[:, 3].astype(int).tolist(),
            **({"optim_nfev": stats[:, 4].astype(int).tolist(), "optim_lsmr_iterations": stats[:, 6].astype(int).tolist()}
               if solver == "trf" else {}),
            "statistic": f"median of {reps} after 1 warm-up",
            "workload": f"BASELINE config 4: {F} frames x {C} views x {A} individuals x {J} joints, ransac + optim",
            "note": "wall time per stage through the drop-in numpy API (host<->device copies included)"}


def config5_gpu(device, pose_model, frames, cams_dev, steps=5):
    """BASELINE config 5 on one GPU, as one hipGraph per frame (mqhip.frame_graph.FramePoseGraph): the
    Swin-S Mask R-CNN detector on all 8 views (1536x2048) -> the 4 best detections of every view as static
    crop-box slots (mq_det_topk_boxes, step 1's truncation + margin expansion) -> ViTPose flip test + UDP
    decode on those 32 crops -> score mask -> omnidir DLT, captured once and replayed per frame; then
    (host) one BoT-SORT update per view on the frame's detections and the ResNet-152 ID classifier on the
    tracked boxes.  With random weights the detector scores sit near 0.5, so the box selection and the
    trackers run with thresholds 0 (every detection eligible).  `steps` frames timed back to back after
    warm-ups (frames resident in HBM; each replay first copies its frame into the graph's input)."""
    import numpy as np
    import torch
    from mqhip.detector import SwinDetectorHip, make_random_weights
    from mqhip.frame_graph import FramePoseGraph
    from mqhip.resnet_id import ResNetIdHip, make_random_weights as id_weights, patch_bounds
    from mqhip.tracker import BOTSORT_CFG, BotSort
    det = SwinDetectorHip(make_random_weights(seed=0), device=device)
    idm = ResNetIdHip(id_weights(152, seed=0), depth=152, device=device)
    trk_cfg = dict(BOTSORT_CFG, track_high_thresh=0.0, track_low_thresh=0.0, new_track_thresh=0.0)
    trackers = [BotSort(**trk_cfg) for _ in range(N_VIEWS)]
    dev = torch.device("cuda", device)
    cfg = pose_model.cfg
    fg = FramePoseGraph(det, pose_model, cams_dev, n_views=N_VIEWS, height=IMG_H, width=IMG_W, k=N_ANIMALS,
                        det_score_thr=0.0, tri_score_thr=TRI_THR)

    def track_and_id(fr):
        dboxes, dscores, _ = fg.det_out
        hb = dboxes[:, :N_ANIMALS].double().cpu().numpy()
        hs = dscores[:, :N_ANIMALS].double().cpu().numpy()
        rows = []
        for v in range(N_VIEWS):
            for r in trackers[v].update(np.hstack([hb[v], hs[v][:, None], np.zeros((N_ANIMALS, 1))]), None):
                pb = patch_bounds((IMG_H, IMG_W), r[:4])
                if pb is not None:
                    rows.append((v, pb[2], pb[0], pb[3], pb[1]))
        if rows:
            x, _ = idm.preprocess(fr, rows)
            idm.forward(x)
        return len(rows)

    def timed(fn):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        out = [fn(i) for i in range(steps)]
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) * 1e3 / steps, out

    fr_of = lambda i: frames[i % frames.shape[0]]  # noqa: E731
    for i in range(2):
        fg.eager(fr_of(i))
    det_ms, _ = timed(lambda i: det.forward(fr_of(i)))
    id_rows = [(v, 100 + 300 * a, 200, 400 + 300 * a, 700) for v in range(N_VIEWS) for a in range(N_ANIMALS)]
    id_ms, _ = timed(lambda i: idm.forward(idm.preprocess(fr_of(i), id_rows)[0]))
    eager_ms, _ = timed(lambda i: fg.eager(fr_of(i)))
    fg.capture()
    for i in range(2):
        fg.run(fr_of(i))
    graph_ms, _ = timed(lambda i: fg.run(fr_of(i)))
    ms, nid = timed(lambda i: (fg.run(fr_of(i)), track_and_id(fr_of(i)))[1])
    n_valid = int(fg.valid.sum().item())
    log(f"config 5: detector {det_ms:.2f} ms, ID (32 boxes) {id_ms:.2f} ms, slice eager {eager_ms:.2f} ms, "
        f"graph replay {graph_ms:.2f} ms, with tracker + ID {ms:.2f} ms / frame")
    return {"workload": "BASELINE config 5 per GPU: Swin-S Mask R-CNN on 8 views 1536x2048 -> 4 best detections "
                        "per view (static top-k, step 1 box expansion) -> ViTPose-%s flip test + UDP decode (32 "
                        "crops) -> omnidir DLT, one hipGraph per frame; BoT-SORT per view (host) -> ResNet-152 ID "
                        "on the tracked boxes" % cfg.name,
            "ms_per_frame": round(graph_ms, 3),
            "slice": "BASELINE config 5 as defined: detector + crops + ViTPose-%s flip test + decode + DLT, "
                     "hipGraph replay per frame" % cfg.name,
            "individuals_frames_per_s": round(N_ANIMALS / (graph_ms * 1e-3), 2),
            "ms_per_frame_eager": round(eager_ms, 3),
            "ms_per_frame_with_tracker_and_id": round(ms, 3),
            "individuals_frames_per_s_with_tracker_and_id": round(N_ANIMALS / (ms * 1e-3), 2),
            "detector_ms_per_frame": round(det_ms, 3),
            "id_classifier_ms_per_frame": round(id_ms, 3), "id_classifier_boxes_timed": len(id_rows),
            "id_boxes_per_frame": round(sum(nid) / steps, 1),
            "valid_box_slots": n_valid, "frames_timed": steps,
            "data": "random detector, pose and ID weights, random frames (the detector returns 100 boxes per view; "
                    "box selection and trackers at thresholds 0)"}


def clip_lift(kp, cams_np, device, clips=1, rank=0, world=1, config=None, camera_group=None, return_kp3d=False):
    """The step-4 lift (Viterbi 2D filter, DLT triangulation, optim_points, reprojection errors; the
    default config_tmpl.toml path) of the keypoints every rank produced in the timed region, gathered in
    frame order: kp (F, C, A, J, 3) -> wall seconds (BASELINE config 3's last stage).  Each rank's frames are
    its own synthetic sequence, so the gathered frames are `clips` clips (one per rank) of A individuals; as in
    step4_aniposefiltering.proc on a sharded run, rank r lifts the individuals i = r (mod world) of the
    clips x A, batched in one solve (every rank holds the gathered keypoints; the caller takes the max).
    config / camera_group / return_kp3d: the step-4 config (default config_tmpl.toml), the camera group (default
    the HIP CameraGroup on `device`) and the rank's kp3d in the result -- for the CPU test of the exchange and
    split (tests/test_multiproc_gloo.py, with oracle stand-ins)."""
    import numpy as np
    import torch
    from mqhip import io as mqio
    from mqhip.geometry import CameraGroup
    from src.pipeline.step4_aniposefiltering import CONFIG_TMPL, filter_2d, reconstruct_3d
    Ft, C, A = kp.shape[:3]
    kp = kp.reshape((clips, Ft // clips) + kp.shape[1:])                         # (clips, F, C, A, J, 3)
    kp2d = np.ascontiguousarray(kp.transpose(0, 3, 1, 2, 4, 5).reshape((clips * A, Ft // clips) + kp.shape[2:3] + kp.shape[4:])).astype(np.float64)   # (clips*A, F, C, J, 3)
    kp2d = np.ascontiguousarray(kp2d[rank::world])
    config = mqio.load_toml(CONFIG_TMPL) if config is None else config
    cg = CameraGroup.from_dicts(cams_np, device=device) if camera_group is None else camera_group
    on_gpu = device is not None and torch.cuda.is_available()
    if on_gpu:
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    kf = filter_2d(kp2d, device=device)
    t1 = time.perf_counter()
    kp3d, _, _, _ = reconstruct_3d(kf, cg, config)
    if on_gpu:
        torch.cuda.synchronize(device)
    t2 = time.perf_counter()
    A2, F = kp2d.shape[:2]
    extra = {"kp3d": kp3d} if return_kp3d else {}
    return {**extra, "frames": int(F), "clips": int(clips), "individuals": int(A * clips), "individuals_per_rank": int(A2),
            "ms": round((t2 - t0) * 1e3, 3),
            "viterbi_ms": round((t1 - t0) * 1e3, 3), "triangulate_optim_ms": round((t2 - t1) * 1e3, 3),
            "finite_3d_fraction": round(float(np.isfinite(kp3d).mean()), 4),
            "what": "step 4 (config_tmpl.toml: Viterbi filter, DLT, optim_points, reprojection errors) on the 2D "
                    "keypoints of every frame of the timed region, gathered from all ranks (one clip per rank); "
                    "the individuals split over the ranks (i = rank mod world), ms = the slowest rank"}


class Pipeline:
    """One step of the headline workload on HBM-resident inputs: `fps` synchronized frames x 8 views x 4
    individuals -> crop -> ViT flip test -> decode -> score mask -> omnidir DLT per frame, all on the
    current stream."""

    def __init__(self, model, cams_dev, fps, boxes_all):
        import torch
        self.model, self.cams, self.fps = model, cams_dev, fps
        dev = model.dev
        J = model.cfg.n_joints
        self.n = n = fps * N_VIEWS * N_ANIMALS
        self.boxes_all = boxes_all                               # (frames, C*A, 4) view-major, on the device
        self.box_frame = torch.arange(n, device=dev, dtype=torch.int32) // N_ANIMALS  # image within the step
        self.crops = torch.empty((n, 3, 256, 192), device=dev)
        self.center = torch.empty((n, 2), device=dev)
        self.scale = torch.empty((n, 2), device=dev)
        self.hm = torch.empty((n, J, 64, 48), device=dev)
        self.kp = torch.empty((n, J, 2), device=dev, dtype=torch.float64)
        self.score = torch.empty((n, J), device=dev)
        self.am = torch.empty((n, J), device=dev, dtype=torch.int32)
        self.p3d = torch.empty((fps, N_ANIMALS * J, 3), device=dev, dtype=torch.float64)
        self.crop_done = None

    def step(self, frames, f0, log=None):
        """frames: (>= fps, C, H, W, 3) u8 device tensor holding this step's frames from index 0; f0: the
        index of the first of them in boxes_all; log: optional (n, J, 3) f32 slot for the keypoints."""
        import torch
        from mqhip import _lib
        m = self.model
        lib, ctx, s = m.lib, m.ctx, _lib.stream_ptr(m.dev)
        J = m.cfg.n_joints
        bx = self.boxes_all[f0:f0 + self.fps].reshape(-1, 4)
        _lib.check(lib.mq_crop_udp(ctx.handle, _lib.ptr(frames), IMG_H * IMG_W * 3, IMG_H, IMG_W, _lib.ptr(bx),
                                   _lib.ptr(self.box_frame), self.n, _lib.ptr(self.crops), _lib.ptr(self.center),
                                   _lib.ptr(self.scale), s), "crop")
        if self.crop_done is not None:
            self.crop_done.record()
        _lib.check(lib.mq_vitpose_forward(m.handle, _lib.ptr(self.crops), self.n, 1, _lib.ptr(self.hm), s), "forward")
        _lib.check(lib.mq_decode_udp(ctx.handle, _lib.ptr(self.hm), self.n, J, 64, 48, _lib.ptr(self.center),
                                     _lib.ptr(self.scale), _lib.ptr(self.kp), _lib.ptr(self.score), _lib.ptr(self.am),
                                     None, s), "decode")
        # step1 (KP_THR) + step4 (score_threshold) masking, then (C, A*J, 2) per frame
        bad = (self.score < TRI_THR).unsqueeze(-1)
        pts = torch.where(bad, torch.full_like(self.kp, float("nan")), self.kp)
        pts = pts.view(self.fps, N_VIEWS, N_ANIMALS * J, 2)
        for f in range(self.fps):
            pf = pts[f].contiguous()
            _lib.check(lib.mq_triangulate_dlt(ctx.handle, _lib.ptr(self.cams), N_VIEWS, _lib.ptr(pf),
                                              N_ANIMALS * J, 1, _lib.ptr(self.p3d[f]), s), "dlt")
        if log is not None:
            log[:, :, :2] = self.kp.float()
            log[:, :, 2] = self.score


def multi_frame_batches(model, cams_dev, boxes_all, frames, counts=(2, 4), steps=20, warmup=3):
    """BASELINE config 3's per-GPU batch choice: the same step with `fps` frames per launch sequence
    (M = fps x 64 x 192 GEMM rows), ms per step and individuals x frames / s per setting."""
    import torch
    out = {}
    P = frames.shape[0]
    for fps in counts:
        pipe = Pipeline(model, cams_dev, fps, boxes_all)
        slots = P // fps
        for i in range(warmup):
            pipe.step(frames[(i % slots) * fps:], (i % slots) * fps)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            pipe.step(frames[(i % slots) * fps:], (i % slots) * fps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out[f"fps{fps}"] = {"ms_per_step": round(dt * 1e3, 3), "frames_per_step": fps,
                            "gemm_rows": fps * N_VIEWS * N_ANIMALS * 2 * model.cfg.tokens,
                            "individuals_frames_per_s": round(fps * N_ANIMALS / dt, 3)}
        log(f"frames per step {fps}: {dt * 1e3:.2f} ms per step, {fps * N_ANIMALS / dt:.1f} individuals x frames/s")
        del pipe
    return out


def with_h2d_upload(model, cams_dev, boxes_all, steps=30, warmup=3):
    """The headline step with each frame's 8 views uploaded from pinned host memory (8 x 9.4 MB) on a
    second stream into a double-buffered device slot, overlapped with the previous step's compute; the
    crop of step i waits for its upload, the upload of frame i+1 waits for step i-1's crop (which read
    that slot).  Also the upload alone (ms and GB/s)."""
    import torch
    dev = model.dev
    P = boxes_all.shape[0]
    host = torch.randint(0, 256, (2, N_VIEWS, IMG_H, IMG_W, 3), dtype=torch.uint8).pin_memory()
    slots = torch.empty((2, 1, N_VIEWS, IMG_H, IMG_W, 3), dtype=torch.uint8, device=dev)
    cs = torch.cuda.Stream(device=dev)
    up_done = [torch.cuda.Event() for _ in range(2)]
    crop_done = [torch.cuda.Event() for _ in range(2)]
    pipe = Pipeline(model, cams_dev, 1, boxes_all)
    main = torch.cuda.current_stream(dev)

    def upload(i):
        with torch.cuda.stream(cs):
            if i >= 2:
                cs.wait_event(crop_done[i % 2])
            slots[i % 2, 0].copy_(host[i % 2], non_blocking=True)
            up_done[i % 2].record(cs)

    def run(n):
        upload(0)
        for i in range(n):
            if i + 1 < n:
                upload(i + 1)
            main.wait_event(up_done[i % 2])
            pipe.crop_done = crop_done[i % 2]
            pipe.step(slots[i % 2], i % P)
        torch.cuda.synchronize(dev)

    run(warmup)
    t0 = time.perf_counter()
    run(steps)
    dt = (time.perf_counter() - t0) / steps
    # the upload alone
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    for i in range(steps):
        slots[i % 2, 0].copy_(host[i % 2], non_blocking=True)
    torch.cuda.synchronize(dev)
    up = (time.perf_counter() - t1) / steps
    nbytes = N_VIEWS * IMG_H * IMG_W * 3
    log(f"with overlapped H2D: {dt * 1e3:.2f} ms per step; upload alone {up * 1e3:.2f} ms ({nbytes / up / 1e9:.1f} GB/s)")
    return {"value": round(N_ANIMALS / dt, 3), "ms_per_step": round(dt * 1e3, 3),
            "h2d_ms_per_frame": round(up * 1e3, 3), "h2d_gb_per_s": round(nbytes / up / 1e9, 2),
            "bytes_per_frame": nbytes, "steps": steps,
            "what": "config 2 step with the frame's 8 views uploaded from pinned host memory on a second stream, "
                    "double-buffered and overlapped with the previous step (the headline keeps frames resident)"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the multi-rank path on a one-GPU box (never set by the driver): MQ_BENCH_SHARE_GPU=1
    # puts every rank on device LOCAL_RANK % device_count and MQ_BENCH_BACKEND=gloo exchanges the
    # keypoints and timings through host tensors (RCCL refuses two ranks on one GPU).
    backend = os.environ.get("MQ_BENCH_BACKEND", "nccl")
    if os.environ.get("MQ_BENCH_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
    # MQ_BENCH_DIST=1 (never set by the driver): the process group, the keypoint all-gather and the
    # max-over-ranks timing also at world 1 -- an RCCL rehearsal of the N > 1 code on a one-GPU box
    dist_on = world > 1 or os.environ.get("MQ_BENCH_DIST") == "1"
    if dist_on:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    xdev = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live

    from mqhip import _lib, synth
    from mqhip.geometry import CameraGroup
    from mqhip.pose import VitPoseHip
    from mqhip.shard import gather_keypoints
    from mqhip.weights import CONFIGS, make_random_weights

    cfg = CONFIGS[args.model]
    # seeded random weights; the 1x1 head is scaled so heatmap peaks score above the thresholds and the
    # clip lift has points to triangulate (synth.confident_head; same FLOPs and launches)
    weights = synth.confident_head(make_random_weights(cfg, seed=0, device=dev))
    model = VitPoseHip(cfg, weights, device=local, graph=args.graph)
    del weights
    lib = model.lib
    extras = rank == 0 and world == 1 and not args.no_extras

    # ---------------- synthetic, HBM-resident inputs (this rank's frames)
    cams_np = synth.make_cameras(N_VIEWS)
    group = CameraGroup.from_dicts(cams_np, device=local)
    cams_dev = group.cams_tensor()
    FPS = args.frames_per_step
    NF = args.resident_frames * max(FPS, 4 if extras else 1)          # resident frames (4 per frame slot)
    skel = synth.make_skeletons(N_ANIMALS, NF, seed=2 + rank)
    kp2d = synth.make_kp2d(cams_np, skel, seed=3 + rank)            # (A, F, C, J, 3)
    boxes = []
    for f in range(NF):
        tight = synth.boxes_from_kp2d(kp2d[:, f].transpose(1, 0, 2, 3))  # (C, A, 4)
        boxes.append(synth.expand_boxes(tight.reshape(-1, 4)))
    boxes = torch.from_numpy(np.stack(boxes)).to(dev)                  # (NF, C*A, 4) view-major
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    frames = torch.randint(0, 256, (NF, N_VIEWS, IMG_H, IMG_W, 3), generator=g, device=dev, dtype=torch.uint8)
    pipe = Pipeline(model, cams_dev, FPS, boxes)
    n = pipe.n
    slots = NF // FPS
    kp_log = torch.empty((args.steps, n, cfg.n_joints, 3), device=dev, dtype=torch.float32)

    def step(i, log_slot=None):
        f0 = (i % slots) * FPS
        pipe.step(frames[f0:f0 + FPS], f0, None if log_slot is None else kp_log[log_slot])

    log(f"model ready; {args.warmup} warm-up + {args.steps} timed steps")
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    timing = not args.graph
    if timing:
        _lib.check(lib.mq_vitpose_timing(model.handle, 1), "timing")
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, log_slot=i)
    # (this rank's compute ends here: one host synchronisation, so the exchange below is timed on its own)
    torch.cuda.synchronize(dev)
    t_steps = time.perf_counter()
    # the one exchange step: every rank's per-view 2D keypoints, in frame order (mqhip.shard)
    per_frame = kp_log.view(args.steps, FPS, N_VIEWS, N_ANIMALS, cfg.n_joints, 3).flatten(0, 1)
    if dist_on:
        gathered = gather_keypoints(per_frame.to(xdev), world * args.steps * FPS, world)
    else:
        gathered = per_frame
    torch.cuda.synchronize(dev)
    t_gather = time.perf_counter()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if timing:
        _lib.check(lib.mq_vitpose_timing(model.handle, 0), "timing")
    # per rank: the timed steps (crop -> ViT -> decode -> DLT) and the keypoint all-gather alone, so a multi-GPU run
    # separates compute from exchange
    rank_times = [[(t_steps - t0) * 1e3, (t_gather - t_steps) * 1e3]]
    if dist_on:
        t = torch.tensor([dt], device=xdev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        mine = torch.tensor(rank_times[0], device=xdev, dtype=torch.float64)
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        rank_times = [p.tolist() for p in parts]

    roof = None
    if timing:
        avg_ms, cnt, fl = C.c_double(), C.c_int(), C.c_int64()
        _lib.check(lib.mq_vitpose_timing_result(model.handle, C.byref(avg_ms), C.byref(cnt), C.byref(fl)),
                   "timing_result")
        achieved = fl.value / (avg_ms.value * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_fc1_gemm.json")
        if os.path.exists(pmc):
            try:
                with open(pmc) as f:
                    traffic = json.load(f).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
                "traffic_source": "profiles/pmc_fc1_gemm.json: rocprofv3 --pmc 2*FETCH_SIZE + WRITE_SIZE per launch "
                                  "(gfx950 corrections; Infinity-Cache hits included); algorithmic 170,414,080 B",
                "kernel": "%s (FFN fc1, M=%d N=%d K=%d)" % (
                    "gemm_pp_kernel<EPI_GELU_BF16>" if lib.mq_get_tuning(12) == 1 else "gemm256_kernel<EPI_GELU_BF16>",
                    2 * n * cfg.tokens, cfg.ffn, cfg.embed_dims),
                "flops_per_launch": fl.value, "avg_launch_ms": round(avg_ms.value, 5), "launches": cnt.value,
                "launches_timed": "fc1 of layers 7, 15, 23, 31 in every timed step (HIP event pairs on the forward's "
                                  "stream; each pair idles the GPU ~4 us on either side of its launch)"}

    frames_done = world * args.steps * FPS
    value = frames_done * N_ANIMALS / dt
    crops_per_s = frames_done * N_VIEWS * N_ANIMALS / dt
    model_tflops = crops_per_s * 2 * cfg.flops_per_forward() / 1e12
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "individuals×frames/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic: seeded random ViTPose weights (1x1 head scaled so peaks pass the score thresholds), "
                "random uint8 1536x2048 frames, boxes from projected synthetic skeletons, 8 omnidir cameras with "
                "the reference's intrinsics",
        "config": {"workload": "BASELINE config 2 per GPU: 1 frame x 8 views x 4 individuals = 32 crops, "
                               "ViTPose-%s 256x192 flip test (64 forwards), UDP decode, omnidir DLT" % cfg.name,
                   "frames_per_step_per_gpu": FPS, "crops_per_step_per_gpu": n,
                   "parallelism": "frame-shard x%d (RCCL all-gather of 2D keypoints)" % world},
        "individuals_views_frames_per_s": round(value * N_VIEWS, 3),
        "crops_per_s": round(crops_per_s, 3),
        "end_to_end_model_tflops": round(model_tflops, 2),
        "end_to_end_mfma_frac": round(model_tflops / (world * PEAK_BF16_TFLOPS), 4),
        "roofline": roof,
        "ranks": [{"rank": r, "steps_ms": round(a, 3), "ms_per_step": round(a / args.steps, 3),
                   "gather_ms": round(b, 3)} for r, (a, b) in enumerate(rank_times)],
        "gather_ms_max": round(max(b for _, b in rank_times), 3),
        "gather_bytes_per_rank": int(args.steps * FPS * N_VIEWS * N_ANIMALS * cfg.n_joints * 3 * 4),
    }
    log(f"timed region {dt:.3f} s")
    if not args.no_lift:
        # BASELINE config 3's last stage: the clip lift of every frame the ranks just processed, its individuals
        # split over the ranks as in run_demo's sharded step 4; the slowest rank's time
        cl = clip_lift(gathered.cpu().numpy(), cams_np, local, clips=world, rank=rank, world=world)
        if dist_on:
            t = torch.tensor([cl["ms"]], device=xdev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cl["ms"] = round(float(t.item()), 3)
        if rank == 0:
            cl["value_with_lift"] = round(frames_done * N_ANIMALS / (dt + cl["ms"] * 1e-3), 3)
            result["clip_lift"] = cl
            log(f"clip lift of {cl['frames']} gathered frames: {cl['ms']:.1f} ms")
    if extras:
        # steady state: the same step back to back for >= 3 s (the driver's utilisation sampler needs more than
        # the short timed region to see the GPU busy; the chip's clock under sustained load is what it reports)
        torch.cuda.synchronize(dev)
        n_s, t_s = 0, time.perf_counter()
        while time.perf_counter() - t_s < 3.0:
            for _ in range(20):
                step(n_s)
                n_s += 1
            torch.cuda.synchronize(dev)
        t_s = time.perf_counter() - t_s
        result["sustained"] = {"steps": n_s, "seconds": round(t_s, 3), "ms_per_step": round(t_s / n_s * 1e3, 3),
                               "value": round(n_s * FPS * N_ANIMALS / t_s, 3),
                               "what": "the timed step repeated back to back for >= 3 s after the timed region "
                                       "(steady-state clock); not the headline"}
        log(f"sustained: {n_s} steps in {t_s:.2f} s")
        result["multi_frame_batches"] = multi_frame_batches(model, cams_dev, boxes, frames)
        result["with_h2d"] = with_h2d_upload(model, cams_dev, boxes)
        result["value_with_h2d"] = result["with_h2d"]["value"]
    if rank == 0 and world == 1 and not args.no_lift:
        result["lift_config4"] = lift_gpu(local)
        result["lift_config4_lm"] = lift_gpu(local, solver="lm")
    if rank == 0 and world == 1 and not args.no_config5:
        result["config5"] = config5_gpu(local, model, frames[:, :N_VIEWS] if frames.dim() == 5 else frames, cams_dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["parity_3d_mm"] = parity_3d(local)
        result["cpu_baseline"] = cpu_baseline(cams_np)
        if "lift_config4" in result:
            result["lift_config4"]["speedup_vs_cpu_port"] = round(
                result["cpu_baseline"]["config4_lift"]["total_s"] * 1e3 / result["lift_config4"]["total_ms"], 1)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
