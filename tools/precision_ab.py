"""Precision A/B of the ViT residual updates in ONE process and on identical inputs:
MQ_TUNE_VIT_RESID_F32 = 1 (proj / fc2 add their f32 accumulators to the residual stream in the GEMM epilogue,
rounds 1-3) against 0 (proj / fc2 round their branch outputs to bf16, the LayerNorm passes add them; round 4).
  (a) seeded random ViT-H weights (full-scale branches: every residual update at its natural size) on 32 seeded
      crops against the fp32 oracle forward (oracle/vitpose.py on the GPU, TF32 off): heatmap max|dH| / max|H| per
      crop, argmax agreement on all joints and on the unclear ones (top-2 margin <= 5e-2 of max|H|);
  (b) the marker scenes of tests/parity3d.py (branches scaled 1/32): the HIP chain's parity figures against ONE
      oracle chain per scene.
python tools/precision_ab.py [--scenes 1:7,8:7] [--crops 32]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"), os.path.join(ROOT, "tests")]
KEY = 23  # MQ_TUNE_VIT_RESID_F32


def forward_ab(lib, n):
    import torch
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_H, make_random_weights
    from oracle.vitpose import forward_flip_test
    w = make_random_weights(VIT_H, seed=0, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.randn((n, 3, 256, 192), generator=g, device="cuda")
    prev = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.no_grad():
            ref = forward_flip_test(x, w, VIT_H)[0].float()
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = prev
    flat = ref.flatten(2)
    top2 = flat.topk(2, dim=-1).values
    unclear = (top2[..., 0] - top2[..., 1]) / flat.abs().amax(-1) <= 5e-2
    out, hms = {}, {}
    for knob in (1, 0):
        assert lib.mq_set_tuning(KEY, knob) == 0
        model = VitPoseHip(VIT_H, w, device=0, graph=False)
        got = model.forward(x, flip_test=True).float()
        del model
        rel = ((got - ref).abs().flatten(1).amax(1) / ref.abs().flatten(1).amax(1)).cpu().numpy()
        am = got.flatten(2).argmax(-1) == flat.argmax(-1)
        hms[knob] = got
        out["resid_f32_epilogue" if knob else "bf16_branch_outputs"] = {
            "max_rel_err": round(float(rel.max()), 6), "median_rel_err": round(float(np.median(rel)), 6),
            "argmax_agreement": round(float(am.float().mean()), 5),
            "argmax_agreement_unclear": round(float(am[unclear].float().mean()), 5),
            "unclear_joints": int(unclear.sum())}
    d = (hms[0] - hms[1]).abs().flatten(1).amax(1) / ref.abs().flatten(1).amax(1)
    out["between_paths_max_rel"] = round(float(d.max()), 6)
    assert lib.mq_set_tuning(KEY, 0) == 0
    return out


def scenes_ab(lib, scenes):
    import parity3d
    w = parity3d.make_weights()
    config = parity3d.load_config()
    keys = ("clear_fraction", "argmax_equal_on_clear", "kp_max_abs_px", "kp_p99_abs_px_clear", "kp_max_abs_px_clear",
            "n_clear_over_tol", "kp3d_dlt_mm_all_clear_median", "kp3d_dlt_mm_all_clear_p99",
            "kp3d_dlt_mm_every_point_median", "kp3d_dlt_mm_every_point_p99", "kp3d_mm_every_point_median",
            "kp3d_mm_every_point_p99", "kp3d_optim_mm_all_clear_median", "kp3d_optim_mm_all_clear_p99")
    out = {}
    for item in scenes.split(","):
        nf, seed = (int(v) for v in item.split(":"))
        scene = parity3d.make_scene(n_frames=nf, seed=seed)
        ora = parity3d.oracle_chain(scene, w, config)
        res = {}
        for knob in (1, 0):
            assert lib.mq_set_tuning(KEY, knob) == 0
            hip = parity3d.hip_chain(scene, w, config)
            # unclear joints too: argmax agreement over every (crop, joint)
            am_all = np.concatenate([(h[2] == o[2]).ravel() for h, o in zip(hip["per_frame"], ora["per_frame"])])
            fig = parity3d.compare(scene, hip, ora, config["triangulation"]["score_threshold"])
            r = {k: fig[k] for k in keys if k in fig}
            r["argmax_equal_all_joints"] = float(am_all.mean())
            res["resid_f32_epilogue" if knob else "bf16_branch_outputs"] = r
        out[f"{nf}f_seed{seed}"] = res
        assert lib.mq_set_tuning(KEY, 0) == 0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="1:7,8:7")
    ap.add_argument("--crops", type=int, default=32)
    a = ap.parse_args()
    from mqhip import _lib
    lib = _lib.Context.get(0).lib
    print(json.dumps({"random_weights_full_scale": forward_ab(lib, a.crops)}), flush=True)
    if a.scenes:
        print(json.dumps({"marker_scenes": scenes_ab(lib, a.scenes)}), flush=True)


if __name__ == "__main__":
    main()
