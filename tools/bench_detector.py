"""Time the Swin-S Mask R-CNN detector (BASELINE config 5's detection stage) on one MI355X:
8 views of 1536x2048 uint8 frames per step, eager and hipGraph-replayed.

python tools/bench_detector.py [--views 8] [--steps 10] [--graph] [--lib PATH]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--lib", default=None, help="time this build of libmq_hip.so (A/B of two builds)")
    args = ap.parse_args()
    if args.lib:
        import torch  # noqa: F401  (torch's HIP runtime first, as everywhere else)
        from mqhip import _lib
        _lib.load(os.path.abspath(args.lib))
    import numpy as np
    import torch
    from mqhip.detector import SwinDetectorHip
    from oracle import swin_det as sd  # seeded random weights only (no oracle arithmetic is timed)
    w = sd.make_weights(sd.SWIN_S, seed=0)
    det = SwinDetectorHip(w, device=0)
    rng = np.random.default_rng(0)
    fr = torch.from_numpy(rng.integers(0, 256, (args.views, 1536, 2048, 3), dtype=np.uint8)).cuda()
    for _ in range(2):
        out = det.forward(fr)
    torch.cuda.synchronize()
    res = {"views": args.views, "frame": "1536x2048 uint8 BGR", "model": "Swin-S Mask R-CNN bbox (random weights)"}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = det.forward(fr)
    torch.cuda.synchronize()
    res["eager_ms_per_frame"] = (time.perf_counter() - t0) * 1e3 / args.steps
    res["detections"] = [int(c) for c in out[2].cpu()]
    # A/B in this process: the FPN / RPN 3x3 convolutions through im2col + GEMM instead of implicit GEMMs
    det.implicit_conv = False
    for _ in range(2):
        ref = det.forward(fr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ref = det.forward(fr)
    torch.cuda.synchronize()
    res["eager_ms_per_frame_im2col_convs"] = (time.perf_counter() - t0) * 1e3 / args.steps
    res["im2col_path_same_counts"] = bool(torch.equal(ref[2], out[2]))
    det.implicit_conv = True
    if args.graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            det.forward(fr)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            gout = det.forward(fr)
        g.replay()
        torch.cuda.synchronize()
        same = all(torch.equal(a, b) for a, b in zip(gout, out))
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.replay()
        torch.cuda.synchronize()
        res["graph_ms_per_frame"] = (time.perf_counter() - t0) * 1e3 / args.steps
        res["graph_equals_eager"] = bool(same)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
