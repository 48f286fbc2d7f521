"""Time the ViTPose-H flip-test forward at the bench shape (32 crops = 64 images) under the
same-result routing knobs, in one process, eager and graph-replayed, and check that every variant
gives bit-identical heatmaps.  Usage: python tools/vit_probe.py [--iters N] [--knob KEY=V1,V2,...]
(KEY one of include/mq_hip.h MQ_TUNE_*; the first value is the reference and is restored at exit).

Round 2 used it to measure a two-lane forward (image halves on two streams, fork / join by events,
bit-identical): 20.1 ms against 16.9 ms for one lane (profiles/r02z_vit_lanes_probe.log), so the
lanes were removed again."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--knob", default="20=1,0", help="KEY=V1,V2,... (default: head-major vs row-major QKV)")
    ap.add_argument("--crops", type=int, default=32)
    ap.add_argument("--lib", default=None, help="another build of libmq_hip.so (A/B across builds)")
    args = ap.parse_args()
    import torch
    from mqhip import _lib
    if args.lib:
        # an older build may lack newer entry points: bind only the ones it exports
        import ctypes
        probe = ctypes.CDLL(os.path.abspath(args.lib))
        for name in list(_lib._SIGS):
            if not hasattr(probe, name):
                del _lib._SIGS[name]
        _lib.ABI_VERSION = probe.mq_abi_version()  # an A/B build may predate the current ABI
        _lib.load(os.path.abspath(args.lib))  # first load wins: every later load() returns this build
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_H, make_random_weights

    dev = torch.device("cuda", 0)
    w = make_random_weights(VIT_H, seed=0, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    crops = torch.randn((args.crops, 3, 256, 192), generator=g, device=dev)
    models = {gr: VitPoseHip(VIT_H, w, device=0, graph=gr) for gr in (False, True)}
    del w
    lib = models[False].lib
    s = _lib.stream_ptr(dev)
    key, vals = args.knob.split("=")
    key = int(key)
    vals = [int(v) for v in vals.split(",")]
    ref = None
    for rnd in range(args.rounds):
        for gr, model in models.items():
            for ln in vals:
                _lib.check(lib.mq_set_tuning(key, ln), "knob")
                hm = torch.empty((args.crops, 17, 64, 48), device=dev)
                for _ in range(2):
                    _lib.check(lib.mq_vitpose_forward(model.handle, _lib.ptr(crops), args.crops, 1, _lib.ptr(hm), s),
                               "forward")
                torch.cuda.synchronize()
                if ref is None:
                    ref = hm.clone()
                same = bool(torch.equal(hm, ref))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    _lib.check(lib.mq_vitpose_forward(model.handle, _lib.ptr(crops), args.crops, 1, _lib.ptr(hm), s),
                               "forward")
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.iters
                print(f"r={rnd} {'graph' if gr else 'eager'} knob {key}={ln}: {ms:.3f} ms per forward "
                      f"({args.crops / (ms * 1e-3) / 8:.1f} ind x frames/s at 8 views)  bit-identical={same}",
                      flush=True)
    _lib.check(lib.mq_set_tuning(key, vals[0]), "knob")


if __name__ == "__main__":
    main()
