"""Time the ResNet-152 ID classifier forward (random weights) on n boxes, in one process, under the
same-result GEMM routing knob MQ_TUNE_GEMM_TILE64 (64x64 tiles for GEMMs that cannot fill the CUs with
128x128 ones) on and off and the implicit-GEMM convolutions on and off, and check that every variant
gives identical probabilities.

python tools/id_probe.py [n_boxes ...]      (default: 13 32 -- a config-5 frame's tracked boxes, 32)
python tools/id_probe.py --lib PATH [n ...]  (that build only, default routing: one line per size with the
                                             forward time and a digest of the probabilities, for A/B of two
                                             builds in two processes)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    import torch
    from mqhip import _lib
    from mqhip.resnet_id import ResNetIdHip, make_random_weights
    argv = sys.argv[1:]
    quick = None
    if argv[:1] == ["--lib"]:
        quick = argv[1]
        argv = argv[2:]
        _lib.load(os.path.abspath(quick))
    sizes = [int(a) for a in argv] or [13, 32]
    m = ResNetIdHip(make_random_weights(152, seed=0), depth=152)
    lib = m.ctx.lib
    if quick:
        import hashlib
        for n in sizes:
            g = torch.Generator(device="cuda").manual_seed(n)
            x = torch.randn((n, 224, 224, 3), device="cuda", generator=g).to(torch.bfloat16)
            for _ in range(3):
                _, probs = m.forward(x)
            torch.cuda.synchronize()
            digest = hashlib.sha1(probs.cpu().numpy().tobytes()).hexdigest()[:16]
            for rnd in range(3):
                t0 = time.perf_counter()
                for _ in range(10):
                    m.forward(x)
                torch.cuda.synchronize()
                print(f"{os.path.basename(os.path.dirname(quick))} r={rnd} ResNet-152 ID forward, {n} boxes: "
                      f"{(time.perf_counter() - t0) * 100:.3f} ms  probs sha1 {digest}", flush=True)
        return
    old = lib.mq_get_tuning(19)
    try:
        for n in sizes:
            x = torch.randn((n, 224, 224, 3), device="cuda").to(torch.bfloat16)
            ref = None
            for rnd in range(3):
                for t64, implicit in ((1, True), (1, False), (0, True)):
                    m.implicit_conv = implicit
                    _lib.check(lib.mq_set_tuning(19, t64), "knob")
                    for _ in range(2):
                        _, probs = m.forward(x)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = probs.clone()
                    same = bool(torch.equal(probs, ref))
                    t0 = time.perf_counter()
                    for _ in range(10):
                        m.forward(x)
                    torch.cuda.synchronize()
                    print(f"r={rnd} ResNet-152 ID forward, {n} boxes, tile64={t64} implicit_conv={implicit}: "
                          f"{(time.perf_counter() - t0) * 100:.2f} ms  identical={same}", flush=True)
    finally:
        lib.mq_set_tuning(19, old)


if __name__ == "__main__":
    main()
