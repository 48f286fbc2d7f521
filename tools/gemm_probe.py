"""Time the ViT GEMM shapes through mq_gemm_bf16 (hipEvents on the launch stream).

python tools/gemm_probe.py [--iters N] [--shape fc1|fc2|qkv|proj|dc1|dc2|all]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))

COLD = False
SHAPES = {  # name: (M, N, K, epilogue)  for 64 forwards x 192 tokens, ViT-H
    "qkv": (12288, 3840, 1280, 0),
    "proj": (12288, 1280, 1280, 2),  # (until round 4: the f32 residual epilogue)
    "proj_bf16": (12288, 1280, 1280, 0),  # round 4 on: bf16 branch output
    "fc1": (12288, 5120, 1280, 1),
    "fc2": (12288, 1280, 5120, 2),
    "dc1": (12288, 4096, 1280, 0),
    "fc2_bf16": (12288, 1280, 5120, 0),  # round 4 on: bf16 branch output
    "dc2": (49152, 4096, 256, 0),
    "f32": (12288, 1280, 5120, 4),   # fc2 shape, plain f32 epilogue
    "fc1_f32": (12288, 5120, 1280, 4),
    "fc1_bf16": (12288, 5120, 1280, 0),
    "n5120_k5120": (12288, 5120, 5120, 0),
    "m8192": (8192, 5120, 1280, 0),
    # one tile per CU on 240 / 120 CUs (the epilogue's store cost against the number of CUs storing at once)
    "fc1_m3072": (3072, 5120, 1280, 1),
    "fc1_m1536": (1536, 5120, 1280, 1),
    "bf16_m3072": (3072, 5120, 1280, 0),
    "bf16_m1536": (1536, 5120, 1280, 0),
    # ragged tiles (partial M and N tiles, one and several K-steps)
    "odd_gelu": (700, 520, 320, 1),
    "odd_bf16": (1000, 264, 2048, 0),
    "odd_k64": (300, 264, 64, 6),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shape", default="all")
    ap.add_argument("--variants", default="pp,il,torch", help="GEMM routes to A/B in this process: pp, il, small, w4 (LDS-DMA), w4v (VGPR-staged), torch")
    ap.add_argument("--cold", action="store_true",
                    help="evict L2/Infinity Cache (384 MB write) before every launch; time each launch alone")
    args = ap.parse_args()
    global COLD
    COLD = args.cold
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    names = list(SHAPES) if args.shape == "all" else args.shape.split(",")
    res = {}
    variants = args.variants.split(",")
    for rnd in range(2):
        for var in variants:
            if var == "torch":
                for name in names:
                    res[f"{name}/{var}/r{rnd}"] = bench_torch(torch, name, args.iters)
                    print(f"{name} v={var} r={rnd}", res[f"{name}/{var}/r{rnd}"], flush=True)
                continue
            # routing knobs (include/mq_hip.h): pp = ping-pong (default), il = interleaved K-step, small = 128x128
            _lib.check(ctx.lib.mq_set_tuning(12, 0 if var == "il" else 1), "tuning")
            _lib.check(ctx.lib.mq_set_tuning(2, 1 if var == "small" else 0), "tuning")
            _lib.check(ctx.lib.mq_set_tuning(27, {"w4": 1, "w4v": 2}.get(var, 0)), "tuning")
            for name in names:
                res[f"{name}/{var}/r{rnd}"] = bench_one(ctx, _lib, torch, name, args.iters)
                print(f"{name} v={var} r={rnd}", res[f"{name}/{var}/r{rnd}"], flush=True)
    _lib.check(ctx.lib.mq_set_tuning(12, 1), "tuning")
    _lib.check(ctx.lib.mq_set_tuning(2, 0), "tuning")
    _lib.check(ctx.lib.mq_set_tuning(27, 0), "tuning")
    print(json.dumps(res))


def bench_torch(torch, name, iters):
    """torch.matmul (hipBLASLt) on the same shape, bf16 out, no fused epilogue -- a reference point."""
    M, N, K, epi = SHAPES[name]
    A = (torch.rand((M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((N, K), device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    out = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(A, W.t(), out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.matmul(A, W.t(), out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return {"M": M, "N": N, "K": K, "ms": round(ms, 4), "tflops": round(2 * M * N * K / (ms * 1e-3) / 1e12, 1)}


def bench_one(ctx, _lib, torch, name, iters):
    if True:
        M, N, K, epi = SHAPES[name]
        A = (torch.rand((M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand((N, K), device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.zeros((N,), device="cuda")
        Cm = torch.zeros((M, N), device="cuda", dtype=torch.bfloat16 if epi in (0, 1) else torch.float32)
        s = _lib.stream_ptr()

        def run():
            _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), _lib.ptr(bias), None,
                                            M, N, K, K, K, N, 0, epi, s), name)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        if COLD:
            flush = torch.empty((384 << 20) // 4, device="cuda")
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
            for a, b in ev:
                flush.fill_(1.0)
                a.record()
                run()
                b.record()
            torch.cuda.synchronize()
            ms = sum(a.elapsed_time(b) for a, b in ev) / iters
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
        tf = 2 * M * N * K / (ms * 1e-3) / 1e12
        return {"M": M, "N": N, "K": K, "ms": round(ms, 4), "tflops": round(tf, 1)}


if __name__ == "__main__":
    main()
