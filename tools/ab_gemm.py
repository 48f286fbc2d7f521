"""A/B two builds of libmq_hip.so in ONE process (box-to-box clock spread is ~8 %, so A/B numbers
are only taken side by side): time mq_gemm_bf16 on the ViT-H GEMM shapes (and optionally the
attention) through each library, alternating, with hipEvents on the launch stream, and check that the
two give bit-identical outputs.

python tools/ab_gemm.py --a macaque-3d-pose-estimation_amd/lib_prev/libmq_hip.so \
                        --b macaque-3d-pose-estimation_amd/lib/libmq_hip.so [--shape fc1,fc2] [--iters 20]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))
from gemm_probe import SHAPES  # noqa: E402  (same shape table)


def open_lib(path):
    lib = C.CDLL(os.path.abspath(path))  # RTLD_LOCAL: the two builds keep their own symbols
    vp, i32 = C.c_void_p, C.c_int
    lib.mq_create.argtypes = [i32, C.POINTER(vp)]
    lib.mq_gemm_bf16.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]
    lib.mq_attention_bf16.argtypes = [vp, vp, vp, i32, i32, i32, i32, vp]
    lib.mq_layernorm.argtypes = [vp, vp, vp, vp, vp, i32, i32, C.c_float, i32, vp]
    lib.mq_add_layernorm.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, C.c_float, vp]
    ctx = vp()
    assert lib.mq_create(0, C.byref(ctx)) == 0
    return lib, ctx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--shape", default="qkv,proj,fc1,fc2,dc1,dc2")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--attention", action="store_true")
    ap.add_argument("--layernorm", action="store_true", help="also time mq_layernorm (ViT-H rows, bf16 and f32 out)")
    ap.add_argument("--add-layernorm", action="store_true",
                    help="also time mq_add_layernorm at the bench's rows, 64 images x 192 tokens (x += p1 [+ p2], stored or not)")
    args = ap.parse_args()
    import torch
    libs = {"A": open_lib(args.a), "B": open_lib(args.b)}
    dev = torch.device("cuda", 0)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for name in [n for n in args.shape.split(",") if n]:
        M, N, K, epi = SHAPES[name]
        a = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn((N, K), generator=g, device=dev) / K ** 0.5).to(torch.bfloat16)
        bias = torch.randn((N,), generator=g, device=dev)
        f32 = epi in (2, 3, 4, 5)
        c0 = torch.randn((M, N), generator=g, device=dev)
        outs = {}
        for rnd in range(args.rounds):
            for key, (lib, ctx) in libs.items():
                c = c0.clone() if f32 else torch.empty((M, N), device=dev, dtype=torch.bfloat16)
                run = lambda: lib.mq_gemm_bf16(ctx, P(a), P(w), P(c), P(bias), None, M, N, K, K, K, N, 0, epi, s)  # noqa
                assert run() == 0
                torch.cuda.synchronize()
                if rnd == 0:
                    outs[key] = c.clone()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / args.iters * 1e3
                print(f"{name} {key} r={rnd}: {us:.1f} us  {2 * M * N * K / (us * 1e-6) / 1e12:.0f} TFLOP/s", flush=True)
        print(f"{name}: A and B bit-identical = {bool(torch.equal(outs['A'], outs['B']))}", flush=True)
    if args.attention:
        n, T, D, H = 64, 192, 1280, 16
        qkv = torch.randn((n * T, 3 * D), generator=g, device=dev).to(torch.bfloat16)
        for rnd in range(args.rounds):
            for key, (lib, ctx) in libs.items():
                out = torch.empty((n * T, D), device=dev, dtype=torch.bfloat16)
                for _ in range(3):
                    lib.mq_attention_bf16(ctx, P(qkv), P(out), n, T, D, H, s)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    lib.mq_attention_bf16(ctx, P(qkv), P(out), n, T, D, H, s)
                e1.record()
                torch.cuda.synchronize()
                print(f"attention {key} r={rnd}: {e0.elapsed_time(e1) / args.iters * 1e3:.1f} us", flush=True)

    if args.layernorm:
        rows, dim = 64 * 192, 1280
        x = torch.randn((rows, dim), generator=g, device=dev) * 3 + 0.5
        gam = torch.randn((dim,), generator=g, device=dev)
        bet = torch.randn((dim,), generator=g, device=dev)
        for out_f32 in (0, 1):
            outs = {}
            for rnd in range(args.rounds):
                for key, (lib, ctx) in libs.items():
                    y = torch.empty((rows, dim), device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
                    run = lambda: lib.mq_layernorm(ctx, P(x), P(gam), P(bet), P(y), rows, dim, 1e-6, out_f32, s)  # noqa: E731
                    for _ in range(3):
                        assert run() == 0
                    torch.cuda.synchronize()
                    outs.setdefault(key, y.clone())
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / args.iters * 1e3
                    nbytes = rows * dim * (4 + (4 if out_f32 else 2))
                    print(f"layernorm out_f32={out_f32} {key} r={rnd}: {us:.2f} us  {nbytes / (us * 1e-6) / 1e12:.2f} TB/s",
                          flush=True)
            print(f"layernorm out_f32={out_f32}: A and B bit-identical = {bool(torch.equal(outs['A'], outs['B']))}",
                  flush=True)

    if args.add_layernorm:
        rows, dim = 64 * 192, 1280
        x0 = torch.randn((rows, dim), generator=g, device=dev) * 3 + 0.5
        p1 = torch.randn((rows, dim), generator=g, device=dev).to(torch.bfloat16)
        p2 = torch.randn((rows, dim), generator=g, device=dev).to(torch.bfloat16)
        gam = torch.randn((dim,), generator=g, device=dev)
        bet = torch.randn((dim,), generator=g, device=dev)
        for nadd, store in ((2, 1), (1, 0), (2, 0)):
            outs = {}
            for rnd in range(args.rounds):
                for key, (lib, ctx) in libs.items():
                    x = x0.clone()
                    y = torch.empty((rows, dim), device=dev, dtype=torch.bfloat16)
                    q2 = P(p2) if nadd == 2 else None
                    run = lambda: lib.mq_add_layernorm(ctx, P(x), P(p1), q2, store, P(gam), P(bet), P(y), rows, dim,  # noqa
                                                       1e-6, s)
                    assert run() == 0
                    torch.cuda.synchronize()
                    outs.setdefault(key, (x.clone(), y.clone()))
                    for _ in range(2):
                        run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / args.iters * 1e3
                    nbytes = rows * dim * (4 + 2 * nadd + 4 * store + 2)
                    print(f"add_layernorm nadd={nadd} store={store} {key} r={rnd}: {us:.2f} us  "
                          f"{nbytes / (us * 1e-6) / 1e12:.2f} TB/s", flush=True)
            same = torch.equal(outs["A"][0], outs["B"][0]) and torch.equal(outs["A"][1], outs["B"][1])
            print(f"add_layernorm nadd={nadd} store={store}: A and B bit-identical = {same}", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
