"""A/B of PP_DIAG diagnostic builds of libmq_hip.so (csrc/gemm_pp.hip: one part of the ping-pong mainloop taken
out; results are garbage, only the time means something) against the shipped library, in one process.

Build: make -C macaque-3d-pose-estimation_amd/csrc OUT=../lib_diag<n> EXTRA=-DPP_DIAG=<n>
Run:   python tools/gemm_diag.py [--shape fc1,qkv] [--diag 2,10,26]   (PP_DIAG bits: csrc/gemm_pp.hip)
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gemm_probe import SHAPES  # noqa: E402

PKG = os.path.join(ROOT, "macaque-3d-pose-estimation_amd")
BITS = {1: "no counted vmcnt waits", 2: "no LDS-DMA", 4: "no barriers", 8: "fragment reads once", 16: "no epilogue", 32: "epilogue without stores", 64: "epilogue stores L2-resident", 128: "both groups' epilogues in one interval (removed; git history)",
        256: "epilogue stores lane-linear per wave", 1024: "deferred-store kernel (removed; git history)",
        512: "epilogue arithmetic first, then the stores", 4096: "static priority for group 1",
        8192: "no priority changes", 16384: "half-tile kernel with the streamed epilogue (removed; git history)",
        32768: "no lgkmcnt(0) opening the MFMA segments"}


def what(d):
    if d >= 100000:  # lib_diag1000NN: a build with PP_GROUP_M = NN (the tile walk's M-group)
        return f"GROUP_M {d - 100000}"
    return "shipped" if d == 0 else ", ".join(v for b, v in BITS.items() if d & b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="fc1,qkv,fc2_bf16")
    ap.add_argument("--diag", default="16,32,64")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", action="store_true",
                    help="also compare each build's output with the shipped library's, bit for bit (for diag builds that "
                         "keep the results, e.g. 1024)")
    ap.add_argument("--attention", action="store_true",
                    help="time mq_attention_bf16 (ViT-H, 64 images) from lib_attdiag<n> builds (-DATT_DIAG=<n>, vit_ops.hip)")
    args = ap.parse_args()
    import torch
    vp, i32 = C.c_void_p, C.c_int
    libs = {}
    for d in [0] + [int(x) for x in args.diag.split(",")]:
        sub = "lib" if d == 0 else (f"lib_attdiag{d}" if args.attention else f"lib_diag{d}")
        path = os.path.join(PKG, sub, "libmq_hip.so")
        lib = C.CDLL(path)
        lib.mq_create.argtypes = [i32, C.POINTER(vp)]
        lib.mq_gemm_bf16.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]
        lib.mq_attention_bf16.argtypes = [vp, vp, vp, i32, i32, i32, i32, vp]
        ctx = vp()
        assert lib.mq_create(0, C.byref(ctx)) == 0, path
        libs[d] = (lib, ctx)
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    if args.attention:
        attention(args, torch, libs, s)
        return
    for name in args.shape.split(","):
        M, N, K, epi = SHAPES[name]
        A = (torch.rand((M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand((N, K), device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.zeros((N,), device="cuda")
        Cm = torch.zeros((M, N), device="cuda", dtype=torch.bfloat16 if epi in (0, 1) else torch.float32)
        keys = list(libs)
        for rnd in range(args.rounds):
            # the order rotates every round, so no build always runs first (the clock ramps within a round)
            for d in keys[rnd % len(keys):] + keys[:rnd % len(keys)]:
                lib, ctx = libs[d]
                if d & 256 and M * N * 2 < (32 << 20):  # (the lane-linear store region is 32 MiB)
                    continue
                def run():
                    assert lib.mq_gemm_bf16(ctx, C.c_void_p(A.data_ptr()), C.c_void_p(W.data_ptr()),
                                            C.c_void_p(Cm.data_ptr()), C.c_void_p(bias.data_ptr()), None, M, N, K, K, K,
                                            N, 0, epi, s) == 0
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / args.iters * 1e3
                res.setdefault((name, d), []).append(us)
        if args.check:
            outs = {}
            for d, (lib, ctx) in libs.items():
                if d & 256 and M * N * 2 < (32 << 20):
                    continue
                Cm.fill_(7.0)
                assert lib.mq_gemm_bf16(ctx, C.c_void_p(A.data_ptr()), C.c_void_p(W.data_ptr()), C.c_void_p(Cm.data_ptr()),
                                        C.c_void_p(bias.data_ptr()), None, M, N, K, K, K, N, 0, epi, s) == 0
                torch.cuda.synchronize()
                outs[d] = Cm.clone()
            for d in outs:
                if d:
                    same = bool(torch.equal(outs[0].view(torch.int16) if outs[0].dtype == torch.bfloat16 else outs[0],
                                            outs[d].view(torch.int16) if outs[d].dtype == torch.bfloat16 else outs[d]))
                    print(f"{name} diag {d}: bit-identical to shipped = {same}", flush=True)
        for d in libs:
            if (name, d) not in res:
                continue
            v = sorted(res[(name, d)])
            print(f"{name} diag {d} ({what(d)}): median {v[len(v) // 2]:.1f} us  all {[round(x, 1) for x in res[(name, d)]]}",
                  flush=True)


ATT_BITS = {1: "no K/V/Q loads", 2: "no exponentials", 4: "no PV MFMAs", 8: "no stores", 16: "no QK MFMAs",
            32: "no K fragment reads"}


def attention(args, torch, libs, s):
    n, T, D, H = 64, 192, 1280, 16
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    qkv = torch.randn((n * T, 3 * D), generator=g, device="cuda").to(torch.bfloat16)
    out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
    res = {}
    for rnd in range(args.rounds):
        for d, (lib, ctx) in libs.items():
            def run():
                assert lib.mq_attention_bf16(ctx, C.c_void_p(qkv.data_ptr()), C.c_void_p(out.data_ptr()), n, T, D, H,
                                             s) == 0
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(d, []).append(e0.elapsed_time(e1) / args.iters * 1e3)
    for d, v in res.items():
        w = "shipped" if d == 0 else ", ".join(t for b, t in ATT_BITS.items() if d & b)
        print(f"attention diag {d} ({w}): median {sorted(v)[len(v) // 2]:.1f} us  all {[round(x, 1) for x in v]}",
              flush=True)


if __name__ == "__main__":
    main()
