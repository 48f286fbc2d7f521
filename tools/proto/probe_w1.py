"""Prototype A/B (tools/proto/gemm_w1.hip, one wave per SIMD, 128 x 256 tiles) against the shipped ping-pong
GEMM (mq_gemm_bf16, plain bf16 epilogue, no bias) on the ViT-H GEMM shapes, in one process, alternating;
the prototype's output is checked against torch (fp32 accumulate of the same bf16 operands).
python tools/proto/probe_w1.py [--iters 20] [--rounds 3]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))
SHAPES = {"qkv": (12288, 3840, 1280), "fc1": (12288, 5120, 1280), "fc2": (12288, 1280, 5120),
          "proj": (12288, 1280, 1280), "dc1": (12288, 4096, 1280)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shape", default="fc1,qkv,fc2,proj,dc1")
    a = ap.parse_args()
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    proto = C.CDLL(os.path.join(ROOT, "tools", "proto", "libproto_w1.so"))
    vp, i32 = C.c_void_p, C.c_int
    proto.proto_gemm_w1.argtypes = [vp, vp, vp, i32, i32, i32, i32, vp]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    for name in a.shape.split(","):
        M, N, K = SHAPES[name]
        A = torch.empty((M, K), device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
        W = (torch.empty((N, K), device=dev).uniform_(-1, 1, generator=g) / K ** 0.5).to(torch.bfloat16)
        Cp = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        Cq = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        runs = {
            "pingpong": lambda: ctx.lib.mq_gemm_bf16(ctx.handle, P(A), P(W), P(Cp), None, None, M, N, K, K, K, N, 0, 0, s),
            "w1proto": lambda: proto.proto_gemm_w1(P(A), P(W), P(Cq), M, N, K, cus, s),
        }
        for k, f in runs.items():
            assert f() == 0, k
        torch.cuda.synchronize()
        ref = (A.float() @ W.float().t())
        for k, c in (("pingpong", Cp), ("w1proto", Cq)):
            err = (c.float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"{name} {k}: max rel err vs fp32 {err:.2e}", flush=True)
        print(f"{name}: pingpong == w1proto bitwise: {bool(torch.equal(Cp, Cq))}", flush=True)
        for rnd in range(a.rounds):
            for k, f in runs.items():
                for _ in range(3):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.iters * 1e3
                print(f"{name} {k} r={rnd}: {us:.1f} us  {2 * M * N * K / (us * 1e-6) / 1e12:.0f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
