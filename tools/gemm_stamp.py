"""Per-segment timing of the ping-pong GEMM mainloop from a PP_STAMP diagnostic build of libmq_hip.so
(never the shipped library): s_memtime after each of the 8 barriers of K-steps 4-7 in block 0, for wave 0
(group 0) and wave 4 (group 1, the same SIMD).  Prints the cycle gap between consecutive barriers.

Build: make -C macaque-3d-pose-estimation_amd/csrc OUT=../lib_stamp EXTRA=-DPP_STAMP
Run:   python tools/gemm_stamp.py [--shape fc1]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from gemm_probe import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "macaque-3d-pose-estimation_amd", "lib_stamp", "libmq_hip.so"))
    ap.add_argument("--shape", default="fc1,dc1,fc2_bf16")
    args = ap.parse_args()
    import torch
    lib = C.CDLL(args.lib)
    vp, i32 = C.c_void_p, C.c_int
    lib.mq_create.argtypes = [i32, C.POINTER(vp)]
    lib.mq_gemm_bf16.argtypes = [vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp]
    ctx = vp()
    assert lib.mq_create(0, C.byref(ctx)) == 0
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name in args.shape.split(","):
        M, N, K, epi = SHAPES[name]
        A = (torch.rand((M, K), device="cuda") * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand((N, K), device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.zeros((N,), device="cuda")
        Cm = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
        st = torch.zeros((128,), device="cuda", dtype=torch.int64)
        for _ in range(5):
            assert lib.mq_gemm_bf16(ctx, C.c_void_p(A.data_ptr()), C.c_void_p(W.data_ptr()), C.c_void_p(Cm.data_ptr()),
                                    C.c_void_p(bias.data_ptr()), C.c_void_p(st.data_ptr()), M, N, K, K, K, N, 0, epi,
                                    s) == 0
        torch.cuda.synchronize()
        t = st.cpu().tolist()
        for grp in (0, 1):
            ts = t[grp * 64: grp * 64 + 64]   # (arrival, release) per barrier, 8 barriers per K-step
            own = [ts[2 * i + 2] - ts[2 * i + 1] for i in range(31)]    # release -> next arrival: own segment
            wait = [ts[2 * i + 1] - ts[2 * i] for i in range(32)]        # arrival -> release: waiting
            print(f"{name} group {grp} own segment cycles:", own, flush=True)
            print(f"{name} group {grp} barrier wait cycles:", wait, flush=True)
            comp = own[0::2] if grp == 0 else own[1::2]
            load = own[1::2] if grp == 0 else own[0::2]
            print(f"{name} group {grp}: mean own segment after open_mfma (MFMA) {sum(own[0::2]) / len(own[0::2]):.0f}, "
                  f"after bar (load) {sum(own[1::2]) / len(own[1::2]):.0f}; mean wait {sum(wait) / len(wait):.0f}",
                  flush=True)


if __name__ == "__main__":
    main()
