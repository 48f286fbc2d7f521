"""Per-256x256-tile error map of mq_gemm_bf16 (EPI_F32) against fp32 on multi-tile grids, with the K-slice that
explains a bad tile: the tool that located the sibling-wave race of the round-3 two-phase ping-pong draft."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))
import torch
from mqhip import _lib
torch.backends.cuda.matmul.allow_tf32 = False
ctx = _lib.Context.get(0)
for (M, N, K) in [(4096, 5120, 256), (4096, 5120, 128), (12288, 5120, 1280)]:
    g = torch.Generator(device="cuda"); g.manual_seed(0)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    ref = A.float() @ W.float().t() + bias
    C = torch.empty((M, N), device="cuda")
    _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(C), _lib.ptr(bias), None, M, N, K,
                                    K, K, N, 0, 4, _lib.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    err = (C - ref).abs()
    tm, tn = M // 256, N // 256
    te = err.view(tm, 256, tn, 256).amax(dim=(1, 3))
    bad = (te > 0.05).nonzero().tolist()
    print(f"M{M} N{N} K{K}: max err {err.max().item():.3f}, bad tiles {len(bad)} of {tm * tn}: {bad[:40]}")
    if bad:
        i, j = bad[0]
        sub = err[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256]
        rows = (sub.amax(dim=1) > 0.05).nonzero().flatten().tolist()
        cols = (sub.amax(dim=0) > 0.05).nonzero().flatten().tolist()
        print("  first bad tile rows:", rows[:8], "...", len(rows), " cols:", cols[:8], "...", len(cols))
        # which K-slice: compare with the products of each 64-slice removed
        for s in range(K // 64):
            A2 = A.float().clone(); A2[:, s * 64:(s + 1) * 64] = 0
            r2 = (A2 @ W.float().t() + bias)[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256]
            d = (C[i * 256:(i + 1) * 256, j * 256:(j + 1) * 256] - r2).abs().max().item()
            print(f"  minus slice {s}: max diff {d:.3f}")
