"""Attention launch time against the number of workgroups (images x 16 heads): with two resident
workgroups per CU, 256 and 512 workgroups should take about one workgroup lifetime each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    T, D, H = 192, 1280, 16
    s = _lib.stream_ptr()
    for ver in (1, 2):
        assert ctx.lib.mq_set_tuning(17, ver) == 0
        for n in (8, 16, 24, 32, 40, 48, 56, 64, 128):
            qkv = torch.randn((n * T, 3 * D), device="cuda").to(torch.bfloat16)
            out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
            for _ in range(3):
                ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, s)
            e1.record()
            torch.cuda.synchronize()
            print(f"v{ver} images={n} workgroups={n * H}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
    ctx.lib.mq_set_tuning(17, 1)


if __name__ == "__main__":
    main()
