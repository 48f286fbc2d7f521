"""Time mq_attention_bf16 at the ViT-H bench shape (64 images x 192 tokens, 16 heads x 80): the
shipped kernel (v2) against the first-generation one (v1, MQ_TUNE_ATTENTION_V2 = 0) in one process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def main():
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    n, T, D, H = 64, 192, 1280, 16
    qkv = torch.randn((n * T, 3 * D), device="cuda").to(torch.bfloat16)
    out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
    s = _lib.stream_ptr()
    for rnd in range(3):
        for ver in (0, 1):
            assert ctx.lib.mq_set_tuning(17, ver) == 0
            for _ in range(3):
                ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, s)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            print(f"attention v{ver + 1} r={rnd}: {us:.1f} us  "
                  f"({2 * 2 * n * H * T * T * (D // H) / (us * 1e-6) / 1e12:.0f} TFLOP/s)", flush=True)
    ctx.lib.mq_set_tuning(17, 1)


if __name__ == "__main__":
    main()
