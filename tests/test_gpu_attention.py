"""GPU numerics of mq_attention_bf16 (the encoder's global MHSA) vs a PyTorch fp32 reference.

Inputs are bf16; the reference runs softmax(q k^T / sqrt(dh)) v in fp32 on the same bf16
values.  The kernel rounds P to bf16 before the PV MFMA and the output to bf16, so the
tolerance is 1.5e-2 relative to max|v| (bf16 has 8 mantissa bits).
"""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _ref(qkv, n, T, D, H):
    import torch
    x = qkv.float().view(n, T, 3, H, D // H).permute(2, 0, 3, 1, 4)   # 3, n, H, T, dh
    q, k, v = x[0], x[1], x[2]
    a = torch.softmax(q @ k.transpose(-1, -2) / (D // H) ** 0.5, dim=-1)
    return (a @ v).permute(0, 2, 1, 3).reshape(n * T, D)


@pytest.mark.parametrize("n,T,D,H", [(3, 192, 1280, 16), (2, 192, 768, 12), (2, 64, 320, 4), (1, 96, 1280, 16),
                                     (64, 192, 1280, 16)])
def test_attention_matches_fp32(n, T, D, H):
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(n * 7 + T)
    qkv = (torch.randn((n * T, 3 * D), generator=g, device="cuda") * 2).to(torch.bfloat16)
    out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, _lib.stream_ptr()),
               "mq_attention_bf16")
    torch.cuda.synchronize()
    ref = _ref(qkv, n, T, D, H)
    vmax = qkv.float().abs().max().item()
    err = (out.float() - ref).abs().max().item()
    assert err <= 1.5e-2 * vmax, (err, vmax)


def test_attention_rejects_bad_shapes():
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    qkv = torch.zeros((100, 3 * 1280), device="cuda", dtype=torch.bfloat16)
    out = torch.zeros((100, 1280), device="cuda", dtype=torch.bfloat16)
    assert ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), 1, 100, 1280, 16, None) != 0
    assert ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), 1, 96, 1280, 10, None) != 0


def test_attention_spiky_scores_match_fp32():
    """A few very large keys per query: the row max dominates and most P underflow -- the softmax
    must still be normalised per query (checks the lane-local 1/l of the transposed output)."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    n, T, D, H = 2, 192, 1280, 16
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    qkv = torch.randn((n * T, 3 * D), generator=g, device="cuda")
    qkv[7, D:2 * D] *= 12.0                     # one key row much larger
    qkv[200, D:2 * D] *= -9.0
    qkv = qkv.to(torch.bfloat16)
    out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H, _lib.stream_ptr()),
               "mq_attention_bf16")
    torch.cuda.synchronize()
    ref = _ref(qkv, n, T, D, H)
    vmax = qkv[:, 2 * D:].float().abs().max().item()
    assert (out.float() - ref).abs().max().item() <= 1.5e-2 * vmax


@pytest.mark.parametrize("n,D,H", [(64, 1280, 16), (3, 768, 12)])
def test_attention_kring_equals_compiler_loop(n, D, H):
    """the 192-token QK^T streams K fragments through an inline-asm ring with hand-counted lgkmcnt
    waits that the compiler's waitcnt pass does not see; MQ_TUNE_ATTN_KRING = 0 routes the same shape to the
    compiler-scheduled loop of the generic instantiation.  Same MFMA order per output: bit for bit."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    T = 192
    g = torch.Generator(device="cuda")
    g.manual_seed(31 + n)
    qkv = (torch.randn((n * T, 3 * D), generator=g, device="cuda") * 2).to(torch.bfloat16)
    outs = {}
    old = ctx.lib.mq_get_tuning(24)
    try:
        for ring in (1, 0):
            assert ctx.lib.mq_set_tuning(24, ring) == 0
            out = torch.empty((n * T, D), device="cuda", dtype=torch.bfloat16)
            _lib.check(ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H,
                                                 _lib.stream_ptr()), "mq_attention_bf16")
            torch.cuda.synchronize()
            outs[ring] = out
    finally:
        ctx.lib.mq_set_tuning(24, old)
    assert torch.equal(outs[1], outs[0])
