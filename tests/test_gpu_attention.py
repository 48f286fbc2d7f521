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


@pytest.mark.parametrize("n,T,D,H", [(3, 192, 1280, 16), (2, 192, 768, 12), (2, 64, 320, 4), (1, 96, 1280, 16)])
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


@pytest.mark.parametrize("n", [1, 7, 64])
def test_attention_persistent_bitwise_equals_per_item(n):
    """The persistent T=192 kernel (MQ_TUNE_ATTENTION_PERSIST, K/V of the next (image, head) staged
    under the current one's compute) runs the same arithmetic as the one-workgroup-per-item kernel:
    outputs must match bit for bit, including grids with fewer items than workgroups."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    T, D, H = 192, 1280, 16
    g = torch.Generator(device="cuda")
    g.manual_seed(100 + n)
    qkv = (torch.randn((n * T, 3 * D), generator=g, device="cuda") * 2).to(torch.bfloat16)
    outs = []
    old = ctx.lib.mq_get_tuning(15)
    try:
        for persist in (0, 1):
            assert ctx.lib.mq_set_tuning(15, persist) == 0
            out = torch.full((n * T, D), float("nan"), device="cuda", dtype=torch.bfloat16)
            _lib.check(ctx.lib.mq_attention_bf16(ctx.handle, _lib.ptr(qkv), _lib.ptr(out), n, T, D, H,
                                                 _lib.stream_ptr()), "mq_attention_bf16")
            outs.append(out)
    finally:
        ctx.lib.mq_set_tuning(15, old)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
