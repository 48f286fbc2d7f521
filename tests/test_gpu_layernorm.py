"""GPU: mq_layernorm (the ViT-H pre-norms, mmpretrain LayerNorm eps 1e-6, and the detector's Swin norms)
against torch's fp32 layer_norm: f32 output to 2e-6 relative, bf16 output within one bf16 rounding of the
fp32 value; ragged row counts (a wave handles several rows) and every dimension class of the kernel."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.mark.parametrize("rows", [1, 5, 7, 8, 9, 12288, 12289])
@pytest.mark.parametrize("dim", [96, 384, 768, 1280, 1536, 3072])
def test_layernorm_matches_fp32(rows, dim):
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(rows * 7 + dim)
    x = torch.randn((rows, dim), generator=g, device="cuda") * 3 + 0.5
    gam = torch.randn((dim,), generator=g, device="cuda")
    bet = torch.randn((dim,), generator=g, device="cuda")
    ref = torch.nn.functional.layer_norm(x.double(), (dim,), gam.double(), bet.double(), 1e-6)
    for out_f32 in (1, 0):
        y = torch.full((rows + 1, dim), 7.0, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
        _lib.check(ctx.lib.mq_layernorm(ctx.handle, _lib.ptr(x), _lib.ptr(gam), _lib.ptr(bet), _lib.ptr(y), rows, dim,
                                        1e-6, out_f32, _lib.stream_ptr()), "mq_layernorm")
        torch.cuda.synchronize()
        assert (y[rows] == 7.0).all(), "wrote past the last row"
        got = y[:rows].double()
        scale = ref.abs().max().item()
        if out_f32:
            assert (got - ref).abs().max().item() <= 2e-6 * scale
        else:
            # one bf16 rounding (2^-8 relative) of a value within the f32 error
            assert ((got - ref).abs() <= ref.abs() * 2.0 ** -8 + 2e-6 * scale).all()


@pytest.mark.parametrize("rows", [1, 7, 9, 12288, 12289])
@pytest.mark.parametrize("dim", [96, 384, 1280, 3072])
@pytest.mark.parametrize("nadd,store", [(1, 0), (1, 1), (2, 0), (2, 1)])
def test_add_layernorm_matches_fp32(rows, dim, nadd, store):
    """mq_add_layernorm (ABI 5): x += p1 (+= p2) with bf16 branch outputs, x stored when asked, y = LN(x) in
    bf16 -- the residual updates of the ViT / Swin pre-norm blocks fused into the next norm.  x after the
    update is exactly float32 (x + p1) + p2; y within one bf16 rounding of the fp32 LayerNorm of it."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(rows * 13 + dim + 100 * nadd + store)
    x = torch.randn((rows, dim), generator=g, device="cuda") * 3 + 0.5
    p1 = (torch.randn((rows, dim), generator=g, device="cuda")).to(torch.bfloat16)
    p2 = (torch.randn((rows, dim), generator=g, device="cuda") * 0.5).to(torch.bfloat16)
    gam = torch.randn((dim,), generator=g, device="cuda")
    bet = torch.randn((dim,), generator=g, device="cuda")
    want_x = x + p1.float()
    if nadd == 2:
        want_x = want_x + p2.float()
    ref = torch.nn.functional.layer_norm(want_x.double(), (dim,), gam.double(), bet.double(), 1e-6)
    x0 = x.clone()
    y = torch.full((rows + 1, dim), 7.0, device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_add_layernorm(ctx.handle, _lib.ptr(x), _lib.ptr(p1), _lib.ptr(p2) if nadd == 2 else None,
                                        store, _lib.ptr(gam), _lib.ptr(bet), _lib.ptr(y), rows, dim, 1e-6,
                                        _lib.stream_ptr()), "mq_add_layernorm")
    torch.cuda.synchronize()
    assert (y[rows] == 7.0).all(), "wrote past the last row"
    assert torch.equal(x, want_x if store else x0)
    got = y[:rows].double()
    scale = ref.abs().max().item()
    assert ((got - ref).abs() <= ref.abs() * 2.0 ** -8 + 2e-6 * scale).all()
