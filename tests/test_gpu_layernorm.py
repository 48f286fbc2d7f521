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
