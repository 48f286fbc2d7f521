"""Sub-pixel implicit-GEMM ConvTranspose2d(k4, s2, p1) + BatchNorm + ReLU (mq_deconv_subpixel_bf16): the
ViTPose head's second deconvolution (model/pose/ViTPose_huge_macaque_256x192.py: HeatmapHead
deconv_out_channels (256, 256), kernel 4) without the 16-tap column buffer and col2im pass.  Checked against
torch's fp32 conv_transpose2d on the same bf16 operands (weights with the BN scale folded in, as packed)."""
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,h,w,ch,cout,relu", [(64, 32, 24, 256, 256, 1), (1, 5, 3, 256, 256, 1),
                                                (3, 8, 6, 64, 256, 0), (2, 17, 11, 128, 512, 1)])
def test_deconv_subpixel_matches_conv_transpose(n, h, w, ch, cout, relu):
    import torch.nn.functional as F
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(n * 100 + h + w + ch)
    x = torch.randn((n, h, w, ch), generator=g, device="cuda").to(torch.bfloat16)
    wt = torch.randn((ch, cout, 4, 4), generator=g, device="cuda") / (2 * ch ** 0.5)
    scale = 0.5 + torch.rand((cout,), generator=g, device="cuda")
    shift = torch.randn((cout,), generator=g, device="cuda") * 0.1
    packed = torch.empty((4 * cout, 4 * ch), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_deconv_subpixel_pack(ctx.handle, _lib.ptr(wt), _lib.ptr(scale), _lib.ptr(packed), ch, cout,
                                               _lib.stream_ptr()), "pack")
    shift4 = shift.repeat(4).contiguous()
    out = torch.empty((n, 2 * h, 2 * w, cout), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_deconv_subpixel_bf16(ctx.handle, _lib.ptr(x), n, h, w, ch, _lib.ptr(packed),
                                               _lib.ptr(shift4), _lib.ptr(out), cout, relu, _lib.stream_ptr()),
               "deconv")
    torch.cuda.synchronize()
    wref = (wt * scale.view(1, cout, 1, 1)).to(torch.bfloat16).float()
    ref = F.conv_transpose2d(x.permute(0, 3, 1, 2).float(), wref, stride=2, padding=1) + shift.view(1, cout, 1, 1)
    if relu:
        ref = ref.clamp_min(0)
    ref = ref.permute(0, 2, 3, 1)
    err = (out.float() - ref).abs().max().item()
    # bf16 output rounding (2^-8 relative) plus f32 accumulation-order differences
    assert err <= 8e-3 * ref.abs().max().item() + 1e-6, err
    # every output pixel class and the image borders (taps outside the input read zeros)
    for py in (0, 1):
        for px in (0, 1):
            e = (out.float()[:, py::2, px::2] - ref[:, py::2, px::2]).abs().max().item()
            assert e <= 8e-3 * ref.abs().max().item() + 1e-6, (py, px, e)


def test_deconv_subpixel_rejects_bad_shapes():
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    x = torch.zeros((1, 4, 4, 96), device="cuda", dtype=torch.bfloat16)
    wp = torch.zeros((1024, 384), device="cuda", dtype=torch.bfloat16)
    out = torch.zeros((1, 8, 8, 256), device="cuda", dtype=torch.bfloat16)
    # ch not a multiple of 64, cout not a multiple of 256
    assert ctx.lib.mq_deconv_subpixel_bf16(ctx.handle, _lib.ptr(x), 1, 4, 4, 96, _lib.ptr(wp), None, _lib.ptr(out),
                                           256, 1, _lib.stream_ptr()) == -2
    assert ctx.lib.mq_deconv_subpixel_bf16(ctx.handle, _lib.ptr(x), 1, 4, 4, 64, _lib.ptr(wp), None, _lib.ptr(out),
                                           200, 1, _lib.stream_ptr()) == -2
