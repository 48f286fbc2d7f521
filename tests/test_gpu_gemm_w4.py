"""GPU: the one-wave-per-SIMD 256x256 GEMM (csrc/gemm_w4.hip, MQ_TUNE_GEMM_W4 = key 27) against the ping-pong
kernel.  Both accumulate every output in the same order (32-deep MFMA steps in ascending K, then bias, then the
epilogue op), so the bf16 outputs must be the same bits: plain, GELU and ReLU epilogues, full and ragged tiles,
one-round and multi-tile persistent walks; and the whole ViT-H forward (whose qkv GEMM stores head-major) must give
the same heatmaps with the kernel on and off, eager and graph-replayed."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

KEY = 27  # include/mq_hip.h MQ_TUNE_GEMM_W4


def _run_routes(M, N, K, epi, seed=0, variant=1):
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    outs = []
    old = ctx.lib.mq_get_tuning(KEY)
    try:
        for w4 in (0, variant):
            assert ctx.lib.mq_set_tuning(KEY, w4) == 0
            Cm = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
            _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), _lib.ptr(bias), None,
                                            M, N, K, K, K, N, 0, epi, _lib.stream_ptr()), "mq_gemm_bf16")
            outs.append(Cm)
    finally:
        ctx.lib.mq_set_tuning(KEY, old)
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t() + bias
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    elif epi == 6:
        ref = ref.clamp_min(0)
    return outs, ref, (A.float().abs() @ W.float().abs().t()).max().item() + 1.0


@pytest.mark.parametrize("epi", [0, 1, 6])
@pytest.mark.parametrize("M,N,K", [(12288, 1280, 1280), (12288, 3840, 1280), (12288, 5120, 1280), (12288, 1280, 5120),
                                   (12288, 4096, 1280), (700, 512, 320), (4196, 2056, 192), (3000, 1280, 5120),
                                   (256, 256, 128), (1000, 264, 2048)])
@pytest.mark.parametrize("variant", [1, 2], ids=["dma", "vgpr"])
def test_gemm_w4_bitwise_equals_pingpong(epi, M, N, K, variant):
    import torch
    (pp, w4), ref, scale = _run_routes(M, N, K, epi, variant=variant)
    assert torch.equal(pp.view(torch.int16), w4.view(torch.int16))
    err = (w4.float() - ref).abs().max().item()
    assert err <= 2e-3 * scale + 0.01 * scale, (err, scale)


@pytest.mark.parametrize("variant", [1, 2], ids=["dma", "vgpr"])
@pytest.mark.parametrize("n", [32, 3])
def test_vit_h_forward_w4_equals_pingpong(n, variant):
    import torch
    from mqhip import _lib
    from mqhip.pose import VitPoseHip
    from mqhip.weights import CONFIGS, make_random_weights
    cfg = CONFIGS["huge"]
    w = make_random_weights(cfg, seed=11, device="cuda")
    crops = torch.randn((n, 3, 256, 192), device="cuda")
    ctx = _lib.Context.get(0)
    old = ctx.lib.mq_get_tuning(KEY)
    try:
        assert ctx.lib.mq_set_tuning(KEY, 0) == 0
        pp = VitPoseHip(cfg, w, graph=False).forward(crops, flip_test=True).clone()
        assert ctx.lib.mq_set_tuning(KEY, variant) == 0
        eager = VitPoseHip(cfg, w, graph=False).forward(crops, flip_test=True).clone()
        gmodel = VitPoseHip(cfg, w, graph=True)
        out = torch.empty_like(pp)
        for _ in range(2):
            gmodel.forward(crops, flip_test=True, out=out)
        torch.cuda.synchronize()
    finally:
        ctx.lib.mq_set_tuning(KEY, old)
    assert torch.isfinite(pp).all()
    assert torch.equal(eager, pp)
    assert torch.equal(out, pp)
