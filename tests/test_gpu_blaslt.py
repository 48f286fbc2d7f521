"""hipBLASLt routing of the ViT's plain bias GEMMs (MQ_TUNE_GEMM_BLASLT, csrc/blaslt.hip).  A library kernel is
used only where its whole output on the tuning input equals the hand kernel's bit for bit (no split-K), so the
forward's heatmaps are the same bits with the route on or off: eager and graph-captured, at the bench's batch
(32 crops, flip test: M = 12,288) and at a ragged one."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

KEY = 26  # include/mq_hip.h MQ_TUNE_GEMM_BLASLT


@pytest.mark.parametrize("n", [32, 3])
def test_vit_h_forward_blaslt_route_equals_hand_kernels(n):
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
        hand = VitPoseHip(cfg, w, graph=False).forward(crops, flip_test=True).clone()
        assert ctx.lib.mq_set_tuning(KEY, 1) == 0
        model = VitPoseHip(cfg, w, graph=False)
        routed = [model.forward(crops, flip_test=True).clone() for _ in range(2)]   # the first call tunes
        gmodel = VitPoseHip(cfg, w, graph=True)
        out = torch.empty_like(hand)
        for _ in range(2):
            gmodel.forward(crops, flip_test=True, out=out)
        torch.cuda.synchronize()
    finally:
        ctx.lib.mq_set_tuning(KEY, old)
    assert torch.isfinite(hand).all()
    for r in routed:
        assert torch.equal(r, hand)
    assert torch.equal(out, hand)
    rows = 2 * n * 192
    plans = {(p["M"], p["N"], p["K"]): p for p in _lib.gemm_plans()}
    print(sorted(plans.values(), key=lambda p: (p["M"], p["N"], p["K"])))
    for shape in ((rows, 1280, 1280), (rows, 1280, 5120), (rows, 4096, 1280)):   # proj, fc2, deconv 1
        assert shape in plans, shape
        p = plans[shape]
        assert 0 <= p["bit_identical"] <= p["candidates"]
        if p["hipblaslt"]:
            assert p["bit_identical"] > 0 and 0 < p["hipblaslt_ms"] < p["hand_ms"]
