"""GPU numerics of the bf16 MFMA GEMM building block (mq_gemm_bf16) vs a PyTorch fp32 reference.

Inputs are bf16; the reference multiplies the same bf16 values in fp32 (torch matmul
with TF32 off), so only the accumulation order differs: tolerance 2e-3 relative to
the row's |A||W| scale, plus bf16 output rounding where the epilogue emits bf16.
"""
import ctypes as C

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _run(M, N, K, epi, aux_rows=0, seed=0):
    import torch
    from mqhip import _lib
    torch.backends.cuda.matmul.allow_tf32 = False
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    ref = A.float() @ W.float().t() + bias
    aux = None
    if epi in (0, 1):
        Cm = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
    elif epi == 2:
        Cm = torch.randn((M, N), generator=g, device="cuda")
        ref = ref + Cm
    elif epi == 3:
        aux = torch.randn((aux_rows, N), generator=g, device="cuda")
        ref = ref + aux[torch.arange(M, device="cuda") % aux_rows]
        Cm = torch.empty((M, N), device="cuda")
    elif epi == 4:
        Cm = torch.empty((M, N), device="cuda")
    else:
        Cm = torch.empty((M // aux_rows, N, aux_rows), device="cuda")
        ref = ref.view(M // aux_rows, aux_rows, N).permute(0, 2, 1)
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    rc = ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), _lib.ptr(bias), _lib.ptr(aux), M, N,
                              K, K, K, N, aux_rows, epi, _lib.stream_ptr())
    _lib.check(rc, "mq_gemm_bf16")
    torch.cuda.synchronize()
    scale = (A.float().abs() @ W.float().abs().t()).max().item() + 1.0
    err = (Cm.float() - ref).abs().max().item()
    return err, scale


@pytest.fixture(params=[(0, 0), (1, 0)], ids=["interleaved", "pingpong"])
def staging(request):
    """Both 256x256 kernels: the interleaved-K-step kernel (gemm_bf16.hip gemm256_kernel) and the
    ping-pong kernel (gemm_pp.hip), selected by MQ_TUNE_GEMM_PINGPONG (key 12)."""
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    keys = (12, 2)
    old = [ctx.lib.mq_get_tuning(k) for k in keys]
    for k, v in zip(keys, (request.param[0], 0)):
        assert ctx.lib.mq_set_tuning(k, v) == 0
    yield request.param
    for k, v in zip(keys, old):
        ctx.lib.mq_set_tuning(k, v)


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4])
def test_gemm_256_path_all_epilogues(epi, staging):
    err, scale = _run(700, 512, 320, epi, aux_rows=192)
    tol = 2e-3 * scale + (0.01 * scale if epi in (0, 1) else 0.0)
    assert err <= tol, (err, tol)


@pytest.mark.parametrize("M,N,K", [(12288, 1280, 1280), (1024, 3840, 1280), (512, 5120, 256), (4196, 5120, 256)])
def test_gemm_vit_shapes(M, N, K, staging):
    err, scale = _run(M, N, K, 4)
    assert err <= 2e-3 * scale


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("M,N", [(12288, 1280), (1000, 1280), (4196, 5120)])
def test_gemm_tile_rows_default_policy(epi, M, N):
    """Default policy (256x256 tiles, interleaved K-step) on narrow (one tile per CU) and wide
    grids: every epilogue, ragged M, residual read-modify-write."""
    err, scale = _run(M, N, 256, epi, aux_rows=192)
    tol = 2e-3 * scale + (0.01 * scale if epi in (0, 1) else 0.0)
    assert err <= tol, (err, tol)


def _run_pair(M, N, K, epi, aux_rows, seed=0):
    """The same GEMM through the interleaved-K-step kernel and the ping-pong kernel."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") * 0.05).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    aux = torch.randn((aux_rows, N), generator=g, device="cuda")
    C0 = torch.randn((M, N), generator=g, device="cuda")
    if epi in (0, 1, 6):
        C0 = C0.to(torch.bfloat16)
    outs = []
    old = ctx.lib.mq_get_tuning(12)
    try:
        for pp in (0, 1):
            assert ctx.lib.mq_set_tuning(12, pp) == 0
            Cm = C0.clone()
            _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), _lib.ptr(bias),
                                            _lib.ptr(aux), M, N, K, K, K, N, aux_rows, epi, _lib.stream_ptr()),
                       "mq_gemm_bf16")
            outs.append(Cm)
    finally:
        ctx.lib.mq_set_tuning(12, old)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 6])
@pytest.mark.parametrize("M,N,K", [(12288, 1280, 1280), (700, 512, 320), (4196, 5120, 256), (2048, 3840, 1280),
                                   (1000, 1280, 2048), (3000, 1280, 5120), (4096, 2048, 64), (4196, 2056, 64),
                                   (4196, 2056, 192), (12288, 5120, 1280), (12288, 3840, 1280), (12288, 1280, 5120),
                                   (6000, 2560, 320)])
def test_gemm_pingpong_bitwise_equals_interleaved(epi, M, N, K):
    """Both kernels accumulate every output in the same order (32-deep MFMA steps in ascending K,
    then bias, then the epilogue op), so the ping-pong kernel must reproduce the other bit for bit,
    on full and ragged tiles and multi-tile persistent walks."""
    import torch
    outs = _run_pair(M, N, K, epi, aux_rows=192)
    bits = [o.view(torch.int16) if o.dtype == torch.bfloat16 else o.view(torch.int32) for o in outs]
    assert torch.equal(bits[0], bits[1])


def test_gemm_force_small_matches_fp32():
    """MQ_TUNE_GEMM_FORCE_SMALL routes every GEMM to the 128x128 kernel: still correct."""
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    old = ctx.lib.mq_get_tuning(2)
    try:
        assert ctx.lib.mq_set_tuning(2, 1) == 0
        for epi in (0, 1, 2, 4):
            err, scale = _run(700, 512, 320, epi)
            assert err <= 2e-3 * scale + (0.01 * scale if epi in (0, 1) else 0.0)
    finally:
        ctx.lib.mq_set_tuning(2, old)


def test_gemm_small_path_nchw():
    err, scale = _run(2 * 3072, 17, 256, 5, aux_rows=3072)
    assert err <= 2e-3 * scale


def test_gemm_small_path_narrow():
    err, scale = _run(300, 128, 128, 4)
    assert err <= 2e-3 * scale


def test_gemm_rejects_bad_k():
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    A = torch.zeros((64, 40), device="cuda", dtype=torch.bfloat16)
    W = torch.zeros((64, 40), device="cuda", dtype=torch.bfloat16)
    Cm = torch.zeros((64, 64), device="cuda")
    rc = ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), None, None, 64, 64, 40, 40, 40, 64,
                              0, 4, _lib.stream_ptr())
    assert rc != 0


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("M,N,K", [(2548, 256, 2304), (637, 512, 4608), (2548, 1024, 256), (100, 2048, 512),
                                   (1000, 96, 320), (50, 17, 1024)])
def test_gemm_tile64_bitwise_equals_tile128(epi, M, N, K):
    """GEMMs too small to occupy every CU with 128x128 tiles (the ID classifier's stage-3/4 convolutions
    at a frame's dozen boxes) run on 64x64 tiles: same K order per output, so the bits of the 128x128
    kernel (MQ_TUNE_GEMM_TILE64 = 0), and within the bf16 tolerance of the fp32 product."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(M + N + K)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    aux_rows = 7 if epi == 5 else 3
    aux = torch.randn((aux_rows, N), generator=g, device="cuda")
    C0 = torch.randn((M, N), generator=g, device="cuda")
    if epi in (0, 1, 6):
        C0 = C0.to(torch.bfloat16)
    if epi == 5:
        M = (M // aux_rows) * aux_rows
        A, C0 = A[:M].contiguous(), torch.zeros((M, N), device="cuda")
    outs = []
    old = ctx.lib.mq_get_tuning(19)
    try:
        for t64 in (0, 1):
            assert ctx.lib.mq_set_tuning(19, t64) == 0
            Cm = C0.clone()
            _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(Cm), _lib.ptr(bias),
                                            _lib.ptr(aux), M, N, K, K, K, N, aux_rows, epi, _lib.stream_ptr()),
                       "mq_gemm_bf16")
            outs.append(Cm)
    finally:
        ctx.lib.mq_set_tuning(19, old)
    torch.cuda.synchronize()
    bits = [o.view(torch.int16) if o.dtype == torch.bfloat16 else o.view(torch.int32) for o in outs]
    assert torch.equal(bits[0], bits[1])
    prod = A.float() @ W.float().t() + bias
    if epi == 1:
        prod = torch.nn.functional.gelu(prod)
    elif epi == 6:
        prod = prod.clamp_min(0)
    elif epi == 2:
        prod = prod + C0
    elif epi == 3:
        prod = prod + aux[torch.arange(M, device="cuda") % aux_rows]
    got = outs[1].float()
    if epi == 5:  # NCHW: out[img][n][pix]
        got = got.view(M // aux_rows, N, aux_rows).permute(0, 2, 1).reshape(M, N)
    tol = 2e-3 * prod.abs().max().item() + (0.01 * prod.abs().max().item() if epi in (0, 1, 6) else 0.0)
    assert (got - prod).abs().max().item() <= tol


@pytest.mark.parametrize("M,N,K", [(2548, 1024, 256), (637, 2048, 512), (40768, 256, 64), (100, 512, 128)])
def test_gemm_resid_relu_equals_resid_then_relu(M, N, K):
    """mq_gemm_resid_relu_bf16 (ResNet bottleneck conv3 + identity + ReLU in one epilogue) gives the bits of
    the residual GEMM followed by the separate ReLU pass (mq_id_relu_bf16) it replaces."""
    import torch
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(M * 7 + N + K)
    A = torch.randn((M, K), generator=g, device="cuda").to(torch.bfloat16)
    W = (torch.randn((N, K), generator=g, device="cuda") / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g, device="cuda")
    X0 = torch.randn((M, N), generator=g, device="cuda")
    X1, X2 = X0.clone(), X0.clone()
    out1 = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
    out2 = torch.empty_like(out1)
    s = _lib.stream_ptr()
    _lib.check(ctx.lib.mq_gemm_resid_relu_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(X1), _lib.ptr(bias),
                                               _lib.ptr(out1), M, N, K, K, K, N, s), "fused")
    _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(A), _lib.ptr(W), _lib.ptr(X2), _lib.ptr(bias), None, M, N, K,
                                    K, K, N, 0, 2, s), "resid")
    _lib.check(ctx.lib.mq_id_relu_bf16(ctx.handle, _lib.ptr(X2), _lib.ptr(out2), X2.numel(), s), "relu")
    torch.cuda.synchronize()
    ref = (X0 + A.float() @ W.float().t() + bias).clamp_min(0)
    assert (X1 - ref).abs().max().item() <= 2e-3 * ref.abs().max().item()
    # the separate path may take the 256x256 kernels at large M (same K order): bit-equal wherever both ran
    # the 128x128 / 64x64 kernel, else within rounding
    if ((M + 255) // 256) * ((N + 255) // 256) < 128:
        assert torch.equal(X1, X2) and torch.equal(out1, out2)
    else:
        assert (X1 - X2).abs().max().item() <= 1e-5 * ref.abs().max().item()
