"""GPU ID classifier (mqhip/resnet_id.py, csrc/resnet_id.hip) vs the oracle (oracle/resnet_id.py):
classify_patches' slice + cv2 resize and the inferencer's ResizeEdge / CenterCrop / normalisation
bit-exact; im2col / max-pool bit-exact; GAP + fc + softmax within 1e-5; the full ResNet-152 in bf16
against the fp32 restatement within the tolerance written below (parity unpinned vs mmpretrain)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def frames():
    rng = np.random.default_rng(0)
    f = rng.integers(0, 256, (2, 480, 640, 3), dtype=np.uint8)
    f[1, 100:300, 200:500] = (f[1, 100:300, 200:500] // 4 + 90)   # some smooth-ish structure
    return f


BOXES = [(0, 10, 20, 200, 300), (1, 192, 30, 640, 478), (0, 0, 0, 224, 224), (1, 5, 7, 6, 8), (0, 600, 400, 640, 480),
         (1, 17, 3, 465, 451), (0, 100, 50, 101, 470)]   # (view, x0, y0, x1, y1): any size, 2x (448), identity, 1x1


def _model(depth=152, seed=0):
    from mqhip import resnet_id as rid
    sd = rid.make_random_weights(depth, seed=seed)
    return sd, rid.ResNetIdHip(sd, depth=depth)


def test_crop_resize_and_preprocess_bit_exact(frames):
    from mqhip import resnet_id as rid
    from oracle import resnet_id as orid
    from oracle.swin_det import resize_linear_u8
    sd = rid.make_random_weights(50)
    m = rid.ResNetIdHip(sd, depth=50)
    dev = torch.as_tensor(frames).cuda()
    x, pat = m.preprocess(dev, BOXES)
    torch.cuda.synchronize()
    pat, x = pat.cpu().numpy(), x.float().cpu()
    for i, (v, x0, y0, x1, y1) in enumerate(BOXES):
        patch = frames[v, y0:y1, x0:x1]
        ref = resize_linear_u8(np.ascontiguousarray(patch), 224, 224)
        assert np.array_equal(pat[i], ref), i
        xo = orid.preprocess(patch).permute(1, 2, 0).to(torch.bfloat16).float()
        assert torch.equal(x[i], xo), i


@pytest.mark.parametrize("c,k,s,p", [(3, 7, 2, 3), (64, 3, 1, 1), (64, 3, 2, 1), (128, 1, 2, 0), (24, 3, 2, 1)])
def test_im2col_matches_unfold(c, k, s, p):
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda").manual_seed(c + k)
    n, h, w = 2, 15, 12
    x = torch.randn((n, h, w, c), generator=g, device="cuda").to(torch.bfloat16)
    kpad = (k * k * c + 31) // 32 * 32
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    out = torch.full((n * oh * ow, kpad), 7.0, device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_id_im2col(ctx.handle, _lib.ptr(x), n, h, w, c, k, k, s, p, kpad, _lib.ptr(out),
                                    _lib.stream_ptr()), "mq_id_im2col")
    cols = F.unfold(x.float().permute(0, 3, 1, 2), (k, k), padding=p, stride=s)
    ref = cols.view(n, c, k * k, -1).permute(0, 3, 2, 1).reshape(n * oh * ow, k * k * c)
    ref = F.pad(ref, (0, kpad - k * k * c))
    assert torch.equal(out.float(), ref)


def test_maxpool_and_head():
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn((3, 17, 14, 64), generator=g, device="cuda").to(torch.bfloat16)
    out = torch.empty((3, 9, 7, 64), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_id_maxpool(ctx.handle, _lib.ptr(x), 3, 17, 14, 64, _lib.ptr(out), _lib.stream_ptr()), "mp")
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(out.float(), ref)
    feat = torch.randn((3, 49, 2048), generator=g, device="cuda")
    fw = torch.randn((6, 2048), generator=g, device="cuda") * 0.02
    fb = torch.randn((6,), generator=g, device="cuda")
    lg, pr = torch.empty((3, 6), device="cuda"), torch.empty((3, 6), device="cuda")
    _lib.check(ctx.lib.mq_id_head(ctx.handle, _lib.ptr(feat), 3, 49, 2048, _lib.ptr(fw), _lib.ptr(fb), 6, _lib.ptr(lg),
                                  _lib.ptr(pr), _lib.stream_ptr()), "head")
    rl = feat.mean(1) @ fw.t() + fb
    torch.testing.assert_close(lg, rl, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(pr, torch.softmax(rl, 1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("depth", [50, 152])
def test_resnet_matches_fp32_oracle(frames, depth):
    """bf16 operands / f32 accumulation vs the fp32 restatement: logits within 3e-2 * (max |logit| + 1),
    probabilities within 2e-2, and the same label wherever the oracle's top-2 probability margin > 0.05."""
    from oracle import resnet_id as orid
    sd, m = _model(depth, seed=depth)
    dev = torch.as_tensor(frames).cuda()
    x, _ = m.preprocess(dev, BOXES)
    lg, pr = m.forward(x)
    torch.cuda.synchronize()
    xo = torch.stack([orid.preprocess(frames[v, y0:y1, x0:x1]) for v, x0, y0, x1, y1 in BOXES])
    with torch.no_grad():
        rl, rp = orid.forward(sd, xo, depth)
    lg, pr = lg.cpu(), pr.cpu()
    scale = rl.abs().max() + 1
    assert (lg - rl).abs().max() <= 3e-2 * scale, ((lg - rl).abs().max(), scale)
    assert (pr - rp).abs().max() <= 2e-2, (pr - rp).abs().max()
    top2 = rp.topk(2, dim=1).values
    sure = (top2[:, 0] - top2[:, 1]) > 0.05
    assert torch.equal(pr.argmax(1)[sure], rp.argmax(1)[sure])


def test_classify_equals_oracle_classify_patches(frames):
    """classify (all views' boxes in one batch) vs the oracle's classify_patches per view, including an empty
    slice (label -1, score 0) and a negative-start box (numpy wrap-around)."""
    from oracle import resnet_id as orid
    sd, m = _model(50, seed=7)
    boxes = [np.array([(10, 20, 200, 300), (5, 5, 5, 90), (-30, 100, 630, 400)]), np.array([(200, 100, 648, 548)])]
    got = m.classify(frames, boxes)
    for v in range(2):
        patches = [frames[v][y1:y2, x1:x2] for (x1, y1, x2, y2) in boxes[v]]
        ref = orid.classify_patches(sd, patches, depth=50)
        for a, b in zip(got[v], ref):
            assert a["pred_label"] == b["pred_label"]
            assert abs(a["pred_score"] - b["pred_score"]) <= 2e-2
    assert got[0][1] == {"pred_label": -1, "pred_score": 0.0}


def test_step1_classify_patches_and_process_frame(frames, monkeypatch):
    """step1 classify_patches(id_model, patches) (step1:140-163) with the MI355X model vs the oracle, and
    process_frame_multiview(..., id_model=...) giving every tracked box its classified id columns."""
    from oracle import resnet_id as orid
    from src.pipeline import step1_proc2d as s1
    sd, m = _model(50, seed=11)
    patches = [frames[0, 20:300, 10:200], frames[1, 0:0, 5:9], frames[1, 30:478, 192:640], frames[0, 5:6, 7:8]]
    got = s1.classify_patches(m, patches)
    ref = orid.classify_patches(sd, patches, depth=50)
    for a, b in zip(got, ref):
        assert a["pred_label"] == b["pred_label"] and abs(a["pred_score"] - b["pred_score"]) <= 2e-2
    assert got[1] == {"pred_label": -1, "pred_score": 0.0}

    from types import SimpleNamespace

    def fake_pose(model, imgs, bbs):
        return [[SimpleNamespace(pred_instances=SimpleNamespace(keypoints=np.zeros((1, 17, 2)),
                                                                keypoint_scores=np.ones((1, 17), np.float32)))
                 for _ in b] for b in bbs]
    monkeypatch.setattr(s1, "inference_topdown_batch", fake_pose)
    tracks = [np.array([[10, 20, 200, 300, 1], [300, 100, 500, 400, 2]], float), np.array([[192, 30, 640, 478, 5]], float)]
    sm = [s1.KeypointSmoother(), s1.KeypointSmoother()]
    rows = s1.process_frame_multiview(None, [frames[0], frames[1]], tracks, sm, 0, id_model=m)
    for v in range(2):
        boxes, _ = s1.filter_tracks(tracks[v])
        ref = orid.classify_patches(sd, [frames[v][y1:y2, x1:x2] for (x1, y1, x2, y2) in boxes], depth=50)
        for row, r in zip(rows[v], ref):
            assert abs(row[7] - r["pred_score"]) <= 2e-2
            if abs(r["pred_score"] - s1.ID_CONF_THR) > 2e-2:
                assert row[6] == (r["pred_label"] if r["pred_score"] >= s1.ID_CONF_THR else -1)


@pytest.mark.parametrize("n,h,w,c,k,s,p,cout,epi", [(13, 56, 56, 64, 3, 1, 1, 64, 6), (13, 56, 56, 256, 1, 2, 0, 512, 4),
                                                    (13, 56, 56, 128, 3, 2, 1, 128, 6), (13, 14, 14, 256, 3, 1, 1, 256, 6),
                                                    (3, 7, 7, 512, 3, 1, 1, 512, 0), (2, 15, 12, 64, 3, 2, 1, 24, 4)])
def test_implicit_conv_equals_im2col_gemm(n, h, w, c, k, s, p, cout, epi):
    """mq_id_conv_bf16 (the A tile of each K-step gathered from the tap-shifted input pixels, zero padding from
    out-of-range DMA offsets) gives the bits of mq_id_im2col + mq_gemm_bf16: same K order, same tiles."""
    from mqhip import _lib
    ctx = _lib.Context.get(0)
    g = torch.Generator(device="cuda").manual_seed(n + h + c + k + s)
    x = torch.randn((n, h, w, c), generator=g, device="cuda").to(torch.bfloat16)
    wt = (torch.randn((cout, k * k * c), generator=g, device="cuda") / (k * c ** 0.5)).to(torch.bfloat16)
    bias = torch.randn((cout,), generator=g, device="cuda")
    oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    M = n * oh * ow
    dt = torch.float32 if epi == 4 else torch.bfloat16
    got = torch.empty((M, cout), device="cuda", dtype=dt)
    _lib.check(ctx.lib.mq_id_conv_bf16(ctx.handle, _lib.ptr(x), n, h, w, c, k, s, p, _lib.ptr(wt), _lib.ptr(bias),
                                       _lib.ptr(got), cout, epi, _lib.stream_ptr()), "mq_id_conv_bf16")
    cols = torch.empty((M, k * k * c), device="cuda", dtype=torch.bfloat16)
    _lib.check(ctx.lib.mq_id_im2col(ctx.handle, _lib.ptr(x), n, h, w, c, k, k, s, p, k * k * c, _lib.ptr(cols),
                                    _lib.stream_ptr()), "mq_id_im2col")
    ref = torch.empty_like(got)
    # the explicit GEMM takes the 256x256 kernels at large M x N; the implicit one always the 128 / 64 tiles
    big = ((M + 255) // 256) * ((cout + 255) // 256) >= 128 and cout >= 256
    old = ctx.lib.mq_get_tuning(2)
    try:
        assert ctx.lib.mq_set_tuning(2, 1) == 0   # the explicit GEMM on the same small-tile kernel
        _lib.check(ctx.lib.mq_gemm_bf16(ctx.handle, _lib.ptr(cols), _lib.ptr(wt), _lib.ptr(ref), _lib.ptr(bias), None,
                                        M, cout, k * k * c, k * k * c, k * k * c, cout, 0, epi, _lib.stream_ptr()),
                   "gemm")
    finally:
        ctx.lib.mq_set_tuning(2, old)
    torch.cuda.synchronize()
    assert torch.equal(got, ref), (big, (got.float() - ref.float()).abs().max().item())


def test_classifier_implicit_conv_matches_im2col(frames):
    """The whole ResNet-152 forward with the implicit convolutions equals the im2col path bit for bit."""
    _, m = _model(152, seed=1)
    dev = torch.as_tensor(frames).cuda()
    x, _ = m.preprocess(dev, BOXES)
    outs = []
    for implicit in (False, True):
        m.implicit_conv = implicit
        outs.append([t.clone() for t in m.forward(x)])
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
