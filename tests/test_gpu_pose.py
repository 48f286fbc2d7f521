"""GPU parity: crop, ViTPose forward (bf16 MFMA) and UDP decode of libmq_hip vs the oracle."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

# bf16 heatmaps vs the fp32 oracle: max|dH| <= 2e-2 * max|H| per sample
HM_TOL = 2e-2
# share of clear joints on the seeded random ViT-H of the config-2 batch test (noise-like maps)
RANDOM_CLEAR_MIN = 0.15


def _frames_and_boxes(n_views=3, seed=0):
    from mqhip import synth
    rng = np.random.default_rng(seed)
    frames = rng.integers(0, 256, size=(n_views, 300, 400, 3), dtype=np.uint8)
    boxes = []
    frame_idx = []
    for v in range(n_views):
        for _ in range(3):
            x1, y1 = rng.uniform(-40, 350), rng.uniform(-40, 250)
            w, h = rng.uniform(10, 160), rng.uniform(10, 200)
            boxes.append([x1, y1, x1 + w, y1 + h])
            frame_idx.append(v)
    return frames, np.array(boxes, dtype=np.float32), np.array(frame_idx, dtype=np.int32)


def test_crop_bit_exact():
    import torch
    from mqhip.pose import crop_boxes
    from oracle.crop import preprocess, topdown_crop
    frames, boxes, fidx = _frames_and_boxes()
    crops, center, scale = crop_boxes(torch.from_numpy(frames).cuda(), torch.from_numpy(boxes).cuda(),
                                      torch.from_numpy(fidx).cuda())
    crops, center, scale = crops.cpu().numpy(), center.cpu().numpy(), scale.cpu().numpy()
    for i in range(len(boxes)):
        c_u8, c, s = topdown_crop(frames[fidx[i]], boxes[i])
        np.testing.assert_array_equal(center[i], c)
        np.testing.assert_array_equal(scale[i], s)
        np.testing.assert_array_equal(crops[i], preprocess(c_u8))


def _peaky_heatmaps(n, J=17, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:64, 0:48]
    hm = rng.normal(0, 0.02, (n, J, 64, 48)).astype(np.float32)
    for i in range(n):
        for k in range(J):
            cx, cy = rng.uniform(-2, 49), rng.uniform(-2, 65)
            hm[i, k] += np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * 2.0 ** 2)).astype(np.float32)
    hm[0, 3] = -np.abs(hm[0, 3])  # max <= 0 -> loc -1 + wrap-around reads
    hm[1, 0] = -np.abs(hm[1, 0])
    return hm


def test_decode_matches_oracle():
    import torch
    from mqhip.pose import decode_heatmaps
    from oracle.decode import decode_batch, udp_decode
    n = 6
    hm = _peaky_heatmaps(n)
    rng = np.random.default_rng(1)
    center = rng.uniform(100, 1500, (n, 2)).astype(np.float32)
    scale = rng.uniform(50, 400, (n, 2)).astype(np.float32)
    kp, score, am, kp_hm = decode_heatmaps(torch.from_numpy(hm).cuda(), torch.from_numpy(center).cuda(),
                                           torch.from_numpy(scale).cuda())
    rkp, rsc, ram = decode_batch(hm, center, scale)
    np.testing.assert_array_equal(am.cpu().numpy(), ram)          # bit-exact argmax
    np.testing.assert_array_equal(score.cpu().numpy(), rsc)       # peak values
    kp_hm = kp_hm.cpu().numpy()
    for i in range(n):
        from oracle.decode import refine_keypoints_dark_udp, get_heatmap_maximum
        locs, vals, _ = get_heatmap_maximum(hm[i].copy())
        ref = refine_keypoints_dark_udp(locs[None].copy(), hm[i].copy())[0]
        np.testing.assert_allclose(kp_hm[i], ref, rtol=0, atol=2e-4)
    np.testing.assert_allclose(kp.cpu().numpy(), rkp, rtol=0, atol=2e-2)


def _run_vit(cfg_name, n_crops, seed=0):
    import torch
    from mqhip.pose import VitPoseHip
    from mqhip.weights import CONFIGS, make_random_weights
    from oracle.vitpose import forward_flip_test
    cfg = CONFIGS[cfg_name]
    w = make_random_weights(cfg, seed=seed, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(seed + 1)
    crops = torch.randn((n_crops, 3, 256, 192), generator=g, device="cuda", dtype=torch.float32)
    model = VitPoseHip(cfg, w, graph=False)
    got = model.forward(crops, flip_test=True)
    torch.cuda.synchronize()
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        ref, _, _ = forward_flip_test(crops, w, cfg)
    return got.float().cpu().numpy(), ref.float().cpu().numpy()


@pytest.mark.parametrize("cfg_name,n", [("tiny", 3), ("base", 2), ("huge", 2)])
def test_vitpose_heatmaps_vs_fp32_oracle(cfg_name, n):
    got, ref = _run_vit(cfg_name, n)
    assert np.all(np.isfinite(got))
    for i in range(n):
        scale = np.abs(ref[i]).max()
        err = np.abs(got[i] - ref[i]).max()
        assert err <= HM_TOL * scale, f"{cfg_name} sample {i}: max|d|={err:.3e} vs {HM_TOL}*{scale:.3e}"


def test_vitpose_graph_replay_matches_eager():
    import torch
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_TINY, make_random_weights
    w = make_random_weights(VIT_TINY, seed=3, device="cuda")
    crops = torch.randn((4, 3, 256, 192), device="cuda")
    eager = VitPoseHip(VIT_TINY, w, graph=False).forward(crops).clone()
    model = VitPoseHip(VIT_TINY, w, graph=True)
    out = torch.empty_like(eager)
    for _ in range(3):
        model.forward(crops, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


@pytest.mark.parametrize("cfg_name,n", [("tiny", 3), ("huge", 32)])
def test_vitpose_qkv_head_major_matches_row_major(cfg_name, n):
    """The qkv GEMM writing Q / K / V head-major (MQ_TUNE_QKV_HEAD_MAJOR = 1, the attention then reads each
    head's rows contiguously) gives the heatmaps of the row-major layout bit for bit; n = 32 takes the ViT-H
    qkv GEMM through the ping-pong kernel, n = 3 through the small-tile kernel."""
    import torch
    from mqhip import _lib
    from mqhip.pose import VitPoseHip
    from mqhip.weights import CONFIGS, make_random_weights
    cfg = CONFIGS[cfg_name]
    w = make_random_weights(cfg, seed=5, device="cuda")
    crops = torch.randn((n, 3, 256, 192), device="cuda")
    model = VitPoseHip(cfg, w, graph=False)
    ctx = _lib.Context.get(0)
    old = ctx.lib.mq_get_tuning(20)
    outs = []
    try:
        for hm in (0, 1):
            assert ctx.lib.mq_set_tuning(20, hm) == 0
            outs.append(model.forward(crops).clone())
    finally:
        ctx.lib.mq_set_tuning(20, old)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])


def test_topdown_end_to_end_vs_oracle():
    """crop -> ViT-tiny (flip) -> decode; argmax exact wherever the top-2 margin is clear."""
    import torch
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_TINY, make_random_weights
    from oracle.crop import preprocess, topdown_crop
    from oracle.decode import decode_batch
    from oracle.vitpose import forward_flip_test
    frames, boxes, fidx = _frames_and_boxes(seed=4)
    w = make_random_weights(VIT_TINY, seed=5, device="cuda")
    model = VitPoseHip(VIT_TINY, w, graph=False)
    kp, score, am = model.topdown(torch.from_numpy(frames).cuda(), torch.from_numpy(boxes).cuda(),
                                  torch.from_numpy(fidx).cuda())
    crops, cs, ss = [], [], []
    for i in range(len(boxes)):
        c_u8, c, s = topdown_crop(frames[fidx[i]], boxes[i])
        crops.append(preprocess(c_u8))
        cs.append(c)
        ss.append(s)
    x = torch.from_numpy(np.stack(crops)).cuda()
    with torch.no_grad():
        ref_hm, _, _ = forward_flip_test(x, w, VIT_TINY)
    ref_hm = ref_hm.cpu().numpy()
    rkp, rsc, ram = decode_batch(ref_hm, np.stack(cs), np.stack(ss))
    am = am.cpu().numpy()
    flat = ref_hm.reshape(ref_hm.shape[0], ref_hm.shape[1], -1)
    top2 = np.sort(flat, axis=-1)[..., -2:]
    margin = (top2[..., 1] - top2[..., 0]) / np.abs(flat).max(axis=-1)
    clear = margin > 5e-2
    assert clear.sum() > 0
    np.testing.assert_array_equal(am[clear], ram[clear])


def test_vitpose_h_config2_batch_vs_fp32_oracle():
    """BASELINE config 2 at the bench's own batch: one frame of 8 views at 2048x1536 x 4 individuals =
    32 crops through ``VitPoseHip.topdown`` (UDP crop -> ViT-H flip test = 64 forwards -> decode), the
    shapes that route every ViT-H GEMM through the 256x256 ping-pong kernel, the head-major qkv, the
    64-image attention and the sub-pixel deconv.  All 32 flip-averaged heatmaps vs the fp32 oracle
    (oracle/vitpose.py, run on the GPU with TF32 off) on the same crops: max|dH| <= 2e-2 max|H| per crop;
    the decoded argmax equals the oracle's wherever the oracle's top-2 margin exceeds 5e-2 max|H|
    (model/pose/...macaque.py:54-110, step1_proc2d.py:294-298)."""
    import torch
    from mqhip import synth
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_H, make_random_weights
    from oracle.decode import decode_batch
    from oracle.vitpose import forward_flip_test
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(4, 1, seed=7), noise_px=0.0, drop=0.0)   # (A, 1, C, J, 3)
    frames = synth.make_frames(8, kp2d[:, 0].transpose(1, 0, 2, 3), seed=8)
    boxes = synth.expand_boxes(synth.boxes_from_kp2d(kp2d[:, 0].transpose(1, 0, 2, 3)).reshape(-1, 4))
    fidx = np.repeat(np.arange(8, dtype=np.int32), 4)
    w = make_random_weights(VIT_H, seed=11, device="cuda")
    model = VitPoseHip(VIT_H, w, graph=True)
    fr = torch.from_numpy(frames).cuda()
    crops, center, scale = model.crop(fr, torch.from_numpy(boxes).cuda(), torch.from_numpy(fidx).cuda())
    hm = model.forward(crops, flip_test=True)
    kp, score, am, _ = model.decode(hm, center, scale)
    kp_t, score_t, am_t = model.topdown(fr, torch.from_numpy(boxes).cuda(), torch.from_numpy(fidx).cuda())
    torch.cuda.synchronize()
    assert torch.equal(am, am_t) and torch.equal(score, score_t) and torch.equal(kp, kp_t)
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        ref, _, _ = forward_flip_test(crops, w, VIT_H)
    got, ref = hm.float().cpu().numpy(), ref.float().cpu().numpy()
    assert got.shape == (32, 17, 64, 48)
    for i in range(32):
        s = np.abs(ref[i]).max()
        err = np.abs(got[i] - ref[i]).max()
        assert err <= HM_TOL * s, f"crop {i}: max|d|={err:.3e} vs {HM_TOL}*{s:.3e}"
    rkp, rsc, ram = decode_batch(ref, center.cpu().numpy(), scale.cpu().numpy())
    flat = ref.reshape(32, 17, -1)
    top2 = np.sort(flat, axis=-1)[..., -2:]
    clear = (top2[..., 1] - top2[..., 0]) / np.abs(flat).max(axis=-1) > 5e-2
    # seeded random weights give noise-like maps: few joints have a clear top-2 margin, and every one of
    # them must decode to the oracle's argmax; the keypoint tolerance on realistic peaks is the marker-scene
    # test below (test_vitpose_h_config2_marker_keypoints)
    print(f"random-weight heatmaps: clear fraction {clear.mean():.3f}")
    assert clear.mean() >= RANDOM_CLEAR_MIN
    np.testing.assert_array_equal(am.cpu().numpy()[clear], ram[clear])


# Stated tolerances of the config-2 keypoint test below (marker scene, see mqhip/synth.py "marker scenes"):
KP_CLEAR_MIN = 0.6       # share of (crop, joint) whose top-2 heatmap margin exceeds 5e-2 max|H|
KP_TOL_PX = 0.5          # image-space keypoint tolerance on clear, Taylor-regime joints
KP_TAYLOR_MIN = 0.3      # share of (crop, joint) that is clear AND whose DARK step stays in half a cell


def test_vitpose_h_config2_marker_keypoints():
    """Config 2 (8 views x 4 individuals, ViTPose-H, flip test) on a marker scene, where the heatmaps have one
    smooth peak per joint as a trained model's do: the HIP path (crop -> bf16 forward ->
    decode) against the oracle (crop -> fp32 forward on the GPU, TF32 off -> decode).  Stated: the clear
    fraction is at least KP_CLEAR_MIN; the argmax is bit-exact on every clear joint; keypoints agree within
    KP_TOL_PX on clear joints whose DARK step stays inside half a heatmap cell (step1_proc2d.py:294-312,
    model/pose/...macaque.py:4-14)."""
    import torch
    from mqhip import synth
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_H
    from oracle.decode import decode_batch
    from oracle.vitpose import forward_flip_test
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(4, 1, seed=7), noise_px=0.0, drop=0.0)   # (A, 1, C, J, 3)
    tight = synth.boxes_from_kp2d(kp2d[:, 0].transpose(1, 0, 2, 3))                          # (C, A, 4)
    frames = synth.render_markers(kp2d[:, 0].transpose(1, 0, 2, 3), tight, seed=8)
    boxes = synth.expand_boxes(tight.reshape(-1, 4))
    fidx = np.repeat(np.arange(8, dtype=np.int32), 4)
    w = synth.marker_weights(VIT_H, device="cuda")
    model = VitPoseHip(VIT_H, w, graph=True)
    fr = torch.from_numpy(frames).cuda()
    crops, center, scale = model.crop(fr, torch.from_numpy(boxes).cuda(), torch.from_numpy(fidx).cuda())
    hm = model.forward(crops, flip_test=True)
    kp, score, am, _ = model.decode(hm, center, scale)
    torch.cuda.synchronize()
    prev = (torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32)
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    try:
        with torch.no_grad():
            ref, _, _ = forward_flip_test(crops, w, VIT_H)
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = prev
    got, ref = hm.float().cpu().numpy(), ref.float().cpu().numpy()
    for i in range(32):
        assert np.abs(got[i] - ref[i]).max() <= HM_TOL * np.abs(ref[i]).max()
    cs, ss = center.cpu().numpy(), scale.cpu().numpy()
    rkp, rsc, ram = decode_batch(ref, cs, ss)
    flat = ref.reshape(32, 17, -1)
    top2 = np.sort(flat, axis=-1)[..., -2:]
    clear = (top2[..., 1] - top2[..., 0]) / np.abs(flat).max(axis=-1) > 5e-2
    print(f"clear fraction {clear.mean():.3f}")
    assert clear.mean() >= KP_CLEAR_MIN
    np.testing.assert_array_equal(am.cpu().numpy()[clear], ram[clear])
    # Taylor regime: the oracle's DARK step stays within half a heatmap cell of its argmax cell
    cell = np.stack([ram % 48 / 47.0, ram // 48 / 63.0], axis=-1) * ss[:, None] + cs[:, None] - 0.5 * ss[:, None]
    taylor = np.abs(rkp - cell).max(axis=-1) <= 0.5 * ss.max(axis=-1)[:, None] / 63.0
    ok = clear & taylor
    dall = np.abs(kp.cpu().numpy().astype(np.float64) - rkp).max(axis=-1)
    d = dall[ok]
    print(f"clear+taylor {ok.mean():.3f}; max |dkp| {d.max():.4f} px; p99 {np.percentile(d, 99):.4f} px; "
          f"all clear joints: max {dall[clear].max():.4f} px, p99 {np.percentile(dall[clear], 99):.4f} px")
    assert ok.mean() >= KP_TAYLOR_MIN and d.max() <= KP_TOL_PX
    np.testing.assert_allclose(score.cpu().numpy()[clear], rsc[clear], rtol=HM_TOL)


# precision budget of the round-4 residual path (bf16 branch outputs added in the LayerNorm passes) against the
# f32 read-modify-write epilogues of rounds 1-3 (MQ_TUNE_VIT_RESID_F32), full-scale random-weight ViT-H
# (tools/precision_ab.py, profiles/r05e_precision_ab.log)
RESID_BF16_ERR_BUDGET = 1.25   # max rel heatmap error of the bf16 path <= this x the f32-epilogue path's


def test_vit_residual_precision_ab_full_scale_branches():
    """the same crops and full-scale random ViT-H weights (every residual update at its natural size)
    through both residual paths in one process, against the fp32 oracle: both within HM_TOL per crop, and the
    bf16-branch path's worst error within RESID_BF16_ERR_BUDGET of the f32-epilogue path's."""
    import torch
    from mqhip import _lib
    from mqhip.pose import VitPoseHip
    from mqhip.weights import VIT_H, make_random_weights
    from oracle.vitpose import forward_flip_test
    ctx = _lib.Context.get(0)
    w = make_random_weights(VIT_H, seed=3, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    crops = torch.randn((8, 3, 256, 192), generator=g, device="cuda", dtype=torch.float32)
    with torch.no_grad():
        torch.backends.cuda.matmul.allow_tf32 = False
        torch.backends.cudnn.allow_tf32 = False
        ref = forward_flip_test(crops, w, VIT_H)[0].float().cpu().numpy()
    errs = {}
    old = ctx.lib.mq_get_tuning(23)
    try:
        for knob in (1, 0):
            assert ctx.lib.mq_set_tuning(23, knob) == 0
            model = VitPoseHip(VIT_H, w, graph=False)
            got = model.forward(crops, flip_test=True).float().cpu().numpy()
            del model
            errs[knob] = np.array([np.abs(got[i] - ref[i]).max() / np.abs(ref[i]).max() for i in range(8)])
    finally:
        ctx.lib.mq_set_tuning(23, old)
    print("max rel err: f32 epilogue %.5f, bf16 branches %.5f" % (errs[1].max(), errs[0].max()))
    assert errs[1].max() <= HM_TOL and errs[0].max() <= HM_TOL
    assert errs[0].max() <= RESID_BF16_ERR_BUDGET * errs[1].max()
