"""GPU: BASELINE config 5 as one hipGraph-captured per-frame slice (mqhip.frame_graph.FramePoseGraph):
Swin-S Mask R-CNN on every view -> static top-k crop boxes (mq_det_topk_boxes) -> UDP crop -> ViTPose
flip test -> UDP decode -> score mask -> omnidir DLT, over the reference's per-frame path
(step1_proc2d.py:226-298).

* mq_det_topk_boxes equals the host mirror of step 1 (score > thr, filter_tracks' int() truncation and
  degenerate-box filter, expand_boxes) bit for bit, empty slots included;
* graph replay equals the eager launch sequence bit for bit on every output (detections, boxes, keypoints,
  scores, 3D points), for two different frames fed through the same captured graph;
* full size (8 views x 2048x1536, full Swin-S, ViT-H): replay == eager, and the detector's backbone stages
  and FPN levels of the captured frame match the fp32 oracle (oracle/swin_det.py run on the GPU) within
  3e-2 max (the stage tolerance of tests/test_gpu_detector.py).
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _host_topk(boxes, scores, counts, k, thr):
    from src.pipeline.step1_proc2d import expand_boxes, filter_tracks
    n = boxes.shape[0]
    out = np.tile(np.array([0, 0, 192, 256], np.float32), (n * k, 1))
    tight = np.zeros((n * k, 4), np.float32)
    valid = np.zeros(n * k, np.int32)
    for i in range(n):
        c = int(counts[i])
        keep = scores[i, :c] > thr
        b, _ = filter_tracks(np.hstack([boxes[i, :c][keep], np.zeros((keep.sum(), 1))]))
        b = b[:k]
        if len(b):
            out[i * k:i * k + len(b)] = expand_boxes(b)
            tight[i * k:i * k + len(b)] = b
            valid[i * k:i * k + len(b)] = 1
    return out, tight, valid


def test_det_topk_boxes_matches_step1_host_mirror():
    import torch
    from mqhip import _lib
    from mqhip.frame_graph import DESIRED_AR, MAX_MARGIN, MIN_MARGIN
    ctx = _lib.Context.get(0)
    rng = np.random.default_rng(0)
    n, D, k, thr = 9, 100, 4, 0.6
    x1 = rng.uniform(-30, 1900, (n, D))
    y1 = rng.uniform(-30, 1400, (n, D))
    w = rng.uniform(-3, 400, (n, D))
    h = rng.uniform(-3, 500, (n, D))
    w[:, ::7] = rng.uniform(0.1, 0.9, w[:, ::7].shape)        # degenerate after int() truncation
    boxes = np.stack([x1, y1, x1 + w, y1 + h], -1).astype(np.float32)
    scores = -np.sort(-rng.uniform(0, 1, (n, D)), axis=1).astype(np.float32)
    counts = rng.integers(0, D + 1, n).astype(np.int32)
    counts[0], counts[1] = 0, 3
    b_d, s_d, c_d = (torch.from_numpy(a).cuda() for a in (boxes, scores, counts))
    ob = torch.empty((n * k, 4), device="cuda")
    ot = torch.empty((n * k, 4), device="cuda")
    oi = torch.empty((n * k,), device="cuda", dtype=torch.int32)
    ov = torch.empty((n * k,), device="cuda", dtype=torch.int32)
    _lib.check(ctx.lib.mq_det_topk_boxes(ctx.handle, _lib.ptr(b_d), _lib.ptr(s_d), _lib.ptr(c_d), n, D, k, thr,
                                         MIN_MARGIN, MAX_MARGIN, DESIRED_AR, _lib.ptr(ob), _lib.ptr(ot), _lib.ptr(oi),
                                         _lib.ptr(ov), _lib.stream_ptr()), "topk")
    torch.cuda.synchronize()
    hb, ht, hv = _host_topk(boxes, scores, counts, k, thr)
    np.testing.assert_array_equal(ov.cpu().numpy(), hv)
    np.testing.assert_array_equal(ob.cpu().numpy(), hb)
    np.testing.assert_array_equal(ot.cpu().numpy(), ht)
    np.testing.assert_array_equal(oi.cpu().numpy(), np.repeat(np.arange(n), k))
    assert hv.sum() > 0 and (hv == 0).sum() > 0
    assert ctx.lib.mq_det_topk_boxes(ctx.handle, _lib.ptr(b_d), _lib.ptr(s_d), _lib.ptr(c_d), n, D, D + 1, thr,
                                     MIN_MARGIN, MAX_MARGIN, DESIRED_AR, _lib.ptr(ob), _lib.ptr(ot), _lib.ptr(oi),
                                     _lib.ptr(ov), None) != 0


def _outputs(fg):
    dboxes, dscores, dcount = fg.det_out
    return [t.clone() for t in (dboxes, dscores, dcount, fg.boxes, fg.valid, fg.kp, fg.score, fg.argmax, fg.p3d)]


def _bits_equal(a, b):
    import torch
    return a.shape == b.shape and torch.equal(a.view(torch.uint8) if a.dtype != torch.uint8 else a,
                                              b.view(torch.uint8) if b.dtype != torch.uint8 else b)


def _slice(swin_cfg, vit_cfg, views, H, W, seed, scale=(800, 800)):
    import torch
    from mqhip import synth
    from mqhip.detector import SwinDetectorHip
    from mqhip.frame_graph import FramePoseGraph
    from mqhip.geometry import CameraGroup
    from mqhip.pose import VitPoseHip
    from mqhip.weights import make_random_weights
    from oracle import swin_det as sd
    wdet = sd.make_weights(swin_cfg, seed=seed)
    det = SwinDetectorHip(wdet, cfg=swin_cfg, device=0, scale=scale)
    pose = VitPoseHip(vit_cfg, make_random_weights(vit_cfg, seed=seed, device="cuda"), graph=False)
    cams = CameraGroup.from_dicts(synth.make_cameras(views)).cams_tensor()
    fg = FramePoseGraph(det, pose, cams, n_views=views, height=H, width=W, k=4, det_score_thr=0.0)
    rng = np.random.default_rng(seed)
    frames = [torch.from_numpy(rng.integers(0, 256, (views, H, W, 3), dtype=np.uint8)).cuda() for _ in range(2)]
    return fg, frames, wdet


def _check_replay_equals_eager(fg, frames):
    import torch
    eager = []
    for fr in frames:
        fg.eager(fr)
        torch.cuda.synchronize()
        eager.append(_outputs(fg))
    fg.capture()
    for fr, ref in zip(frames + frames[:1], eager + eager[:1]):
        fg.run(fr)
        torch.cuda.synchronize()
        got = _outputs(fg)
        for i, (a, b) in enumerate(zip(got, ref)):
            assert _bits_equal(a, b), i
    assert int(eager[0][4].sum()) > 0           # some slots hold detections
    assert not torch.equal(eager[0][5], eager[1][5])   # the two frames differ


def test_frame_graph_replay_equals_eager_small():
    from mqhip.weights import VIT_TINY
    small = dict(embed=96, depths=(2, 2, 2, 2), heads=(3, 6, 12, 24), window=7, mlp_ratio=4)
    fg, frames, _ = _slice(small, VIT_TINY, 8, 384, 512, 3, scale=(256, 256))
    _check_replay_equals_eager(fg, frames)


@pytest.mark.timeout(600)
def test_frame_graph_full_size_replay_and_detector_parity():
    import torch
    from mqhip.weights import VIT_H
    from oracle import swin_det as sd
    fg, frames, wdet = _slice(sd.SWIN_S, VIT_H, 8, 1536, 2048, 5)
    _check_replay_equals_eager(fg, frames)
    # backbone stages and FPN levels of frame 1 (the last one replayed is frame 0: re-run eagerly)
    fr = frames[1]
    _, _, _, it = fg.det.forward(fr, keep_intermediates=True)
    g = fg.det.geometry(1536, 2048)
    wd = {k: v.cuda() for k, v in wdet.items()}
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    for v in (0, 5):
        x, _, _ = sd.preprocess(fr[v].cpu().numpy())
        with torch.no_grad():
            feats = sd.swin_forward(x.cuda(), wd, sd.SWIN_S)
            P = sd.fpn_forward(feats, wd)
        for s in range(4):
            Hs, Ws = g["sizes"][s]
            got = it["outs"][s].float().view(8, Hs, Ws, -1)[v]
            exp = feats[s][0].permute(1, 2, 0)
            err = (got - exp).abs().max().item()
            assert err <= 3e-2 * exp.abs().max().item(), (v, s, err)
        for lv in range(5):
            h, w = g["levels"][lv]
            got = it["P"][lv].view(8, h, w, 256)[v]
            exp = P[lv][0].permute(1, 2, 0)
            err = (got - exp).abs().max().item()
            assert err <= 3e-2 * exp.abs().max().item(), (v, lv, err)
