"""CPU: the marker scene used by the end-to-end parity tests (mqhip/synth.py "marker scenes"): seeded ViTPose
weights that are a matched filter for two-tone joint markers.  Known-answer checks of the construction on the
fp32 oracle (oracle/vitpose.py), no GPU:
  * one isolated marker of joint j whose centre line sits between crop columns 4h+1 and 4h+2 peaks at heatmap
    pixel (row, h) in the plain forward AND, through the flip test's flip-back + FLIP_INDICES re-index, in the
    flipped forward (the flip-equivariance a trained model learns);
  * on the config-2 scene (ViT-B, a few crops) most joints have a clear top-2 margin and most peaks sit on
    their own joint's marker.
"""
import numpy as np
import pytest
import torch


def _cfg(layers):
    from mqhip.weights import VitPoseConfig
    return VitPoseConfig("b%d" % layers, 768, layers, 12, 3072)


def _crop_with_marker(j, x0, y0, sigma=4.0, amp=1.5):
    from mqhip import synth
    col = synth.marker_colours()[j] * amp
    yy, xx = np.mgrid[0:256, 0:192].astype(np.float64)
    al = np.exp(-((xx - x0) ** 2 + (yy - y0) ** 2) / (2 * sigma * sigma))
    dev = np.where((xx < x0)[..., None], col[0], col[1]) * al[..., None]        # (256, 192, 3) normalised RGB
    return torch.from_numpy(dev.transpose(2, 0, 1)[None].astype(np.float32))


@pytest.mark.parametrize("j,h,row", [(0, 20, 30), (1, 11, 17), (2, 31, 40), (9, 24, 52), (16, 7, 9)])
def test_isolated_marker_peaks_at_its_pixel_in_both_forwards(j, h, row):
    from mqhip import synth
    from oracle.vitpose import forward_flip_test
    cfg = _cfg(0)
    w = synth.marker_weights(cfg)
    x = _crop_with_marker(j, 4 * h + 1.5, 4 * row - 0.5)
    with torch.no_grad():
        avg, plain, flip_raw = forward_flip_test(x, w, cfg)
    back = flip_raw.flip(-1)[:, synth.FLIP_INDICES]
    for hm in (plain, back, avg):
        a = int(hm[0, j].argmax())
        assert (a // 48, a % 48) == (row, h)
    # every other joint's map stays below half of this joint's peak at the marker
    peak = float(avg[0, j].max())
    others = [float(avg[0, k].max()) for k in range(17) if k != j]
    assert max(others) <= 0.55 * peak


def test_marker_weights_are_bf16_exact():
    from mqhip import synth
    cfg = _cfg(2)
    w = synth.marker_weights(cfg)
    for k, v in w.items():
        assert torch.equal(v, v.to(torch.bfloat16).float()), k


def test_config2_marker_scene_peaks_on_the_joints():
    from mqhip import synth
    from oracle.crop import preprocess, topdown_crop
    from oracle.decode import decode_batch
    from oracle.postprocess import expand_boxes
    from oracle.vitpose import forward_flip_test
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(4, 1, seed=7), noise_px=0.0, drop=0.0)[:, 0]   # (A, C, J, 3)
    truth = kp2d.transpose(1, 0, 2, 3)                                                             # (C, A, J, 3)
    tight = synth.boxes_from_kp2d(truth)
    views = [0, 3, 6]
    frames = synth.render_markers(truth[views], tight[views], seed=8)
    crops, cs, ss, tru = [], [], [], []
    for k, c in enumerate(views):
        bb = expand_boxes(tight[c])
        for a in range(4):
            cu8, ctr, scl = topdown_crop(frames[k], bb[a])
            crops.append(preprocess(cu8))
            cs.append(ctr)
            ss.append(scl)
            tru.append(truth[c, a, :, :2])
    cfg = _cfg(12)
    w = synth.marker_weights(cfg)
    with torch.no_grad():
        hm = forward_flip_test(torch.from_numpy(np.stack(crops)), w, cfg)[0].numpy()
    kp, sc, am = decode_batch(hm, np.stack(cs), np.stack(ss))
    flat = hm.reshape(hm.shape[0], 17, -1)
    top2 = np.sort(flat, axis=-1)[..., -2:]
    clear = (top2[..., 1] - top2[..., 0]) / np.abs(flat).max(axis=-1) > 5e-2
    found = np.linalg.norm(kp - np.stack(tru), axis=-1) < 12.0       # frame pixels
    print(f"clear {clear.mean():.3f} found {found.mean():.3f} score median {np.median(sc):.3f}")
    assert clear.mean() >= 0.6 and found.mean() >= 0.55 and np.median(sc) >= 0.5
