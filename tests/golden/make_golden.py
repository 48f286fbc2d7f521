"""Generate the committed golden fixtures under tests/golden/ from the oracle.

The reference ships no tests, golden vectors or fixtures and
its Python could not be executed here, so these vectors
are produced by the oracle restatement on seeded synthetic inputs.  They pin the
oracle against regressions; known-answer tests in tests/test_oracle_kat.py pin
its semantics.  Regenerate with:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "macaque-3d-pose-estimation_amd"))


def geometry():
    from mqhip import synth
    from mqhip.geometry import OmnidirCamera
    from oracle.geometry import CameraGroupOracle
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(2, 4)
    kp2d = synth.make_kp2d(cams, skel, seed=7)
    o = CameraGroupOracle(cams)
    A, F, C, J, _ = kp2d.shape
    p = kp2d.transpose(2, 0, 1, 3, 4).reshape(C, -1, 3)
    pts = p[..., :2].copy()
    pts[p[..., 2] < 0.5] = np.nan
    pts[:, 0] = np.nan
    pts[1:, 1] = np.nan
    rows = np.stack([OmnidirCamera.from_dict(c).param_row() for c in cams])
    p3 = o.triangulate(pts)
    r3, rpk, rp2, rerr = o.triangulate_ransac(pts)
    np.savez_compressed(os.path.join(HERE, "geometry.npz"), cam_rows=rows, skel=skel, pts=pts,
                        project=o.project(skel.reshape(-1, 3)), undistort=o.undistort(pts), dlt=p3,
                        reproj_mean=o.reprojection_error(p3, pts, mean=True), ransac_p3d=r3, ransac_picked=rpk,
                        ransac_p2d=rp2, ransac_err=rerr,
                        K=np.stack([c["K"] for c in cams]), xi=np.stack([c["xi"] for c in cams]),
                        D=np.stack([c["D"] for c in cams]), rvec=np.stack([c["rvec"] for c in cams]),
                        tvec=np.stack([c["tvec"] for c in cams]))


def viterbi():
    from mqhip import synth
    from oracle.viterbi import step4_filter
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(1, 30)
    kp2d = synth.make_kp2d(cams, skel, drop=0.3, seed=11)[:, :, :3]
    kp2d[0, 5:9, 1, 2] = 0
    kp2d[0, 12, 0, 4, :2] += 300
    out = step4_filter(kp2d)
    np.savez_compressed(os.path.join(HERE, "viterbi.npz"), kp2d=kp2d, kp2d_f=out)


def decode():
    from oracle.decode import decode_batch
    rng = np.random.default_rng(21)
    yy, xx = np.mgrid[0:64, 0:48]
    hm = rng.normal(0, 0.02, (2, 17, 64, 48)).astype(np.float32)
    truth = rng.uniform([2, 2], [45, 61], (2, 17, 2))
    for i in range(2):
        for k in range(17):
            cx, cy = truth[i, k]
            hm[i, k] += np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / 8.0).astype(np.float32)
    hm[1, 4] = -np.abs(hm[1, 4])
    center = np.array([[500, 400], [1200, 800]], dtype=np.float32)
    scale = np.array([[150, 200], [300, 400]], dtype=np.float32)
    kp, sc, am = decode_batch(hm, center, scale)
    np.savez_compressed(os.path.join(HERE, "decode.npz"), heatmaps=hm, center=center, scale=scale, kp=kp,
                        score=sc, argmax=am, truth=truth)


def crop():
    from oracle.crop import topdown_crop
    rng = np.random.default_rng(31)
    frame = rng.integers(0, 256, (120, 160, 3), dtype=np.uint8)
    boxes = np.array([[10, 12, 90, 110], [-20, -10, 60, 70], [100, 50, 170, 140], [40.3, 20.7, 41.9, 25.2]],
                     dtype=np.float32)
    crops, centers, scales = [], [], []
    for b in boxes:
        c, ce, s = topdown_crop(frame, b)
        crops.append(c)
        centers.append(ce)
        scales.append(s)
    crops = np.stack(crops)
    np.savez_compressed(os.path.join(HERE, "crop.npz"), frame=frame, boxes=boxes, crops_u8=crops,
                        center=np.stack(centers), scale=np.stack(scales))


def vit_tiny():
    import torch
    from mqhip.weights import VIT_TINY, make_random_weights
    from oracle.vitpose import forward_flip_test
    w = make_random_weights(VIT_TINY, seed=0, device="cpu")
    g = torch.Generator()
    g.manual_seed(1)
    x = torch.randn((1, 3, 256, 192), generator=g)
    with torch.no_grad():
        avg, _, _ = forward_flip_test(x, w, VIT_TINY)
    np.savez_compressed(os.path.join(HERE, "vit_tiny.npz"), heatmaps=avg.numpy())


if __name__ == "__main__":
    geometry()
    viterbi()
    decode()
    crop()
    vit_tiny()
    print("golden fixtures written to", HERE)
