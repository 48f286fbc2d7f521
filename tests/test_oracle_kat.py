"""CPU: known-answer tests that pin the oracle's semantics (no GPU, no reference execution).

The reference ships no tests or fixtures, so the oracle is
pinned by first-principles answers: noise-free projections triangulate back
exactly, reprojection error vanishes on consistent data, Viterbi leaves a clean
track unchanged, a sampled Gaussian decodes at its centre, and crops of constant
or integer-shifted images come out exact.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def scene():
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(2, 5)
    return cams, skel, CameraGroupOracle(cams)


def test_noise_free_dlt_recovers_truth(scene):
    cams, skel, o = scene
    X = skel.reshape(-1, 3)
    np.testing.assert_allclose(o.triangulate(o.project(X)), X, rtol=0, atol=1e-6)


def test_undistort_is_pinhole_normalisation(scene):
    """undistort(project(X)) == (R X + t)_xy / z: the form the [R|t] DLT assumes (row a11)."""
    cams, skel, o = scene
    X = skel.reshape(-1, 3)
    uv = o.project(X)
    und = o.undistort(uv)
    for c, cam in enumerate(o.cameras):
        M = cam.extrinsics_mat()
        Xc = X @ M[:3, :3].T + M[:3, 3]
        np.testing.assert_allclose(und[c], Xc[:, :2] / Xc[:, 2:3], rtol=0, atol=1e-12)


def test_reprojection_error_zero_on_consistent_data(scene):
    cams, skel, o = scene
    X = skel.reshape(-1, 3)
    uv = o.project(X)
    e = o.reprojection_error(X, uv, mean=True)
    assert np.nanmax(np.abs(e)) < 1e-9
    # fewer than 2 cameras -> NaN (denom < 1.5)
    uv1 = uv.copy()
    uv1[1:] = np.nan
    assert np.all(np.isnan(o.reprojection_error(X, uv1, mean=True)))


def test_ransac_noise_free_uses_all_cameras(scene):
    cams, skel, o = scene
    X = skel.reshape(-1, 3)[:6]
    uv = o.project(X)
    p3, picked, p2, err = o.triangulate_ransac(uv)
    np.testing.assert_allclose(p3, X, atol=1e-6)
    assert picked.all()            # first subset (all cameras) is already below 0.5 px
    assert np.all(err < 1e-6)


def test_ransac_edge_cases(scene):
    cams, skel, o = scene
    uv = o.project(skel.reshape(-1, 3)[:3])
    uv[:, 0] = np.nan              # seen by nobody
    uv[1:, 1] = np.nan             # seen by one camera
    p3, picked, p2, err = o.triangulate_ransac(uv)
    assert np.all(np.isnan(p3[:2])) and np.all(err[:2] == 0) and not picked[:, :2].any()
    assert np.isfinite(p3[2]).all()


def test_viterbi_keeps_clean_track():
    from oracle.viterbi import viterbi_path
    F = 50
    t = np.arange(F)
    pts = np.stack([100 + 3.0 * t, 200 + 2.0 * np.sin(t / 5)], axis=1)[:, None, :]
    sc = np.full((F, 1), 0.9)
    out, scores, idx = viterbi_path(pts.copy(), sc.copy(), n_back=3, thres_dist=25, return_indices=True)
    np.testing.assert_array_equal(out, pts[:, 0])
    assert np.all(idx == 0)


def test_viterbi_bridges_gap_with_older_particle():
    from oracle.viterbi import viterbi_path
    F = 20
    pts = np.stack([np.linspace(0, 40, F), np.zeros(F)], axis=1)[:, None, :]
    sc = np.full((F, 1), 0.9)
    pts[10] = np.nan
    out, scores, idx = viterbi_path(pts.copy(), sc.copy(), n_back=3, thres_dist=25, return_indices=True)
    # frame 10 re-uses frame 9's point (particle index 0 at frame 10 = frame 9 with score / 2)
    np.testing.assert_array_equal(out[10], pts[9, 0])
    assert scores[10] == pytest.approx(0.45)


def test_viterbi_missing_everywhere():
    from oracle.viterbi import viterbi_path
    pts = np.full((5, 1, 2), np.nan)
    out, scores = viterbi_path(pts, np.zeros((5, 1)), 3, 25)
    np.testing.assert_array_equal(out, -1)
    np.testing.assert_array_equal(scores, 0.001)


def test_decode_recovers_gaussian_centre():
    from oracle.decode import udp_decode
    yy, xx = np.mgrid[0:64, 0:48]
    cx, cy = 20.3, 31.7
    hm = np.zeros((17, 64, 48), dtype=np.float32)
    hm[:] = np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * 2.0 ** 2))
    kp, sc, idx = udp_decode(hm)
    kp_hm = kp[0] / np.array([192, 256]) * np.array([47, 63])
    np.testing.assert_allclose(kp_hm, np.tile([cx, cy], (17, 1)), atol=0.05)
    assert np.all(idx == 32 * 48 + 20)


def test_decode_nonpositive_map_keeps_minus_one_lineage():
    from oracle.decode import get_heatmap_maximum
    hm = -np.ones((2, 64, 48), dtype=np.float32)
    locs, vals, idx = get_heatmap_maximum(hm)
    np.testing.assert_array_equal(locs, -1)
    np.testing.assert_array_equal(idx, 0)


def test_gaussian_table_matches_hip_constants():
    import os
    import re
    from oracle.decode import gaussian_kernel_1d
    src = open(os.path.join(os.path.dirname(__file__), "..", "macaque-3d-pose-estimation_amd", "csrc",
                            "imgproc.hip")).read()
    body = src[src.index("kGauss11[11] = {"):]
    body = body[:body.index("};")]
    vals = np.array([float(v) for v in re.findall(r"([0-9.]+(?:e-?[0-9]+)?)f", body)], dtype=np.float32)
    np.testing.assert_array_equal(vals, gaussian_kernel_1d(11))


def test_crop_constant_image_is_constant_inside():
    from oracle.crop import topdown_crop
    img = np.full((200, 300, 3), 77, dtype=np.uint8)
    c, ce, s = topdown_crop(img, np.array([50, 40, 150, 160], np.float32))
    # inside the source image the bilinear weights sum to 32768 exactly
    assert c[128, 96].tolist() == [77, 77, 77]
    assert set(np.unique(c)) <= set(range(0, 78))


def test_crop_matrix_maps_box_centre_to_crop_centre():
    from oracle.crop import bbox_xyxy2cs, fix_aspect_ratio, udp_warp_matrix
    b = np.array([[10, 20, 110, 220]], np.float32)
    c, s = bbox_xyxy2cs(b)
    s = fix_aspect_ratio(s)
    m = udp_warp_matrix(c[0], s[0]).astype(np.float64)
    p = m @ np.array([c[0][0], c[0][1], 1.0])
    np.testing.assert_allclose(p, [95.5, 127.5], atol=1e-4)   # (W-1)/2, (H-1)/2 in UDP


def test_optim_points_oracle_reduces_cost():
    """scipy TRF with the reference arguments (cameras.py:1166-1180) lowers the objective."""
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle, optim_points
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(1, 30)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=0.1)
    o = CameraGroupOracle(cams)
    pts = kp2d[0].transpose(1, 0, 2, 3)  # (C, F, J, 3)
    p2 = pts[..., :2].copy()
    p2[pts[..., 2] < 0.5] = np.nan
    init = o.triangulate(p2.reshape(8, -1, 2)).reshape(30, 17, 3)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    p3, jl, res, ssf, x0 = optim_points(o, p2, init, cons, weak, scale_smooth=3, scale_length=5,
                                        scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3,
                                        return_result=True)
    r0 = o._error_fun_triangulation(x0, p2, np.array(cons), np.array(weak), ssf, 5, 2, 3, 'soft_l1', 2)
    assert res.cost < 0.5 * np.sum(r0 ** 2)
    assert jl.shape == (31,) and np.isfinite(p3).all()
    assert np.nanmedian(np.linalg.norm(p3 - skel[0], axis=-1)) < 10.0


@pytest.mark.parametrize("min_cams", [2, 3])
def test_batched_ransac_oracle_equals_loop_oracle(min_cams):
    """triangulate_ransac_batched (used for clip-sized parity, config 4) returns exactly what the
    loop restatement of cameras.py:639-743 returns: same picks, same p3d / errors bit for bit,
    including points seen by 0, 1 or 2 cameras."""
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(2, 3), noise_px=2.0, drop=0.35, seed=7)
    pts = kp2d[..., :2].copy()
    pts[kp2d[..., 2] < 0.5] = np.nan
    flat = np.ascontiguousarray(pts.transpose(2, 0, 1, 3, 4).reshape(8, -1, 2))
    flat[:, 0] = np.nan
    flat[1:, 1] = np.nan
    flat[2:, 2] = np.nan
    o = CameraGroupOracle(cams)
    loop = o.triangulate_ransac(flat, min_cams=min_cams)
    fast = o.triangulate_ransac_batched(flat, min_cams=min_cams)
    for a, b in zip(loop, fast):
        np.testing.assert_array_equal(a, b)


def test_jointlenfix_oracle_residual_and_nfev_cap():
    """cameras.py:1192-1415: the fixed-length residual is the free one with the lengths pinned,
    the sparsity drops the length columns, and scipy stops at max_nfev = 15."""
    from mqhip import synth
    from oracle.geometry import (CameraGroupOracle, jac_sparsity_triangulation_jointlenfix,
                                 optim_points_jointlenfix)
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(1, 20)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=0.1)
    o = CameraGroupOracle(cams)
    pts = kp2d[0].transpose(1, 0, 2, 3)
    p2 = pts[..., :2].copy()
    p2[pts[..., 2] < 0.5] = np.nan
    init = o.triangulate(p2.reshape(8, -1, 2)).reshape(20, 17, 3)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    jl = np.linspace(50, 300, len(cons) + len(weak))
    x = init.ravel().copy()
    x[~np.isfinite(x)] = 0
    r_fix = o._error_fun_triangulation_jointlenfix(x, p2, jl, np.array(cons), np.array(weak), 2.0, 5, 2, 3,
                                                   'soft_l1', 2)
    r_free = o._error_fun_triangulation(np.hstack([x, jl]), p2, np.array(cons), np.array(weak), 2.0, 5, 2, 3,
                                        'soft_l1', 2)
    np.testing.assert_array_equal(r_fix, r_free)
    A = jac_sparsity_triangulation_jointlenfix(p2, np.array(cons), np.array(weak), 2)
    assert A.shape == (len(r_fix), x.size)
    p3, jl_out, res, ssf, x0 = optim_points_jointlenfix(o, p2, init, jl, cons, weak, scale_smooth=3,
                                                        scale_length=5, scale_length_weak=2, n_deriv_smooth=2,
                                                        reproj_error_threshold=3, max_nfev=3, ftol=1e-12,
                                                        return_result=True)
    assert res.nfev <= 3 and jl_out is jl and p3.shape == init.shape


def test_batched_viterbi_oracle_equals_loop_oracle():
    """step4_filter_batched (clip-sized parity, config 4) == the loop restatement of
    filter_pose.py:48-186 as driven by step4:142-167, value for value (gaps, placeholders)."""
    from mqhip import synth
    from oracle.viterbi import step4_filter, step4_filter_batched
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(2, 30), noise_px=6.0, drop=0.45, seed=11)
    kp2d[0, 5:12, 3] = 0          # a camera loses animal 0 for 7 frames
    np.testing.assert_array_equal(step4_filter(kp2d), step4_filter_batched(kp2d))
