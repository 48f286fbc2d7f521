"""GPU parity: float64 geometry kernels of libmq_hip vs the numpy oracle."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _setup(n_animals=4, n_frames=12, seed=3):
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(n_animals, n_frames)
    kp2d = synth.make_kp2d(cams, skel, seed=seed)
    g = CameraGroup.from_dicts(cams)
    o = CameraGroupOracle(cams)
    return cams, skel, kp2d, g, o


def _points(kp2d, score_thr=0.5):
    # (A,F,C,J,3) -> (C, A*F*J, 2) with NaN where score < thr (step4:225-226)
    A, F, C, J, _ = kp2d.shape
    p = kp2d.transpose(2, 0, 1, 3, 4).reshape(C, A * F * J, 3).copy()
    pts = p[..., :2].copy()
    pts[p[..., 2] < score_thr] = np.nan
    return pts


def test_project_and_undistort_bit_exact():
    cams, skel, kp2d, g, o = _setup()
    X = skel.reshape(-1, 3)
    np.testing.assert_array_equal(g.project(X), o.project(X))
    pts = _points(kp2d)
    np.testing.assert_array_equal(g.undistort_points(pts), o.undistort(pts))


def test_triangulate_dlt_matches_oracle():
    cams, skel, kp2d, g, o = _setup()
    pts = _points(kp2d)
    got = g.triangulate(pts)
    ref = o.triangulate(pts)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref[:, 0])
    np.testing.assert_allclose(got[ok], ref[ok], rtol=0, atol=1e-6)


def test_triangulate_noise_free_recovers_truth():
    cams, skel, kp2d, g, o = _setup()
    X = skel.reshape(-1, 3)
    uv = o.project(X)
    got = g.triangulate(uv)
    np.testing.assert_allclose(got, X, rtol=0, atol=1e-6)


def test_reprojection_error_matches_oracle():
    cams, skel, kp2d, g, o = _setup()
    pts = _points(kp2d)
    p3 = o.triangulate(pts)
    for mean in (False, True):
        got = g.reprojection_error(p3, pts, mean=mean)
        ref = o.reprojection_error(p3, pts, mean=mean)
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-9, equal_nan=True)


def test_triangulate_ransac_matches_oracle():
    cams, skel, kp2d, g, o = _setup(n_animals=2, n_frames=6)
    pts = _points(kp2d)
    # edge cases: a point seen by 0 cams and one seen by 1 cam
    pts[:, 0] = np.nan
    pts[1:, 1] = np.nan
    for min_cams in (2, 3):
        p3, picked, p2, err = g.triangulate_ransac(pts, min_cams=min_cams)
        r3, rpicked, r2, rerr = o.triangulate_ransac(pts, min_cams=min_cams)
        np.testing.assert_array_equal(picked, rpicked)
        assert np.array_equal(np.isnan(p3), np.isnan(r3))
        np.testing.assert_allclose(p3, r3, rtol=0, atol=1e-6, equal_nan=True)
        np.testing.assert_allclose(err, rerr, rtol=1e-9, atol=1e-9)
        np.testing.assert_array_equal(p2, r2)


def test_mvpose_pinv_dlt_matches_oracle():
    from mqhip.geometry import triangulate_pinv
    from oracle.geometry import mct_triangulate_points
    cams, skel, kp2d, g, o = _setup()
    pts = _points(kp2d)
    und = o.undistort(pts)
    use = ~np.isnan(und[..., 0]).T  # (N, C)
    und0 = np.where(np.isnan(und), 0.0, und)
    pmat = [o.cameras[c].extrinsics_mat()[:3] for c in range(len(cams))]
    ref = mct_triangulate_points(und0, use, pmat)
    got = triangulate_pinv(g, und0, use)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6, equal_nan=True)


def test_viterbi_matches_oracle():
    from mqhip import synth
    from mqhip.geometry import viterbi_filter
    from oracle.viterbi import step4_filter
    cams = synth.make_cameras(8)
    skel = synth.make_skeletons(2, 40)
    kp2d = synth.make_kp2d(cams, skel, drop=0.3, seed=5)
    # jumps and long gaps exercise the -100 clamp and the missing particle
    kp2d[0, 10:14, 2, 3] = 0
    kp2d[1, 20, 4, 5, :2] += 400
    got = viterbi_filter(kp2d)                     # (A,F,C,J,3)
    ref = step4_filter(kp2d)                       # (F,J,A,3,C)
    ref = ref.transpose(2, 0, 4, 1, 3)
    np.testing.assert_array_equal(got, ref)
