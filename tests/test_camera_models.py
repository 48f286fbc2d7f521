"""The pinhole ``Camera`` and ``FisheyeCamera`` models of aniposelib (cameras.py:173-426).

CPU: known-answer checks of the oracle's restatements of cv2.undistortPoints / cv2.projectPoints and
cv2.fisheye.undistortPoints / projectPoints (OpenCV 4.11; cv2 itself is absent, so parity with OpenCV is
unpinned): zero-distortion closed forms, round trips, the pinhole ``icdist < 0`` exit and the fisheye
non-convergence sentinel (-1e6, -1e6).

GPU: every geometry entry point on camera groups of each model and on a mixed group, against the
oracle: pinhole undistort / project bit for bit; fisheye within 1e-12 relative (the device atan / tan may
differ from glibc's by an ulp); DLT, reprojection error and RANSAC as for omnidir groups
(tests/test_gpu_geometry.py); optim_points within the scipy band of tests/test_gpu_optim.py.
"""
import numpy as np
import pytest

from conftest import gpu_available



def _mixed():
    from mqhip import synth
    om = synth.make_cameras(8)
    pin = synth.make_cameras_model(8, "pinhole")
    fis = synth.make_cameras_model(8, "fisheye")
    return om[:2] + pin[2:5] + fis[5:]


def _cams(kind):
    from mqhip import synth
    if kind == "mixed":
        return _mixed()
    return synth.make_cameras_model(8, kind)


def _cam_frame_dict(model, dist, f=1000.0, c=(1000.0, 750.0)):
    m = np.array([[f, 2.0, c[0]], [0.0, f * 1.01, c[1]], [0.0, 0.0, 1.0]])
    return dict(name="k", matrix=m, distortions=np.asarray(dist, dtype=np.float64), rotation=np.zeros(3),
                translation=np.zeros(3), fisheye=model == "fisheye", omnidir=False)


# ------------------------------------------------------------------------------------------ CPU oracle

def test_pinhole_zero_distortion_closed_form():
    from oracle.geometry import PinholeCam
    cam = PinholeCam(_cam_frame_dict("pinhole", np.zeros(5)))
    X = np.array([[100.0, -50.0, 1500.0], [0.0, 0.0, 800.0], [-300.0, 220.0, 2100.0]])
    uv = cam.project(X)
    m = cam.K
    np.testing.assert_array_equal(uv[:, 0], X[:, 0] * (1.0 / X[:, 2]) * m[0, 0] + m[0, 2])
    np.testing.assert_array_equal(uv[:, 1], X[:, 1] * (1.0 / X[:, 2]) * m[1, 1] + m[1, 2])
    np.testing.assert_allclose(cam.undistort_points(uv), X[:, :2] / X[:, 2:], rtol=0, atol=1e-15)


def test_pinhole_round_trip_and_negative_icdist_exit():
    from oracle.geometry import PinholeCam
    cam = PinholeCam(_cam_frame_dict("pinhole", [-0.08, 0.02, 1e-3, -2e-3, 0.004]))
    rng = np.random.default_rng(0)
    xy = rng.uniform(-0.3, 0.3, (50, 2))
    uv = cam.project(np.c_[xy * 1000.0, np.full(50, 1000.0)])
    np.testing.assert_allclose(cam.undistort_points(uv), xy, rtol=0, atol=1e-9)  # 5 fixed-point steps
    bad = PinholeCam(_cam_frame_dict("pinhole", [-50.0, 0, 0, 0, 0]))
    p = np.array([[1000.0 + 0.4 * 1000.0, 750.0]])                    # r2 = 0.16: 1 - 8 < 0
    np.testing.assert_array_equal(bad.undistort_points(p), [[(p[0, 0] - 1000.0) * (1.0 / 1000.0), 0.0]])


def test_fisheye_zero_distortion_is_equidistant():
    from oracle.geometry import FisheyeCam
    cam = FisheyeCam(_cam_frame_dict("fisheye", np.zeros(4)))
    uv = cam.project(np.array([[1.0, 0.0, 1.0], [0.0, 0.0, 5.0]]))    # 45 degrees off axis; on axis
    np.testing.assert_allclose(uv[0], [1000.0 * np.pi / 4 + 1000.0, 750.0], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(uv[1], [1000.0, 750.0])
    und = cam.undistort_points(uv)
    np.testing.assert_allclose(und, [[1.0, 0.0], [0.0, 0.0]], rtol=0, atol=1e-12)


def test_fisheye_round_trip_and_non_convergence_sentinel():
    from oracle.geometry import FisheyeCam
    cam = FisheyeCam(_cam_frame_dict("fisheye", [0.02, -0.004, 1e-3, -5e-4]))
    rng = np.random.default_rng(1)
    xy = rng.uniform(-1.0, 1.0, (50, 2))
    uv = cam.project(np.c_[xy * 100.0, np.full(50, 100.0)])
    np.testing.assert_allclose(cam.undistort_points(uv), xy, rtol=0, atol=1e-9)
    # theta (1 - 0.6 theta^2) never reaches theta_d = 1.2: Newton does not converge -> (-1e6, -1e6)
    bad = FisheyeCam(_cam_frame_dict("fisheye", [-0.6, 0, 0, 0]))
    p = np.array([[1000.0 + 1.2 * 1000.0, 750.0]])
    np.testing.assert_array_equal(bad.undistort_points(p), [[-1e6, -1e6]])


@pytest.mark.parametrize("kind", ["pinhole", "fisheye", "mixed"])
def test_oracle_dlt_recovers_truth(kind):
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle
    o = CameraGroupOracle(_cams(kind))
    X = synth.make_skeletons(1, 3).reshape(-1, 3)
    np.testing.assert_allclose(o.triangulate(o.project(X)), X, rtol=0, atol=1e-6)


# ------------------------------------------------------------------------------------------ GPU parity

def _points(cams, n_frames=8, seed=3, drop=0.1):
    from mqhip import synth
    skel = synth.make_skeletons(2, n_frames)
    kp2d = synth.make_kp2d(cams, skel, seed=seed, drop=drop)
    A, F, C, J, _ = kp2d.shape
    p = kp2d.transpose(2, 0, 1, 3, 4).reshape(C, A * F * J, 3)
    pts = p[..., :2].copy()
    pts[p[..., 2] < 0.5] = np.nan
    return skel, pts


@pytest.mark.parametrize("kind", ["pinhole", "fisheye", "mixed"])
@pytest.mark.gpu
def test_gpu_project_and_undistort_match_oracle(kind):
    if not gpu_available():
        pytest.skip("needs a HIP device")
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle
    cams = _cams(kind)
    g, o = CameraGroup.from_dicts(cams), CameraGroupOracle(cams)
    skel, pts = _points(cams)
    X = skel.reshape(-1, 3)
    # edge points: the principal point of each camera (r = 0) and a NaN
    pts[:, 0] = [[float(np.asarray(c["matrix"])[0, 2]), float(np.asarray(c["matrix"])[1, 2])]
                 if not c.get("omnidir") else [np.nan, np.nan] for c in cams]
    exact = kind == "pinhole"
    gp, op = g.project(X), o.project(X)
    gu, ou = g.undistort_points(pts), o.undistort(pts)
    if exact:
        np.testing.assert_array_equal(gp, op)
        np.testing.assert_array_equal(gu, ou)
    else:
        np.testing.assert_allclose(gp, op, rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(gu, ou, rtol=1e-12, atol=1e-15, equal_nan=True)


@pytest.mark.gpu
def test_gpu_edge_branches_match_oracle():
    """The pinhole icdist < 0 exit and the fisheye non-convergence sentinel on the GPU."""
    if not gpu_available():
        pytest.skip("needs a HIP device")
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle
    cams = [_cam_frame_dict("pinhole", [-50.0, 0, 0, 0, 0]), _cam_frame_dict("fisheye", [-0.6, 0, 0, 0])]
    g, o = CameraGroup.from_dicts(cams), CameraGroupOracle(cams)
    pts = np.array([[[1400.0, 750.0], [1001.0, 751.0], [2200.0, 750.0]]] * 2)
    got, ref = g.undistort_points(pts), o.undistort(pts)
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=0)
    assert got[1, 2, 0] == -1e6 and got[0, 0, 1] == 0.0


@pytest.mark.parametrize("kind", ["pinhole", "fisheye", "mixed"])
@pytest.mark.gpu
def test_gpu_dlt_reprojection_ransac_match_oracle(kind):
    if not gpu_available():
        pytest.skip("needs a HIP device")
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle
    cams = _cams(kind)
    g, o = CameraGroup.from_dicts(cams), CameraGroupOracle(cams)
    skel, pts = _points(cams, n_frames=4)
    pts[:, 0] = np.nan
    pts[1:, 1] = np.nan
    got = g.triangulate(pts)
    ref = o.triangulate(pts)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6, equal_nan=True)
    X = skel.reshape(-1, 3)
    np.testing.assert_allclose(g.triangulate(o.project(X)), X, rtol=0, atol=1e-6)
    for mean in (False, True):
        np.testing.assert_allclose(g.reprojection_error(ref, pts, mean=mean), o.reprojection_error(ref, pts, mean=mean),
                                   rtol=1e-9, atol=1e-9, equal_nan=True)
    p3, picked, p2, err = g.triangulate_ransac(pts, min_cams=2)
    r3, rpicked, r2, rerr = o.triangulate_ransac(pts, min_cams=2)
    np.testing.assert_array_equal(picked, rpicked)
    np.testing.assert_allclose(p3, r3, rtol=0, atol=1e-6, equal_nan=True)
    np.testing.assert_allclose(err, rerr, rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(p2, r2)


@pytest.mark.parametrize("kind", ["pinhole", "fisheye", "mixed"])
@pytest.mark.gpu
def test_gpu_optim_points_matches_scipy(kind):
    """optim_points with the model's analytic Jacobian (csrc/optim.hip) against scipy's TRF on the
    oracle's residuals: the band and cost criteria of tests/test_gpu_optim.py."""
    if not gpu_available():
        pytest.skip("needs a HIP device")
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle, optim_points
    args = dict(scale_smooth=3, scale_length=5, scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3)
    cams = _cams(kind)
    F = 24
    skel = synth.make_skeletons(1, F)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=0.1, seed=4)
    o = CameraGroupOracle(cams)
    pts = kp2d[0].transpose(1, 0, 2, 3)
    p2 = pts[..., :2].copy()
    p2[pts[..., 2] < 0.5] = np.nan
    init = o.triangulate(p2.reshape(8, -1, 2)).reshape(F, 17, 3)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    sa = optim_points(o, p2, init, cons, weak, ftol=1e-3, return_result=True, **args)
    sb = optim_points(o, p2, init, cons, weak, ftol=1e-10, return_result=True, **args)
    p3g, jlg = CameraGroup.from_dicts(cams).optim_points(p2, init, constraints=cons, constraints_weak=weak, **args)
    band = np.linalg.norm(sa[0] - sb[0], axis=-1)
    dev = np.linalg.norm(p3g - sa[0], axis=-1)
    assert np.median(dev) <= max(np.median(band), 1.0), (np.median(dev), np.median(band))
    assert np.percentile(dev, 99) <= max(np.percentile(band, 99), 5.0)
    r = o._error_fun_triangulation(np.hstack([p3g.ravel(), jlg]), p2, np.array(cons), np.array(weak), sa[3],
                                   args["scale_length"], args["scale_length_weak"], args["reproj_error_threshold"],
                                   "soft_l1", args["n_deriv_smooth"])
    assert 0.5 * np.sum(r ** 2) <= sa[2].cost * (1 + 1e-3), (0.5 * np.sum(r ** 2), sa[2].cost)


@pytest.mark.gpu
def test_gpu_unknown_model_row_gives_nan():
    """A camera row whose model slot (include/mq_hip.h slot 22) is not 0, 1 or 2 yields NaN from every
    geometry entry point instead of silently running another model."""
    if not gpu_available():
        pytest.skip("needs a HIP device")
    import torch
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    cams = synth.make_cameras(3)
    g = CameraGroup.from_dicts(cams)
    rows = g.cams_tensor().clone()
    rows[1, 22] = 7.0
    g._cams_dev = rows
    X = synth.make_skeletons(1, 2).reshape(-1, 3)
    uv = g.project(X)
    assert np.isfinite(uv[[0, 2]]).all() and np.isnan(uv[1]).all()
    und = g.undistort_points(uv.copy())
    assert np.isnan(und[1]).all() and np.isfinite(und[[0, 2]]).all()


@pytest.mark.gpu
def test_gpu_closed_forms_without_the_oracle():
    """the GPU camera models against closed forms that do not go through oracle/geometry.py (so a
    misreading of OpenCV shared by the oracle and the kernels cannot pass): zero-distortion pinhole = the
    pinhole projection fx X/Z + cx; zero-distortion fisheye = equidistant f atan(r) / r; undistort(project(X))
    = X / Z for distorted models; the pinhole icdist < 0 exit returns the undistorted seed ((u - cx) / fx, 0)
    and the fisheye non-convergence sentinel is (-1e6, -1e6)."""
    if not gpu_available():
        pytest.skip("needs a HIP device")
    from mqhip.geometry import CameraGroup
    X = np.array([[100.0, -50.0, 1500.0], [0.0, 0.0, 800.0], [-300.0, 220.0, 2100.0], [1.0, 0.0, 1.0]])
    g = CameraGroup.from_dicts([_cam_frame_dict("pinhole", np.zeros(5)), _cam_frame_dict("fisheye", np.zeros(4))])
    uv = g.project(X)
    f, fy, cx, cy = 1000.0, 1010.0, 1000.0, 750.0
    np.testing.assert_allclose(uv[0, :, 0], f * X[:, 0] / X[:, 2] + cx, rtol=1e-15, atol=1e-9)
    np.testing.assert_allclose(uv[0, :, 1], fy * X[:, 1] / X[:, 2] + cy, rtol=1e-15, atol=1e-9)
    r = np.hypot(X[:, 0], X[:, 1]) / X[:, 2]
    sc = np.where(r > 0, np.arctan(r) / np.where(r > 0, r, 1.0), 1.0)
    np.testing.assert_allclose(uv[1, :, 0], f * sc * X[:, 0] / X[:, 2] + cx, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(uv[1, 3], [f * np.pi / 4 + cx, cy], rtol=0, atol=1e-9)
    np.testing.assert_allclose(g.undistort_points(uv), np.broadcast_to(X[:, :2] / X[:, 2:], (2, 4, 2)), rtol=0,
                               atol=1e-12)
    # distorted round trips
    gd = CameraGroup.from_dicts([_cam_frame_dict("pinhole", [-0.08, 0.02, 1e-3, -2e-3, 0.004]),
                                 _cam_frame_dict("fisheye", [0.02, -0.004, 1e-3, -5e-4])])
    rng = np.random.default_rng(5)
    xy = rng.uniform(-0.3, 0.3, (64, 2))
    Xd = np.c_[xy * 1000.0, np.full(64, 1000.0)]
    np.testing.assert_allclose(gd.undistort_points(gd.project(Xd)), np.broadcast_to(xy, (2, 64, 2)), rtol=0, atol=1e-9)
    # the two exit branches, by their defining values
    ge = CameraGroup.from_dicts([_cam_frame_dict("pinhole", [-50.0, 0, 0, 0, 0]), _cam_frame_dict("fisheye", [-0.6, 0, 0, 0])])
    und = ge.undistort_points(np.array([[[1400.0, 750.0]], [[2200.0, 750.0]]]))
    np.testing.assert_allclose(und[0, 0], [0.4, 0.0], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(und[1, 0], [-1e6, -1e6])
