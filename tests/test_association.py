"""Step-2 geometry affinity (geometry_affinity2, step2_crossviewmatching.py:373-432): the oracle's
known answers on CPU, and mq_geometry_affinity vs the oracle on the GPU (float64, 1e-9)."""
import numpy as np
import pytest

from conftest import gpu_available
from oracle.association import calc_dist_btw_lines, geometry_affinity2


def _scene(seed, n_cam=4, n_ind=3, J=17, noise=0.0, spread=600.0):
    """Cameras on a ring looking at the origin; individuals = clusters of J points; detections =
    normalized (undistorted) projections, i.e. what step 2 feeds geometry_affinity2."""
    rng = np.random.default_rng(seed)
    pmats, tvecs = [], []
    for c in range(n_cam):
        ang = 2 * np.pi * c / n_cam
        center = np.array([2000 * np.cos(ang), 2000 * np.sin(ang), 300.0])
        fwd = -center / np.linalg.norm(center)
        up = np.array([0, 0, 1.0])
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        R = np.stack([right, down, fwd])
        t = -R @ center
        pmats.append(np.hstack([R, t[:, None]]))
        tvecs.append(t)
    inds = [rng.normal(0, 150, size=(J, 3)) + rng.uniform(-spread, spread, size=3) for _ in range(n_ind)]
    return pmats, tvecs, inds, rng


def _project(P, X):
    Xc = X @ P[:, :3].T + P[:, 3]
    return Xc[:, :2] / Xc[:, 2:3]


def _frame(pmats, inds, rng, dets_per_cam, noise=0.0, low_score_frac=0.1):
    pts, dim = [], [0]
    for c, who in enumerate(dets_per_cam):
        for i in who:
            xy = _project(pmats[c], inds[i]) + rng.normal(0, noise, size=(inds[i].shape[0], 2))
            s = rng.uniform(0.2, 1.0, size=(inds[i].shape[0], 1))
            s[rng.random(s.shape) < low_score_frac] = 0.05
            pts.append(np.hstack([xy, s]))
        dim.append(dim[-1] + len(who))
    return np.array(pts), np.array(dim)


def test_line_distance_known_answer():
    # x axis through the origin and a line parallel to y at z = 7: distance 7
    v1 = np.array([0, 0, 0, 1, 0, 0.0])
    v2 = np.array([3, -2, 7, 3, 5, 7.0])
    assert abs(calc_dist_btw_lines(v1, v2) - 7.0) < 1e-12


def test_oracle_affinity_known_answers():
    # Known answers of the reference normalisation (step2:419-431): the z-score runs over every entry
    # below 2*Dth2 *including the zero diagonal*, so the diagonal holds the row maximum, the same
    # individual seen from two cameras sits just below it (rays meet up to the detection noise),
    # and pairs on one camera or of different individuals (rays ~1 m apart) are 0.
    pmats, tvecs, inds, rng = _scene(0, n_cam=3, n_ind=2, spread=900.0)
    pts, dim = _frame(pmats, inds, rng, [[0, 1], [1, 0], [0]], noise=1e-3, low_score_frac=0.0)
    aff = geometry_affinity2(pts, dim, pmats, tvecs)
    np.testing.assert_array_equal(aff, aff.T)
    diag = np.diag(aff)
    assert np.all(diag == diag[0]) and diag[0] > 0.9
    for i, j in [(0, 3), (0, 4), (3, 4), (1, 2)]:  # same individual, different cameras
        assert 0 < aff[i, j] < diag[0], (i, j, aff[i, j])
    for i, j in [(0, 1), (2, 3), (0, 2), (1, 3), (1, 4), (2, 4)]:  # same camera / other individual
        assert aff[i, j] == 0, (i, j, aff[i, j])


def test_oracle_affinity_too_few_keypoints_is_far():
    # fewer than 3 keypoints scored above THR_KP by both detections -> distance 2*Dth2 -> affinity 0
    pmats, tvecs, inds, rng = _scene(3, n_cam=2, n_ind=1)
    pts, dim = _frame(pmats, inds, rng, [[0], [0]], noise=1e-3, low_score_frac=0.0)
    pts[1, 2:, 2] = 0.1                            # "> thr" is strict: 0.1 does not qualify
    aff = geometry_affinity2(pts, dim, pmats, tvecs)
    assert aff[0, 1] == 0 and aff[1, 0] == 0


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
def test_gpu_affinity_matches_oracle_batched():
    from mqhip.association import dimgroup_to_cams, geometry_affinity_batch
    from mqhip.geometry import CameraGroup, OmnidirCamera
    pmats, tvecs, inds, rng = _scene(1, n_cam=6, n_ind=4)
    layouts = [
        [[0, 1, 2, 3]] * 6,                               # every individual in every view (M = 24)
        [[0, 1], [2], [], [3, 1, 0], [0], [2, 3]],        # a camera without detections
        [[0]],                                            # M = 1: std 0 -> NaN, as numpy gives
        [[0, 1], [0, 1], [1]],
        [[3], [3], [2], [2, 3], [1], [0, 1, 2]],
    ]
    frames = [_frame(pmats, inds, rng, lay, noise=2e-3, low_score_frac=0.15) for lay in layouts]
    Mmax = max(p.shape[0] for p, _ in frames)
    J = inds[0].shape[0]
    pts = np.zeros((len(frames), Mmax, J, 3))
    cod = np.full((len(frames), Mmax), -1, dtype=np.int32)
    for b, (p, dim) in enumerate(frames):
        pts[b, :p.shape[0]] = p
        cod[b, :p.shape[0]] = dimgroup_to_cams(dim, p.shape[0])
    g = CameraGroup([OmnidirCamera.from_projection(P) for P in pmats])
    got = geometry_affinity_batch(g, pts, cod)
    for b, (p, dim) in enumerate(frames):
        M = p.shape[0]
        ref = geometry_affinity2(p, dim, pmats, tvecs)
        np.testing.assert_allclose(got[b, :M, :M], ref, rtol=0, atol=1e-9, equal_nan=True)
        assert np.all(got[b, M:, :] == 0) and np.all(got[b, :, M:] == 0)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
def test_step2_mirror_signature_matches_oracle():
    from src.pipeline.step2_crossviewmatching import geometry_affinity2 as mirror
    pmats, tvecs, inds, rng = _scene(2, n_cam=4, n_ind=3)
    pts, dim = _frame(pmats, inds, rng, [[0, 1, 2], [2, 1], [0, 2], [1]], noise=1e-3)
    camparam = {"camera_id": [f"c{i}" for i in range(4)], "pmat": pmats, "tvecs": tvecs}
    got = mirror(pts, dim, "unused.yaml", camparam=camparam)
    ref = geometry_affinity2(pts, dim, pmats, tvecs)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-9, equal_nan=True)
    with pytest.raises(FileNotFoundError):  # as the reference: get_camparam opens config.yaml
        mirror(pts, dim, "unused.yaml")
