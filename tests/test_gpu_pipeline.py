"""GPU: the drop-in entry points (src/...) end to end against the oracle.

* step4_aniposefiltering.proc on a synthetic results directory (kp2d.pickle,
  calibration.toml, config.yaml) vs the oracle composition of step4:140-331
  (Viterbi chains identical, kp3d within the optim_points band, scores exact,
  reprojection errors 1e-6 px).
* anipose filter_pose_viterbi shim (incl. its input mutation) vs the oracle.
* multicam_toolbox undistortPoints / triangulatePoints (camparam path) vs the oracle.
* step1 multi-view batch == per-view inference_topdown, alldata.json rows.
"""
import os

import numpy as np
import pytest
import yaml

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

TRI = dict(scale_smooth=3, scale_length=5, scale_length_weak=2, n_deriv_smooth=2, reproj_error_threshold=3)


def _cams(kind):
    from mqhip import synth
    if kind == "omnidir":
        return synth.make_cameras(8)
    # mixed: 2 omnidir, 3 pinhole, 3 fisheye cameras in one calibration.toml (cameras.py:1972-1982)
    return (synth.make_cameras(8)[:2] + synth.make_cameras_model(8, "pinhole")[2:5] +
            synth.make_cameras_model(8, "fisheye")[5:])


def _results_dir(tmp_path, A=2, F=36, kind="omnidir"):
    from mqhip import io as mqio
    from mqhip import synth
    cams = _cams(kind)
    skel = synth.make_skeletons(A, F)
    kp2d = synth.make_kp2d(cams, skel, noise_px=2.0, drop=0.1)       # (A,F,C,J,3)
    rd = tmp_path / "results" / "demo"
    rd.mkdir(parents=True)
    synth.write_calibration_toml(cams, str(rd / "calibration.toml"))
    mqio.dump_pickle(kp2d, str(rd / "kp2d.pickle"))
    cal = tmp_path / "calib"
    cal.mkdir()
    with open(cal / "config.yaml", "w") as f:
        yaml.safe_dump({"camera_id": [int(c["name"]) for c in cams]}, f)
    return cams, kp2d, str(tmp_path / "results"), str(cal / "config.yaml")


@pytest.mark.parametrize("kind", ["omnidir", "mixed"])
def test_step4_proc_matches_oracle(tmp_path, kind):
    """step 4 end to end; "mixed": a calibration.toml holding omnidir, pinhole and fisheye cameras, loaded
    through CameraGroup.load into the three models."""
    from mqhip import io as mqio
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle, optim_points
    from oracle.viterbi import step4_filter
    from src.pipeline import step4_aniposefiltering as step4
    cams, kp2d, root, cfg = _results_dir(tmp_path, kind=kind)
    data = step4.proc("demo", root, cfg, 17, redo=True)
    rd = os.path.join(root, "demo")
    got = mqio.load_array_pickle(os.path.join(rd, "kp3d.pickle"))
    assert set(got) == {"kp3d", "kp3d_score", "kp3d_err", "joint_len"}
    kp2d_f = mqio.load_array_pickle(os.path.join(rd, "kp2d_f.pickle"))
    ref_f = step4_filter(kp2d)
    np.testing.assert_array_equal(kp2d_f, ref_f)
    o = CameraGroupOracle(cams)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    kp = ref_f.transpose((2, 4, 0, 1, 3))
    A, C, F, J, _ = kp.shape
    for a in range(A):
        p2 = kp[a, ..., :2].copy()
        sc = kp[a, ..., 2].copy()
        p2[sc < 0.5] = np.nan
        init = o.triangulate(p2.reshape(C, -1, 2)).reshape(F, J, 3)
        ra = optim_points(o, p2, init, cons, weak, ftol=1e-3, **TRI)[0]
        rb = optim_points(o, p2, init, cons, weak, ftol=1e-10, **TRI)[0]
        band = np.linalg.norm(ra - rb, axis=-1)
        dev = np.linalg.norm(got["kp3d"][a] - ra, axis=-1)
        assert np.median(dev) <= max(np.median(band), 1.0)
        assert np.percentile(dev, 99) <= max(np.percentile(band, 99), 5.0)
        good = ~np.isnan(p2[..., 0])
        s = sc.copy()
        s[~good] = 2
        s3 = s.min(axis=0)
        s3[good.sum(0) < 1] = np.nan
        np.testing.assert_array_equal(got["kp3d_score"][a], s3)
        err = o.reprojection_error(got["kp3d"][a].reshape(-1, 3), p2.reshape(C, -1, 2), mean=True).reshape(F, J)
        err[good.sum(0) < 1] = np.nan
        np.testing.assert_allclose(got["kp3d_err"][a], err, rtol=0, atol=1e-6)
    assert len(got["joint_len"]) == A and got["joint_len"][0].shape == (31,)
    assert np.load(os.path.join(rd, "joint_len.npy")).shape == (A, 31)
    assert data["kp3d"].shape == (A, F, J, 3)


def test_step4_non_optim_branches_match_oracle(tmp_path):
    """optim = false: plain DLT (num_cams >= 2) and RANSAC min_cams = 3 (step4:290-318)."""
    from mqhip import io as mqio
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle
    from oracle.viterbi import step4_filter
    from src.pipeline import step4_aniposefiltering as step4
    cams, kp2d, root, cfg = _results_dir(tmp_path, A=2, F=6)
    kp2d_f = step4_filter(kp2d)
    g = CameraGroup.from_dicts(cams)
    o = CameraGroupOracle(cams)
    conf = mqio.load_toml(step4.CONFIG_TMPL)
    kp = kp2d_f.transpose((2, 4, 0, 1, 3))
    A, C, F, J, _ = kp.shape
    for ransac in (False, True):
        conf["triangulation"].update(optim=False, ransac=ransac)
        kp3d, S, E, _ = step4.reconstruct_3d(kp2d_f, g, conf)
        for a in range(A):
            p2 = kp[a, ..., :2].copy()
            sc = kp[a, ..., 2].copy()
            p2[sc < 0.5] = np.nan
            flat = p2.reshape(C, -1, 2)
            if ransac:
                p3, picked, p2s, err = o.triangulate_ransac(flat, min_cams=3)
                good = ~np.isnan(p2s.reshape(C, F, J, 2)[..., 0])
                nc = picked.sum(0).sum(1).reshape(F, J).astype(float)
            else:
                p3 = o.triangulate(flat)
                err = o.reprojection_error(p3, flat, mean=True)
                good = ~np.isnan(p2[..., 0])
                nc = good.sum(0).astype(float)
            s = sc.copy()
            s[~good] = 2
            s3 = s.min(0)
            s3[nc < 2] = np.nan
            err = err.reshape(F, J).copy()
            err[nc < 2] = np.nan
            np.testing.assert_allclose(kp3d[a], p3.reshape(F, J, 3), rtol=0, atol=1e-6)
            np.testing.assert_array_equal(S[a], s3)
            np.testing.assert_allclose(E[a], err, rtol=0, atol=1e-6)


def test_filter_pose_viterbi_shim_matches_oracle():
    from mqhip import synth
    from oracle.viterbi import STEP4_FILTER_CONFIG, filter_pose_viterbi as ofilter
    from src.third_party.anipose import filter_pose as af
    cams = synth.make_cameras(8)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(1, 60), noise_px=3.0, drop=0.2)
    pts = np.ascontiguousarray(kp2d[0, :, 2][:, :, None, :])           # (F,J,1,3) of camera 2
    a, b = pts.copy(), pts.copy()
    p, s = af.filter_pose_viterbi(STEP4_FILTER_CONFIG, a, [])
    op, os_ = ofilter(STEP4_FILTER_CONFIG, b, [])
    np.testing.assert_array_equal(p, op)
    np.testing.assert_array_equal(s, os_)
    np.testing.assert_array_equal(a, b)                                # same input mutation
    np.testing.assert_array_equal(af.wrap_points(p, s)[:, :, 0, 2], s)


def test_multicam_toolbox_shim_matches_oracle():
    from mqhip import synth
    from mqhip.geometry import rodrigues
    from oracle.geometry import CameraGroupOracle, mct_triangulate_points
    from src.utils import multicam_toolbox as mct
    cams = synth.make_cameras(8)
    o = CameraGroupOracle(cams)
    X = synth.make_skeletons(1, 4).reshape(-1, 3)
    uv = o.project(X) + np.random.default_rng(0).normal(0, 1.0, (8, len(X), 2))
    camparam = {"camera_id": [c["name"] for c in cams], "K": [c["K"] for c in cams],
                "xi": [c["xi"] for c in cams], "D": [c["D"] for c in cams],
                "pmat": [np.hstack([rodrigues(c["rvec"]), np.asarray(c["tvec"]).reshape(3, 1)]) for c in cams]}
    und = mct.undistortPoints(None, list(uv), omnidir=True, camparam=camparam)
    np.testing.assert_allclose(np.stack(und), o.undistort(uv), rtol=0, atol=1e-12)
    use = np.random.default_rng(1).random((len(X), 8)) < 0.7
    use[0] = False
    use[1, 1:] = False
    P = mct.triangulatePoints(None, und, use, True, camparam=camparam)
    ref = mct_triangulate_points(np.stack(und), use, camparam["pmat"])
    np.testing.assert_allclose(P, ref, rtol=0, atol=1e-6)
    assert np.isnan(P[:2]).all()


def test_step1_multiview_batch_matches_per_view(tmp_path):
    import torch
    from mqhip import synth
    from src.pipeline import step1_proc2d as s1
    cfgp = tmp_path / "vit_tiny.py"
    cfgp.write_text("model = dict(type='TopdownPoseEstimator', backbone=dict(type='mmpretrain.VisionTransformer', "
                    "arch='tiny'))\n")
    model = s1.init_pose_model(str(cfgp), None, device="cuda:0")
    assert model.cfg.name == "tiny"
    cams = synth.make_cameras(4)
    kp2d = synth.make_kp2d(cams, synth.make_skeletons(2, 1), noise_px=0.0, drop=0.0)[:, 0]   # (A,C,J,3)
    frames = synth.make_frames(4, kp2d.transpose(1, 0, 2, 3), height=1536, width=2048)
    boxes = synth.boxes_from_kp2d(kp2d.transpose(1, 0, 2, 3))                              # (C,A,4)
    tracks = [np.hstack([boxes[c], np.array([[1], [2]]), np.ones((2, 1))]).astype(np.float64) for c in range(4)]
    sm_b = [s1.KeypointSmoother() for _ in range(4)]
    rows_b = s1.process_frame_multiview(model, list(frames), tracks, sm_b, 0)
    for c in range(4):
        sm = s1.KeypointSmoother()
        rows = s1.process_frame(model, frames[c], tracks[c], sm, 0)
        assert len(rows) == len(rows_b[c]) == 2
        for r, rb in zip(rows, rows_b[c]):
            assert r[:5] == rb[:5] and r[6:] == rb[6:]
            np.testing.assert_allclose(np.array(r[5], dtype=float), np.array(rb[5], dtype=float), rtol=0,
                                       atol=1e-3, equal_nan=True)
    out = s1.process_single_cam([frames[0]] * 3, [tracks[0]] * 3, str(tmp_path / "cam0"), model)
    assert os.path.exists(tmp_path / "cam0" / "alldata.json") and len(out) == 3
    assert np.load(tmp_path / "cam0" / "frame_num.npy").tolist() == [0, 1, 2]
    torch.cuda.synchronize()


def _template(tmp_path, **tri):
    """A copy of configs/config_tmpl.toml with [triangulation] keys overridden (how a reference
    user switches step 4 to RANSAC: by editing the template, step4:102)."""
    from mqhip import io as mqio
    from src.pipeline import step4_aniposefiltering as step4
    conf = mqio.load_toml(step4.CONFIG_TMPL)
    conf["triangulation"].update(tri)
    p = tmp_path / "config_tmpl.toml"
    mqio.dump_toml(conf, str(p))
    return str(p)


def _oracle_scores_errors(o, kp_a, p3):
    C, F, J, _ = kp_a.shape
    p2 = kp_a[..., :2].copy()
    sc = kp_a[..., 2].copy()
    p2[sc < 0.5] = np.nan
    good = ~np.isnan(p2[..., 0])
    s = sc.copy()
    s[~good] = 2
    s3 = s.min(axis=0)
    s3[good.sum(0) < 1] = np.nan
    err = o.reprojection_error(p3.reshape(-1, 3), p2.reshape(C, -1, 2), mean=True).reshape(F, J)
    err[good.sum(0) < 1] = np.nan
    return p2, s3, err


def test_step4_proc_config4_ransac_then_optim(tmp_path, monkeypatch):
    """BASELINE config 4 end to end: a 300-frame clip, 8 views x 4 individuals x 17 joints through
    step4.proc with ransac = true, optim = true (step4:228-291: Viterbi -> triangulate_ransac
    (min_cams 2) -> optim_points -> reprojection error / scores).  Oracle composition: the batched
    Viterbi and RANSAC restatements (pinned bit-for-bit to the loop restatements on CPU) and scipy
    TRF with the reference's arguments per animal.  Tolerances: kp2d_f identical; RANSAC picks
    identical, p3d/err 1e-6; kp3d within 1 mm median / 5 mm p99 of scipy (SURVEY 8(d) floor) and
    no worse in cost than scipy + 0.1 %; scores exact; reprojection errors 1e-6 px."""
    from mqhip import io as mqio
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    from oracle.geometry import CameraGroupOracle, optim_points
    from oracle.viterbi import step4_filter_batched
    from src.pipeline import step4_aniposefiltering as step4
    cams, kp2d, root, cfg = _results_dir(tmp_path, A=4, F=300)
    monkeypatch.setattr(step4, "CONFIG_TMPL", _template(tmp_path, ransac=True, optim=True))
    step4.proc("demo", root, cfg, 17, redo=True)
    rd = os.path.join(root, "demo")
    got = mqio.load_array_pickle(os.path.join(rd, "kp3d.pickle"))
    kp2d_f = mqio.load_array_pickle(os.path.join(rd, "kp2d_f.pickle"))
    ref_f = step4_filter_batched(kp2d)
    np.testing.assert_array_equal(kp2d_f, ref_f)
    o = CameraGroupOracle(cams)
    g = CameraGroup.from_dicts(cams)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    kp = ref_f.transpose((2, 4, 0, 1, 3))                               # (A, C, F, J, 3)
    A, C, F, J, _ = kp.shape
    pts = kp[..., :2].copy()
    pts[kp[..., 2] < 0.5] = np.nan
    flat = np.ascontiguousarray(pts.transpose(1, 0, 2, 3, 4).reshape(C, -1, 2))
    ro = o.triangulate_ransac_batched(flat, min_cams=2)
    rg = g.triangulate_ransac(flat, min_cams=2)
    np.testing.assert_array_equal(rg[1], ro[1])                          # picked subsets
    np.testing.assert_allclose(rg[0], ro[0], rtol=0, atol=1e-6)
    np.testing.assert_allclose(rg[3], ro[3], rtol=0, atol=1e-6)
    init = ro[0].reshape(A, F, J, 3)
    for a in range(A):
        p2, s3, _ = _oracle_scores_errors(o, kp[a], init[a])
        sa = optim_points(o, p2, init[a], cons, weak, ftol=1e-3, return_result=True, **TRI)
        dev = np.linalg.norm(got["kp3d"][a] - sa[0], axis=-1)
        assert np.median(dev) <= 1.0 and np.percentile(dev, 99) <= 5.0, (a, np.median(dev),
                                                                           np.percentile(dev, 99))
        cg = 0.5 * np.sum(o._error_fun_triangulation(
            np.hstack([got["kp3d"][a].ravel(), got["joint_len"][a]]), p2, np.array(cons), np.array(weak), sa[3],
            TRI["scale_length"], TRI["scale_length_weak"], TRI["reproj_error_threshold"], "soft_l1",
            TRI["n_deriv_smooth"]) ** 2)
        assert cg <= sa[2].cost * (1 + 1e-3), (a, cg, sa[2].cost)
        _, s3, err = _oracle_scores_errors(o, kp[a], got["kp3d"][a])
        np.testing.assert_array_equal(got["kp3d_score"][a], s3)
        np.testing.assert_allclose(got["kp3d_err"][a], err, rtol=0, atol=1e-6)
    assert len(got["joint_len"]) == A


def test_step4_proc_fixed_joint_lengths(tmp_path):
    """calib/joint_len.npy present -> optim_points_jointlenfix with its median (step4:179-183,
    259-270) and kp3d_fxdJointLen.pickle (:334-336), vs scipy TRF at max_nfev = 15."""
    from mqhip import io as mqio
    from mqhip import synth
    from oracle.geometry import CameraGroupOracle, optim_points_jointlenfix
    from oracle.viterbi import step4_filter_batched
    from src.pipeline import step4_aniposefiltering as step4
    cams, kp2d, root, cfg = _results_dir(tmp_path, A=2, F=40)
    skel = synth.make_skeletons(2, 40)
    cons = synth.constraint_indices(synth.CONSTRAINTS)
    weak = synth.constraint_indices(synth.CONSTRAINTS_WEAK)
    jl_runs = np.array([[np.median(np.linalg.norm(skel[a][:, i] - skel[a][:, j], axis=1)) for i, j in cons + weak]
                        for a in range(2)])
    np.save(os.path.join(os.path.dirname(cfg), "joint_len.npy"), jl_runs)
    step4.proc("demo", root, cfg, 17, redo=True)
    rd = os.path.join(root, "demo")
    assert not os.path.exists(os.path.join(rd, "kp3d.pickle"))
    got = mqio.load_array_pickle(os.path.join(rd, "kp3d_fxdJointLen.pickle"))
    jl = np.median(jl_runs, axis=0)
    o = CameraGroupOracle(cams)
    kp = step4_filter_batched(kp2d).transpose((2, 4, 0, 1, 3))
    for a in range(2):
        np.testing.assert_array_equal(got["joint_len"][a], jl)
        p2, _, _ = _oracle_scores_errors(o, kp[a], np.zeros((40, 17, 3)))
        init = o.triangulate(p2.reshape(8, -1, 2)).reshape(40, 17, 3)
        sa = optim_points_jointlenfix(o, p2, init, jl, cons, weak, ftol=1e-3, max_nfev=15, return_result=True,
                                      **TRI)
        dev = np.linalg.norm(got["kp3d"][a] - sa[0], axis=-1)
        assert np.median(dev) <= 1.0 and np.percentile(dev, 99) <= 5.0, (a, np.median(dev))
        _, s3, err = _oracle_scores_errors(o, kp[a], got["kp3d"][a])
        np.testing.assert_array_equal(got["kp3d_score"][a], s3)
        np.testing.assert_allclose(got["kp3d_err"][a], err, rtol=0, atol=1e-6)


def test_step4_proc_from_h5_calibration(tmp_path, monkeypatch):
    """step4.proc with cam_intrinsic.h5 / cam_extrinsic_optim.h5 next to config.yaml (read through a
    stand-in h5py module; h5py is absent here) rebuilds calibration.toml from them (step4:101-138) and
    gives the same kp3d, bit for bit, as the run on the synthetic calibration.toml of the same cameras."""
    import shutil
    from _fakes import calibration_h5_store, install_fake_h5py
    from mqhip import io as mqio
    from src.pipeline import step4_aniposefiltering as step4
    cams, kp2d, root, cfg = _results_dir(tmp_path, A=2, F=24)
    step4.proc("demo", root, cfg, 17, redo=True)
    ref = mqio.load_array_pickle(os.path.join(root, "demo", "kp3d.pickle"))
    store = calibration_h5_store(cams, os.path.dirname(cfg))
    install_fake_h5py(monkeypatch, store)
    for path in store:
        open(path, "wb").close()
    os.remove(os.path.join(root, "demo", "calibration.toml"))
    shutil.rmtree(os.path.join(root, "demo", "kp2d_f.pickle"), ignore_errors=True)
    step4.proc("demo", root, cfg, 17, redo=True)
    got = mqio.load_array_pickle(os.path.join(root, "demo", "kp3d.pickle"))
    assert os.path.exists(os.path.join(root, "demo", "calibration.toml"))
    for k in ("kp3d", "kp3d_score", "kp3d_err"):
        np.testing.assert_array_equal(got[k], ref[k])
