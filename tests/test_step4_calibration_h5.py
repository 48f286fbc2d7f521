"""CPU: step 4's calibration writer (reference step4_aniposefiltering.py:101-138) against a stand-in
h5py module (h5py is absent in this image).  Field by field: the 8-camera template
(configs/calibration_tmpl.toml), ``mtx[:2, :] /= 2``, the ravel of dist / xi / D, K as stored, the name
= the camera id, rvec / tvec raveled; then step4.proc's own load of the written file
(CameraGroup.load(...).subset_cameras_names(ID), step4:212-213) gives the synthetic cameras' rows."""
import os

import numpy as np
import pytest
import yaml

from _fakes import calibration_h5_store, install_fake_h5py


def _setup(tmp_path, monkeypatch, n_cams=8, order=None):
    from mqhip import synth
    cams = synth.make_cameras(n_cams)
    cal = tmp_path / "calib"
    cal.mkdir()
    ids = [int(c["name"]) for c in cams]
    if order is not None:
        ids = [ids[i] for i in order]
    with open(cal / "config.yaml", "w") as f:
        yaml.safe_dump({"camera_id": ids}, f)
    install_fake_h5py(monkeypatch, calibration_h5_store(cams, str(cal)))
    rd = tmp_path / "results" / "demo"
    rd.mkdir(parents=True)
    return cams, [str(i) for i in ids], str(cal / "config.yaml"), str(rd)


@pytest.mark.parametrize("order", [None, [3, 1, 0, 2, 7, 6, 5, 4]])
def test_write_calibration_fields(tmp_path, monkeypatch, order):
    from mqhip import io as mqio
    from src.pipeline import step4_aniposefiltering as step4
    cams, ids, cfg, rd = _setup(tmp_path, monkeypatch, order=order)
    step4.write_calibration(cfg, rd, ids)
    got = mqio.load_toml(os.path.join(rd, "calibration.toml"))
    assert list(got) == [f"cam_{i}" for i in range(8)]
    by_name = {str(c["name"]): c for c in cams}
    for i, k in enumerate(ids):
        e, c = got[f"cam_{i}"], by_name[k]
        assert list(e) == ["name", "size", "matrix", "distortions", "rotation", "translation", "fisheye", "omnidir",
                           "xi", "K", "D"]                                 # template keys first, then xi / K / D
        assert e["name"] == k and e["size"] == [2048, 1536] and e["fisheye"] is False and e["omnidir"] is True
        np.testing.assert_array_equal(np.array(e["matrix"]), np.asarray(c["matrix"]))   # (2 x mtx)[:2] / 2
        np.testing.assert_array_equal(e["distortions"], np.ravel(c["distortions"])[:4])
        np.testing.assert_array_equal(e["xi"], np.ravel(c["xi"]))
        np.testing.assert_array_equal(np.array(e["K"]), np.asarray(c["K"]))
        np.testing.assert_array_equal(e["D"], np.ravel(c["D"]))
        np.testing.assert_array_equal(e["rotation"], np.ravel(c["rvec"]))
        np.testing.assert_array_equal(e["translation"], np.ravel(c["tvec"]))
        assert len(e["xi"]) == 1 and len(e["D"]) == 4 and len(e["rotation"]) == 3


def test_write_calibration_keeps_template_entries_and_rejects_a_ninth_camera(tmp_path, monkeypatch):
    """Fewer cameras than the template: the remaining template entries keep their zeros and names "k+1";
    more than eight: KeyError, as the reference's calib['cam_8'] lookup."""
    from mqhip import io as mqio
    from src.pipeline import step4_aniposefiltering as step4
    cams, ids, cfg, rd = _setup(tmp_path, monkeypatch, n_cams=5)
    step4.write_calibration(cfg, rd, ids)
    got = mqio.load_toml(os.path.join(rd, "calibration.toml"))
    assert len(got) == 8
    for i in range(5, 8):
        e = got[f"cam_{i}"]
        assert e["name"] == str(i + 1) and e["matrix"] == [[0.0] * 3] * 3 and e["rotation"] == [0, 0, 0]
        assert "xi" not in e
    with pytest.raises(KeyError):
        step4.write_calibration(cfg, rd, ids + ["a", "b", "c", "d"])


def test_step4_proc_writes_and_loads_h5_calibration(tmp_path, monkeypatch):
    """step4.proc with the two h5 files present rebuilds calibration.toml from them (a stale toml is
    overwritten) and hands step 4's reconstruction the camera group of the config's IDs; the GPU stages
    are stubbed here and run for real in tests/test_gpu_pipeline.py::test_step4_proc_from_h5_calibration."""
    from mqhip import io as mqio
    from mqhip import synth
    from src.pipeline import step4_aniposefiltering as step4
    cams, ids, cfg, rd = _setup(tmp_path, monkeypatch, order=[3, 1, 0, 2, 7, 6, 5, 4])
    for path in calibration_h5_store(cams, os.path.dirname(cfg)):
        open(path, "wb").close()                                           # proc tests for the files
    with open(os.path.join(rd, "calibration.toml"), "w") as f:
        f.write("[cam_0]\nname = \"stale\"\n")
    mqio.dump_pickle(np.zeros((1, 2, 8, 17, 3)), os.path.join(rd, "kp2d.pickle"))
    seen = {}
    monkeypatch.setattr(step4, "filter_2d", lambda kp2d, device=0: np.zeros((2, 17, 1, 3, 8)))

    def fake_reconstruct(kp2d_f, cgroup, config, joint_len_median=None, verbose=False):
        seen["names"] = cgroup.get_names()
        seen["rows"] = np.stack([c.param_row() for c in cgroup.cameras])
        return np.zeros((1, 2, 17, 3)), np.zeros((1, 2, 17)), np.zeros((1, 2, 17)), [np.zeros(31)]

    monkeypatch.setattr(step4, "reconstruct_3d", fake_reconstruct)
    step4.proc("demo", os.path.dirname(rd), cfg, 17, redo=True)
    assert seen["names"] == ids
    by_name = {str(c["name"]): c for c in cams}
    np.testing.assert_array_equal(seen["rows"], synth.camera_array([by_name[k] for k in ids]))
