"""CPU: CameraGroup.from_dicts / load build the camera model of each calibration dict
(cameras.py:1972-1982: ``fisheye`` -> FisheyeCamera, ``omnidir`` -> OmnidirCamera, otherwise the
pinhole Camera), and each model packs the 24-double camera row of include/mq_hip.h (slot 22 = model,
slot 23 = the pinhole's k3).  No GPU call."""
import numpy as np
import pytest


def _dicts():
    from mqhip import synth
    return synth.make_cameras(3)


def test_omnidir_dicts_build_omnidir_cameras():
    from mqhip.geometry import CameraGroup, OmnidirCamera
    g = CameraGroup.from_dicts(_dicts())
    assert all(isinstance(c, OmnidirCamera) for c in g.cameras)
    assert g.get_names() == [d["name"] for d in _dicts()]
    assert all(c.param_row()[22] == 0 for c in g.cameras)


@pytest.mark.parametrize("flags,cls", [({"omnidir": False, "fisheye": False}, "Camera"),
                                       ({"fisheye": True}, "FisheyeCamera"),
                                       ({"fisheye": True, "omnidir": True}, "FisheyeCamera"),
                                       ({}, "Camera")])
def test_model_follows_the_dict_flags(flags, cls):
    from mqhip import geometry
    from mqhip.geometry import CameraGroup
    ds = _dicts()
    d = {k: v for k, v in ds[1].items() if k not in ("omnidir", "fisheye")}
    d["distortions"] = np.zeros(4) if cls == "FisheyeCamera" else np.zeros(5)
    d.update(flags)
    ds[1] = d
    g = CameraGroup.from_dicts(ds)
    assert type(g.cameras[1]) is getattr(geometry, cls)
    assert type(g.cameras[0]) is geometry.OmnidirCamera


def test_pinhole_row_layout():
    from mqhip import synth
    from mqhip.geometry import Camera, CameraGroup, rodrigues
    d = synth.make_cameras_model(2, "pinhole")[1]
    cam = CameraGroup.from_dicts([d]).cameras[0]
    assert type(cam) is Camera
    row = cam.param_row()
    m = d["matrix"]
    np.testing.assert_array_equal(row[:6], [m[0, 0], m[1, 1], 0.0, m[0, 2], m[1, 2], 0.0])  # skew unused by cv2
    np.testing.assert_array_equal(row[6:10], d["distortions"][:4])
    np.testing.assert_array_equal(row[10:19], rodrigues(d["rotation"]).ravel())
    np.testing.assert_array_equal(row[19:22], d["translation"])
    assert row[22] == 1 and row[23] == d["distortions"][4]
    # 4 coefficients: k3 = 0; 8 with zero rational terms: accepted; non-zero rational terms: not implemented
    assert Camera(matrix=m, dist=d["distortions"][:4]).param_row()[23] == 0
    Camera(matrix=m, dist=np.r_[d["distortions"], np.zeros(3)]).param_row()
    with pytest.raises(NotImplementedError, match="rational"):
        Camera(matrix=m, dist=np.r_[d["distortions"], 0.1, 0, 0], name="x").param_row()


def test_fisheye_row_layout():
    from mqhip import synth
    from mqhip.geometry import CameraGroup, FisheyeCamera
    d = synth.make_cameras_model(2, "fisheye")[0]
    cam = CameraGroup.from_dicts([d]).cameras[0]
    assert type(cam) is FisheyeCamera
    row = cam.param_row()
    np.testing.assert_array_equal(row[6:10], d["distortions"])
    assert row[2] == 0 and row[5] == 0 and row[22] == 2 and row[23] == 0
    with pytest.raises(NotImplementedError, match="fisheye"):
        FisheyeCamera(matrix=d["matrix"], dist=np.zeros(5)).param_row()


def test_get_dict_flags_like_the_reference():
    """cameras.py:191-199, 361-364, 479-485 (OmnidirCamera writes the capitalised 'Omnidir' key)."""
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    ds = synth.make_cameras(1) + synth.make_cameras_model(2, "pinhole")[1:] + synth.make_cameras_model(1, "fisheye")
    out = CameraGroup.from_dicts(ds).get_dicts()
    assert out[0]["Omnidir"] is True and "fisheye" not in out[1] and out[2]["fisheye"] is True
    assert out[1]["distortions"] == list(ds[1]["distortions"])


def test_load_pinhole_and_fisheye_calibration_toml(tmp_path):
    from mqhip import io as mqio
    from mqhip import synth
    from mqhip.geometry import Camera, CameraGroup, FisheyeCamera
    pin = synth.make_cameras_model(2, "pinhole")
    fis = synth.make_cameras_model(2, "fisheye")
    calib = {}
    for i, d in enumerate([pin[0], fis[1]]):
        calib[f"cam_{i}"] = {"name": str(d["name"]), "size": [2048, 1536], "matrix": np.asarray(d["matrix"]).tolist(),
                             "distortions": np.ravel(d["distortions"]).tolist(), "rotation": np.ravel(d["rotation"]).tolist(),
                             "translation": np.ravel(d["translation"]).tolist(), "fisheye": bool(d["fisheye"])}
    p = tmp_path / "calibration.toml"
    mqio.dump_toml(calib, str(p))
    g = CameraGroup.load(str(p))
    assert [type(c) for c in g.cameras] == [Camera, FisheyeCamera]
    np.testing.assert_array_equal(g.cameras[1].dist, fis[1]["distortions"])


def test_group_parameter_accessors_and_device_rows():
    """cameras.py:1849-1882: rotations / translations get and set; the setters re-pack the device rows."""
    from mqhip import synth
    from mqhip.geometry import CameraGroup, rodrigues
    g = CameraGroup.from_dicts(synth.make_cameras_model(3, "pinhole"))
    r = g.get_rotations()
    t = g.get_translations()
    assert r.shape == (3, 3) and t.shape == (3, 3)
    g._cams_dev = "stale"               # stands in for packed device rows
    g.set_rotations(r[::-1])
    assert g._cams_dev is None          # re-packed on next use
    np.testing.assert_array_equal(g.get_rotations(), r[::-1])
    np.testing.assert_array_equal(g.cameras[0].param_row()[10:19], rodrigues(r[2]).ravel())
    g.set_translations(t + 1.0)
    np.testing.assert_array_equal(g.get_translations(), t + 1.0)
    g.set_names(["a", "b", "c"])
    assert g.get_names() == ["a", "b", "c"]
    c = g.copy()
    c.cameras[0].set_focal_length(5.0)
    assert g.cameras[0].get_focal_length() != 5.0 and c.cameras[0].get_focal_length(both=True) == (5.0, 5.0)


def test_resize_and_dump_load_round_trip(tmp_path):
    """cameras.py:269-277, 1998-2017: resize scales matrix and size; dump -> load keeps pinhole and fisheye
    cameras (an omnidir camera's 'Omnidir' key reloads as pinhole, as in the reference)."""
    from mqhip import synth
    from mqhip.geometry import Camera, CameraGroup, FisheyeCamera, OmnidirCamera
    ds = synth.make_cameras_model(2, "pinhole")[:1] + synth.make_cameras_model(2, "fisheye")[1:] + \
        synth.make_cameras(3)[2:]
    g = CameraGroup.from_dicts(ds)
    g.metadata = {"adjusted": True}
    p = tmp_path / "calib.toml"
    g.dump(str(p))
    h = CameraGroup.load(str(p))
    assert [type(c) for c in h.cameras] == [Camera, FisheyeCamera, Camera]
    assert h.metadata == {"adjusted": True}
    for a, b in zip(g.cameras[:2], h.cameras[:2]):
        np.testing.assert_array_equal(a.param_row(), b.param_row())
    m0 = g.cameras[0].get_camera_matrix().copy()
    g.resize_cameras(0.5)
    np.testing.assert_array_equal(g.cameras[0].get_camera_matrix()[:2], m0[:2] * 0.5)
    assert g.cameras[0].get_camera_matrix()[2, 2] == 1 and tuple(g.cameras[0].get_size()) == (1024.0, 768.0)
    assert isinstance(g.cameras[2], OmnidirCamera)


def test_synthetic_mixed_calibration_toml_round_trip(tmp_path):
    """synth.write_calibration_toml writes pinhole / fisheye dicts in Camera.get_dict's layout next to the
    omnidir ones (the step-4 GPU test's mixed calibration); CameraGroup.load gives the same camera rows."""
    from mqhip import synth
    from mqhip.geometry import Camera, CameraGroup, FisheyeCamera, OmnidirCamera
    cams = synth.make_cameras(8)[:2] + synth.make_cameras_model(8, "pinhole")[2:5] + \
        synth.make_cameras_model(8, "fisheye")[5:]
    p = tmp_path / "calibration.toml"
    synth.write_calibration_toml(cams, str(p))
    g = CameraGroup.load(str(p))
    assert [type(c) for c in g.cameras] == [OmnidirCamera] * 2 + [Camera] * 3 + [FisheyeCamera] * 3
    for a, b in zip(g.cameras, CameraGroup.from_dicts(cams).cameras):
        np.testing.assert_array_equal(a.param_row(), b.param_row())
