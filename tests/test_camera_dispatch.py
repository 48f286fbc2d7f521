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


def test_device_rows_follow_camera_setters_and_shared_subsets(monkeypatch):
    """cams_tensor re-packs the rows on every call, so a setter on a camera object (not only the
    group's setters), on an OmnidirCamera's K / xi / D, or through a parent group that shares the camera
    objects with a subset group, is never answered with stale rows; load_dicts updates the cameras in place
    (cameras.py:1994-1996), so subset groups see the reloaded values.  Device rows on the CPU here."""
    import torch
    from mqhip import synth
    from mqhip.geometry import CameraGroup
    g = CameraGroup.from_dicts(synth.make_cameras(3))
    sub = g.subset_cameras([2, 0])
    for grp in (g, sub):
        monkeypatch.setattr(grp, "_dev", lambda: torch.device("cpu"))
    r0 = g.cams_tensor().clone()
    assert g.cams_tensor() is g.cams_tensor()                        # unchanged rows: no re-upload
    g.cameras[0].set_K(np.asarray(g.cameras[0].K) * 2.0)
    np.testing.assert_array_equal(g.cams_tensor()[0, 0].item(), 2.0 * r0[0, 0].item())
    np.testing.assert_array_equal(sub.cams_tensor()[1].numpy(), g.cams_tensor()[0].numpy())
    g.cameras[2].set_rotation([0.1, 0.2, 0.3])
    np.testing.assert_array_equal(sub.cams_tensor()[0].numpy(), g.cameras[2].param_row())
    d = synth.make_cameras(3, seed_ext=7)
    g.load_dicts([{**c, "rotation": c["rvec"], "translation": c["tvec"]} for c in d])
    assert sub.cameras[0] is g.cameras[2]
    np.testing.assert_array_equal(sub.cams_tensor()[0, 19:22].numpy(), np.ravel(d[2]["tvec"]))
    assert not np.array_equal(sub.cams_tensor().numpy(), r0[[2, 0]].numpy())


def test_integration_stub_cam_rows_runs_and_matches_the_library_rows():
    """INTEGRATION.md's Option-B stub packs camera rows through mqhip.geometry (no cv2).
    Its ``_cam_rows`` is executed here on reference-style camera objects (get_dict() as cameras.py:191-199,
    361-364, 479-485) with torch's .cuda() stubbed, and must equal synth.camera_array."""
    import os
    import re
    from types import SimpleNamespace
    from mqhip import geometry as mq
    from mqhip import synth
    text = open(os.path.join(os.path.dirname(__file__), "..", "INTEGRATION.md")).read()
    block = re.search(r"```python\n(.*?)```", text, re.S).group(1)
    src = block[block.index("def _cam_rows"):block.index("def triangulate")]
    fake_torch = SimpleNamespace(from_numpy=lambda a: SimpleNamespace(cuda=lambda: a))
    ns = {"np": np, "torch": fake_torch, "_mq": mq}
    exec(src, ns)

    class RefStyle:                                   # what the reference's OmnidirCamera.get_dict returns
        def __init__(self, c):
            self.c = c

        def get_dict(self):
            c = self.c
            return {"name": c["name"], "size": list(c["size"]), "matrix": np.asarray(c["matrix"]).tolist(),
                    "distortions": np.ravel(c["distortions"]).tolist(), "rotation": np.ravel(c["rvec"]).tolist(),
                    "translation": np.ravel(c["tvec"]).tolist(), "Omnidir": True, "xi": c["xi"], "K": c["K"],
                    "D": c["D"]}

    cams = synth.make_cameras(4)
    np.testing.assert_array_equal(ns["_cam_rows"]([RefStyle(c) for c in cams]), synth.camera_array(cams))
    pin = synth.make_cameras_model(2, "pinhole")
    ref = np.stack([mq.Camera.from_dict(d).param_row() for d in pin])
    np.testing.assert_array_equal(ns["_cam_rows"]([mq.Camera.from_dict(d) for d in pin]), ref)
