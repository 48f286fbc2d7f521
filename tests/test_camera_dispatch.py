"""CPU: CameraGroup.from_dicts / load honour the camera model of each calibration dict
(cameras.py:1972-1982).  Omnidir dicts build OmnidirCameras; fisheye and pinhole dicts raise
instead of being pushed through the omnidir kernels (which would silently return garbage)."""
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


@pytest.mark.parametrize("flags,kind", [({"omnidir": False, "fisheye": False}, "pinhole"),
                                        ({"fisheye": True}, "fisheye"),
                                        ({}, "pinhole")])
def test_non_omnidir_dicts_raise(flags, kind):
    from mqhip.geometry import CameraGroup
    ds = _dicts()
    d = {k: v for k, v in ds[1].items() if k not in ("omnidir", "fisheye")}
    d.update(flags)
    ds[1] = d
    with pytest.raises(NotImplementedError, match=kind):
        CameraGroup.from_dicts(ds)


def test_load_pinhole_calibration_toml_raises(tmp_path):
    from mqhip import io as mqio
    from mqhip.geometry import CameraGroup
    calib = {f"cam_{i}": {"name": str(d["name"]), "size": [2048, 1536],
                          "matrix": np.asarray(d["matrix"]).tolist(), "distortions": [0.0] * 5,
                          "rotation": np.ravel(d["rvec"]).tolist(), "translation": np.ravel(d["tvec"]).tolist()}
             for i, d in enumerate(_dicts())}
    p = tmp_path / "calibration.toml"
    mqio.dump_toml(calib, str(p))
    with pytest.raises(NotImplementedError, match="pinhole"):
        CameraGroup.load(str(p))
