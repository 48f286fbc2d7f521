"""Multi-view geometry on MI355X: the aniposelib ``CameraGroup`` surface used by step 4.

Mirrors ``/root/reference/src/third_party/aniposelib/cameras.py`` (Camera :173-337,
FisheyeCamera :339-426, OmnidirCamera :429-555, CameraGroup :557-2017) for the calls step 4 makes
(``src/pipeline/step4_aniposefiltering.py``:212-291): ``load``,
``subset_cameras_names``, ``triangulate``, ``triangulate_ransac``,
``reprojection_error``, ``project``, ``optim_points``.  Inputs/outputs are numpy
float64 like the reference; the arithmetic runs in libmq_hip (float64 HIP kernels).
Shape errors raise AssertionError and unknown camera names IndexError, as in the
reference.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def rodrigues(rvec):
    """cv2.Rodrigues(rvec) (host-side parameter packing only): R = (c I + (1 - c) r r^T) + s [r]_x
    entry by entry, as OpenCV's cvRodrigues2 / Affine3::rotation evaluate it."""
    r = np.asarray(rvec, dtype=np.float64).ravel()
    th = np.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2])
    if th < np.finfo(np.float64).eps:
        return np.eye(3)
    c, s = np.cos(th), np.sin(th)
    c1 = 1.0 - c
    it = 1.0 / th
    x, y, z = r[0] * it, r[1] * it, r[2] * it
    rrt = np.array([[x * x, x * y, x * z], [x * y, y * y, y * z], [x * z, y * z, z * z]])
    r_x = np.array([[0.0, -z, y], [z, 0.0, -x], [-y, x, 0.0]])
    return (c * np.eye(3) + c1 * rrt) + s * r_x


# camera row slot 22 (include/mq_hip.h, csrc/camera.hpp)
MODEL_OMNIDIR, MODEL_PINHOLE, MODEL_FISHEYE = 0, 1, 2


class Camera:
    """Pinhole camera with the field names of aniposelib's Camera (cameras.py:173-337); the
    undistortion / projection (cv2.undistortPoints / cv2.projectPoints, distortions k1, k2, p1, p2[, k3])
    run in libmq_hip (csrc/camera.hpp)."""

    model = MODEL_PINHOLE
    n_dist = 5

    def __init__(self, matrix=None, dist=None, size=None, rvec=None, tvec=None, name=None, extra_dist=False):
        self.matrix = np.eye(3) if matrix is None else np.asarray(matrix, dtype=np.float64)
        self.dist = np.zeros(self.n_dist) if dist is None else np.asarray(dist, dtype=np.float64).ravel()
        self.size = size
        self.rvec = np.zeros(3) if rvec is None else np.asarray(rvec, dtype=np.float64).ravel()
        self.tvec = np.zeros(3) if tvec is None else np.asarray(tvec, dtype=np.float64).ravel()
        self.name = None if name is None else str(name)
        self.extra_dist = extra_dist
        self.R = None  # explicit rotation (from_projection); otherwise rodrigues(rvec)

    @classmethod
    def from_dict(cls, d):
        """cameras.py:201-212 load_dict keys."""
        return cls(matrix=d.get("matrix"), dist=d.get("distortions"), size=d.get("size"),
                   rvec=d.get("rotation", d.get("rvec")), tvec=d.get("translation", d.get("tvec")), name=d.get("name"))

    def load_dict(self, d):
        """cameras.py:201-207: reload this camera's parameters in place from a dict."""
        self.set_camera_matrix(d['matrix'])
        self.set_rotation(d['rotation'])
        self.set_translation(d['translation'])
        self.set_distortions(d['distortions'])
        self.set_name(d['name'])
        self.set_size(d['size'])

    def get_dict(self):
        """cameras.py:191-199."""
        return {"name": self.get_name(), "size": list(self.size) if self.size is not None else None,
                "matrix": self.matrix.tolist(), "distortions": self.dist.tolist(), "rotation": self.rvec.tolist(),
                "translation": self.tvec.tolist()}

    def get_name(self):
        return self.name

    def get_camera_matrix(self):
        return self.matrix

    def get_distortions(self):
        return self.dist

    def get_rotation(self):
        return self.rvec

    def get_translation(self):
        return self.tvec

    def get_extrinsics_mat(self):
        M = np.eye(4)
        M[:3, :3] = rodrigues(self.rvec) if self.R is None else self.R
        M[:3, 3] = self.tvec
        return M

    # cameras.py:214-299 accessors (host-side parameters; a CameraGroup re-packs its rows on every call and
    # re-uploads them when they changed, so any setter -- on the camera or on a group -- takes effect)
    def set_camera_matrix(self, matrix):
        self.matrix = np.array(matrix, dtype=np.float64)

    def set_focal_length(self, fx, fy=None):
        self.matrix[0, 0] = fx
        self.matrix[1, 1] = fx if fy is None else fy

    def get_focal_length(self, both=False):
        fx, fy = self.matrix[0, 0], self.matrix[1, 1]
        return (fx, fy) if both else (fx + fy) / 2.0

    def set_distortions(self, dist):
        self.dist = np.array(dist, dtype=np.float64).ravel()

    def set_rotation(self, rvec):
        self.rvec = np.array(rvec, dtype=np.float64).ravel()
        self.R = None

    def set_translation(self, tvec):
        self.tvec = np.array(tvec, dtype=np.float64).ravel()

    def set_name(self, name):
        self.name = str(name)

    def set_size(self, size):
        self.size = size

    def get_size(self):
        return self.size

    def resize_camera(self, scale):
        """cameras.py:269-277."""
        size = self.get_size()
        self.set_size((size[0] * scale, size[1] * scale))
        m = self.get_camera_matrix() * scale
        m[2, 2] = 1
        self.set_camera_matrix(m)

    def copy(self):
        import copy as _copy
        return _copy.deepcopy(self)

    def _extrinsic_rows(self, row):
        row[10:19] = (rodrigues(self.rvec) if self.R is None else self.R).ravel()
        row[19:22] = self.tvec[:3]
        row[22] = self.model

    def param_row(self):
        """24-double camera row (include/mq_hip.h): fx, fy, 0, cx, cy, 0, k1, k2, p1, p2, R, t, model, k3.
        cv2.projectPoints / undistortPoints take 4, 5, 8, 12 or 14 coefficients; the rational, thin-prism
        and tilt terms past the fifth must be zero here."""
        d = self.dist
        if d.size < 4 or np.any(d[5:] != 0):
            raise NotImplementedError(f"camera {self.name!r}: pinhole distortions must be (k1, k2, p1, p2[, k3]) "
                                      f"(the rational / thin-prism / tilt terms are not implemented), got {d.size}")
        m = self.matrix
        row = np.zeros(24)
        row[0:6] = [m[0, 0], m[1, 1], 0.0, m[0, 2], m[1, 2], 0.0]
        row[6:10] = d[:4]
        row[23] = d[4] if d.size > 4 else 0.0
        self._extrinsic_rows(row)
        return row


class FisheyeCamera(Camera):
    """aniposelib's FisheyeCamera (cameras.py:339-426): cv2.fisheye.undistortPoints / projectPoints,
    distortions k1..k4, alpha 0."""

    model = MODEL_FISHEYE
    n_dist = 4

    def get_dict(self):
        d = super().get_dict()
        d["fisheye"] = True
        return d

    def param_row(self):
        d = self.dist
        if d.size != 4:
            raise NotImplementedError(f"camera {self.name!r}: fisheye distortions must be (k1, k2, k3, k4)")
        m = self.matrix
        row = np.zeros(24)
        row[0:6] = [m[0, 0], m[1, 1], 0.0, m[0, 2], m[1, 2], 0.0]
        row[6:10] = d
        self._extrinsic_rows(row)
        return row


class OmnidirCamera(Camera):
    """Parameter holder with the OmnidirCamera field names (cameras.py:429-555)."""

    model = MODEL_OMNIDIR
    n_dist = 4

    def __init__(self, matrix=None, dist=None, size=None, rvec=None, tvec=None, xi=None, K=None, D=None,
                 name=None, extra_dist=False):
        super().__init__(matrix=matrix, dist=dist, size=size, rvec=rvec, tvec=tvec, name=name, extra_dist=extra_dist)
        self.xi = np.zeros(1) if xi is None else np.asarray(xi, dtype=np.float64).ravel()
        self.K = np.zeros((3, 3)) if K is None else np.asarray(K, dtype=np.float64)
        self.D = np.zeros(4) if D is None else np.asarray(D, dtype=np.float64).ravel()

    @staticmethod
    def from_projection(P, name=None):
        """A camera whose extrinsics are the given 3x4 [R|t] (multicam_toolbox pmat)."""
        P = np.asarray(P, dtype=np.float64)
        cam = OmnidirCamera(tvec=P[:, 3], name=name)
        cam.R = P[:, :3].copy()
        return cam

    @staticmethod
    def from_dict(d):
        return OmnidirCamera(matrix=d.get("matrix"), dist=d.get("distortions"), size=d.get("size"),
                             rvec=d.get("rotation", d.get("rvec")), tvec=d.get("translation", d.get("tvec")),
                             xi=d.get("xi"), K=d.get("K"), D=d.get("D"), name=d.get("name"))

    def load_dict(self, d):
        """cameras.py:442-451."""
        super().load_dict(d)
        self.set_xi(d['xi'])
        self.set_K(d['K'])
        self.set_D(d['D'])

    def get_xi(self):
        return self.xi

    def set_xi(self, xi):
        self.xi = np.array(xi, dtype=np.float64).ravel()

    def get_K(self):
        return self.K

    def set_K(self, K):
        self.K = np.array(K, dtype=np.float64)

    def get_D(self):
        return self.D

    def set_D(self, D):
        self.D = np.array(D, dtype=np.float64).ravel()

    def get_dict(self):
        d = super().get_dict()
        d.update({"Omnidir": True, "xi": self.xi, "K": self.K, "D": self.D})
        return d

    def param_row(self):
        row = np.zeros(24)
        row[0:6] = [self.K[0, 0], self.K[1, 1], self.K[0, 1], self.K[0, 2], self.K[1, 2], float(self.xi[0])]
        row[6:10] = self.D[:4]
        self._extrinsic_rows(row)
        return row


class CameraGroup:
    def __init__(self, cameras, metadata=None, device: int = 0):
        self.cameras = list(cameras)
        self.metadata = {} if metadata is None else metadata
        self.device = device
        self._cams_dev = None
        self._cams_host = None

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_dicts(arr, device: int = 0):
        """cameras.py:1972-1982: the camera model is chosen per dict -- ``fisheye`` -> FisheyeCamera,
        ``omnidir`` -> OmnidirCamera, otherwise the pinhole Camera; groups may mix models."""
        cams = []
        for d in arr:
            if d.get("fisheye", False):
                cams.append(FisheyeCamera.from_dict(d))
            elif d.get("omnidir", False):
                cams.append(OmnidirCamera.from_dict(d))
            else:
                cams.append(Camera.from_dict(d))
        return CameraGroup(cams, device=device)

    def get_dicts(self):
        """cameras.py:1966-1970."""
        return [c.get_dict() for c in self.cameras]

    @staticmethod
    def load(path, device: int = 0):
        """cameras.py:2006-2013 (TOML calibration; every camera model)."""
        try:
            import tomllib as _toml  # py >= 3.11
        except ImportError:  # pragma: no cover - py3.10 image
            import tomli as _toml
        with open(path, "rb") as f:
            master = _toml.load(f)
        keys = sorted([k for k in master.keys() if k != "metadata"])
        items = [master[k] for k in keys]
        g = CameraGroup.from_dicts(items, device=device)
        g.metadata = master.get("metadata", {})
        return g

    def get_names(self):
        return [c.get_name() for c in self.cameras]

    # cameras.py:1849-1889, 1994-2017: host-side parameter access; setters invalidate the device rows
    def invalidate(self):
        """Drop the cached device rows (cams_tensor re-packs on every call anyway)."""
        self._cams_dev = None
        self._cams_host = None

    def copy(self):
        import copy as _copy
        return CameraGroup([c.copy() for c in self.cameras], _copy.copy(self.metadata), self.device)

    def set_rotations(self, rvecs):
        for cam, rvec in zip(self.cameras, rvecs):
            cam.set_rotation(rvec)
        self.invalidate()

    def set_translations(self, tvecs):
        for cam, tvec in zip(self.cameras, tvecs):
            cam.set_translation(tvec)
        self.invalidate()

    def get_rotations(self):
        return np.array([cam.get_rotation() for cam in self.cameras])

    def get_translations(self):
        return np.array([cam.get_translation() for cam in self.cameras])

    def set_names(self, names):
        for cam, name in zip(self.cameras, names):
            cam.set_name(name)

    def average_error(self, p2ds, median=False):
        """cameras.py:1883-1889: mean (or median) per-point reprojection error of the DLT points."""
        p3ds = self.triangulate(p2ds)
        errors = self.reprojection_error(p3ds, p2ds, mean=True)
        return np.median(errors) if median else np.mean(errors)

    def load_dicts(self, arr):
        """cameras.py:1994-1996: each camera reloads its parameters in place (subset groups and outside
        references to the camera objects see the new values)."""
        for cam, d in zip(self.cameras, arr):
            cam.load_dict(d)
        self.invalidate()

    def dump(self, fname):
        """cameras.py:1998-2004: TOML with cam_<i> tables and the metadata.  As in the reference, an
        OmnidirCamera's dict carries the key 'Omnidir' (cameras.py:479-485) while from_dicts tests 'omnidir',
        so a dumped omnidir group loads back as pinhole cameras; the pipeline's own calibration.toml is
        written by step 4 with 'omnidir = true'."""
        from .io import dump_toml
        dicts = self.get_dicts()
        master = {f"cam_{i}": _toml_ready(d) for i, d in enumerate(dicts)}
        master["metadata"] = self.metadata
        dump_toml(master, fname)

    def resize_cameras(self, scale):
        for cam in self.cameras:
            cam.resize_camera(scale)
        self.invalidate()

    def subset_cameras(self, indices):
        return CameraGroup([self.cameras[i] for i in indices], self.metadata, self.device)

    def subset_cameras_names(self, names):
        cur = self.get_names()
        d = dict(zip(cur, range(len(cur))))
        idx = []
        for n in names:
            if n not in d:
                raise IndexError("name {} not part of camera names: {}".format(n, cur))
            idx.append(d[n])
        return self.subset_cameras(idx)

    # ------------------------------------------------------------------ device plumbing
    def _dev(self):
        return torch.device("cuda", self.device)

    def cams_tensor(self):
        """The (C, 24) f64 device rows.  Re-packed from the cameras on every call (the reference reads the
        parameters on every call too; C x 24 doubles is cheap) and re-uploaded only when they changed, so a
        setter on a camera, on this group or on a group sharing the camera objects is never missed."""
        rows = np.stack([c.param_row() for c in self.cameras])
        if self._cams_dev is None or self._cams_host is None or rows.tobytes() != self._cams_host.tobytes():
            self._cams_host = rows
            self._cams_dev = torch.from_numpy(rows.copy()).to(self._dev())
        return self._cams_dev

    def _ctx(self):
        return _lib.Context.get(self.device)

    def _to_dev(self, a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(self._dev())

    # ------------------------------------------------------------------ API
    def project(self, points):
        """Nx3 -> CxNx2 (cameras.py:573-584)."""
        p = np.asarray(points, dtype=np.float64).reshape(-1, 3)
        n, C = p.shape[0], len(self.cameras)
        ctx = self._ctx()
        out = torch.empty((C, n, 2), dtype=torch.float64, device=self._dev())
        p_d = self._to_dev(p)  # keep device temporaries alive until the call is enqueued
        _lib.check(ctx.lib.mq_camera_project(ctx.handle, _lib.ptr(self.cams_tensor()), C, _lib.ptr(p_d),
                                              n, _lib.ptr(out), _lib.stream_ptr(self._dev())), "mq_camera_project")
        return out.cpu().numpy()

    def undistort_points(self, points):
        pts = np.asarray(points, dtype=np.float64)
        C = len(self.cameras)
        assert pts.shape[0] == C
        shape = pts.shape
        flat = pts.reshape(C, -1, 2)
        n = flat.shape[1]
        ctx = self._ctx()
        out = torch.empty((C, n, 2), dtype=torch.float64, device=self._dev())
        flat_d = self._to_dev(flat)
        _lib.check(ctx.lib.mq_camera_undistort(ctx.handle, _lib.ptr(self.cams_tensor()), C,
                                                _lib.ptr(flat_d), n, _lib.ptr(out),
                                                _lib.stream_ptr(self._dev())), "mq_camera_undistort")
        return out.cpu().numpy().reshape(shape)

    def triangulate(self, points, undistort=True, progress=False):
        """CxNx2 -> Nx3 (cameras.py:593-637)."""
        assert points.shape[0] == len(self.cameras), \
            "Invalid points shape, first dim should be equal to" \
            " number of cameras ({}), but shape is {}".format(len(self.cameras), points.shape)
        one_point = False
        if len(points.shape) == 2:
            points = points.reshape(-1, 1, 2)
            one_point = True
        C, n, _ = points.shape
        ctx = self._ctx()
        out = torch.empty((n, 3), dtype=torch.float64, device=self._dev())
        pts_d = self._to_dev(points)
        _lib.check(ctx.lib.mq_triangulate_dlt(ctx.handle, _lib.ptr(self.cams_tensor()), C,
                                              _lib.ptr(pts_d), n, 1 if undistort else 0, _lib.ptr(out),
                                              _lib.stream_ptr(self._dev())), "mq_triangulate_dlt")
        res = out.cpu().numpy()
        return res[0] if one_point else res

    def triangulate_ransac(self, points, undistort=True, min_cams=2, progress=False, threshold=0.5):
        """CxNx2 -> (p3d Nx3, picked CxNx1, p2ds CxNx2, errors N) (cameras.py:639-743)."""
        assert points.shape[0] == len(self.cameras), \
            "Invalid points shape, first dim should be equal to" \
            " number of cameras ({}), but shape is {}".format(len(self.cameras), points.shape)
        if not undistort:
            raise NotImplementedError("triangulate_ransac(undistort=False) is not on the reference's path")
        C, n, _ = points.shape
        ctx = self._ctx()
        dev = self._dev()
        p3d = torch.empty((n, 3), dtype=torch.float64, device=dev)
        picked = torch.empty((C, n), dtype=torch.uint8, device=dev)
        p2d = torch.empty((C, n, 2), dtype=torch.float64, device=dev)
        err = torch.empty((n,), dtype=torch.float64, device=dev)
        pts_d = self._to_dev(points)
        _lib.check(ctx.lib.mq_triangulate_ransac(ctx.handle, _lib.ptr(self.cams_tensor()), C,
                                                 _lib.ptr(pts_d), n, int(min_cams), float(threshold),
                                                 _lib.ptr(p3d), _lib.ptr(picked), _lib.ptr(p2d), _lib.ptr(err),
                                                 _lib.stream_ptr(dev)), "mq_triangulate_ransac")
        return (p3d.cpu().numpy(), picked.cpu().numpy().astype(bool).reshape(C, n, 1), p2d.cpu().numpy(),
                err.cpu().numpy())

    def reprojection_error(self, p3ds, p2ds, mean=False):
        """cameras.py:746-783."""
        one_point = False
        if len(p3ds.shape) == 1 and len(p2ds.shape) == 2:
            p3ds = p3ds.reshape(1, 3)
            p2ds = p2ds.reshape(-1, 1, 2)
            one_point = True
        C, n, _ = p2ds.shape
        assert p3ds.shape == (n, 3), \
            "shapes of 2D and 3D points are not consistent: 2D={}, 3D={}".format(p2ds.shape, p3ds.shape)
        ctx = self._ctx()
        dev = self._dev()
        out = torch.empty((n,) if mean else (C, n, 2), dtype=torch.float64, device=dev)
        p3_d, p2_d = self._to_dev(p3ds), self._to_dev(p2ds)
        _lib.check(ctx.lib.mq_reproj_error(ctx.handle, _lib.ptr(self.cams_tensor()), C, _lib.ptr(p3_d),
                                           _lib.ptr(p2_d), n, 1 if mean else 0, _lib.ptr(out),
                                           _lib.stream_ptr(dev)), "mq_reproj_error")
        errors = out.cpu().numpy()
        if one_point:
            errors = float(errors[0]) if mean else errors.reshape(-1, 2)
        return errors

    def optim_points(self, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4, scale_length=2,
                     scale_length_weak=0.5, reproj_error_threshold=15, reproj_loss='soft_l1', n_deriv_smooth=1,
                     scores=None, verbose=False):
        """cameras.py:1116-1190 on the GPU (see mqhip.optim)."""
        from .optim import optim_points_gpu
        return optim_points_gpu(self, points, p3ds, constraints=constraints, constraints_weak=constraints_weak,
                                scale_smooth=scale_smooth, scale_length=scale_length,
                                scale_length_weak=scale_length_weak, reproj_error_threshold=reproj_error_threshold,
                                reproj_loss=reproj_loss, n_deriv_smooth=n_deriv_smooth, scores=scores,
                                verbose=verbose)

    def optim_points_jointlenfix(self, points, p3ds, joint_len, constraints=(), constraints_weak=(), scale_smooth=4,
                                 scale_length=2, scale_length_weak=0.5, reproj_error_threshold=15,
                                 reproj_loss='soft_l1', n_deriv_smooth=1, scores=None, verbose=False):
        """cameras.py:1192-1415: lengths fixed to joint_len, p3d only; the reference caps scipy at
        max_nfev=15 (the initial evaluation + 14 trial steps): the trf solver takes the same cap, the LM solver
        at most 14 trial steps."""
        from .optim import optim_points_gpu
        joint_len = np.asarray(joint_len, dtype=np.float64).ravel()
        p3, _ = optim_points_gpu(self, points, p3ds, constraints=constraints, constraints_weak=constraints_weak,
                                 scale_smooth=scale_smooth, scale_length=scale_length,
                                 scale_length_weak=scale_length_weak, reproj_error_threshold=reproj_error_threshold,
                                 reproj_loss=reproj_loss, n_deriv_smooth=n_deriv_smooth, scores=scores,
                                 verbose=verbose, joint_len=joint_len, max_iter=14, max_nfev=15)
        return p3, joint_len


def _toml_ready(d):
    """numpy arrays / scalars of a camera dict as TOML-serialisable lists and floats."""
    out = {}
    for k, v in d.items():
        if isinstance(v, np.ndarray):
            out[k] = v.tolist()
        elif isinstance(v, (np.floating, np.integer)):
            out[k] = v.item()
        elif v is None:
            continue
        else:
            out[k] = v
    return out


def triangulate_pinv(cams: CameraGroup, und, frame_use):
    """multicam_toolbox.triangulatePoints on the GPU: und (C,N,2) undistorted, frame_use (N,C) bool."""
    und = np.asarray(und, dtype=np.float64)
    C, n, _ = und.shape
    ctx = cams._ctx()
    dev = cams._dev()
    use = torch.from_numpy(np.ascontiguousarray(frame_use, dtype=np.uint8)).to(dev)
    out = torch.empty((n, 3), dtype=torch.float64, device=dev)
    und_d = cams._to_dev(und)
    _lib.check(ctx.lib.mq_triangulate_pinv(ctx.handle, _lib.ptr(cams.cams_tensor()), C, _lib.ptr(und_d),
                                           _lib.ptr(use), n, _lib.ptr(out), _lib.stream_ptr(dev)),
               "mq_triangulate_pinv")
    return out.cpu().numpy()


def viterbi_filter(kp2d, score_threshold=0.3, n_back=3, offset_threshold=25, device: int = 0):
    """Batched filter_pose_viterbi over kp2d (A,F,C,J,3) -> filtered (A,F,C,J,3) (step4:142-167)."""
    kp = np.ascontiguousarray(kp2d, dtype=np.float64)
    A, F, C, J, _ = kp.shape
    ctx = _lib.Context.get(device)
    dev = torch.device("cuda", device)
    src = torch.from_numpy(kp).to(dev)
    out = torch.empty_like(src)
    _lib.check(ctx.lib.mq_viterbi_filter(ctx.handle, _lib.ptr(src), A, F, C, J, float(score_threshold), int(n_back),
                                         float(offset_threshold), _lib.ptr(out), _lib.stream_ptr(dev)),
               "mq_viterbi_filter")
    return out.cpu().numpy()
