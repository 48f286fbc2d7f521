"""ORACLE (test infrastructure only): float64 restatement of the anipose / mvpose
geometry on the hot path.

Sources restated (all under /root/reference):
* ``src/third_party/aniposelib/cameras.py``:20-32 (triangulate_simple),
  498-516 (OmnidirCamera.undistort_points / project), 593-637 (triangulate),
  639-743 (triangulate_possible / triangulate_ransac), 746-783 (reprojection_error),
  1116-1190 (optim_points), 1560-1620 (_error_fun_triangulation),
  1670-1697 (_initialize_params_triangulation), 1714-1793 (_jac_sparsity_triangulation),
  129-145 (medfilt_data / interpolate_data).
* ``src/third_party/aniposelib/utils.py``:9-15 (make_M).
* ``src/utils/multicam_toolbox.py``:393-486 (undistortPoints / triangulatePoints).
* cv2.omnidir.projectPoints / undistortPoints / cv2.Rodrigues (opencv-contrib 4.11,
  not installed; restated from the published Mei-model algorithm -- see DESIGN.md,
  "parity unpinned" for the undistort final step).
"""
from __future__ import annotations

import itertools

import numpy as np
from scipy import optimize, signal
from scipy.sparse import dok_matrix


# ----------------------------------------------------------------------------- cameras

def rodrigues(rvec):
    """cv2.Rodrigues(rvec) -> 3x3 (calibration.cpp cvRodrigues2; the same expression as
    Affine3::rotation, which cv2.fisheye.projectPoints uses): r = rvec / theta,
    R = (c I + (1 - c) r r^T) + s [r]_x evaluated entry by entry as OpenCV's Matx expression
    does; theta < DBL_EPSILON returns I."""
    r = np.asarray(rvec, dtype=np.float64).ravel()
    th = np.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2])
    if th < np.finfo(np.float64).eps:
        return np.eye(3)
    c = np.cos(th)
    s = np.sin(th)
    c1 = 1.0 - c
    it = 1.0 / th
    x, y, z = r[0] * it, r[1] * it, r[2] * it
    rrt = np.array([[x * x, x * y, x * z], [x * y, y * y, y * z], [x * z, y * z, z * z]])
    r_x = np.array([[0.0, -z, y], [z, 0.0, -x], [-y, x, 0.0]])
    return (c * np.eye(3) + c1 * rrt) + s * r_x


def make_M(rvec, tvec):
    """utils.py:9-15 -- 4x4 [R|t; 0 0 0 1]."""
    out = np.zeros((4, 4))
    out[:3, :3] = rodrigues(rvec)
    out[:3, 3] = np.asarray(tvec, dtype=np.float64).ravel()
    out[3, 3] = 1
    return out


class OmnidirCam:
    """cameras.py:429-555 OmnidirCamera (only the hot-path methods)."""

    def __init__(self, d):
        self.name = str(d["name"])
        self.K = np.asarray(d["K"], dtype=np.float64)
        self.xi = float(np.ravel(d["xi"])[0])
        self.D = np.asarray(d["D"], dtype=np.float64).ravel()[:4]
        self.rvec = np.asarray(d["rvec"] if "rvec" in d else d["rotation"], dtype=np.float64).ravel()
        self.tvec = np.asarray(d["tvec"] if "tvec" in d else d["translation"], dtype=np.float64).ravel()

    def extrinsics_mat(self):
        return make_M(self.rvec, self.tvec)

    def undistort_points(self, pts):
        """cameras.py:498-507 -> cv2.omnidir.undistortPoints(pts, K, D, xi, I).

        Mei model: normalise with skew, 20 Gauss-Seidel fixed-point iterations
        removing (k1,k2,p1,p2), lift to the unit sphere, R = I, then the pinhole
        reprojection (Xs/Zs) -- the form consistent with the [R|t] DLT of
        cameras.py:20-32 (unpinned against opencv-contrib 4.11).
        """
        shape = pts.shape
        p = np.asarray(pts, dtype=np.float64).reshape(-1, 2)
        fx, fy, cx, cy, s = self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2], self.K[0, 1]
        k1, k2, p1, p2 = self.D
        xi = self.xi
        ppx = (p[:, 0] * fy - cx * fy - s * (p[:, 1] - cy)) / (fx * fy)
        ppy = (p[:, 1] - cy) / fy
        x = ppx.copy()
        y = ppy.copy()
        for _ in range(20):
            r2 = x * x + y * y
            r4 = r2 * r2
            x = (ppx - 2 * p1 * x * y - p2 * (r2 + 2 * x * x)) / (1 + k1 * r2 + k2 * r4)
            y = (ppy - 2 * p2 * x * y - p1 * (r2 + 2 * y * y)) / (1 + k1 * r2 + k2 * r4)
        r2 = x * x + y * y
        a = r2 + 1
        b = 2 * xi * r2
        cc = r2 * xi * xi - 1
        Zs = (-b + np.sqrt(b * b - 4 * a * cc)) / (2 * a)
        Xw = x * (Zs + xi)
        Yw = y * (Zs + xi)
        nrm = np.sqrt(Xw * Xw + Yw * Yw + Zs * Zs)
        Xs, Ys, Zn = Xw / nrm, Yw / nrm, Zs / nrm
        out = np.stack([Xs / Zn, Ys / Zn], axis=-1)
        return out.reshape(shape)

    def project(self, p3d):
        """cameras.py:509-516 -> cv2.omnidir.projectPoints(p, rvec, tvec, K, xi, D)."""
        X = np.asarray(p3d, dtype=np.float64).reshape(-1, 3)
        R = rodrigues(self.rvec)
        t = self.tvec
        Xc0 = R[0, 0] * X[:, 0] + R[0, 1] * X[:, 1] + R[0, 2] * X[:, 2] + t[0]
        Xc1 = R[1, 0] * X[:, 0] + R[1, 1] * X[:, 1] + R[1, 2] * X[:, 2] + t[1]
        Xc2 = R[2, 0] * X[:, 0] + R[2, 1] * X[:, 1] + R[2, 2] * X[:, 2] + t[2]
        nrm = np.sqrt(Xc0 * Xc0 + Xc1 * Xc1 + Xc2 * Xc2)
        xs, ys, zs = Xc0 / nrm, Xc1 / nrm, Xc2 / nrm
        xu = xs / (zs + self.xi)
        yu = ys / (zs + self.xi)
        k1, k2, p1, p2 = self.D
        r2 = xu * xu + yu * yu
        r4 = r2 * r2
        xd = xu * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu * yu + p2 * (r2 + 2 * xu * xu)
        yd = yu * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * yu * yu) + 2 * p2 * xu * yu
        K = self.K
        u = K[0, 0] * xd + K[0, 1] * yd + K[0, 2]
        v = K[1, 1] * yd + K[1, 2]
        return np.stack([u, v], axis=-1)

    def reprojection_error(self, p3d, p2d):
        """cameras.py:326-328 (Camera.reprojection_error)."""
        proj = self.project(p3d).reshape(p2d.shape)
        return p2d - proj


class PinholeCam:
    """cameras.py:173-337 Camera (the hot-path methods) on cv2.undistortPoints / cv2.projectPoints
    (OpenCV 4.11 undistort.dispatch.cpp cvUndistortPointsInternal, calibration.cpp
    cvProjectPoints2Internal) restated for the 4- or 5-coefficient model (k1, k2, p1, p2[, k3]); the
    rational / thin-prism / tilt terms are zero, and the camera matrix's skew entry is not used by
    either function.  cv2 is absent here: parity with OpenCV itself is unpinned."""

    model = 1

    def __init__(self, d):
        self.name = str(d["name"])
        self.K = np.asarray(d["matrix"], dtype=np.float64)
        dist = np.asarray(d.get("distortions", np.zeros(5)), dtype=np.float64).ravel()
        if dist.size < 4 or np.any(dist[5:] != 0):
            raise NotImplementedError("pinhole distortion must be (k1, k2, p1, p2[, k3])")
        self.dist = np.zeros(5)
        self.dist[:min(5, dist.size)] = dist[:5]
        self.rvec = np.asarray(d["rvec"] if "rvec" in d else d["rotation"], dtype=np.float64).ravel()
        self.tvec = np.asarray(d["tvec"] if "tvec" in d else d["translation"], dtype=np.float64).ravel()

    def extrinsics_mat(self):
        return make_M(self.rvec, self.tvec)

    def undistort_points(self, pts):
        """cameras.py:310-316 -> cv2.undistortPoints(pts, K, dist): criteria COUNT 5 (the default of
        the 6-argument overload), R = P = I."""
        shape = pts.shape
        p = np.asarray(pts, dtype=np.float64).reshape(-1, 2)
        fx, fy, cx, cy = self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]
        ifx, ify = 1.0 / fx, 1.0 / fy
        k0, k1, k2, k3, k4 = self.dist
        out = np.empty_like(p)
        for i in range(p.shape[0]):
            u, v = p[i, 0], p[i, 1]
            x = (u - cx) * ifx
            y = (v - cy) * ify
            x0, y0 = x, y
            for _ in range(5):
                r2 = x * x + y * y
                icdist = (1 + ((0.0 * r2 + 0.0) * r2 + 0.0) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2)
                if icdist < 0:
                    x = (u - cx) * ifx
                    y = (v - cy) * ify
                    break
                dx = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + 0.0 * r2 + 0.0 * r2 * r2
                dy = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + 0.0 * r2 + 0.0 * r2 * r2
                x = (x0 - dx) * icdist
                y = (y0 - dy) * icdist
            out[i] = x, y
        return out.reshape(shape)

    def project(self, p3d):
        """cameras.py:318-323 -> cv2.projectPoints(p, rvec, tvec, K, dist)."""
        X = np.asarray(p3d, dtype=np.float64).reshape(-1, 3)
        R = rodrigues(self.rvec)
        t = self.tvec
        x = R[0, 0] * X[:, 0] + R[0, 1] * X[:, 1] + R[0, 2] * X[:, 2] + t[0]
        y = R[1, 0] * X[:, 0] + R[1, 1] * X[:, 1] + R[1, 2] * X[:, 2] + t[1]
        z = R[2, 0] * X[:, 0] + R[2, 1] * X[:, 1] + R[2, 2] * X[:, 2] + t[2]
        with np.errstate(divide="ignore"):
            iz = np.where(z != 0, 1.0 / z, 1.0)
        x = x * iz
        y = y * iz
        k0, k1, k2, k3, k4 = self.dist
        r2 = x * x + y * y
        r4 = r2 * r2
        r6 = r4 * r2
        a1 = 2 * x * y
        a2 = r2 + 2 * x * x
        a3 = r2 + 2 * y * y
        cdist = 1 + k0 * r2 + k1 * r4 + k4 * r6
        xd = x * cdist + k2 * a1 + k3 * a2
        yd = y * cdist + k2 * a3 + k3 * a1
        u = xd * self.K[0, 0] + self.K[0, 2]
        v = yd * self.K[1, 1] + self.K[1, 2]
        return np.stack([u, v], axis=-1)

    def reprojection_error(self, p3d, p2d):
        """cameras.py:325-327."""
        proj = self.project(p3d).reshape(p2d.shape)
        return p2d - proj


class FisheyeCam(PinholeCam):
    """cameras.py:339-426 FisheyeCamera on cv2.fisheye.undistortPoints / cv2.fisheye.projectPoints
    (OpenCV 4.11 fisheye.cpp) restated: equidistant model theta_d = theta (1 + k1 theta^2 + ... +
    k4 theta^8), alpha (skew) 0 as in the reference's calls.  Parity with OpenCV itself is unpinned."""

    model = 2

    def __init__(self, d):
        self.name = str(d["name"])
        self.K = np.asarray(d["matrix"], dtype=np.float64)
        dist = np.asarray(d.get("distortions", np.zeros(4)), dtype=np.float64).ravel()
        if dist.size != 4:
            raise NotImplementedError("fisheye distortion must be (k1, k2, k3, k4)")
        self.dist = dist.copy()
        self.rvec = np.asarray(d["rvec"] if "rvec" in d else d["rotation"], dtype=np.float64).ravel()
        self.tvec = np.asarray(d["tvec"] if "tvec" in d else d["translation"], dtype=np.float64).ravel()

    def undistort_points(self, pts):
        """cameras.py:376-382 -> cv2.fisheye.undistortPoints(pts, K, D): Newton on theta, criteria
        MAX_ITER + EPS (10, 1e-8) (the binding's default); a point that does not converge, or whose
        theta changes sign, comes out as (-1e6, -1e6)."""
        shape = pts.shape
        p = np.asarray(pts, dtype=np.float64).reshape(-1, 2)
        f0, f1, c0, c1 = self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]
        k0, k1, k2, k3 = self.dist
        out = np.empty_like(p)
        for i in range(p.shape[0]):
            pw0 = (p[i, 0] - c0) / f0
            pw1 = (p[i, 1] - c1) / f1
            theta_d = np.sqrt(pw0 * pw0 + pw1 * pw1)
            theta_d = min(max(-np.pi / 2.0, theta_d), np.pi / 2.0)
            converged = False
            theta = theta_d
            scale = 0.0
            if abs(theta_d) > 1e-8:
                for _ in range(10):
                    t2 = theta * theta
                    t4 = t2 * t2
                    t6 = t4 * t2
                    t8 = t6 * t2
                    a, b, c, e = k0 * t2, k1 * t4, k2 * t6, k3 * t8
                    fix = (theta * (1 + a + b + c + e) - theta_d) / (1 + 3 * a + 5 * b + 7 * c + 9 * e)
                    theta = theta - fix
                    if abs(fix) < 1e-8:
                        converged = True
                        break
                scale = np.tan(theta) / theta_d
            else:
                converged = True
            flipped = (theta_d < 0 and theta > 0) or (theta_d > 0 and theta < 0)
            if converged and not flipped:
                out[i] = pw0 * scale, pw1 * scale
            else:
                out[i] = -1000000.0, -1000000.0
        return out.reshape(shape)

    def project(self, p3d):
        """cameras.py:384-390 -> cv2.fisheye.projectPoints(p, rvec, tvec, K, D)."""
        X = np.asarray(p3d, dtype=np.float64).reshape(-1, 3)
        R = rodrigues(self.rvec)
        t = self.tvec
        Y0 = R[0, 0] * X[:, 0] + R[0, 1] * X[:, 1] + R[0, 2] * X[:, 2] + t[0]
        Y1 = R[1, 0] * X[:, 0] + R[1, 1] * X[:, 1] + R[1, 2] * X[:, 2] + t[1]
        Y2 = R[2, 0] * X[:, 0] + R[2, 1] * X[:, 1] + R[2, 2] * X[:, 2] + t[2]
        Y2 = np.where(np.abs(Y2) < np.finfo(np.float64).tiny, 1.0, Y2)
        x0 = Y0 / Y2
        x1 = Y1 / Y2
        r = np.sqrt(x0 * x0 + x1 * x1)
        th = np.arctan(r)
        th2 = th * th
        th3 = th2 * th
        th4 = th2 * th2
        th5 = th4 * th
        th6 = th3 * th3
        th7 = th6 * th
        th8 = th4 * th4
        th9 = th8 * th
        k0, k1, k2, k3 = self.dist
        theta_d = th + k0 * th3 + k1 * th5 + k2 * th7 + k3 * th9
        big = r > 1e-8
        with np.errstate(divide="ignore", invalid="ignore"):
            cdist = np.where(big, theta_d * (1.0 / np.where(big, r, 1.0)), 1.0)
        u = (x0 * cdist) * self.K[0, 0] + self.K[0, 2]
        v = (x1 * cdist) * self.K[1, 1] + self.K[1, 2]
        return np.stack([u, v], axis=-1)


def make_cam(d):
    """cameras.py:1972-1982: the model of each calibration dict (fisheye, else omnidir, else pinhole)."""
    if isinstance(d, (OmnidirCam, PinholeCam)):
        return d
    if d.get("fisheye", False):
        return FisheyeCam(d)
    if d.get("omnidir", False):
        return OmnidirCam(d)
    return PinholeCam(d)


def triangulate_simple(points, camera_mats):
    """cameras.py:20-32 -- homogeneous DLT, last right-singular vector of the 2k x 4 system."""
    num_cams = len(camera_mats)
    A = np.zeros((num_cams * 2, 4))
    for i in range(num_cams):
        x, y = points[i]
        mat = camera_mats[i]
        A[i * 2] = x * mat[2] - mat[0]
        A[i * 2 + 1] = y * mat[2] - mat[1]
    u, s, vh = np.linalg.svd(A, full_matrices=True)
    p3d = vh[-1]
    return p3d[:3] / p3d[3]


class CameraGroupOracle:
    """cameras.py:557-783 CameraGroup hot-path methods."""

    def __init__(self, cam_dicts):
        self.cameras = [make_cam(c) for c in cam_dicts]

    def subset(self, idx):
        g = CameraGroupOracle([])
        g.cameras = [self.cameras[i] for i in idx]
        return g

    def project(self, p3d):
        p3d = np.asarray(p3d, dtype=np.float64).reshape(-1, 3)
        return np.stack([c.project(p3d) for c in self.cameras])

    def undistort(self, points):
        return np.stack([c.undistort_points(np.copy(points[i])) for i, c in enumerate(self.cameras)])

    def triangulate(self, points, undistort=True):
        """cameras.py:593-637."""
        assert points.shape[0] == len(self.cameras)
        one_point = False
        if points.ndim == 2:
            points = points.reshape(-1, 1, 2)
            one_point = True
        if undistort:
            points = self.undistort(points)
        n_cams, n_points, _ = points.shape
        out = np.full((n_points, 3), np.nan)
        cam_mats = np.array([c.extrinsics_mat() for c in self.cameras])
        for ip in range(n_points):
            subp = points[:, ip, :]
            good = ~np.isnan(subp[:, 0])
            if np.sum(good) >= 2:
                out[ip] = triangulate_simple(subp[good], cam_mats[good])
        if one_point:
            out = out[0]
        return out

    def reprojection_error(self, p3ds, p2ds, mean=False):
        """cameras.py:746-783."""
        one_point = False
        if p3ds.ndim == 1 and p2ds.ndim == 2:
            p3ds = p3ds.reshape(1, 3)
            p2ds = p2ds.reshape(-1, 1, 2)
            one_point = True
        n_cams, n_points, _ = p2ds.shape
        assert p3ds.shape == (n_points, 3)
        errors = np.empty((n_cams, n_points, 2))
        for cnum, cam in enumerate(self.cameras):
            errors[cnum] = cam.reprojection_error(p3ds, p2ds[cnum])
        if mean:
            errors_norm = np.linalg.norm(errors, axis=2)
            good = ~np.isnan(errors_norm)
            errors_norm[~good] = 0
            denom = np.sum(good, axis=0).astype('float64')
            denom[denom < 1.5] = np.nan
            errors = np.sum(errors_norm, axis=0) / denom
        if one_point:
            if mean:
                errors = float(errors[0])
            else:
                errors = errors.reshape(-1, 2)
        return errors

    def triangulate_possible(self, points, undistort=True, min_cams=2, threshold=0.5):
        """cameras.py:639-722 for n_possible = 1 (the triangulate_ransac path).

        Subsets come from ``itertools.product`` over ``[(cam, 0), None]`` for each
        camera with a non-NaN point, in ascending camera order; the first subset
        whose error drops below ``threshold`` ends the search (``best`` starts at 200).
        """
        n_cams, n_points, n_possible, _ = points.shape
        assert n_cams == len(self.cameras)
        out = np.full((n_points, 3), np.nan)
        picked_vals = np.zeros((n_cams, n_points, n_possible), dtype=bool)
        errors = np.zeros(n_points)
        points_2d = np.full((n_cams, n_points, 2), np.nan)
        for ip in range(n_points):
            present = {}
            for c in range(n_cams):
                for k in range(n_possible):
                    if not np.isnan(points[c, ip, k, 0]):
                        present.setdefault(c, []).append((c, k))
            for c in present:
                present[c].append(None)
            best_point = None
            best_error = 200
            n_cams_max = len(present)
            for picked in itertools.product(*present.values()):
                picked = [p for p in picked if p is not None]
                if len(picked) < min_cams and len(picked) != n_cams_max:
                    continue
                cnums = [p[0] for p in picked]
                xnums = [p[1] for p in picked]
                pts = points[cnums, ip, xnums]
                cc = self.subset(cnums)
                if len(cnums) == 0:
                    continue  # 0-camera subset: p3d NaN, err NaN -> never accepted
                p3d = cc.triangulate(pts, undistort=undistort)
                err = cc.reprojection_error(p3d, pts, mean=True)
                if err < best_error:
                    best_point = dict(error=err, point=p3d[:3], points=pts, picked=picked)
                    best_error = err
                    if best_error < threshold:
                        break
            if best_point is not None:
                out[ip] = best_point['point']
                cn = [p[0] for p in best_point['picked']]
                xn = [p[1] for p in best_point['picked']]
                picked_vals[cn, ip, xn] = True
                errors[ip] = best_point['error']
                points_2d[cn, ip] = best_point['points']
        return out, picked_vals, points_2d, errors

    def triangulate_ransac(self, points, undistort=True, min_cams=2):
        """cameras.py:724-743."""
        n_cams, n_points, _ = points.shape
        return self.triangulate_possible(points.reshape(n_cams, n_points, 1, 2),
                                         undistort=undistort, min_cams=min_cams)

    def triangulate_ransac_batched(self, points, min_cams=2, threshold=0.5):
        """Same result as ``triangulate_ransac`` (cameras.py:639-743, n_possible = 1), batched
        for clip-sized inputs (config 4: 20,400 points x <= 247 subsets).

        Points are grouped by their set of cameras with a non-NaN observation; within a group
        every subset of ``itertools.product`` order is triangulated for all of the group's
        points in one stacked ``np.linalg.svd`` call on exactly the (2k x 4) matrices of
        ``triangulate_simple`` (no padding, so each SVD is the one the loop version computes).
        The loop's selection rule -- keep a subset iff err < best (best starts at 200), stop
        at the first best < threshold -- reduces to: the first subset with err < threshold,
        else the first occurrence of the minimum error below 200 (NaN errors never win).
        tests/test_oracle_kat.py checks it against ``triangulate_ransac`` pick for pick."""
        C, N, _ = points.shape
        assert C == len(self.cameras)
        und = self.undistort(points)
        mats = np.array([c.extrinsics_mat()[:3] for c in self.cameras])
        out = np.full((N, 3), np.nan)
        picked = np.zeros((C, N, 1), dtype=bool)
        errors = np.zeros(N)
        p2 = np.full((C, N, 2), np.nan)
        present = ~np.isnan(points[:, :, 0])                       # (C, N)
        codes = (present.astype(np.int64) << np.arange(C)[:, None]).sum(0)
        for code in np.unique(codes):
            ips = np.flatnonzero(codes == code)
            cams_p = [c for c in range(C) if (code >> c) & 1]
            n = len(cams_p)
            if n < 2:
                continue    # 0 or 1 camera: p3d NaN, error stays 0 (cameras.py:675)
            errs, p3s, subsets = [], [], []
            for s in range(1 << n):
                sub = [cams_p[i] for i in range(n) if not (s >> (n - 1 - i)) & 1]
                k = len(sub)
                if (k < min_cams and k != n) or k < 2:
                    continue
                x = und[sub][:, ips]                                 # (k, P, 2)
                A = np.empty((len(ips), 2 * k, 4))
                for i, c in enumerate(sub):
                    A[:, 2 * i] = x[i, :, 0:1] * mats[c, 2] - mats[c, 0]
                    A[:, 2 * i + 1] = x[i, :, 1:2] * mats[c, 2] - mats[c, 1]
                vh = np.linalg.svd(A, full_matrices=True)[2]
                p3 = vh[:, -1, :3] / vh[:, -1, 3:4]
                en = np.stack([np.linalg.norm(points[c, ips] - self.cameras[c].project(p3), axis=1)
                               for c in sub], axis=1)                # (P, k)
                # per point: the loop version's np.sum over its (k, 1) error column
                errs.append(np.sum(en, axis=1) / float(k))
                p3s.append(p3)
                subsets.append(sub)
            E = np.array(errs)                                       # (S, P)
            Ef = np.where(np.isnan(E), np.inf, E)
            hit = Ef < threshold
            first_hit = np.argmax(hit, axis=0)
            best = np.argmin(Ef, axis=0)
            sel = np.where(hit.any(axis=0), first_hit, best)
            ok = Ef[sel, np.arange(len(ips))] < 200
            for j, ip in enumerate(ips):
                if not ok[j]:
                    continue
                s = sel[j]
                out[ip] = p3s[s][j]
                errors[ip] = E[s, j]
                picked[subsets[s], ip, 0] = True
                p2[subsets[s], ip] = points[subsets[s], ip]
        return out, picked, p2, errors

    # ------------------------------------------------------------------ optim_points
    def _error_fun_triangulation(self, params, p2ds, constraints, constraints_weak,
                                 scale_smooth, scale_length, scale_length_weak,
                                 reproj_error_threshold, reproj_loss, n_deriv_smooth):
        """cameras.py:1560-1620."""
        n_cams, n_frames, n_joints, _ = p2ds.shape
        n_3d = n_frames * n_joints * 3
        n_c = len(constraints)
        p3ds = params[:n_3d].reshape((n_frames, n_joints, 3))
        jl = np.array(params[n_3d:n_3d + n_c])
        jlw = np.array(params[n_3d + n_c:])
        p3ds_flat = p3ds.reshape(-1, 3)
        p2ds_flat = p2ds.reshape((n_cams, -1, 2))
        errors = self.reprojection_error(p3ds_flat, p2ds_flat)
        errors_reproj = errors[~np.isnan(p2ds_flat)]
        rp = reproj_error_threshold
        errors_reproj = np.abs(errors_reproj)
        if reproj_loss == 'huber':
            bad = errors_reproj > rp
            errors_reproj[bad] = rp * (2 * np.sqrt(errors_reproj[bad] / rp) - 1)
        elif reproj_loss == 'soft_l1':
            errors_reproj = rp * 2 * (np.sqrt(1 + errors_reproj / rp) - 1)
        errors_smooth = np.diff(p3ds, n=n_deriv_smooth, axis=0).ravel() * scale_smooth
        el = np.empty((len(constraints), n_frames))
        for cix, (a, b) in enumerate(constraints):
            lengths = np.linalg.norm(p3ds[:, a] - p3ds[:, b], axis=1)
            el[cix] = 100 * (lengths - jl[cix]) / jl[cix]
        el = el.ravel() * scale_length
        elw = np.empty((len(constraints_weak), n_frames))
        for cix, (a, b) in enumerate(constraints_weak):
            lengths = np.linalg.norm(p3ds[:, a] - p3ds[:, b], axis=1)
            elw[cix] = 100 * (lengths - jlw[cix]) / jlw[cix]
        elw = elw.ravel() * scale_length_weak
        return np.hstack([errors_reproj, errors_smooth, el, elw])

    def _error_fun_triangulation_jointlenfix(self, params, p2ds, joint_len, constraints, constraints_weak,
                                             scale_smooth, scale_length, scale_length_weak,
                                             reproj_error_threshold, reproj_loss, n_deriv_smooth):
        """cameras.py:1355-1415: params = p3d only; the lengths are the fixed ``joint_len``
        (strong first, then weak).  Otherwise the residual set of _error_fun_triangulation."""
        n_cams, n_frames, n_joints, _ = p2ds.shape
        n_3d = n_frames * n_joints * 3
        n_c = len(constraints)
        jl = np.asarray(joint_len, dtype=np.float64)
        x = np.hstack([np.asarray(params, dtype=np.float64)[:n_3d], jl[:n_c], jl[n_c:]])
        return self._error_fun_triangulation(x, p2ds, constraints, constraints_weak, scale_smooth,
                                             scale_length, scale_length_weak, reproj_error_threshold,
                                             reproj_loss, n_deriv_smooth)


def medfilt_data(values, size=15):
    """cameras.py:129-133."""
    padsize = size + 5
    vpad = np.pad(values, (padsize, padsize), mode='reflect')
    vpadf = signal.medfilt(vpad, kernel_size=size)
    return vpadf[padsize:-padsize]


def interpolate_data(vals):
    """cameras.py:135-145."""
    nans = np.isnan(vals)
    out = np.copy(vals)
    try:
        out[nans] = np.interp(nans.nonzero()[0], (~nans).nonzero()[0], vals[~nans])
    except ValueError:
        out[:] = 0
    return out


def initialize_params_triangulation(p3ds, constraints, constraints_weak):
    """cameras.py:1670-1697."""
    jl = np.empty(len(constraints))
    jlw = np.empty(len(constraints_weak))
    for cix, (a, b) in enumerate(constraints):
        jl[cix] = np.median(np.linalg.norm(p3ds[:, a] - p3ds[:, b], axis=1))
    for cix, (a, b) in enumerate(constraints_weak):
        jlw[cix] = np.median(np.linalg.norm(p3ds[:, a] - p3ds[:, b], axis=1))
    all_lengths = np.hstack([jl, jlw])
    med = np.median(all_lengths)
    if med == 0:
        med = 1e-3
    mad = np.median(np.abs(all_lengths - med))
    jl[jl == 0] = med
    jlw[jlw == 0] = med
    jl[jl > med + mad * 5] = med
    jlw[jlw > med + mad * 5] = med
    return np.hstack([p3ds.ravel(), jl, jlw])


def jac_sparsity_triangulation(p2ds, constraints, constraints_weak, n_deriv_smooth=1):
    """cameras.py:1714-1793."""
    n_cams, n_frames, n_joints, _ = p2ds.shape
    n_c = len(constraints)
    n_cw = len(constraints_weak)
    p2ds_flat = p2ds.reshape((n_cams, -1, 2))
    point_indices = np.zeros(p2ds_flat.shape, dtype='int32')
    for i in range(p2ds_flat.shape[1]):
        point_indices[:, i] = i
    point_indices_3d = np.arange(n_frames * n_joints).reshape((n_frames, n_joints))
    good = ~np.isnan(p2ds_flat)
    n_errors_reproj = np.sum(good)
    n_errors_smooth = (n_frames - n_deriv_smooth) * n_joints * 3
    n_errors_lengths = n_c * n_frames
    n_errors_lengths_weak = n_cw * n_frames
    n_errors = n_errors_reproj + n_errors_smooth + n_errors_lengths + n_errors_lengths_weak
    n_3d = n_frames * n_joints * 3
    n_params = n_3d + n_c + n_cw
    point_indices_good = point_indices[good]
    A = dok_matrix((n_errors, n_params), dtype='int16')
    ix_reproj = np.arange(n_errors_reproj)
    for k in range(3):
        A[ix_reproj, point_indices_good * 3 + k] = 1
    frames = np.arange(n_frames - n_deriv_smooth)
    for j in range(n_joints):
        for n in range(n_deriv_smooth + 1):
            pa = point_indices_3d[frames, j]
            pb = point_indices_3d[frames + n, j]
            for k in range(3):
                A[n_errors_reproj + pa * 3 + k, pb * 3 + k] = 1
    start = n_errors_reproj + n_errors_smooth
    frames = np.arange(n_frames)
    for cix, (a, b) in enumerate(constraints):
        A[start + cix * n_frames + frames, n_3d + cix] = 1
    for cix, (a, b) in enumerate(constraints):
        pa = point_indices_3d[frames, a]
        pb = point_indices_3d[frames, b]
        for k in range(3):
            A[start + cix * n_frames + frames, pa * 3 + k] = 1
            A[start + cix * n_frames + frames, pb * 3 + k] = 1
    start = n_errors_reproj + n_errors_smooth + n_errors_lengths
    for cix, (a, b) in enumerate(constraints_weak):
        A[start + cix * n_frames + frames, n_3d + n_c + cix] = 1
    for cix, (a, b) in enumerate(constraints_weak):
        pa = point_indices_3d[frames, a]
        pb = point_indices_3d[frames, b]
        for k in range(3):
            A[start + cix * n_frames + frames, pa * 3 + k] = 1
            A[start + cix * n_frames + frames, pb * 3 + k] = 1
    return A


def optim_init(p3ds, constraints, constraints_weak, scale_smooth):
    """cameras.py:1146-1150: x0 (interpolated p3d + limb lengths, non-finite -> 0) and scale_smooth_full."""
    p3ds_intp = np.apply_along_axis(interpolate_data, 0, p3ds)
    p3ds_med = np.apply_along_axis(medfilt_data, 0, p3ds_intp, size=7)
    default_smooth = 1.0 / np.mean(np.abs(np.diff(p3ds_med, axis=0)))
    scale_smooth_full = scale_smooth * default_smooth
    x0 = initialize_params_triangulation(p3ds_intp, constraints, constraints_weak)
    x0[~np.isfinite(x0)] = 0
    return x0, scale_smooth_full


def optim_points(cgroup, points, p3ds, constraints=(), constraints_weak=(), scale_smooth=4,
                 scale_length=2, scale_length_weak=0.5, reproj_error_threshold=15,
                 reproj_loss='soft_l1', n_deriv_smooth=1, ftol=1e-3, return_result=False):
    """cameras.py:1116-1190 -- scipy TRF with a 2-point FD sparse Jacobian, loss 'linear'."""
    n_cams, n_frames, n_joints, _ = points.shape
    assert n_cams == len(cgroup.cameras)
    constraints = np.array(constraints)
    constraints_weak = np.array(constraints_weak)
    x0, scale_smooth_full = optim_init(p3ds, constraints, constraints_weak, scale_smooth)
    jac = jac_sparsity_triangulation(points, constraints, constraints_weak, n_deriv_smooth)
    res = optimize.least_squares(
        cgroup._error_fun_triangulation, x0=x0, jac_sparsity=jac, loss='linear', ftol=ftol,
        args=(points, constraints, constraints_weak, scale_smooth_full, scale_length,
              scale_length_weak, reproj_error_threshold, reproj_loss, n_deriv_smooth))
    p3ds_new = res.x[:p3ds.size].reshape(p3ds.shape)
    joint_len = res.x[p3ds.size:]
    if return_result:
        return p3ds_new, joint_len, res, scale_smooth_full, x0
    return p3ds_new, joint_len


def jac_sparsity_triangulation_jointlenfix(p2ds, constraints, constraints_weak, n_deriv_smooth=1):
    """cameras.py:1272-1352: the pattern of jac_sparsity_triangulation without the length
    columns (n_params = F*J*3; length residuals depend on the two joints' points only)."""
    A = jac_sparsity_triangulation(p2ds, constraints, constraints_weak, n_deriv_smooth)
    n_cams, n_frames, n_joints, _ = p2ds.shape
    return A.tocsr()[:, :n_frames * n_joints * 3]


def optim_points_jointlenfix(cgroup, points, p3ds, joint_len, constraints=(), constraints_weak=(),
                             scale_smooth=4, scale_length=2, scale_length_weak=0.5,
                             reproj_error_threshold=15, reproj_loss='soft_l1', n_deriv_smooth=1,
                             ftol=1e-3, max_nfev=15, return_result=False):
    """cameras.py:1192-1270 -- scipy TRF on p3d only (lengths fixed to ``joint_len``),
    ftol 1e-3 and **max_nfev = 15** as in the reference."""
    n_cams, n_frames, n_joints, _ = points.shape
    assert n_cams == len(cgroup.cameras)
    constraints = np.array(constraints)
    constraints_weak = np.array(constraints_weak)
    p3ds_intp = np.apply_along_axis(interpolate_data, 0, p3ds)
    p3ds_med = np.apply_along_axis(medfilt_data, 0, p3ds_intp, size=7)
    default_smooth = 1.0 / np.mean(np.abs(np.diff(p3ds_med, axis=0)))
    scale_smooth_full = scale_smooth * default_smooth
    x0 = initialize_params_triangulation(p3ds_intp, constraints, constraints_weak)
    x0[~np.isfinite(x0)] = 0
    x0 = x0[:p3ds.size]
    jac = jac_sparsity_triangulation_jointlenfix(points, constraints, constraints_weak, n_deriv_smooth)
    res = optimize.least_squares(
        cgroup._error_fun_triangulation_jointlenfix, x0=x0, jac_sparsity=jac, loss='linear', ftol=ftol,
        max_nfev=max_nfev,
        args=(points, joint_len, constraints, constraints_weak, scale_smooth_full, scale_length,
              scale_length_weak, reproj_error_threshold, reproj_loss, n_deriv_smooth))
    p3ds_new = res.x[:p3ds.size].reshape(p3ds.shape)
    if return_result:
        return p3ds_new, joint_len, res, scale_smooth_full, x0
    return p3ds_new, joint_len


# ----------------------------------------------------------------------------- mvpose DLT

def mct_triangulate_points(pos_2d_undist, frame_use, pmat):
    """multicam_toolbox.py:433-486 -- inhomogeneous DLT: X = pinv(A[:,:3]) A[:,3], P = -X."""
    n_frame, n_cam = frame_use.shape
    P = np.zeros((n_frame, 3))
    U = pos_2d_undist
    for i_frame in range(n_frame):
        if np.sum(frame_use[i_frame, :]) < 2:
            P[i_frame, :] = np.nan
            continue
        A = []
        for i_cam in range(n_cam):
            if frame_use[i_frame, i_cam]:
                a1 = U[i_cam][i_frame, 0] * pmat[i_cam][2, :] - pmat[i_cam][0, :]
                a2 = U[i_cam][i_frame, 1] * pmat[i_cam][2, :] - pmat[i_cam][1, :]
                A.append(np.vstack((a1, a2)))
        A = np.vstack(A)
        X = np.matmul(np.linalg.pinv(A[:, :3]), A[:, 3])
        P[i_frame, :] = -X
    return P
