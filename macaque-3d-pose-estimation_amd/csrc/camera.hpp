// Camera models of aniposelib's CameraGroup (cameras.py:173-555) as float64 device functions:
// undistort (pixel -> normalised image plane) and project (world -> pixel) for the three models
// CameraGroup.from_dicts builds (cameras.py:1972-1982).  The row's `model` slot selects one:
//
//   0  OmnidirCamera  cv2.omnidir.undistortPoints / projectPoints (Mei model; k1, k2, p1, p2, xi, skew)
//   1  Camera         cv2.undistortPoints / projectPoints (k1, k2, p1, p2 in slots 6-9, k3 in slot 23;
//                     the matrix's skew entry is not used by either OpenCV function)
//   2  FisheyeCamera  cv2.fisheye.undistortPoints / projectPoints (k1..k4 in slots 6-9, alpha = 0)
//
// Each function restates the OpenCV 4.11 routine with its operation order (the translation units are
// built with -ffp-contract=off) so that the numpy restatements in oracle/geometry.py give the same bits;
// the fisheye model also calls atan / tan, which may differ from glibc's by an ulp.
#pragma once
#include "common.hpp"

namespace mq {

enum CamModel { CAM_OMNIDIR = 0, CAM_PINHOLE = 1, CAM_FISHEYE = 2 };

// the row's model as an int; -1 (no model) for a non-integral slot
__device__ __forceinline__ int cam_model(const CamParams& cp) {
  return cp.model == (double)(int)cp.model ? (int)cp.model : -1;
}

// cv2.omnidir.undistortPoints(p, K, D, xi, R = I) restated (oracle/geometry.py OmnidirCam).
__device__ __forceinline__ void omni_undistort(const CamParams& cp, double u, double v, double& ox, double& oy) {
  const double fx = cp.fx, fy = cp.fy, cx = cp.cx, cy = cp.cy, s = cp.skew;
  const double ppx = (u * fy - cx * fy - s * (v - cy)) / (fx * fy);
  const double ppy = (v - cy) / fy;
  double x = ppx, y = ppy;
  for (int it = 0; it < 20; ++it) {
    const double r2 = x * x + y * y;
    const double r4 = r2 * r2;
    x = (ppx - 2 * cp.p1 * x * y - cp.p2 * (r2 + 2 * x * x)) / (1 + cp.k1 * r2 + cp.k2 * r4);
    y = (ppy - 2 * cp.p2 * x * y - cp.p1 * (r2 + 2 * y * y)) / (1 + cp.k1 * r2 + cp.k2 * r4);
  }
  const double xi = cp.xi;
  const double r2 = x * x + y * y;
  const double a = r2 + 1;
  const double b = 2 * xi * r2;
  const double cc = r2 * xi * xi - 1;
  const double Zs = (-b + sqrt(b * b - 4 * a * cc)) / (2 * a);
  const double Xw = x * (Zs + xi), Yw = y * (Zs + xi);
  const double nrm = sqrt(Xw * Xw + Yw * Yw + Zs * Zs);
  const double Xs = Xw / nrm, Ys = Yw / nrm, Zn = Zs / nrm;
  ox = Xs / Zn;
  oy = Ys / Zn;
}

// cv2.omnidir.projectPoints(X, rvec, tvec, K, xi, D) restated.
__device__ __forceinline__ void omni_project(const CamParams& cp, double X, double Y, double Z, double& u,
                                             double& v) {
  const double* R = cp.R;
  const double x0 = R[0] * X + R[1] * Y + R[2] * Z + cp.t[0];
  const double x1 = R[3] * X + R[4] * Y + R[5] * Z + cp.t[1];
  const double x2 = R[6] * X + R[7] * Y + R[8] * Z + cp.t[2];
  const double nrm = sqrt(x0 * x0 + x1 * x1 + x2 * x2);
  const double xs = x0 / nrm, ys = x1 / nrm, zs = x2 / nrm;
  const double xu = xs / (zs + cp.xi), yu = ys / (zs + cp.xi);
  const double r2 = xu * xu + yu * yu;
  const double r4 = r2 * r2;
  const double xd = xu * (1 + cp.k1 * r2 + cp.k2 * r4) + 2 * cp.p1 * xu * yu + cp.p2 * (r2 + 2 * xu * xu);
  const double yd = yu * (1 + cp.k1 * r2 + cp.k2 * r4) + cp.p1 * (r2 + 2 * yu * yu) + 2 * cp.p2 * xu * yu;
  u = cp.fx * xd + cp.skew * yd + cp.cx;
  v = cp.fy * yd + cp.cy;
}

// cv2.undistortPoints(p, K, dist) (undistort.dispatch.cpp cvUndistortPointsInternal): criteria COUNT 5,
// no tilt, R = P = I; the rational and thin-prism terms are zero (numerator of icdist = 1, their
// deltas + 0).  A negative icdist restores the undistorted-only estimate and stops.
__device__ __forceinline__ void pinhole_undistort(const CamParams& cp, double u, double v, double& ox, double& oy) {
  const double ifx = 1. / cp.fx, ify = 1. / cp.fy;
  double x = (u - cp.cx) * ifx, y = (v - cp.cy) * ify;
  const double x0 = x, y0 = y;
  for (int j = 0; j < 5; ++j) {
    const double r2 = x * x + y * y;
    const double icdist = 1 / (1 + ((cp.k3 * r2 + cp.k2) * r2 + cp.k1) * r2);
    if (icdist < 0) {
      x = (u - cp.cx) * ifx;
      y = (v - cp.cy) * ify;
      break;
    }
    const double dx = 2 * cp.p1 * x * y + cp.p2 * (r2 + 2 * x * x);
    const double dy = cp.p1 * (r2 + 2 * y * y) + 2 * cp.p2 * x * y;
    x = (x0 - dx) * icdist;
    y = (y0 - dy) * icdist;
  }
  ox = x;
  oy = y;
}

// cv2.projectPoints(X, rvec, tvec, K, dist) (calibration.cpp cvProjectPoints2Internal).
__device__ __forceinline__ void pinhole_project(const CamParams& cp, double X, double Y, double Z, double& u,
                                                double& v) {
  const double* R = cp.R;
  double x = R[0] * X + R[1] * Y + R[2] * Z + cp.t[0];
  double y = R[3] * X + R[4] * Y + R[5] * Z + cp.t[1];
  double z = R[6] * X + R[7] * Y + R[8] * Z + cp.t[2];
  z = z != 0 ? 1. / z : 1;
  x *= z;
  y *= z;
  const double r2 = x * x + y * y, r4 = r2 * r2, r6 = r4 * r2;
  const double a1 = 2 * x * y, a2 = r2 + 2 * x * x, a3 = r2 + 2 * y * y;
  const double cdist = 1 + cp.k1 * r2 + cp.k2 * r4 + cp.k3 * r6;
  const double xd = x * cdist + cp.p1 * a1 + cp.p2 * a2;
  const double yd = y * cdist + cp.p1 * a3 + cp.p2 * a1;
  u = xd * cp.fx + cp.cx;
  v = yd * cp.fy + cp.cy;
}

// cv2.fisheye.undistortPoints(p, K, D) (fisheye.cpp): Newton on theta, criteria MAX_ITER + EPS (10, 1e-8);
// a point that does not converge or whose theta changes sign is written as (-1e6, -1e6).
__device__ __forceinline__ void fisheye_undistort(const CamParams& cp, double u, double v, double& ox, double& oy) {
  const double k0 = cp.k1, k1 = cp.k2, k2 = cp.p1, k3 = cp.p2;
  const double pw0 = (u - cp.cx) / cp.fx, pw1 = (v - cp.cy) / cp.fy;
  double theta_d = sqrt(pw0 * pw0 + pw1 * pw1);
  constexpr double HALF_PI = 3.1415926535897932384626433832795 / 2.;
  theta_d = fmin(fmax(-HALF_PI, theta_d), HALF_PI);
  bool converged = false;
  double theta = theta_d, scale = 0.0;
  if (fabs(theta_d) > 1e-8) {
    for (int j = 0; j < 10; ++j) {
      const double t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
      const double a = k0 * t2, b = k1 * t4, c = k2 * t6, e = k3 * t8;
      const double fix = (theta * (1 + a + b + c + e) - theta_d) / (1 + 3 * a + 5 * b + 7 * c + 9 * e);
      theta = theta - fix;
      if (fabs(fix) < 1e-8) {
        converged = true;
        break;
      }
    }
    scale = tan(theta) / theta_d;
  } else {
    converged = true;
  }
  const bool flipped = (theta_d < 0 && theta > 0) || (theta_d > 0 && theta < 0);
  if (converged && !flipped) {
    ox = pw0 * scale;
    oy = pw1 * scale;
  } else {
    ox = -1000000.0;
    oy = -1000000.0;
  }
}

// cv2.fisheye.projectPoints(X, rvec, tvec, K, D), alpha = 0 (fisheye.cpp).
__device__ __forceinline__ void fisheye_project(const CamParams& cp, double X, double Y, double Z, double& u,
                                                double& v) {
  const double* R = cp.R;
  const double y0 = R[0] * X + R[1] * Y + R[2] * Z + cp.t[0];
  const double y1 = R[3] * X + R[4] * Y + R[5] * Z + cp.t[1];
  double y2 = R[6] * X + R[7] * Y + R[8] * Z + cp.t[2];
  if (fabs(y2) < 2.2250738585072014e-308) y2 = 1;  // DBL_MIN
  const double x0 = y0 / y2, x1 = y1 / y2;
  const double r = sqrt(x0 * x0 + x1 * x1);
  const double th = atan(r);
  const double th2 = th * th, th3 = th2 * th, th4 = th2 * th2, th5 = th4 * th, th6 = th3 * th3, th7 = th6 * th,
               th8 = th4 * th4, th9 = th8 * th;
  const double theta_d = th + cp.k1 * th3 + cp.k2 * th5 + cp.p1 * th7 + cp.p2 * th9;
  const double cdist = r > 1e-8 ? theta_d * (1.0 / r) : 1;
  u = (x0 * cdist) * cp.fx + cp.cx;
  v = (x1 * cdist) * cp.fy + cp.cy;
}

// A row whose model slot is none of the three (not a row the host packer writes) gives NaN: garbage in,
// visibly invalid out, instead of a silently wrong model.
__device__ __forceinline__ void cam_undistort(const CamParams& cp, double u, double v, double& ox, double& oy) {
  switch (cam_model(cp)) {
    case CAM_OMNIDIR: omni_undistort(cp, u, v, ox, oy); break;
    case CAM_PINHOLE: pinhole_undistort(cp, u, v, ox, oy); break;
    case CAM_FISHEYE: fisheye_undistort(cp, u, v, ox, oy); break;
    default: ox = oy = __builtin_nan(""); break;
  }
}

__device__ __forceinline__ void cam_project(const CamParams& cp, double X, double Y, double Z, double& u, double& v) {
  switch (cam_model(cp)) {
    case CAM_OMNIDIR: omni_project(cp, X, Y, Z, u, v); break;
    case CAM_PINHOLE: pinhole_project(cp, X, Y, Z, u, v); break;
    case CAM_FISHEYE: fisheye_project(cp, X, Y, Z, u, v); break;
    default: u = v = __builtin_nan(""); break;
  }
}

}  // namespace mq
