// Device pieces shared by the two optim_points solvers (optim.hip: Levenberg-Marquardt + PCG;
// optim_trf.hip: scipy's trust-region-reflective + lsmr): the reprojection loss and the three camera
// models' projections with their analytic d(u, v)/dX.
#pragma once
#include "camera.hpp"

namespace mq {

__device__ __forceinline__ const CamParams& cam_at(const double* cams, int c) {
  return *reinterpret_cast<const CamParams*>(cams + 24 * c);
}

// r = rho(|e|) and dr/de (cameras.py:1581-1590: abs first, then the loss).
__device__ __forceinline__ void reproj_loss(double e, double rp, int loss, double& r, double& dr) {
  const double a = fabs(e), sg = e < 0 ? -1.0 : 1.0;
  if (loss == 1) {
    const double s = sqrt(1 + a / rp);
    r = rp * 2 * (s - 1);
    dr = sg / s;
  } else if (loss == 2 && a > rp) {
    r = rp * (2 * sqrt(a / rp) - 1);
    dr = sg * sqrt(rp / a);
  } else {
    r = a;
    dr = sg;
  }
}

// cv2.omnidir.projectPoints (same arithmetic as camera.hpp omni_project) plus
// the analytic d(u,v)/dX.
__device__ __forceinline__ void omni_project_jac(const CamParams& cp, const double* X, double& u, double& v, double* Ju,
                                                 double* Jv) {
  const double* R = cp.R;
  const double x0 = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + cp.t[0];
  const double x1 = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + cp.t[1];
  const double x2 = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + cp.t[2];
  const double nrm = sqrt(x0 * x0 + x1 * x1 + x2 * x2);
  const double xs = x0 / nrm, ys = x1 / nrm, zs = x2 / nrm;
  const double xu = xs / (zs + cp.xi), yu = ys / (zs + cp.xi);
  const double r2 = xu * xu + yu * yu;
  const double r4 = r2 * r2;
  const double rad = 1 + cp.k1 * r2 + cp.k2 * r4;
  const double xd = xu * rad + 2 * cp.p1 * xu * yu + cp.p2 * (r2 + 2 * xu * xu);
  const double yd = yu * rad + cp.p1 * (r2 + 2 * yu * yu) + 2 * cp.p2 * xu * yu;
  u = cp.fx * xd + cp.skew * yd + cp.cx;
  v = cp.fy * yd + cp.cy;
  // xu = x0 / w, yu = x1 / w with w = x2 + xi |Xc|
  const double w = x2 + cp.xi * nrm;
  const double dw[3] = {cp.xi * x0 / nrm, cp.xi * x1 / nrm, 1 + cp.xi * x2 / nrm};
  const double drad = 2 * (cp.k1 + 2 * cp.k2 * r2);
  const double a11 = rad + xu * drad * xu + 2 * cp.p1 * yu + 6 * cp.p2 * xu;
  const double a12 = xu * drad * yu + 2 * cp.p1 * xu + 2 * cp.p2 * yu;
  const double a21 = yu * drad * xu + 2 * cp.p1 * xu + 2 * cp.p2 * yu;
  const double a22 = rad + yu * drad * yu + 6 * cp.p1 * yu + 2 * cp.p2 * xu;
  double gxu[3], gyu[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    gxu[i] = ((i == 0 ? 1.0 : 0.0) - xu * dw[i]) / w;
    gyu[i] = ((i == 1 ? 1.0 : 0.0) - yu * dw[i]) / w;
  }
#pragma unroll
  for (int jx = 0; jx < 3; ++jx) {
    const double Gx = gxu[0] * R[jx] + gxu[1] * R[3 + jx] + gxu[2] * R[6 + jx];
    const double Gy = gyu[0] * R[jx] + gyu[1] * R[3 + jx] + gyu[2] * R[6 + jx];
    const double dxd = a11 * Gx + a12 * Gy, dyd = a21 * Gx + a22 * Gy;
    Ju[jx] = cp.fx * dxd + cp.skew * dyd;
    Jv[jx] = cp.fy * dyd;
  }
}

// cv2.projectPoints (camera.hpp pinhole_project: u, v bit for bit) plus the analytic d(u,v)/dX.
__device__ __forceinline__ void pinhole_project_jac(const CamParams& cp, const double* X, double& u, double& v,
                                                    double* Ju, double* Jv) {
  pinhole_project(cp, X[0], X[1], X[2], u, v);
  const double* R = cp.R;
  const double z = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + cp.t[2];
  const double iz = z != 0 ? 1. / z : 1;
  const double x = (R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + cp.t[0]) * iz;
  const double y = (R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + cp.t[1]) * iz;
  const double r2 = x * x + y * y, r4 = r2 * r2;
  const double cdist = 1 + cp.k1 * r2 + cp.k2 * r4 + cp.k3 * r4 * r2;
  const double dc = 2 * (cp.k1 + 2 * cp.k2 * r2 + 3 * cp.k3 * r4);  // d cdist / dx = dc x
  const double a11 = cdist + x * dc * x + 2 * cp.p1 * y + 6 * cp.p2 * x;
  const double a12 = x * dc * y + 2 * cp.p1 * x + 2 * cp.p2 * y;
  const double a21 = y * dc * x + 2 * cp.p1 * x + 2 * cp.p2 * y;
  const double a22 = cdist + y * dc * y + 6 * cp.p1 * y + 2 * cp.p2 * x;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    // x = Xc0 / Xc2, y = Xc1 / Xc2
    const double gx = (R[j] - x * R[6 + j]) * iz, gy = (R[3 + j] - y * R[6 + j]) * iz;
    Ju[j] = cp.fx * (a11 * gx + a12 * gy);
    Jv[j] = cp.fy * (a21 * gx + a22 * gy);
  }
}

// cv2.fisheye.projectPoints (camera.hpp fisheye_project) plus the analytic d(u,v)/dX:
// (xd, yd) = g(r) (x, y), g = theta_d(atan r) / r, so d xd / dx = g + x^2 g' / r and so on.
__device__ __forceinline__ void fisheye_project_jac(const CamParams& cp, const double* X, double& u, double& v,
                                                    double* Ju, double* Jv) {
  fisheye_project(cp, X[0], X[1], X[2], u, v);
  const double* R = cp.R;
  double z = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + cp.t[2];
  if (fabs(z) < 2.2250738585072014e-308) z = 1;
  const double x = (R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + cp.t[0]) / z;
  const double y = (R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + cp.t[1]) / z;
  const double r = sqrt(x * x + y * y);
  double g = 1, gr = 0;  // g and g' / r
  if (r > 1e-8) {
    const double th = atan(r), t2 = th * th, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
    const double td = th * (1 + cp.k1 * t2 + cp.k2 * t4 + cp.p1 * t6 + cp.p2 * t8);
    const double dtd = 1 + 3 * cp.k1 * t2 + 5 * cp.k2 * t4 + 7 * cp.p1 * t6 + 9 * cp.p2 * t8;
    g = td / r;
    gr = (dtd / (1 + r * r) - g) / (r * r);
  }
  const double a11 = g + x * x * gr, a12 = x * y * gr, a22 = g + y * y * gr;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double gx = (R[j] - x * R[6 + j]) / z, gy = (R[3 + j] - y * R[6 + j]) / z;
    Ju[j] = cp.fx * (a11 * gx + a12 * gy);
    Jv[j] = cp.fy * (a12 * gx + a22 * gy);
  }
}

__device__ __forceinline__ void project_jac(const CamParams& cp, const double* X, double& u, double& v, double* Ju,
                                            double* Jv) {
  switch (cam_model(cp)) {
    case CAM_OMNIDIR: omni_project_jac(cp, X, u, v, Ju, Jv); break;
    case CAM_PINHOLE: pinhole_project_jac(cp, X, u, v, Ju, Jv); break;
    case CAM_FISHEYE: fisheye_project_jac(cp, X, u, v, Ju, Jv); break;
    default:  // not a row the host packer writes (camera.hpp)
      u = v = __builtin_nan("");
      for (int k = 0; k < 3; ++k) Ju[k] = Jv[k] = 0.0;
      break;
  }
}

}  // namespace mq
