// float64 multi-view geometry kernels (anipose / mvpose lift).
// Compiled with -ffp-contract=off so every expression rounds like the numpy oracle.
#include "common.hpp"
#include "camera.hpp"
#include "geometry.hpp"

namespace mq {

__device__ __forceinline__ const CamParams& cam_at(const double* cams, int c) {
  return *reinterpret_cast<const CamParams*>(cams + 24 * c);
}

// One-sided (Hestenes) Jacobi SVD of an m x N matrix held as N columns of length M
// (unused rows zero).  Returns the right singular vectors in V and the column
// norms (singular values) in sig.
template <int M, int N>
__device__ __forceinline__ void jacobi_svd(double (&a)[N][M], double (&V)[N][N], double (&sig)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < N - 1; ++p) {
#pragma unroll
      for (int q = p + 1; q < N; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
          alpha += a[p][i] * a[p][i];
          beta += a[q][i] * a[q][i];
          gamma += a[p][i] * a[q][i];
        }
        if (fabs(gamma) > 1e-15 * sqrt(alpha * beta) && gamma != 0.0) {
          rotated = true;
          const double zeta = (beta - alpha) / (2.0 * gamma);
          const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double c = 1.0 / sqrt(1.0 + t * t);
          const double s = c * t;
#pragma unroll
          for (int i = 0; i < M; ++i) {
            const double ap = a[p][i], aq = a[q][i];
            a[p][i] = c * ap - s * aq;
            a[q][i] = s * ap + c * aq;
          }
#pragma unroll
          for (int i = 0; i < N; ++i) {
            const double vp = V[p][i], vq = V[q][i];
            V[p][i] = c * vp - s * vq;
            V[q][i] = s * vp + c * vq;
          }
        }
      }
    }
    if (!rotated) break;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) s += a[j][i] * a[j][i];
    sig[j] = sqrt(s);
  }
}

// Homogeneous DLT (cameras.py:20-32) over the cameras flagged in `use`.
template <int MAXC>
__device__ __forceinline__ void dlt_point(const double* cams, int C, const double* ux, const double* uy,
                                          unsigned use, double out[3]) {
  double a[4][2 * MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const bool on = (c < C) && ((use >> c) & 1u);
    if (on) {
      const CamParams& cp = cam_at(cams, c);
      const double P0[4] = {cp.R[0], cp.R[1], cp.R[2], cp.t[0]};
      const double P1[4] = {cp.R[3], cp.R[4], cp.R[5], cp.t[1]};
      const double P2[4] = {cp.R[6], cp.R[7], cp.R[8], cp.t[2]};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k][2 * c] = ux[c] * P2[k] - P0[k];
        a[k][2 * c + 1] = uy[c] * P2[k] - P1[k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k][2 * c] = 0.0;
        a[k][2 * c + 1] = 0.0;
      }
    }
  }
  double V[4][4], sig[4];
  jacobi_svd<2 * MAXC, 4>(a, V, sig);
  int jmin = 0;
#pragma unroll
  for (int j = 1; j < 4; ++j)
    if (sig[j] < sig[jmin]) jmin = j;
  double v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = V[jmin][k];
  out[0] = v[0] / v[3];
  out[1] = v[1] / v[3];
  out[2] = v[2] / v[3];
}


// ------------------------------------------------------------------ step-2 geometry affinity
// geometry_affinity2 (step2_crossviewmatching.py:373-432) batched over B frames of up to M detections
// (cam_of_det < 0 marks padding).  Three launches: rays, pairwise mean ray distance, per-frame z-score
// + logistic.  Operation order follows the reference (numpy), compiled without FMA contraction.

// 3x3 inverse (adjugate / determinant) of the camera rotation: deproject uses np.linalg.inv(R).
__device__ __forceinline__ void inv3(const double* R, double* Ri) {
  const double c00 = R[4] * R[8] - R[5] * R[7], c01 = R[5] * R[6] - R[3] * R[8], c02 = R[3] * R[7] - R[4] * R[6];
  const double det = R[0] * c00 + R[1] * c01 + R[2] * c02;
  const double id = 1.0 / det;
  Ri[0] = c00 * id;
  Ri[1] = (R[2] * R[7] - R[1] * R[8]) * id;
  Ri[2] = (R[1] * R[5] - R[2] * R[4]) * id;
  Ri[3] = c01 * id;
  Ri[4] = (R[0] * R[8] - R[2] * R[6]) * id;
  Ri[5] = (R[2] * R[3] - R[0] * R[5]) * id;
  Ri[6] = c02 * id;
  Ri[7] = (R[1] * R[6] - R[0] * R[7]) * id;
  Ri[8] = (R[0] * R[4] - R[1] * R[3]) * id;
}

// deproject (step2:327-355) at depth 0 and 1000: rays[b][i][k] = (near xyz, far xyz)
__global__ void affinity_rays_kernel(const double* __restrict__ cams, int C, const double* __restrict__ pts,
                                     const int32_t* __restrict__ cam_of_det, int BM, int J,
                                     double* __restrict__ rays) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= BM * J) return;
  const int det = idx / J;
  const int c = cam_of_det[det];
  double* r = rays + (size_t)idx * 6;
  if (c < 0 || c >= C) {  // padding (an out-of-range camera index is treated as padding too)
    for (int e = 0; e < 6; ++e) r[e] = 0.0;
    return;
  }
  const CamParams& cp = cam_at(cams, c);
  double Ri[9];
  inv3(cp.R, Ri);
  const double x = pts[(size_t)idx * 3], y = pts[(size_t)idx * 3 + 1];
  const double dn[3] = {0.0 * x - cp.t[0], 0.0 * y - cp.t[1], 0.0 * 1.0 - cp.t[2]};
  const double df[3] = {x * 1000.0 - cp.t[0], y * 1000.0 - cp.t[1], 1.0 * 1000.0 - cp.t[2]};
#pragma unroll
  for (int row = 0; row < 3; ++row) {
    r[row] = (Ri[3 * row] * dn[0] + Ri[3 * row + 1] * dn[1]) + Ri[3 * row + 2] * dn[2];
    r[3 + row] = (Ri[3 * row] * df[0] + Ri[3 * row + 1] * df[1]) + Ri[3 * row + 2] * df[2];
  }
}

// calc_dist_btw_lines (step2:359-369)
__device__ __forceinline__ double line_dist(const double* v1, const double* v2) {
  double d1[3], d2[3];
  const double a0 = v1[3] - v1[0], a1 = v1[4] - v1[1], a2 = v1[5] - v1[2];
  const double b0 = v2[3] - v2[0], b1 = v2[4] - v2[1], b2 = v2[5] - v2[2];
  const double na = sqrt((a0 * a0 + a1 * a1) + a2 * a2), nb = sqrt((b0 * b0 + b1 * b1) + b2 * b2);
  d1[0] = a0 / na; d1[1] = a1 / na; d1[2] = a2 / na;
  d2[0] = b0 / nb; d2[1] = b1 / nb; d2[2] = b2 / nb;
  const double c0 = d1[1] * d2[2] - d1[2] * d2[1];
  const double c1 = d1[2] * d2[0] - d1[0] * d2[2];
  const double c2 = d1[0] * d2[1] - d1[1] * d2[0];
  const double num = ((v2[0] - v1[0]) * c0 + (v2[1] - v1[1]) * c1) + (v2[2] - v1[2]) * c2;
  return fabs(num) / sqrt((c0 * c0 + c1 * c1) + c2 * c2);
}

// pairwise mean ray distance; dist = -1 marks a padding pair (excluded from the statistics)
__global__ void affinity_dist_kernel(const double* __restrict__ rays, const double* __restrict__ pts,
                                     const int32_t* __restrict__ cam_of_det, int C, int B, int M, int J,
                                     double thr_kp, double* __restrict__ dist) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * M * M) return;
  const int b = (int)(idx / ((int64_t)M * M));
  const int i = (int)((idx / M) % M), j = (int)(idx % M);
  const int ci = cam_of_det[b * M + i], cj = cam_of_det[b * M + j];
  double d;
  if (ci < 0 || cj < 0 || ci >= C || cj >= C) {
    d = -1.0;
  } else if (i == j) {
    d = 0.0;
  } else if (ci == cj) {
    d = 300.0;
  } else {
    const int lo = i < j ? i : j, hi = i < j ? j : i;  // the reference fills (i, j) and (j, i) from i < j
    const double* ri = rays + ((size_t)(b * M + lo) * J) * 6;
    const double* rj = rays + ((size_t)(b * M + hi) * J) * 6;
    const double* si = pts + ((size_t)(b * M + lo) * J) * 3;
    const double* sj = pts + ((size_t)(b * M + hi) * J) * 3;
    double sum = 0.0;
    int cnt = 0;
    for (int k = 0; k < J; ++k) {
      if (si[k * 3 + 2] > thr_kp && sj[k * 3 + 2] > thr_kp) {
        sum = sum + line_dist(ri + k * 6, rj + k * 6);
        ++cnt;
      }
    }
    d = cnt >= 3 ? sum / (double)cnt : 300.0;
  }
  dist[idx] = d;
}

// per frame: mean / std (two-pass, ddof 0) over the entries < 2*Dth2, logistic(-5 z), 0 where > Dth2
__global__ __launch_bounds__(256) void affinity_norm_kernel(const double* __restrict__ dist, int M,
                                                            double* __restrict__ out) {
  const int b = blockIdx.x;
  const double* d = dist + (size_t)b * M * M;
  double* o = out + (size_t)b * M * M;
  __shared__ double red[256];
  __shared__ int redc[256];
  double s = 0.0;
  int c = 0;
  for (int e = threadIdx.x; e < M * M; e += blockDim.x) {
    const double v = d[e];
    if (v >= 0.0 && v < 300.0) {
      s += v;
      ++c;
    }
  }
  red[threadIdx.x] = s;
  redc[threadIdx.x] = c;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      red[threadIdx.x] += red[threadIdx.x + w];
      redc[threadIdx.x] += redc[threadIdx.x + w];
    }
    __syncthreads();
  }
  const double mean = red[0] / (double)redc[0];
  const int cnt = redc[0];
  __syncthreads();
  double q = 0.0;
  for (int e = threadIdx.x; e < M * M; e += blockDim.x) {
    const double v = d[e];
    if (v >= 0.0 && v < 300.0) q += (v - mean) * (v - mean);
  }
  red[threadIdx.x] = q;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double sd = sqrt(red[0] / (double)cnt);
  for (int e = threadIdx.x; e < M * M; e += blockDim.x) {
    const double v = d[e];
    double a;
    if (v < 0.0 || v > 150.0) {
      a = 0.0;
    } else {
      const double z = -(v - mean) / sd;
      a = 1.0 / (1.0 + exp(-5.0 * z));
    }
    o[e] = a;
  }
}

// ------------------------------------------------------------------ kernels
__global__ void undistort_kernel(const double* __restrict__ cams, int C, const double* __restrict__ pts,
                                 double* __restrict__ out, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * N) return;
  const int c = i / N;
  double ox, oy;
  cam_undistort(cam_at(cams, c), pts[2 * i], pts[2 * i + 1], ox, oy);
  out[2 * i] = ox;
  out[2 * i + 1] = oy;
}

__global__ void project_kernel(const double* __restrict__ cams, int C, const double* __restrict__ p3d,
                               double* __restrict__ out, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * N) return;
  const int c = i / N, n = i % N;
  double u, v;
  cam_project(cam_at(cams, c), p3d[3 * n], p3d[3 * n + 1], p3d[3 * n + 2], u, v);
  out[2 * i] = u;
  out[2 * i + 1] = v;
}

// CameraGroup.triangulate (cameras.py:593-637): optional undistort, >= 2 views.
// 64-thread launches: the bound lifts the default 1024-thread VGPR cap, under which the 2C x 4
// f64 DLT matrix of the Jacobi SVD spilled to scratch (115 us for one frame's 68 points).
template <int MAXC>
__global__ __launch_bounds__(64) void triangulate_kernel(const double* __restrict__ cams, int C, const double* __restrict__ pts, int N,
                                   int undistort, double* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double ux[MAXC], uy[MAXC];
  unsigned use = 0;
  int cnt = 0;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    ux[c] = 0;
    uy[c] = 0;
    if (c < C) {
      const double u = pts[2 * ((size_t)c * N + n)], v = pts[2 * ((size_t)c * N + n) + 1];
      double x = u, y = v;
      if (undistort) cam_undistort(cam_at(cams, c), u, v, x, y);
      ux[c] = x;
      uy[c] = y;
      if (!(x != x)) {
        use |= 1u << c;
        ++cnt;
      }
    }
  }
  double r[3] = {NAN, NAN, NAN};
  if (cnt >= 2) dlt_point<MAXC>(cams, C, ux, uy, use, r);
  out[3 * n] = r[0];
  out[3 * n + 1] = r[1];
  out[3 * n + 2] = r[2];
}

// CameraGroup.reprojection_error (cameras.py:746-783).
__global__ void reproj_kernel(const double* __restrict__ cams, int C, const double* __restrict__ p3d,
                              const double* __restrict__ p2d, int N, int mean, double* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const double X = p3d[3 * n], Y = p3d[3 * n + 1], Z = p3d[3 * n + 2];
  double sum = 0.0, cnt = 0.0;
  for (int c = 0; c < C; ++c) {
    double u, v;
    cam_project(cam_at(cams, c), X, Y, Z, u, v);
    const size_t o = 2 * ((size_t)c * N + n);
    const double ex = p2d[o] - u, ey = p2d[o + 1] - v;
    if (!mean) {
      out[o] = ex;
      out[o + 1] = ey;
    } else {
      const double nr = sqrt(ex * ex + ey * ey);
      if (!(nr != nr)) {
        sum = sum + nr;
        cnt = cnt + 1.0;
      }
    }
  }
  if (mean) out[n] = (cnt < 1.5) ? NAN : sum / cnt;
}

// triangulate_ransac -> triangulate_possible (cameras.py:639-743), n_possible = 1.
// One wave per point; lanes walk the itertools.product order (bit m-1-i of the
// subset index = "camera position i dropped") 64 subsets at a time and stop at
// the first chunk holding an error < threshold, which reproduces the serial
// early exit exactly; otherwise the first strict minimum below 200 wins.
template <int MAXC>
__global__ __launch_bounds__(64) void ransac_kernel(const double* __restrict__ cams, int C,
                                                    const double* __restrict__ pts, int N, int min_cams,
                                                    double threshold, double* __restrict__ out_p3d,
                                                    uint8_t* __restrict__ out_picked, double* __restrict__ out_p2d,
                                                    double* __restrict__ out_err) {
  const int n = blockIdx.x;
  const int lane = threadIdx.x;
  if (n >= N) return;
  double raw_u[MAXC], raw_v[MAXC], ux[MAXC], uy[MAXC];
  int pos2cam[MAXC];
  int m = 0;
  unsigned und_ok = 0;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    raw_u[c] = raw_v[c] = ux[c] = uy[c] = 0;
    if (c < C) {
      const size_t o = 2 * ((size_t)c * N + n);
      raw_u[c] = pts[o];
      raw_v[c] = pts[o + 1];
      if (!(raw_u[c] != raw_u[c])) {
        cam_undistort(cam_at(cams, c), raw_u[c], raw_v[c], ux[c], uy[c]);
        if (!(ux[c] != ux[c])) und_ok |= 1u << c;
        pos2cam[m] = c;
        ++m;
      }
    }
  }
  const int nsub = 1 << m;
  int chosen = -1;
  double best_err = 200.0;
  int best_s = 0x7fffffff;
  if (m >= 2) {
    for (int base = 0; base < nsub; base += 64) {
      const int s = base + lane;
      double err = NAN;
      if (s < nsub) {
        unsigned use = 0;
        int k = 0;
        for (int i = 0; i < m; ++i)
          if (!((s >> (m - 1 - i)) & 1)) {
            use |= 1u << pos2cam[i];
            ++k;
          }
        if (!(k < min_cams && k != m) && k >= 2) {
          double p[3] = {NAN, NAN, NAN};
          if (__popc(use & und_ok) >= 2) dlt_point<MAXC>(cams, C, ux, uy, use & und_ok, p);
          double sum = 0.0, cnt = 0.0;
          for (int c = 0; c < C; ++c) {
            if (!((use >> c) & 1u)) continue;
            double u, v;
            cam_project(cam_at(cams, c), p[0], p[1], p[2], u, v);
            const double ex = raw_u[c] - u, ey = raw_v[c] - v;
            const double nr = sqrt(ex * ex + ey * ey);
            if (!(nr != nr)) {
              sum = sum + nr;
              cnt = cnt + 1.0;
            }
          }
          err = (cnt < 1.5) ? NAN : sum / cnt;
        }
      }
      // first subset (smallest s) in this chunk with err < threshold
      const bool hit = err < threshold;
      const unsigned long long hits = __ballot(hit);
      if (hits) {
        chosen = base + __ffsll((long long)hits) - 1;
        break;
      }
      // running strict minimum, ties keep the earlier subset
      double e = (err < 200.0) ? err : INFINITY;
      int es = (err < 200.0) ? s : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double e2 = __shfl_xor(e, o, 64);
        const int s2 = __shfl_xor(es, o, 64);
        if (e2 < e || (e2 == e && s2 < es)) {
          e = e2;
          es = s2;
        }
      }
      if (es != 0x7fffffff && (e < best_err || (e == best_err && es < best_s))) {
        best_err = e;
        best_s = es;
      }
    }
    if (chosen < 0 && best_s != 0x7fffffff) chosen = best_s;
  }
  if (lane != 0) return;
  double p[3] = {NAN, NAN, NAN};
  double err = 0.0;
  unsigned use = 0;
  if (chosen >= 0) {
    for (int i = 0; i < m; ++i)
      if (!((chosen >> (m - 1 - i)) & 1)) use |= 1u << pos2cam[i];
    if (__popc(use & und_ok) >= 2) dlt_point<MAXC>(cams, C, ux, uy, use & und_ok, p);
    double sum = 0.0, cnt = 0.0;
    for (int c = 0; c < C; ++c) {
      if (!((use >> c) & 1u)) continue;
      double u, v;
      cam_project(cam_at(cams, c), p[0], p[1], p[2], u, v);
      const double ex = raw_u[c] - u, ey = raw_v[c] - v;
      const double nr = sqrt(ex * ex + ey * ey);
      if (!(nr != nr)) {
        sum = sum + nr;
        cnt = cnt + 1.0;
      }
    }
    err = (cnt < 1.5) ? NAN : sum / cnt;
  }
  out_p3d[3 * n] = p[0];
  out_p3d[3 * n + 1] = p[1];
  out_p3d[3 * n + 2] = p[2];
  out_err[n] = err;
  for (int c = 0; c < C; ++c) {
    const bool on = (use >> c) & 1u;
    out_picked[(size_t)c * N + n] = on ? 1 : 0;
    out_p2d[2 * ((size_t)c * N + n)] = on ? raw_u[c] : NAN;
    out_p2d[2 * ((size_t)c * N + n) + 1] = on ? raw_v[c] : NAN;
  }
}

// mvpose inhomogeneous DLT (multicam_toolbox.py:433-486): X = pinv(A[:, :3]) A[:, 3], P = -X.
template <int MAXC>
__global__ void pinv_dlt_kernel(const double* __restrict__ cams, int C, const double* __restrict__ und,
                                const uint8_t* __restrict__ use_mask, int N, double* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double a[3][2 * MAXC], b[2 * MAXC];
  int cnt = 0;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    bool on = false;
    double x = 0, y = 0;
    if (c < C) {
      on = use_mask[(size_t)n * C + c] != 0;
      x = und[2 * ((size_t)c * N + n)];
      y = und[2 * ((size_t)c * N + n) + 1];
    }
    if (on) {
      ++cnt;
      const CamParams& cp = cam_at(cams, c);
      const double P0[4] = {cp.R[0], cp.R[1], cp.R[2], cp.t[0]};
      const double P1[4] = {cp.R[3], cp.R[4], cp.R[5], cp.t[1]};
      const double P2[4] = {cp.R[6], cp.R[7], cp.R[8], cp.t[2]};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        a[k][2 * c] = x * P2[k] - P0[k];
        a[k][2 * c + 1] = y * P2[k] - P1[k];
      }
      b[2 * c] = x * P2[3] - P0[3];
      b[2 * c + 1] = y * P2[3] - P1[3];
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) a[k][2 * c] = a[k][2 * c + 1] = 0.0;
      b[2 * c] = b[2 * c + 1] = 0.0;
    }
  }
  if (cnt < 2) {
    out[3 * n] = out[3 * n + 1] = out[3 * n + 2] = NAN;
    return;
  }
  double V[3][3], sig[3];
  jacobi_svd<2 * MAXC, 3>(a, V, sig);
  const double smax = fmax(fmax(sig[0], sig[1]), sig[2]);
  double X[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if (sig[j] > 1e-15 * smax) {
      double ub = 0;
#pragma unroll
      for (int i = 0; i < 2 * MAXC; ++i) ub += a[j][i] * b[i];
      const double w = ub / (sig[j] * sig[j]);
#pragma unroll
      for (int k = 0; k < 3; ++k) X[k] += V[j][k] * w;
    }
  }
  out[3 * n] = -X[0];
  out[3 * n + 1] = -X[1];
  out[3 * n + 2] = -X[2];
}

// ------------------------------------------------------------------ Viterbi (filter_pose.py:48-186)
// scipy log_ndtr (Faddeeva form): x < -1: log(erfcx(-t)/2) - t^2, else log1p(-erfc(t)/2), t = x/sqrt(2),
// erfc(t) = exp(-t^2) erfcx(t) (t >= 0) or 2 - exp(-t^2) erfcx(-t).
__device__ __forceinline__ double log_ndtr_d(double x) {
  const double t = x * 0.70710678118654752440;
  if (x < -1.0) return log(erfcx(-t) / 2) - t * t;
  const double e = (t < 0) ? (2. - exp(-t * t) * erfcx(-t)) : exp(-t * t) * erfcx(t);
  return log1p(-e / 2);
}

// log(Phi((d+2)/s) - Phi((d-2)/s)) evaluated as scipy's logsumexp(b=[1,-1]) does, clamped at -100.
__device__ __forceinline__ double trans_logprob(double d, double thres) {
  const double hi = log_ndtr_d((d + 2) / thres);
  const double lo = log_ndtr_d((d - 2) / thres);
  double r;
  if (hi > lo) {
    r = log1p(-exp(lo - hi)) + hi;
  } else if (hi == lo) {
    r = -INFINITY;
  } else {
    r = NAN;
  }
  if (r < -100) r = -100;
  return r;
}

// The Viterbi filter in two launches (filter_pose.py:48-120, chain = (animal, camera, joint)):
//  1. viterbi_trans_kernel, one thread per (chain, frame i, particle q of frame i, particle p of
//     frame i-1): the transition log-probability log(Phi((d+2)/s) - Phi((d-2)/s)) -- the fp64
//     log_ndtr work, which is all of the arithmetic -- for every chain and frame in parallel; the
//     (q, p) = (0, 0) thread of each frame also records the frame's particles (x, y, score, log score)
//     and their count;
//  2. viterbi_dp_kernel, one thread per chain: the max-product recursion over frames on those
//     records (a few adds and compares per frame, the next frame's inputs loaded while the current
//     one is combined), back-pointers and the backtracked path in LDS, then the output rows.
// Same operations in the same order per value as the single-pass form, so outputs are identical.
struct VitChain {
  const double* kp;
  int F, C, J, n_back;
  double score_thr;
  __device__ const double* at(int a, int c, int j, int f) const {
    return kp + ((((size_t)a * F + f) * C + c) * J + j) * 3;
  }
  __device__ bool valid(const double* p) const {
    const bool masked = p[2] < score_thr;  // points_full[scores < thr] = NaN
    return !masked && !(p[0] != p[0]);
  }
  // particles of frame i: (x, y, score * 2^-jj) for valid frames i-jj, jj < n_back
  __device__ int particles(int a, int c, int j, int i, double* px, double* py, double* ps) const {
    int s = 0;
    double w = 1.0;
    for (int jj = 0; jj < n_back && jj < 8; ++jj) {
      if (i - jj < 0) break;
      const double* p = at(a, c, j, i - jj);
      if (valid(p)) {
        px[s] = p[0];
        py[s] = p[1];
        ps[s] = p[2] * w;
        ++s;
      }
      w = w * 0.5;
    }
    if (s == 0) {
      px[0] = -1;
      py[0] = -1;
      ps[0] = 0.001;
      s = 1;
    }
    return s;
  }
};

struct VitBufs {
  double* trans;  // [chain][F][NB][NB]: P(q of frame i | p of frame i-1)
  double* part;   // [chain][F][NB][4]: x, y, score, log(score)
  int8_t* cnt;    // [chain][F]: particle count
  int8_t* bk;     // [chain][F][NB]: back-pointers when they do not fit in LDS
};

__global__ void viterbi_trans_kernel(VitChain V, int chains, double thres_dist, VitBufs W) {
  const int NB = V.n_back;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t per_chain = (size_t)V.F * NB * NB;
  if (tid >= (size_t)chains * per_chain) return;
  const int ch = (int)(tid / per_chain);
  const int rem = (int)(tid - (size_t)ch * per_chain);
  const int i = rem / (NB * NB), q = (rem / NB) % NB, p = rem % NB;
  const int j = ch % V.J, c = (ch / V.J) % V.C, a = ch / (V.J * V.C);
  double bx[8], by[8], bs[8];
  const int vb = V.particles(a, c, j, i, bx, by, bs);
  if (q == 0 && p == 0) {
    double* rec = W.part + ((size_t)ch * V.F + i) * NB * 4;
    for (int k = 0; k < vb; ++k) {
      rec[4 * k] = bx[k];
      rec[4 * k + 1] = by[k];
      rec[4 * k + 2] = bs[k];
      rec[4 * k + 3] = log(bs[k]);
    }
    W.cnt[(size_t)ch * V.F + i] = (int8_t)vb;
  }
  if (i == 0) return;
  double ax[8], ay[8], as[8];
  const int va = V.particles(a, c, j, i - 1, ax, ay, as);
  if (q >= vb || p >= va) return;
  double P;
  if (bx[q] == -1 || ax[p] == -1) {
    P = log(0.001);
  } else {
    const double dx = ax[p] - bx[q], dy = ay[p] - by[q];
    P = trans_logprob(sqrt(dx * dx + dy * dy), thres_dist);
  }
  W.trans[tid] = P;
}

constexpr int VIT_DP_THREADS = 64;

// Back-pointers (then the backtracked path in slot 0 of each frame): blockDim.x * F * NB bytes of LDS
// when that fits (the block size is chosen by the launcher), else the global fallback in W.bk.
template <int NB>
__global__ void __launch_bounds__(VIT_DP_THREADS) viterbi_dp_kernel(VitChain V, int chains, VitBufs W,
                                                                    double* __restrict__ out, int bk_in_lds) {
  extern __shared__ int8_t lds_bk[];
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= chains) return;
  const int F = V.F;
  const int j = ch % V.J, c = (ch / V.J) % V.C, a = ch / (V.J * V.C);
  int8_t* bk = bk_in_lds ? lds_bk + (size_t)threadIdx.x * F * NB : W.bk + (size_t)ch * F * NB;
  const double* tr = W.trans + (size_t)ch * F * NB * NB;
  const double* part = W.part + (size_t)ch * F * NB * 4;
  const int8_t* cnt = W.cnt + (size_t)ch * F;
  double Tp[NB], Tc[NB];
  int va = cnt[0];
#pragma unroll
  for (int p = 0; p < NB; ++p) Tp[p] = (p < va) ? part[4 * p + 3] : -INFINITY;
  // inputs of frame i: count, log scores, transitions; frame i+1's are loaded before frame i is combined
  auto load = [&](int i, int& n, double (&lg)[NB], double (&t)[NB * NB]) {
    n = cnt[i];
#pragma unroll
    for (int k = 0; k < NB; ++k) lg[k] = part[((size_t)i * NB + k) * 4 + 3];
#pragma unroll
    for (int k = 0; k < NB * NB; ++k) t[k] = tr[(size_t)i * NB * NB + k];
  };
  int vb_n = 1;
  double lg_n[NB], t_n[NB * NB];
  if (F > 1) load(1, vb_n, lg_n, t_n);
  for (int i = 1; i < F; ++i) {
    const int vb = vb_n;
    double lg[NB], t[NB * NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) lg[k] = lg_n[k];
#pragma unroll
    for (int k = 0; k < NB * NB; ++k) t[k] = t_n[k];
    if (i + 1 < F) load(i + 1, vb_n, lg_n, t_n);
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      double best = -INFINITY;
      int arg = 0;
#pragma unroll
      for (int p = 0; p < NB; ++p) {
        if (p >= va) continue;
        const double v = Tp[p] + t[q * NB + p];
        // np.max / np.argmax semantics: first maximum, a NaN wins and sticks
        if (p == 0) {
          best = v;
          arg = 0;
        } else if (!(best != best) && ((v != v) || v > best)) {
          best = v;
          arg = p;
        }
      }
      Tc[q] = (q < vb) ? best + lg[q] : -INFINITY;
      bk[i * NB + q] = (int8_t)arg;
    }
#pragma unroll
    for (int q = 0; q < NB; ++q) Tp[q] = Tc[q];
    va = vb;
  }
  // backtrack from the first argmax of the last frame; the path goes into slot 0 of each frame
  int cur = 0;
#pragma unroll
  for (int p = 1; p < NB; ++p)
    if (p < va && Tp[p] > Tp[cur]) cur = p;
  for (int i = F - 1; i >= 0; --i) {
    const int nxt = i > 0 ? bk[i * NB + cur] : 0;
    bk[i * NB] = (int8_t)cur;
    cur = nxt;
  }
  for (int i = 0; i < F; ++i) {  // output rows (independent loads)
    const double* r = part + ((size_t)i * NB + bk[i * NB]) * 4;
    double* o = out + ((((size_t)a * F + i) * V.C + c) * V.J + j) * 3;
    o[0] = r[0];
    o[1] = r[1];
    o[2] = r[2];
  }
}

// ------------------------------------------------------------------ launchers
int omnidir_undistort(const double* cams, int C, const double* pts, double* out, int N, hipStream_t s) {
  const int tot = C * N;
  if (tot <= 0) return 0;
  hipLaunchKernelGGL(undistort_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, cams, C, pts, out, N);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int omnidir_project(const double* cams, int C, const double* p3d, double* out, int N, hipStream_t s) {
  const int tot = C * N;
  if (tot <= 0) return 0;
  hipLaunchKernelGGL(project_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, cams, C, p3d, out, N);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int triangulate_dlt(const double* cams, int C, const double* pts, int N, int undistort, double* out, hipStream_t s) {
  if (N <= 0) return 0;
  if (C <= 8)
    hipLaunchKernelGGL(triangulate_kernel<8>, dim3((N + 63) / 64), dim3(64), 0, s, cams, C, pts, N, undistort, out);
  else if (C <= 16)
    hipLaunchKernelGGL(triangulate_kernel<16>, dim3((N + 63) / 64), dim3(64), 0, s, cams, C, pts, N, undistort, out);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int reprojection_error(const double* cams, int C, const double* p3d, const double* p2d, int N, int mean, double* out,
                       hipStream_t s) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(reproj_kernel, dim3((N + 127) / 128), dim3(128), 0, s, cams, C, p3d, p2d, N, mean, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int triangulate_ransac(const double* cams, int C, const double* pts, int N, int min_cams, double threshold,
                       double* p3d, uint8_t* picked, double* p2d, double* err, hipStream_t s) {
  if (N <= 0) return 0;
  if (C <= 8)
    hipLaunchKernelGGL(ransac_kernel<8>, dim3(N), dim3(64), 0, s, cams, C, pts, N, min_cams, threshold, p3d, picked,
                       p2d, err);
  else if (C <= 16)
    hipLaunchKernelGGL(ransac_kernel<16>, dim3(N), dim3(64), 0, s, cams, C, pts, N, min_cams, threshold, p3d, picked,
                       p2d, err);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int triangulate_pinv(const double* cams, int C, const double* und, const uint8_t* use, int N, double* out,
                     hipStream_t s) {
  if (N <= 0) return 0;
  if (C <= 8)
    hipLaunchKernelGGL(pinv_dlt_kernel<8>, dim3((N + 63) / 64), dim3(64), 0, s, cams, C, und, use, N, out);
  else if (C <= 16)
    hipLaunchKernelGGL(pinv_dlt_kernel<16>, dim3((N + 63) / 64), dim3(64), 0, s, cams, C, und, use, N, out);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -1;
}


int geometry_affinity(const double* cams, int C, const double* pts, const int32_t* cam_of_det, int B, int M, int J,
                      double thr_kp, double* rays, double* dist, double* out, hipStream_t s) {
  if (B <= 0 || M <= 0) return 0;
  const int bmj = B * M * J;
  if (bmj > 0)
    hipLaunchKernelGGL(affinity_rays_kernel, dim3((bmj + 255) / 256), dim3(256), 0, s, cams, C, pts, cam_of_det,
                       B * M, J, rays);
  const int64_t pairs = (int64_t)B * M * M;
  hipLaunchKernelGGL(affinity_dist_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, s, rays, pts,
                     cam_of_det, C, B, M, J, thr_kp, dist);
  hipLaunchKernelGGL(affinity_norm_kernel, dim3(B), dim3(256), 0, s, dist, M, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t viterbi_scratch_bytes(int A, int F, int C, int J, int n_back) {
  const size_t chains = (size_t)A * C * J;
  const size_t rows = chains * F;
  return rows * n_back * (n_back + 4) * sizeof(double) + rows + rows * n_back + 512;
}

// scratch: viterbi_scratch_bytes() -- transitions, particle records, particle counts, back-pointers.
int viterbi_filter(const double* kp, int A, int F, int C, int J, double score_thr, int n_back, double thres_dist,
                   void* scratch, double* out, hipStream_t s) {
  const int chains = A * C * J;
  if (chains <= 0 || F <= 0) return 0;
  if (n_back > 3 || n_back < 1) return -2;
  const size_t rows = (size_t)chains * F;
  char* w = static_cast<char*>(scratch);
  VitBufs W;
  W.trans = reinterpret_cast<double*>(w);
  W.part = reinterpret_cast<double*>(w + rows * n_back * n_back * sizeof(double));
  W.cnt = reinterpret_cast<int8_t*>(w + rows * n_back * (n_back + 4) * sizeof(double));
  W.bk = W.cnt + rows;
  VitChain V{kp, F, C, J, n_back, score_thr};
  const size_t work = rows * n_back * n_back;
  hipLaunchKernelGGL(viterbi_trans_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, V, chains, thres_dist,
                     W);
  // as many chains per block as their back-pointers fit in LDS (64 at 300 frames), else global
  int threads = VIT_DP_THREADS;
  while (threads > 8 && (size_t)threads * F * n_back > 160 * 1024) threads >>= 1;
  const int in_lds = (size_t)threads * F * n_back <= 160 * 1024;
  const size_t lds = in_lds ? (size_t)threads * F * n_back : 0;
  const dim3 grid((chains + threads - 1) / threads);
  switch (n_back) {
    case 1: hipLaunchKernelGGL(viterbi_dp_kernel<1>, grid, dim3(threads), lds, s, V, chains, W, out, in_lds); break;
    case 2: hipLaunchKernelGGL(viterbi_dp_kernel<2>, grid, dim3(threads), lds, s, V, chains, W, out, in_lds); break;
    default: hipLaunchKernelGGL(viterbi_dp_kernel<3>, grid, dim3(threads), lds, s, V, chains, W, out, in_lds); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
