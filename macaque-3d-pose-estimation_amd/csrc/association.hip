// Step-2 cross-view matching on MI355X: matchSVT (step2_crossviewmatching.py:130-216), batched
// over keyframes.  One workgroup per keyframe runs the whole ADMM loop; nothing returns to the host
// between iterations.
//
// The reference takes a full SVD of the symmetric matrix M = Y/mu + X every iteration and keeps
// Q = U max(s - lambda/mu, 0) V^T.  For symmetric M = E diag(l) E^T that is
//   Q = sum_k sign(l_k) max(|l_k| - lambda/mu, 0) e_k e_k^T,
// so the kernel keeps an eigenbasis E instead: cyclic parallel Jacobi (round-robin pairing, N/2
// disjoint rotations per round, two-sided updates in LDS), warm-started from the previous iteration's
// E -- M moves little between ADMM iterations, so E^T M E is already nearly diagonal and one or two
// sweeps re-diagonalise it.  The elementwise steps (block zeroing per camera, diagonal 1, clip,
// symmetrise, dual update, primal / dual residuals, mu adaptation) follow the reference's order.
// The dual-stochastic projection (myproj2dpam) is off in the reference's MODEL_CFG (step2:30) and
// not implemented here; the host API rejects it.
//
// Layout: S, X, Y, W per keyframe (B, Nmax, Nmax) float64 row-major in HBM (X, Y, W in the context's
// association workspace, L2-resident); A, E, T (Ne x (Ne+1), Ne = N rounded up to even) in LDS.
#include "common.hpp"
#include "geometry.hpp"

namespace mq {
namespace {

constexpr int SVT_THREADS = 256;
constexpr int SVT_WAVES = SVT_THREADS / 64;
constexpr int SVT_MAX_N = 64;
constexpr int SVT_MAX_SWEEPS = 24;
// a rotation is applied when |a_pq| > SVT_OFF_TOL * ||M||_F (the Frobenius norm is invariant)
constexpr double SVT_OFF_TOL = 1e-14;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// block reductions in a fixed order (butterfly per wave, then wave 0..3 in order): deterministic
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < SVT_WAVES; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ double block_max(double v, double* red) {
  v = wave_max_d(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < SVT_WAVES; ++i) s = fmax(s, red[i]);
  return s;
}

// round r of the round-robin schedule on Ne players: pair m
__device__ __forceinline__ void rr_pair(int Ne, int r, int m, int& p, int& q) {
  const int n1 = Ne - 1;
  int a, b;
  if (m == 0) {
    a = r;
    b = n1;
  } else {
    a = (r + m) % n1;
    b = (r - m + n1) % n1;
  }
  p = a < b ? a : b;
  q = a < b ? b : a;
}

__global__ __launch_bounds__(SVT_THREADS) void match_svt_kernel(
    const double* __restrict__ S, const int32_t* __restrict__ n_det, const int32_t* __restrict__ cam_of_det,
    int Nmax, double alpha, double lambda, double mu0, double tol, int max_iter, int pselect, double* __restrict__ ws,
    uint8_t* __restrict__ match, double* __restrict__ x_out, int32_t* __restrict__ iters) {
  extern __shared__ double lds[];
  __shared__ double red[SVT_WAVES];
  __shared__ double rot_c[SVT_MAX_N / 2], rot_s[SVT_MAX_N / 2];
  __shared__ int rot_p[SVT_MAX_N / 2], rot_q[SVT_MAX_N / 2], rot_on[SVT_MAX_N / 2];
  __shared__ double fdiag[SVT_MAX_N];
  __shared__ int cam[SVT_MAX_N];

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int N = n_det[b];
  const size_t NN = (size_t)Nmax * Nmax;
  uint8_t* mb = match + (size_t)b * NN;
  if (N <= 0) {
    for (int e = tid; e < Nmax * Nmax; e += SVT_THREADS) mb[e] = 0;
    if (x_out)
      for (int e = tid; e < Nmax * Nmax; e += SVT_THREADS) x_out[(size_t)b * NN + e] = 0.0;
    if (tid == 0) iters[b] = -1;
    return;
  }
  const int Ne = N + (N & 1);
  const int ld = Ne + 1;
  double* A = lds;
  double* E = A + Ne * ld;
  double* T = E + Ne * ld;

  const double* Sb = S + (size_t)b * NN;
  double* X = ws + (size_t)b * 3 * NN;
  double* Y = X + NN;
  double* W = Y + NN;
  for (int i = tid; i < N; i += SVT_THREADS) cam[i] = cam_of_det[(size_t)b * Nmax + i];

  // S[diag] = 0; S = (S + S^T) / 2; X = S; Y = 0; W = alpha - S  (step2:148-155)
  for (int e = tid; e < N * N; e += SVT_THREADS) {
    const int i = e / N, j = e % N;
    const double sij = i == j ? 0.0 : Sb[i * Nmax + j];
    const double sji = i == j ? 0.0 : Sb[j * Nmax + i];
    const double s = (sij + sji) / 2.0;
    X[i * Nmax + j] = s;
    Y[i * Nmax + j] = 0.0;
    W[i * Nmax + j] = alpha - s;
  }
  for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
    const int i = e / Ne, j = e % Ne;
    E[i * ld + j] = i == j ? 1.0 : 0.0;
  }
  __syncthreads();

  double mu = mu0;
  int it = 0;
  for (it = 0; it < max_iter; ++it) {
    // M = Y / mu + X into T (zero padding row / column when N is odd)
    double fro = 0.0;
    for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
      const int i = e / Ne, j = e % Ne;
      double m = 0.0;
      if (i < N && j < N) m = Y[i * Nmax + j] / mu + X[i * Nmax + j];
      T[i * ld + j] = m;
      fro += m * m;
    }
    fro = block_sum(fro, red);  // contains a barrier: T is complete
    const double off_tol = SVT_OFF_TOL * sqrt(fro);

    // A = E^T (M E), symmetrised
    for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
      const int i = e / Ne, j = e % Ne;
      double acc = 0.0;
      for (int k = 0; k < Ne; ++k) acc += T[i * ld + k] * E[k * ld + j];
      A[i * ld + j] = acc;
    }
    __syncthreads();
    for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
      const int i = e / Ne, j = e % Ne;
      double acc = 0.0;
      for (int k = 0; k < Ne; ++k) acc += E[k * ld + i] * A[k * ld + j];
      T[i * ld + j] = acc;
    }
    __syncthreads();
    for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
      const int i = e / Ne, j = e % Ne;
      A[i * ld + j] = (T[i * ld + j] + T[j * ld + i]) / 2.0;
    }
    __syncthreads();

    // Jacobi sweeps until every off-diagonal entry is below off_tol
    for (int sweep = 0; sweep < SVT_MAX_SWEEPS; ++sweep) {
      double off = 0.0;
      for (int e = tid; e < Ne * Ne; e += SVT_THREADS) {
        const int i = e / Ne, j = e % Ne;
        if (i < j) off = fmax(off, fabs(A[i * ld + j]));
      }
      off = block_max(off, red);
      if (!(off > off_tol)) break;  // uniform across the block
      for (int r = 0; r < Ne - 1; ++r) {
        if (tid < Ne / 2) {
          int p, q;
          rr_pair(Ne, r, tid, p, q);
          const double apq = A[p * ld + q];
          double c = 1.0, s = 0.0;
          int on = 0;
          if (fabs(apq) > off_tol) {
            // symmetric Schur 2x2: J^T [app apq; apq aqq] J diagonal, J = [c s; -s c]
            const double tau = (A[q * ld + q] - A[p * ld + p]) / (2.0 * apq);
            const double t = tau >= 0.0 ? 1.0 / (tau + sqrt(1.0 + tau * tau)) : -1.0 / (-tau + sqrt(1.0 + tau * tau));
            c = 1.0 / sqrt(1.0 + t * t);
            s = t * c;
            on = 1;
          }
          rot_c[tid] = c;
          rot_s[tid] = s;
          rot_p[tid] = p;
          rot_q[tid] = q;
          rot_on[tid] = on;
        }
        __syncthreads();
        // rows: A <- J^T A
        for (int e = tid; e < (Ne / 2) * Ne; e += SVT_THREADS) {
          const int m = e / Ne, k = e % Ne;
          if (!rot_on[m]) continue;
          const int p = rot_p[m], q = rot_q[m];
          const double c = rot_c[m], s = rot_s[m];
          const double ap = A[p * ld + k], aq = A[q * ld + k];
          A[p * ld + k] = c * ap - s * aq;
          A[q * ld + k] = s * ap + c * aq;
        }
        __syncthreads();
        // columns: A <- A J, E <- E J
        for (int e = tid; e < (Ne / 2) * Ne; e += SVT_THREADS) {
          const int m = e / Ne, k = e % Ne;
          if (!rot_on[m]) continue;
          const int p = rot_p[m], q = rot_q[m];
          const double c = rot_c[m], s = rot_s[m];
          const double ap = A[k * ld + p], aq = A[k * ld + q];
          A[k * ld + p] = c * ap - s * aq;
          A[k * ld + q] = s * ap + c * aq;
          const double ep = E[k * ld + p], eq = E[k * ld + q];
          E[k * ld + p] = c * ep - s * eq;
          E[k * ld + q] = s * ep + c * eq;
        }
        __syncthreads();
      }
    }

    // singular value thresholding on the eigenvalues: f = sign(l) max(|l| - lambda/mu, 0)
    const double thr = lambda / mu;
    for (int k = tid; k < Ne; k += SVT_THREADS) {
      const double l = A[k * ld + k];
      const double sh = fmax(fabs(l) - thr, 0.0);
      fdiag[k] = l < 0.0 ? -sh : sh;
    }
    __syncthreads();
    // Q = E diag(f) E^T into T
    for (int e = tid; e < N * N; e += SVT_THREADS) {
      const int i = e / N, j = e % N;
      double acc = 0.0;
      for (int k = 0; k < Ne; ++k) acc += (E[i * ld + k] * fdiag[k]) * E[j * ld + k];
      T[i * ld + j] = acc;
    }
    __syncthreads();
    // X = Q - (W + Y)/mu; same-camera blocks 0; diagonal 1 (pselect); clip [0, 1]  -> A
    for (int e = tid; e < N * N; e += SVT_THREADS) {
      const int i = e / N, j = e % N;
      double x = T[i * ld + j] - (W[i * Nmax + j] + Y[i * Nmax + j]) / mu;
      if (cam[i] == cam[j]) x = 0.0;
      if (pselect == 1 && i == j) x = 1.0;
      x = fmin(fmax(x, 0.0), 1.0);
      A[i * ld + j] = x;
    }
    __syncthreads();
    // X = (X + X^T)/2; Y += mu (X - Q); residuals
    double pr = 0.0, dr = 0.0;
    for (int e = tid; e < N * N; e += SVT_THREADS) {
      const int i = e / N, j = e % N;
      const double xn = (A[i * ld + j] + A[j * ld + i]) / 2.0;
      const double q = T[i * ld + j];
      const double x0 = X[i * Nmax + j];
      Y[i * Nmax + j] = Y[i * Nmax + j] + mu * (xn - q);
      X[i * Nmax + j] = xn;
      pr += (xn - q) * (xn - q);
      dr += (xn - x0) * (xn - x0);
    }
    pr = block_sum(pr, red);
    dr = block_sum(dr, red);
    const double pRes = sqrt(pr) / N;
    const double dRes = mu * sqrt(dr) / N;
    if (pRes < tol && dRes < tol) break;
    if (pRes > 10.0 * dRes)
      mu *= 2.0;
    else if (dRes > 10.0 * pRes)
      mu /= 2.0;
  }
  __syncthreads();  // X complete in global memory for the whole block
  // X = (X + X^T)/2; match = X > 0.5
  for (int e = tid; e < Nmax * Nmax; e += SVT_THREADS) {
    const int i = e / Nmax, j = e % Nmax;
    double x = 0.0;
    if (i < N && j < N) x = (X[i * Nmax + j] + X[j * Nmax + i]) / 2.0;
    mb[e] = (i < N && j < N && x > 0.5) ? 1 : 0;
    if (x_out) x_out[(size_t)b * NN + e] = x;
  }
  if (tid == 0) iters[b] = it < max_iter ? it : max_iter - 1;
}

}  // namespace

size_t match_svt_workspace_bytes(int B, int Nmax) { return (size_t)B * 3 * Nmax * Nmax * sizeof(double) + 256; }

int match_svt(const double* S, const int32_t* n_det, const int32_t* cam_of_det, int B, int Nmax, double alpha,
              double lambda, double mu, double tol, int max_iter, int pselect, void* ws, uint8_t* match,
              double* x_out, int32_t* iters, hipStream_t s) {
  if (B <= 0) return 0;
  if (Nmax < 1 || Nmax > SVT_MAX_N) return -2;
  const int Ne = Nmax + (Nmax & 1);
  const size_t lds = (size_t)3 * Ne * (Ne + 1) * sizeof(double);
  static size_t attr_lds = 0;  // dynamic LDS above the 64 KB default needs the attribute (static LDS counts too)
  if (lds > attr_lds) {
    if (hipFuncSetAttribute((const void*)match_svt_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -1;
    attr_lds = lds;
  }
  hipLaunchKernelGGL(match_svt_kernel, dim3(B), dim3(SVT_THREADS), lds, s, S, n_det, cam_of_det, Nmax, alpha, lambda,
                     mu, tol, max_iter, pselect, static_cast<double*>(ws), match, x_out, iters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
