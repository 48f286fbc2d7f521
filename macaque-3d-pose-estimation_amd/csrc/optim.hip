// optim_points on the GPU (row a16): the aniposelib bundle-style refinement of
// 3D keypoints, cameras.py:1116-1190 (objective :1560-1620, parameter layout
// :1670-1697) and the fixed-length variant :1192-1415.
//
// Objective (identical residual set to the reference, per animal b):
//   x = [p3d (F*J*3), L (n_strong + n_weak)]
//   reprojection   r = rho(|p2d - project(X)|) per non-NaN coordinate
//                  (rho = soft_l1 2 rp (sqrt(1+|e|/rp)-1), huber, or |e|)
//   smoothness     r = ssf * diff^n(p3d over frames)         (np.diff order n)
//   lengths        r = s * 100 (|Xa - Xb| - L) / L           (s = strong / weak scale)
//
// Solver (MI355X-native, replaces scipy TRF + 2-point finite differences):
// Levenberg-Marquardt on the analytic Jacobian.  The normal matrix is never
// formed globally: it is applied as
//   H p = R_fj p_fj (3x3 reprojection blocks) + J_len^T (J_len p) + ssf^2 (D^T D (x) I) p + lam diag(H) p
// and each LM step is solved by preconditioned conjugate gradients.  The
// preconditioner is exact for everything except the cross-joint length
// couplings: one block-banded (3x3 blocks, bandwidth n) Cholesky per joint
// series over frames, plus a diagonal for the length variables.
//
// Determinism: every reduction is a fixed-order per-block / per-series sum, so
// results are bitwise reproducible run to run.
#include <algorithm>
#include <cstdio>
#include <vector>

#include "camera.hpp"
#include "common.hpp"
#include "optim_dev.hpp"

namespace mq {
namespace {

constexpr int OPT_MAXJ = 32;
constexpr int OPT_MAXL = 64;
constexpr int OPT_MAXN = 3;
constexpr int OPT_FS = 9 + 36 * OPT_MAXN;  // doubles per frame record of the factored preconditioner
constexpr int OPT_MAXK = 16;               // chunks of a series in the chunked substitutions (one lane quad each)

// Chunks the LDS preconditioner splits a series of F frames into: about sqrt(F), at most 16 (one wave of
// lane quads), each at least n frames long.  Chunk c is frames [c F / K, (c + 1) F / K).
__host__ __device__ inline int opt_chunks(int F, int n) {
  int k = 1;
  while ((k + 1) * (k + 1) <= F) ++k;
  k = k < OPT_MAXK ? k : OPT_MAXK;
  const int kn = F / (n > 0 ? n : 1);
  k = k < kn ? k : kn;
  return k > 1 ? k : 1;
}
constexpr int OPT_MAXC = 16;
constexpr int OPT_MAXIT = 128;  // PCG iterations per LM step (upper bound)
constexpr int OPT_THREADS = 128;

// -DOPT_PROFILE builds (tools only, never the shipped library): wall-clock time per phase of the LDS
// preconditioner kernel, summed over its blocks and printed by optim_points at the end of a solve.
#ifdef OPT_PROFILE
__device__ unsigned long long g_opt_prof[9];
#define OPT_PROF_BEGIN() \
  unsigned long long prof_t[9]; \
  prof_t[0] = wall_clock64()
#define OPT_PROF(k) prof_t[k] = wall_clock64()
#define OPT_PROF_END()                                                               \
  do {                                                                               \
    if (threadIdx.x == 0) {                                                          \
      for (int k = 1; k < 9; ++k) atomicAdd(&g_opt_prof[k], prof_t[k] - prof_t[k - 1]); \
      atomicAdd(&g_opt_prof[0], 1ull);                                               \
    }                                                                                \
  } while (0)
#else
#define OPT_PROF_BEGIN() (void)0
#define OPT_PROF(k) (void)0
#define OPT_PROF_END() (void)0
#endif

struct OptDims {
  int B, C, F, J, NL, nS, fix, n, loss;
  int NX, NV;
  double rp, s_len, s_len_weak, tol2;
  double c[OPT_MAXN + 1];
};

struct OptBufs {
  const double* cams;
  const double* p2d;
  const int* cons;    // [NL][2]
  const double* ssf;  // [B]
  const double* ctl;  // [B][2]: lambda, accept flag
  double *g, *diag, *R, *lenJ, *costF, *cost;
  double *d, *r, *z, *P0, *P1, *q, *fac, *pinvL, *rzJ, *pq, *pqF, *qLf;
  double* mn;  // [B][J][F][18 n]: the M / N blocks again, contiguous per series (LDS-DMA staging)
};

__device__ __forceinline__ double dtd(int f, int g, int F, int n, const double* c) {
  const int lo = max(0, max(f, g) - n), hi = min(min(f, g), F - 1 - n);
  double s = 0;
  for (int i = lo; i <= hi; ++i) s += c[f - i] * c[g - i];
  return s;
}

constexpr int OPT_RTHREADS = 512;  // the per-animal reductions over frames (one block per animal)

template <int NT = OPT_THREADS>
__device__ double block_sum(double v, double* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  const double out = red[0];
  __syncthreads();
  return out;
}

// ---------------------------------------------------------------------------------------------
// Residuals, cost and (mode 0) the Gauss-Newton pieces for one (frame, animal).
__global__ void __launch_bounds__(OPT_THREADS) optim_eval_kernel(OptDims D, OptBufs Bf, const double* __restrict__ x,
                                                                  int mode) {
  const int f = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int J = D.J, J3 = J * 3, F = D.F, n = D.n;
  __shared__ double sx[OPT_MAXJ * 3];
  __shared__ double slen[OPT_MAXL][5];
  __shared__ double ssg[OPT_MAXJ * 3], ssd[OPT_MAXJ * 3];
  __shared__ double red[OPT_THREADS];
  __shared__ int scons[2 * OPT_MAXL];  // the constraint list, read NL times by every joint thread below
  const double* xb = x + (size_t)b * D.NV;
  if (t < J3) sx[t] = xb[(size_t)f * J3 + t];
  if (t < 2 * D.NL) scons[t] = Bf.cons[t];
  __syncthreads();
  double cost = 0;
  const double ssf = Bf.ssf[b];
  if (t < D.NL) {  // joint-length residuals (cameras.py:1600-1616)
    const int a = scons[2 * t], c2 = scons[2 * t + 1];
    const double L = xb[D.NX + t];
    const double s = t < D.nS ? D.s_len : D.s_len_weak;
    const double dx = sx[3 * a] - sx[3 * c2], dy = sx[3 * a + 1] - sx[3 * c2 + 1], dz = sx[3 * a + 2] - sx[3 * c2 + 2];
    const double nr = sqrt(dx * dx + dy * dy + dz * dz);
    const double r = 100 * (nr - L) / L * s;
    cost += r * r;
    const double k = nr > 0 ? s * 100 / L / nr : 0.0;
    slen[t][0] = k * dx;
    slen[t][1] = k * dy;
    slen[t][2] = k * dz;
    slen[t][3] = -s * 100 * nr / (L * L);
    slen[t][4] = r;
    if (mode == 0) {
      double* o = Bf.lenJ + (((size_t)b * F + f) * D.NL + t) * 5;
#pragma unroll
      for (int i = 0; i < 5; ++i) o[i] = slen[t][i];
    }
  }
  if (t < J3 && F > n) {  // temporal smoothness (np.diff order n over frames)
    auto row = [&](int i) {
      double s = 0;
      for (int m = 0; m <= n; ++m) s += D.c[m] * xb[(size_t)(i + m) * J3 + t];
      return s * ssf;
    };
    if (f <= F - 1 - n) {
      const double rs = row(f);
      cost += rs * rs;
    }
    if (mode == 0) {
      double gs = 0;
      for (int i = max(0, f - n); i <= min(f, F - 1 - n); ++i) gs += D.c[f - i] * ssf * row(i);
      ssg[t] = gs;
      ssd[t] = ssf * ssf * dtd(f, f, F, n, D.c);
    }
  } else if (t < J3) {
    ssg[t] = 0;
    ssd[t] = 0;
  }
  __syncthreads();
  if (t < J) {  // reprojection, one thread per joint over all cameras
    double Rm[6] = {0, 0, 0, 0, 0, 0}, gr[3] = {0, 0, 0};
    const double X[3] = {sx[3 * t], sx[3 * t + 1], sx[3 * t + 2]};
    for (int c = 0; c < D.C; ++c) {
      const double* pp = Bf.p2d + ((((size_t)b * D.C + c) * F + f) * J + t) * 2;
      const double px = pp[0], py = pp[1];
      if (isnan(px) && isnan(py)) continue;
      double u, v, Ju[3], Jv[3];
      project_jac(cam_at(Bf.cams, c), X, u, v, Ju, Jv);
#pragma unroll
      for (int comp = 0; comp < 2; ++comp) {
        const double obs = comp ? py : px;
        if (isnan(obs)) continue;
        double r, dr;
        reproj_loss(obs - (comp ? v : u), D.rp, D.loss, r, dr);
        cost += r * r;
        const double* Jp = comp ? Jv : Ju;
        const double j0 = -dr * Jp[0], j1 = -dr * Jp[1], j2 = -dr * Jp[2];
        Rm[0] += j0 * j0;
        Rm[1] += j0 * j1;
        Rm[2] += j0 * j2;
        Rm[3] += j1 * j1;
        Rm[4] += j1 * j2;
        Rm[5] += j2 * j2;
        gr[0] += j0 * r;
        gr[1] += j1 * r;
        gr[2] += j2 * r;
      }
    }
    if (mode == 0) {
      double dg[3] = {Rm[0], Rm[3], Rm[5]};
      for (int k = 0; k < D.NL; ++k) {
        const int a = scons[2 * k], c2 = scons[2 * k + 1];
        const double sgn = (a == t) ? 1.0 : (c2 == t ? -1.0 : 0.0);
        if (sgn == 0.0) continue;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          gr[i] += sgn * slen[k][i] * slen[k][4];
          dg[i] += slen[k][i] * slen[k][i];
        }
      }
      double* Ro = Bf.R + (((size_t)b * F + f) * J + t) * 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) Ro[i] = Rm[i];
      const size_t o = (size_t)b * D.NV + (size_t)f * J3 + 3 * t;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        Bf.g[o + i] = gr[i] + ssg[3 * t + i];
        Bf.diag[o + i] = dg[i] + ssd[3 * t + i];
      }
    }
  }
  const double tot = block_sum(cost, red);
  if (t == 0) Bf.costF[(size_t)b * F + f] = tot;
}

// Sums over frames of the per-frame length terms, for every length variable: OPT_RCH frame chunks
// (f = c, c + OPT_RCH, ...) per length, each an unrolled run of independent loads, then the chunk
// partials in a fixed order -- deterministic, and latency-bound on ~F / OPT_RCH / 8 round trips
// instead of F.  qLf: [F][NL] (qL partials); lenJ: [F][NL][5] (gradient l[4] l[3], diagonal l[3]^2).
constexpr int OPT_RCH = OPT_RTHREADS / 32;
__device__ __forceinline__ void len_partials(const OptDims& D, const double* __restrict__ qLf,
                                             const double* __restrict__ lenJ, double (*pa)[OPT_MAXL],
                                             double (*pb)[OPT_MAXL], int t) {
  const int ch = t / 32;
  constexpr int UF = 512 / OPT_RCH;  // frames per chunk held in registers: every load of a clip up to 512 frames in flight at once
  for (int l = t % 32; l < D.NL; l += 32) {
    double a = 0, bsum = 0;
    double va[UF], vb[UF];
#pragma unroll
    for (int k = 0; k < UF; ++k) {
      const int f = ch + k * OPT_RCH;
      va[k] = vb[k] = 0.0;
      if (f < D.F) {
        if (qLf) {
          va[k] = qLf[(size_t)f * D.NL + l];
        } else {
          const double* q = lenJ + ((size_t)f * D.NL + l) * 5;
          va[k] = q[4];
          vb[k] = q[3];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < UF; ++k) {  // the sums in ascending frame order, as before
      if (ch + k * OPT_RCH < D.F) {
        if (qLf) {
          a += va[k];
        } else {
          a += va[k] * vb[k];
          bsum += vb[k] * vb[k];
        }
      }
    }
    for (int f = ch + UF * OPT_RCH; f < D.F; f += OPT_RCH) {  // longer clips (global-memory route)
      if (qLf) {
        a += qLf[(size_t)f * D.NL + l];
      } else {
        const double* q = lenJ + ((size_t)f * D.NL + l) * 5;
        a += q[4] * q[3];
        bsum += q[3] * q[3];
      }
    }
    pa[ch][l] = a;
    if (pb) pb[ch][l] = bsum;
  }
}

__device__ __forceinline__ double len_combine(const double (*p)[OPT_MAXL], int l) {
  double s = p[0][l];
#pragma unroll
  for (int c = 1; c < OPT_RCH; ++c) s += p[c][l];
  return s;
}

// cost[b] = sum_f costF (fixed order); mode 0 also reduces the length-variable gradient and diagonal.
__global__ void __launch_bounds__(OPT_RTHREADS) optim_reduce_kernel(OptDims D, OptBufs Bf, double* cost_out, int mode) {
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ double red[OPT_RTHREADS];
  double s = 0;
  for (int f = t; f < D.F; f += OPT_RTHREADS) s += Bf.costF[(size_t)b * D.F + f];
  const double tot = block_sum<OPT_RTHREADS>(s, red);
  if (t == 0) cost_out[b] = 0.5 * tot;  // scipy's cost convention
  if (mode == 0 && !D.fix) {
    __shared__ double pg[OPT_RCH][OPT_MAXL], pe[OPT_RCH][OPT_MAXL];
    len_partials(D, nullptr, Bf.lenJ + (size_t)b * D.F * D.NL * 5, pg, pe, t);
    __syncthreads();
    if (t < D.NL) {
      Bf.g[(size_t)b * D.NV + D.NX + t] = len_combine(pg, t);
      Bf.diag[(size_t)b * D.NV + D.NX + t] = len_combine(pe, t);
    }
  }
}

__device__ __forceinline__ double damp_of(double dg) { return fmax(dg, 1e-12); }

// Block-banded Cholesky of the per-joint preconditioner (thread per (animal, joint)).
// fac[((b*J + j)*F + f)*OPT_FS] holds the factor pre-multiplied for the two substitutions:
//   [0 .. 8]                      I_f = inv(L_ff) (lower)
//   [9 + 9(d-1) ..]   d = 1..n    M_{f,d} = I_f L_{f,f-d}          (zero for f - d < 0)
//   [9 + 9n + 9(d-1)..] d = 1..n  N_{f,d} = I_f^T L_{f+d,f}^T      (zero for f + d >= F)
//   [9 + 18n + 9(k-1)..] k = 1..n G_{f,k}: forward response of frame f to its chunk's incoming y_{a-k}
//   [9 + 27n + 9(k-1)..] k = 1..n H_{f,k}: backward response of frame f to the incoming z_{e+k-1}
// (chunks [a, e) as opt_chunks; G / H are written by the LDS factor kernel only, for the chunked
// substitutions of optim_precond_lds_kernel)
// so that L y = r is y_f = I_f r_f - sum_d M_{f,d} y_{f-d} and L^T z = y is
// z_f = I_f^T y_f - sum_d N_{f,d} z_{f+d}: the I_f r_f / I_f^T y_f products leave the sequential
// recurrence and run frame-parallel.  The factor recurrence is latency-bound: the last NN frames'
// blocks stay in registers and frame f+1's inputs are loaded while frame f is factored.
struct FacRec {
  double inv[9];
  double L[OPT_MAXN][9];  // L[d-1] = L_{f,f-d}
};

// Indices of the constraints touching joint j, into ck[OPT_MAXL]; returns their count.
__device__ __forceinline__ int joint_cons(const OptDims& D, const OptBufs& Bf, int j, int* ck) {
  int n = 0;
  for (int k = 0; k < D.NL; ++k)
    if (Bf.cons[2 * k] == j || Bf.cons[2 * k + 1] == j) ck[n++] = k;
  return n;
}

// Diagonal block of joint j at frame f: reprojection Gauss-Newton block + limb-length terms +
// smoothness + lam * damped diagonal.
template <int NN>
__device__ __forceinline__ void assemble_block(const OptDims& D, const OptBufs& Bf, const int* ck, int nck, int b,
                                               int j, int f, double s2, double lam, double (&A)[3][3]) {
  const int F = D.F, J = D.J;
  const double* Rm = Bf.R + (((size_t)b * F + f) * J + j) * 6;
  A[0][0] = Rm[0]; A[0][1] = Rm[1]; A[0][2] = Rm[2];
  A[1][0] = Rm[1]; A[1][1] = Rm[3]; A[1][2] = Rm[4];
  A[2][0] = Rm[2]; A[2][1] = Rm[4]; A[2][2] = Rm[5];
  const double* lb = Bf.lenJ + ((size_t)b * F + f) * D.NL * 5;
  for (int t = 0; t < nck; ++t) {
    const double* l = lb + ck[t] * 5;
    const double l0 = l[0], l1 = l[1], l2 = l[2];
    A[0][0] += l0 * l0; A[0][1] += l0 * l1; A[0][2] += l0 * l2;
    A[1][0] += l1 * l0; A[1][1] += l1 * l1; A[1][2] += l1 * l2;
    A[2][0] += l2 * l0; A[2][1] += l2 * l1; A[2][2] += l2 * l2;
  }
  const double* dg = Bf.diag + (size_t)b * D.NV + (size_t)f * J * 3 + 3 * j;
  const double sd = s2 * dtd(f, f, F, NN, D.c);
  A[0][0] += sd + lam * damp_of(dg[0]);
  A[1][1] += sd + lam * damp_of(dg[1]);
  A[2][2] += sd + lam * damp_of(dg[2]);
}

// 1/sqrt(x) for normal positive x: the hardware estimate refined by one Newton step (the factor only
// preconditions the solve, so it needs accuracy, not IEEE rounding)
__device__ __forceinline__ double rsq_f64(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = fma(-0.5 * x * y, y, 0.5);
  return fma(y, e, y);
}

// One step of the block-banded Cholesky recurrence: from frame f's diagonal block A and the last
// NN frames' factor blocks W (W[k-1] = frame f-k), the blocks L_{f,f-d} and inv(L_ff).
template <int NN>
__device__ __forceinline__ void factor_frame(const OptDims& D, double s2, int f, double (&A)[3][3],
                                             const FacRec (&W)[NN], FacRec& cur, const double* offs = nullptr) {
  // Only the structural non-zeros are formed: inv(L_ii) is lower triangular, so L_{f,i} = M inv(L_ii)^T
  // needs the k <= c terms of each entry; with no older block the product is off * inv(L_ii)^T alone;
  // and A_f only feeds its lower triangle to the Cholesky below.  (Zero terms added nothing before:
  // the same values, a third fewer dependent f64 operations on the sequential chain.)
  const int F = D.F;
#pragma unroll
  for (int d = NN; d >= 1; --d) {
    const int i = f - d;
    if (i < 0) {
#pragma unroll
      for (int e = 0; e < 9; ++e) cur.L[d - 1][e] = 0.0;
      continue;
    }
    // s2 dtd(f, f - d): precomputed by the LDS kernel (offs[d - 1], frame-parallel), else formed here
    const double off = offs ? offs[d - 1] : s2 * dtd(f, i, F, NN, D.c);
    const double* Ii = W[d - 1].inv;  // inv(L_ii) (lower)
    bool older = false;
#pragma unroll
    for (int e = d + 1; e <= NN; ++e) older |= f - e >= 0;
    if (!older) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) cur.L[d - 1][3 * r + c] = r <= c ? off * Ii[3 * c + r] : 0.0;
      continue;
    }
    double M[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) M[r][c] = (r == c) ? off : 0.0;
#pragma unroll
    for (int e = d + 1; e <= NN; ++e) {
      if (f - e < 0) continue;
      const double* Lf = cur.L[e - 1];          // L_{f, f-e}
      const double* Li = W[d - 1].L[e - d - 1];  // L_{i, f-e}
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          M[r][c] -= Lf[3 * r] * Li[3 * c] + Lf[3 * r + 1] * Li[3 * c + 1] + Lf[3 * r + 2] * Li[3 * c + 2];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      cur.L[d - 1][3 * r + 0] = M[r][0] * Ii[0];
      cur.L[d - 1][3 * r + 1] = M[r][0] * Ii[3] + M[r][1] * Ii[4];
      cur.L[d - 1][3 * r + 2] = M[r][0] * Ii[6] + M[r][1] * Ii[7] + M[r][2] * Ii[8];
    }
  }
#pragma unroll
  for (int d = 1; d <= NN; ++d) {
    if (f - d < 0) continue;
    const double* Lf = cur.L[d - 1];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c)
        A[r][c] -= Lf[3 * r] * Lf[3 * c] + Lf[3 * r + 1] * Lf[3 * c + 1] + Lf[3 * r + 2] * Lf[3 * c + 2];
  }
  // 3x3 Cholesky by reciprocal square roots: the recurrence's latency chain is three v_rsq_f64 (+ one
  // Newton step each) instead of three IEEE square roots and five IEEE divisions.  Only inv(L_ff) and
  // the off-diagonal blocks are kept, so L_ff's own diagonal is never formed.
  const double i00 = rsq_f64(fmax(A[0][0], 1e-300));
  const double l10 = A[1][0] * i00, l20 = A[2][0] * i00;
  const double i11 = rsq_f64(fmax(A[1][1] - l10 * l10, 1e-300));
  const double l21 = (A[2][1] - l20 * l10) * i11;
  const double i22 = rsq_f64(fmax(A[2][2] - l20 * l20 - l21 * l21, 1e-300));
  const double i10 = -l10 * i00 * i11;
  const double i21 = -l21 * i11 * i22;
  const double i20 = -(l20 * i00 + l21 * i10) * i22;
  cur.inv[0] = i00; cur.inv[1] = 0; cur.inv[2] = 0;
  cur.inv[3] = i10; cur.inv[4] = i11; cur.inv[5] = 0;
  cur.inv[6] = i20; cur.inv[7] = i21; cur.inv[8] = i22;
}

// M_{f,d} = I_f L_{f,f-d} and N_{f,d} = (L_{f+d,f} I_f)^T (the record layout above).
__device__ __forceinline__ void premul_M(const double* I, const double* Lf, double* o) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) o[3 * r + c] = I[3 * r] * Lf[c] + I[3 * r + 1] * Lf[3 + c] + I[3 * r + 2] * Lf[6 + c];
}
__device__ __forceinline__ void premul_N(const double* Ii, const double* Lf, double* o) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) o[3 * r + c] = Lf[3 * c] * Ii[r] + Lf[3 * c + 1] * Ii[3 + r] + Lf[3 * c + 2] * Ii[6 + r];
}

// Global-memory factorization, one thread per (animal, joint): for clips too long for LDS.
template <int NN>
__device__ void factor_series(const OptDims& D, const OptBufs& Bf, int b, int j, double lam) {
  const int F = D.F, J = D.J;
  const double ssf = Bf.ssf[b];
  const double s2 = F > NN ? ssf * ssf : 0.0;
  double* fb = Bf.fac + ((size_t)b * J + j) * F * OPT_FS;
  int ck[OPT_MAXL];
  const int nck = joint_cons(D, Bf, j, ck);
  FacRec W[NN];  // W[k-1] = frame f-k
  double An[3][3];
  assemble_block<NN>(D, Bf, ck, nck, b, j, 0, s2, lam, An);
  for (int f = 0; f < F; ++f) {
    double A[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) A[r][c] = An[r][c];
    if (f + 1 < F) assemble_block<NN>(D, Bf, ck, nck, b, j, f + 1, s2, lam, An);
    FacRec cur;
    factor_frame<NN>(D, s2, f, A, W, cur);
    double* o = fb + (size_t)f * OPT_FS;
#pragma unroll
    for (int e = 0; e < 9; ++e) o[e] = cur.inv[e];
#pragma unroll
    for (int d = 1; d <= NN; ++d) {
      premul_M(cur.inv, cur.L[d - 1], o + 9 * d);
      if (f - d >= 0) premul_N(W[d - 1].inv, cur.L[d - 1], fb + (size_t)(f - d) * OPT_FS + 9 + 9 * NN + 9 * (d - 1));
      if (f + d >= F) {
#pragma unroll
        for (int e = 0; e < 9; ++e) o[9 + 9 * NN + 9 * (d - 1) + e] = 0.0;
      }
    }
#pragma unroll
    for (int k = NN - 1; k >= 1; --k) W[k] = W[k - 1];
    W[0] = cur;
  }
}

__device__ __forceinline__ void length_pinv(const OptDims& D, const OptBufs& Bf, int b, double lam) {
  if (D.fix) return;
  for (int k = 0; k < D.NL; ++k) {
    const double E = Bf.diag[(size_t)b * D.NV + D.NX + k];
    Bf.pinvL[(size_t)b * OPT_MAXL + k] = 1.0 / (E + lam * damp_of(E) + 1e-300);
  }
}

__global__ void __launch_bounds__(64) optim_factor_kernel(OptDims D, OptBufs Bf) {
  const int b = blockIdx.x, j = threadIdx.x;
  const int J = D.J;
  const double lam = Bf.ctl[2 * b];
  if (j == J) {
    length_pinv(D, Bf, b, lam);
    return;
  }
  if (j > J) return;
  if (D.n == 1) factor_series<1>(D, Bf, b, j, lam);
  else if (D.n == 2) factor_series<2>(D, Bf, b, j, lam);
  else factor_series<3>(D, Bf, b, j, lam);
}

// The factorization with the series in LDS, one 256-thread block per (joint, animal):
//   1. all threads assemble the diagonal blocks A_f (frame-parallel);
//   2. thread 0 runs the Cholesky recurrence on LDS operands (inv(L_ff), L_{f,f-d} into LDS);
//   3. all threads write I_f and the pre-multiplied M / N blocks (frame-parallel).
// Only the recurrence's own arithmetic is sequential.  LDS: optim_factor_lds_bytes.
template <int NN>
__global__ void __launch_bounds__(256) optim_factor_lds_kernel(OptDims D, OptBufs Bf) {
  const int j = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int F = D.F, J = D.J;
  const double lam = Bf.ctl[2 * b];
  if (j == J) {  // the length variables' diagonal, one thread per length
    if (!D.fix && t < D.NL) {
      const double E = Bf.diag[(size_t)b * D.NV + D.NX + t];
      Bf.pinvL[(size_t)b * OPT_MAXL + t] = 1.0 / (E + lam * damp_of(E) + 1e-300);
    }
    return;
  }
  constexpr int RS = 9 + 9 * NN;  // record doubles: inv(L_ff), L_{f,f-1..n}
  extern __shared__ double lds_opt[];
  double* sA = lds_opt;               // [F][6] upper triangle of A_f
  double* sRec = sA + (size_t)F * 6;  // [F][RS]
  double* sOff = sRec + (size_t)F * RS;  // [F][NN] s2 dtd(f, f - d): the recurrence's only other inputs
  const double ssf = Bf.ssf[b];
  const double s2 = F > NN ? ssf * ssf : 0.0;
  __shared__ int s_ck[OPT_MAXL];
  __shared__ int s_nck;
  if (t == 0) s_nck = joint_cons(D, Bf, j, s_ck);
  __syncthreads();
  const int nck = s_nck;
  for (int f = t; f < F; f += 256) {
    double A[3][3];
    assemble_block<NN>(D, Bf, s_ck, nck, b, j, f, s2, lam, A);
    double* o = sA + 6 * f;
    o[0] = A[0][0]; o[1] = A[0][1]; o[2] = A[0][2];
    o[3] = A[1][1]; o[4] = A[1][2]; o[5] = A[2][2];
#pragma unroll
    for (int d = 1; d <= NN; ++d) sOff[(size_t)f * NN + d - 1] = f - d >= 0 ? s2 * dtd(f, f - d, F, NN, D.c) : 0.0;
  }
  __syncthreads();
  if (t == 0) {
    FacRec W[NN];
#pragma unroll 2  // the W rotation becomes register renaming (n = 2)
    for (int f = 0; f < F; ++f) {
      const double* a = sA + 6 * f;
      double A[3][3];
      A[0][0] = a[0]; A[0][1] = a[1]; A[0][2] = a[2];
      A[1][0] = a[1]; A[1][1] = a[3]; A[1][2] = a[4];
      A[2][0] = a[2]; A[2][1] = a[4]; A[2][2] = a[5];
      FacRec cur;
      factor_frame<NN>(D, s2, f, A, W, cur, sOff + (size_t)f * NN);
      double* o = sRec + (size_t)f * RS;
#pragma unroll
      for (int e = 0; e < 9; ++e) o[e] = cur.inv[e];
#pragma unroll
      for (int d = 0; d < NN; ++d)
#pragma unroll
        for (int e = 0; e < 9; ++e) o[9 + 9 * d + e] = cur.L[d][e];
#pragma unroll
      for (int k = NN - 1; k >= 1; --k) W[k] = W[k - 1];
      W[0] = cur;
    }
  }
  __syncthreads();
  double* fb = Bf.fac + ((size_t)b * J + j) * F * OPT_FS;
  double* mnb = Bf.mn + ((size_t)b * J + j) * F * (18 * NN);
  for (int f = t; f < F; f += 256) {
    const double* rec = sRec + (size_t)f * RS;
    double* o = fb + (size_t)f * OPT_FS;
#pragma unroll
    for (int e = 0; e < 9; ++e) o[e] = rec[e];
    double mnv[18 * NN];
#pragma unroll
    for (int d = 1; d <= NN; ++d) {
      premul_M(rec, rec + 9 * d, mnv + 9 * (d - 1));
      double* on = mnv + 9 * NN + 9 * (d - 1);
      if (f + d < F) {
        premul_N(rec, sRec + (size_t)(f + d) * RS + 9 * d, on);
      } else {
#pragma unroll
        for (int e = 0; e < 9; ++e) on[e] = 0.0;
      }
    }
#pragma unroll
    for (int e = 0; e < 18 * NN; ++e) {
      o[9 + e] = mnv[e];
      mnb[(size_t)f * 18 * NN + e] = mnv[e];
    }
  }
  // Chunk responses for the chunked substitutions: thread per (direction, chunk, incoming column).
  // Forward, chunk c >= 1 over [a, e): the column (k, comp) is the solution over the chunk of
  // g_f = -sum_d M_{f,d} X_{f-d} with X = unit vector comp at frame a - k, zero at the other incoming
  // frames, g inside the chunk.  Backward, chunk c <= K - 2: h_f = -sum_d N_{f,d} X_{f+d} from a unit
  // vector at frame e + k - 1.  M / N are re-formed from the LDS factor (premul_M / premul_N, the same
  // arithmetic as the records above).
  const int K = opt_chunks(F, NN);
  constexpr int NC = 3 * NN;
  const int per_dir = (K - 1) * NC;
  for (int tt = t; tt < 2 * per_dir; tt += 256) {
    const bool back = tt >= per_dir;
    const int u = back ? tt - per_dir : tt;
    const int c = back ? u / NC : 1 + u / NC;  // forward chunks 1 .. K-1, backward 0 .. K-2
    const int col = u % NC, k = col / 3 + 1, comp = col % 3;
    const int a = c * F / K, e = (c + 1) * F / K;
    double X[NN][3];  // X[d-1]: the value d frames back (forward) / ahead (backward)
#pragma unroll
    for (int d = 0; d < NN; ++d)
#pragma unroll
      for (int r = 0; r < 3; ++r) X[d][r] = (d == k - 1 && r == comp) ? 1.0 : 0.0;
    // forward: X[d-1] at frame a is frame a - d, so the unit sits at d = k; backward: X[d-1] at frame
    // e - 1 is frame e - 1 + d, unit at d = k -- the same initial pattern
    const int len = e - a;
    for (int s2 = 0; s2 < len; ++s2) {
      const int f = back ? e - 1 - s2 : a + s2;
      const double* rec = sRec + (size_t)f * RS;
      double gv[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int d = NN; d >= 1; --d) {
        double Mb[9];
        if (!back) {
          premul_M(rec, rec + 9 * d, Mb);
        } else if (f + d < F) {
          premul_N(rec, sRec + (size_t)(f + d) * RS + 9 * d, Mb);
        } else {
#pragma unroll
          for (int i = 0; i < 9; ++i) Mb[i] = 0.0;
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) gv[r] = gv[r] - Mb[3 * r] * X[d - 1][0] - Mb[3 * r + 1] * X[d - 1][1] - Mb[3 * r + 2] * X[d - 1][2];
      }
      double* o = fb + (size_t)f * OPT_FS + 9 + (back ? 27 : 18) * NN + 9 * (k - 1);
#pragma unroll
      for (int r = 0; r < 3; ++r) o[3 * r + comp] = gv[r];
#pragma unroll
      for (int d = NN - 1; d >= 1; --d)
#pragma unroll
        for (int r = 0; r < 3; ++r) X[d][r] = X[d - 1][r];
#pragma unroll
      for (int r = 0; r < 3; ++r) X[0][r] = gv[r];
    }
  }
}

size_t optim_factor_lds_bytes(int F, int NN) { return (size_t)F * (15 + 10 * NN) * sizeof(double); }

// Sum over the J + 1 series of the r.z partials of PCG iteration it, by the whole wave: lane l loads
// partial l (one load per lane, a single round trip) and an xor butterfly adds them, so every lane
// of every wave that asks ends with the same bits (each step adds the same two values, commuted).
// Every lane of the calling wave must be active.
__device__ __forceinline__ double rz_at(const OptDims& D, const OptBufs& Bf, int b, int it) {
  const int lane = threadIdx.x & 63;
  const double* p = Bf.rzJ + ((size_t)b * (OPT_MAXIT + 1) + it) * (D.J + 1);
  double v = lane <= D.J ? p[lane] : 0.0;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// rz_at for several iterations at once, the butterflies interleaved so every step's cross-lane moves share
// one wait (the same additions, so the same bits as separate rz_at calls)
template <int NI>
__device__ __forceinline__ void rz_at_n(const OptDims& D, const OptBufs& Bf, int b, const int (&its)[NI],
                                        double (&out)[NI]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const double* p = Bf.rzJ + ((size_t)b * (OPT_MAXIT + 1) + its[i]) * (D.J + 1);
    out[i] = lane <= D.J ? p[lane] : 0.0;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    double w[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) w[i] = __shfl_xor(out[i], m);
#pragma unroll
    for (int i = 0; i < NI; ++i) out[i] += w[i];
  }
}

__device__ __forceinline__ bool pcg_done(const OptDims& D, const OptBufs& Bf, int b, int it) {
  const double r0 = rz_at(D, Bf, b, 0);
  if (!(r0 > 0)) return true;
  if (it == 0) return false;
  const double ri = rz_at(D, Bf, b, it);
  return !(ri > D.tol2 * r0);
}

// z = M^-1 r for one joint series (and the length diagonal for j == J); it < 0: init (d = 0, r = -g),
// else first d += alpha p_it, r -= alpha q_it.  Writes the series' r.z partial to rzJ[it + 1].
// Both substitutions keep the last NN solution vectors in registers and load frame f+-1's
// inputs while frame f is solved (the recurrence is latency-bound, one thread per series).
// Global-memory form of optim_precond_lds_kernel, for clips too long for LDS.
template <int NN>
__device__ double solve_series(const OptDims& D, const OptBufs& Bf, int b, int j, int it, double alpha,
                               const double* __restrict__ P) {
  const int F = D.F, J = D.J, J3 = 3 * J;
  const size_t base = (size_t)b * D.NV + 3 * j;
  const double* __restrict__ fb = Bf.fac + ((size_t)b * J + j) * F * OPT_FS;
  double* __restrict__ z = Bf.z;
  double* __restrict__ r = Bf.r;
  double* __restrict__ dd = Bf.d;
  const double* __restrict__ g = Bf.g;
  const double* __restrict__ q = Bf.q;
  struct In {
    double rec[9 + 9 * NN];  // I_f, M_{f,1..n}
    double r[3], d[3], p[3], q[3];
  };
  auto load_in = [&](int f, In& x) {
    const double* rc = fb + (size_t)f * OPT_FS;
#pragma unroll
    for (int e = 0; e < 9 + 9 * NN; ++e) x.rec[e] = rc[e];
    const size_t o = base + (size_t)f * J3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (it < 0) {
        x.r[i] = -g[o + i];
      } else {
        x.r[i] = r[o + i];
        x.d[i] = dd[o + i];
        x.p[i] = P[o + i];
        x.q[i] = q[o + i];
      }
    }
  };
  double Y[NN][3];
#pragma unroll
  for (int k = 0; k < NN; ++k) Y[k][0] = Y[k][1] = Y[k][2] = 0.0;
  In nx;
  load_in(0, nx);
  for (int f = 0; f < F; ++f) {  // forward: y_f = I_f r_f - sum_d M_{f,d} y_{f-d}
    const In cu = nx;
    if (f + 1 < F) load_in(f + 1, nx);
    const size_t o = base + (size_t)f * J3;
    double rr[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (it < 0) {
        dd[o + i] = 0.0;
        rr[i] = cu.r[i];
      } else {
        dd[o + i] = cu.d[i] + alpha * cu.p[i];
        rr[i] = cu.r[i] - alpha * cu.q[i];
      }
      r[o + i] = rr[i];
    }
    const double* I = cu.rec;
    double w[3] = {I[0] * rr[0], I[3] * rr[0] + I[4] * rr[1], I[6] * rr[0] + I[7] * rr[1] + I[8] * rr[2]};
#pragma unroll
    for (int d = NN; d >= 1; --d) {
      const double* M = cu.rec + 9 * d;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        w[i] -= M[3 * i] * Y[d - 1][0] + M[3 * i + 1] * Y[d - 1][1] + M[3 * i + 2] * Y[d - 1][2];
    }
    z[o] = w[0];
    z[o + 1] = w[1];
    z[o + 2] = w[2];
#pragma unroll
    for (int k = NN - 1; k >= 1; --k) {
      Y[k][0] = Y[k - 1][0];
      Y[k][1] = Y[k - 1][1];
      Y[k][2] = Y[k - 1][2];
    }
    Y[0][0] = w[0];
    Y[0][1] = w[1];
    Y[0][2] = w[2];
  }
  // backward: z_f = I_f^T y_f - sum_d N_{f,d} z_{f+d}.  Frame f needs its own record, y_f, r_f.
  struct Bk {
    double inv[9];
    double N[NN][9];
    double y[3], r[3];
  };
  auto load_bk = [&](int f, Bk& x) {
    const double* rc = fb + (size_t)f * OPT_FS;
#pragma unroll
    for (int e = 0; e < 9; ++e) x.inv[e] = rc[e];
#pragma unroll
    for (int d = 0; d < NN; ++d)
#pragma unroll
      for (int e = 0; e < 9; ++e) x.N[d][e] = rc[9 + 9 * NN + 9 * d + e];
    const size_t o = base + (size_t)f * J3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      x.y[i] = z[o + i];
      x.r[i] = r[o + i];
    }
  };
  double Z[NN][3];
#pragma unroll
  for (int k = 0; k < NN; ++k) Z[k][0] = Z[k][1] = Z[k][2] = 0.0;
  double rz = 0;
  Bk bn;
  load_bk(F - 1, bn);
  for (int f = F - 1; f >= 0; --f) {
    const Bk bc = bn;
    if (f > 0) load_bk(f - 1, bn);
    const double* I = bc.inv;
    double w[3] = {I[0] * bc.y[0] + I[3] * bc.y[1] + I[6] * bc.y[2], I[4] * bc.y[1] + I[7] * bc.y[2], I[8] * bc.y[2]};
#pragma unroll
    for (int d = NN; d >= 1; --d) {
      const double* N = bc.N[d - 1];
#pragma unroll
      for (int i = 0; i < 3; ++i)
        w[i] -= N[3 * i] * Z[d - 1][0] + N[3 * i + 1] * Z[d - 1][1] + N[3 * i + 2] * Z[d - 1][2];
    }
    const size_t o = base + (size_t)f * J3;
    z[o] = w[0];
    z[o + 1] = w[1];
    z[o + 2] = w[2];
    rz += bc.r[0] * w[0] + bc.r[1] * w[1] + bc.r[2] * w[2];
#pragma unroll
    for (int k = NN - 1; k >= 1; --k) {
      Z[k][0] = Z[k - 1][0];
      Z[k][1] = Z[k - 1][1];
      Z[k][2] = Z[k - 1][2];
    }
    Z[0][0] = w[0];
    Z[0][1] = w[1];
    Z[0][2] = w[2];
  }
  return rz;
}

__global__ void __launch_bounds__(64) optim_precond_kernel(OptDims D, OptBufs Bf, int it) {
  const int b = blockIdx.x, j = threadIdx.x;
  const int J = D.J;
  double alpha = 0;
  const double* P = (it & 1) ? Bf.P1 : Bf.P0;
  if (it >= 0) {  // (the whole wave: rz_at)
    if (pcg_done(D, Bf, b, it)) return;
    const double pq = Bf.pq[(size_t)b * (OPT_MAXIT + 1) + it];
    if (!(pq > 0)) return;
    alpha = rz_at(D, Bf, b, it) / pq;
  }
  if (j > J) return;
  const size_t base = (size_t)b * D.NV;
  double rz = 0;
  if (j == J) {
    if (!D.fix)
      for (int k = 0; k < D.NL; ++k) {
        const size_t o = base + D.NX + k;
        double r;
        if (it < 0) {
          Bf.d[o] = 0;
          r = -Bf.g[o];
        } else {
          Bf.d[o] += alpha * P[o];
          r = Bf.r[o] - alpha * Bf.q[o];
        }
        Bf.r[o] = r;
        const double z = r * Bf.pinvL[(size_t)b * OPT_MAXL + k];
        Bf.z[o] = z;
        rz += r * z;
      }
  } else if (D.n == 1) {
    rz = solve_series<1>(D, Bf, b, j, it, alpha, P);
  } else if (D.n == 2) {
    rz = solve_series<2>(D, Bf, b, j, it, alpha, P);
  } else {
    rz = solve_series<3>(D, Bf, b, j, it, alpha, P);
  }
  Bf.rzJ[((size_t)b * (OPT_MAXIT + 1) + (it + 1)) * (J + 1) + j] = rz;
}

// Broadcast lane K of each lane quad to the quad (DPP quad_perm, no LDS round trip).
template <int K>
__device__ __forceinline__ double quad_bcast(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)u, K * 0x55, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), K * 0x55, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// w -= a . v and p -= b . v as two fma chains, interleaved in issue order (the scheduler otherwise
// emits one chain after the other, and in-order issue then puts both on the latency path)
__device__ __forceinline__ void fma3_pair(double& w, double& p, const double (&a)[3], const double (&b)[3],
                                          const double (&v)[3]) {
  asm("v_fma_f64 %0, -%2, %8, %0\n\t"
      "v_fma_f64 %1, -%5, %8, %1\n\t"
      "v_fma_f64 %0, -%3, %9, %0\n\t"
      "v_fma_f64 %1, -%6, %9, %1\n\t"
      "v_fma_f64 %0, -%4, %10, %0\n\t"
      "v_fma_f64 %1, -%7, %10, %1"
      : "+v"(w), "+v"(p)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(v[0]), "v"(v[1]), "v"(v[2]));
}

// One sequential substitution over the series, run by lanes 0..3: lane q = 0, 1, 2 owns row q of
// the 3-vector (lane 3 repeats row 2), and the new vector reaches every lane by three DPP
// broadcasts.  Forward (BACK false): out_f = in_f - sum_d A[f][d] out_{f-d}; backward:
// out_f = in_f - sum_d A[f][n + d] out_{f+d}, with A[f] the 18n M / N doubles of frame f.  The
// terms are summed farthest frame first, and only the nearest frame's three products wait on the
// previous step: the far terms of step s + 1 (in_{s+1} - sum_{d >= 2} ...) are formed during step s,
// off the latency chain.  Operands are read from LDS two steps ahead (three register sets).
//
// Chunked form: the quad solves frames [f0, f0 + len) with zero incoming vectors; every quad of the
// wave runs the same trip count L >= len (chunk lengths differ by one), and the steps past len write a
// pad slot out[3 * pad + i] instead of a frame.
template <int NN, bool BACK>
__device__ __forceinline__ void lane_substitution(const double* __restrict__ smn, const double* __restrict__ in,
                                                  double* __restrict__ out, int f0, int len, int L, int pad,
                                                  int t) {
#pragma clang fp contract(fast)
  const int q = t & 3, i = q < 3 ? q : 2;
  const int F = L;
  double V[NN][3];
#pragma unroll
  for (int k = 0; k < NN; ++k) V[k][0] = V[k][1] = V[k][2] = 0.0;
  struct Ops {
    double a[NN][3];
    double in;
  };
  auto frame = [&](int s) {
    const int sc = min(s, len - 1);
    return BACK ? f0 + len - 1 - sc : f0 + sc;
  };
  auto load = [&](int s, Ops& o) {
    const int f = frame(s);
    const double* A = smn + (size_t)f * (18 * NN) + (BACK ? 9 * NN : 0) + 3 * i;
#pragma unroll
    for (int d = 0; d < NN; ++d) {
      o.a[d][0] = A[9 * d];
      o.a[d][1] = A[9 * d + 1];
      o.a[d][2] = A[9 * d + 2];
    }
    o.in = in[3 * f + i];
    __builtin_amdgcn_sched_barrier(0);  // keep the look-ahead loads ahead of the step they overlap
  };
  // in - sum_{d = NN .. 2} a[d-1] . W[d-1-shift] (farthest first): the far terms of a step; shift 1
  // when formed one step early (step s + 1's V[d-1] is step s's V[d-2]).  dmin = 3 leaves out the
  // d = 2 terms (formed by fma3_pair below).
  auto far = [&](const Ops& o, int shift, int dmin) {
    double p = o.in;
#pragma unroll
    for (int d = NN; d >= dmin; --d)
      p = p - o.a[d - 1][0] * V[d - 1 - shift][0] - o.a[d - 1][1] * V[d - 1 - shift][1] -
          o.a[d - 1][2] * V[d - 1 - shift][2];
    return p;
  };
  double part;
  auto step = [&](int s, const Ops& cur, const Ops& nxt) {
    const int f = s < len ? frame(s) : pad;
    double w = part;
    if constexpr (NN >= 2) {
      // this step's nearest-frame terms and step s + 1's d = 2 terms, both on V[0], as two
      // interleaved fma chains: the far chain fills the latency of the critical one (same operation
      // order as the plain expression, so the same rounding)
      part = far(nxt, 1, 3);
      fma3_pair(w, part, cur.a[0], nxt.a[1], V[0]);
    } else {
      w = w - cur.a[0][0] * V[0][0] - cur.a[0][1] * V[0][1] - cur.a[0][2] * V[0][2];
      part = nxt.in;
    }
    out[3 * f + i] = w;     // lanes 2 and 3 store the same value
#pragma unroll
    for (int k = NN - 1; k >= 1; --k) {
      V[k][0] = V[k - 1][0];
      V[k][1] = V[k - 1][1];
      V[k][2] = V[k - 1][2];
    }
    V[0][0] = quad_bcast<0>(w);
    V[0][1] = quad_bcast<1>(w);
    V[0][2] = quad_bcast<2>(w);
  };
  // the look-ahead loads are unconditional (clamped to the last step) so that the LDS counter
  // wait before a step covers only the operands it uses
  Ops ra, rb, rc;
  load(0, ra);
  load(min(1, F - 1), rb);
  part = far(ra, 0, 2);
  // whole rounds of three steps without exits (an exit between the steps would let the compiler sink
  // the far terms behind the next step's latency chain), then the 0 - 2 remaining steps
  const int F3 = F - F % 3;
  int s = 0;
  for (; s < F3; s += 3) {
    load(min(s + 2, F - 1), rc);
    step(s, ra, rb);
    load(min(s + 3, F - 1), ra);
    step(s + 1, rb, rc);
    load(min(s + 4, F - 1), rb);
    step(s + 2, rc, ra);
  }
  if (s < F) {
    load(min(s + 2, F - 1), rc);
    step(s, ra, rb);
    if (s + 1 < F) step(s + 1, rb, rc);
  }
}

// The same preconditioner step with the series staged in LDS: one 256-thread block per (joint
// series, animal).  The two substitutions are split into K chunks (opt_chunks, ~sqrt(F)) solved at
// once, one lane quad each, and stitched together through the chunk responses G / H of the factor
// record, so the sequential depth is ~F / K + K steps instead of F:
//   1. all threads: r_f = r_f - alpha q_f, d_f += alpha p_f, u_f = I_f r_f; stage M / N blocks and the
//      chunk-boundary G / H blocks;
//   2. quad c:      y^_f = u_f - sum_d M_{f,d} y^_{f-d} over chunk c, zero incoming  (forward)
//   3. lanes < 3n:  the true last n vectors of each chunk, chunk by chunk:
//                   S_c[k] = y_{a_c - k} = y^_{a_c - k} + sum_j G_{a_c - k, j} S_{c-1}[j]
//   4. all threads: y_f = y^_f + sum_k G_{f,k} S_c[k];  v_f = I_f^T y_f
//   5-7.            the same backward (N, H, chunks from the last), z_f = z^_f + sum_k H_{f,k} T_c[k]
//   8. all threads: write r, z; block-reduce r.z.
// A sequential step is 3n fused products per lane on LDS operands (lane_substitution).  Run from
// global memory the same recurrence waits on loads left in another XCD's L2.  LDS:
// optim_precond_lds_bytes.
template <int NN>
__global__ void __launch_bounds__(256) optim_precond_lds_kernel(OptDims D, OptBufs Bf, int it) {
  const int j = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int F = D.F, J = D.J, J3 = 3 * J;
  const double* P = (it & 1) ? Bf.P1 : Bf.P0;
  // false when this animal's PCG has finished (every wave: rz_at is a wave reduction).  The series blocks
  // ask only after issuing their staging loads, so the rz / pq reads share their memory round trip.
  auto pcg_alpha = [&](double& a) -> bool {
    a = 0;
    if (it < 0) return true;
    const double pq = Bf.pq[(size_t)b * (OPT_MAXIT + 1) + it];
    double rz2[2];
    rz_at_n<2>(D, Bf, b, {0, it}, rz2);  // pcg_done's two sums, the second also alpha's numerator
    if (!(rz2[0] > 0) || (it > 0 && !(rz2[1] > D.tol2 * rz2[0]))) return false;
    if (!(pq > 0)) return false;
    a = rz2[1] / pq;
    return true;
  };
  double alpha = 0;
  const size_t base = (size_t)b * D.NV;
  if (j == J) {  // the length variables: diagonal preconditioner, one thread per length
    if (!pcg_alpha(alpha)) return;
    __shared__ double srz[OPT_MAXL];
    const int NLa = D.fix ? 0 : D.NL;
    if (t < NLa) {
      const size_t o = base + D.NX + t;
      double r;
      if (it < 0) {
        Bf.d[o] = 0;
        r = -Bf.g[o];
      } else {
        Bf.d[o] += alpha * P[o];
        r = Bf.r[o] - alpha * Bf.q[o];
      }
      Bf.r[o] = r;
      const double z = r * Bf.pinvL[(size_t)b * OPT_MAXL + t];
      Bf.z[o] = z;
      srz[t] = r * z;
    }
    __syncthreads();
    if (t == 0) {
      double rz = 0;
      for (int k = 0; k < NLa; ++k) rz += srz[k];  // length order, as before
      Bf.rzJ[((size_t)b * (OPT_MAXIT + 1) + (it + 1)) * (J + 1) + j] = rz;
    }
    return;
  }
  OPT_PROF_BEGIN();
  constexpr int MN = 18 * NN;  // M and N doubles per frame
  constexpr int GB = 9 * NN;   // G (or H) doubles per frame
  const int K = opt_chunks(F, NN);
  const int L = (F + K - 1) / K;  // longest chunk
  extern __shared__ double lds_opt[];
  const int MNP = (F * MN + 127) / 128 * 128;  // M / N image padded to whole 1-KiB DMA instructions
  double* smn = lds_opt;                  // [F][MN]
  double* sr = smn + (size_t)MNP;         // [F][3] r
  double* su = sr + (size_t)F * 3;        // [F + 1][3] u, then v (+ pad frame)
  double* sz = su + (size_t)(F + 1) * 3;  // [F + 1][3] y^, then z^ / z (+ pad frame)
  double* sPhi = sz + (size_t)(F + 1) * 3;  // [K][NN][GB] G at each chunk's last NN frames (of chunk c-1)
  double* sPsi = sPhi + (size_t)K * NN * GB;  // [K][NN][GB] H at the first NN frames of chunk c+1
  double* sS = sPsi + (size_t)K * NN * GB;    // [K][NN][3] true incoming vectors, forward
  double* sT = sS + (size_t)K * NN * 3;       // [K][NN][3] backward
  const double* __restrict__ fb = Bf.fac + ((size_t)b * J + j) * F * OPT_FS;
  // Stage M / N and the chunk-boundary G / H blocks into LDS and update r / d for this series.  The
  // loads of all three are issued before any of their stores (one round trip to memory instead of one
  // per loop iteration: each trip is ~2 us when the factor was written on another XCD).
  // this thread's frames t and t + 256: their I blocks serve the staging and phase 4, and their G blocks
  // (phase 4) are loaded with the staging loads, so phase 4 waits on no global load of its own
  double Iv[2][9], Gv[2][GB];
  {
    constexpr int UG = (2 * OPT_MAXK * NN * GB + 255) / 256;    // G / H loads per thread
    const double* __restrict__ gg = Bf.g;
    const double* __restrict__ rin = Bf.r;
    const double* __restrict__ qq = Bf.q;
    const double* __restrict__ pp = P;
    double* __restrict__ dd = Bf.d;
    // r / d inputs of frames t and t + 256 (F <= 512 on this path: the LDS image caps F near 450)
    double a0v[2][3], a1v[2][3], a2v[2][3], a3v[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int f = t + 256 * h;
      if (f < F) {
        const size_t o = base + (size_t)f * J3 + 3 * j;
        const double* I = fb + (size_t)f * OPT_FS;
#pragma unroll
        for (int e = 0; e < 9; ++e) Iv[h][e] = I[e];
#pragma unroll
        for (int e = 0; e < GB; ++e) Gv[h][e] = I[9 + 18 * NN + e];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          if (it < 0) {
            a0v[h][i] = gg[o + i];
          } else {
            a0v[h][i] = dd[o + i];
            a1v[h][i] = pp[o + i];
            a2v[h][i] = rin[o + i];
            a3v[h][i] = qq[o + i];
          }
        }
      }
    }
    double gv[UG];
#pragma unroll
    for (int u2 = 0; u2 < UG; ++u2) {
      const int idx = t + 256 * u2;
      const bool back = idx >= K * NN * GB;
      const int u = back ? idx - K * NN * GB : idx;
      const int c = u / (NN * GB), k = (u / GB) % NN + 1, e = u % GB;
      gv[u2] = 0.0;
      if (idx < 2 * K * NN * GB) {
        if (!back && c >= 2) gv[u2] = fb[(size_t)(c * F / K - k) * OPT_FS + 9 + 18 * NN + e];
        if (back && c <= K - 3) gv[u2] = fb[(size_t)((c + 1) * F / K + k - 1) * OPT_FS + 9 + 27 * NN + e];
      }
    }
    // M / N: the contiguous copy of the series (Bf.mn) by LDS-DMA, 1 KiB per wave instruction (16 B per
    // lane); the last instruction's lanes past the end re-read the series' last 16 B into the pad
    {
      const char* src = reinterpret_cast<const char*>(Bf.mn + ((size_t)b * J + j) * F * MN);
      const int nbytes = F * MN * 8, nins = MNP * 8 / 1024;
      for (int ins = t >> 6; ins < nins; ins += 4) {
        const int off = min(ins * 1024 + (t & 63) * 16, nbytes - 16);
        __builtin_amdgcn_global_load_lds(MQ_LDS_GLOBAL(src + off), MQ_LDS_LOCAL(reinterpret_cast<char*>(smn) + ins * 1024),
                                         16, 0, 0);
      }
    }
    if (!pcg_alpha(alpha)) {  // nothing to do: let the LDS-DMA land before the workgroup's LDS is released
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      return;
    }
#pragma unroll
    for (int u2 = 0; u2 < UG; ++u2) {
      const int idx = t + 256 * u2;
      if (idx < 2 * K * NN * GB) sPhi[idx] = gv[u2];  // sPsi follows sPhi
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int f = t + 256 * h;
      if (f < F) {
        const size_t o = base + (size_t)f * J3 + 3 * j;
        double rr[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          double dn;
          if (it < 0) {
            dn = 0.0;
            rr[i] = -a0v[h][i];
          } else {
            dn = a0v[h][i] + alpha * a1v[h][i];
            rr[i] = a2v[h][i] - alpha * a3v[h][i];
          }
          dd[o + i] = dn;
          sr[3 * f + i] = rr[i];
        }
        su[3 * f] = Iv[h][0] * rr[0];
        su[3 * f + 1] = Iv[h][3] * rr[0] + Iv[h][4] * rr[1];
        su[3 * f + 2] = Iv[h][6] * rr[0] + Iv[h][7] * rr[1] + Iv[h][8] * rr[2];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA of M / N
  __syncthreads();
  OPT_PROF(1);
  const int cq = t >> 2;  // this lane's chunk in the substitutions
  const int a0 = cq * F / K, a1 = (cq + 1) * F / K;
  if (cq < K) lane_substitution<NN, false>(smn, su, sz, a0, a1 - a0, L, F, t);
  __syncthreads();
  OPT_PROF(2);
  // phase 3 (stitching): lane t < 3n owns row (k, r) of the incoming vectors and exchanges them through
  // LDS within the wave (LDS operations of a wave complete in order); the G rows do not depend on the
  // recurrence, so only one LDS round trip and n x 3 fmas sit on each step's chain
  if (t < 3 * NN) {
    const int k = t / 3 + 1, r = t % 3;
    for (int c = 1; c < K; ++c) {
      const int a = c * F / K;
      double v = sz[3 * (a - k) + r];
      if (c >= 2) {
        const double* G = sPhi + ((size_t)c * NN + k - 1) * GB + 3 * r;
        const double* Sp = sS + (size_t)(c - 1) * NN * 3;
#pragma unroll
        for (int jj = 0; jj < NN; ++jj) v += G[9 * jj] * Sp[3 * jj] + G[9 * jj + 1] * Sp[3 * jj + 1] + G[9 * jj + 2] * Sp[3 * jj + 2];
      }
      sS[((size_t)c * NN + k - 1) * 3 + r] = v;
    }
  }
  __syncthreads();
  OPT_PROF(3);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = t + 256 * h;
    if (f >= F) break;
    const int c = ((f + 1) * K + F - 1) / F - 1;
    double y[3] = {sz[3 * f], sz[3 * f + 1], sz[3 * f + 2]};
    if (c >= 1) {
      const double* G = Gv[h];
      const double* Sc = sS + (size_t)c * NN * 3;
#pragma unroll
      for (int k = 0; k < NN; ++k)
#pragma unroll
        for (int r = 0; r < 3; ++r)
          y[r] += G[9 * k + 3 * r] * Sc[3 * k] + G[9 * k + 3 * r + 1] * Sc[3 * k + 1] + G[9 * k + 3 * r + 2] * Sc[3 * k + 2];
    }
    const double* I = Iv[h];
    su[3 * f] = I[0] * y[0] + I[3] * y[1] + I[6] * y[2];
    su[3 * f + 1] = I[4] * y[1] + I[7] * y[2];
    su[3 * f + 2] = I[8] * y[2];
  }
  // phase 7's H blocks, in flight during the backward substitution
  double Hv[2][GB];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = t + 256 * h;
    if (f < F) {
#pragma unroll
      for (int e = 0; e < GB; ++e) Hv[h][e] = fb[(size_t)f * OPT_FS + 9 + 27 * NN + e];
    }
  }
  __syncthreads();
  OPT_PROF(4);
  if (cq < K) lane_substitution<NN, true>(smn, su, sz, a0, a1 - a0, L, F, t);
  __syncthreads();
  OPT_PROF(5);
  if (t < 3 * NN) {  // backward stitching, as the forward one
    const int k = t / 3 + 1, r = t % 3;
    for (int c = K - 2; c >= 0; --c) {
      const int e = (c + 1) * F / K;
      double v = sz[3 * (e + k - 1) + r];
      if (c <= K - 3) {
        const double* H = sPsi + ((size_t)c * NN + k - 1) * GB + 3 * r;
        const double* Tn = sT + (size_t)(c + 1) * NN * 3;
#pragma unroll
        for (int jj = 0; jj < NN; ++jj) v += H[9 * jj] * Tn[3 * jj] + H[9 * jj + 1] * Tn[3 * jj + 1] + H[9 * jj + 2] * Tn[3 * jj + 2];
      }
      sT[((size_t)c * NN + k - 1) * 3 + r] = v;
    }
  }
  __syncthreads();
  OPT_PROF(6);
  double rz = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = t + 256 * h;
    if (f >= F) break;
    const int c = ((f + 1) * K + F - 1) / F - 1;
    double z[3] = {sz[3 * f], sz[3 * f + 1], sz[3 * f + 2]};
    if (c <= K - 2) {
      const double* H = Hv[h];
      const double* Tc = sT + (size_t)c * NN * 3;
#pragma unroll
      for (int k = 0; k < NN; ++k)
#pragma unroll
        for (int r = 0; r < 3; ++r)
          z[r] += H[9 * k + 3 * r] * Tc[3 * k] + H[9 * k + 3 * r + 1] * Tc[3 * k + 1] + H[9 * k + 3 * r + 2] * Tc[3 * k + 2];
    }
    const size_t o = base + (size_t)f * J3 + 3 * j;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      Bf.r[o + i] = sr[3 * f + i];
      Bf.z[o + i] = z[i];
      rz += sr[3 * f + i] * z[i];
    }
  }
  __syncthreads();
  OPT_PROF(7);
  double* red = lds_opt;  // r / z are in registers or global memory now
  red[t] = rz;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) Bf.rzJ[((size_t)b * (OPT_MAXIT + 1) + (it + 1)) * (J + 1) + j] = red[0];
  OPT_PROF(8);
  OPT_PROF_END();
}

size_t optim_precond_lds_bytes(int F, int NN) {
  const size_t K = (size_t)opt_chunks(F, NN);
  const size_t mnp = ((size_t)F * 18 * NN + 127) / 128 * 128;
  const size_t n = mnp + (size_t)F * 3 + (size_t)(F + 1) * 6 + 2 * K * NN * 9 * NN + 2 * K * NN * 3;
  return std::max(n, (size_t)256) * sizeof(double);
}

// q = (H + lam diag(H)) p_it with p_it = z + beta p_{it-1} (computed here, written to P[it & 1]).
// Every load that does not depend on beta (the constraint list and this frame's length-Jacobian rows into
// LDS, the R row and damping diagonal into registers) is issued together with the rz reads, so the
// kernel waits on one memory round trip before the p loads instead of one per dependent step (the
// per-joint constraint loop used to load cons / lenJ from global memory on every trip round it).
__global__ void __launch_bounds__(OPT_THREADS) optim_matvec_kernel(OptDims D, OptBufs Bf, int it) {
  const int f = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int F = D.F, J = D.J, J3 = 3 * J, n = D.n, NL = D.NL;
  __shared__ double sp[2 * OPT_MAXN + 1][OPT_MAXJ * 3];
  __shared__ double spL[OPT_MAXL], stk[OPT_MAXL];
  __shared__ double slen[OPT_MAXL * 5];
  __shared__ int scons[2 * OPT_MAXL];
  __shared__ double red[OPT_THREADS];
  static_assert(2 * OPT_MAXL <= OPT_THREADS, "one constraint index per thread");
  const size_t base = (size_t)b * D.NV;
  const double* lf = Bf.lenJ + ((size_t)b * F + f) * NL * 5;
  for (int k = t; k < 5 * NL; k += OPT_THREADS) slen[k] = lf[k];
  if (t < 2 * NL) scons[t] = Bf.cons[t];
  double Rr[3] = {0.0, 0.0, 0.0}, dgo = 0.0;
  if (t < J3) {
    const int j = t / 3, comp = t % 3;
    const double* Rm = Bf.R + (((size_t)b * F + f) * J + j) * 6;
    const int ix[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
    Rr[0] = Rm[ix[comp][0]];
    Rr[1] = Rm[ix[comp][1]];
    Rr[2] = Rm[ix[comp][2]];
    dgo = Bf.diag[base + (size_t)f * J3 + t];
  }
  const double lam = Bf.ctl[2 * b];
  const double ssf = Bf.ssf[b];
  // z and the previous direction of the 2n + 1 frames this block couples, loaded before the done check too
  const double* Pp = (it & 1) ? Bf.P0 : Bf.P1;
  constexpr int NW = 2 * OPT_MAXN + 1;
  double zv[NW], pv[NW], zl = 0.0, pl = 0.0;
  if (t < J3) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int ff = f + w - n;
      zv[w] = pv[w] = 0.0;
      if (w <= 2 * n && ff >= 0 && ff < F) {
        const size_t o = base + (size_t)ff * J3 + t;
        zv[w] = Bf.z[o];
        if (it > 0) pv[w] = Pp[o];
      }
    }
  }
  if (t < NL && !D.fix) {
    const size_t o = base + D.NX + t;
    zl = Bf.z[o];
    if (it > 0) pl = Pp[o];
  }
  // pcg_done and beta from the same three rz reads
  double rz3[3];
  rz_at_n<3>(D, Bf, b, {0, it, it > 0 ? it - 1 : 0}, rz3);
  const double r0 = rz3[0];
  const double ri = it == 0 ? r0 : rz3[1];
  const double rim = it == 0 ? 1.0 : rz3[2];
  if (!(r0 > 0) || (it > 0 && !(ri > D.tol2 * r0))) return;  // pcg_done: the whole block
  const double beta = it == 0 ? 0.0 : ri / rim;
  double* Pc = (it & 1) ? Bf.P1 : Bf.P0;
  if (t < J3) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int ff = f + w - n;
      if (w > 2 * n || ff < 0 || ff >= F) continue;
      const double p = it == 0 ? zv[w] : zv[w] + beta * pv[w];
      sp[w][t] = p;
      if (w == n) Pc[base + (size_t)ff * J3 + t] = p;
    }
  }
  if (t < NL) {
    double p = 0;
    if (!D.fix) {
      p = it == 0 ? zl : zl + beta * pl;
      if (f == 0) Pc[base + D.NX + t] = p;
    }
    spL[t] = p;
  }
  __syncthreads();
  const double* p0 = sp[n];
  if (t < NL) {
    const double* l = slen + 5 * t;
    const int a = scons[2 * t], c2 = scons[2 * t + 1];
    const double tk = l[0] * (p0[3 * a] - p0[3 * c2]) + l[1] * (p0[3 * a + 1] - p0[3 * c2 + 1]) +
                      l[2] * (p0[3 * a + 2] - p0[3 * c2 + 2]) + l[3] * spL[t];
    stk[t] = tk;
    if (!D.fix) Bf.qLf[((size_t)b * F + f) * NL + t] = l[3] * tk;
  }
  __syncthreads();
  double pq = 0;
  if (t < J3) {
    const int j = t / 3, comp = t % 3;
    double q = Rr[0] * p0[3 * j] + Rr[1] * p0[3 * j + 1] + Rr[2] * p0[3 * j + 2];
    for (int k = 0; k < NL; ++k) {
      const int a = scons[2 * k], c2 = scons[2 * k + 1];
      if (a != j && c2 != j) continue;
      const double gk = slen[5 * k + comp];
      q += (a == j ? gk : -gk) * stk[k];
    }
    if (F > n) {
      const double s2 = ssf * ssf;
      for (int df = -n; df <= n; ++df) {
        const int ff = f + df;
        if (ff < 0 || ff >= F) continue;
        q += s2 * dtd(f, ff, F, n, D.c) * sp[df + n][t];
      }
    }
    const size_t o = base + (size_t)f * J3 + t;
    q += lam * damp_of(dgo) * p0[t];
    Bf.q[o] = q;
    pq = p0[t] * q;
  }
  const double tot = block_sum(pq, red);
  if (t == 0) Bf.pqF[(size_t)b * F + f] = tot;
}

// Length part of q and the full p.q (fixed-order reductions over frames).  (Folding this into the matvec's
// last-arriving block needs a device-scope release per block; the L2 write-back that implies made the
// matvec 4x slower, profiles/r04p_*.)
__global__ void __launch_bounds__(OPT_RTHREADS) optim_reduce_pq_kernel(OptDims D, OptBufs Bf, int it) {
  const int b = blockIdx.x, t = threadIdx.x;
  __shared__ double red[OPT_RTHREADS];
  const double* P = (it & 1) ? Bf.P1 : Bf.P0;
  const size_t base = (size_t)b * D.NV;
  __shared__ double part[OPT_RCH][OPT_MAXL];
  double s = 0;
  // the partial loads go out before the "PCG finished" check (stale values are then only discarded)
  for (int f = t; f < D.F; f += OPT_RTHREADS) s += Bf.pqF[(size_t)b * D.F + f];
  if (!D.fix) len_partials(D, Bf.qLf + (size_t)b * D.F * D.NL, nullptr, part, nullptr, t);
  if (pcg_done(D, Bf, b, it)) return;  // the whole block
  __syncthreads();
  if (!D.fix && t < D.NL) {
    double qL = len_combine(part, t);
    const size_t o = base + D.NX + t;
    qL += Bf.ctl[2 * b] * damp_of(Bf.diag[o]) * P[o];
    Bf.q[o] = qL;
    s += P[o] * qL;
  }
  const double tot = block_sum<OPT_RTHREADS>(s, red);
  if (t == 0) Bf.pq[(size_t)b * (OPT_MAXIT + 1) + it] = tot;
}

__global__ void optim_axpy_kernel(const double* x, const double* d, double* xt, int NX, int NV, int B, int fix) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)B * NV) return;
  const int k = (int)(i % NV);
  xt[i] = (fix && k >= NX) ? x[i] : x[i] + d[i];
}

// Predicted cost reduction of the Gauss-Newton model for the step d (one workgroup per batch element):
// pred = -g.d - d.H.d / 2.  The PCG iterate solves (H + lam Dm) d = -g over a Krylov space that holds d, so
// d.(H + lam Dm).d = -g.d and pred = (-g.d + lam d.Dm.d) / 2 from two dot products (fixed lengths excluded).
__global__ __launch_bounds__(256) void optim_pred_kernel(OptDims D, OptBufs Bf, double* pred) {
  const int b = blockIdx.x;
  const int nv = D.fix ? D.NX : D.NV;
  const size_t o = (size_t)b * D.NV;
  double gd = 0.0, dd = 0.0;
  for (int k = threadIdx.x; k < nv; k += 256) {
    const double dk = Bf.d[o + k];
    gd += Bf.g[o + k] * dk;
    dd += damp_of(Bf.diag[o + k]) * dk * dk;
  }
  __shared__ double sg[256], sd[256];
  sg[threadIdx.x] = gd;
  sd[threadIdx.x] = dd;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      sg[threadIdx.x] += sg[threadIdx.x + w];
      sd[threadIdx.x] += sd[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) pred[b] = 0.5 * (-sg[0] + Bf.ctl[2 * b] * sd[0]);
}

__global__ void optim_accept_kernel(double* x, const double* xt, const double* ctl, int NV, int B) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)B * NV) return;
  if (ctl[2 * (i / NV) + 1] != 0.0) x[i] = xt[i];
}

}  // namespace

int g_optim_precond_lds = 1;
// LM inner-solve cap and stop rule (MQ_TUNE_OPTIM_PCG_ITERS / MQ_TUNE_OPTIM_STOP).  On clean synthetic 2D
// (config 4) 20 PCG iterations and scipy's first-small-step stop landed within 3e-4 of scipy's cost
// (tools/optim_probe.py).  On ViT-derived 2D (the marker-scene oracle chain, tools/optim_parity_probe.py,
// profiles/r04h_optim_parity_probe_stop_rules.log) that stopped up to 1.0 % above scipy's cost and 34 mm (p99)
// from the converged solution; 40 iterations with the test required on two accepted steps in a row land
// within 1e-4 of scipy's cost and closer to the converged solution than scipy's own ftol 1e-3 stop.
int g_optim_pcg_iters = 40;
int g_optim_stop = 6;        // stop rule bits: 1 model-agreement ratio > 0.25 (scipy trf), 2 two steps in a row,
                             // 4 the test at ftol / 2 (tools/optim_parity_probe.py on the marker scenes of seeds 7-9:
                             // ftol alone stopped up to 1.5 % above scipy's cost on one; ftol / 2 at or below it on all,
                             // profiles/r04r_optim_parity_probe_seeds.log)

size_t optim_workspace_bytes(int B, int F, int J, int NL) {
  const size_t NV = (size_t)F * J * 3 + NL;
  size_t n = 0;
  n += (size_t)B * NV * 9;                       // g diag d r z P0 P1 q xt
  n += (size_t)B * F * J * 6;                    // R
  n += (size_t)B * F * NL * 5;                   // lenJ
  n += (size_t)B * F * 2;                        // costF pqF
  n += (size_t)B * F * NL;                       // qLf
  n += (size_t)B * J * F * OPT_FS + (size_t)B * OPT_MAXL;  // fac pinvL
  n += (size_t)B * J * F * 18 * OPT_MAXN + 2;               // mn (+ 16-B alignment)
  n += (size_t)B * (OPT_MAXIT + 1) * (J + 2);    // rzJ, pq
  n += (size_t)B * 5;                            // cost, cost_t + pred (2), ctl(2)
  n += (size_t)NL + 2 + B;                       // constraint pairs (int32), ssf
  return n * sizeof(double);
}

// Host driver.  x: device (B, NV) in/out.  cons/ssf/stats: host.  ws: device workspace of
// optim_workspace_bytes().  stats[b*4 + {0,1,2,3}] = initial cost, final cost, LM iterations, status
// (1 ftol, 2 max_iter, 3 damping overflow).
int optim_points(const double* cams, int C, const double* p2d, double* x, int B, int F, int J, const int* cons_host,
                 int n_strong, int n_weak, const double* ssf_host, double scale_length, double scale_length_weak,
                 double rp, int loss, int n_deriv, int fix_lengths, int max_iter, double ftol, void* ws,
                 double* stats, hipStream_t s) {
  const int NL = n_strong + n_weak;
  if (B <= 0 || F <= 0 || J <= 0) return 0;
  if (J > OPT_MAXJ || NL > OPT_MAXL || C > OPT_MAXC || C < 1 || n_deriv < 1 || n_deriv > OPT_MAXN) return -2;
  OptDims D{};
  D.B = B;
  D.C = C;
  D.F = F;
  D.J = J;
  D.NL = NL;
  D.nS = n_strong;
  D.fix = fix_lengths;
  D.n = n_deriv;
  D.loss = loss;
  D.NX = F * J * 3;
  D.NV = D.NX + NL;
  D.rp = rp;
  D.s_len = scale_length;
  D.s_len_weak = scale_length_weak;
  D.tol2 = 1e-10;
  {  // np.diff(., n) coefficients: (-1)^(n-m) C(n, m)
    int binom = 1;
    for (int m = 0; m <= n_deriv; ++m) {
      D.c[m] = (((n_deriv - m) & 1) ? -1.0 : 1.0) * binom;
      binom = binom * (n_deriv - m) / (m + 1);
    }
  }
  const size_t NVB = (size_t)B * D.NV;
  double* w = static_cast<double*>(ws);
  OptBufs Bf{};
  auto take = [&](size_t cnt) {
    double* p = w;
    w += cnt;
    return p;
  };
  Bf.g = take(NVB);
  Bf.diag = take(NVB);
  Bf.d = take(NVB);
  Bf.r = take(NVB);
  Bf.z = take(NVB);
  Bf.P0 = take(NVB);
  Bf.P1 = take(NVB);
  Bf.q = take(NVB);
  double* xt = take(NVB);
  Bf.R = take((size_t)B * F * J * 6);
  Bf.lenJ = take((size_t)B * F * NL * 5);
  Bf.costF = take((size_t)B * F);
  Bf.pqF = take((size_t)B * F);
  Bf.qLf = take((size_t)B * F * NL);
  Bf.fac = take((size_t)B * J * F * OPT_FS);
  Bf.mn = take((size_t)B * J * F * 18 * OPT_MAXN + 2);
  if (reinterpret_cast<uintptr_t>(Bf.mn) & 15) ++Bf.mn;  // 16-B aligned for the LDS-DMA
  Bf.pinvL = take((size_t)B * OPT_MAXL);
  Bf.rzJ = take((size_t)B * (OPT_MAXIT + 1) * (J + 1));
  Bf.pq = take((size_t)B * (OPT_MAXIT + 1));
  Bf.cost = take(B);
  double* cost_t = take(2 * (size_t)B);   // trial costs, then the predicted reductions (one copy back)
  double* pred_d = cost_t + B;
  double* ctl = take(2 * (size_t)B);
  Bf.ctl = ctl;
  Bf.cams = cams;
  Bf.p2d = p2d;
  // small host-side inputs go to the device through the workspace tail
  int* cons_d = reinterpret_cast<int*>(take((NL * 2 + 1) / 2 + 1));
  double* ssf_d = take(B);
  Bf.cons = cons_d;
  Bf.ssf = ssf_d;
  if (hipMemcpyAsync(cons_d, cons_host, sizeof(int) * 2 * NL, hipMemcpyHostToDevice, s) != hipSuccess) return -3;
  if (hipMemcpyAsync(ssf_d, ssf_host, sizeof(double) * B, hipMemcpyHostToDevice, s) != hipSuccess) return -3;

  const int npcg = std::max(1, std::min(g_optim_pcg_iters, OPT_MAXIT));
  const dim3 gridFB(F, B);
  const int ew_blocks = (int)((NVB + 255) / 256);
  std::vector<double> lam(B, 1e-3), cost(B), costt(2 * B), hctl(2 * B, 0.0);
  std::vector<int> active(B, 1), iters(B, 0), status(B, 2), small(B, 0);
  const bool stop_ratio = (g_optim_stop & 1) != 0, stop_twice = (g_optim_stop & 2) != 0;
  const double ftol_test = (g_optim_stop & 4) ? 0.5 * ftol : ftol;

  // preconditioner step: series staged in LDS when they fit (every clip up to ~450 frames at n = 2)
  const size_t lds_b = optim_precond_lds_bytes(F, D.n);
  const size_t fac_lds_b = optim_factor_lds_bytes(F, D.n);
  const bool fac_lds = g_optim_precond_lds && fac_lds_b + 512 <= 160 * 1024;  // + the static constraint list
  // the chunked LDS apply reads the chunk responses that only the LDS factor kernel writes
  const bool use_lds = fac_lds && lds_b + 1024 <= 160 * 1024 && F <= 512;  // (two frames per thread)
  auto precond = [&](int it) {
    if (!use_lds) {
      hipLaunchKernelGGL(optim_precond_kernel, dim3(B), dim3(64), 0, s, D, Bf, it);
      return;
    }
    const dim3 grid(J + 1, B);
    if (D.n == 1) hipLaunchKernelGGL(optim_precond_lds_kernel<1>, grid, dim3(256), lds_b, s, D, Bf, it);
    else if (D.n == 2) hipLaunchKernelGGL(optim_precond_lds_kernel<2>, grid, dim3(256), lds_b, s, D, Bf, it);
    else hipLaunchKernelGGL(optim_precond_lds_kernel<3>, grid, dim3(256), lds_b, s, D, Bf, it);
  };
  // factorization: the LDS kernel whenever the series fits (its footprint is smaller than the apply's)
  auto factor = [&]() {
    if (!fac_lds) {
      hipLaunchKernelGGL(optim_factor_kernel, dim3(B), dim3(64), 0, s, D, Bf);
      return;
    }
    const dim3 grid(J + 1, B);
    if (D.n == 1) hipLaunchKernelGGL(optim_factor_lds_kernel<1>, grid, dim3(256), fac_lds_b, s, D, Bf);
    else if (D.n == 2) hipLaunchKernelGGL(optim_factor_lds_kernel<2>, grid, dim3(256), fac_lds_b, s, D, Bf);
    else hipLaunchKernelGGL(optim_factor_lds_kernel<3>, grid, dim3(256), fac_lds_b, s, D, Bf);
  };
  if (use_lds || fac_lds) {
    static std::atomic<unsigned> attr{0};
    if (first_on_device(attr)) {
      const int mx = 160 * 1024;
      // (dynamic + static LDS may not exceed the CU's 160 KB, or the call fails and leaves a sticky error;
      // both kernels keep under 1 KB of static LDS)
      (void)hipFuncSetAttribute((const void*)optim_precond_lds_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 1024);
      (void)hipFuncSetAttribute((const void*)optim_precond_lds_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 1024);
      (void)hipFuncSetAttribute((const void*)optim_precond_lds_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 1024);
      (void)hipFuncSetAttribute((const void*)optim_factor_lds_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 512);
      (void)hipFuncSetAttribute((const void*)optim_factor_lds_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 512);
      (void)hipFuncSetAttribute((const void*)optim_factor_lds_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, mx - 512);
    }
  }
  auto eval = [&](const double* xx, int mode, double* out) {
    hipLaunchKernelGGL(optim_eval_kernel, gridFB, dim3(OPT_THREADS), 0, s, D, Bf, xx, mode);
    hipLaunchKernelGGL(optim_reduce_kernel, dim3(B), dim3(OPT_RTHREADS), 0, s, D, Bf, out, mode);
  };
  eval(x, 0, Bf.cost);
  if (hipMemcpyAsync(cost.data(), Bf.cost, sizeof(double) * B, hipMemcpyDeviceToHost, s) != hipSuccess) return -3;
  if (hipStreamSynchronize(s) != hipSuccess) return -3;
  for (int b = 0; b < B; ++b) {
    stats[4 * b + 0] = cost[b];
    if (!(cost[b] > 0)) {  // already exact (or NaN input): nothing to do
      active[b] = 0;
      status[b] = 1;
    }
  }
  for (int iter = 0; iter < max_iter; ++iter) {
    bool any = false;
    for (int b = 0; b < B; ++b) any |= active[b] != 0;
    if (!any) break;
    for (int b = 0; b < B; ++b) {
      hctl[2 * b] = lam[b];
      hctl[2 * b + 1] = 0;
    }
    if (hipMemcpyAsync(ctl, hctl.data(), sizeof(double) * 2 * B, hipMemcpyHostToDevice, s) != hipSuccess) return -3;
    (void)hipMemsetAsync(Bf.rzJ, 0, sizeof(double) * (size_t)B * (OPT_MAXIT + 1) * (J + 2), s);
    factor();
    precond(-1);
    for (int it = 0; it < npcg; ++it) {
      hipLaunchKernelGGL(optim_matvec_kernel, gridFB, dim3(OPT_THREADS), 0, s, D, Bf, it);
      hipLaunchKernelGGL(optim_reduce_pq_kernel, dim3(B), dim3(OPT_RTHREADS), 0, s, D, Bf, it);
      precond(it);
    }
    hipLaunchKernelGGL(optim_axpy_kernel, dim3(ew_blocks), dim3(256), 0, s, x, Bf.d, xt, D.NX, D.NV, B, D.fix);
    if (stop_ratio) hipLaunchKernelGGL(optim_pred_kernel, dim3(B), dim3(256), 0, s, D, Bf, pred_d);
    eval(xt, 1, cost_t);
    if (hipMemcpyAsync(costt.data(), cost_t, sizeof(double) * (stop_ratio ? 2 * B : B), hipMemcpyDeviceToHost, s) !=
        hipSuccess)
      return -3;
    if (hipStreamSynchronize(s) != hipSuccess) return -3;
    bool accepted_any = false;
    for (int b = 0; b < B; ++b) {
      if (!active[b]) continue;
      iters[b]++;
      if (costt[b] < cost[b]) {  // accept
        const double dF = cost[b] - costt[b];
        hctl[2 * b + 1] = 1;
        accepted_any = true;
        // scipy's ftol test on an accepted step; with stop bit 1 also its model-agreement condition
        // (trf: dF < ftol F and ratio > 0.25), with bit 2 on two accepted steps in a row
        bool ft = dF < ftol_test * cost[b];
        if (ft && stop_ratio) ft = dF > 0.25 * costt[B + b];
        small[b] = ft ? small[b] + 1 : 0;
        if (small[b] >= (stop_twice ? 2 : 1)) {
          active[b] = 0;
          status[b] = 1;
        }
        cost[b] = costt[b];
        lam[b] = std::max(lam[b] / 3.0, 1e-12);
      } else {
        small[b] = 0;  // "two accepted steps in a row": a rejected step in between breaks the run
        lam[b] *= 4.0;
        if (lam[b] > 1e12) {
          active[b] = 0;
          status[b] = 3;
        }
      }
    }
    if (accepted_any) {
      if (hipMemcpyAsync(ctl, hctl.data(), sizeof(double) * 2 * B, hipMemcpyHostToDevice, s) != hipSuccess) return -3;
      hipLaunchKernelGGL(optim_accept_kernel, dim3(ew_blocks), dim3(256), 0, s, x, xt, ctl, D.NV, B);
      eval(x, 0, Bf.cost);
    }
  }
  if (hipStreamSynchronize(s) != hipSuccess) return -3;
#ifdef OPT_PROFILE
  {
    unsigned long long h[9];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_opt_prof), sizeof(h));
    const double n = h[0] ? (double)h[0] : 1.0;
    fprintf(stderr, "opt_prof blocks %llu us/block:", h[0]);
    for (int k = 1; k < 9; ++k) fprintf(stderr, " %.2f", h[k] / n / 100.0);  // wall clock: 100 MHz
    fprintf(stderr, "\n");
  }
#endif
  for (int b = 0; b < B; ++b) {
    stats[4 * b + 1] = cost[b];
    stats[4 * b + 2] = iters[b];
    stats[4 * b + 3] = status[b];
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace mq
