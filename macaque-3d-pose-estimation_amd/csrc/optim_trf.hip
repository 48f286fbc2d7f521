// optim_points, scipy-faithful solver (row a16; the parity default since ABI 7).
//
// The reference refines 3D points with scipy.optimize.least_squares(method='trf', jac_sparsity=...,
// loss='linear', ftol=1e-3) (cameras.py:1166-1180).  Without bounds and with a sparse Jacobian that is
// scipy 1.15.3's trf_no_bounds with tr_solver='lsmr' (optimize/_lsq/trf.py:401-540), restated step for step:
//   * J and g = J^T f at every accepted x; gtol / max_nfev tests at the top of the loop;
//   * the damping of the lsmr step from the 1-D quadratic along -g inside the trust region (regularize);
//   * gn = lsmr(J, f, damp) with atol = btol = 1e-6, conlim 1e8, maxiter min(m, n)  (sparse/linalg lsmr.py);
//   * S = orth([g, gn]), B_S = (J S)^T (J S), g_S = S^T g; solve_trust_region_2d; update_tr_radius;
//     check_termination (ftol with the ratio > 0.25 condition, xtol 1e-8).
// oracle/trf.py restates the same algorithm in this file's phase order and is pinned bit for bit against scipy
// (tests/test_oracle_trf.py).  What differs here: the Jacobian is analytic (scipy: 2-point differences, which
// move scipy's own answer by < 0.2 mm on the marker scenes, profiles/r05*), and the reductions run in a fixed
// order of their own (so floating-point results are not scipy's bits).
//
// Work decomposition (one animal = one independent problem; B animals per call, batched in every launch):
//   * a workgroup owns a block of FB (<= 4) consecutive frames of one animal: its reprojection rows (camera x
//     joint x {u, v}), smoothness rows (np.diff order n, row i at frame i) and limb-length rows (m space), and
//     its 3 J parameters per frame (n space); the length variables belong to block 0;
//   * lsmr is two launches per iteration: phase 1 (u = J v - alpha u; the previous iteration's recurrences and
//     the x / h / hbar updates), phase 2 (the previous iteration's stop test, then v = J^T u - beta v).  Every
//     workgroup reduces the norms it needs from the previous launch's per-block partials itself, in the same
//     fixed order, so every workgroup holds the same scalars bit for bit and no launch waits on another
//     workgroup.  The host checks the per-animal done flags every few iterations;
//   * the trust-region logic (2x2 subproblem, radius, termination) runs on the host from the partials.
#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <initializer_list>
#include <limits>
#include <vector>

#include "camera.hpp"
#include "common.hpp"
#include "optim_dev.hpp"

namespace mq {
namespace {

constexpr int TRF_THREADS = 256;
constexpr int TRF_FB = 4;  // frames per workgroup (at most; fewer when a block's rows would not fit in LDS)
// (5 measured slower on config 4: 23.1 vs 20.9 ms for 240 instead of 300 workgroups; profiles/r06k_*)
constexpr int TRF_MAXJ = 32, TRF_MAXL = 64, TRF_MAXN = 3;
static_assert(TRF_FB * TRF_MAXJ * 3 <= 2 * TRF_THREADS, "a block's parameters: at most two per thread");
constexpr int TRF_NS = 24;  // lsmr state doubles per slot

// -DTRF_PROFILE builds (tools only, never the shipped library): wall-clock time per phase of the two lsmr
// kernels, block TRF_PROFILE_BLOCK (default 0) of animal 0, summed over launches and printed at the end of
// optim_points_trf.
#ifdef TRF_PROFILE
__device__ unsigned long long g_trf_prof[2][12];
#define TRF_PROF_BEGIN() \
  unsigned long long prof_t[12]; \
  prof_t[0] = wall_clock64()
#ifndef TRF_PROFILE_BLOCK
#define TRF_PROFILE_BLOCK 0
#endif
#define TRF_PROF(k) prof_t[k] = wall_clock64()
#define TRF_PROF_END(kern, last)                                                       \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x == TRF_PROFILE_BLOCK && blockIdx.y == 0) {       \
      for (int k = 1; k <= last; ++k) atomicAdd(&g_trf_prof[kern][k], prof_t[k] - prof_t[k - 1]); \
      atomicAdd(&g_trf_prof[kern][0], 1ull);                                           \
    }                                                                                   \
  } while (0)
#else
#define TRF_PROF_BEGIN() (void)0
#define TRF_PROF(k) (void)0
#define TRF_PROF_END(kern, last) (void)0
#endif

struct TrfDims {
  int B, C, F, J, NL, nS, fix, n, loss;
  int NX, NV, MR, MRrep, NB, FB;
  int NBV;  // slots of the J^T partials: NB + 1 when the length variables have a workgroup of their own, else NB
  double rp, s_len, s_len_weak;
  double c[TRF_MAXN + 1];
  double atol, btol, ctol;
};

struct TrfBufs {
  const double* cams;
  const double* p2d;
  const int* cons;
  const int* jadj;  // per joint the constraints touching it, ascending l: [J + 1] offsets, then codes 2 l + (second end)
  const double* ssf;
  const int* act;  // [B] the animal takes part in this launch
  int* done;       // [B] lsmr finished
  double *fres, *ftr, *Jrep, *lenJ;
  double *g, *u, *vraw, *vn, *h, *hbar, *xl, *s1, *s2;
  double* fpart;  // [B][NB][4]: sum r^2 at x, sum r^2 at the trial point, rows (host-mapped)
  double* fL;     // [B][NB][NL]: sum over the block's frames of dL * r_len at x
  double* upart;  // [2][B][NB]
  double* vpart;  // [2][B][NBV][2]: sum v^2, max |v| (slot NB, if NBV = NB + 1: the length variables)
  double* xpart;  // [2][B][NB]
  double* Lpart;  // [B][NB][NL]
  double* npart;  // [B][NB][TRF_NPF] (host-mapped)
  double* jpart;  // [B][NB][4] (host-mapped)
  double* gpart;  // [B][NBV][2]: |g|^2, max |g| (host-mapped)
  double* hitn;   // [B]: lsmr's final iteration count (host-mapped)
  int* hdone;     // [B]: copy of done (host-mapped), polled by the host between chunks
  double* st;     // [2][B][TRF_NS]
  double* lctl;   // [B][4]: damp, normb, maxiter, final lsmr itn
  double* coef;   // [B][4]
};

// Sum over the workgroup; every thread returns the same bits (xor butterflies add the same two values,
// commuted, and the wave sums combine in one fixed order).
__device__ __forceinline__ double block_sum_all(double v, double* red) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v += __shfl_xor(v, m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__device__ __forceinline__ double block_max_all(double v, double* red) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) v = fmax(v, __shfl_xor(v, m));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  return s;
}

// sum_i p[i * stride] over i < count, the same value in every thread of every workgroup that asks
__device__ __forceinline__ double reduce_parts(const double* __restrict__ p, int count, int stride, double* red) {
  double v = 0.0;
  for (int i = threadIdx.x; i < count; i += TRF_THREADS) v += p[(size_t)i * stride];
  return block_sum_all(v, red);
}

// scipy.sparse.linalg._isolve.lsqr._sym_ortho (np.sign(0) = 0)
__device__ __forceinline__ double sgn0(double a) { return a > 0 ? 1.0 : (a < 0 ? -1.0 : 0.0); }
__device__ __forceinline__ void sym_ortho(double a, double b, double& c, double& s, double& r) {
  if (b == 0) {
    c = sgn0(a);
    s = 0;
    r = fabs(a);
  } else if (a == 0) {
    c = 0;
    s = sgn0(b);
    r = fabs(b);
  } else if (fabs(b) > fabs(a)) {
    const double tau = a / b;
    s = sgn0(b) / sqrt(1 + tau * tau);
    c = s * tau;
    r = b / s;
  } else {
    const double tau = b / a;
    c = sgn0(a) / sqrt(1 + tau * tau);
    s = c * tau;
    r = a / c;
  }
}


// Global -> LDS staging with every load of a thread issued before its LDS stores (a plain copy loop waits on
// each load before the next iteration's: one memory round trip per element a thread copies).  stage16: 16-B
// loads, src and dst 16-B aligned, n even; stage8: 8-B loads, any alignment.
typedef double trf_d2 __attribute__((ext_vector_type(2)));
template <int U = 8>
__device__ __forceinline__ void stage16(double* __restrict__ dst, const double* __restrict__ src, int n) {
  const int n2 = n >> 1;
  const trf_d2* s2 = reinterpret_cast<const trf_d2*>(src);
  trf_d2* d2 = reinterpret_cast<trf_d2*>(dst);
  for (int base = 0; base < n2; base += TRF_THREADS * U) {
    trf_d2 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // (an out-of-range lane re-reads element 0: no conditional array writes)
      const int i = base + u * TRF_THREADS + (int)threadIdx.x;
      r[u] = s2[i < n2 ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * TRF_THREADS + (int)threadIdx.x;
      if (i < n2) d2[i] = r[u];
    }
  }
}
template <int U = 8>
__device__ __forceinline__ void stage8(double* __restrict__ dst, const double* __restrict__ src, int n) {
  for (int base = 0; base < n; base += TRF_THREADS * U) {
    double r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * TRF_THREADS + (int)threadIdx.x;
      r[u] = src[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * TRF_THREADS + (int)threadIdx.x;
      if (i < n) dst[i] = r[u];
    }
  }
}

// Several copies at once, in two halves: load() issues the first U8 * TRF_THREADS doubles of s8 (8-B loads) and
// U* * TRF_THREADS 16-B vectors of a, b, c into registers; store() writes them to LDS, then copies whatever is
// left of a larger array (more joints or cameras than the sizes chosen) in further rounds.  Everything a
// kernel loads goes between the two halves, so the launch waits on one memory round trip (a load whose value
// is stored or summed right away costs a round trip of its own: the wait sits before the use).  U = 0 leaves a
// segment to the further rounds alone.
struct StageSeg {
  double* dst;
  const double* src;
  int n;
};
template <int U8, int UA, int UB, int UC>
struct Stager {
  StageSeg s8, a, b, c;
  double r8[U8 > 0 ? U8 : 1];
  trf_d2 ra[UA > 0 ? UA : 1], rb[UB > 0 ? UB : 1], rc[UC > 0 ? UC : 1];
  __device__ __forceinline__ void load() {
    const int t = threadIdx.x;
    const int na = a.n >> 1, nb = b.n >> 1, nc = c.n >> 1;
    const trf_d2 *sa = reinterpret_cast<const trf_d2*>(a.src), *sb = reinterpret_cast<const trf_d2*>(b.src),
                 *sc = reinterpret_cast<const trf_d2*>(c.src);
#pragma unroll
    for (int u = 0; u < U8; ++u) {  // (an out-of-range lane re-reads element 0: no conditional loads)
      const int i = u * TRF_THREADS + t;
      r8[u] = s8.src[i < s8.n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int i = u * TRF_THREADS + t;
      ra[u] = sa[i < na ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = u * TRF_THREADS + t;
      rb[u] = sb[i < nb ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < UC; ++u) {
      const int i = u * TRF_THREADS + t;
      rc[u] = sc[i < nc ? i : 0];
    }
  }
  __device__ __forceinline__ void store() {
    const int t = threadIdx.x;
    const int na = a.n >> 1, nb = b.n >> 1, nc = c.n >> 1;
#pragma unroll
    for (int u = 0; u < U8; ++u) {
      const int i = u * TRF_THREADS + t;
      if (i < s8.n) s8.dst[i] = r8[u];
    }
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int i = u * TRF_THREADS + t;
      if (i < na) reinterpret_cast<trf_d2*>(a.dst)[i] = ra[u];
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int i = u * TRF_THREADS + t;
      if (i < nb) reinterpret_cast<trf_d2*>(b.dst)[i] = rb[u];
    }
#pragma unroll
    for (int u = 0; u < UC; ++u) {
      const int i = u * TRF_THREADS + t;
      if (i < nc) reinterpret_cast<trf_d2*>(c.dst)[i] = rc[u];
    }
    constexpr int D8 = U8 * TRF_THREADS, DA = 2 * UA * TRF_THREADS, DB = 2 * UB * TRF_THREADS,
                  DC = 2 * UC * TRF_THREADS;
    if (s8.n > D8) stage8(s8.dst + D8, s8.src + D8, s8.n - D8);
    if (a.n > DA) stage16(a.dst + DA, a.src + DA, a.n - DA);
    if (b.n > DB) stage16(b.dst + DB, b.src + DB, b.n - DB);
    if (c.n > DC) stage16(c.dst + DC, c.src + DC, c.n - DC);
  }
};

// np.diff coefficient m of the kernel arguments by constant indices (a runtime index into the by-value
// TrfDims made the compiler copy it to scratch: a memory round trip per use)
__device__ __forceinline__ double dcoef(const TrfDims& D, int m) {
  return m == 0 ? D.c[0] : (m == 1 ? D.c[1] : (m == 2 ? D.c[2] : D.c[3]));
}

// frame of flat row i in a block of rows `per` wide (i < TRF_FB * per): comparisons, no integer division
__device__ __forceinline__ int trf_frame_of(int i, int per) {
  int fl = 0;
#pragma unroll
  for (int k = 1; k < TRF_FB; ++k) fl += i >= k * per;
  return fl;
}

// lsmr state slot
enum {
  S_ALPHABAR, S_RHO, S_RHOBAR, S_CBAR, S_SBAR, S_ZETABAR, S_ZETA, S_BETADD, S_BETAD, S_RHODOLD, S_TAUTILDEOLD,
  S_THETATILDE, S_D, S_NORMA2, S_MAXRBAR, S_MINRBAR, S_ITN, S_NORMR, S_NORMAR, S_NORMA, S_CONDA,
  S_CHAT, S_SHAT, S_ALPHAHAT  // sym_ortho(alphabar, damp) of the next iteration (depends on neither norm)
};
static_assert(S_ALPHAHAT < TRF_NS, "lsmr state slot");

// ---------------------------------------------------------------------------------------------------------
// Residuals (and, mode 1, the Jacobian) at x for the block's frames.  fout: m vector [B][F][MR]:
//   [(j C + c) 2 + comp] reprojection (0 where the coordinate is NaN), [MRrep + 3 j + k] smoothness (frames
//   f < F - n), [MRrep + 3 J + l] limb lengths.  Partials: sum r^2 (slot 0 at x / 1 at a trial point), rows.
__global__ void __launch_bounds__(TRF_THREADS) trf_eval_kernel(TrfDims D, TrfBufs Bf, const double* __restrict__ x,
                                                              double* __restrict__ fout, int mode) {
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  if (!Bf.act[b]) return;
  const int J = D.J, C = D.C, J3 = 3 * J, n = D.n, F = D.F, NL = D.NL;
  const int f0 = blk * D.FB, nf = min(D.FB, F - f0);
  __shared__ double sx[(TRF_FB + TRF_MAXN) * TRF_MAXJ * 3];
  __shared__ double sL[TRF_MAXL];
  __shared__ int scons[2 * TRF_MAXL];
  __shared__ double sLr[TRF_FB][TRF_MAXL];
  __shared__ double red[4];
  const double* xb = x + (size_t)b * D.NV;
  const int nfx = min(nf + n, F - f0);
  stage8(sx, xb + (size_t)f0 * J3, nfx * J3);
  if (t < NL) sL[t] = xb[D.NX + t];
  if (t < 2 * NL) scons[t] = Bf.cons[t];
  __syncthreads();
  const double ssf = Bf.ssf[b];
  double cost = 0.0, rows = 0.0;
  const int nrep = J * C, ntask = nrep + J3 + NL;
  for (int task = t; task < nf * ntask; task += TRF_THREADS) {
    const int fl = task / ntask, r = task - fl * ntask, f = f0 + fl;
    double* fo = fout + ((size_t)b * F + f) * D.MR;
    if (r < nrep) {  // reprojection (cameras.py:1579-1590): rho(|p2d - project(X)|) per non-NaN coordinate
      const int j = r / C, c = r - j * C;
      const double* pp = Bf.p2d + ((((size_t)b * C + c) * F + f) * J + j) * 2;
      const double px = pp[0], py = pp[1];
      double res[2] = {0.0, 0.0}, jr[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      if (!(isnan(px) && isnan(py))) {
        const double X[3] = {sx[fl * J3 + 3 * j], sx[fl * J3 + 3 * j + 1], sx[fl * J3 + 3 * j + 2]};
        double pu, pv, Ju[3], Jv[3];
        project_jac(cam_at(Bf.cams, c), X, pu, pv, Ju, Jv);
#pragma unroll
        for (int comp = 0; comp < 2; ++comp) {
          const double obs = comp ? py : px;
          if (isnan(obs)) continue;
          double rr, dr;
          reproj_loss(obs - (comp ? pv : pu), D.rp, D.loss, rr, dr);
          res[comp] = rr;
          cost += rr * rr;
          rows += 1.0;
          const double* Jp = comp ? Jv : Ju;
#pragma unroll
          for (int k = 0; k < 3; ++k) jr[3 * comp + k] = -dr * Jp[k];
        }
      }
      fo[2 * r] = res[0];
      fo[2 * r + 1] = res[1];
      if (mode == 1) {
        double* jo = Bf.Jrep + (((size_t)b * F + f) * nrep + r) * 6;
#pragma unroll
        for (int k = 0; k < 6; ++k) jo[k] = jr[k];
      }
    } else if (r < nrep + J3) {  // smoothness: np.diff(p3ds, n, axis=0) * scale_smooth (:1595)
      const int q = r - nrep;
      double val = 0.0;
      if (f < F - n) {
        // np.diff applied n times (numpy's order of the differences), in registers
        const double x0 = sx[fl * J3 + q], x1 = sx[(fl + 1) * J3 + q];
        double dd = x1 - x0;
        if (n >= 2) {
          const double x2 = sx[(fl + 2) * J3 + q];
          const double e1 = x2 - x1;
          if (n == 2) {
            dd = e1 - dd;
          } else {
            const double x3 = sx[(fl + 3) * J3 + q];
            dd = ((x3 - x2) - e1) - (e1 - dd);
          }
        }
        val = dd * ssf;
        cost += val * val;
        rows += 1.0;
      }
      fo[D.MRrep + q] = val;
    } else {  // limb lengths (:1597-1616): 100 (|Xa - Xb| - L) / L * scale
      const int l = r - nrep - J3;
      const int a = scons[2 * l], c2 = scons[2 * l + 1];
      const double L = sL[l], s = l < D.nS ? D.s_len : D.s_len_weak;
      const double dx = sx[fl * J3 + 3 * a] - sx[fl * J3 + 3 * c2];
      const double dy = sx[fl * J3 + 3 * a + 1] - sx[fl * J3 + 3 * c2 + 1];
      const double dz = sx[fl * J3 + 3 * a + 2] - sx[fl * J3 + 3 * c2 + 2];
      const double nr = sqrt(dx * dx + dy * dy + dz * dz);
      const double val = 100 * (nr - L) / L * s;
      cost += val * val;
      rows += 1.0;
      fo[D.MRrep + J3 + l] = val;
      if (mode == 1) {
        const double k = nr > 0 ? s * 100 / L / nr : 0.0;
        double* lo = Bf.lenJ + (((size_t)b * F + f) * NL + l) * 4;
        lo[0] = k * dx;
        lo[1] = k * dy;
        lo[2] = k * dz;
        lo[3] = -s * 100 * nr / (L * L);
        sLr[fl][l] = lo[3] * val;
      }
    }
  }
  cost = block_sum_all(cost, red);
  rows = block_sum_all(rows, red);
  double* fp = Bf.fpart + ((size_t)b * D.NB + blk) * 4;
  if (t == 0) {
    fp[mode == 1 ? 0 : 1] = cost;
    fp[2] = rows;
  }
  if (mode == 1 && t < NL) {
    double s = 0.0;
    for (int fl = 0; fl < nf; ++fl) s += sLr[fl][t];
    Bf.fL[((size_t)b * D.NB + blk) * NL + t] = s;
  }
}

// ---------------------------------------------------------------------------------------------------------
// Latency structure of the per-iteration kernels: every global load that does not depend on a norm (the
// partials, the block's m rows, its Jacobian rows, the n-space entries) is issued first, into LDS or registers;
// then ONE combined reduction of the partials; then the arithmetic from LDS.  A launch thus waits on one memory
// round trip before its arithmetic instead of one per dependent step.

// sums of up to three partial values, every thread of the workgroup holding the same bits
__device__ __forceinline__ void block_sum3_all(double& a, double& b, double& c, double* red /* [12] */) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    a += __shfl_xor(a, m);
    b += __shfl_xor(b, m);
    c += __shfl_xor(c, m);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = a;
    red[4 + w] = b;
    red[8 + w] = c;
  }
  __syncthreads();
  a = (red[0] + red[1]) + (red[2] + red[3]);
  b = (red[4] + red[5]) + (red[6] + red[7]);
  c = (red[8] + red[9]) + (red[10] + red[11]);
  __syncthreads();
}

// Length variables of block 0: sum over the NB blocks of the per-block partials lp[bb * NL + l], fixed order
// (G threads per length, blocks bb = g, g + G, ...; then the G group sums in order).  The first LEN_U partials
// of a thread are loaded early (length_preload, issued with the kernel's other loads); length_sums adds them,
// then any further ones, and leaves out[l] in LDS.
constexpr int LEN_U = 16;
__device__ __forceinline__ void length_preload(const TrfDims& D, const double* __restrict__ lp, double* v) {
  const int NL = D.NL, NB = D.NB, t = threadIdx.x;
  const int G = NL > 0 ? TRF_THREADS / NL : 1;
  const int l = NL > 0 ? t % NL : 0, g = NL > 0 ? t / NL : 0;
#pragma unroll
  for (int u = 0; u < LEN_U; ++u) {
    const int bb = g + u * G;
    v[u] = lp[(size_t)(bb < NB ? bb : 0) * NL + l];
  }
}
__device__ __forceinline__ void length_sums(const TrfDims& D, const double* __restrict__ lp, const double* v,
                                            double* part /*[256]*/, double* out) {
  const int NL = D.NL, NB = D.NB, t = threadIdx.x;
  const int G = NL > 0 ? TRF_THREADS / NL : 1;
  double s = 0.0;
  if (t < G * NL) {
    const int l = t % NL, g = t / NL;
#pragma unroll
    for (int u = 0; u < LEN_U; ++u)
      if (g + u * G < NB) s += v[u];
    for (int bb = g + LEN_U * G; bb < NB; bb += G) s += lp[(size_t)bb * NL + l];
  }
  part[t] = s;
  __syncthreads();
  if (t < NL) {
    double a = 0.0;
    for (int g = 0; g < G; ++g) a += part[g * NL + t];
    out[t] = a;
  }
  __syncthreads();
}

// The length variables, in a workgroup of their own (the last of a J^T launch, blockIdx.x == NB) when the grid
// (for TRF_NOMINAL_B animals) leaves a CU for it (D.NBV == NB + 1): v = the sum over the frames of dL * u_len
// (the per-block sums of the m-space launch: Lpart, or fL for MODE 0 / 1) / beta, minus beta vn in MODE 2; its
// partials go to slot NB.  Done by block 0 alongside its frames, the NB x NL sums make that block, and so the
// launch, 1.2 us longer (profiles/r05x_*); on a grid that already has more workgroups than CUs an extra one
// costs more than that (config 4: 4 % slower, profiles/r05z_*), and block 0 keeps them.
template <int MODE>
__device__ __forceinline__ void jt_lengths(const TrfDims& D, const TrfBufs& Bf, int par, int b, double* red,
                                           double* spart, double* sLs) {
  const int t = threadIdx.x, NL = D.NL, NB = D.NB;
  const double normb = Bf.lctl[4 * b + 1];
  const double* up = Bf.upart + ((size_t)par * D.B + b) * NB;
  double pu = 0.0;
  if (MODE == 2 && t < NB) pu = up[t];
  const size_t nb = (size_t)b * D.NV;
  const bool lens = !D.fix && NL > 0;
  double vnL = 0.0;
  if (MODE == 2 && lens && t < NL) vnL = Bf.vn[nb + D.NX + t];
  const double* lp = (MODE == 2 ? Bf.Lpart : Bf.fL) + (size_t)b * NB * NL;
  double lv[LEN_U];
  if (lens) length_preload(D, lp, lv);
  if (!Bf.act[b] || (MODE > 0 && Bf.done[b])) return;
  if (MODE == 2)
    for (int i = t + TRF_THREADS; i < NB; i += TRF_THREADS) pu += up[i];
  if (lens) length_sums(D, lp, lv, spart, sLs);
  double beta = 1.0;
  if (MODE == 1) beta = normb;
  if (MODE == 2) {  // (the same reduction, in the same order, as every other workgroup's)
    double d1 = 0.0, d2 = 0.0;
    block_sum3_all(pu, d1, d2, red);
    beta = sqrt(pu);
  }
  const double ib = 1.0 / beta;
  double vsq = 0.0, vmax = 0.0;
  if (t < NL) {
    double v = 0.0;
    if (lens) {
      const double acc = sLs[t] * ib;
      v = MODE == 2 ? vnL * -beta + acc : acc;
      vsq = v * v;
      vmax = fabs(v);
    }
    (MODE == 0 ? Bf.g : Bf.vraw)[nb + D.NX + t] = v;
  }
  vsq = block_sum_all(vsq, red);
  if (MODE == 0) vmax = block_max_all(vmax, red);
  if (t == 0) {
    double* vp = MODE == 0 ? Bf.gpart + ((size_t)b * D.NBV + NB) * 2
                           : Bf.vpart + (((size_t)par * D.B + b) * D.NBV + NB) * 2;
    vp[0] = vsq;
    vp[1] = vmax;
  }
}

// v = J^T (u / beta) - beta vn for the block's parameters (blockIdx.x < NB; the length variables: jt_lengths).
//   MODE 0: g = J^T f (u = fres, beta = 1, no vn); partials (sum g^2, max |g|) in gpart
//   MODE 1: lsmr's start, v = J^T (f / normb)
//   MODE 2: lsmr phase 2 of iteration k: v_k = J^T (u_k / beta_k) - beta_k v_{k-1}  (par = k & 1)
// Dynamic LDS: the m rows of frames [f0 - n, f0 + nf) (raw; scaled by 1 / beta where they are used, as scipy's
// in-place u *= 1 / beta), the block's Jacobian rows and the per-camera products of 3a.
template <int MODE>
__global__ void __launch_bounds__(TRF_THREADS) trf_jt_kernel(TrfDims D, TrfBufs Bf, int par) {
  TRF_PROF_BEGIN();
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int J = D.J, C = D.C, J3 = 3 * J, n = D.n, F = D.F, NL = D.NL, NB = D.NB;
  const int f0 = blk * D.FB, nf = min(D.FB, F - f0);
  __shared__ double red[12];
  __shared__ __attribute__((aligned(16))) double slj[TRF_FB * TRF_MAXL * 4];
  __shared__ int sadj[TRF_MAXJ + 1 + 2 * TRF_MAXL];
  __shared__ double spart[TRF_THREADS];
  __shared__ double sLs[TRF_MAXL];
  extern __shared__ double lds_jt[];
  if (blk == NB) {  // (only launched when D.NBV == NB + 1)
    jt_lengths<MODE>(D, Bf, par, b, red, spart, sLs);
    return;
  }
  const int fa = max(0, f0 - n), nrow = (f0 + nf - fa) * D.MR;
  double* su = lds_jt;
  double* sj = lds_jt + (((size_t)(D.FB + D.n) * D.MR + 1) & ~(size_t)1);
  double* sprod = sj + (size_t)D.FB * J * C * 6;
  const double* uin = MODE == 2 ? Bf.u : Bf.fres;
  // 1. loads independent of beta, all issued before the first wait
  const double ssf = Bf.ssf[b], normb = Bf.lctl[4 * b + 1];
  const double* up = Bf.upart + ((size_t)par * D.B + b) * NB;
  double pu = 0.0;
  if (MODE == 2 && t < NB) pu = up[t];
  const size_t nb = (size_t)b * D.NV;
  double vn0 = 0.0, vn1 = 0.0, vnL = 0.0;  // the thread's (at most two) parameters and a length variable
  const bool lblk = blk == 0 && D.NBV == NB;   // block 0 holds the length variables
  if (MODE == 2) {
    if (t < nf * J3) vn0 = Bf.vn[nb + (size_t)f0 * J3 + t];
    if (t + TRF_THREADS < nf * J3) vn1 = Bf.vn[nb + (size_t)f0 * J3 + t + TRF_THREADS];
    if (lblk && t < NL && !D.fix) vnL = Bf.vn[nb + D.NX + t];
  }
  const bool lens = lblk && !D.fix && NL > 0;
  const double* lp = (MODE == 2 ? Bf.Lpart : Bf.fL) + (size_t)b * NB * NL;
  double lv[LEN_U];
  if (lens) length_preload(D, lp, lv);
  const int nadj = J + 1 + 2 * NL;
  const int adj = Bf.jadj[t < nadj ? t : 0];
  // the m rows (FB + n frames of MR: up to 2560 doubles in the first round, 7 x 354 for 17 joints, 8 cameras,
  // 31 constraints), the Jacobian rows (3584: 4 frames x 17 joints x 8 cameras x 6) and the length rows (512:
  // 4 frames x 32 constraints x 4)
  Stager<0, 5, 7, 1> st{StageSeg{nullptr, nullptr, 0}, StageSeg{su, uin + ((size_t)b * F + fa) * D.MR, nrow},
                        StageSeg{sj, Bf.Jrep + ((size_t)b * F + f0) * J * C * 6, nf * J * C * 6},
                        StageSeg{slj, Bf.lenJ + ((size_t)b * F + f0) * NL * 4, nf * NL * 4}};
  st.load();
  // the animal's flags, read with the rest (a block of a finished animal has loaded for nothing; every address
  // above is inside the workspace whatever the flags)
  if (!Bf.act[b] || (MODE > 0 && Bf.done[b])) return;
  TRF_PROF(1);
  // then the stores (and the rare second rounds)
  if (t < nadj) sadj[t] = adj;
  st.store();
  if (MODE == 2)
    for (int i = t + TRF_THREADS; i < NB; i += TRF_THREADS) pu += up[i];
  if (lens) length_sums(D, lp, lv, spart, sLs);
  TRF_PROF(2);
  // 2. the norm
  double beta = 1.0;
  if (MODE == 1) beta = normb;
  if (MODE == 2) {
    double d1 = 0.0, d2 = 0.0;
    block_sum3_all(pu, d1, d2, red);  // (also the barrier after the staging stores)
    beta = sqrt(pu);
  } else {
    __syncthreads();
  }
  const double ib = 1.0 / beta;
  TRF_PROF(3);
  // 3a. the reprojection products, one thread per (frame, joint, camera) row pair: lanes read consecutive rows
  // (a thread per parameter summing over the cameras read rows 96 dwords apart, all in two LDS banks); the
  // three products per row pair go to sprod[fl][c][3 j + k]
  {
    const int JC = J * C, NT = nf * JC;
    const float iC = 1.0f / (float)C;
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // (NT <= 3 TRF_THREADS for 4 frames x 17 joints x 8 cameras; more loop)
      for (int i = k * TRF_THREADS + t; i < NT; i += 3 * TRF_THREADS) {
        const int fl = trf_frame_of(i, JC), jc = i - fl * JC;
        const int j = (int)(((float)jc + 0.5f) * iC), c = jc - j * C;
        const trf_d2* jr2 = reinterpret_cast<const trf_d2*>(sj + (size_t)i * 6);
        const trf_d2 ju = *reinterpret_cast<const trf_d2*>(su + (size_t)(f0 + fl - fa) * D.MR + 2 * jc);
        const trf_d2 a0 = jr2[0], a1 = jr2[1], a2 = jr2[2];  // (d/dX, d/dY, d/dZ of u; then of v)
        const double u0 = ju.x * ib, u1 = ju.y * ib;
        double* pr = sprod + ((size_t)fl * C + c) * J3 + 3 * j;
        pr[0] = a0.x * u0 + a1.y * u1;
        pr[1] = a0.y * u0 + a2.x * u1;
        pr[2] = a1.x * u0 + a2.y * u1;
      }
    }
  }
  __syncthreads();
  // 3b. one thread per parameter: the camera products in camera order, the smoothness and length terms
  double vsq = 0.0, vmax = 0.0;
  const int ntask = nf * J3;
  for (int task = t, it = 0; task < ntask; task += TRF_THREADS, ++it) {
    const int fl = task / J3, q = task - fl * J3, j = q / 3, kk = q - 3 * j, f = f0 + fl;
    const double* uf = su + (size_t)(f - fa) * D.MR;
    double acc = 0.0;
    const double* pr = sprod + (size_t)fl * C * J3 + q;
#pragma unroll 4
    for (int c = 0; c < C; ++c) acc += pr[(size_t)c * J3];
    for (int m = 0; m <= n; ++m) {  // smoothness rows i = f - m hold frame f with coefficient c[m]
      const int i = f - m;
      if (i >= 0 && i < F - n) acc += ssf * dcoef(D, m) * (su[(size_t)(i - fa) * D.MR + D.MRrep + q] * ib);
    }
    for (int e = sadj[j], ee = sadj[j + 1]; e < ee; ++e) {  // the constraints touching joint j, ascending l
      const int code = sadj[J + 1 + e], l = code >> 1;
      const double term = slj[(fl * NL + l) * 4 + kk] * (uf[D.MRrep + J3 + l] * ib);
      if (code & 1) acc -= term;
      else acc += term;
    }
    const size_t o = nb + (size_t)f * J3 + q;
    const double v = MODE == 2 ? (it == 0 ? vn0 : vn1) * -beta + acc : acc;
    (MODE == 0 ? Bf.g : Bf.vraw)[o] = v;
    vsq += v * v;
    vmax = fmax(vmax, fabs(v));
  }
  if (lblk && t < NL) {  // the length variables: sum over frames of dL * u_len
    const size_t o = nb + D.NX + t;
    double v = 0.0;
    if (!D.fix) {
      const double acc = sLs[t] * ib;
      v = MODE == 2 ? vnL * -beta + acc : acc;
      vsq += v * v;
      vmax = fmax(vmax, fabs(v));
    }
    (MODE == 0 ? Bf.g : Bf.vraw)[o] = v;
  }
  TRF_PROF(4);
  vsq = block_sum_all(vsq, red);
  if (MODE == 0) vmax = block_max_all(vmax, red);
  if (t == 0) {
    double* vp = MODE == 0 ? Bf.gpart + ((size_t)b * D.NBV + blk) * 2
                           : Bf.vpart + (((size_t)par * D.B + b) * D.NBV + blk) * 2;
    vp[0] = vsq;
    vp[1] = vmax;
  }
  TRF_PROF(5);
  if (MODE == 2) TRF_PROF_END(1, 5);
}

// ---------------------------------------------------------------------------------------------------------
// lsmr phase 1 of iteration k (k >= 1; pp = (k - 1) & 1, par = k & 1): alpha_{k-1}, beta_{k-1} and
// ||x_{k-2}|| from the partials; FIRST (k = 1) starts the recurrences (lsmr.py:205-239); otherwise the stop test
// of iteration k - 2 (lsmr.py:413-441, with ||x_{k-2}||: when it passes x_{k-2} is the answer and nothing more
// runs), then iteration k - 1's recurrences (:301-410) and the hbar / x / h updates; then u_k = J v_{k-1} -
// alpha_{k-1} u_{k-1} for the block's rows.
__device__ __forceinline__ void lsmr_recurrence(double* S, double alpha, double beta, double damp, double& chb,
                                                double& cx, double& ch) {
  // (lsmr.py:305's rotation of alphabar and damp was computed with the previous iteration's recurrences, off
  // the chain that waits on this iteration's norms)
  const double chat = S[S_CHAT], shat = S[S_SHAT], alphahat = S[S_ALPHAHAT];
  const double rhoold = S[S_RHO];
  double c, s, rho;
  sym_ortho(alphahat, beta, c, s, rho);
  const double thetanew = s * alpha;
  S[S_ALPHABAR] = c * alpha;
  sym_ortho(S[S_ALPHABAR], damp, S[S_CHAT], S[S_SHAT], S[S_ALPHAHAT]);
  const double rhobarold = S[S_RHOBAR];
  const double zetaold = S[S_ZETA];
  const double thetabar = S[S_SBAR] * rho;
  const double rhotemp = S[S_CBAR] * rho;
  double cbar, sbar, rhobar;
  sym_ortho(S[S_CBAR] * rho, thetanew, cbar, sbar, rhobar);
  const double zeta = cbar * S[S_ZETABAR];
  const double zetabar = -sbar * S[S_ZETABAR];
  chb = -(thetabar * rho / (rhoold * rhobarold));
  cx = zeta / (rho * rhobar);
  ch = -(thetanew / rho);
  const double betaacute = chat * S[S_BETADD];
  const double betacheck = -shat * S[S_BETADD];
  const double betahat = c * betaacute;
  const double betadd = -s * betaacute;
  const double thetatildeold = S[S_THETATILDE];
  double ctildeold, stildeold, rhotildeold;
  sym_ortho(S[S_RHODOLD], thetabar, ctildeold, stildeold, rhotildeold);
  const double thetatilde = stildeold * rhobar;
  const double rhodold = ctildeold * rhobar;
  const double betad = -stildeold * S[S_BETAD] + ctildeold * betahat;
  const double tautildeold = (zetaold - thetatildeold * S[S_TAUTILDEOLD]) / rhotildeold;
  const double taud = (zeta - thetatilde * tautildeold) / rhodold;
  const double d = S[S_D] + betacheck * betacheck;
  const double bt = betad - taud;
  const double normr = sqrt(d + bt * bt + betadd * betadd);
  double normA2 = S[S_NORMA2] + beta * beta;
  const double normA = sqrt(normA2);
  normA2 = normA2 + alpha * alpha;
  const double itn = S[S_ITN] + 1;
  const double maxrbar = fmax(S[S_MAXRBAR], rhobarold);
  const double minrbar = itn > 1 ? fmin(S[S_MINRBAR], rhobarold) : S[S_MINRBAR];
  const double condA = fmax(maxrbar, rhotemp) / fmin(minrbar, rhotemp);
  S[S_RHO] = rho;
  S[S_RHOBAR] = rhobar;
  S[S_CBAR] = cbar;
  S[S_SBAR] = sbar;
  S[S_ZETABAR] = zetabar;
  S[S_ZETA] = zeta;
  S[S_BETADD] = betadd;
  S[S_BETAD] = betad;
  S[S_RHODOLD] = rhodold;
  S[S_TAUTILDEOLD] = tautildeold;
  S[S_THETATILDE] = thetatilde;
  S[S_D] = d;
  S[S_NORMA2] = normA2;
  S[S_MAXRBAR] = maxrbar;
  S[S_MINRBAR] = minrbar;
  S[S_ITN] = itn;
  S[S_NORMR] = normr;
  S[S_NORMAR] = fabs(zetabar);
  S[S_NORMA] = normA;
  S[S_CONDA] = condA;
}

// the stop test of lsmr.py:413-441 from a state slot and ||x||; 0 = go on
__device__ __forceinline__ int lsmr_istop(const TrfDims& D, const double* S, double normx, double normb,
                                          double maxiter) {
  const double normr = S[S_NORMR], normar = S[S_NORMAR], normA = S[S_NORMA], condA = S[S_CONDA];
  const double itn = S[S_ITN];
  const double test1 = normr / normb;
  const double test2 = (normA * normr) != 0 ? normar / (normA * normr) : INFINITY;
  const double test3 = 1 / condA;
  const double t1 = test1 / (1 + normA * normx / normb);
  const double rtol = D.btol + D.atol * normA * normx / normb;
  int istop = 0;
  if (itn >= maxiter) istop = 7;
  if (1 + test3 <= 1) istop = 6;
  if (1 + test2 <= 1) istop = 5;
  if (1 + t1 <= 1) istop = 4;
  if (test3 <= D.ctol) istop = 3;
  if (test2 <= D.atol) istop = 2;
  if (test1 <= rtol) istop = 1;
  return istop;
}

template <bool FIRST>
__global__ void __launch_bounds__(TRF_THREADS) trf_lsmr1_kernel(TrfDims D, TrfBufs Bf, int par) {
  TRF_PROF_BEGIN();
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int J = D.J, C = D.C, J3 = 3 * J, n = D.n, F = D.F, NL = D.NL, NB = D.NB;
  const int f0 = blk * D.FB, nf = min(D.FB, F - f0);
  const int pp = par ^ 1;
  __shared__ double red[12];
  __shared__ double sv[(TRF_FB + TRF_MAXN) * TRF_MAXJ * 3];
  __shared__ double sL[TRF_MAXL];
  __shared__ double sLu[TRF_FB][TRF_MAXL];
  __shared__ __attribute__((aligned(16))) double slj[TRF_FB * TRF_MAXL * 4];
  __shared__ int scons[2 * TRF_MAXL];
  __shared__ double sS[TRF_NS];
  __shared__ double scoef[4];
  __shared__ int sstop;
  extern __shared__ double lds_l1[];
  double* sm = lds_l1;                                                   // the block's m rows (u_{k-1}, raw)
  double* sj = lds_l1 + (((size_t)D.FB * D.MR + 1) & ~(size_t)1);       // its Jacobian rows
  const size_t nb = (size_t)b * D.NV;
  // 1. loads independent of the norms, all issued before the first wait
  const double damp = Bf.lctl[4 * b], normb = Bf.lctl[4 * b + 1], maxiter = Bf.lctl[4 * b + 2], ssf = Bf.ssf[b];
  const double* vp = Bf.vpart + ((size_t)pp * D.B + b) * D.NBV * 2;
  const double* upp = Bf.upart + ((size_t)pp * D.B + b) * NB;
  const double* xp = Bf.xpart + ((size_t)pp * D.B + b) * NB;
  double pa = 0.0, pb = 0.0, px = 0.0;
  if (t < D.NBV) pa = vp[2 * t];
  if (!FIRST && t < NB) {
    pb = upp[t];
    px = xp[t];
  }
  const double stv = (!FIRST && t < TRF_NS) ? Bf.st[((size_t)pp * D.B + b) * TRF_NS + t] : 0.0;
  const int nfx = min(nf + n, F - f0);
  // the thread's n-space entries: (at most two) parameters and block 0's length variable
  double h0 = 0.0, h1 = 0.0, hL = 0.0, hb0 = 0.0, hb1 = 0.0, hbL = 0.0, x0 = 0.0, x1 = 0.0, xL = 0.0;
  const size_t o0 = nb + (size_t)f0 * J3 + t, o1 = o0 + TRF_THREADS, oL = nb + D.NX + t;
  const bool e0 = t < nf * J3, e1 = t + TRF_THREADS < nf * J3, eL = blk == 0 && t < NL && !D.fix;
  if (!FIRST) {
    if (e0) {
      h0 = Bf.h[o0];
      hb0 = Bf.hbar[o0];
      x0 = Bf.xl[o0];
    }
    if (e1) {
      h1 = Bf.h[o1];
      hb1 = Bf.hbar[o1];
      x1 = Bf.xl[o1];
    }
    if (eL) {
      hL = Bf.h[oL];
      hbL = Bf.hbar[oL];
      xL = Bf.xl[oL];
    }
  }
  const double lv = (t < NL && !D.fix) ? Bf.vraw[nb + D.NX + t] : 0.0;
  const int cv = Bf.cons[t < 2 * NL ? t : 0];
  const double* uin = FIRST ? Bf.fres : Bf.u;
  // v_raw of frames [f0, f0 + nf + n) (up to 512 doubles: 7 frames x 17 joints x 3), the m rows (up to 1536:
  // 4 frames x 384), the Jacobian rows (3584) and the length rows (512)
  Stager<2, 3, 7, 1> st{StageSeg{sv, Bf.vraw + nb + (size_t)f0 * J3, nfx * J3},
                        StageSeg{sm, uin + ((size_t)b * F + f0) * D.MR, nf * D.MR},
                        StageSeg{sj, Bf.Jrep + ((size_t)b * F + f0) * J * C * 6, nf * J * C * 6},
                        StageSeg{slj, Bf.lenJ + ((size_t)b * F + f0) * NL * 4, nf * NL * 4}};
  st.load();
  // the animal's flags, read with the rest (as in trf_jt_kernel)
  if (!Bf.act[b] || Bf.done[b]) return;
  TRF_PROF(1);
  // then the stores (and the rare second rounds)
  if (!FIRST && t < TRF_NS) sS[t] = stv;
  if (t < NL) sL[t] = lv;
  if (t < 2 * NL) scons[t] = cv;
  st.store();
  for (int i = t + TRF_THREADS; i < D.NBV; i += TRF_THREADS) pa += vp[2 * i];
  if (!FIRST)
    for (int i = t + TRF_THREADS; i < NB; i += TRF_THREADS) {
      pb += upp[i];
      px += xp[i];
    }
  TRF_PROF(2);
  // 2. the norms (one combined reduction; also the barrier after the staging stores)
  block_sum3_all(pa, pb, px, red);
  TRF_PROF(3);
  const double alpha = sqrt(pa);
  const double beta = FIRST ? normb : sqrt(pb);
  // v_{k-1} = v_raw / alpha: scipy's in-place v *= 1 / alpha, applied by every reader of sv / sL to the raw
  // value it reads (the same product, so the same bits, with no pass over LDS and no barrier before the rows)
  const double ia = 1.0 / alpha;
  // 3. lane 0 of the last wave: the stop test and the recurrences (a serial chain of divisions and square
  // roots, in registers); meanwhile the other waves compute the m-space rows, which need only alpha and beta:
  // u_k = (u_{k-1} / beta) * -alpha + J v_{k-1}   (lsmr.py:284-286).  (If the test stops the run, the rows
  // written here are never read: every later lsmr launch returns on the done flag.)
  constexpr int RT = TRF_THREADS - 64;  // the recurrence thread; m-space workers t < MW
  const int MW = FIRST ? TRF_THREADS : RT;
  if (t == RT) {
    double S[TRF_NS];
#pragma unroll
    for (int i = 0; i < TRF_NS; ++i) S[i] = FIRST ? 0.0 : sS[i];
    double chb = 0.0, cx = 0.0, ch = 0.0;
    int istop = 0;
    if (FIRST) {
      S[S_ZETABAR] = alpha * beta;
      S[S_ALPHABAR] = alpha;
      sym_ortho(alpha, damp, S[S_CHAT], S[S_SHAT], S[S_ALPHAHAT]);
      S[S_RHO] = 1;
      S[S_RHOBAR] = 1;
      S[S_CBAR] = 1;
      S[S_SBAR] = 0;
      S[S_BETADD] = beta;
      S[S_RHODOLD] = 1;
      S[S_NORMA2] = alpha * alpha;
      S[S_MINRBAR] = 1e+100;
      S[S_ITN] = 0;
      if (!(alpha * beta != 0)) istop = 8;  // normar == 0 (or normb == 0): x = 0 (lsmr.py:247-256)
    } else {
      // the test and the recurrences side by side (independent chains; the recurrence's results are dropped
      // when the test stops the run)
      const double itn0 = S[S_ITN];
      if (itn0 >= 1) istop = lsmr_istop(D, S, sqrt(px), normb, maxiter);
      lsmr_recurrence(S, alpha, beta, damp, chb, cx, ch);
      if (istop) S[S_ITN] = itn0;
    }
    if (istop && blk == 0) {
      Bf.done[b] = istop;
      Bf.lctl[4 * b + 3] = S[S_ITN];
      Bf.hitn[b] = S[S_ITN];
      Bf.hdone[b] = istop;
    }
    sstop = istop;
    scoef[0] = chb;
    scoef[1] = cx;
    scoef[2] = ch;
    if (blk == 0 && !istop) {
      double* So = Bf.st + ((size_t)par * D.B + b) * TRF_NS;
#pragma unroll
      for (int i = 0; i < TRF_NS; ++i) So[i] = S[i];
    }
#ifdef TRF_PROFILE
    if (!FIRST && blk == TRF_PROFILE_BLOCK && b == 0) atomicAdd(&g_trf_prof[1][8], wall_clock64() - prof_t[3]);  // the recurrence
#endif
  }
  const double ib = 1.0 / beta;
  const int nrep = J * C;
  double usq = 0.0;
  if (t < MW) {
    // reprojection rows, up to three row pairs per thread with their LDS reads issued together (frame and joint
    // from comparisons and a float reciprocal instead of integer divisions)
    const int NR = nf * nrep;
    const float iC = 1.0f / (float)C;
    for (int base = t; base < NR; base += 3 * MW) {
      trf_d2 a0[3], a1[3], a2[3], um[3];
      double v0[3], v1[3], v2[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int i0 = base + k * MW, i = i0 < NR ? i0 : 0;
        const int fl = trf_frame_of(i, nrep), r = i - fl * nrep;
        const int j = (int)(((float)r + 0.5f) * iC);
        const trf_d2* jr2 = reinterpret_cast<const trf_d2*>(sj + (size_t)i * 6);
        a0[k] = jr2[0];
        a1[k] = jr2[1];
        a2[k] = jr2[2];
        um[k] = *reinterpret_cast<const trf_d2*>(sm + (size_t)fl * D.MR + 2 * r);
        const double* v = sv + fl * J3 + 3 * j;
        v0[k] = v[0] * ia;
        v1[k] = v[1] * ia;
        v2[k] = v[2] * ia;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int i = base + k * MW;
        if (i < NR) {
          const int fl = trf_frame_of(i, nrep), r = i - fl * nrep;
          const double ju = a0[k].x * v0[k] + a0[k].y * v1[k] + a1[k].x * v2[k];
          const double jv = a1[k].y * v0[k] + a2[k].x * v1[k] + a2[k].y * v2[k];
          const double un0 = (um[k].x * ib) * -alpha + ju, un1 = (um[k].y * ib) * -alpha + jv;
          trf_d2 o;
          o.x = un0;
          o.y = un1;
          *reinterpret_cast<trf_d2*>(Bf.u + ((size_t)b * F + f0 + fl) * D.MR + 2 * r) = o;
          usq += un0 * un0;
          usq += un1 * un1;
        }
      }
    }
    TRF_PROF(8);
    // smoothness rows
    const float iJ3 = 1.0f / (float)J3;
    for (int i = t; i < nf * J3; i += MW) {
      const int fl = (int)(((float)i + 0.5f) * iJ3), q = i - fl * J3, f = f0 + fl;
      double un = 0.0;
      if (f < F - n) {
        double jv = 0.0;
        for (int m = 0; m <= n; ++m) jv += ssf * dcoef(D, m) * (sv[(fl + m) * J3 + q] * ia);
        un = (sm[(size_t)fl * D.MR + D.MRrep + q] * ib) * -alpha + jv;
      }
      Bf.u[((size_t)b * F + f) * D.MR + D.MRrep + q] = un;
      usq += un * un;
    }
    TRF_PROF(9);
    // limb-length rows
    const float iNL = NL > 0 ? 1.0f / (float)NL : 0.0f;
    for (int i = t; i < nf * NL; i += MW) {
      const int fl = (int)(((float)i + 0.5f) * iNL), l = i - fl * NL, f = f0 + fl;
      const int a = scons[2 * l], c2 = scons[2 * l + 1];
      const double* lj = slj + (fl * NL + l) * 4;
      const double* va = sv + fl * J3 + 3 * a;
      const double* vc = sv + fl * J3 + 3 * c2;
      double jv = lj[0] * (va[0] * ia - vc[0] * ia) + lj[1] * (va[1] * ia - vc[1] * ia) +
                  lj[2] * (va[2] * ia - vc[2] * ia);
      if (!D.fix) jv += lj[3] * (sL[l] * ia);
      const double un = (sm[(size_t)fl * D.MR + D.MRrep + J3 + l] * ib) * -alpha + jv;
      Bf.u[((size_t)b * F + f) * D.MR + D.MRrep + J3 + l] = un;
      usq += un * un;
      sLu[fl][l] = lj[3] * un;
    }
  }
  TRF_PROF(4);
  __syncthreads();
  TRF_PROF(5);
  if (sstop) {
    if (FIRST) {  // x = 0
      if (e0) Bf.xl[o0] = 0.0;
      if (e1) Bf.xl[o1] = 0.0;
      if (eL) Bf.xl[oL] = 0.0;
    }
    return;
  }
  // 4. n space: hbar, x, h (lsmr.py:396-403)
  const double chb = scoef[0], cx = scoef[1], ch = scoef[2];
  double xsq = 0.0;
  auto upd = [&](bool e, size_t o, double v, double h, double hb, double x) {
    if (!e) return;
    Bf.vn[o] = v;
    if (FIRST) {
      Bf.h[o] = v;
      Bf.hbar[o] = 0.0;
      Bf.xl[o] = 0.0;
    } else {
      const double hbn = hb * chb + h;
      const double xn = x + cx * hbn;
      Bf.hbar[o] = hbn;
      Bf.xl[o] = xn;
      Bf.h[o] = h * ch + v;
      xsq += xn * xn;
    }
  };
  upd(e0, o0, e0 ? sv[t] * ia : 0.0, h0, hb0, x0);
  upd(e1, o1, e1 ? sv[t + TRF_THREADS] * ia : 0.0, h1, hb1, x1);
  upd(eL, oL, eL ? sL[t] * ia : 0.0, hL, hbL, xL);
  TRF_PROF(6);
  block_sum3_all(usq, xsq, pa, red);
  if (t == 0) {
    Bf.upart[((size_t)par * D.B + b) * NB + blk] = usq;
    Bf.xpart[((size_t)par * D.B + b) * NB + blk] = xsq;
  }
  if (t < NL) {
    double s2 = 0.0;
    for (int fl = 0; fl < nf; ++fl) s2 += sLu[fl][t];
    Bf.Lpart[((size_t)b * NB + blk) * NL + t] = s2;
  }
  TRF_PROF(7);
  if (!FIRST) TRF_PROF_END(0, 7);
#ifdef TRF_PROFILE
  if (!FIRST && t == 0 && blk == TRF_PROFILE_BLOCK && b == 0) {  // the m-space split: rows from phase 3's start
    atomicAdd(&g_trf_prof[0][8], prof_t[8] - prof_t[3]);
    atomicAdd(&g_trf_prof[0][9], prof_t[9] - prof_t[8]);
    atomicAdd(&g_trf_prof[0][10], prof_t[4] - prof_t[9]);
  }
#endif
}

// ---------------------------------------------------------------------------------------------------------
// m-space products J a (and J c) without storage: partials sum (Ja)^2, sum (Jc)^2, sum (Ja)(Jc).
__global__ void __launch_bounds__(TRF_THREADS) trf_jv_kernel(TrfDims D, TrfBufs Bf, const double* __restrict__ va,
                                                            const double* __restrict__ vc) {
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  if (!Bf.act[b]) return;
  const int J = D.J, C = D.C, J3 = 3 * J, n = D.n, F = D.F, NL = D.NL;
  const int f0 = blk * D.FB, nf = min(D.FB, F - f0);
  __shared__ double red[4];
  __shared__ double sa[(TRF_FB + TRF_MAXN) * TRF_MAXJ * 3], sc[(TRF_FB + TRF_MAXN) * TRF_MAXJ * 3];
  __shared__ double saL[TRF_MAXL], scL[TRF_MAXL];
  __shared__ int scons[2 * TRF_MAXL];
  const size_t nb = (size_t)b * D.NV;
  const int nfx = min(nf + n, F - f0);
  for (int i = t; i < nfx * J3; i += TRF_THREADS) {
    sa[i] = va[nb + (size_t)f0 * J3 + i];
    sc[i] = vc ? vc[nb + (size_t)f0 * J3 + i] : 0.0;
  }
  if (t < NL) {
    saL[t] = D.fix ? 0.0 : va[nb + D.NX + t];
    scL[t] = (D.fix || !vc) ? 0.0 : vc[nb + D.NX + t];
  }
  if (t < 2 * NL) scons[t] = Bf.cons[t];
  __syncthreads();
  const double ssf = Bf.ssf[b];
  const int nrep = J * C, ntask = nrep + J3 + NL;
  double saa = 0.0, scc = 0.0, sac = 0.0;
  for (int task = t; task < nf * ntask; task += TRF_THREADS) {
    const int fl = task / ntask, r = task - fl * ntask, f = f0 + fl;
    if (r < nrep) {
      const int j = r / C;
      const double* jr = Bf.Jrep + (((size_t)b * F + f) * nrep + r) * 6;
      const double* a = sa + fl * J3 + 3 * j;
      const double* c = sc + fl * J3 + 3 * j;
#pragma unroll
      for (int comp = 0; comp < 2; ++comp) {
        const double ja = jr[3 * comp] * a[0] + jr[3 * comp + 1] * a[1] + jr[3 * comp + 2] * a[2];
        const double jc = jr[3 * comp] * c[0] + jr[3 * comp + 1] * c[1] + jr[3 * comp + 2] * c[2];
        saa += ja * ja;
        scc += jc * jc;
        sac += ja * jc;
      }
    } else if (r < nrep + J3) {
      const int q = r - nrep;
      if (f < F - n) {
        double ja = 0.0, jc = 0.0;
        for (int m = 0; m <= n; ++m) {
          ja += ssf * dcoef(D, m) * sa[(fl + m) * J3 + q];
          jc += ssf * dcoef(D, m) * sc[(fl + m) * J3 + q];
        }
        saa += ja * ja;
        scc += jc * jc;
        sac += ja * jc;
      }
    } else {
      const int l = r - nrep - J3;
      const int a = scons[2 * l], c2 = scons[2 * l + 1];
      const double* lj = Bf.lenJ + (((size_t)b * F + f) * NL + l) * 4;
      double ja = 0.0, jc = 0.0;
#pragma unroll
      for (int kk = 0; kk < 3; ++kk) {
        ja += lj[kk] * (sa[fl * J3 + 3 * a + kk] - sa[fl * J3 + 3 * c2 + kk]);
        jc += lj[kk] * (sc[fl * J3 + 3 * a + kk] - sc[fl * J3 + 3 * c2 + kk]);
      }
      ja += lj[3] * saL[l];
      jc += lj[3] * scL[l];
      saa += ja * ja;
      scc += jc * jc;
      sac += ja * jc;
    }
  }
  saa = block_sum_all(saa, red);
  scc = block_sum_all(scc, red);
  sac = block_sum_all(sac, red);
  if (t == 0) {
    double* jp = Bf.jpart + ((size_t)b * D.NB + blk) * 4;
    jp[0] = saa;
    jp[1] = scc;
    jp[2] = sac;
  }
}

// ---------------------------------------------------------------------------------------------------------
// n-space operations of the trust-region step, with per-block partials in npart[b][blk][field] (a field per
// operation, so an operation can read the previous one's partials while it writes its own):
//   0 XNORM  x.x                                                     field 0
//   1 DOTS   g.gn                                                    field 1  (gn = lsmr's x)
//   2 S1T    s1 = g * c0;  s2 = gn - c1 * s1;  s2.s2                 field 2  (Gram-Schmidt of [g, gn]; c0 = 1 / |g|,
//            c1 = (g.gn) / |g| from gpart and field 1, reduced by every workgroup)
//   3 S2     s2 = s2 * c2;  g.s1, g.s2                                fields 3, 4  (c2 = 1 / |s2| from field 2, 0 if 0)
//   4 STEP   xt = x + (s1 p0 + s2 p1);  step.step                    field 5  (p = coef[0..1], from the host)
//   5 ACCEPT x = xt
enum { OP_XNORM, OP_DOTS, OP_S1T, OP_S2, OP_STEP, OP_ACCEPT };
constexpr int TRF_NPF = 8;  // npart fields
__global__ void __launch_bounds__(TRF_THREADS) trf_nops_kernel(TrfDims D, TrfBufs Bf, double* __restrict__ x,
                                                              double* __restrict__ xt, int op) {
  const int blk = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  if (!Bf.act[b]) return;
  const int J3 = 3 * D.J, F = D.F;
  const int f0 = blk * D.FB, nf = min(D.FB, F - f0);
  __shared__ double red[4];
  const double* cf = Bf.coef + 4 * (size_t)b;
  const size_t nb = (size_t)b * D.NV;
  const double* nbp = Bf.npart + (size_t)b * D.NB * TRF_NPF;
  double c0 = 0.0, c1 = 0.0, c2 = 0.0;
  if (op == OP_S1T) {
    const double ng = sqrt(reduce_parts(Bf.gpart + (size_t)b * D.NBV * 2, D.NBV, 2, red));
    c0 = 1.0 / ng;
    c1 = reduce_parts(nbp + 1, D.NB, TRF_NPF, red) / ng;
  } else if (op == OP_S2) {
    const double nt = sqrt(reduce_parts(nbp + 2, D.NB, TRF_NPF, red));
    c2 = nt > 0 ? 1.0 / nt : 0.0;
  }
  double p0 = 0.0, p1 = 0.0;
  auto one = [&](size_t o) {
    switch (op) {
      case OP_XNORM: p0 += x[o] * x[o]; break;
      case OP_DOTS: p0 += Bf.g[o] * Bf.xl[o]; break;
      case OP_S1T: {
        const double s1 = Bf.g[o] * c0;
        const double tt = Bf.xl[o] - c1 * s1;
        Bf.s1[o] = s1;
        Bf.s2[o] = tt;
        p0 += tt * tt;
        break;
      }
      case OP_S2: {
        const double s2 = Bf.s2[o] * c2;
        Bf.s2[o] = s2;
        p0 += Bf.g[o] * Bf.s1[o];
        p1 += Bf.g[o] * s2;
        break;
      }
      case OP_STEP: {
        const double st = Bf.s1[o] * cf[0] + Bf.s2[o] * cf[1];
        xt[o] = x[o] + st;
        p0 += st * st;
        break;
      }
      default: x[o] = xt[o]; break;
    }
  };
  for (int i = t; i < nf * J3; i += TRF_THREADS) one(nb + (size_t)f0 * J3 + i);
  if (blk == 0 && t < D.NL) {
    const size_t o = nb + D.NX + t;
    if (!D.fix) one(o);
    else if (op == OP_STEP) xt[o] = x[o];  // the fixed lengths ride along
    else if (op == OP_XNORM) p0 += 0.0;
  }
  p0 = block_sum_all(p0, red);
  p1 = block_sum_all(p1, red);
  if (t == 0) {
    const int fld = op <= OP_S2 ? op : 5 + (op - OP_STEP);
    double* np = Bf.npart + ((size_t)b * D.NB + blk) * TRF_NPF + fld;
    np[0] = p0;
    if (op == OP_S2) np[1] = p1;
  }
}

// ---------------------------------------------------------------------------------------------------------
// Host: the 2-D trust-region subproblem (common.py solve_trust_region_2d).  np.roots of the quartic is
// replaced by its real roots found by bracketing between the critical points (the roots of the derivative,
// recursively) and bisecting; a root the polynomial only touches is not bracketed (numpy's companion
// eigenvalues of such a root are a near-real complex pair, excluded there too unless exactly real).
double poly_eval(const double* c, int d, double t) {
  double v = c[0];
  for (int i = 1; i <= d; ++i) v = v * t + c[i];
  return v;
}

void poly_real_roots(const double* cin, int din, std::vector<double>& out) {
  out.clear();
  int s = 0;
  while (s <= din && cin[s] == 0.0) ++s;  // leading zeros (np.roots strips them)
  const int d = din - s;
  if (d <= 0) return;
  const double* c = cin + s;
  if (d == 1) {
    out.push_back(-c[1] / c[0]);
    return;
  }
  if (d == 2) {
    const double disc = c[1] * c[1] - 4 * c[0] * c[2];
    if (disc < 0) return;
    const double q = -0.5 * (c[1] + (c[1] >= 0 ? sqrt(disc) : -sqrt(disc)));
    if (q != 0) {
      out.push_back(q / c[0]);
      out.push_back(c[2] / q);
    } else {
      out.push_back(0.0);
      out.push_back(0.0);
    }
    std::sort(out.begin(), out.end());
    return;
  }
  double dc[8];
  for (int i = 0; i < d; ++i) dc[i] = c[i] * (d - i);
  std::vector<double> crit;
  poly_real_roots(dc, d - 1, crit);
  double R = 0.0;
  for (int i = 1; i <= d; ++i) R = std::max(R, std::fabs(c[i] / c[0]));
  R += 1.0;
  std::vector<double> pts;
  pts.push_back(-R);
  for (double x : crit)
    if (x > -R && x < R) pts.push_back(x);
  pts.push_back(R);
  std::sort(pts.begin(), pts.end());
  for (size_t i = 0; i + 1 < pts.size(); ++i) {
    double a = pts[i], b = pts[i + 1];
    double fa = poly_eval(c, d, a), fb = poly_eval(c, d, b);
    if (fa == 0.0) {
      if (out.empty() || out.back() != a) out.push_back(a);
      continue;
    }
    if (fb == 0.0 || (fa < 0) == (fb < 0)) continue;
    for (int it = 0; it < 200; ++it) {
      const double m = 0.5 * (a + b);
      if (m <= a || m >= b) break;
      const double fm = poly_eval(c, d, m);
      if (fm == 0.0) {
        a = b = m;
        break;
      }
      if ((fm < 0) == (fa < 0)) {
        a = m;
        fa = fm;
      } else {
        b = m;
      }
    }
    out.push_back(0.5 * (a + b));
  }
  if (poly_eval(c, d, pts.back()) == 0.0) out.push_back(pts.back());
}

void solve_trust_region_2d(const double B[3], const double g[2], double Delta, double p[2]) {
  // cho_factor (upper) + cho_solve, p = -B^-1 g, if B is positive definite and p lies inside
  const double b00 = B[0], b01 = B[1], b11 = B[2];
  if (b00 > 0) {
    const double r00 = std::sqrt(b00), r01 = b01 / r00, s = b11 - r01 * r01;
    if (s > 0) {
      const double r11 = std::sqrt(s);
      const double y0 = g[0] / r00, y1 = (g[1] - r01 * y0) / r11;  // R^T y = g
      const double q1 = y1 / r11, q0 = (y0 - r01 * q1) / r00;      // R q = y
      const double pn0 = -q0, pn1 = -q1;
      if (pn0 * pn0 + pn1 * pn1 <= Delta * Delta) {
        p[0] = pn0;
        p[1] = pn1;
        return;
      }
    }
  }
  const double a = b00 * Delta * Delta, b = b01 * Delta * Delta, c = b11 * Delta * Delta;
  const double d = g[0] * Delta, f = g[1] * Delta;
  const double co[5] = {-b + d, 2 * (a - c + f), 6 * b, 2 * (-a + c + f), -b - d};
  std::vector<double> ts;
  poly_real_roots(co, 4, ts);
  if (ts.empty()) {
    // No sign change (numpy's companion eigenvalues would all be complex here, and scipy's argmin over an empty
    // set raises): the quartic's touching points -- critical points where it is zero to rounding -- are the
    // boundary candidates; failing those, the Cauchy point -Delta g / |g|.
    const double dco[4] = {4 * co[0], 3 * co[1], 2 * co[2], co[3]};
    std::vector<double> crit;
    poly_real_roots(dco, 3, crit);
    double scale = 0.0;
    for (double v : co) scale = std::max(scale, std::fabs(v));
    for (double tt : crit) {
      double mag = 0.0;  // |c_i t^(4-i)| summed: the rounding scale of the polynomial's value at t
      for (int i = 0; i <= 4; ++i) mag += std::fabs(co[i]) * std::pow(std::fabs(tt), 4 - i);
      if (std::fabs(poly_eval(co, 4, tt)) <= 64 * 2.220446049250313e-16 * (mag > 0 ? mag : scale)) ts.push_back(tt);
    }
    if (ts.empty()) {
      const double gn = std::sqrt(g[0] * g[0] + g[1] * g[1]);
      p[0] = gn > 0 ? -Delta * g[0] / gn : 0.0;
      p[1] = gn > 0 ? -Delta * g[1] / gn : -Delta;
      return;
    }
  }
  double best = std::numeric_limits<double>::infinity();
  p[0] = 0.0;
  p[1] = -Delta;
  bool any = false;
  for (double tt : ts) {
    const double q0 = Delta * (2 * tt / (1 + tt * tt)), q1 = Delta * ((1 - tt * tt) / (1 + tt * tt));
    const double val = 0.5 * (q0 * (b00 * q0 + b01 * q1) + q1 * (b01 * q0 + b11 * q1)) + (g[0] * q0 + g[1] * q1);
    if (!any || val < best) {
      best = val;
      p[0] = q0;
      p[1] = q1;
      any = true;
    }
  }
}

}  // namespace

}  // namespace mq

extern int mq_fail_host(const std::string& msg, int code);

// The 2-D trust-region subproblem on the host (no HIP call): what optim_points' driver solves each trial step,
// exposed so the CPU tests compare it with the numpy restatement (oracle/trf.py, scipy 1.15.3 common.py).
extern "C" int mq_trust_region_2d(const double* B, const double* g, double Delta, double* p) {
  if (!B || !g || !p) return mq_fail_host("mq_trust_region_2d: null argument", -1);
  if (!(Delta > 0) || !std::isfinite(Delta)) return mq_fail_host("mq_trust_region_2d: Delta must be finite and > 0", -2);
  mq::solve_trust_region_2d(B, g, Delta, p);
  return 0;
}

namespace mq {

int g_optim_trf_chunk = 16;
int g_optim_trf_fb = TRF_FB;

namespace {
constexpr size_t TRF_UP_ARENA = 64 * 1024;
struct TrfHostStage {  // per host thread: pinned staging of optim_points_trf's small transfers (never freed)
  char* up = nullptr;
  size_t up_cap = 0, up_off = 0;
  double* down = nullptr;  // host-mapped, coherent: the partials the host reads, written there by the kernels
  double* down_dev = nullptr;
  size_t down_cap = 0;
  bool dirty = false;  // a call is using the buffers (set at entry, cleared by a call that completes)
};
thread_local TrfHostStage g_trf_stage;
constexpr int TRF_MAX_DEV = 16;
struct TrfDevCache {  // per host thread and device: capture stream, polling events, the lsmr chunk graph
  hipStream_t cap = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipGraphExec_t exec = nullptr;
  int chunk = 0;
  size_t jt_lds = 0, l1_lds = 0;
  TrfDims D{};
  TrfBufs Bf{};
};
thread_local TrfDevCache g_trf_dev[TRF_MAX_DEV];
}  // namespace  // lsmr iterations launched (one captured graph) between two reads of the done flags

// dynamic LDS of the two per-iteration kernels for FB frames per block
size_t trf_jt_lds(int FB, int n, int MR, int J, int C) {
  return ((((size_t)(FB + n) * MR + 1) & ~(size_t)1) + (size_t)FB * J * C * 9) * sizeof(double);
}
size_t trf_l1_lds(int FB, int MR, int J, int C) {
  return ((((size_t)FB * MR + 1) & ~(size_t)1) + (size_t)FB * J * C * 6) * sizeof(double);
}
constexpr size_t TRF_DYN_LDS = 128 * 1024;  // (the kernels' static LDS stays under 24 KB)
// Frames per workgroup.  `fit`: the most (<= TRF_FB and the MQ_TUNE_OPTIM_TRF_FB cap) whose rows fit in LDS.  The
// per-iteration kernels are latency-bound chains, so fewer frames per workgroup shorten each one's chain while
// the grid still has a CU per workgroup: the smallest count whose grid, for TRF_NOMINAL_B animals, fits the
// nominal CUs (TRF_NOMINAL_CUS below), else `fit` (profiles/r05u_*: 24 frames x 4 animals 8 % faster at 1 frame than at 4; 300 x 4,
// which fills the CUs at 4, 60 % slower at 1).  The choice depends on F, not on the batch, so an animal's
// result does not depend on which animals share its call (the reductions follow the blocks).  Monotonic in
// `fit`, so the workspace, sized at the deepest smoothing order, never has fewer blocks than a call.
constexpr int TRF_NOMINAL_B = 4;  // the reference's four individuals
// The block decomposition (frames per workgroup, the length variables' own workgroup) is sized for a nominal
// MI355X (256 CUs), not for the device at hand: the reductions follow the blocks, so an optim_points result
// depends, bit for bit, only on the problem and MQ_TUNE_OPTIM_TRF_FB -- the same on every device and every rank
// of a sharded step 4.  On a device with fewer CUs the same blocks simply take more rounds.
constexpr long long TRF_NOMINAL_CUS = 256;
static int trf_cu_count() { return (int)TRF_NOMINAL_CUS; }
int trf_frames_per_block(int J, int C, int NL, int n, int F) {
  const int MR = (J * C * 2 + J * 3 + NL + 1) & ~1;
  int fit = 1;
  for (int fb = std::min(TRF_FB, std::max(1, g_optim_trf_fb)); fb > 1; --fb)
    if (trf_jt_lds(fb, n, MR, J, C) <= TRF_DYN_LDS && trf_l1_lds(fb, MR, J, C) <= TRF_DYN_LDS) {
      fit = fb;
      break;
    }
  const long long cus = trf_cu_count();
  for (int fb = 1; fb < fit; ++fb)
    if ((long long)TRF_NOMINAL_B * ((F + fb - 1) / fb) <= cus) return fb;
  return fit;
}

size_t optim_trf_workspace_bytes(int B, int F, int J, int C, int NL) {
  const size_t NV = (size_t)F * J * 3 + NL, MR = ((size_t)J * C * 2 + (size_t)J * 3 + NL + 1) & ~(size_t)1;
  const int FB = trf_frames_per_block(J, C, NL, TRF_MAXN, F);
  const size_t NB = ((size_t)F + FB - 1) / FB;
  size_t n = 0;
  n += (size_t)B * F * MR * 3;           // fres ftr u
  n += (size_t)B * F * J * C * 6;        // Jrep
  n += (size_t)B * F * NL * 4;           // lenJ
  n += (size_t)B * NV * 10;              // g vraw vn h hbar xl s1 s2 xt (+1)
  n += (size_t)B * NB * (NL + 2 + 2 + NL) + 4 * (size_t)B * (NB + 1);  // fL upart xpart Lpart vpart (the host-read
                                                                         // partials are host-mapped)
  n += 2 * (size_t)B * TRF_NS + (size_t)B * 8;
  n += (size_t)NL + 2 + 2 * (size_t)B + 16;  // cons, act, done, ssf
  n += ((size_t)J + 1 + 2 * (size_t)NL) / 2 + 1;  // jadj
  return n * sizeof(double) + 256;
}

// Host driver (the trf_no_bounds loop).  x: device (B, NV) in/out.  stats[8 b + ...]: 0 initial cost, 1 final
// cost, 2 iterations (njev - 1), 3 status (scipy's: 0 max_nfev, 1 gtol, 2 ftol, 3 xtol, 4 ftol and xtol),
// 4 nfev, 5 njev, 6 lsmr iterations in total, 7 largest lsmr run.
int optim_points_trf(const double* cams, int C, const double* p2d, double* x, int B, int F, int J, const int* cons_host,
                     int n_strong, int n_weak, const double* ssf_host, double scale_length, double scale_length_weak,
                     double rp, int loss, int n_deriv, int fix_lengths, int max_nfev_arg, double ftol, void* ws,
                     double* stats, hipStream_t s) {
  const int NL = n_strong + n_weak;
  if (B <= 0 || F <= 0 || J <= 0) return 0;
  if (J > TRF_MAXJ || NL > TRF_MAXL || C > 16 || C < 1 || n_deriv < 1 || n_deriv > TRF_MAXN) return -2;
  TrfDims D{};
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
  D.MRrep = J * C * 2;
  D.MR = (D.MRrep + J * 3 + NL + 1) & ~1;  // even: 16-B aligned rows for the LDS staging
  D.FB = trf_frames_per_block(J, C, NL, n_deriv, F);
  D.NB = (F + D.FB - 1) / D.FB;
  D.NBV = (long long)TRF_NOMINAL_B * (D.NB + 1) <= trf_cu_count() ? D.NB + 1 : D.NB;  // (batch-independent too)
  D.rp = rp;
  D.s_len = scale_length;
  D.s_len_weak = scale_length_weak;
  D.atol = 1e-6;
  D.btol = 1e-6;
  D.ctol = 1.0 / 1e8;
  {
    int binom = 1;
    for (int m = 0; m <= n_deriv; ++m) {
      D.c[m] = (((n_deriv - m) & 1) ? -1.0 : 1.0) * binom;
      binom = binom * (n_deriv - m) / (m + 1);
    }
  }
  const int NB = D.NB;
  const size_t NVB = (size_t)B * D.NV, MB = (size_t)B * F * D.MR;
  double* w = static_cast<double*>(ws);
  auto take = [&](size_t cnt) {
    double* p = w;
    w += cnt;
    return p;
  };
  TrfBufs Bf{};
  Bf.fres = take(MB);
  Bf.ftr = take(MB);
  Bf.u = take(MB);
  Bf.Jrep = take((size_t)B * F * J * C * 6);
  Bf.lenJ = take((size_t)B * F * NL * 4);
  Bf.g = take(NVB);
  Bf.vraw = take(NVB);
  Bf.vn = take(NVB);
  Bf.h = take(NVB);
  Bf.hbar = take(NVB);
  Bf.xl = take(NVB);
  Bf.s1 = take(NVB);
  Bf.s2 = take(NVB);
  double* xt = take(NVB);
  Bf.fL = take((size_t)B * NB * NL);
  Bf.upart = take(2 * (size_t)B * NB);
  Bf.vpart = take(2 * (size_t)B * (NB + 1) * 2);
  Bf.xpart = take(2 * (size_t)B * NB);
  Bf.Lpart = take((size_t)B * NB * NL);
  Bf.st = take(2 * (size_t)B * TRF_NS);
  // the host-written inputs, one contiguous run in upload order, so that each group of them the driver sends
  // together (call setup; lsmr setup: lctl, done, act; a trial: act, coef) is one copy
  int* cons_d = reinterpret_cast<int*>(take(((size_t)NL * 2 + 1) / 2 + 1));
  int* jadj_d = reinterpret_cast<int*>(take(((size_t)J + 1 + 2 * (size_t)NL) / 2 + 1));
  double* ssf_d = take(B);
  Bf.lctl = take(4 * (size_t)B);
  int* done_d = reinterpret_cast<int*>(take(((size_t)B + 1) / 2 + 1));
  int* act_d = reinterpret_cast<int*>(take(((size_t)B + 1) / 2 + 1));
  Bf.coef = take(4 * (size_t)B);
  char* const ctl_end = reinterpret_cast<char*>(w);
  Bf.cams = cams;
  Bf.p2d = p2d;
  Bf.cons = cons_d;
  Bf.jadj = jadj_d;
  Bf.ssf = ssf_d;
  Bf.act = act_d;
  Bf.done = done_d;
  // Every small transfer of the driver goes through pinned memory: a copy from or to pageable memory waits for
  // the stream (tens of microseconds per copy, several per trust-region iteration).  Uploads are staged in an
  // arena that is recycled at each stream synchronisation (a copy still queued reads its own slot); downloads
  // land in pinned arrays read after the synchronisation that follows them.
  TrfHostStage& hs = g_trf_stage;
  // (a previous call that failed half way may have left copies from the arena, or kernels writing the host-mapped
  // partials, in flight on its stream)
  if (hs.dirty) (void)hipDeviceSynchronize();
  hs.dirty = true;
  const size_t down_n = (size_t)B * NB * (4 + TRF_NPF + 4) + (size_t)B * (NB + 1) * 2 + 2 * (size_t)B;
  if (hs.up_cap < TRF_UP_ARENA) {
    if (hs.up) (void)hipHostFree(hs.up);
    hs.up = nullptr;
    if (hipHostMalloc((void**)&hs.up, TRF_UP_ARENA, hipHostMallocPortable) != hipSuccess) return -3;
    hs.up_cap = TRF_UP_ARENA;
  }
  if (hs.down_cap < down_n) {
    if (hs.down) (void)hipHostFree(hs.down);
    hs.down = hs.down_dev = nullptr;
    hs.down_cap = 0;
    if (hipHostMalloc((void**)&hs.down, sizeof(double) * down_n,
                      hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) !=
        hipSuccess)
      return -3;
    if (hipHostGetDevicePointer((void**)&hs.down_dev, hs.down, 0) != hipSuccess) return -3;
    hs.down_cap = down_n;
  }
  // the partials the host reads: written by the kernels straight into host memory (no copy, no copy kernel)
  double* hf = hs.down;                      // [B][NB][4] eval: sum r^2 at x, at the trial point, rows
  double* hg = hf + (size_t)B * NB * 4;      // [B][NBV][2] J^T f: |g|^2, max |g| (NBV <= NB + 1)
  double* hn = hg + (size_t)B * (NB + 1) * 2;  // [B][NB][TRF_NPF] n-space operations
  double* hj = hn + (size_t)B * NB * TRF_NPF;  // [B][NB][4] J a, J c products
  double* hitn = hj + (size_t)B * NB * 4;    // [B] lsmr iterations
  volatile int* hdone = reinterpret_cast<volatile int*>(hitn + B);  // [B] lsmr's done flags
  {
    const size_t o_g = (size_t)(hg - hf), o_n = (size_t)(hn - hf), o_j = (size_t)(hj - hf), o_i = (size_t)(hitn - hf);
    Bf.fpart = hs.down_dev;
    Bf.gpart = hs.down_dev + o_g;
    Bf.npart = hs.down_dev + o_n;
    Bf.jpart = hs.down_dev + o_j;
    Bf.hitn = hs.down_dev + o_i;
    Bf.hdone = reinterpret_cast<int*>(hs.down_dev + o_i + B);
  }
  hs.up_off = 0;
  auto sync = [&]() {
    hs.up_off = 0;
    return hipStreamSynchronize(s) == hipSuccess;
  };
  auto H2D = [&](void* d, const void* h, size_t bytes) {
    if (bytes > TRF_UP_ARENA) return false;
    if (hs.up_off + bytes > hs.up_cap && !sync()) return false;
    char* st = hs.up + hs.up_off;
    std::memcpy(st, h, bytes);
    hs.up_off += (bytes + 255) & ~(size_t)255;
    return hipMemcpyAsync(d, st, bytes, hipMemcpyHostToDevice, s) == hipSuccess;
  };
  // several host arrays into the device run [d0, d1) with one copy (the bytes between them are padding)
  struct Seg {
    void* d;
    const void* h;
    size_t bytes;
  };
  auto H2Drun = [&](void* d0, void* d1, std::initializer_list<Seg> segs) {
    const size_t bytes = (size_t)(static_cast<char*>(d1) - static_cast<char*>(d0));
    if (bytes > TRF_UP_ARENA) return false;
    if (hs.up_off + bytes > hs.up_cap && !sync()) return false;
    char* st = hs.up + hs.up_off;
    std::memset(st, 0, bytes);
    for (const Seg& g : segs)
      if (g.bytes) std::memcpy(st + (static_cast<char*>(g.d) - static_cast<char*>(d0)), g.h, g.bytes);
    hs.up_off += (bytes + 255) & ~(size_t)255;
    return hipMemcpyAsync(d0, st, bytes, hipMemcpyHostToDevice, s) == hipSuccess;
  };
  // J^T's constraint terms per joint (trf_jt_kernel): the constraints with the joint as their first end (+) or,
  // failing that, their second end (-), in ascending order of l
  std::vector<int> jadj(J + 1 + 2 * NL, 0);
  for (int j = 0, e = 0; j < J; ++j) {
    jadj[j] = e;
    for (int l = 0; l < NL; ++l) {
      if (cons_host[2 * l] == j) jadj[J + 1 + e++] = 2 * l;
      else if (cons_host[2 * l + 1] == j) jadj[J + 1 + e++] = 2 * l + 1;
    }
    jadj[j + 1] = e;
  }
  std::vector<int> act(B, 1), doneh(B, 1);
  // (lctl, done and coef are sent before their first reads; zeros until then)
  if (!H2Drun(cons_d, ctl_end,
              {{cons_d, cons_host, sizeof(int) * 2 * NL}, {jadj_d, jadj.data(), sizeof(int) * jadj.size()},
               {ssf_d, ssf_host, sizeof(double) * B}, {act_d, act.data(), sizeof(int) * B}}))
    return -3;

  const dim3 grid(NB, B), blk(TRF_THREADS);
  const dim3 gridj(D.NBV, B);  // J^T launches (with the length variables' workgroup when NBV = NB + 1)
  const size_t jt_lds = trf_jt_lds(D.FB, D.n, D.MR, J, C), l1_lds = trf_l1_lds(D.FB, D.MR, J, C);
  {
    static std::atomic<unsigned> attr{0};
    if (first_on_device(attr)) {
      const int mx = (int)TRF_DYN_LDS;
      (void)hipFuncSetAttribute((const void*)trf_jt_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      (void)hipFuncSetAttribute((const void*)trf_jt_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      (void)hipFuncSetAttribute((const void*)trf_jt_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      (void)hipFuncSetAttribute((const void*)trf_lsmr1_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
      (void)hipFuncSetAttribute((const void*)trf_lsmr1_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    }
  }
  if (jt_lds > TRF_DYN_LDS || l1_lds > TRF_DYN_LDS) return -2;
  // lsmr's iterations run as a captured graph of `chunk` (even) iterations, replayed until every done flag is
  // set: the kernels take only the slot parity, so one graph serves every chunk of the call.  Captured on a
  // private stream (the caller's may be the legacy default stream, which cannot be captured), replayed on s.
  // The instantiated graph is kept per host thread and device and reused while the call's dimensions, buffers and
  // chunk are the same (instantiating costs a few hundred microseconds).
  const int chunk = std::max(2, (g_optim_trf_chunk + 1) & ~1);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= TRF_MAX_DEV) return -3;
  TrfDevCache& dc = g_trf_dev[dev];
  if (!dc.cap && hipStreamCreateWithFlags(&dc.cap, hipStreamNonBlocking) != hipSuccess) return -3;
  // (the polling events order nothing but the host's read of the done flags, which a stale read only delays by a
  // chunk: no system-scope cache fence at each chunk boundary)
  for (auto& e : dc.ev)
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
      return -3;
  hipEvent_t* done_ev = dc.ev;
  if (!dc.exec || dc.chunk != chunk || dc.jt_lds != jt_lds || dc.l1_lds != l1_lds ||
      std::memcmp(&dc.D, &D, sizeof(D)) != 0 || std::memcmp(&dc.Bf, &Bf, sizeof(Bf)) != 0) {
    if (dc.exec) (void)hipGraphExecDestroy(dc.exec);
    dc.exec = nullptr;
    hipGraph_t graph = nullptr;
    if (hipStreamBeginCapture(dc.cap, hipStreamCaptureModeThreadLocal) != hipSuccess) return -3;
    for (int i = 0; i < chunk; ++i) {
      hipLaunchKernelGGL(trf_lsmr1_kernel<false>, grid, blk, l1_lds, dc.cap, D, Bf, i & 1);
      hipLaunchKernelGGL(trf_jt_kernel<2>, gridj, blk, jt_lds, dc.cap, D, Bf, i & 1);
    }
    if (hipStreamEndCapture(dc.cap, &graph) != hipSuccess) return -3;
    const bool ok = hipGraphInstantiate(&dc.exec, graph, nullptr, nullptr, 0) == hipSuccess;
    (void)hipGraphDestroy(graph);
    if (!ok) {
      dc.exec = nullptr;
      return -3;
    }
    dc.chunk = chunk;
    dc.jt_lds = jt_lds;
    dc.l1_lds = l1_lds;
    std::memcpy(&dc.D, &D, sizeof(D));
    std::memcpy(&dc.Bf, &Bf, sizeof(Bf));
  }
  const hipGraphExec_t lsmr_exec = dc.exec;
  std::vector<double> ctl(4 * (size_t)B), coef(4 * (size_t)B, 0.0);
  auto upload_act = [&]() { return H2D(act_d, act.data(), sizeof(int) * B); };
  // per-animal sums of a partial field over the blocks (fixed order)
  auto sum_field = [&](const double* p, int stride, int field, int b) {
    double v = 0.0;
    for (int k = 0; k < NB; ++k) v += p[((size_t)b * NB + k) * stride + field];
    return v;
  };
  // At a point p (x, or a trial point), for the animals in act: J, f, cost (mode 1), g = J^T f with its norms,
  // |p|, and J g (the next iteration's `regularize`).  Launched, then read after the next synchronisation.
  std::vector<double> cost(B), gnorm2(B), ginf(B), rows(B), xnorm(B), areg(B);
  auto launch_jac = [&](double* p) {
    hipLaunchKernelGGL(trf_eval_kernel, grid, blk, 0, s, D, Bf, p, Bf.fres, 1);
    hipLaunchKernelGGL(trf_jt_kernel<0>, gridj, blk, jt_lds, s, D, Bf, 0);
    hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, p, xt, (int)OP_XNORM);
    hipLaunchKernelGGL(trf_jv_kernel, grid, blk, 0, s, D, Bf, (const double*)Bf.g, (const double*)nullptr);
  };
  auto read_jac = [&](int b) {
    cost[b] = 0.5 * sum_field(hf, 4, 0, b);
    rows[b] = sum_field(hf, 4, 2, b);
    double gs = 0.0, m = 0.0;
    for (int k = 0; k < D.NBV; ++k) {
      gs += hg[((size_t)b * D.NBV + k) * 2];
      m = std::max(m, hg[((size_t)b * D.NBV + k) * 2 + 1]);
    }
    gnorm2[b] = gs;
    ginf[b] = m;
    xnorm[b] = std::sqrt(sum_field(hn, TRF_NPF, 0, b));
    areg[b] = 0.5 * sum_field(hj, 4, 0, b);
  };
  auto jac_and_grad = [&]() -> bool {
    launch_jac(x);
    if (!sync()) return false;
    for (int b = 0; b < B; ++b) {
      if (!act[b]) continue;
      cost[b] = 0.5 * sum_field(hf, 4, 0, b);
      rows[b] = sum_field(hf, 4, 2, b);
      double gs = 0.0, m = 0.0;
      for (int k = 0; k < D.NBV; ++k) {
        gs += hg[((size_t)b * D.NBV + k) * 2];
        m = std::max(m, hg[((size_t)b * D.NBV + k) * 2 + 1]);
      }
      gnorm2[b] = gs;
      ginf[b] = m;
      xnorm[b] = std::sqrt(sum_field(hn, TRF_NPF, 0, b));
      areg[b] = 0.5 * sum_field(hj, 4, 0, b);
    }
    return true;
  };

  const int nparam = fix_lengths ? D.NX : D.NV;
  const long long max_nfev = max_nfev_arg > 0 ? max_nfev_arg : 100LL * (fix_lengths ? D.NX : D.NV);
  const double xtol = 1e-8, gtol = 1e-8;
  enum { RUN, STOP };
  std::vector<int> state(B, RUN), status(B, 0), lsmr_total(B, 0), lsmr_max(B, 0);
  std::vector<long long> nfev(B, 1), njev(B, 1);
  std::vector<double> Delta(B), damp(B), BS(3 * (size_t)B), gS(2 * (size_t)B), cost_new(B), actual(B);
  if (!jac_and_grad()) return -3;
  for (int b = 0; b < B; ++b) {
    stats[8 * b + 0] = cost[b];
    Delta[b] = xnorm[b] == 0 ? 1.0 : xnorm[b];
  }
  for (;;) {
    bool any = false;
    for (int b = 0; b < B; ++b) {
      act[b] = 0;
      if (state[b] != RUN) continue;
      if (ginf[b] < gtol) status[b] = 1;  // trf.py:463-465 (ftol stops end the loop below)
      if (status[b] != 0 || nfev[b] == max_nfev) {
        state[b] = STOP;
        continue;
      }
      act[b] = 1;
      any = true;
    }
    if (!any) break;
    // regularize: the 1-D quadratic along -g inside the trust region (trf.py:480-484; J g from jac_and_grad)
    for (int b = 0; b < B; ++b) {
      ctl[4 * b] = ctl[4 * b + 1] = ctl[4 * b + 2] = ctl[4 * b + 3] = 0.0;
      doneh[b] = act[b] ? 0 : 1;
      if (!act[b]) continue;
      const double a = areg[b];
      const double bq = -gnorm2[b];
      const double to_tr = Delta[b] / std::sqrt(gnorm2[b]);
      double ag = 0.0 * (a * 0.0 + bq);
      const double y1 = to_tr * (a * to_tr + bq);
      if (y1 < ag) ag = y1;
      if (a != 0) {
        const double ext = -0.5 * bq / a;
        if (0 < ext && ext < to_tr) {
          const double y2 = ext * (a * ext + bq);
          if (y2 < ag) ag = y2;
        }
      }
      const double reg = -ag / (Delta[b] * Delta[b]);
      damp[b] = std::sqrt(0.0 + reg);
      ctl[4 * b] = damp[b];
      ctl[4 * b + 1] = std::sqrt(2.0 * cost[b]);  // norm(f)
      ctl[4 * b + 2] = std::min(rows[b], (double)nparam);
    }
    if (!H2Drun(Bf.lctl, act_d + B,
                {{Bf.lctl, ctl.data(), sizeof(double) * ctl.size()}, {done_d, doneh.data(), sizeof(int) * B},
                 {act_d, act.data(), sizeof(int) * B}}))
      return -3;
    for (int b = 0; b < B; ++b) hdone[b] = doneh[b];  // (no kernel writes it before this iteration's lsmr)
    // lsmr(J, f, damp)
    hipLaunchKernelGGL(trf_jt_kernel<1>, gridj, blk, jt_lds, s, D, Bf, 0);
    hipLaunchKernelGGL(trf_lsmr1_kernel<true>, grid, blk, l1_lds, s, D, Bf, 1);
    hipLaunchKernelGGL(trf_jt_kernel<2>, gridj, blk, jt_lds, s, D, Bf, 1);
    int k = 2;  // the next iteration; every chunk starts at an even one
    double maxit = 0.0;
    for (int b = 0; b < B; ++b)
      if (act[b]) maxit = std::max(maxit, ctl[4 * b + 2]);
    // chunks run back to back: the kernels write the done flags into host memory too, and the host reads them
    // once chunk i - 1 has finished, while chunk i runs (a finished animal's kernels return at once), so no
    // chunk waits on the host
    int ci = 0;
    for (;; ++ci) {
      if (hipGraphLaunch(lsmr_exec, s) != hipSuccess) return -3;
      k += chunk;
      if (hipEventRecord(done_ev[ci & 1], s) != hipSuccess) return -3;
      if (ci == 0) continue;
      if (hipEventSynchronize(done_ev[(ci - 1) & 1]) != hipSuccess) return -3;
      bool all = true;
      for (int b = 0; b < B; ++b) all &= hdone[b] != 0;
      if (all) break;
      if (k > maxit + 4 + 2 * chunk) return -7;  // the device test stops every run by maxiter
    }
    // S = orth([g, gn]) by Gram-Schmidt (its coefficients reduced on the device), g_S and B_S (trf.py:489-493),
    // with one synchronisation
    hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, x, xt, (int)OP_DOTS);
    hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, x, xt, (int)OP_S1T);
    hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, x, xt, (int)OP_S2);
    hipLaunchKernelGGL(trf_jv_kernel, grid, blk, 0, s, D, Bf, (const double*)Bf.s1, (const double*)Bf.s2);
    if (!sync()) return -3;
    for (int b = 0; b < B; ++b) {
      if (!act[b]) continue;
      const int it = (int)hitn[b];
      lsmr_total[b] += it;
      lsmr_max[b] = std::max(lsmr_max[b], it);
      gS[2 * b] = sum_field(hn, TRF_NPF, 3, b);
      gS[2 * b + 1] = sum_field(hn, TRF_NPF, 4, b);
      BS[3 * b] = sum_field(hj, 4, 0, b);
      BS[3 * b + 1] = sum_field(hj, 4, 2, b);
      BS[3 * b + 2] = sum_field(hj, 4, 1, b);
    }
    // the trial steps (trf.py:496-540), every animal until it accepts, terminates or runs out of evaluations
    std::vector<int> trial(B, 0);
    for (int b = 0; b < B; ++b) {
      trial[b] = act[b];
      actual[b] = -1;
    }
    std::vector<double> pred(B), step_norm(B);
    for (;;) {
      bool anyt = false;
      for (int b = 0; b < B; ++b) {
        act[b] = trial[b] && actual[b] <= 0 && nfev[b] < max_nfev;
        trial[b] = act[b];
        if (!act[b]) continue;
        anyt = true;
        double p[2];
        solve_trust_region_2d(&BS[3 * b], &gS[2 * b], Delta[b], p);
        coef[4 * b] = p[0];
        coef[4 * b + 1] = p[1];
        const double q = p[0] * (BS[3 * b] * p[0] + BS[3 * b + 1] * p[1]) + p[1] * (BS[3 * b + 1] * p[0] + BS[3 * b + 2] * p[1]);
        pred[b] = -(0.5 * q + (p[0] * gS[2 * b] + p[1] * gS[2 * b + 1]));
      }
      if (!anyt) break;
      if (!H2Drun(act_d, Bf.coef + coef.size(),
                  {{act_d, act.data(), sizeof(int) * B}, {Bf.coef, coef.data(), sizeof(double) * coef.size()}}))
        return -3;
      hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, x, xt, (int)OP_STEP);
      // the residuals at the trial point with the Jacobian, g, |xt| and J g there, on the bet that the step is
      // accepted (it mostly is): an accepted step then needs no further evaluation or synchronisation.  A
      // rejected one loses nothing the next trial needs (that uses x, s1, s2 and the host's B_S, g_S).
      launch_jac(xt);
      if (!sync()) return -3;
      for (int b = 0; b < B; ++b) {
        if (!act[b]) continue;
        nfev[b]++;
        const double sh = std::sqrt(sum_field(hn, TRF_NPF, 5, b));
        step_norm[b] = sh;
        const double cn = 0.5 * sum_field(hf, 4, 0, b);
        if (!std::isfinite(cn)) {
          Delta[b] = 0.25 * sh;
          actual[b] = -1;
          continue;
        }
        cost_new[b] = cn;
        actual[b] = cost[b] - cn;
        double ratio;
        if (pred[b] > 0) ratio = actual[b] / pred[b];
        else if (pred[b] == actual[b] && actual[b] == 0) ratio = 1;
        else ratio = 0;
        double Dn = Delta[b];
        if (ratio < 0.25) Dn = 0.25 * sh;
        else if (ratio > 0.75 && sh > 0.95 * Delta[b]) Dn *= 2.0;
        const bool ft = actual[b] < ftol * cost[b] && ratio > 0.25;
        const bool xt_ok = sh < xtol * (xtol + xnorm[b]);
        const int term = (ft && xt_ok) ? 4 : ft ? 2 : xt_ok ? 3 : 0;
        if (term) {
          status[b] = term;
          trial[b] = 0;
          continue;
        }
        Delta[b] = Dn;
      }
    }
    // accepted steps: x = x_new, with J, g, |x| and J g at x as the last trial evaluated them (trf.py:522-540)
    bool anya = false;
    for (int b = 0; b < B; ++b) {
      act[b] = state[b] == RUN && actual[b] > 0;
      if (!act[b]) continue;
      anya = true;
      njev[b]++;
      read_jac(b);  // (the partials of the animal's last trial: it stopped trying at its accepted step)
    }
    if (anya) {
      if (!upload_act()) return -3;
      hipLaunchKernelGGL(trf_nops_kernel, grid, blk, 0, s, D, Bf, x, xt, (int)OP_ACCEPT);
    }
  }
#ifdef TRF_PROFILE
  {
    unsigned long long h[2][12];
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_trf_prof), sizeof(h));
    for (int kk = 0; kk < 2; ++kk) {
      const double nn = h[kk][0] ? (double)h[kk][0] : 1.0;
      fprintf(stderr, "trf_prof %s launches %llu us/launch:", kk ? "jt2" : "lsmr1", h[kk][0]);
      for (int k = 1; k < 12; ++k) fprintf(stderr, " %.2f", h[kk][k] / nn / 100.0);  // wall clock: 100 MHz
      fprintf(stderr, "\n");
    }
  }
#endif
  if (!sync()) return -3;  // (the staging arena is the next call's)
  hs.dirty = false;
  for (int b = 0; b < B; ++b) {
    stats[8 * b + 1] = cost[b];
    stats[8 * b + 2] = (double)(njev[b] - 1);
    stats[8 * b + 3] = status[b];
    stats[8 * b + 4] = (double)nfev[b];
    stats[8 * b + 5] = (double)njev[b];
    stats[8 * b + 6] = lsmr_total[b];
    stats[8 * b + 7] = lsmr_max[b];
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace mq
