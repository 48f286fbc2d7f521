// Host-side initialisation of optim_points (cameras.py:1116-1150 + _initialize_params_triangulation
// :1670-1697), bit for bit the numpy arithmetic the reference runs before its solver:
//
//   * NaN gaps of every (joint, axis) series filled by np.interp over the frame index (edge values
//     outside the known range; an all-NaN series becomes 0)                       (interpolate_data)
//   * scale_smooth_full = scale_smooth / mean|diff(medfilt7(series))| -- medfilt_data's reflect pad by
//     size + 5, zero-padded 7-wide running median, and np.mean's summation order over the array laid out
//     frames-fastest: 8192-element buffered chunks, each summed pairwise (numpy's pairwise_sum)
//   * limb lengths: per constraint the median over frames of the 3D distance ((dx^2 + dy^2) + dz^2 under
//     the square root, as np.linalg.norm reduces), 0 -> median of all, > median + 5 MAD -> median
//   * x0 = [interpolated p3d, strong lengths, weak lengths], non-finite -> 0
//
// Pure host code (no HIP call), compiled without FMA contraction so that every expression rounds as
// numpy's does.  One thread per animal for long clips (>= ~1200 frames).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "mq_hip.h"

namespace {

constexpr long NPY_BUFSIZE = 8192;   // numpy's default ufunc buffer (reductions are chunked by it)
constexpr long PW_BLOCKSIZE = 128;

// numpy's pairwise_sum_DOUBLE (unit stride)
double pairwise_sum(const double* a, long n) {
  if (n < 8) {
    double res = 0.;
    for (long i = 0; i < n; ++i) res += a[i];
    return res;
  }
  if (n <= PW_BLOCKSIZE) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    long i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  long n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// np.mean of a contiguous buffer (reduction buffered in NPY_BUFSIZE chunks)
double np_mean(const std::vector<double>& v) {
  double s = 0.;
  for (long i = 0; i < (long)v.size(); i += NPY_BUFSIZE)
    s += pairwise_sum(v.data() + i, std::min(NPY_BUFSIZE, (long)v.size() - i));
  return s / (double)v.size();
}

// np.median of n finite values (destroys v): middle value, or the mean of the two middle values
double np_median(double* v, long n) {
  if (n <= 0) return NAN;
  for (long i = 0; i < n; ++i)
    if (std::isnan(v[i])) return NAN;
  const long k = n / 2;
  std::nth_element(v, v + k, v + n);
  const double hi = v[k];
  if (n % 2) return hi;
  const double lo = *std::max_element(v, v + k);
  return (lo + hi) / 2.0;
}

// np.interp of the NaN positions of one series (stride s): xp / fp = the finite frames
void interpolate_series(double* x, long F, long s) {
  long first = -1, last = -1;
  for (long f = 0; f < F; ++f)
    if (!std::isnan(x[f * s])) {
      if (first < 0) first = f;
      last = f;
    }
  if (first < 0) {
    for (long f = 0; f < F; ++f) x[f * s] = 0.0;
    return;
  }
  long prev = -1;   // last finite frame before f
  for (long f = 0; f < F; ++f) {
    if (!std::isnan(x[f * s])) {
      prev = f;
      continue;
    }
    if (f < first) {
      x[f * s] = x[first * s];          // left = fp[0]
      continue;
    }
    if (f > last) {
      x[f * s] = x[last * s];           // right = fp[-1]
      continue;
    }
    long next = f + 1;
    while (std::isnan(x[next * s])) ++next;
    const double x0 = (double)prev, x1 = (double)next, y0 = x[prev * s], y1 = x[next * s];
    const double slope = (y1 - y0) / (x1 - x0);
    double r = slope * ((double)f - x0) + y0;
    if (std::isnan(r)) {
      r = slope * ((double)f - x1) + y1;
      if (std::isnan(r) && y0 == y1) r = y0;
    }
    x[f * s] = r;   // written after next was found: later NaN frames interpolate between finite frames
  }
}

// the middle of 7 values by the optimal 16-comparator sorting network (the values are finite here:
// every series is gap-filled first); the median is one of the inputs, so any exact sort gives it
inline double median7(const double* in) {
  double a[7] = {in[0], in[1], in[2], in[3], in[4], in[5], in[6]};
  auto cx = [&](int i, int j) {
    const double lo = a[i] < a[j] ? a[i] : a[j], hi = a[i] < a[j] ? a[j] : a[i];
    a[i] = lo;
    a[j] = hi;
  };
  cx(0, 6); cx(2, 3); cx(4, 5);
  cx(0, 2); cx(1, 4); cx(3, 6);
  cx(0, 1); cx(2, 5); cx(3, 4);
  cx(1, 2); cx(4, 6);
  cx(2, 3); cx(4, 5);
  cx(1, 2); cx(3, 4); cx(5, 6);
  return a[3];
}

// medfilt_data (cameras.py:129-133): reflect pad by size + 5, zero pad size // 2, running median.
// v: scratch of at least F + 2 (size + 5) + 2 (size / 2) doubles.
void median_filter(const double* x, long F, long s, int size, double* out, double* v) {
  const long pad = size + 5, h = size / 2;
  const long n = F + 2 * pad;
  for (long i = 0; i < h; ++i) v[i] = v[n + h + i] = 0.0;
  for (long i = 0; i < n; ++i) {
    long j = i - pad;   // np.pad mode="reflect" (no edge repeat)
    const long period = 2 * (F - 1);
    if (F == 1) {
      j = 0;
    } else {
      j = ((j % period) + period) % period;
      if (j >= F) j = period - j;
    }
    v[i + h] = x[j * s];
  }
  if (size == 7) {
    for (long f = 0; f < F; ++f) out[f] = median7(v + f + pad);   // window centre f + pad
    return;
  }
  std::vector<double> w(size);
  for (long f = 0; f < F; ++f) {
    const long c = f + pad;   // window centre in the reflect-padded array
    for (int k = 0; k < size; ++k) w[k] = v[c + k];
    std::sort(w.begin(), w.end());
    out[f] = w[size / 2];
  }
}

void prepare_one(const double* p3d, long F, long J, const int32_t* cons, int nS, int nW, double scale_smooth,
                 double* x0, double* ssf) {
  const long NV = F * J * 3;
  std::vector<double> intp(p3d, p3d + NV);
  for (long i = 0; i < J * 3; ++i) {
    bool gap = false;
    for (long f = 0; f < F && !gap; ++f) gap = std::isnan(intp[f * J * 3 + i]);
    if (gap) interpolate_series(intp.data() + i, F, J * 3);
  }
  // smoothness scale: medfilt per series, |diff| laid out [joint][axis][frame]
  std::vector<double> med(F), dif, scratch(F + 2 * (7 + 5) + 2 * (7 / 2));
  dif.reserve((size_t)std::max<long>(F - 1, 0) * J * 3);
  for (long i = 0; i < J * 3; ++i) {
    median_filter(intp.data() + i, F, J * 3, 7, med.data(), scratch.data());
    for (long f = 0; f + 1 < F; ++f) dif.push_back(std::fabs(med[f + 1] - med[f]));
  }
  const double m = dif.empty() ? NAN : np_mean(dif);
  *ssf = scale_smooth * (1.0 / m);
  // limb lengths
  const int nC = nS + nW;
  std::vector<double> len(nC), col(F);
  for (int c = 0; c < nC; ++c) {
    const long a = cons[2 * c], b = cons[2 * c + 1];
    for (long f = 0; f < F; ++f) {
      const double* pa = intp.data() + (f * J + a) * 3;
      const double* pb = intp.data() + (f * J + b) * 3;
      const double dx = pa[0] - pb[0], dy = pa[1] - pb[1], dz = pa[2] - pb[2];
      col[f] = std::sqrt((dx * dx + dy * dy) + dz * dz);
    }
    len[c] = np_median(col.data(), F);
  }
  if (nC > 0) {
    std::vector<double> tmp(len);
    double md = np_median(tmp.data(), nC);
    if (md == 0) md = 1e-3;
    for (int c = 0; c < nC; ++c) tmp[c] = std::fabs(len[c] - md);
    const double mad = np_median(tmp.data(), nC);
    for (int c = 0; c < nC; ++c) {
      if (len[c] == 0) len[c] = md;
      if (len[c] > md + mad * 5) len[c] = md;
    }
  }
  for (long i = 0; i < NV; ++i) x0[i] = std::isfinite(intp[i]) ? intp[i] : 0.0;
  for (int c = 0; c < nC; ++c) x0[NV + c] = std::isfinite(len[c]) ? len[c] : 0.0;
}

}  // namespace

extern int mq_fail_host(const std::string& msg, int code);

extern "C" int mq_optim_prepare(const double* p3ds, int B, int F, int J, const int32_t* constraints, int n_strong,
                                int n_weak, double scale_smooth, double* x0, double* ssf) {
  if (!p3ds || !x0 || !ssf) return mq_fail_host("mq_optim_prepare: null argument", -1);
  if (B < 0 || F < 0 || J < 0 || n_strong < 0 || n_weak < 0) return mq_fail_host("mq_optim_prepare: negative size", -2);
  if (n_strong + n_weak > 0 && !constraints) return mq_fail_host("mq_optim_prepare: null constraints", -1);
  for (int k = 0; k < 2 * (n_strong + n_weak); ++k)
    if (constraints[k] < 0 || constraints[k] >= J) return mq_fail_host("mq_optim_prepare: constraint joint out of range", -2);
  const long nx = (long)F * J * 3 + n_strong + n_weak;
  std::vector<std::thread> pool;
  for (int b = 0; b < B; ++b) {
    auto job = [=]() {
      prepare_one(p3ds + (size_t)b * F * J * 3, F, J, constraints, n_strong, n_weak, scale_smooth, x0 + (size_t)b * nx,
                  ssf + b);
    };
    if (B == 1 || (long)F * J < 20000)  // ~0.3 ms per animal at 300 frames: threads cost more than they save
      job();
    else
      pool.emplace_back(job);
  }
  for (auto& t : pool) t.join();
  return 0;
}
