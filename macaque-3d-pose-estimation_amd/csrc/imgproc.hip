// Crop and heatmap-decode kernels.  Compiled with -ffp-contract=off: every
// floating-point step here follows the operation order of the restated reference
// (oracle/crop.py, oracle/decode.py) so results are bit-reproducible against it.
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

// ------------------------------------------------------------------ UDP crop
// GetBBoxCenterScale(1.25) -> _fix_aspect_ratio(0.75) -> get_udp_warp_matrix ->
// cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) fixed-point -> bgr2rgb ->
// (x - mean) / std.   One block per (output row, box), one thread per output column.
struct BoxWarp {
  float c0, c1, s0, s1;
  double M[6];  // inverse map dst -> src
};

__device__ __forceinline__ BoxWarp box_warp(const float* bb, int out_w, int out_h) {
  BoxWarp w;
  const float x1 = bb[0], y1 = bb[1], x2 = bb[2], y2 = bb[3];
  const float sw = (x2 - x1) * 1.25f, sh = (y2 - y1) * 1.25f;
  w.c0 = (x2 + x1) * 0.5f;
  w.c1 = (y2 + y1) * 0.5f;
  const float ar = 0.75f;
  if (sw > sh * ar) {
    w.s0 = sw;
    w.s1 = sw / ar;
  } else {
    w.s0 = sh * ar;
    w.s1 = sh;
  }
  const double in0 = (double)(w.c0 * 2.0f), in1 = (double)(w.c1 * 2.0f);
  const double s0 = (double)w.s0, s1 = (double)w.s1;
  const double sx = (double)(out_w - 1) / s0;
  const double sy = (double)(out_h - 1) / s1;
  float m[6];
  m[0] = (float)(1.0 * sx);
  m[1] = (float)(-0.0 * sx);
  m[2] = (float)(sx * ((-0.5 * in0 * 1.0 + 0.5 * in1 * 0.0) + 0.5 * s0));
  m[3] = (float)(0.0 * sy);
  m[4] = (float)(1.0 * sy);
  m[5] = (float)(sy * ((-0.5 * in0 * 0.0 - 0.5 * in1 * 1.0) + 0.5 * s1));
  double M[6];
  for (int i = 0; i < 6; ++i) M[i] = (double)m[i];
  double D = M[0] * M[4] - M[1] * M[3];
  D = D != 0 ? 1.0 / D : 0.0;
  const double A11 = M[4] * D, A22 = M[0] * D;
  M[0] = A11;
  M[1] *= -D;
  M[3] *= -D;
  M[4] = A22;
  const double b1 = -M[0] * M[2] - M[1] * M[5];
  const double b2 = -M[3] * M[2] - M[4] * M[5];
  M[2] = b1;
  M[5] = b2;
  for (int i = 0; i < 6; ++i) w.M[i] = M[i];
  return w;
}

__global__ void crop_udp_kernel(const uint8_t* __restrict__ frames, int64_t fstride, int H, int W,
                                const float* __restrict__ boxes, const int32_t* __restrict__ box_frame,
                                float* __restrict__ crops, float* __restrict__ center, float* __restrict__ scale,
                                int out_w, int out_h) {
  const int y = blockIdx.x;
  const int n = blockIdx.y;
  const int x = threadIdx.x;
  const BoxWarp bw = box_warp(boxes + 4 * n, out_w, out_h);
  if (y == 0 && x == 0) {
    center[2 * n] = bw.c0;
    center[2 * n + 1] = bw.c1;
    scale[2 * n] = bw.s0;
    scale[2 * n + 1] = bw.s1;
  }
  if (x >= out_w) return;
  const int X0 = __double2int_rn((bw.M[1] * (double)y + bw.M[2]) * 1024.0) + 16;
  const int Y0 = __double2int_rn((bw.M[4] * (double)y + bw.M[5]) * 1024.0) + 16;
  const int ad = __double2int_rn(bw.M[0] * (double)x * 1024.0);
  const int bd = __double2int_rn(bw.M[3] * (double)x * 1024.0);
  const int X = (X0 + ad) >> 5;
  const int Y = (Y0 + bd) >> 5;
  const int sx = X >> 5, sy = Y >> 5;
  const int fx = X & 31, fy = Y & 31;
  const int w00 = (32 - fy) * (32 - fx) * 32, w01 = (32 - fy) * fx * 32;
  const int w10 = fy * (32 - fx) * 32, w11 = fy * fx * 32;
  const uint8_t* img = frames + (int64_t)box_frame[n] * fstride;
  int acc[3] = {0, 0, 0};
#pragma unroll
  for (int tap = 0; tap < 4; ++tap) {
    const int yy = sy + (tap >> 1), xx = sx + (tap & 1);
    const int wgt = tap == 0 ? w00 : tap == 1 ? w01 : tap == 2 ? w10 : w11;
    if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
      const uint8_t* p = img + ((int64_t)yy * W + xx) * 3;
      acc[0] += p[0] * wgt;
      acc[1] += p[1] * wgt;
      acc[2] += p[2] * wgt;
    }
  }
  const float mean[3] = {123.675f, 116.28f, 103.53f};
  const float stdv[3] = {58.395f, 57.12f, 57.375f};
  const int64_t plane = (int64_t)out_h * out_w;
  float* out = crops + (int64_t)n * 3 * plane + (int64_t)y * out_w + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int v = (acc[2 - c] + 16384) >> 15;  // rgb channel c = bgr channel 2-c
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    out[c * plane] = ((float)v - mean[c]) / stdv[c];
  }
}

int crop_udp(const uint8_t* frames, int64_t frame_stride, int img_h, int img_w, const float* boxes,
             const int32_t* box_frame, int n, float* crops, float* center, float* scale, hipStream_t s) {
  if (n <= 0) return 0;
  const int out_w = 192, out_h = 256;
  hipLaunchKernelGGL(crop_udp_kernel, dim3(out_h, n), dim3(256), 0, s, frames, frame_stride, img_h, img_w, boxes,
                     box_frame, crops, center, scale, out_w, out_h);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------ flip average
// avg[n][k][y][x] = (h[n][k][y][x] + h[n + N][fi[k]][y][W-1-x]) * 0.5
__global__ void flip_average_kernel(const float* __restrict__ hm, float* __restrict__ avg, int N, int K, int HH,
                                    int WW, const int32_t* __restrict__ fi) {
  const int64_t plane = (int64_t)HH * WW;
  const int64_t total = (int64_t)N * K * plane;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % WW);
    const int y = (int)((i / WW) % HH);
    const int k = (int)((i / plane) % K);
    const int n = (int)(i / (plane * K));
    const float a = hm[i];
    const float b = hm[(((int64_t)(n + N) * K + fi[k]) * HH + y) * WW + (WW - 1 - x)];
    avg[i] = (a + b) * 0.5f;
  }
}

int flip_average(const float* hm_all, float* avg, int n, int joints, int h, int w, const int32_t* flip_idx,
                 hipStream_t s) {
  const int64_t total = (int64_t)n * joints * h * w;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(flip_average_kernel, dim3(blocks), dim3(256), 0, s, hm_all, avg, n, joints, h, w, flip_idx);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ------------------------------------------------------------------ UDP / DARK-UDP decode
// The 11-tap Gaussian of cv2.getGaussianKernel(11, sigma 0 -> 2.0), computed in
// float64 and rounded to float32 (oracle/decode.py:gaussian_kernel_1d; a CPU
// test pins this table against it).
__constant__ float kGauss11[11] = {
    0.00881222914904356f, 0.027143577113747597f, 0.06511405855417252f, 0.12164907157421112f,
    0.17699836194515228f, 0.2005654126405716f,   0.17699836194515228f, 0.12164907157421112f,
    0.06511405855417252f, 0.027143577113747597f, 0.00881222914904356f};

// Stage 1: one block per (instance, joint): first argmax, separable blur of the
// 5-px zero-padded map, rescale to the original max, clip [1e-3, 50], log.
__global__ __launch_bounds__(256) void decode_blur_kernel(const float* __restrict__ avg, int K, int HH, int WW,
                                                          float* __restrict__ work, int32_t* __restrict__ argmax,
                                                          float* __restrict__ score) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int nk = blockIdx.x;
  const int plane = HH * WW;
  const int PR = HH + 10;  // padded rows
  float* hmap = sm;                 // HH*WW
  float* rows = sm + plane;         // PR*WW (row-filtered padded rows)
  __shared__ float red_v[256];
  __shared__ int red_i[256];
  const float* src = avg + (int64_t)nk * plane;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < plane; i += blockDim.x) {
    const float v = src[i];
    hmap[i] = v;
    if (v > bv || (v == bv && i < bi) || (v != v && bv == bv)) {  // NaN counts as max (np.argmax)
      bv = v;
      bi = i;
    }
  }
  red_v[threadIdx.x] = bv;
  red_i[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      const float v2 = red_v[threadIdx.x + o];
      const int i2 = red_i[threadIdx.x + o];
      const float v1 = red_v[threadIdx.x];
      const int i1 = red_i[threadIdx.x];
      const bool n1 = v1 != v1, n2 = v2 != v2;
      bool take2;
      if (n1 || n2)
        take2 = n2 && (!n1 || i2 < i1);
      else
        take2 = (v2 > v1) || (v2 == v1 && i2 < i1);
      if (take2) {
        red_v[threadIdx.x] = v2;
        red_i[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  const float origin_max = red_v[0];
  if (threadIdx.x == 0) {
    argmax[nk] = red_i[0];
    score[nk] = origin_max;
  }
  // row pass over the padded map: rows[r][x] = sum_t g[t] * dr[r][x + t]
  for (int i = threadIdx.x; i < PR * WW; i += blockDim.x) {
    const int r = i / WW, x = i % WW;
    const int yy = r - 5;
    float acc;
    if (yy < 0 || yy >= HH) {
      acc = 0.f;
    } else {
      const float* hr = hmap + yy * WW;
      // padded column x + t  <->  original column x + t - 5
      int c = x - 5;
      acc = kGauss11[0] * ((c >= 0 && c < WW) ? hr[c] : 0.f);
      for (int t = 1; t < 11; ++t) {
        c = x + t - 5;
        acc = acc + kGauss11[t] * ((c >= 0 && c < WW) ? hr[c] : 0.f);
      }
    }
    rows[i] = acc;
  }
  __syncthreads();
  // column pass -> blurred (stored back into hmap), track its max
  float lmax = -INFINITY;
  for (int i = threadIdx.x; i < plane; i += blockDim.x) {
    const int y = i / WW, x = i % WW;
    float acc = kGauss11[0] * rows[y * WW + x];
    for (int t = 1; t < 11; ++t) acc = acc + kGauss11[t] * rows[(y + t) * WW + x];
    hmap[i] = acc;
    lmax = fmaxf(lmax, acc);
  }
  __syncthreads();
  red_v[threadIdx.x] = lmax;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red_v[threadIdx.x] = fmaxf(red_v[threadIdx.x], red_v[threadIdx.x + o]);
    __syncthreads();
  }
  const float ratio = origin_max / red_v[0];
  float* dst = work + (int64_t)nk * plane;
  for (int i = threadIdx.x; i < plane; i += blockDim.x) {
    float v = hmap[i] * ratio;
    v = fminf(fmaxf(v, 0.001f), 50.0f);
    dst[i] = logf(v);
  }
}

// Element of numpy's flattened edge-padded (K, H+2, W+2) log map with Python
// negative-index wrap-around (refine_keypoints_dark_udp reads through it for
// joints whose max <= 0, loc = -1).
__device__ __forceinline__ float padded_at(const float* work_inst, int K, int HH, int WW, long idx) {
  const long per = (long)(HH + 2) * (WW + 2);
  const long total = per * K;
  if (idx < 0) idx += total;
  const int k = (int)(idx / per);
  const int rem = (int)(idx % per);
  int pr = rem / (WW + 2) - 1, pc = rem % (WW + 2) - 1;
  pr = pr < 0 ? 0 : (pr >= HH ? HH - 1 : pr);
  pc = pc < 0 ? 0 : (pc >= WW ? WW - 1 : pc);
  return work_inst[((long)k * HH + pr) * WW + pc];
}

// Stage 2: one thread per (instance, joint): DARK-UDP Newton step (float32
// derivatives, float64 Hessian inverse), heatmap -> input -> image space.
__global__ void decode_refine_kernel(const float* __restrict__ work, const int32_t* __restrict__ argmax,
                                     const float* __restrict__ score, int N, int K, int HH, int WW,
                                     const float* __restrict__ center, const float* __restrict__ scale, int in_w,
                                     int in_h, double* __restrict__ kp_img, float* __restrict__ kp_hm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * K) return;
  const int n = i / K, k = i % K;
  const float* wi = work + (long)n * K * HH * WW;
  float lx, ly;
  if (score[i] <= 0.f) {
    lx = -1.f;
    ly = -1.f;
  } else {
    lx = (float)(argmax[i] % WW);
    ly = (float)(argmax[i] / WW);
  }
  const int W2 = WW + 2;
  const float fidx = lx + 1.f + (ly + 1.f) * (float)W2;
  const long index = (long)fidx + (long)W2 * (HH + 2) * k;
  const float i_ = padded_at(wi, K, HH, WW, index);
  const float ix1 = padded_at(wi, K, HH, WW, index + 1);
  const float iy1 = padded_at(wi, K, HH, WW, index + W2);
  const float ix1y1 = padded_at(wi, K, HH, WW, index + W2 + 1);
  const float ix1_y1_ = padded_at(wi, K, HH, WW, index - W2 - 1);
  const float ix1_ = padded_at(wi, K, HH, WW, index - 1);
  const float iy1_ = padded_at(wi, K, HH, WW, index - W2);
  const float dx = 0.5f * (ix1 - ix1_);
  const float dy = 0.5f * (iy1 - iy1_);
  const float dxx = ix1 - 2.f * i_ + ix1_;
  const float dxy = 0.5f * (ix1y1 - ix1 - iy1 + i_ + i_ - ix1_ - iy1_ + ix1_y1_);
  const float dyy = iy1 - 2.f * i_ + iy1_;
  const double eps = 1.1920928955078125e-07;
  // inv([[a b][c d]]) by LU with partial pivoting (LAPACK getrf/getrs order)
  double a = (double)dxx + eps, b = (double)dxy + 0.0, c = (double)dxy + 0.0, d = (double)dyy + eps;
  bool swap = fabs(c) > fabs(a);
  double p = swap ? c : a, q = swap ? d : b, r = swap ? a : c, s = swap ? b : d;
  const double l = r * (1.0 / p);
  const double u22 = s - l * q;
  double inv[2][2];
  for (int j = 0; j < 2; ++j) {
    double b1 = (j == 0) ? (swap ? 0.0 : 1.0) : (swap ? 1.0 : 0.0);
    double b2 = (j == 0) ? (swap ? 1.0 : 0.0) : (swap ? 0.0 : 1.0);
    b2 = b2 - l * b1;
    b2 = b2 / u22;
    b1 = b1 - b2 * q;
    b1 = b1 / p;
    inv[0][j] = b1;
    inv[1][j] = b2;
  }
  const double stx = inv[0][0] * (double)dx + inv[0][1] * (double)dy;
  const double sty = inv[1][0] * (double)dx + inv[1][1] * (double)dy;
  const float kx = (float)((double)lx - stx);
  const float ky = (float)((double)ly - sty);
  if (kp_hm) {
    kp_hm[2 * i] = kx;
    kp_hm[2 * i + 1] = ky;
  }
  const double ix = (double)kx / (double)(WW - 1) * (double)in_w;
  const double iy = (double)ky / (double)(HH - 1) * (double)in_h;
  const float s0 = scale[2 * n], s1 = scale[2 * n + 1];
  const float h0 = 0.5f * s0, h1 = 0.5f * s1;
  kp_img[2 * i] = ix / (double)in_w * (double)s0 + (double)center[2 * n] - (double)h0;
  kp_img[2 * i + 1] = iy / (double)in_h * (double)s1 + (double)center[2 * n + 1] - (double)h1;
}

int udp_decode(const float* avg, int n, int joints, int h, int w, const float* center, const float* scale, int in_w,
               int in_h, float* work, double* kp_img, float* score, int32_t* argmax, float* kp_hm, hipStream_t s) {
  if (n <= 0) return 0;
  const size_t lds = (size_t)(h * w + (h + 10) * w) * sizeof(float);
  hipLaunchKernelGGL(decode_blur_kernel, dim3(n * joints), dim3(256), lds, s, avg, joints, h, w, work, argmax, score);
  const int tot = n * joints;
  hipLaunchKernelGGL(decode_refine_kernel, dim3((tot + 127) / 128), dim3(128), 0, s, work, argmax, score, n, joints, h,
                     w, center, scale, in_w, in_h, kp_img, kp_hm);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
