// Step-1 ID classifier kernels: the patch preprocessing of classify_patches + mmpretrain's test
// pipeline, and the non-GEMM layers of the ResNet-152 collar-ID model
// (model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py:41-73; step1_proc2d.py:140-163).
// The convolutions are im2col + mq_gemm_bf16 (bias = folded BatchNorm, ReLU epilogue); the host side
// (mqhip/resnet_id.py) sequences them.  Activations are NHWC: bf16 between convolutions, the
// residual stream of each stage in f32.
#include "common.hpp"
#include "idcls.hpp"

namespace mq {
namespace {

constexpr float ID_MEAN[3] = {123.675f, 116.28f, 103.53f};  // RGB (data_preprocessor, to_rgb=True)
constexpr float ID_STD[3] = {58.395f, 57.12f, 57.375f};

// cv::resize INTER_LINEAR coefficients of one output index (resize.cpp, fixed point, 11-bit weights):
// fx = (float)((d + 0.5) * scale - 0.5) with scale = 1 / (dst / src), floor, clamp to the border.
__device__ __forceinline__ void lin_coef(int d, int src, int dst, int& s0, int& s1, int& a0, int& a1) {
  const double scale = 1.0 / ((double)dst / (double)src);
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) f = 0.f, s = 0;
  if (s >= src - 1) f = 0.f, s = src - 1;
  s0 = s;
  s1 = min(s + 1, src - 1);
  a0 = (int)rintf((1.f - f) * 2048.f);
  a1 = (int)rintf(f * 2048.f);
}

// the u8 vertical pass of cv2's INTER_LINEAR (VResizeLinearVec_32s8u rounding)
__device__ __forceinline__ int lin_vert(int h0, int h1, int b0, int b1) {
  const int v = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
  return min(max((v + 2) >> 2, 0), 255);
}

// patches: box b = (frame, x0, y0, x1, y1), the numpy slice img[y0:y1, x0:x1] (non-empty) ->
// cv2.resize(patch, (out_size, out_size), INTER_LINEAR) u8 (n, out, out, 3).  An exact 2x
// downscale takes cv2's INTER_AREA fast path (mean of the 2x2 block, +2 >> 2).
__global__ __launch_bounds__(256) void id_crop_resize_kernel(const uint8_t* __restrict__ frames, int64_t fstride,
                                                             int W, const int32_t* __restrict__ boxes, int n,
                                                             int out_size, uint8_t* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)out_size * out_size;
  if (idx >= n * per) return;
  const int b = (int)(idx / per);
  const int p = (int)(idx - (int64_t)b * per);
  const int dy = p / out_size, dx = p - (p / out_size) * out_size;
  const int32_t* bx = boxes + 5 * b;
  const uint8_t* f = frames + bx[0] * fstride;
  const int x0 = bx[1], y0 = bx[2];
  const int sw = bx[3] - bx[1], sh = bx[4] - bx[2];
  uint8_t* o = out + ((int64_t)b * per + p) * 3;
  auto px = [&](int y, int x, int c) { return (int)f[((int64_t)(y0 + y) * W + (x0 + x)) * 3 + c]; };
  if (sw == 2 * out_size && sh == 2 * out_size) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
      o[c] = (uint8_t)((px(2 * dy, 2 * dx, c) + px(2 * dy, 2 * dx + 1, c) + px(2 * dy + 1, 2 * dx, c) +
                        px(2 * dy + 1, 2 * dx + 1, c) + 2) >> 2);
    return;
  }
  int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
  lin_coef(dx, sw, out_size, sx0, sx1, a0, a1);
  lin_coef(dy, sh, out_size, sy0, sy1, b0, b1);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int h0 = px(sy0, sx0, c) * a0 + px(sy0, sx1, c) * a1;
    const int h1 = px(sy1, sx0, c) * a0 + px(sy1, sx1, c) * a1;
    o[c] = (uint8_t)lin_vert(h0, h1, b0, b1);
  }
}

// ResizeEdge(scale=edge, edge='short') of a square in_size image (cv2 INTER_LINEAR to edge x edge),
// CenterCrop(crop) at offset round((edge - crop) / 2), BGR -> RGB, (x - mean) / std -> bf16 NHWC
// (n, crop, crop, 3).
__global__ __launch_bounds__(256) void id_edge_crop_kernel(const uint8_t* __restrict__ in, int n, int in_size,
                                                           int edge, int crop, int off, bf16_t* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)crop * crop;
  if (idx >= n * per) return;
  const int b = (int)(idx / per);
  const int p = (int)(idx - (int64_t)b * per);
  const int dy = p / crop + off, dx = p - (p / crop) * crop + off;
  int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
  lin_coef(dx, in_size, edge, sx0, sx1, a0, a1);
  lin_coef(dy, in_size, edge, sy0, sy1, b0, b1);
  const uint8_t* s = in + (int64_t)b * in_size * in_size * 3;
  bf16_t* o = out + ((int64_t)b * per + p) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {  // output channel c (RGB) reads source channel 2 - c (BGR)
    const int sc = 2 - c;
    const int h0 = (int)s[(sy0 * in_size + sx0) * 3 + sc] * a0 + (int)s[(sy0 * in_size + sx1) * 3 + sc] * a1;
    const int h1 = (int)s[(sy1 * in_size + sx0) * 3 + sc] * a0 + (int)s[(sy1 * in_size + sx1) * 3 + sc] * a1;
    o[c] = f32_to_bf16(((float)lin_vert(h0, h1, b0, b1) - ID_MEAN[c]) / ID_STD[c]);
  }
}

// im2col of a bf16 NHWC map for a kh x kw / stride / zero-pad convolution: out (n * oh * ow, kpad) with
// k = (ky * kw + kx) * c + ch, zero for padding taps and k >= kh * kw * c.  Channels in groups of 8
// (16-B moves) when c % 8 == 0.
__global__ __launch_bounds__(256) void im2col_bf16_kernel(const bf16_t* __restrict__ x, int n, int h, int w, int c,
                                                          int kh, int kw, int stride, int pad, int oh, int ow, int kpad,
                                                          bf16_t* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool vec = (c & 7) == 0 && (kpad & 7) == 0;
  const int gk = vec ? kpad / 8 : kpad;
  const int64_t rows = (int64_t)n * oh * ow;
  if (idx >= rows * gk) return;
  const int64_t row = idx / gk;
  const int kg = (int)(idx - row * gk);
  const int img = (int)(row / ((int64_t)oh * ow));
  const int rp = (int)(row - (int64_t)img * oh * ow);
  const int oy = rp / ow, ox = rp - (rp / ow) * ow;
  const int k = vec ? kg * 8 : kg;
  if (k >= kh * kw * c) {
    if (vec)
      *reinterpret_cast<uint4*>(out + row * kpad + k) = make_uint4(0, 0, 0, 0);
    else
      out[row * kpad + k] = 0;
    return;
  }
  const int tap = k / c, ch = k - (k / c) * c;
  const int ky = tap / kw, kx = tap - (tap / kw) * kw;
  const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
  const bool in = iy >= 0 && iy < h && ix >= 0 && ix < w;
  const bf16_t* src = x + (((int64_t)img * h + iy) * w + ix) * c + ch;
  if (vec)
    *reinterpret_cast<uint4*>(out + row * kpad + k) = in ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
  else
    out[row * kpad + k] = in ? *src : (bf16_t)0;
}

__device__ __forceinline__ float bf16_to_f32(bf16_t v) { return __uint_as_float((unsigned)v << 16); }

// MaxPool2d(3, stride 2, padding 1) on bf16 NHWC (padding never wins)
__global__ __launch_bounds__(256) void maxpool3s2_kernel(const bf16_t* __restrict__ x, int n, int h, int w, int c,
                                                         int oh, int ow, bf16_t* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= (int64_t)n * oh * ow * c) return;
  const int ch = (int)(idx % c);
  const int64_t pix = idx / c;
  const int ox = (int)(pix % ow), oy = (int)((pix / ow) % oh), img = (int)(pix / ((int64_t)ow * oh));
  float m = -INFINITY;
  bf16_t best = 0;
  for (int ky = 0; ky < 3; ++ky) {
    const int iy = oy * 2 - 1 + ky;
    if (iy < 0 || iy >= h) continue;
    for (int kx = 0; kx < 3; ++kx) {
      const int ix = ox * 2 - 1 + kx;
      if (ix < 0 || ix >= w) continue;
      const bf16_t v = x[(((int64_t)img * h + iy) * w + ix) * c + ch];
      const float fv = bf16_to_f32(v);
      if (fv > m) m = fv, best = v;
    }
  }
  out[idx] = best;
}

// x = relu(x) in place (f32 residual stream) and y = bf16(x) (the next convolution's operand)
__global__ __launch_bounds__(256) void relu_bf16_kernel(float* __restrict__ x, bf16_t* __restrict__ y, int64_t n4) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  float4 v = reinterpret_cast<float4*>(x)[i];
  v.x = fmaxf(v.x, 0.f);
  v.y = fmaxf(v.y, 0.f);
  v.z = fmaxf(v.z, 0.f);
  v.w = fmaxf(v.w, 0.f);
  reinterpret_cast<float4*>(x)[i] = v;
  reinterpret_cast<uint2*>(y)[i] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
}

// GlobalAveragePooling + LinearClsHead.fc + softmax, one block per image: x f32 (n, hw, c) ->
// logits / probs f32 (n, ncls).  Fixed-order reductions.
__global__ __launch_bounds__(1024) void gap_fc_softmax_kernel(const float* __restrict__ x, int hw, int c,
                                                              const float* __restrict__ fc_w,
                                                              const float* __restrict__ fc_b, int ncls,
                                                              float* __restrict__ logits, float* __restrict__ probs) {
  extern __shared__ float sh_id[];
  float* pooled = sh_id;      // [c]
  float* red = sh_id + c;     // [1024]
  const int b = blockIdx.x, t = threadIdx.x;
  const float* xb = x + (int64_t)b * hw * c;
  // channels t and t + 1024 together, 8 pixels of each per batch of loads (16 loads in flight); every
  // channel still sums its pixels in ascending order
  for (int ch0 = t; ch0 < c; ch0 += 2048) {
    const int ch1 = ch0 + 1024;
    const bool has1 = ch1 < c;
    float s0 = 0.f, s1 = 0.f;
    for (int p0 = 0; p0 < hw; p0 += 8) {
      float v0[8], v1[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int pp = p0 + u;
        v0[u] = pp < hw ? xb[(int64_t)pp * c + ch0] : 0.f;
        v1[u] = (pp < hw && has1) ? xb[(int64_t)pp * c + ch1] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (p0 + u < hw) {
          s0 += v0[u];
          s1 += v1[u];
        }
    }
    pooled[ch0] = s0 / (float)hw;
    if (has1) pooled[ch1] = s1 / (float)hw;
  }
  __syncthreads();
  float lg[ID_MAX_CLASSES];
  for (int k = 0; k < ncls; ++k) {
    float s = 0.f;
    for (int ch = t; ch < c; ch += 1024) s += fc_w[(int64_t)k * c + ch] * pooled[ch];
    red[t] = s;
    __syncthreads();
    for (int o = 512; o > 0; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    lg[k] = red[0] + fc_b[k];
    __syncthreads();
  }
  if (t == 0) {
    float m = -INFINITY;
    for (int k = 0; k < ncls; ++k) m = fmaxf(m, lg[k]);
    float s = 0.f;
    for (int k = 0; k < ncls; ++k) s += expf(lg[k] - m);
    for (int k = 0; k < ncls; ++k) {
      logits[b * ncls + k] = lg[k];
      probs[b * ncls + k] = expf(lg[k] - m) / s;
    }
  }
}

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

int id_crop_resize(const uint8_t* frames, int64_t fstride, int W, const int32_t* boxes, int n, int out_size,
                   uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(id_crop_resize_kernel, grid_for((int64_t)n * out_size * out_size), dim3(256), 0, s, frames,
                     fstride, W, boxes, n, out_size, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int id_edge_crop(const uint8_t* in, int n, int in_size, int edge, int crop, int off, bf16_t* out, hipStream_t s) {
  hipLaunchKernelGGL(id_edge_crop_kernel, grid_for((int64_t)n * crop * crop), dim3(256), 0, s, in, n, in_size, edge,
                     crop, off, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int im2col_bf16(const bf16_t* x, int n, int h, int w, int c, int kh, int kw, int stride, int pad, int kpad,
                bf16_t* out, hipStream_t s) {
  const int oh = (h + 2 * pad - kh) / stride + 1, ow = (w + 2 * pad - kw) / stride + 1;
  const bool vec = (c % 8) == 0 && (kpad % 8) == 0;
  const int64_t total = (int64_t)n * oh * ow * (vec ? kpad / 8 : kpad);
  hipLaunchKernelGGL(im2col_bf16_kernel, grid_for(total), dim3(256), 0, s, x, n, h, w, c, kh, kw, stride, pad, oh, ow,
                     kpad, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int maxpool3s2(const bf16_t* x, int n, int h, int w, int c, bf16_t* out, hipStream_t s) {
  const int oh = (h - 1) / 2 + 1, ow = (w - 1) / 2 + 1;
  hipLaunchKernelGGL(maxpool3s2_kernel, grid_for((int64_t)n * oh * ow * c), dim3(256), 0, s, x, n, h, w, c, oh, ow,
                     out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int relu_bf16(float* x, bf16_t* y, int64_t count, hipStream_t s) {
  hipLaunchKernelGGL(relu_bf16_kernel, grid_for(count / 4), dim3(256), 0, s, x, y, count / 4);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int gap_fc_softmax(const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int ncls, float* logits,
                   float* probs, hipStream_t s) {
  hipLaunchKernelGGL(gap_fc_softmax_kernel, dim3(n), dim3(1024), (c + 1024) * sizeof(float), s, x, hw, c, fc_w, fc_b,
                     ncls, logits, probs);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
