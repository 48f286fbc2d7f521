// Step-1 detector (Swin-S Mask R-CNN, bbox only) kernels for gfx950 -- everything of the detector
// that is not a GEMM or a LayerNorm (those reuse gemm_bf16 / gemm_pp / layernorm):
//
//   det_resize_patch   cv2.resize(INTER_LINEAR, fixed point) + BGR->RGB + mean/std + zero pad,
//                      written straight as the 4x4 patch-embed im2col operand (bf16, K padded to 64)
//   window_attention   Swin W-MSA / SW-MSA: one wave per (image, window, head); the zero pad, the
//                      cyclic shift, window partition / reverse and the crop are folded into the
//                      token gather / scatter; relative position bias and the -100 shift mask are
//                      added to S in registers; 16x16x32 bf16 MFMA for K Q^T and V^T P^T
//   merge_gather       PatchMerging's nn.Unfold(2, 2) order (c * 4 + kh * 2 + kw)
//   upsample_add       FPN top-down: lo += nearest(hi)
//   im2col3x3          NHWC f32 -> bf16 (rows, 9 C), tap-major K = (ky * 3 + kx) * C + c, zero pad 1
//   subsample2         P6 = max_pool2d(P5, 1, stride 2)
//   rpn_scores / rpn_decode   sigmoid, per-level top-k (one stable rocprim radix sort on (segment, score) keys),
//                      anchors + delta2bbox + clip + w,h > 0
//   nms_sort / nms_mask / nms_sweep   mmcv batched_nms: level offsets, descending-score order
//                      (ties: candidate order), bitmask IoU (inter > thr * union), greedy sweep
//   roi_align          mmcv RoIAlign (aligned, adaptive sampling, avg) on the map_roi_levels level
//   rcnn_decode        softmax, delta2bbox (0.1, 0.1, 0.2, 0.2), rescale, score_thr
//
// Box arithmetic follows mmdet's operation order in float32 (compiled without FMA contraction).
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "common.hpp"
#include "detector.hpp"

namespace mq {
namespace {

constexpr float LOG2E = 1.4426950408889634f;

// ------------------------------------------------------------------ resize + normalise + patch im2col
// One thread per (token, k): token = (img, ty, tx) of the padded (hp x wp) image / 4, k < 64.
__global__ __launch_bounds__(256) void det_resize_patch_kernel(const uint8_t* __restrict__ frames, int64_t fstride,
                                                               int H, int W, int nh, int nw, int hp, int wp,
                                                               const int32_t* __restrict__ xofs,
                                                               const int32_t* __restrict__ xa,
                                                               const int32_t* __restrict__ yofs,
                                                               const int32_t* __restrict__ ya, int64_t total,
                                                               bf16_t* __restrict__ A) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int k = (int)(idx & 63);
  const int64_t tok = idx >> 6;
  const int tw = wp / 4, th = hp / 4;
  const int tx = (int)(tok % tw);
  const int ty = (int)((tok / tw) % th);
  const int img = (int)(tok / ((int64_t)tw * th));
  float v = 0.f;
  if (k < 48) {
    const int c = k >> 4, kh = (k >> 2) & 3, kw = k & 3;
    const int y = ty * 4 + kh, x = tx * 4 + kw;
    if (y < nh && x < nw) {
      const uint8_t* f = frames + img * fstride;
      const int sc = 2 - c;  // BGR source
      const int sx = xofs[x], sy = yofs[y];
      const int sx1 = min(sx + 1, W - 1), sy1 = min(sy + 1, H - 1);
      const int a0 = xa[2 * x], a1 = xa[2 * x + 1], b0 = ya[2 * y], b1 = ya[2 * y + 1];
      const int h0 = (int)f[((int64_t)sy * W + sx) * 3 + sc] * a0 + (int)f[((int64_t)sy * W + sx1) * 3 + sc] * a1;
      const int h1 = (int)f[((int64_t)sy1 * W + sx) * 3 + sc] * a0 + (int)f[((int64_t)sy1 * W + sx1) * 3 + sc] * a1;
      const int vv = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
      const int u = min(max((vv + 2) >> 2, 0), 255);
      const float mean = c == 0 ? 123.675f : (c == 1 ? 116.28f : 103.53f);
      const float stdv = c == 0 ? 58.395f : (c == 1 ? 57.12f : 57.375f);
      v = ((float)u - mean) / stdv;
    }
  }
  A[idx] = f32_to_bf16(v);
}

// ------------------------------------------------------------------ Swin window attention
constexpr int WIN = 7, WT = 49, WPAD = 64, HD = 32;
constexpr int KROW = 40;  // LDS row stride in bf16 (80 B): conflict-free 16-B column reads

__device__ __forceinline__ int region_of(int p, int Pp, int shift) {
  return p < Pp - WIN ? 0 : (p < Pp - shift ? 1 : 2);
}

// one wave per (image, window, head)
__global__ __launch_bounds__(256) void window_attention_kernel(const bf16_t* __restrict__ qkv,
                                                               const float* __restrict__ qkv_bias,
                                                               const float* __restrict__ rel_table,
                                                               bf16_t* __restrict__ out, int n_units, int H, int W,
                                                               int C, int heads, int shift, float scale) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[4][WPAD * KROW];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[4][WPAD * KROW];
  __shared__ float rel[4][176];
  __shared__ int tokidx[4][WPAD];
  __shared__ int region[4][WPAD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int unit = blockIdx.x * 4 + wave;
  const bool active = unit < n_units;
  const int Hp = (H + WIN - 1) / WIN * WIN, Wp = (W + WIN - 1) / WIN * WIN;
  const int nWw = Wp / WIN, nW = (Hp / WIN) * nWw;
  const int head = active ? unit % heads : 0;
  const int win = active ? (unit / heads) % nW : 0;
  const int img = active ? unit / (heads * nW) : 0;
  const int wy = win / nWw, wx = win % nWw;
  const int ld = 3 * C;
  // token table: shifted-frame window token -> original token row (-1 = zero pad, -2 = beyond 49)
  {
    const int t = lane;
    int ti = -2, rg = 0;
    if (t < WT) {
      const int py = wy * WIN + t / WIN, px = wx * WIN + t % WIN;
      const int oy = (py + shift) % Hp, ox = (px + shift) % Wp;
      ti = (oy < H && ox < W) ? (img * H + oy) * W + ox : -1;
      rg = shift > 0 ? region_of(py, Hp, shift) * 3 + region_of(px, Wp, shift) : 0;
    }
    tokidx[wave][t] = ti;
    region[wave][t] = rg;
  }
  for (int i = lane; i < 169; i += 64) rel[wave][i] = rel_table[i * heads + head];
  __syncthreads();
  // K and V rows into LDS (4 x 16-B chunks of 32 d per token); pad tokens = the qkv bias
  for (int c = lane; c < WPAD * 4; c += 64) {
    const int t = c >> 2, ch = c & 3;
    const int ti = tokidx[wave][t];
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (ti >= 0) {
      kv = *reinterpret_cast<const uint4*>(qkv + (size_t)ti * ld + C + head * HD + ch * 8);
      vv = *reinterpret_cast<const uint4*>(qkv + (size_t)ti * ld + 2 * C + head * HD + ch * 8);
    } else if (ti == -1) {
      const float* kb = qkv_bias + C + head * HD + ch * 8;
      const float* vb = qkv_bias + 2 * C + head * HD + ch * 8;
      kv = make_uint4(pack_bf16x2(kb[0], kb[1]), pack_bf16x2(kb[2], kb[3]), pack_bf16x2(kb[4], kb[5]),
                      pack_bf16x2(kb[6], kb[7]));
      vv = make_uint4(pack_bf16x2(vb[0], vb[1]), pack_bf16x2(vb[2], vb[3]), pack_bf16x2(vb[4], vb[5]),
                      pack_bf16x2(vb[6], vb[7]));
    }
    *reinterpret_cast<uint4*>(&Ks[wave][t * KROW + ch * 8]) = kv;
    *reinterpret_cast<uint4*>(&Vs[wave][t * KROW + ch * 8]) = vv;
  }
  // Q^T fragments (B operand: k = d 8 g + j, column = query l16) straight from global
  const int l16 = lane & 15, g = lane >> 4;
  bf16x8 qf[4];
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) {
    const int ti = tokidx[wave][qb * 16 + l16];
    if (ti >= 0) {
      qf[qb] = *reinterpret_cast<const bf16x8*>(qkv + (size_t)ti * ld + head * HD + g * 8);
    } else if (ti == -1) {
      const float* qb_ = qkv_bias + head * HD + g * 8;
      const uint4 u = make_uint4(pack_bf16x2(qb_[0], qb_[1]), pack_bf16x2(qb_[2], qb_[3]),
                                 pack_bf16x2(qb_[4], qb_[5]), pack_bf16x2(qb_[6], qb_[7]));
      qf[qb] = __builtin_bit_cast(bf16x8, u);
    } else {
      qf[qb] = bf16x8{};
    }
  }
  __syncthreads();
  if (!active) return;
  // S^T[kb][qb]: keys kb*16 + 4 g + e (rows), query qb*16 + l16 (column)
  f32x4 S[4][4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[wave][(kb * 16 + l16) * KROW + g * 8]);
#pragma unroll
    for (int qb = 0; qb < 4; ++qb)
      S[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qb], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
  }
  // + relative position bias + shift mask, softmax over the 49 keys of each query
  bf16x8 P[4][2];
  float linv[4];
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) {
    const int q = qb * 16 + l16;
    const int qi = q / WIN, qj = q % WIN;
    const int qr = region[wave][q];
    float m = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = kb * 16 + 4 * g + e;
        float s = -INFINITY;
        if (k < WT) {
          const int ki = k / WIN, kj = k % WIN;
          s = S[kb][qb][e] * scale + rel[wave][(qi - ki + WIN - 1) * (2 * WIN - 1) + (qj - kj + WIN - 1)];
          if (shift > 0 && region[wave][k] != qr) s += -100.0f;
        }
        S[kb][qb][e] = s;
        m = fmaxf(m, s);
      }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = __builtin_amdgcn_exp2f((S[kb][qb][e] - m) * LOG2E);
        S[kb][qb][e] = pv;
        l += pv;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    linv[qb] = 1.0f / l;
    // B operand of P^T: element j of lane group g = key 32 ks + 16 (j >> 2) + 4 g + (j & 3)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        P[qb][ks][e] = (__bf16)S[2 * ks][qb][e];
        P[qb][ks][4 + e] = (__bf16)S[2 * ks + 1][qb][e];
      }
  }
  // O^T[dt][qb] = V^T P^T: rows d = dt*16 + 4 g + e, column = query
  f32x4 O[2][4];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) O[dt][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int trq = l16 >> 2, trp = l16 & 3;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const int ra = 2 * ks * 16 + 4 * g + trq;
      const bf16_t* pa = &Vs[wave][ra * KROW + dt * 16 + 4 * trp];
      const short4v v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) short4v*)MQ_LDS_LOCAL(pa));
      const short4v v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) short4v*)MQ_LDS_LOCAL(pa + 16 * KROW));
      bf16x8 vb;
      __builtin_memcpy(&vb, &v0, 8);
      __builtin_memcpy(reinterpret_cast<char*>(&vb) + 8, &v1, 8);
#pragma unroll
      for (int qb = 0; qb < 4; ++qb) O[dt][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb, P[qb][ks], O[dt][qb], 0, 0, 0);
    }
  }
  // scatter back to the original token rows (window reverse + roll back + crop)
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) {
    const int q = qb * 16 + l16;
    const int ti = q < WT ? tokidx[wave][q] : -1;
    if (ti < 0) continue;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const uint2 o = make_uint2(pack_bf16x2(O[dt][qb][0] * linv[qb], O[dt][qb][1] * linv[qb]),
                                 pack_bf16x2(O[dt][qb][2] * linv[qb], O[dt][qb][3] * linv[qb]));
      *reinterpret_cast<uint2*>(out + (size_t)ti * C + head * HD + dt * 16 + 4 * g) = o;
    }
  }
}

// ------------------------------------------------------------------ small layout kernels
__global__ void merge_gather_kernel(const float* __restrict__ x, int H, int W, int C, int64_t total,
                                    float* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C4 = 4 * C;
  const int f = (int)(idx % C4);
  const int64_t row = idx / C4;
  const int H2 = (H + 1) / 2, W2 = (W + 1) / 2;
  const int j = (int)(row % W2), i = (int)((row / W2) % H2);
  const int img = (int)(row / ((int64_t)W2 * H2));
  const int c = f >> 2, kh = (f >> 1) & 1, kw = f & 1;
  const int y = 2 * i + kh, xx = 2 * j + kw;
  out[idx] = (y < H && xx < W) ? x[(((int64_t)img * H + y) * W + xx) * C + c] : 0.f;
}

__global__ void upsample_add_kernel(float* __restrict__ lo, const float* __restrict__ hi, int Hl, int Wl, int Hh,
                                    int Wh, int C, int64_t total) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const int64_t p = idx / C;
  const int x = (int)(p % Wl), y = (int)((p / Wl) % Hl);
  const int img = (int)(p / ((int64_t)Wl * Hl));
  // torch 'nearest' with an output size: src = min(floor(dst * in / out), in - 1)
  const float sy = (float)Hh / (float)Hl, sx = (float)Wh / (float)Wl;
  const int ys = min((int)floorf((float)y * sy), Hh - 1), xs = min((int)floorf((float)x * sx), Wh - 1);
  lo[idx] = lo[idx] + hi[(((int64_t)img * Hh + ys) * Wh + xs) * C + c];
}

__global__ void im2col3x3_kernel(const float* __restrict__ x, int H, int W, int C, int64_t total,
                                 bf16_t* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // one thread per 4 channels
  if (idx >= total) return;
  const int C4 = C / 4;
  const int cq = (int)(idx % C4);
  const int tap = (int)((idx / C4) % 9);
  const int64_t p = idx / (C4 * 9);
  const int xx = (int)(p % W), y = (int)((p / W) % H);
  const int img = (int)(p / ((int64_t)W * H));
  const int sy = y + tap / 3 - 1, sx = xx + tap % 3 - 1;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sy >= 0 && sy < H && sx >= 0 && sx < W)
    v = *reinterpret_cast<const float4*>(x + (((int64_t)img * H + sy) * W + sx) * C + cq * 4);
  *reinterpret_cast<uint2*>(out + p * 9 * C + tap * C + cq * 4) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
}

__global__ void subsample2_kernel(const float* __restrict__ x, int H, int W, int C, int Ho, int Wo, int64_t total,
                                  float* __restrict__ out) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int c = (int)(idx % C);
  const int64_t p = idx / C;
  const int xx = (int)(p % Wo), y = (int)((p / Wo) % Ho);
  const int img = (int)(p / ((int64_t)Wo * Ho));
  out[idx] = x[(((int64_t)img * H + 2 * y) * W + 2 * xx) * C + c];
}

// ------------------------------------------------------------------ RPN
// head rows: level-major over the batch -- row(img, l, pos) = n_img * row_off[l] + img * h_l * w_l + pos --
// 15 columns (3 anchor logits, 12 deltas anchor-major).  Scores / ids are image-major (one sort segment
// per (image, level)).
__device__ __forceinline__ int det_level_of(const DetLevels& lv, int row) {
  int l = 0;
  while (l + 1 < lv.n && row >= lv.row_off[l + 1]) ++l;
  return l;
}

// sort key: (segment = image * levels + level) above the descending score, so one stable radix sort
// orders every segment by descending score (ties: lower anchor index first) in place
__global__ void rpn_scores_kernel(const float* __restrict__ head, const DetLevels lv, int rows_per_img, int n_img,
                                  float* __restrict__ scores, int32_t* __restrict__ ids,
                                  unsigned long long* __restrict__ keys) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)rows_per_img * 3;
  if (idx >= (int64_t)n_img * per) return;
  const int img = (int)(idx / per);
  const int local = (int)(idx % per);
  const int a = local % 3, r = local / 3;
  const int l = det_level_of(lv, r);
  const int pos = r - lv.row_off[l];
  const int64_t hrow = (int64_t)n_img * lv.row_off[l] + (int64_t)img * lv.h[l] * lv.w[l] + pos;
  const float x = head[hrow * 15 + a];
  const float sc = 1.0f / (1.0f + expf(-x));
  scores[idx] = sc;
  ids[idx] = local;
  unsigned u = __float_as_uint(sc);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  keys[idx] = ((unsigned long long)(img * lv.n + l) << 32) | (unsigned long long)(~u);
}

// decode the top-k of every (image, level): candidates of an image are level-major, rank order
__global__ void rpn_decode_kernel(const float* __restrict__ head, const float* __restrict__ scores,
                                  const int32_t* __restrict__ sorted_ids, const DetLevels lv, int n_img,
                                  int rows_per_img, float img_h, float img_w, float* __restrict__ boxes,
                                  float* __restrict__ cand_scores, uint8_t* __restrict__ valid,
                                  int8_t* __restrict__ lvl_of) {
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int K = lv.cand_total;
  if (idx >= (int64_t)n_img * K) return;
  const int img = (int)(idx / K), c = (int)(idx % K);
  int l = 0;
  while (l + 1 < lv.n && c >= lv.cand_off[l + 1]) ++l;
  const int r = c - lv.cand_off[l];
  const int64_t seg = (int64_t)img * rows_per_img * 3 + (int64_t)lv.row_off[l] * 3;  // segment start
  const int id = sorted_ids[seg + r];  // index within the image's anchors (level offset included)
  const float s = scores[(int64_t)img * rows_per_img * 3 + id];
  const int local = id - lv.row_off[l] * 3;
  const int pos = local / 3, a = local % 3;
  const int x = pos % lv.w[l], y = pos / lv.w[l];
  const float st = (float)lv.stride[l];
  const float sx = (float)x * st, sy = (float)y * st;
  const float ax1 = lv.base[l][a][0] + sx, ay1 = lv.base[l][a][1] + sy;
  const float ax2 = lv.base[l][a][2] + sx, ay2 = lv.base[l][a][3] + sy;
  const float* d = head + ((int64_t)n_img * lv.row_off[l] + (int64_t)img * lv.h[l] * lv.w[l] + pos) * 15 + 3 + a * 4;
  float b[4];
  delta2bbox(ax1, ay1, ax2, ay2, d[0] * 1.0f + 0.0f, d[1] * 1.0f + 0.0f, d[2] * 1.0f + 0.0f, d[3] * 1.0f + 0.0f,
             img_h, img_w, b);
  float* o = boxes + idx * 4;
  o[0] = b[0];
  o[1] = b[1];
  o[2] = b[2];
  o[3] = b[3];
  cand_scores[idx] = s;
  valid[idx] = (b[2] - b[0] > 0.f) && (b[3] - b[1] > 0.f);
  lvl_of[idx] = (int8_t)l;
}

// ------------------------------------------------------------------ batched NMS
constexpr int NMS_SORT_MAX = 8192;
constexpr int NMS_T = 1024;

__device__ __forceinline__ unsigned long long nms_key(float s, int i) {
  // descending score, ascending index -> ascending u64
  unsigned u = __float_as_uint(s);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // orderable ascending
  return ((unsigned long long)(~u) << 32) | (unsigned)i;
}

// per image: max over valid boxes (level offsets), sort valid candidates, write offset boxes in order
__global__ __launch_bounds__(NMS_T) void nms_sort_kernel(const float* __restrict__ boxes,
                                                          const float* __restrict__ scores,
                                                          const uint8_t* __restrict__ valid,
                                                          const int8_t* __restrict__ lvl, int n_cand,
                                                          int32_t* __restrict__ order, float* __restrict__ sboxes,
                                                          int32_t* __restrict__ n_valid) {
  __shared__ unsigned long long keys[NMS_SORT_MAX];
  __shared__ float red[NMS_T / 64];
  __shared__ int cnt[NMS_T / 64];
  const int img = blockIdx.x, tid = threadIdx.x;
  const float* b = boxes + (size_t)img * n_cand * 4;
  const float* s = scores + (size_t)img * n_cand;
  const uint8_t* v = valid + (size_t)img * n_cand;
  float mx = -INFINITY;
  int nv = 0;
  for (int i = tid; i < n_cand; i += NMS_T)
    if (v[i]) {
      mx = fmaxf(mx, fmaxf(fmaxf(b[i * 4], b[i * 4 + 1]), fmaxf(b[i * 4 + 2], b[i * 4 + 3])));
      ++nv;
    }
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    nv += __shfl_xor(nv, o, 64);
  }
  if ((tid & 63) == 0) red[tid >> 6] = mx, cnt[tid >> 6] = nv;
  int n2 = 1;
  while (n2 < n_cand) n2 <<= 1;
  for (int i = tid; i < n2; i += NMS_T) keys[i] = (i < n_cand && v[i]) ? nms_key(s[i], i) : ~0ull;
  __syncthreads();
  float gmax = red[0];
  int gnv = cnt[0];
  for (int w = 1; w < NMS_T / 64; ++w) gmax = fmaxf(gmax, red[w]), gnv += cnt[w];
  // bitonic sort of n2 keys in LDS
  for (int k = 2; k <= n2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n2; i += NMS_T) {
        const int p = i ^ j;
        if (p > i) {
          const unsigned long long a = keys[i], c = keys[p];
          const bool up = (i & k) == 0;
          if ((a > c) == up) keys[i] = c, keys[p] = a;
        }
      }
      __syncthreads();
    }
  }
  const float off_unit = gmax + 1.0f;
  for (int r = tid; r < gnv; r += NMS_T) {
    const int i = (int)(keys[r] & 0xffffffffu);
    const float off = lvl ? (float)lvl[(size_t)img * n_cand + i] * off_unit : 0.0f;
    order[(size_t)img * n_cand + r] = i;
    float* o = sboxes + ((size_t)img * n_cand + r) * 4;
    o[0] = b[i * 4] + off;
    o[1] = b[i * 4 + 1] + off;
    o[2] = b[i * 4 + 2] + off;
    o[3] = b[i * 4 + 3] + off;
  }
  if (tid == 0) n_valid[img] = gnv;
}

// mask[img][i][w] bit t: sorted box i suppresses sorted box 64 w + t (> i)
__global__ __launch_bounds__(64) void nms_mask_kernel(const float* __restrict__ sboxes,
                                                      const int32_t* __restrict__ n_valid, int n_cand, int words,
                                                      float thr, unsigned long long* __restrict__ mask) {
  const int img = blockIdx.z, rb = blockIdx.y, cb = blockIdx.x;
  const int nv = n_valid[img];
  const int i = rb * 64 + threadIdx.x;
  __shared__ float cbox[64][4];
  const int jj = cb * 64 + threadIdx.x;
  if (jj < nv) {
    const float* q = sboxes + ((size_t)img * n_cand + jj) * 4;
    cbox[threadIdx.x][0] = q[0];
    cbox[threadIdx.x][1] = q[1];
    cbox[threadIdx.x][2] = q[2];
    cbox[threadIdx.x][3] = q[3];
  }
  __syncthreads();
  if (i >= nv || cb * 64 + 63 <= i) {
    if (i < nv) mask[((size_t)img * n_cand + i) * words + cb] = 0ull;
    return;
  }
  const float* a = sboxes + ((size_t)img * n_cand + i) * 4;
  const float a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
  const float sa = (a2 - a0) * (a3 - a1);
  unsigned long long bits = 0ull;
  const int jmax = min(64, nv - cb * 64);
  for (int t = 0; t < jmax; ++t) {
    const int j = cb * 64 + t;
    if (j <= i) continue;
    const float w = fmaxf(fminf(a2, cbox[t][2]) - fmaxf(a0, cbox[t][0]), 0.f);
    const float h = fmaxf(fminf(a3, cbox[t][3]) - fmaxf(a1, cbox[t][1]), 0.f);
    const float inter = w * h;
    const float sb = (cbox[t][2] - cbox[t][0]) * (cbox[t][3] - cbox[t][1]);
    if (inter > thr * ((sa + sb) - inter)) bits |= 1ull << t;
  }
  mask[((size_t)img * n_cand + i) * words + cb] = bits;
}

// block per image: mask rows arrive 64 at a time into LDS (all threads, coalesced); wave 0 runs
// the greedy sweep over them in sorted order, at most max_keep kept.  The removed-candidate mask lives
// in wave 0's registers (lane l holds words l and l + 64), the word of the current 64-candidate chunk
// in scalar registers, so a suppressed candidate costs a bit test and a kept one a single LDS row read;
// kept candidates are recorded by sorted index in LDS and mapped through `order` by all threads at the
// end (a global load per kept candidate used to sit on the sweep's chain).
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long readfirst_u64(unsigned long long v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
__global__ __launch_bounds__(256) void nms_sweep_kernel(const unsigned long long* __restrict__ mask,
                                                        const int32_t* __restrict__ order,
                                                        const int32_t* __restrict__ n_valid, int n_cand, int words,
                                                        int max_keep, int32_t* __restrict__ keep,
                                                        int32_t* __restrict__ n_keep) {
  extern __shared__ unsigned long long rows[];  // 64 * words, then max_keep kept indices (int32)
  int32_t* kidx = reinterpret_cast<int32_t*>(rows + 64 * words);
  __shared__ int s_kept;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int nv = n_valid[img];
  if (tid == 0) s_kept = 0;
  const unsigned long long* mrow = mask + (size_t)img * n_cand * words;
  int kept = 0;  // wave 0's count
  unsigned long long rm0 = 0ull, rm1 = 0ull;  // wave 0: removed-mask words lane, lane + 64
  __syncthreads();
  for (int c0 = 0; c0 < nv; c0 += 64) {
    if (s_kept >= max_keep) break;  // uniform: read after the barrier that published it
    const int nr = min(64, nv - c0);
    for (int e = tid; e < nr * words; e += 256) rows[e] = mrow[(size_t)c0 * words + e];
    __syncthreads();
    if (tid < 64) {
      const int w = c0 >> 6;  // every candidate of the chunk lives in word w
      unsigned long long cur = readlane_u64(w < 64 ? rm0 : rm1, w & 63);
      for (int t = 0; t < nr && kept < max_keep; ++t) {
        if ((cur >> t) & 1ull) continue;
        if (lane == 0) kidx[kept] = c0 + t;
        ++kept;
        const unsigned long long* row = rows + t * words;
        if (lane < words) rm0 |= row[lane];
        if (lane + 64 < words) rm1 |= row[lane + 64];
        cur |= readfirst_u64(row[w]);
      }
      if (lane == 0) s_kept = kept;
    }
    __syncthreads();
  }
  const int k = s_kept;
  for (int r = tid; r < max_keep; r += 256)
    keep[(size_t)img * max_keep + r] = r < k ? order[(size_t)img * n_cand + kidx[r]] : -1;
  if (tid == 0) n_keep[img] = k;
}

// proposals = the first kept candidates' (un-offset) boxes
__global__ void gather_boxes_kernel(const float* __restrict__ boxes, const float* __restrict__ scores,
                                    const int32_t* __restrict__ keep, int n_img, int n_cand, int max_keep,
                                    float* __restrict__ out_boxes, float* __restrict__ out_scores) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_img * max_keep) return;
  const int img = idx / max_keep;
  const int k = keep[idx];
  float* o = out_boxes + (size_t)idx * 4;
  if (k < 0) {
    o[0] = o[1] = o[2] = o[3] = 0.f;
    if (out_scores) out_scores[idx] = 0.f;
    return;
  }
  const float* b = boxes + ((size_t)img * n_cand + k) * 4;
  o[0] = b[0];
  o[1] = b[1];
  o[2] = b[2];
  o[3] = b[3];
  if (out_scores) out_scores[idx] = scores[(size_t)img * n_cand + k];
}

// ------------------------------------------------------------------ RoIAlign
__device__ __forceinline__ void roi_bilinear_w(int H, int W, float y, float x, int& i00, int& i01, int& i10, int& i11,
                                               float& w1, float& w2, float& w3, float& w4, bool& ok) {
  ok = !(y < -1.0f || y > (float)H || x < -1.0f || x > (float)W);
  if (!ok) return;
  if (y <= 0.f) y = 0.f;
  if (x <= 0.f) x = 0.f;
  int yl = (int)y, xl = (int)x, yh, xh;
  if (yl >= H - 1) {
    yh = yl = H - 1;
    y = (float)yl;
  } else {
    yh = yl + 1;
  }
  if (xl >= W - 1) {
    xh = xl = W - 1;
    x = (float)xl;
  } else {
    xh = xl + 1;
  }
  const float ly = y - (float)yl, lx = x - (float)xl;
  const float hy = 1.f - ly, hx = 1.f - lx;
  w1 = hy * hx;
  w2 = hy * lx;
  w3 = ly * hx;
  w4 = ly * lx;
  i00 = yl * W + xl;
  i01 = yl * W + xh;
  i10 = yh * W + xl;
  i11 = yh * W + xh;
}

// block per roi: thread = (channel quad, bin slot of 4); bilinear weights per sample shared by the 4
// channels of a float4 load; the roi's (256, 7, 7) output is staged in LDS and stored contiguously.
// Rows past an image's proposal count are zero.
__global__ __launch_bounds__(256) void roi_align_kernel(const DetFeats fs, const float* __restrict__ rois,
                                                        const int32_t* __restrict__ n_rois, int max_rois,
                                                        bf16_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) bf16_t o_lds[256 * 49];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int img = r / max_rois;
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)r * 256 * 49);
  constexpr int NCH = 256 * 49 * 2 / 16;  // 16-B chunks per roi
  if (r % max_rois >= n_rois[img]) {
    for (int i = tid; i < NCH; i += 256) o[i] = make_uint4(0, 0, 0, 0);
    return;
  }
  const float* rb = rois + (size_t)r * 4;
  const float x1 = rb[0], y1 = rb[1], x2 = rb[2], y2 = rb[3];
  const float scl = sqrtf((x2 - x1) * (y2 - y1));
  int lvl = (int)floorf(log2f(scl / 56.0f + 1e-6f));
  lvl = min(max(lvl, 0), 3);
  const int H = fs.h[lvl], W = fs.w[lvl];
  const float ss = 1.0f / (float)fs.stride[lvl];
  const int cq = tid & 63, slot = tid >> 6;
  const float* f = fs.p[lvl] + (size_t)img * H * W * 256 + cq * 4;
  const float sx = x1 * ss - 0.5f, sy = y1 * ss - 0.5f;
  const float ex = x2 * ss - 0.5f, ey = y2 * ss - 0.5f;
  const float rw = ex - sx, rh = ey - sy;
  const float bw = rw / 7.0f, bh = rh / 7.0f;
  const int gh = (int)ceilf(rh / 7.0f), gw = (int)ceilf(rw / 7.0f);
  const float cnt = (float)max(gh * gw, 1);
  for (int bin = slot; bin < 49; bin += 4) {
    const int ph = bin / 7, pw = bin % 7;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // (issuing the loads of 4 samples together was measured 22 % slower: most bins take 1-4 samples
    // and the kernel is bound by the L2 gather volume, not by load latency)
    for (int iy = 0; iy < gh; ++iy) {
      const float y = sy + (float)ph * bh + ((float)iy + 0.5f) * bh / (float)gh;
      for (int ix = 0; ix < gw; ++ix) {
        const float x = sx + (float)pw * bw + ((float)ix + 0.5f) * bw / (float)gw;
        int i00, i01, i10, i11;
        float w1, w2, w3, w4;
        bool ok;
        roi_bilinear_w(H, W, y, x, i00, i01, i10, i11, w1, w2, w3, w4, ok);
        if (!ok) continue;
        const float4 v1 = *reinterpret_cast<const float4*>(f + (size_t)i00 * 256);
        const float4 v2 = *reinterpret_cast<const float4*>(f + (size_t)i01 * 256);
        const float4 v3 = *reinterpret_cast<const float4*>(f + (size_t)i10 * 256);
        const float4 v4 = *reinterpret_cast<const float4*>(f + (size_t)i11 * 256);
        acc.x += ((w1 * v1.x + w2 * v2.x) + w3 * v3.x) + w4 * v4.x;
        acc.y += ((w1 * v1.y + w2 * v2.y) + w3 * v3.y) + w4 * v4.y;
        acc.z += ((w1 * v1.z + w2 * v2.z) + w3 * v3.z) + w4 * v4.z;
        acc.w += ((w1 * v1.w + w2 * v2.w) + w3 * v3.w) + w4 * v4.w;
      }
    }
    const int c = cq * 4;
    o_lds[(c + 0) * 49 + bin] = f32_to_bf16(acc.x / cnt);
    o_lds[(c + 1) * 49 + bin] = f32_to_bf16(acc.y / cnt);
    o_lds[(c + 2) * 49 + bin] = f32_to_bf16(acc.z / cnt);
    o_lds[(c + 3) * 49 + bin] = f32_to_bf16(acc.w / cnt);
  }
  __syncthreads();
  const uint4* src = reinterpret_cast<const uint4*>(o_lds);
  for (int i = tid; i < NCH; i += 256) o[i] = src[i];
}

// ------------------------------------------------------------------ RCNN post-process
__global__ void rcnn_decode_kernel(const float* __restrict__ rois, const float* __restrict__ head,
                                   const int32_t* __restrict__ n_rois, int n_img, int max_rois, float img_h,
                                   float img_w, float inv_sw, float inv_sh, float score_thr,
                                   float* __restrict__ boxes, float* __restrict__ scores,
                                   uint8_t* __restrict__ valid) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_img * max_rois) return;
  const int img = idx / max_rois;
  const float* h = head + (size_t)idx * 6;
  const float m = fmaxf(h[0], h[1]);
  const float e0 = expf(h[0] - m), e1 = expf(h[1] - m);
  const float s = e0 / (e0 + e1);
  const float* r = rois + (size_t)idx * 4;
  float b[4];
  delta2bbox(r[0], r[1], r[2], r[3], h[2] * 0.1f + 0.0f, h[3] * 0.1f + 0.0f, h[4] * 0.2f + 0.0f,
             h[5] * 0.2f + 0.0f, img_h, img_w, b);
  float* o = boxes + (size_t)idx * 4;
  o[0] = b[0] * inv_sw;
  o[1] = b[1] * inv_sh;
  o[2] = b[2] * inv_sw;
  o[3] = b[3] * inv_sh;
  scores[idx] = s;
  valid[idx] = (idx % max_rois < n_rois[img]) && (s > score_thr);
}


// ------------------------------------------------------------------ static top-k crop boxes (config 5 graph)
// One thread per image.  The detections (score-ordered, det_counts[i] valid) that score above thr and
// are non-degenerate after step 1's int() truncation (filter_tracks, step1_proc2d.py:255-268) fill the
// first k slots in score order; each gets the dynamic-margin expansion + aspect fix of step1:270-292
// in float64 with numpy's operation order (expand_boxes), rounded to float32.  Empty slots: valid 0 and
// a placeholder box (the crop stays in bounds, the caller masks the keypoints).
__global__ void det_topk_boxes_kernel(const float* __restrict__ dboxes, const float* __restrict__ dscores,
                                      const int32_t* __restrict__ dcount, int n_img, int max_det, int k, float thr,
                                      double mn, double mx, double ar_t, float* __restrict__ out,
                                      float* __restrict__ tight, int32_t* __restrict__ img_of,
                                      int32_t* __restrict__ valid) {
  const int img = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n_img) return;
  const int cnt = min(dcount[img], max_det);
  int slot = 0;
  for (int d = 0; d < cnt && slot < k; ++d) {
    if (!(dscores[(size_t)img * max_det + d] > thr)) continue;
    const float* b = dboxes + ((size_t)img * max_det + d) * 4;
    const long long x1 = (long long)b[0], y1 = (long long)b[1], x2 = (long long)b[2], y2 = (long long)b[3];
    if (!(x2 > x1 && y2 > y1)) continue;
    const double w = (double)(x2 - x1), h = (double)(y2 - y1);
    const double cx = (double)x1 + 0.5 * w, cy = (double)y1 + 0.5 * h;
    double frac = (h - 50.0) / (200.0 - 50.0);
    frac = frac < 0.0 ? 0.0 : (frac > 1.0 ? 1.0 : frac);
    const double m = mx - (mx - mn) * frac;
    double wn = w * (1.0 + m), hn = h * (1.0 + m);
    const double ar = wn / hn;
    const bool fix = fabs(ar - ar_t) > 0.20, wide = ar >= ar_t;
    if (fix && !wide) wn = hn * ar_t;
    if (fix && wide) hn = wn / ar_t;
    const double fcx = (double)(float)cx, fcy = (double)(float)cy;
    const double hw = 0.5 * (double)(float)wn, hh = 0.5 * (double)(float)hn;
    const int o = img * k + slot;
    out[4 * o + 0] = (float)(fcx - hw);
    out[4 * o + 1] = (float)(fcy - hh);
    out[4 * o + 2] = (float)(fcx + hw);
    out[4 * o + 3] = (float)(fcy + hh);
    tight[4 * o + 0] = (float)x1;
    tight[4 * o + 1] = (float)y1;
    tight[4 * o + 2] = (float)x2;
    tight[4 * o + 3] = (float)y2;
    img_of[o] = img;
    valid[o] = 1;
    ++slot;
  }
  for (; slot < k; ++slot) {
    const int o = img * k + slot;
    out[4 * o + 0] = 0.f;
    out[4 * o + 1] = 0.f;
    out[4 * o + 2] = 192.f;
    out[4 * o + 3] = 256.f;
    tight[4 * o + 0] = tight[4 * o + 1] = tight[4 * o + 2] = tight[4 * o + 3] = 0.f;
    img_of[o] = img;
    valid[o] = 0;
  }
}


}  // namespace

// ------------------------------------------------------------------ launchers
static inline dim3 blocks_for(int64_t n, int t = 256) { return dim3((unsigned)((n + t - 1) / t)); }

int det_resize_patch(const uint8_t* frames, int64_t fstride, int n_img, int H, int W, int nh, int nw, int hp, int wp,
                     const int32_t* xofs, const int32_t* xa, const int32_t* yofs, const int32_t* ya, bf16_t* A,
                     hipStream_t s) {
  const int64_t total = (int64_t)n_img * (hp / 4) * (wp / 4) * 64;
  hipLaunchKernelGGL(det_resize_patch_kernel, blocks_for(total), dim3(256), 0, s, frames, fstride, H, W, nh, nw, hp, wp,
                     xofs, xa, yofs, ya, total, A);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int window_attention(const bf16_t* qkv, const float* qkv_bias, const float* rel_table, bf16_t* out, int n_img, int H,
                     int W, int C, int heads, int shift, hipStream_t s) {
  if (C != heads * HD || shift < 0 || shift >= WIN) return -2;
  const int Hp = (H + WIN - 1) / WIN * WIN, Wp = (W + WIN - 1) / WIN * WIN;
  const int units = n_img * (Hp / WIN) * (Wp / WIN) * heads;
  const float scale = 1.0f / sqrtf((float)HD);
  hipLaunchKernelGGL(window_attention_kernel, dim3((units + 3) / 4), dim3(256), 0, s, qkv, qkv_bias, rel_table, out,
                     units, H, W, C, heads, shift, scale);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int merge_gather(const float* x, int n_img, int H, int W, int C, float* out, hipStream_t s) {
  const int64_t total = (int64_t)n_img * ((H + 1) / 2) * ((W + 1) / 2) * 4 * C;
  hipLaunchKernelGGL(merge_gather_kernel, blocks_for(total), dim3(256), 0, s, x, H, W, C, total, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int upsample_add(float* lo, const float* hi, int n_img, int Hl, int Wl, int Hh, int Wh, int C, hipStream_t s) {
  const int64_t total = (int64_t)n_img * Hl * Wl * C;
  hipLaunchKernelGGL(upsample_add_kernel, blocks_for(total), dim3(256), 0, s, lo, hi, Hl, Wl, Hh, Wh, C, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int im2col3x3(const float* x, int n_img, int H, int W, int C, bf16_t* out, hipStream_t s) {
  if (C % 4) return -2;
  const int64_t total = (int64_t)n_img * H * W * 9 * (C / 4);
  hipLaunchKernelGGL(im2col3x3_kernel, blocks_for(total), dim3(256), 0, s, x, H, W, C, total, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int subsample2(const float* x, int n_img, int H, int W, int C, float* out, hipStream_t s) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int64_t total = (int64_t)n_img * Ho * Wo * C;
  hipLaunchKernelGGL(subsample2_kernel, blocks_for(total), dim3(256), 0, s, x, H, W, C, Ho, Wo, total, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t nms_workspace_bytes(int n_img, int n_cand) {
  const int words = (n_cand + 63) / 64;
  return (size_t)n_img * n_cand * (4 + 16) + (size_t)n_img * n_cand * words * 8 + (size_t)n_img * 4 + 1024;
}

int nms_batched(const float* boxes, const float* scores, const uint8_t* valid, const int8_t* lvl, int n_img,
                int n_cand, float thr, int max_keep, void* ws, int32_t* keep, int32_t* n_keep, hipStream_t s) {
  if (n_cand > NMS_SORT_MAX) return -2;
  const int words = (n_cand + 63) / 64;
  if (words > 128) return -2;
  char* p = static_cast<char*>(ws);
  int32_t* order = reinterpret_cast<int32_t*>(p);
  p += (size_t)n_img * n_cand * 4;
  float* sboxes = reinterpret_cast<float*>(p);
  p += (size_t)n_img * n_cand * 16;
  unsigned long long* mask = reinterpret_cast<unsigned long long*>(((uintptr_t)p + 255) & ~(uintptr_t)255);
  p = reinterpret_cast<char*>(mask) + (size_t)n_img * n_cand * words * 8;
  int32_t* nv = reinterpret_cast<int32_t*>(p);
  hipLaunchKernelGGL(nms_sort_kernel, dim3(n_img), dim3(NMS_T), 0, s, boxes, scores, valid, lvl, n_cand, order, sboxes,
                     nv);
  hipLaunchKernelGGL(nms_mask_kernel, dim3(words, words, n_img), dim3(64), 0, s, sboxes, nv, n_cand, words, thr, mask);
  hipLaunchKernelGGL(nms_sweep_kernel, dim3(n_img), dim3(256), (size_t)64 * words * 8 + (size_t)max_keep * 4, s, mask,
                     order, nv, n_cand, words, max_keep, keep, n_keep);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

static size_t sort_temp_bytes(size_t n) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, n, 0u, 44u);
  return bytes;
}

size_t rpn_workspace_bytes(int n_img, int rows_per_img, int cand_total, int n_levels) {
  const size_t n = (size_t)n_img * rows_per_img * 3;
  const size_t sort_tmp = sort_temp_bytes(n);
  (void)n_levels;
  const size_t nc = (size_t)n_img * cand_total;
  return n * 32 + ((sort_tmp + 255) & ~(size_t)255) + (size_t)n_img * 6 * 2 * 4 + nc * 24 + 18 * 256 +
         nms_workspace_bytes(n_img, cand_total) + 4096;
}

int rpn_proposals(const float* head, const DetLevels& lv, int n_img, int rows_per_img, float img_h, float img_w,
                  float iou_thr, int max_keep, void* ws, size_t ws_bytes, float* props, float* prop_scores,
                  int32_t* n_props, int32_t* keep_buf, hipStream_t s) {
  const size_t n = (size_t)n_img * rows_per_img * 3;
  const int K = lv.cand_total;
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t b) {
    char* q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  float* sc = reinterpret_cast<float*>(take(n * 4));
  int32_t* ids = reinterpret_cast<int32_t*>(take(n * 4));
  int32_t* ids_sorted = reinterpret_cast<int32_t*>(take(n * 4));
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(take(n * 8));
  unsigned long long* keys_sorted = reinterpret_cast<unsigned long long*>(take(n * 8));
  float* cboxes = reinterpret_cast<float*>(take((size_t)n_img * K * 16));
  float* cscores = reinterpret_cast<float*>(take((size_t)n_img * K * 4));
  uint8_t* cvalid = reinterpret_cast<uint8_t*>(take((size_t)n_img * K));
  int8_t* clvl = reinterpret_cast<int8_t*>(take((size_t)n_img * K));
  void* nms_ws = take(nms_workspace_bytes(n_img, K));
  size_t sort_tmp = sort_temp_bytes(n);
  void* sort_ws = take(sort_tmp);
  if ((size_t)(p - static_cast<char*>(ws)) > ws_bytes) return -5;
  hipLaunchKernelGGL(rpn_scores_kernel, blocks_for((int64_t)n), dim3(256), 0, s, head, lv, rows_per_img, n_img, sc, ids,
                     keys);
  if (rocprim::radix_sort_pairs(sort_ws, sort_tmp, keys, keys_sorted, ids, ids_sorted, n, 0u, 44u, s) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(rpn_decode_kernel, blocks_for((int64_t)n_img * K), dim3(256), 0, s, head, sc, ids_sorted,
                     lv, n_img, rows_per_img, img_h, img_w, cboxes, cscores, cvalid, clvl);
  int rc = nms_batched(cboxes, cscores, cvalid, clvl, n_img, K, iou_thr, max_keep, nms_ws, keep_buf, n_props, s);
  if (rc) return rc;
  hipLaunchKernelGGL(gather_boxes_kernel, blocks_for((int64_t)n_img * max_keep), dim3(256), 0, s, cboxes, cscores,
                     keep_buf, n_img, K, max_keep, props, prop_scores);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int roi_align(const DetFeats& fs, const float* rois, const int32_t* n_rois, int n_img, int max_rois, bf16_t* out,
              hipStream_t s) {
  hipLaunchKernelGGL(roi_align_kernel, dim3(n_img * max_rois), dim3(256), 0, s, fs, rois, n_rois, max_rois, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t rcnn_workspace_bytes(int n_img, int max_rois) {
  return (size_t)n_img * max_rois * 24 + nms_workspace_bytes(n_img, max_rois) + (size_t)n_img * 128 * 4 + 2048;
}

int rcnn_post(const float* rois, const float* head, const int32_t* n_rois, int n_img, int max_rois, float img_h,
              float img_w, float inv_sw, float inv_sh, float score_thr, float iou_thr, int max_det, void* ws,
              float* det_boxes, float* det_scores, int32_t* n_det, int32_t* keep_buf, hipStream_t s) {
  char* p = static_cast<char*>(ws);
  auto take = [&](size_t b) {
    char* q = p;
    p += (b + 255) & ~(size_t)255;
    return q;
  };
  float* boxes = reinterpret_cast<float*>(take((size_t)n_img * max_rois * 16));
  float* scores = reinterpret_cast<float*>(take((size_t)n_img * max_rois * 4));
  uint8_t* valid = reinterpret_cast<uint8_t*>(take((size_t)n_img * max_rois));
  void* nms_ws = take(nms_workspace_bytes(n_img, max_rois));
  hipLaunchKernelGGL(rcnn_decode_kernel, blocks_for((int64_t)n_img * max_rois), dim3(256), 0, s, rois, head, n_rois,
                     n_img, max_rois, img_h, img_w, inv_sw, inv_sh, score_thr, boxes, scores, valid);
  int rc = nms_batched(boxes, scores, valid, nullptr, n_img, max_rois, iou_thr, max_det, nms_ws, keep_buf, n_det, s);
  if (rc) return rc;
  hipLaunchKernelGGL(gather_boxes_kernel, blocks_for((int64_t)n_img * max_det), dim3(256), 0, s, boxes, scores,
                     keep_buf, n_img, max_rois, max_det, det_boxes, det_scores);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int det_topk_boxes(const float* dboxes, const float* dscores, const int32_t* dcount, int n_img, int max_det, int k,
                   float thr, double min_margin, double max_margin, double desired_ar, float* boxes, float* tight,
                   int32_t* img_of, int32_t* valid, hipStream_t s) {
  hipLaunchKernelGGL(det_topk_boxes_kernel, dim3((n_img + 63) / 64), dim3(64), 0, s, dboxes, dscores, dcount, n_img,
                     max_det, k, thr, min_margin, max_margin, desired_ar, boxes, tight, img_of, valid);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
