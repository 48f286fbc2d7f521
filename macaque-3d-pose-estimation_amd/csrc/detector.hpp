// Internal launchers of the detector kernels (detector.hip) and the box arithmetic they share.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mq {

typedef unsigned short bf16_t;

// RPN level geometry of one image (all images of a batch share it)
struct DetLevels {
  int n;                 // levels (5: P2..P6)
  int h[6], w[6];        // feature map sizes
  int stride[6];
  int row_off[6];        // first head row of the level within an image's rows
  int cand_off[6];       // first candidate of the level (top-k per level, level-major)
  int cand_total;
  float base[6][3][4];   // AnchorGenerator base anchors (x1, y1, x2, y2) per ratio
};

// RoIAlign inputs: P2..P5 NHWC f32 (n_img, h, w, 256)
struct DetFeats {
  const float* p[4];
  int h[4], w[4];
  int stride[4];
};

// DeltaXYWHBBoxCoder.decode for one box (deltas already * stds + means), mmdet operation order,
// clipped to [0, img_w] x [0, img_h]
__device__ __forceinline__ void delta2bbox(float x1, float y1, float x2, float y2, float dx, float dy, float dw,
                                           float dh, float img_h, float img_w, float* out) {
  const float max_ratio = 4.135166556742356f;  // |log(16 / 1000)|
  dw = fminf(fmaxf(dw, -max_ratio), max_ratio);
  dh = fminf(fmaxf(dh, -max_ratio), max_ratio);
  const float px = (x1 + x2) * 0.5f, py = (y1 + y2) * 0.5f;
  const float pw = x2 - x1, ph = y2 - y1;
  const float gx = px + pw * dx, gy = py + ph * dy;
  const float gw = pw * expf(dw), gh = ph * expf(dh);
  const float bx1 = gx - gw * 0.5f, by1 = gy - gh * 0.5f, bx2 = gx + gw * 0.5f, by2 = gy + gh * 0.5f;
  out[0] = fminf(fmaxf(bx1, 0.f), img_w);
  out[1] = fminf(fmaxf(by1, 0.f), img_h);
  out[2] = fminf(fmaxf(bx2, 0.f), img_w);
  out[3] = fminf(fmaxf(by2, 0.f), img_h);
}

int det_resize_patch(const uint8_t* frames, int64_t fstride, int n_img, int H, int W, int nh, int nw, int hp, int wp,
                     const int32_t* xofs, const int32_t* xa, const int32_t* yofs, const int32_t* ya, bf16_t* A,
                     hipStream_t s);
int window_attention(const bf16_t* qkv, const float* qkv_bias, const float* rel_table, bf16_t* out, int n_img, int H,
                     int W, int C, int heads, int shift, hipStream_t s);
int merge_gather(const float* x, int n_img, int H, int W, int C, float* out, hipStream_t s);
int upsample_add(float* lo, const float* hi, int n_img, int Hl, int Wl, int Hh, int Wh, int C, hipStream_t s);
int im2col3x3(const float* x, int n_img, int H, int W, int C, bf16_t* out, hipStream_t s);
int subsample2(const float* x, int n_img, int H, int W, int C, float* out, hipStream_t s);
size_t nms_workspace_bytes(int n_img, int n_cand);
int nms_batched(const float* boxes, const float* scores, const uint8_t* valid, const int8_t* lvl, int n_img,
                int n_cand, float thr, int max_keep, void* ws, int32_t* keep, int32_t* n_keep, hipStream_t s);
size_t rpn_workspace_bytes(int n_img, int rows_per_img, int cand_total, int n_levels);
int rpn_proposals(const float* head, const DetLevels& lv, int n_img, int rows_per_img, float img_h, float img_w,
                  float iou_thr, int max_keep, void* ws, size_t ws_bytes, float* props, float* prop_scores,
                  int32_t* n_props, int32_t* keep_buf, hipStream_t s);
int roi_align(const DetFeats& fs, const float* rois, const int32_t* n_rois, int n_img, int max_rois, bf16_t* out,
              hipStream_t s);
size_t rcnn_workspace_bytes(int n_img, int max_rois);
int rcnn_post(const float* rois, const float* head, const int32_t* n_rois, int n_img, int max_rois, float img_h,
              float img_w, float inv_sw, float inv_sh, float score_thr, float iou_thr, int max_det, void* ws,
              float* det_boxes, float* det_scores, int32_t* n_det, int32_t* keep_buf, hipStream_t s);
int det_topk_boxes(const float* dboxes, const float* dscores, const int32_t* dcount, int n_img, int max_det, int k,
                   float thr, double min_margin, double max_margin, double desired_ar, float* boxes, float* tight,
                   int32_t* img_of, int32_t* valid, hipStream_t s);

}  // namespace mq
