// Internal launchers of the ID-classifier kernels (resnet_id.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mq {

typedef unsigned short bf16_t;

constexpr int ID_MAX_CLASSES = 16;

int id_crop_resize(const uint8_t* frames, int64_t fstride, int W, const int32_t* boxes, int n, int out_size,
                   uint8_t* out, hipStream_t s);
int id_edge_crop(const uint8_t* in, int n, int in_size, int edge, int crop, int off, bf16_t* out, hipStream_t s);
int im2col_bf16(const bf16_t* x, int n, int h, int w, int c, int kh, int kw, int stride, int pad, int kpad,
                bf16_t* out, hipStream_t s);
int maxpool3s2(const bf16_t* x, int n, int h, int w, int c, bf16_t* out, hipStream_t s);
int relu_bf16(float* x, bf16_t* y, int64_t count, hipStream_t s);
int gap_fc_softmax(const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int ncls, float* logits,
                   float* probs, hipStream_t s);

}  // namespace mq
