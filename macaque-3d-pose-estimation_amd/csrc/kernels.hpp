// Internal launcher declarations of libmq_hip (not part of the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mq {

enum GemmEpilogue {
  EPI_BF16 = 0,       // C bf16 = acc + bias
  EPI_GELU_BF16 = 1,  // C bf16 = gelu_erf(acc + bias)
  EPI_RESID_F32 = 2,  // C f32 += acc + bias            (residual stream)
  EPI_POS_F32 = 3,    // C f32 = acc + bias + aux[m % aux_rows][n]   (patch embed + pos_embed)
  EPI_F32 = 4,        // C f32 = acc + bias
  EPI_NCHW_F32 = 5,   // C f32 [m / aux_rows][n][m % aux_rows] = acc + bias (1x1 conv -> NCHW)
  EPI_RELU_BF16 = 6,  // C bf16 = max(acc + bias, 0)   (detector convs / fc layers)
  EPI_RESID_RELU = 7, // C f32 = max(C + acc + bias, 0), C2 bf16 = the same (ResNet bottleneck output)
};

struct GemmArgs {
  const unsigned short* A;  // [M][lda] bf16, K-contiguous
  const unsigned short* W;  // [N][ldw] bf16, K-contiguous
  void* C;
  const float* bias;        // [N] or null
  const float* aux;         // epilogue side input
  int M, N, K;
  int lda, ldw, ldc;
  int aux_rows;
  // implicit 3x3 / stride 1 / pad 1 convolution (conv_c > 0): A is the NHWC input, M = n * conv_h * conv_w
  // output pixels, lda = conv_c channels, K = 9 * conv_c in (ky * 3 + kx) * conv_c + c order; the A tile
  // rows of each K-step are gathered from the tap's shifted pixels (zeros outside the image)
  int conv_h = 0, conv_w = 0, conv_c = 0;
  // implicit k x k / stride / pad convolution in the 128x128 / 64x64 kernel (conv_c % 64 == 0): conv_h /
  // conv_w are the INPUT size, M = n * OH * OW output pixels, K = k * k * conv_c in (ky * k + kx) * C + c
  // order (the ID classifier's mq_id_im2col order); the ping-pong conv path takes 3 / 1 / 1 only
  int conv_k = 3, conv_s = 1, conv_p = 1;
  void* C2 = nullptr;       // EPI_RESID_RELU: bf16 copy of the output, ldc
  // EPI_BF16 with head_dim > 0: head-major output, column n of row m at
  // C[((n / head_dim) * M + m) * head_dim + n % head_dim] (the ViT qkv GEMM -> attention; ldc unused)
  int head_dim = 0;
};

// bf16 output address of element (m, n) of a GEMM (row-major, or head-major blocks)
__device__ __forceinline__ unsigned short* gemm_out_bf16(const GemmArgs& p, int m, int n) {
  if (p.head_dim)
    return (unsigned short*)p.C + ((size_t)(n / p.head_dim) * p.M + m) * p.head_dim + (n - (n / p.head_dim) * p.head_dim);
  return (unsigned short*)p.C + (size_t)m * p.ldc + n;
}

int gemm_bf16(const GemmArgs& p, int epi, hipStream_t stream);
// implicit-GEMM 3x3 convolution (ping-pong kernel only; conv_c % 64 == 0)
int conv3x3_bf16(const GemmArgs& p, int epi, hipStream_t stream);
// k x k / stride / pad convolution as an implicit GEMM on the 128x128 / 64x64 kernel (same bits as
// mq_id_im2col + gemm_bf16 on those tiles); conv_c % 64 == 0
int conv_small_bf16(const GemmArgs& p, int epi, hipStream_t stream);
// ConvTranspose2d(k4, s2, p1) as one sub-pixel implicit GEMM (ping-pong kernel): A = NHWC input
// (conv_h x conv_w x conv_c), W = deconv_subpixel_pack output [4 classes x C_out][4 taps x conv_c],
// bias [4 x C_out], C = NHWC (2 conv_h x 2 conv_w x C_out) bf16; C_out % 256 == 0, conv_c % 64 == 0
int deconv_subpixel_bf16(const GemmArgs& p, int epi, hipStream_t stream);
// routing knobs (mq_set_tuning): both settings give correct results
extern bool g_gemm_force_small;  // every GEMM on the 128x128 kernel
extern int g_gemm_tile64;        // 64x64 tiles for GEMMs that cannot fill the CUs with 128x128 ones
// ping-pong 256x256 kernel (gemm_pp.hip): the two wave groups of a block alternate LDS traffic and MFMA
extern int g_gemm_pingpong;
bool gemm_pingpong_fits(const GemmArgs& p, int epi, int num_cus);
int gemm_pingpong(const GemmArgs& p, int epi, int num_cus, hipStream_t stream);
int gemm_pingpong_conv(const GemmArgs& p, int epi, int num_cus, hipStream_t stream);
int gemm_pingpong_deconv(const GemmArgs& p, int epi, int num_cus, hipStream_t stream);
// one-wave-per-SIMD 256x256 kernel, 128 x 128 per wave (gemm_w4.hip): bf16 epilogues, K % 32 == 0
extern int g_gemm_w4;  // MQ_TUNE_GEMM_W4
bool gemm_w4_fits(const GemmArgs& p, int epi);
int gemm_w4(const GemmArgs& p, int epi, int num_cus, hipStream_t stream);

// ViT ops (vit_ops.hip)
int layernorm_f32_bf16(const float* x, const float* gamma, const float* beta, unsigned short* y, int rows, int dim,
                       float eps, hipStream_t s);
int layernorm_f32_f32(const float* x, const float* gamma, const float* beta, float* y, int rows, int dim, float eps,
                      hipStream_t s);
// x += p1 (+= p2) (bf16 branch outputs, added in that order), x written back when store_x, y = LayerNorm(x)
// in bf16: the pre-norm residual updates fused into the next block's norm (p2 may be null)
int add_layernorm_f32_bf16(float* x, const unsigned short* p1, const unsigned short* p2, bool store_x,
                           const float* gamma, const float* beta, unsigned short* y, int rows, int dim, float eps,
                           hipStream_t s);
// head_major: qkv holds the head-major blocks of the qkv GEMM's head_dim output (GemmArgs::head_dim)
extern int g_attn_kring;  // MQ_TUNE_ATTN_KRING
int attention_bf16(const unsigned short* qkv, unsigned short* out, int n_img, int tokens, int dim, int heads,
                   hipStream_t s, bool head_major = false);
int patch_im2col(const float* crops, unsigned short* A, int n_crops, int flip_copies, int img_h, int img_w,
                 int patch, int pad, hipStream_t s);
int deconv_col2im_bn_relu(const unsigned short* cols, const float* scale, const float* shift, unsigned short* out,
                          int n_img, int in_h, int in_w, int ch, hipStream_t s);
int convert_f32_bf16(const float* src, unsigned short* dst, int64_t n, hipStream_t s);
int deconv_weight_pack(const float* w, unsigned short* dst, int cin, int cout, hipStream_t s);
// [cin][cout][4][4] f32 (x scale[co] when scale != null) -> sub-pixel GEMM weights (deconv_subpixel_bf16)
int deconv_subpixel_pack(const float* w, const float* scale, unsigned short* dst, int cin, int cout, hipStream_t s);

// image ops (imgproc.hip)
int crop_udp(const uint8_t* frames, int64_t frame_stride, int img_h, int img_w, const float* boxes,
             const int32_t* box_frame, int n, float* crops, float* center, float* scale, hipStream_t s);
int flip_average(const float* hm_all, float* avg, int n, int joints, int h, int w, const int32_t* flip_idx,
                 hipStream_t s);
int udp_decode(const float* avg, int n, int joints, int h, int w, const float* center, const float* scale,
               int in_w, int in_h, float* work, double* kp_img, float* score, int32_t* argmax, float* kp_hm,
               hipStream_t s);

// optim_points (optim.hip)
extern int g_optim_pcg_iters;
extern int g_optim_stop;  // optim_points stop-rule bits (MQ_TUNE_OPTIM_STOP)
extern int g_optim_precond_lds;  // 1 (default): LDS-staged preconditioner when the series fits; 0: global memory
size_t optim_workspace_bytes(int B, int F, int J, int NL);
int optim_points(const double* cams, int C, const double* p2d, double* x, int B, int F, int J, const int* cons_host,
                 int n_strong, int n_weak, const double* ssf_host, double scale_length, double scale_length_weak,
                 double rp, int loss, int n_deriv, int fix_lengths, int max_iter, double ftol, void* ws,
                 double* stats, hipStream_t s);
// the scipy-faithful trust-region solver (optim_trf.hip); stats (B, 8)
extern int g_optim_trf_chunk;
extern int g_optim_trf_fb;
size_t optim_trf_workspace_bytes(int B, int F, int J, int C, int NL);
int optim_points_trf(const double* cams, int C, const double* p2d, double* x, int B, int F, int J, const int* cons_host,
                     int n_strong, int n_weak, const double* ssf_host, double scale_length, double scale_length_weak,
                     double rp, int loss, int n_deriv, int fix_lengths, int max_nfev, double ftol, void* ws,
                     double* stats, hipStream_t s);

}  // namespace mq
