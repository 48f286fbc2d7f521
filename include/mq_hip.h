/*
 * mq_hip.h -- C ABI of libmq_hip.so, the MI355X (gfx950) implementation of the
 * per-frame 2D->3D pose hot path of sidd-bme/macaque-3d-pose-estimation.
 *
 * Conventions:
 *   - every function returns 0 on success, < 0 on error; mq_last_error() gives text;
 *   - the caller owns every data buffer (device pointers unless stated otherwise);
 *     contexts / models own their weights and workspaces;
 *   - work is stream ordered on the hipStream_t passed as `void* stream`
 *     (NULL = the null stream); nothing synchronises unless stated;
 *   - a context owns per-device scratch (decode, Viterbi, optim_points and affinity
 *     workspaces) and a model owns its activations and mq_topdown staging: calls that
 *     share one mq_ctx (or one mq_vitpose) must be issued on ONE stream (or be ordered
 *     by the caller); use one context per stream for concurrent work;
 *   - missing 2D / 3D data is NaN on the way in and out (Viterbi emits (-1,-1,0.001)
 *     for missing frames exactly like anipose).
 *
 * Camera parameter rows (`cams`, float64, 24 values per camera, device memory):
 *   fx, fy, skew, cx, cy, xi, d0, d1, d2, d3, R00..R22 (row-major, from rvec via
 *   Rodrigues), t0, t1, t2, model, d4.  `model` selects the camera class
 *   CameraGroup.from_dicts builds (cameras.py:1972-1982):
 *     0  OmnidirCamera (cameras.py:429-555): K / xi, d0..d3 = D (k1, k2, p1, p2), d4 = 0;
 *     1  Camera, pinhole (cameras.py:173-337): matrix, d0..d4 = distortions (k1, k2, p1, p2, k3),
 *        xi = skew = 0 (cv2.projectPoints / undistortPoints do not use the matrix's skew);
 *     2  FisheyeCamera (cameras.py:339-426): matrix, d0..d3 = distortions (k1..k4), xi = skew = d4 = 0.
 *   Every geometry entry point below (undistort, project, DLT, RANSAC, reprojection error,
 *   optim_points) runs the model of each row; any other model value gives NaN results.
 */
#ifndef MQ_HIP_H
#define MQ_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history:
 *   1 -- rounds 1-2.
 *   2 -- mq_viterbi_filter accepts n_back in [1, 3] only (was [1, 8]); the timing-ablation tuning keys and
 *        MQ_TUNE_ATTENTION_V2 (key 17, the first-generation attention kernel) were removed and now return -2;
 *        MQ_TUNE_OPTIM_PCG_ITERS defaults to 20 (was 40; optim_points results stay within their tolerance);
 *        mq_det_topk_boxes (config-5 capturable box selection) and mq_optim_prepare (host initialisation) added.
 *   3 -- camera rows carry a model (slot 22: 0 omnidir, 1 pinhole, 2 fisheye) and a fifth distortion
 *        coefficient (slot 23); rows written for ABI 1-2 (zeros there) keep the omnidir meaning.
 *        mq_camera_undistort / mq_camera_project added (mq_omnidir_* are the same functions).
 *   4 -- mq_alldata_json (host: step 1's alldata.json text from row arrays) added.
 *   5 -- mq_add_layernorm added; tuning key MQ_TUNE_OPTIM_STOP (21) added; optim_points defaults to 40 PCG iterations per LM step and
 *        the ftol test on two accepted steps in a row (it lands closer to the converged solution than
 *        scipy's own ftol stop on ViT-derived 2D).
 *   6 -- MQ_TUNE_OPTIM_STOP bit 4: the ftol test at ftol / 2; default 6 (two steps in a row at ftol / 2: at or
 *        below scipy's cost on every marker scene probed, where ftol alone stopped 1.5 % above it on one).
 *   7 -- mq_optim_points takes a solver (0: scipy's trust-region-reflective + lsmr, restated -- the default and
 *        the parity mode; 1: the Levenberg-Marquardt + PCG solver of ABI 1-6) and writes 8 stats per animal;
 *        tuning keys MQ_TUNE_OPTIM_TRF_CHUNK (22), MQ_TUNE_VIT_RESID_F32 (23), MQ_TUNE_ATTN_KRING (24) and
 *        MQ_TUNE_OPTIM_TRF_FB (25) added; tuning key MQ_TUNE_GEMM_BLASLT (26) and mq_gemm_plans added.
 *   8 -- the hipBLASLt route is gone: every GEMM of the library is a hand-written kernel.  MQ_TUNE_GEMM_BLASLT (26)
 *        now returns -2 like any unknown key, and mq_gemm_plans was removed.  MQ_TUNE_GEMM_W4 (27) and the host-only
 *        mq_trust_region_2d added. */
#define MQ_ABI_VERSION 8

typedef struct mq_ctx mq_ctx;
typedef struct mq_vitpose mq_vitpose;

int mq_abi_version(void);
const char* mq_last_error(void);

/* Process-wide knobs for A/B measurement.  The kernel-routing knobs select variants that compute the
 * same results (tested equal); the PCG cap changes only the inner-solve accuracy of optim_points,
 * whose results stay within that stage's tolerance.  No knob can select a variant that computes
 * something else.  Changing one makes the next mq_vitpose_forward re-capture its graph. */
#define MQ_TUNE_GEMM_FORCE_SMALL 2  /* 1: route every GEMM to the 128x128 / 64x64 kernel (default 0; the reference
                                       route of the bitwise implicit-convolution tests) */
#define MQ_TUNE_OPTIM_PCG_ITERS 4   /* cap on the conjugate-gradient iterations per Levenberg-Marquardt step (default 40;
                                       results stay within the optim_points tolerance) */
#define MQ_TUNE_GEMM_PINGPONG 12    /* 1 (default): 256x256 GEMMs with K % 64 == 0 on the ping-pong kernel (wave groups
                                       alternate LDS traffic and MFMA, gemm_pp.hip); 0: the interleaved-K-step kernel */
#define MQ_TUNE_OPTIM_PRECOND_LDS 18 /* 1 (default): optim_points' preconditioner on the series staged in LDS when it
                                        fits; 0: the global-memory substitution kernel (same preconditioner) */
#define MQ_TUNE_GEMM_TILE64 19      /* 1 (default): GEMMs whose 128x128 tiles cannot occupy every CU once take the
                                       64x64-tile kernel (same accumulation order, tested equal); 0: 128x128 */
#define MQ_TUNE_QKV_HEAD_MAJOR 20   /* 1 (default): the ViT qkv GEMM writes Q / K / V head-major (each head's rows
                                       contiguous) for the attention's loads; 0: row-major (same results) */
#define MQ_TUNE_OPTIM_STOP 21       /* optim_points' stop rule on an accepted LM step, bits: 0 = scipy's ftol test
                                       alone (dF < ftol F); 1 = and the step's actual / predicted reduction > 0.25
                                       (scipy trf's condition); 2 = the test passed on two accepted steps in a row;
                                       4 = the test at ftol / 2.  Default 6 (2 | 4).  Levenberg-Marquardt solver only */
#define MQ_TUNE_VIT_RESID_F32 23    /* 1: the ViT's proj / fc2 add their f32 accumulators to the residual stream in the
                                       GEMM epilogue (rounds 1-3); 0 (default): bf16 branch outputs added in the
                                       LayerNorm passes (round 4).  A precision A/B knob */
#define MQ_TUNE_ATTN_KRING 24       /* 1 (default): 192-token attention with the inline-asm K-fragment ring; 0: the
                                       compiler-scheduled loop (bit-identical; the fallback for a toolchain change) */
#define MQ_TUNE_OPTIM_TRF_CHUNK 22  /* lsmr iterations the trust-region solver launches between two reads of its done
                                       flags (default 16, 1..64; same results) */
#define MQ_TUNE_OPTIM_TRF_FB 25     /* most frames per workgroup of the trust-region solver's kernels (default 4, 1..4;
                                       same algorithm, the fixed reduction order follows the blocks) */
#define MQ_TUNE_GEMM_W4 27          /* 1: the ViT's bf16-output GEMMs (qkv, proj, fc1, fc2, deconv 1) on the one-wave-per-SIMD
                                       256x256 kernel (128 x 128 per wave, gemm_w4.hip); 0: the ping-pong kernel.  Same
                                       accumulation order, the same bits */
int mq_set_tuning(int key, int value);
/* Current value of a tuning knob (negative on an unknown key). */
int mq_get_tuning(int key);
/* Bind a context to HIP device `device`. */
int mq_create(int device, mq_ctx** out);
int mq_destroy(mq_ctx* ctx);

/* ======================================================================= pose
 * Replaces mmpose.apis.init_model + inference_topdown for the ViTPose top-down
 * model (reference: src/pipeline/step1_proc2d.py:100-101 init, :294-298 call,
 * model/pose/td-hm_ViTPose-huge_8xb64-210e_coco-256x192_sn_macaque.py:54-110).
 */

/* Create an (empty) ViTPose model: ViT-H = (1280, 32, 16, 5120, 17); ViT-B = (768, 12, 12, 3072, 17). */
int mq_vitpose_create(mq_ctx* ctx, int embed_dims, int num_layers, int num_heads, int ffn_dims, int n_joints,
                      mq_vitpose** out);
int mq_vitpose_destroy(mq_vitpose* model);

/* Load one float32 parameter by its mmpose state_dict name (e.g.
 * "backbone.layers.3.attn.qkv.weight", "head.deconv_layers.1.running_var").
 * `data` is device memory if on_device != 0, host memory otherwise.  Synchronous. */
int mq_vitpose_set_param(mq_vitpose* model, const char* name, const float* data, int64_t numel, int on_device);

/* Verify every parameter was loaded and fold the eval BatchNorms. */
int mq_vitpose_finalize(mq_vitpose* model);

/* Enable (1) / disable (0) hipGraph capture + replay of mq_vitpose_forward. */
int mq_vitpose_set_graph(mq_vitpose* model, int enable);

/* Live kernel timing for roofline reporting: while enabled, eager forwards (graph
 * replay is bypassed) record hipEvents around every FFN fc1 GEMM launch on the
 * launch stream.  _result synchronises on them and returns the average duration
 * (ms) per launch, the launch count, and the algorithmic FLOPs of one launch. */
int mq_vitpose_timing(mq_vitpose* model, int enable);
int mq_vitpose_timing_result(mq_vitpose* model, double* avg_ms, int* count, int64_t* flops_per_launch);

/* GetBBoxCenterScale(1.25) + TopdownAffine(UDP, 192x256) + PoseDataPreprocessor.
 *   frames   : uint8 BGR images, image i at frames + i * frame_stride, each height x width x 3
 *   boxes    : float32 (n, 4) xyxy;  box_frame : int32 (n,) image index of each box
 *   crops    : float32 (n, 3, 256, 192) normalised RGB (the model input)
 *   center, scale : float32 (n, 2)  (PoseDataSample input_center / input_scale)      */
int mq_crop_udp(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int height, int width,
                const float* boxes, const int32_t* box_frame, int n, float* crops, float* center, float* scale,
                void* stream);

/* Heatmaps of n crops: float32 (n, J, 64, 48).  With flip_test the model runs 2n
 * forwards and returns (H + flip_back(H_flip)) * 0.5 (test_cfg flip_mode 'heatmap'). */
int mq_vitpose_forward(mq_vitpose* model, const float* crops, int n, int flip_test, float* heatmaps, void* stream);

/* UDPHeatmap.decode (get_heatmap_maximum + refine_keypoints_dark_udp, blur 11) and
 * add_pred_to_datasample.  kp_img float64 (n, J, 2) image pixels; score float32 (n, J);
 * argmax int32 (n, J) flat heatmap index; kp_hm float32 (n, J, 2) heatmap-space (may be NULL). */
int mq_decode_udp(mq_ctx* ctx, const float* heatmaps, int n, int n_joints, int hm_h, int hm_w,
                  const float* center, const float* scale, double* kp_img, float* score, int32_t* argmax,
                  float* kp_hm, void* stream);

/* crop -> forward(flip) -> decode in one call (inference_topdown batched over boxes of
 * many views).  heatmaps may be NULL. */
int mq_topdown(mq_vitpose* model, const uint8_t* frames, int64_t frame_stride, int height, int width,
               const float* boxes, const int32_t* box_frame, int n, int flip_test, double* kp_img, float* score,
               int32_t* argmax, float* heatmaps, void* stream);

/* bf16 MFMA GEMM building block used by the forward: C[M,N] = A[M,K] * W[N,K]^T + bias
 * (A, W bf16 K-contiguous; leading dims in elements).  epilogue: 0 C bf16, 1 C bf16 with
 * exact-erf GELU, 2 C f32 += (residual), 3 C f32 = . + aux[m % aux_rows][n] (pos_embed),
 * 4 C f32, 5 C f32 scattered to [m / aux_rows][n][m % aux_rows] (NCHW), 6 C bf16 = max(., 0) (ReLU).
 * bias/aux may be NULL. */
int mq_gemm_bf16(mq_ctx* ctx, const void* A, const void* W, void* C, const float* bias, const float* aux, int M,
                 int N, int K, int lda, int ldw, int ldc, int aux_rows, int epilogue, void* stream);

/* k x k / stride / pad convolution as an implicit GEMM (no im2col buffer): x bf16 NHWC (n_img, height, width,
 * ch), ch % 64 == 0; w bf16 (cout, k * k * ch) in the mq_id_im2col order ((ky * k + kx) * ch + c); out
 * (n_img * OH * OW, cout) with epilogue 0 (bf16), 4 (f32) or 6 (ReLU bf16) of mq_gemm_bf16, plus bias.  The
 * same bits as mq_id_im2col + mq_gemm_bf16: the ID classifier's 3x3 and strided 1x1 convolutions. */
int mq_id_conv_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch, int k, int stride,
                    int pad, const uint16_t* w, const float* bias, void* out, int cout, int epilogue, void* stream);

/* C f32 (M, ldc) = max(C + A W^T + bias, 0) and out bf16 (M, ldc) = the same values: a ResNet bottleneck's
 * conv3 + residual add + ReLU in one pass (mmpretrain Bottleneck.forward, the ID classifier
 * model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py backbone), K % 64 == 0. */
int mq_gemm_resid_relu_bf16(mq_ctx* ctx, const void* A, const void* W, float* C, const float* bias, uint16_t* out,
                            int M, int N, int K, int lda, int ldw, int ldc, void* stream);

/* ======================================================================= detector
 * Building blocks of the step-1 detector, Swin-S Mask R-CNN bbox only
 * (model/detection/SWIN-Mask_R-CNN_bbox_only.py:29-226, inference_detector at step1_proc2d.py:226):
 * the GEMMs and LayerNorms of the backbone / FPN / heads go through mq_gemm_bf16 and mq_layernorm;
 * mqhip/detector.py sequences them.  Feature maps are NHWC f32, GEMM operands bf16 (uint16 storage).
 * Pointers are device pointers unless marked host. */

/* cv2.resize(INTER_LINEAR) of uint8 BGR frames (n_img, height, width, 3) to (new_h, new_w) with the
 * 11-bit coefficient tables xofs/xalpha (new_w, 2 per x) and yofs/yalpha (new_h) (device int32), then
 * BGR->RGB, (x - mean) / std, zero pad to (pad_h, pad_w), written as the 4x4 stride-4 patch-embed
 * im2col operand: patches bf16 (n_img * pad_h/4 * pad_w/4, 64), k = c * 16 + kh * 4 + kw, k >= 48 zero. */
int mq_det_resize_patch(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int n_img, int height, int width,
                        int new_h, int new_w, int pad_h, int pad_w, const int32_t* xofs, const int32_t* xalpha,
                        const int32_t* yofs, const int32_t* yalpha, uint16_t* patches, void* stream);

/* LayerNorm over rows of f32 x (rows, dim), dim % 4 == 0 and <= 3072: y bf16 (out_f32 = 0) or f32. */
int mq_layernorm(mq_ctx* ctx, const float* x, const float* gamma, const float* beta, void* y, int rows, int dim,
                 float eps, int out_f32, void* stream);

/* The pre-norm residual update fused in front of a LayerNorm (ABI 5): x (rows, dim) f32 += p1 (+= p2, in that
 * order; the bf16 branch outputs of the previous GEMMs, bias included; p2 may be null), x written back when
 * store_x, y = LayerNorm(x) in bf16.  dim as mq_layernorm.  Used by the ViT (inside mq_vitpose_forward) and
 * the Swin detector's blocks (x = x + attn(norm1 x); x = x + mlp(norm2 x): SWIN-Mask_R-CNN_bbox_only.py:29-61). */
int mq_add_layernorm(mq_ctx* ctx, float* x, const uint16_t* p1, const uint16_t* p2, int store_x, const float* gamma,
                     const float* beta, uint16_t* y, int rows, int dim, float eps, void* stream);

/* Swin (shifted) window attention, window 7, head_dim 32 (dim = 32 * heads): qkv bf16 (n_img * height *
 * width, 3 * dim) of the LayerNorm-ed tokens, qkv_bias f32 (3 * dim) (the q/k/v of the zero-padded
 * tokens), rel_table f32 (169, heads); out bf16 (n_img * height * width, dim).  shift 0 (W-MSA) or 3
 * (SW-MSA); the zero pad to a multiple of 7, the cyclic shift and its -100 mask, window partition
 * and reverse are done inside (ShiftWindowMSA + WindowMSA, mmdet swin.py). */
int mq_window_attention(mq_ctx* ctx, const uint16_t* qkv, const float* qkv_bias, const float* rel_table, uint16_t* out,
                        int n_img, int height, int width, int dim, int heads, int shift, void* stream);

/* PatchMerging gather: x f32 (n_img, height, width, dim) -> out f32 (n_img * ceil(h/2) * ceil(w/2), 4 dim)
 * in nn.Unfold(2, stride 2) order c * 4 + kh * 2 + kw (odd sizes zero padded at the bottom / right). */
int mq_patch_merge_gather(mq_ctx* ctx, const float* x, int n_img, int height, int width, int dim, float* out,
                          void* stream);

/* FPN top-down: lo (n_img, lo_h, lo_w, ch) += nearest-resized hi (n_img, hi_h, hi_w, ch). */
int mq_upsample_add(mq_ctx* ctx, float* lo, const float* hi, int n_img, int lo_h, int lo_w, int hi_h, int hi_w, int ch,
                    void* stream);

/* 3x3 / stride 1 / pad 1 im2col: x f32 NHWC -> out bf16 (n_img * h * w, 9 * ch), k = (ky * 3 + kx) * ch + c. */
int mq_im2col3x3(mq_ctx* ctx, const float* x, int n_img, int height, int width, int ch, uint16_t* out, void* stream);

/* 3x3 / stride 1 / pad 1 convolution as an implicit GEMM (no im2col buffer): x bf16 NHWC (n_img, h, w, ch),
 * ch % 64 == 0; w bf16 (cout, 9 * ch) with k = (ky * 3 + kx) * ch + c (the mq_im2col3x3 order); out
 * (n_img * h * w, ldc) with epilogue 0 (bf16), 4 (f32) or 6 (ReLU bf16) of mq_gemm_bf16, plus bias.
 * Same bits as mq_im2col3x3 + mq_gemm_bf16 on the bf16-rounded input.  Replaces the detector's FPN output
 * convolutions (neck, SWIN-Mask_R-CNN_bbox_only.py:80-89) and the RPN head convolution (rpn_head, :137). */
int mq_conv3x3_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch, const uint16_t* w,
                    const float* bias, void* out, int cout, int ldc, int epilogue, void* stream);

/* ConvTranspose2d(k4, s2, p1) + per-channel affine (eval BatchNorm) + ReLU as ONE implicit GEMM: the four
 * output parity classes are 2x2 convolutions over the input (sub-pixel decomposition), their taps gathered
 * per K-step and the result stored straight into out, bf16 NHWC (n_img, 2 h, 2 w, cout).  x bf16 NHWC
 * (n_img, h, w, ch), ch % 64 == 0, cout % 256 == 0; w_packed = mq_deconv_subpixel_pack of the torch weight
 * [ch][cout][4][4]; shift4 = the BatchNorm shift repeated for the 4 classes (4 * cout floats, may be null).
 * Replaces the head's second deconvolution + col2im (ViTPose HeatmapHead deconv_layers.3/.4/.5,
 * model/pose/td-hm_ViTPose-huge_8xb64-210e_coco-256x192_sn_macaque.py:85-108). */
int mq_deconv_subpixel_pack(mq_ctx* ctx, const float* w, const float* scale, uint16_t* w_packed, int ch, int cout,
                            void* stream);
int mq_deconv_subpixel_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch,
                            const uint16_t* w_packed, const float* shift4, uint16_t* out, int cout, int relu,
                            void* stream);

/* float32 -> bfloat16, round to nearest even (count elements). */
int mq_f32_to_bf16(mq_ctx* ctx, const float* src, uint16_t* dst, int64_t count, void* stream);

/* max_pool2d(kernel 1, stride 2) = every other pixel: x f32 NHWC -> out (n_img, ceil(h/2), ceil(w/2), ch). */
int mq_subsample2(mq_ctx* ctx, const float* x, int n_img, int height, int width, int ch, float* out, void* stream);

/* mmcv batched_nms + nms (offset 0): per image, candidates with valid != 0, visited in descending score
 * order (ties: lower index first), offset by level * (max coordinate + 1) when level != NULL; keep
 * int32 (n_img, max_keep) candidate indices in visiting order (-1 past n_keep). n_cand <= 8192. */
int mq_nms(mq_ctx* ctx, const float* boxes, const float* scores, const uint8_t* valid, const int8_t* level, int n_img,
           int n_cand, float iou_thr, int max_keep, int32_t* keep, int32_t* n_keep, void* stream);

/* RPNHead._predict_by_feat_single + _bbox_post_process for a batch: head f32 rows level-major over the
 * batch (level l, image i, position p at row n_img * sum_{l'<l} h_l' w_l' + i * h_l w_l + p), 15 columns
 * = the 3 anchor logits then 12 deltas (anchor-major); level_hw host
 * int32 (n_levels, 2), strides host int32, base_anchors host f32 (n_levels, 3, 4).  Sigmoid, top nms_pre
 * per level (stable descending), delta2bbox (stds 1, clip to img_h x img_w), w,h > 0, NMS per level,
 * first max_keep: proposals f32 (n_img, max_keep, 4), scores (n_img, max_keep) (may be NULL), counts. */
int mq_rpn_proposals(mq_ctx* ctx, const float* head, int n_img, int n_levels, const int32_t* level_hw,
                     const int32_t* strides, const float* base_anchors, int nms_pre, float img_h, float img_w,
                     float iou_thr, int max_keep, float* proposals, float* scores, int32_t* counts, void* stream);

/* SingleRoIExtractor + RoIAlign(7, sampling 0, aligned): P2..P5 f32 NHWC with 256 channels (level_hw /
 * strides host), rois f32 (n_img, max_rois, 4) with counts per image -> out bf16 (n_img * max_rois,
 * 256 * 49) in (c, 7, 7) order (rows past a count are zero). */
int mq_roi_align(mq_ctx* ctx, const float* p2, const float* p3, const float* p4, const float* p5,
                 const int32_t* level_hw, const int32_t* strides, const float* rois, const int32_t* counts, int n_img,
                 int max_rois, uint16_t* out, void* stream);

/* Shared2FCBBoxHead.predict_by_feat + multiclass_nms (1 class): head f32 (n_img * max_rois, 6) = 2 logits
 * (class, background) + 4 deltas; softmax, delta2bbox (stds 0.1 0.1 0.2 0.2), clip, * (inv_scale_w,
 * inv_scale_h), score > score_thr, NMS, first max_det: det_boxes (n_img, max_det, 4), det_scores, counts. */
int mq_rcnn_post(mq_ctx* ctx, const float* rois, const float* head, const int32_t* counts, int n_img, int max_rois,
                 float img_h, float img_w, float inv_scale_w, float inv_scale_h, float score_thr, float iou_thr,
                 int max_det, float* det_boxes, float* det_scores, int32_t* det_counts, void* stream);

/* Static top-k crop boxes per image from mq_rcnn_post's output, the capturable stand-in for the tracker's
 * box list in the config-5 per-frame graph: per image the first k detections (score order) with score >
 * score_thr whose int()-truncated box has positive extent (step1_proc2d.py:229-240, 255-268), expanded by
 * step 1's dynamic margin + aspect fix in float64 (step1:270-292; margins / aspect as there: 0.2, 0.5,
 * 0.75).  Out (n_img * k slots): boxes f32 (., 4) expanded xyxy, tight f32 (., 4) the truncated box,
 * img_of int32 (.) = image index, valid int32 (.) = 1 for a filled slot (0: placeholder box
 * (0, 0, 192, 256) so the crop stays in bounds). */
int mq_det_topk_boxes(mq_ctx* ctx, const float* det_boxes, const float* det_scores, const int32_t* det_counts,
                      int n_img, int max_det, int k, float score_thr, double min_margin, double max_margin,
                      double desired_ar, float* boxes, float* tight, int32_t* img_of, int32_t* valid, void* stream);

/* ======================================================================= ID classifier
 * Step-1 collar-ID classifier, ResNet-152 + GlobalAveragePooling + LinearClsHead (6 classes)
 * (model/id/sn_resnet152_8xb32_in1k_pretrained_optimized_finetuned.py:41-73), replacing
 * mmpretrain's ImageClassificationInferencer in classify_patches (step1_proc2d.py:140-163).  The
 * convolutions are mq_id_im2col + mq_gemm_bf16 (folded BN bias, MQ_EPI 6 = ReLU); mqhip/resnet_id.py
 * sequences them.  Maps are NHWC. */

/* classify_patches' crop + cv2.resize(patch, (out_size, out_size), INTER_LINEAR): boxes int32 (n, 5) =
 * (frame, x0, y0, x1, y1), the non-empty numpy slice frames[frame][y0:y1, x0:x1]; out u8 (n, out, out, 3). */
int mq_id_crop_resize(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int height, int width,
                      const int32_t* boxes, int n, int out_size, uint8_t* out, void* stream);

/* The inferencer's test pipeline on square u8 BGR images (n, in_size, in_size, 3): ResizeEdge(edge,
 * 'short', cv2 bilinear) + CenterCrop(crop) + to_rgb + (x - mean) / std -> bf16 NHWC (n, crop, crop, 3). */
int mq_id_preprocess(mq_ctx* ctx, const uint8_t* in, int n, int in_size, int edge, int crop, uint16_t* out,
                     void* stream);

/* im2col of a bf16 NHWC map (n, h, w, c) for a kh x kw / stride / zero-pad convolution:
 * out bf16 (n * oh * ow, kpad), k = (ky * kw + kx) * c + ch, zero for k >= kh * kw * c. */
int mq_id_im2col(mq_ctx* ctx, const uint16_t* x, int n, int h, int w, int c, int kh, int kw, int stride, int pad,
                 int kpad, uint16_t* out, void* stream);

/* MaxPool2d(3, 2, 1) on bf16 NHWC -> (n, (h - 1) / 2 + 1, (w - 1) / 2 + 1, c). */
int mq_id_maxpool(mq_ctx* ctx, const uint16_t* x, int n, int h, int w, int c, uint16_t* out, void* stream);

/* x = relu(x) in place (f32, count % 4 == 0) and y = bf16(x). */
int mq_id_relu_bf16(mq_ctx* ctx, float* x, uint16_t* y, int64_t count, void* stream);

/* GlobalAveragePooling + fc (ncls x c f32, bias) + softmax: x f32 (n, hw, c) -> logits, probs f32 (n, ncls). */
int mq_id_head(mq_ctx* ctx, const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int ncls,
               float* logits, float* probs, void* stream);

/* ======================================================================= geometry
 * Replaces aniposelib CameraGroup (cameras.py:593-783), anipose filter_pose_viterbi
 * (filter_pose.py:48-186) and the mvpose DLT (multicam_toolbox.py:393-486).
 */

/* Camera.undistort_points (cameras.py:310-316, 376-382, 498-507; the row's model) for every camera:
 * pts/out float64 (C, N, 2) normalised image coordinates.  mq_omnidir_undistort is the ABI-2 name. */
int mq_camera_undistort(mq_ctx* ctx, const double* cams, int n_cams, const double* pts, int n, double* out,
                        void* stream);
int mq_omnidir_undistort(mq_ctx* ctx, const double* cams, int n_cams, const double* pts, int n, double* out,
                         void* stream);

/* Camera.project (cameras.py:318-323, 384-390, 509-516; the row's model) for every camera:
 * p3d (N, 3) -> out (C, N, 2) pixels.  mq_omnidir_project is the ABI-2 name. */
int mq_camera_project(mq_ctx* ctx, const double* cams, int n_cams, const double* p3d, int n, double* out,
                      void* stream);
int mq_omnidir_project(mq_ctx* ctx, const double* cams, int n_cams, const double* p3d, int n, double* out,
                       void* stream);

/* CameraGroup.triangulate: pts (C, N, 2) raw pixels (undistort != 0) or undistorted; out (N, 3). */
int mq_triangulate_dlt(mq_ctx* ctx, const double* cams, int n_cams, const double* pts, int n, int undistort,
                       double* out, void* stream);

/* CameraGroup.reprojection_error: p3d (N,3), p2d (C,N,2) -> out (C,N,2) or (N,) if mean. */
int mq_reproj_error(mq_ctx* ctx, const double* cams, int n_cams, const double* p3d, const double* p2d, int n,
                    int mean, double* out, void* stream);

/* CameraGroup.triangulate_ransac (triangulate_possible, n_possible = 1):
 * p3d (N,3), picked uint8 (C,N), p2d (C,N,2), err (N).  threshold 0.5 in the reference. */
int mq_triangulate_ransac(mq_ctx* ctx, const double* cams, int n_cams, const double* pts, int n, int min_cams,
                          double threshold, double* p3d, uint8_t* picked, double* p2d, double* err, void* stream);

/* multicam_toolbox.triangulatePoints: und (C,N,2) undistorted, use uint8 (N,C) -> out (N,3). */
int mq_triangulate_pinv(mq_ctx* ctx, const double* cams, int n_cams, const double* und, const uint8_t* use, int n,
                        double* out, void* stream);

/* step-2 cross-view geometry affinity (geometry_affinity2, step2_crossviewmatching.py:373-432),
 * batched over B frames:
 *   points     : float64 (B, M, J, 3) undistorted x, y and keypoint score per detection
 *   cam_of_det : int32 (B, M) camera index of each detection (its dimGroup slot), -1 = padding
 *   affinity   : float64 (B, M, M); padding rows / columns are 0
 * Rays through each keypoint at depth 0 and 1000 (deproject :327-355), mean line distance over the
 * keypoints both detections score above thr_kp (THR_KP = 0.1) when at least 3 qualify, z-score over
 * the frame's entries below 300, logistic(-5 z), 0 beyond 150. */
int mq_geometry_affinity(mq_ctx* ctx, const double* cams, int n_cams, const double* points, const int32_t* cam_of_det,
                         int B, int M, int J, double thr_kp, double* affinity, void* stream);

/* step-2 matchSVT (step2_crossviewmatching.py:130-216) batched over B keyframes:
 *   S          : float64 (B, Nmax, Nmax) affinity W of each keyframe (first n_det[b] rows / columns used)
 *   n_det      : int32 (B) detections per keyframe (0 = empty keyframe), Nmax <= 64
 *   cam_of_det : int32 (B, Nmax) camera index of each detection (the dimGroup slot); detections of one
 *                camera form one zero block of X
 *   alpha, lambda, mu, tol, max_iter, pselect: matchSVT's keywords (step 2 calls alpha 0.5, lambda 50,
 *                mu 64, tol 5e-4, maxIter 500, pselect 1; dual_stochastic_SVT False -- not supported)
 *   match      : uint8 (B, Nmax, Nmax) = X > 0.5 after the final symmetrisation (0 outside n_det)
 *   x_out      : optional float64 (B, Nmax, Nmax) final X (NULL to skip)
 *   iters      : int32 (B) the last iteration index (the reference's info["iter"]; -1 for empty keyframes)
 * The SVD of the symmetric Y/mu + X is taken as its eigen-decomposition (parallel Jacobi in LDS,
 * warm-started across iterations); see association.hip. */
int mq_match_svt(mq_ctx* ctx, const double* S, const int32_t* n_det, const int32_t* cam_of_det, int B, int Nmax,
                 double alpha, double lambda, double mu, double tol, int max_iter, int pselect, uint8_t* match,
                 double* x_out, int32_t* iters, void* stream);

/* filter_pose_viterbi over every (animal, camera, joint) chain of kp (A,F,C,J,3)
 * [x, y, score] (step 4 layout of kp2d.pickle) -> out (A,F,C,J,3).  Scratch is
 * owned by the context.  score_threshold 0.3, n_back 3, offset_threshold 25 in step 4 (n_back 1..3). */
int mq_viterbi_filter(mq_ctx* ctx, const double* kp, int n_animals, int n_frames, int n_cams, int n_joints,
                      double score_threshold, int n_back, double offset_threshold, double* out, void* stream);

/* Global multi-head self-attention of the ViT encoder (mmpretrain MultiheadAttention, qkv_bias,
 * scale 1/sqrt(head_dim)) -- the building block inside mq_vitpose_forward.
 *   qkv  bf16 (n_img * tokens, 3 * dim) = [q | k | v] per token row; out bf16 (n_img * tokens, dim).
 *   tokens % 32 == 0 and <= 192; head_dim = dim / heads in {64, 80}. */
int mq_attention_bf16(mq_ctx* ctx, const uint16_t* qkv, uint16_t* out, int n_img, int tokens, int dim, int heads,
                      void* stream);

/* optim_points' parameter initialisation on the HOST (no HIP call; host pointers): per animal b of
 * p3ds (B, F, J, 3) float64 (NaN = missing) -> x0 (B, F*J*3 + n_strong + n_weak) = [p3d with every NaN gap
 * of a series linearly interpolated over frames (np.interp; an all-NaN series -> 0), median limb lengths
 * (strong then weak; 0 or > median + 5 MAD -> the median of all)], non-finite -> 0, and scale_smooth_full
 * (B) = scale_smooth / mean |diff(medfilt7(series))|: bit for bit the numpy arithmetic of cameras.py:
 * 1116-1150 / 1670-1697 (np.interp, medfilt_data's padding, np.median, np.linalg.norm and np.mean's
 * summation orders).  constraints: int32 (n_strong + n_weak, 2) joint pairs.  One host thread per animal. */
int mq_optim_prepare(const double* p3ds, int B, int F, int J, const int32_t* constraints, int n_strong, int n_weak,
                     double scale_smooth, double* x0, double* scale_smooth_full);

/* step 1's alldata.json text (step1_proc2d.py:345-375: json.dump of the per-frame row lists
 * [track id, x1, y1, x2, y2, [[x, y, score] x J], assigned id, id score]) from the rows as HOST arrays (no
 * HIP call): nrows int32 (n_frames) rows per frame; tid / assigned int64 (n); box float64 (n, 4); kp
 * float64 (n, J, 3); score float64 (n), n = sum(nrows).  Writes the text, byte for byte Python's
 * json.dumps of those lists (float repr, NaN, ", " separators), into out[cap] and its length into *len;
 * -2 if cap is too small.  Replaces the interpreter-bound json.dumps of step 1's writer. */
int mq_alldata_json(int n_frames, const int32_t* nrows, const int64_t* tid, const double* box, const double* kp,
                    int J, const int64_t* assigned, const double* score, char* out, int64_t cap, int64_t* len);

/* The 2-D trust-region subproblem of scipy's trf (scipy 1.15.3 optimize/_lsq/common.py solve_trust_region_2d, called
 * by trf_no_bounds for each trial step of optim_points' least_squares, cameras.py:1166-1180) on the HOST (no HIP
 * call): minimise 0.5 p^T B p + g^T p subject to |p| <= Delta, B = [B[0] B[1]; B[1] B[2]] (host arrays).  The
 * Newton point when B is positive definite and the point lies inside; else the best boundary point among the real
 * roots of scipy's quartic (found by bracketing and bisection instead of np.roots); when the quartic has no sign
 * change, its touching points, then the Cauchy point -Delta g / |g| (scipy raises there).  Writes p[2]. */
int mq_trust_region_2d(const double* B, const double* g, double Delta, double* p);

/* CameraGroup.optim_points (cameras.py:1116-1190) and optim_points_jointlenfix (:1192-1415) for
 * B animals at once.  Replaces scipy least_squares (cameras.py:1166-1180: trf, 2-point sparse Jacobian,
 * loss 'linear', ftol 1e-3; jointlenfix :1246-1260 adds max_nfev 15) on the analytic Jacobian, with
 *   solver 0: the same algorithm, restated (scipy 1.15.3 trf_no_bounds + lsmr: damped lsmr Gauss-Newton step,
 *             2-D subspace trust region, update_tr_radius, check_termination with ftol / xtol 1e-8 / gtol
 *             1e-8); the parity default (csrc/optim_trf.hip);
 *   solver 1: Levenberg-Marquardt + PCG inner solves with its own stop rule (MQ_TUNE_OPTIM_STOP): a
 *             "converged" mode that stops later than scipy (csrc/optim.hip).
 *   p2d  device (B, C, F, J, 2) float64, NaN = missing coordinate
 *   x    device (B, F*J*3 + n_strong + n_weak) in/out: [p3d, strong lengths, weak lengths]
 *        (the reference's _initialize_params_triangulation layout, :1670-1697)
 *   constraints host int32 (n_strong + n_weak, 2) joint pairs; scale_smooth_full host (B)
 *   reproj_loss 0 linear, 1 soft_l1 (reference default), 2 huber
 *   fix_lengths 1: lengths are constants (jointlenfix variant), only p3d is optimised
 *   max_iter solver 0: max_nfev (0 = scipy's default, 100 x parameters; the jointlenfix call passes 15);
 *            solver 1: Levenberg-Marquardt iterations
 *   stats host (B, 8): initial cost, final cost, iterations, status, then for solver 0 nfev, njev, lsmr
 *         iterations in total, the longest lsmr run.  status, solver 0: scipy's (0 max_nfev, 1 gtol, 2 ftol,
 *         3 xtol, 4 ftol + xtol); solver 1: 1 ftol, 2 max_iter, 3 damping overflow. */
int mq_optim_points(mq_ctx* ctx, const double* cams, int n_cams, const double* p2d, double* x, int n_animals,
                    int n_frames, int n_joints, const int32_t* constraints, int n_strong, int n_weak,
                    const double* scale_smooth_full, double scale_length, double scale_length_weak,
                    double reproj_error_threshold, int reproj_loss, int n_deriv_smooth, int fix_lengths,
                    int max_iter, double ftol, int solver, double* stats, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MQ_HIP_H */
