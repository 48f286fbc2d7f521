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
 *   fx, fy, skew, cx, cy, xi, k1, k2, p1, p2, R00..R22 (row-major, from rvec via
 *   Rodrigues), t0, t1, t2, 0, 0.   (OmnidirCamera K / xi / D / rvec / tvec,
 *   /root/reference/src/third_party/aniposelib/cameras.py:429-555)
 */
#ifndef MQ_HIP_H
#define MQ_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQ_ABI_VERSION 1

typedef struct mq_ctx mq_ctx;
typedef struct mq_vitpose mq_vitpose;

int mq_abi_version(void);
const char* mq_last_error(void);

/* Process-wide knobs for A/B measurement.  The kernel-routing knobs select variants that compute the
 * same results (tested equal); the PCG cap changes only the inner-solve accuracy of optim_points,
 * whose results stay within that stage's tolerance.  No knob can select a variant that computes
 * something else.  Changing one makes the next mq_vitpose_forward re-capture its graph. */
#define MQ_TUNE_GEMM_FORCE_SMALL 2  /* 1: route every GEMM to the 128x128 kernel (default 0) */
#define MQ_TUNE_OPTIM_PCG_ITERS 4   /* cap on the conjugate-gradient iterations per Levenberg-Marquardt step (default 20;
                                       results stay within the optim_points tolerance) */
#define MQ_TUNE_GEMM_PINGPONG 12    /* 1 (default): 256x256 GEMMs with K % 64 == 0 on the ping-pong kernel (wave groups
                                       alternate LDS traffic and MFMA, gemm_pp.hip); 0: the interleaved-K-step kernel */
#define MQ_TUNE_ATTENTION_V2 17     /* 1 (default): attention on 16x16x32 QK^T + transposed-output PV (vit_ops.hip
                                       attention2_kernel); 0: the first-generation kernel */
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
 * 4 C f32, 5 C f32 scattered to [m / aux_rows][n][m % aux_rows] (NCHW).  bias/aux may be NULL. */
int mq_gemm_bf16(mq_ctx* ctx, const void* A, const void* W, void* C, const float* bias, const float* aux, int M,
                 int N, int K, int lda, int ldw, int ldc, int aux_rows, int epilogue, void* stream);

/* ======================================================================= geometry
 * Replaces aniposelib CameraGroup (cameras.py:593-783), anipose filter_pose_viterbi
 * (filter_pose.py:48-186) and the mvpose DLT (multicam_toolbox.py:393-486).
 */

/* OmnidirCamera.undistort_points for every camera: pts/out float64 (C, N, 2). */
int mq_omnidir_undistort(mq_ctx* ctx, const double* cams, int n_cams, const double* pts, int n, double* out,
                         void* stream);

/* OmnidirCamera.project for every camera: p3d (N, 3) -> out (C, N, 2). */
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

/* CameraGroup.optim_points (cameras.py:1116-1190) and optim_points_jointlenfix (:1192-1415) for
 * B animals at once.  Replaces scipy least_squares(trf, 2-point sparse Jacobian) with
 * Levenberg-Marquardt on the analytic Jacobian, PCG inner solves.
 *   p2d  device (B, C, F, J, 2) float64, NaN = missing coordinate
 *   x    device (B, F*J*3 + n_strong + n_weak) in/out: [p3d, strong lengths, weak lengths]
 *        (the reference's _initialize_params_triangulation layout, :1670-1697)
 *   constraints host int32 (n_strong + n_weak, 2) joint pairs; scale_smooth_full host (B)
 *   reproj_loss 0 linear, 1 soft_l1 (reference default), 2 huber
 *   fix_lengths 1: lengths are constants (jointlenfix variant), only p3d is optimised
 *   max_iter LM iterations (reference: unbounded / max_nfev 15), ftol scipy-style on accepted steps
 *   stats host (B, 4): initial cost, final cost, LM iterations, status (1 ftol, 2 max_iter, 3 damping). */
int mq_optim_points(mq_ctx* ctx, const double* cams, int n_cams, const double* p2d, double* x, int n_animals,
                    int n_frames, int n_joints, const int32_t* constraints, int n_strong, int n_weak,
                    const double* scale_smooth_full, double scale_length, double scale_length_weak,
                    double reproj_error_threshold, int reproj_loss, int n_deriv_smooth, int fix_lengths,
                    int max_iter, double ftol, double* stats, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MQ_HIP_H */
