// Internal launchers of the float64 geometry kernels (geometry.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mq {
int omnidir_undistort(const double* cams, int C, const double* pts, double* out, int N, hipStream_t s);
int omnidir_project(const double* cams, int C, const double* p3d, double* out, int N, hipStream_t s);
int triangulate_dlt(const double* cams, int C, const double* pts, int N, int undistort, double* out, hipStream_t s);
int reprojection_error(const double* cams, int C, const double* p3d, const double* p2d, int N, int mean, double* out,
                       hipStream_t s);
int triangulate_ransac(const double* cams, int C, const double* pts, int N, int min_cams, double threshold,
                       double* p3d, uint8_t* picked, double* p2d, double* err, hipStream_t s);
int triangulate_pinv(const double* cams, int C, const double* und, const uint8_t* use, int N, double* out,
                     hipStream_t s);
int geometry_affinity(const double* cams, int C, const double* pts, const int32_t* cam_of_det, int B, int M, int J,
                      double thr_kp, double* rays, double* dist, double* out, hipStream_t s);
int viterbi_filter(const double* kp, int A, int F, int C, int J, double score_thr, int n_back, double thres_dist,
                   void* scratch, double* out, hipStream_t s);
size_t viterbi_scratch_bytes(int A, int F, int C, int J, int n_back);
int match_svt(const double* S, const int32_t* n_det, const int32_t* cam_of_det, int B, int Nmax, double alpha,
              double lambda, double mu, double tol, int max_iter, int pselect, void* ws, uint8_t* match,
              double* x_out, int32_t* iters, hipStream_t s);
size_t match_svt_workspace_bytes(int B, int Nmax);
}  // namespace mq
