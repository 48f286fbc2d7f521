// hipBLASLt for the ViT's plain bias GEMMs (bf16 A / W / C, f32 bias, f32 accumulation: fc2, proj and
// deconv 1), used only where the library gives the hand kernel's bits faster.
//
// Per (device, shape, strides, bias or not) the first eager call tunes once: the library's heuristic candidates
// run on a random A with the call's W and bias; a candidate is kept only if its whole output equals the hand
// kernel's bit for bit (which rules out split-K sums: the K sum must run in one accumulator in ascending order,
// as in the hand kernels), and the fastest kept one is used if it beats the hand kernel by 2 %.  Every call gets
// a workspace (256 MiB per host thread and device, allocated outside capture), as the library's probes run them:
// per thread, so that two threads' streams never share one.  Otherwise, or
// before tuning (a call inside stream capture never tunes), the caller runs the hand kernel: either route gives
// the same bits, so where the tuning lands never changes a result.  MQ_TUNE_GEMM_BLASLT = 0 turns the route off.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace mq {

int g_gemm_blaslt = 1;

namespace {

// deterministic bf16 in [-1, 1) (a hash of the index): the tuning input
__global__ void blaslt_fill_kernel(unsigned short* a, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 15;
    x *= 2246822519u;
    x ^= x >> 13;
    x *= 3266489917u;
    x ^= x >> 16;
    const float f = (float)(x >> 8) * (1.0f / 8388608.0f) - 1.0f;
    a[i] = (unsigned short)(__float_as_uint(f) >> 16);
  }
}

// per block: 1 if any element of its grid-stride share differs (no atomics: one store per block)
__global__ void blaslt_differs_kernel(const unsigned short* a, const unsigned short* b, size_t n, int* out) {
  int d = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    d |= a[i] != b[i];
  d = __syncthreads_or(d);
  if (threadIdx.x == 0) out[blockIdx.x] = d;
}

constexpr int CMP_BLOCKS = 1024;

struct Key {
  int dev, M, N, K, lda, ldw, ldc, bias;
  bool operator<(const Key& o) const {
    return std::tie(dev, M, N, K, lda, ldw, ldc, bias) < std::tie(o.dev, o.M, o.N, o.K, o.lda, o.ldw, o.ldc, o.bias);
  }
};

struct Plan {
  bool use_lt = false;
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  float ms_hand = 0.f, ms_lt = 0.f;
  int candidates = 0, identical = 0;
};

std::mutex g_mu;                                      // plans, handles, and a plan's descriptor while it launches
std::map<Key, std::unique_ptr<Plan>> g_plans;
hipblasLtHandle_t g_handle[16] = {};
thread_local void* t_ws[16] = {};
constexpr size_t WS_BYTES = (size_t)256 << 20;

// this thread's workspace on dev (null inside a capture that would have to allocate it)
void* workspace(int dev, hipStream_t s);

// a plain GEMM the library can compute: bf16 out with bias or nothing, no fused side input, no implicit
// convolution, no head-major store, sizes where 256 x 256 tiles fill the device
bool eligible(const GemmArgs& p, int epi) {
  return g_gemm_blaslt && epi == EPI_BF16 && !p.head_dim && !p.aux && !p.C2 && !p.conv_c && p.M >= 256 &&
         p.N >= 256 && p.K % 64 == 0 && p.lda % 8 == 0 && p.ldw % 8 == 0 && p.ldc % 8 == 0;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone;
}

template <class F>
float time_ms(F&& run, hipStream_t s, int reps) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1.f;
  float best = -1.f;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(e0, s);
    if (!run()) {
      best = -1.f;
      break;
    }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (best < 0.f || ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

void destroy(Plan& p) {
  if (p.la) (void)hipblasLtMatrixLayoutDestroy(p.la);
  if (p.lb) (void)hipblasLtMatrixLayoutDestroy(p.lb);
  if (p.lc) (void)hipblasLtMatrixLayoutDestroy(p.lc);
  if (p.desc) (void)hipblasLtMatmulDescDestroy(p.desc);
  p = Plan{};
}

// builds the plan for p's key (called with g_mu held, outside capture); a plan that keeps the hand kernel is a
// valid result too.  Nonzero: a HIP / library failure (the call falls back to the hand kernel).
int tune(const GemmArgs& p, int dev, Plan& plan, hipStream_t s) {
  if (!g_handle[dev] && hipblasLtCreate(&g_handle[dev]) != HIPBLAS_STATUS_SUCCESS) return -1;
  void* ws = workspace(dev, s);
  if (!ws) return -1;
  hipblasLtHandle_t lt = g_handle[dev];
  // C^T[N, M] = W[N, K] * A[M, K]^T in hipBLASLt's column-major view: m = N, n = M, op(W) = T, op(A) = N
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  const hipblasLtEpilogue_t ep = p.bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT;
  const hipDataType bdt = HIP_R_32F;
  if (hipblasLtMatmulDescCreate(&plan.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS ||
      hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)) ||
      hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)) ||
      hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) ||
      (p.bias && (hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &p.bias,
                                                  sizeof(p.bias)) ||
                  hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt,
                                                  sizeof(bdt)))) ||
      hipblasLtMatrixLayoutCreate(&plan.la, HIP_R_16BF, p.K, p.N, p.ldw) ||
      hipblasLtMatrixLayoutCreate(&plan.lb, HIP_R_16BF, p.K, p.M, p.lda) ||
      hipblasLtMatrixLayoutCreate(&plan.lc, HIP_R_16BF, p.N, p.M, p.ldc))
    return -1;
  hipblasLtMatmulPreference_t pref = nullptr;
  const uint64_t ws_max = WS_BYTES;
  if (hipblasLtMatmulPreferenceCreate(&pref) ||
      hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws_max, sizeof(ws_max))) {
    if (pref) (void)hipblasLtMatmulPreferenceDestroy(pref);
    return -1;
  }
  hipblasLtMatmulHeuristicResult_t heur[16];
  int nres = 0;
  (void)hipblasLtMatmulAlgoGetHeuristic(lt, plan.desc, plan.la, plan.lb, plan.lc, plan.lc, pref, 16, heur, &nres);
  (void)hipblasLtMatmulPreferenceDestroy(pref);
  plan.candidates = nres;
  if (nres <= 0) return 0;
  // the tuning operands: a random A (same strides), the call's W and bias, two outputs
  const size_t na = (size_t)p.M * p.lda, nc = (size_t)p.M * p.ldc;
  unsigned short *A = nullptr, *C0 = nullptr, *C1 = nullptr;
  int* diff_d = nullptr;
  auto release = [&]() {
    (void)hipStreamSynchronize(s);
    if (A) (void)hipFree(A);
    if (C0) (void)hipFree(C0);
    if (C1) (void)hipFree(C1);
    if (diff_d) (void)hipFree(diff_d);
  };
  if (hipMalloc(&A, na * 2) || hipMalloc(&C0, nc * 2) || hipMalloc(&C1, nc * 2) ||
      hipMalloc(&diff_d, CMP_BLOCKS * sizeof(int))) {
    release();
    return -1;
  }
  hipLaunchKernelGGL(blaslt_fill_kernel, dim3(2048), dim3(256), 0, s, A, na, 0x9e3779b9u);
  (void)hipMemsetAsync(C0, 0, nc * 2, s);
  GemmArgs q = p;
  q.A = A;
  q.C = C0;
  auto run_hand = [&]() { return gemm_bf16(q, EPI_BF16, s) == 0; };
  if (!run_hand()) {
    release();
    return -1;
  }
  const float alpha = 1.f, beta = 0.f;
  std::vector<int> diff(CMP_BLOCKS);
  std::vector<std::pair<float, int>> kept;  // (best of 4 runs in ms, candidate) of the bit-identical ones
  for (int h = 0; h < nres; ++h) {
    if (heur[h].state != HIPBLAS_STATUS_SUCCESS || heur[h].workspaceSize > WS_BYTES) continue;
    auto run_lt = [&]() {
      return hipblasLtMatmul(lt, plan.desc, &alpha, p.W, plan.la, A, plan.lb, &beta, C1, plan.lc, C1, plan.lc,
                             &heur[h].algo, ws, WS_BYTES, s) == HIPBLAS_STATUS_SUCCESS;
    };
    (void)hipMemsetAsync(C1, 0xff, nc * 2, s);
    if (!run_lt()) continue;
    hipLaunchKernelGGL(blaslt_differs_kernel, dim3(CMP_BLOCKS), dim3(256), 0, s, C0, C1, nc, diff_d);
    if (hipMemcpyAsync(diff.data(), diff_d, CMP_BLOCKS * sizeof(int), hipMemcpyDeviceToHost, s) ||
        hipStreamSynchronize(s))
      break;
    if (std::any_of(diff.begin(), diff.end(), [](int d) { return d != 0; })) continue;
    ++plan.identical;
    (void)run_lt();
    const float ms = time_ms(run_lt, s, 4);  // best of 4 (a single timed run misranks the candidates)
    if (ms > 0.f) kept.emplace_back(ms, h);
  }
  std::sort(kept.begin(), kept.end());
  const float best = kept.empty() ? -1.f : kept[0].first;
  const int best_i = kept.empty() ? -1 : kept[0].second;
  (void)run_hand();
  plan.ms_hand = time_ms(run_hand, s, 4);
  plan.ms_lt = best;
  if (best_i >= 0 && plan.ms_hand > 0.f && best < 0.98f * plan.ms_hand) {
    plan.algo = heur[best_i].algo;
    plan.use_lt = true;
  }
  release();
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

void* workspace(int dev, hipStream_t s) {
  if (!t_ws[dev] && !capturing(s) && hipMalloc(&t_ws[dev], WS_BYTES) != hipSuccess) t_ws[dev] = nullptr;
  return t_ws[dev];
}

// p's plan on dev, tuned now if there is none (g_mu held); null inside a capture that would have to tune.  A
// failed tuning is recorded as a hand-kernel plan.
Plan* find_or_tune(const GemmArgs& p, int dev, hipStream_t s) {
  const Key key{dev, p.M, p.N, p.K, p.lda, p.ldw, p.ldc, p.bias ? 1 : 0};
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second.get();
  if (capturing(s)) return nullptr;
  auto plan = std::make_unique<Plan>();
  if (tune(p, dev, *plan, s)) {
    destroy(*plan);
    (void)hipGetLastError();
  }
  return g_plans.emplace(key, std::move(plan)).first->second.get();
}

bool current_device(int& dev) { return hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 16; }

}  // namespace

int gemm_blaslt(const GemmArgs& p, int epi, hipStream_t s) {
  int dev = 0;
  if (!eligible(p, epi) || !current_device(dev)) return 1;
  std::lock_guard<std::mutex> lock(g_mu);
  Plan* found = find_or_tune(p, dev, s);
  if (!found || !found->use_lt) return 1;
  Plan& plan = *found;
  void* ws = workspace(dev, s);
  if (!ws) return 1;
  if (p.bias && hipblasLtMatmulDescSetAttribute(plan.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &p.bias,
                                                sizeof(p.bias)) != HIPBLAS_STATUS_SUCCESS)
    return -5;
  const float alpha = 1.f, beta = 0.f;
  return hipblasLtMatmul(g_handle[dev], plan.desc, &alpha, p.W, plan.la, p.A, plan.lb, &beta, p.C, plan.lc, p.C,
                         plan.lc, &plan.algo, ws, WS_BYTES, s) == HIPBLAS_STATUS_SUCCESS
             ? 0
             : -5;
}

int gemm_blaslt_prepare(const GemmArgs& p, int epi, hipStream_t s) {
  // the plan only (tuning writes private buffers, not p.C) and this thread's workspace: before a graph capture
  // that will launch p
  int dev = 0;
  if (!eligible(p, epi) || !current_device(dev) || capturing(s)) return 0;
  std::lock_guard<std::mutex> lock(g_mu);
  (void)find_or_tune(p, dev, s);
  (void)workspace(dev, s);
  return 0;
}

int gemm_blaslt_report(int index, int* shape, float* ms) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (index < 0 || index >= (int)g_plans.size()) return -1;
  auto it = g_plans.begin();
  std::advance(it, index);
  const Key& k = it->first;
  const Plan& p = *it->second;
  shape[0] = k.M;
  shape[1] = k.N;
  shape[2] = k.K;
  shape[3] = p.use_lt ? 1 : 0;
  shape[4] = p.candidates;
  shape[5] = p.identical;
  ms[0] = p.ms_hand;
  ms[1] = p.ms_lt;
  return 0;
}

}  // namespace mq
