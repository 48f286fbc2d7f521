// C ABI + native runtime of libmq_hip (include/mq_hip.h).
//
// The ViTPose runtime owns bf16 weights laid out for the MFMA GEMM (K-contiguous,
// deconvs packed as [(ky*4+kx)*Cout + co][Cin]) and a workspace sized for the
// largest batch seen; a forward is ~7 launches per encoder layer, optionally
// captured once into a hipGraph and replayed (keyed on batch size and the
// caller's input/output pointers).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "geometry.hpp"
#include "detector.hpp"
#include "idcls.hpp"
#include "kernels.hpp"
#include "mq_hip.h"

namespace {

thread_local std::string g_err;
// ViT qkv GEMM output head-major for the attention (MQ_TUNE_QKV_HEAD_MAJOR; 0: row-major, same bits)
int g_qkv_head_major = 1;
// MQ_TUNE_VIT_RESID_F32: 1 = the ViT's residual updates as f32 read-modify-write GEMM epilogues (rounds 1-3);
// 0 (default) = bf16 branch outputs added in the LayerNorm passes (round 4).  A precision A/B of that choice.
int g_vit_resid_f32 = 0;
int g_tuning_gen = 0;  // bumped by mq_set_tuning

int fail(const std::string& msg, int code = -1) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(std::string(#expr ": ") + hipGetErrorString(e_), -5); \
  } while (0)

#define K_TRY(expr)                                              \
  do {                                                           \
    int r_ = (expr);                                             \
    if (r_ != 0) return fail(std::string(#expr " failed"), -6);  \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t b) {
    if (b <= bytes) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, b) != hipSuccess) return -1;
    bytes = b;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

}  // namespace

struct mq_ctx {
  int device = 0;
  DevBuf scratch;  // geometry scratch (Viterbi back-pointers)
  DevBuf decode_work;
  DevBuf optim_ws;
  DevBuf assoc_ws;  // step-2 affinity: rays + pairwise distances
  DevBuf det_ws;    // detector post-processing (sort, NMS masks)
  DevBuf dlt_ws;    // mq_triangulate_dlt: undistorted points
};

struct ParamSlot {
  int kind;  // 0 bf16 linear/conv, 1 f32 plain, 2 deconv pack, 3 bn part (f32 host copy)
  int64_t numel;
  void* dst;
  int cin, cout;
  bool loaded = false;
};

struct Layer {
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  unsigned short *wqkv, *wproj, *wfc1, *wfc2;
  float *bqkv, *bproj, *bfc1, *bfc2;
};

struct mq_vitpose {
  mq_ctx* ctx;
  int D, L, H, FF, J;
  int img_h = 256, img_w = 192, patch = 16, pad = 2, dc = 256;
  int gh, gw, T;
  DevBuf weights;  // one arena
  std::vector<Layer> layers;
  unsigned short *w_patch, *w_dc1, *w_dc2, *w_fin;
  float *b_patch, *pos, *lnf_g, *lnf_b, *b_fin;
  float *bn1_scale, *bn1_shift, *bn2_scale, *bn2_shift;
  // deconv 2 as one sub-pixel implicit GEMM (dc % 256 == 0): its f32 weights are kept until finalize,
  // which packs them with the BatchNorm scale folded in (w_dc2) and replicates the shift per class
  bool dc2_subpixel = false;
  float *w_dc2_f32 = nullptr, *bn2_shift4 = nullptr;
  std::vector<float> bn_host[8];  // w1,b1,rm1,rv1,w2,b2,rm2,rv2
  int32_t* flip_idx;
  std::map<std::string, ParamSlot> slots;
  bool finalized = false;
  // workspace
  DevBuf ws;
  int ws_F = 0;
  unsigned short *A0, *Hn, *QKV, *O, *G, *Y1, *cols2, *Y2;
  float *X, *hm_all;
  // graph cache (captured and replayed on a private non-blocking stream that is
  // event-ordered after / before the caller's stream, so callers may pass the
  // legacy null stream, which cannot be captured)
  hipStream_t cap_stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  bool use_graph = false;
  hipGraphExec_t gexec = nullptr;
  int g_n = -1, g_flip = -1, g_gen = -1;
  const void* g_in = nullptr;
  void* g_out = nullptr;
  // live kernel timing (eager forwards only): hipEvent pairs around every FFN fc1
  // GEMM launch, recorded on the stream the kernel is launched on
  bool timing = false;
  int64_t g_rows_timed = 0;
  std::vector<hipEvent_t> t_events;
  size_t t_used = 0;
  DevBuf stage;  // mq_topdown: crops, center / scale, heatmaps (allocated on the model's device)
};

extern "C" {

int mq_abi_version(void) { return MQ_ABI_VERSION; }

// Knobs select between variants that compute the same results (kernel routing, tested equal) or
// bound the inner-solver iterations of optim_points (results within that stage's tolerance).  A change
// bumps the generation so that ViTPose graphs captured under the old routing are re-captured.
int mq_set_tuning(int key, int value) {
  switch (key) {
    case MQ_TUNE_GEMM_FORCE_SMALL:
      mq::g_gemm_force_small = value != 0;
      break;
    case MQ_TUNE_GEMM_PINGPONG:
      mq::g_gemm_pingpong = value != 0;
      break;
    case MQ_TUNE_OPTIM_PCG_ITERS:
      if (value < 1 || value > 128) return fail("mq_set_tuning: PCG iterations must be in [1, 128]", -2);
      mq::g_optim_pcg_iters = value;
      break;
    case MQ_TUNE_OPTIM_PRECOND_LDS:
      mq::g_optim_precond_lds = value != 0;
      break;
    case MQ_TUNE_GEMM_TILE64:
      mq::g_gemm_tile64 = value != 0;
      break;
    case MQ_TUNE_QKV_HEAD_MAJOR:
      g_qkv_head_major = value != 0;
      break;
    case MQ_TUNE_VIT_RESID_F32:
      g_vit_resid_f32 = value != 0;
      break;
    case MQ_TUNE_ATTN_KRING:
      mq::g_attn_kring = value != 0;
      break;
    case MQ_TUNE_OPTIM_STOP:
      if (value < 0 || value > 7) return fail("mq_set_tuning: optim stop rule must be in [0, 7]", -2);
      mq::g_optim_stop = value;
      break;
    case MQ_TUNE_OPTIM_TRF_CHUNK:
      if (value < 1 || value > 64) return fail("mq_set_tuning: lsmr chunk must be in [1, 64]", -2);
      mq::g_optim_trf_chunk = value;
      break;
    case MQ_TUNE_OPTIM_TRF_FB:
      if (value < 1 || value > 4) return fail("mq_set_tuning: frames per workgroup must be in [1, 4]", -2);
      mq::g_optim_trf_fb = value;
      break;
    case MQ_TUNE_GEMM_W4:
      if (value < 0 || value > 2) return fail("mq_set_tuning: GEMM_W4 must be 0, 1 or 2", -2);
      mq::g_gemm_w4 = value;
      break;
    default:
      return fail("mq_set_tuning: unknown key", -2);
  }
  ++g_tuning_gen;
  return 0;
}

int mq_get_tuning(int key) {
  switch (key) {
    case MQ_TUNE_GEMM_FORCE_SMALL: return mq::g_gemm_force_small ? 1 : 0;
    case MQ_TUNE_GEMM_PINGPONG: return mq::g_gemm_pingpong;
    case MQ_TUNE_OPTIM_PCG_ITERS: return mq::g_optim_pcg_iters;
    case MQ_TUNE_OPTIM_PRECOND_LDS: return mq::g_optim_precond_lds;
    case MQ_TUNE_GEMM_TILE64: return mq::g_gemm_tile64;
    case MQ_TUNE_QKV_HEAD_MAJOR: return g_qkv_head_major;
    case MQ_TUNE_VIT_RESID_F32: return g_vit_resid_f32;
    case MQ_TUNE_ATTN_KRING: return mq::g_attn_kring;
    case MQ_TUNE_OPTIM_STOP: return mq::g_optim_stop;
    case MQ_TUNE_OPTIM_TRF_CHUNK: return mq::g_optim_trf_chunk;
    case MQ_TUNE_OPTIM_TRF_FB: return mq::g_optim_trf_fb;
    case MQ_TUNE_GEMM_W4: return mq::g_gemm_w4;
    default: return fail("mq_get_tuning: unknown key", -2);
  }
}

const char* mq_last_error(void) { return g_err.c_str(); }

int mq_create(int device, mq_ctx** out) {
  if (!out) return fail("mq_create: null out");
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail("mq_create: bad device index");
  HIP_TRY(hipSetDevice(device));
  mq_ctx* c = new mq_ctx();
  c->device = device;
  *out = c;
  return 0;
}

int mq_destroy(mq_ctx* ctx) {
  if (!ctx) return 0;
  (void)hipSetDevice(ctx->device);
  ctx->scratch.release();
  ctx->decode_work.release();
  ctx->optim_ws.release();
  ctx->assoc_ws.release();
  ctx->dlt_ws.release();
  ctx->det_ws.release();
  delete ctx;
  return 0;
}

// ----------------------------------------------------------------------------- ViTPose
int mq_vitpose_create(mq_ctx* ctx, int D, int L, int H, int FF, int J, mq_vitpose** out) {
  if (!ctx || !out) return fail("mq_vitpose_create: null argument");
  if (D <= 0 || L <= 0 || H <= 0 || D % H || FF <= 0 || J <= 0 || J > 128) return fail("mq_vitpose_create: bad dims");
  const int dh = D / H;
  if (dh != 64 && dh != 80) return fail("mq_vitpose_create: head dim must be 64 or 80");
  if (D % 64 || FF % 64 || D > 2048) return fail("mq_vitpose_create: dims must be multiples of 64, D <= 2048");
  HIP_TRY(hipSetDevice(ctx->device));
  mq_vitpose* m = new mq_vitpose();
  m->ctx = ctx;
  m->D = D;
  m->L = L;
  m->H = H;
  m->FF = FF;
  m->J = J;
  m->gh = (m->img_h + 2 * m->pad - m->patch) / m->patch + 1;
  m->gw = (m->img_w + 2 * m->pad - m->patch) / m->patch + 1;
  m->T = m->gh * m->gw;
  const int KP = 3 * m->patch * m->patch;
  const int dc = m->dc;
  // arena layout
  std::vector<std::pair<void**, size_t>> plan;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  struct Req {
    std::string name;
    int kind;
    int64_t numel;
    size_t offset;
    int cin, cout;
  };
  std::vector<Req> reqs;
  auto add = [&](const std::string& name, int kind, int64_t numel, size_t elem, int cin = 0, int cout = 0) {
    size_t o = take((size_t)numel * elem);
    reqs.push_back({name, kind, numel, o, cin, cout});
    return o;
  };
  size_t o_wpatch = add("backbone.patch_embed.projection.weight", 0, (int64_t)D * KP, 2);
  size_t o_bpatch = add("backbone.patch_embed.projection.bias", 1, D, 4);
  size_t o_pos = add("backbone.pos_embed", 1, (int64_t)m->T * D, 4);
  struct LOff {
    size_t l1g, l1b, l2g, l2b, wq, wp, w1, w2, bq, bp, b1, b2;
  };
  std::vector<LOff> lo(L);
  for (int i = 0; i < L; ++i) {
    std::string p = "backbone.layers." + std::to_string(i) + ".";
    lo[i].l1g = add(p + "ln1.weight", 1, D, 4);
    lo[i].l1b = add(p + "ln1.bias", 1, D, 4);
    lo[i].wq = add(p + "attn.qkv.weight", 0, (int64_t)3 * D * D, 2);
    lo[i].bq = add(p + "attn.qkv.bias", 1, 3 * D, 4);
    lo[i].wp = add(p + "attn.proj.weight", 0, (int64_t)D * D, 2);
    lo[i].bp = add(p + "attn.proj.bias", 1, D, 4);
    lo[i].l2g = add(p + "ln2.weight", 1, D, 4);
    lo[i].l2b = add(p + "ln2.bias", 1, D, 4);
    lo[i].w1 = add(p + "ffn.layers.0.0.weight", 0, (int64_t)FF * D, 2);
    lo[i].b1 = add(p + "ffn.layers.0.0.bias", 1, FF, 4);
    lo[i].w2 = add(p + "ffn.layers.1.weight", 0, (int64_t)D * FF, 2);
    lo[i].b2 = add(p + "ffn.layers.1.bias", 1, D, 4);
  }
  size_t o_lnfg = add("backbone.ln1.weight", 1, D, 4);
  size_t o_lnfb = add("backbone.ln1.bias", 1, D, 4);
  size_t o_dc1 = add("head.deconv_layers.0.weight", 2, (int64_t)D * dc * 16, 2, D, dc);
  m->dc2_subpixel = dc % 256 == 0;
  size_t o_dc2, o_dc2f = 0, o_shift4 = 0;
  if (m->dc2_subpixel) {
    o_dc2f = add("head.deconv_layers.3.weight", 1, (int64_t)dc * dc * 16, 4);
    o_dc2 = take((size_t)dc * dc * 16 * 2);
    o_shift4 = take((size_t)4 * dc * 4);
  } else {
    o_dc2 = add("head.deconv_layers.3.weight", 2, (int64_t)dc * dc * 16, 2, dc, dc);
  }
  // final 1x1 conv: pad rows to a multiple of 8 is not needed (N masked in the GEMM)
  size_t o_fin = add("head.final_layer.weight", 0, (int64_t)J * dc, 2);
  size_t o_bfin = add("head.final_layer.bias", 1, J, 4);
  const char* bn_names[8] = {"head.deconv_layers.1.weight", "head.deconv_layers.1.bias",
                             "head.deconv_layers.1.running_mean", "head.deconv_layers.1.running_var",
                             "head.deconv_layers.4.weight", "head.deconv_layers.4.bias",
                             "head.deconv_layers.4.running_mean", "head.deconv_layers.4.running_var"};
  size_t o_bn = take(4 * (size_t)dc * 4);
  size_t o_flip = take(128 * 4);
  if (m->weights.ensure(off)) {
    delete m;
    return fail("mq_vitpose_create: hipMalloc of weights failed", -5);
  }
  char* base = m->weights.as<char>();
  for (auto& r : reqs) {
    ParamSlot s;
    s.kind = r.kind;
    s.numel = r.numel;
    s.dst = base + r.offset;
    s.cin = r.cin;
    s.cout = r.cout;
    m->slots[r.name] = s;
  }
  for (int k = 0; k < 8; ++k) {
    ParamSlot s;
    s.kind = 3;
    s.numel = dc;
    s.dst = nullptr;
    s.cin = k;
    s.cout = 0;
    m->slots[bn_names[k]] = s;
  }
  m->w_patch = (unsigned short*)(base + o_wpatch);
  m->b_patch = (float*)(base + o_bpatch);
  m->pos = (float*)(base + o_pos);
  m->layers.resize(L);
  for (int i = 0; i < L; ++i) {
    Layer& ly = m->layers[i];
    ly.ln1_g = (float*)(base + lo[i].l1g);
    ly.ln1_b = (float*)(base + lo[i].l1b);
    ly.ln2_g = (float*)(base + lo[i].l2g);
    ly.ln2_b = (float*)(base + lo[i].l2b);
    ly.wqkv = (unsigned short*)(base + lo[i].wq);
    ly.wproj = (unsigned short*)(base + lo[i].wp);
    ly.wfc1 = (unsigned short*)(base + lo[i].w1);
    ly.wfc2 = (unsigned short*)(base + lo[i].w2);
    ly.bqkv = (float*)(base + lo[i].bq);
    ly.bproj = (float*)(base + lo[i].bp);
    ly.bfc1 = (float*)(base + lo[i].b1);
    ly.bfc2 = (float*)(base + lo[i].b2);
  }
  m->lnf_g = (float*)(base + o_lnfg);
  m->lnf_b = (float*)(base + o_lnfb);
  m->w_dc1 = (unsigned short*)(base + o_dc1);
  m->w_dc2 = (unsigned short*)(base + o_dc2);
  if (m->dc2_subpixel) {
    m->w_dc2_f32 = (float*)(base + o_dc2f);
    m->bn2_shift4 = (float*)(base + o_shift4);
  }
  m->w_fin = (unsigned short*)(base + o_fin);
  m->b_fin = (float*)(base + o_bfin);
  m->bn1_scale = (float*)(base + o_bn);
  m->bn1_shift = m->bn1_scale + dc;
  m->bn2_scale = m->bn1_scale + 2 * dc;
  m->bn2_shift = m->bn1_scale + 3 * dc;
  m->flip_idx = (int32_t*)(base + o_flip);
  // macaque flip pairs (model/pose/macaque.py:15-130); identity beyond 17 joints
  int32_t fi[128];
  const int32_t mac[17] = {0, 2, 1, 4, 3, 6, 5, 8, 7, 10, 9, 12, 11, 14, 13, 16, 15};
  for (int k = 0; k < 128; ++k) fi[k] = (J == 17 && k < 17) ? mac[k] : k;
  HIP_TRY(hipMemcpy(m->flip_idx, fi, sizeof(fi), hipMemcpyHostToDevice));
  *out = m;
  return 0;
}

int mq_vitpose_destroy(mq_vitpose* m) {
  if (!m) return 0;
  (void)hipSetDevice(m->ctx->device);
  if (m->gexec) (void)hipGraphExecDestroy(m->gexec);
  for (hipEvent_t e : m->t_events) (void)hipEventDestroy(e);
  if (m->cap_stream) (void)hipStreamDestroy(m->cap_stream);
  if (m->ev_in) (void)hipEventDestroy(m->ev_in);
  if (m->ev_out) (void)hipEventDestroy(m->ev_out);
  m->weights.release();
  m->ws.release();
  m->stage.release();
  delete m;
  return 0;
}

int mq_vitpose_set_param(mq_vitpose* m, const char* name, const float* data, int64_t numel, int on_device) {
  if (!m || !name || !data) return fail("mq_vitpose_set_param: null argument");
  auto it = m->slots.find(name);
  if (it == m->slots.end()) return fail(std::string("mq_vitpose_set_param: unknown parameter ") + name, -2);
  ParamSlot& s = it->second;
  if (numel != s.numel)
    return fail(std::string("mq_vitpose_set_param: numel mismatch for ") + name + " expected " +
                    std::to_string(s.numel) + " got " + std::to_string(numel),
                -3);
  HIP_TRY(hipSetDevice(m->ctx->device));
  if (s.kind == 3) {
    std::vector<float>& h = m->bn_host[s.cin];
    h.resize(numel);
    if (on_device)
      HIP_TRY(hipMemcpy(h.data(), data, numel * 4, hipMemcpyDeviceToHost));
    else
      std::memcpy(h.data(), data, numel * 4);
    s.loaded = true;
    m->finalized = false;
    return 0;
  }
  const float* src = data;
  void* tmp = nullptr;
  if (!on_device) {
    HIP_TRY(hipMalloc(&tmp, numel * 4));
    HIP_TRY(hipMemcpy(tmp, data, numel * 4, hipMemcpyHostToDevice));
    src = (const float*)tmp;
  }
  int rc = 0;
  if (s.kind == 1) {
    if (hipMemcpy(s.dst, src, numel * 4, hipMemcpyDeviceToDevice) != hipSuccess) rc = -5;
  } else if (s.kind == 0) {
    rc = mq::convert_f32_bf16(src, (unsigned short*)s.dst, numel, nullptr);
  } else if (s.kind == 2) {
    rc = mq::deconv_weight_pack(src, (unsigned short*)s.dst, s.cin, s.cout, nullptr);
  }
  if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -5;
  if (tmp) (void)hipFree(tmp);
  if (rc) return fail(std::string("mq_vitpose_set_param: device copy failed for ") + name, rc);
  s.loaded = true;
  m->finalized = false;
  return 0;
}

int mq_vitpose_finalize(mq_vitpose* m) {
  if (!m) return fail("mq_vitpose_finalize: null model");
  for (auto& kv : m->slots)
    if (!kv.second.loaded) return fail("mq_vitpose_finalize: parameter not loaded: " + kv.first, -2);
  // eval BatchNorm: y = (x - rm) / sqrt(rv + eps) * w + b = x * scale + shift
  std::vector<float> ss(4 * m->dc);
  for (int l = 0; l < 2; ++l) {
    const std::vector<float>* h = &m->bn_host[4 * l];
    for (int c = 0; c < m->dc; ++c) {
      const double sc = (double)h[0][c] / std::sqrt((double)h[3][c] + 1e-5);
      ss[(2 * l) * m->dc + c] = (float)sc;
      ss[(2 * l + 1) * m->dc + c] = (float)((double)h[1][c] - (double)h[2][c] * sc);
    }
  }
  HIP_TRY(hipSetDevice(m->ctx->device));
  HIP_TRY(hipMemcpy(m->bn1_scale, ss.data(), ss.size() * 4, hipMemcpyHostToDevice));
  if (m->dc2_subpixel) {
    std::vector<float> sh4(4 * m->dc);
    for (int c = 0; c < 4; ++c)
      std::memcpy(sh4.data() + c * m->dc, ss.data() + 3 * m->dc, m->dc * sizeof(float));
    HIP_TRY(hipMemcpy(m->bn2_shift4, sh4.data(), sh4.size() * 4, hipMemcpyHostToDevice));
    K_TRY(mq::deconv_subpixel_pack(m->w_dc2_f32, m->bn2_scale, m->w_dc2, m->dc, m->dc, nullptr));
    HIP_TRY(hipDeviceSynchronize());
  }
  m->finalized = true;
  if (m->gexec) {
    (void)hipGraphExecDestroy(m->gexec);
    m->gexec = nullptr;
  }
  return 0;
}

int mq_vitpose_set_graph(mq_vitpose* m, int enable) {
  if (!m) return fail("mq_vitpose_set_graph: null model");
  m->use_graph = enable != 0;
  if (!m->use_graph && m->gexec) {
    (void)hipGraphExecDestroy(m->gexec);
    m->gexec = nullptr;
  }
  return 0;
}

static int ensure_workspace(mq_vitpose* m, int F) {
  if (F <= m->ws_F) return 0;
  const size_t T = m->T, D = m->D, FF = m->FF, dc = m->dc;
  const size_t rows = (size_t)F * T;
  const size_t KP = 3 * m->patch * m->patch;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    size_t o = off;
    off += (bytes + 255) & ~size_t(255);
    return o;
  };
  size_t oA0 = take(rows * KP * 2);
  size_t oX = take(rows * D * 4);
  size_t oH = take(rows * D * 2);
  size_t oQKV = take(rows * 3 * D * 2);
  size_t oO = take(rows * D * 2);
  size_t big = std::max(rows * FF * 2, rows * 16 * dc * 2);  // G and cols1 share
  size_t oG = take(big);
  size_t oY1 = take((size_t)F * 4 * T * dc * 2);
  size_t oC2 = m->dc2_subpixel ? 0 : take((size_t)F * 4 * T * 16 * dc * 2);
  size_t oY2 = take((size_t)F * 16 * T * dc * 2);
  size_t oHM = take((size_t)F * m->J * 16 * T * 4);
  if (m->ws.ensure(off)) return fail("workspace hipMalloc failed", -5);
  char* b = m->ws.as<char>();
  m->A0 = (unsigned short*)(b + oA0);
  m->X = (float*)(b + oX);
  m->Hn = (unsigned short*)(b + oH);
  m->QKV = (unsigned short*)(b + oQKV);
  m->O = (unsigned short*)(b + oO);
  m->G = (unsigned short*)(b + oG);
  m->Y1 = (unsigned short*)(b + oY1);
  m->cols2 = m->dc2_subpixel ? nullptr : (unsigned short*)(b + oC2);
  m->Y2 = (unsigned short*)(b + oY2);
  m->hm_all = (float*)(b + oHM);
  m->ws_F = F;
  if (m->gexec) {
    (void)hipGraphExecDestroy(m->gexec);
    m->gexec = nullptr;
  }
  return 0;
}

// a plain bias GEMM of the forward (proj, fc2, deconv 1): the hand-written kernels only (gemm_pp.hip)
static int gemm_plain(const mq::GemmArgs& g, hipStream_t s) { return mq::gemm_bf16(g, mq::EPI_BF16, s); }

static int launch_forward(mq_vitpose* m, const float* crops, int n, int flip, float* heatmaps, hipStream_t s) {
  const int F = flip ? 2 * n : n;
  const int T = m->T, D = m->D, FF = m->FF, dc = m->dc;
  const int rows = F * T;
  const int KP = 3 * m->patch * m->patch;
  m->g_rows_timed = rows;
  K_TRY(mq::patch_im2col(crops, m->A0, n, flip ? 2 : 1, m->img_h, m->img_w, m->patch, m->pad, s));
  mq::GemmArgs g{};
  g = mq::GemmArgs{m->A0, m->w_patch, m->X, m->b_patch, m->pos, rows, D, KP, KP, KP, D, T};
  K_TRY(mq::gemm_bf16(g, mq::EPI_POS_F32, s));
  // Residual updates: proj and fc2 write their branch outputs (bias included) as bf16 into P1 / P2, and the
  // LayerNorm passes add them to the f32 residual stream X: LN2 normalises x + p1 without storing it, the
  // next block's LN1 adds p1 then p2 (the same order as two separate updates), stores X and normalises.
  // The f32 read-modify-write of X in the GEMM epilogue, which every CU ran at once at the end of proj's /
  // fc2's single tile round, is gone.  P1 / P2 live in the QKV buffer: the attention has read QKV before
  // proj writes P1, and the next qkv GEMM runs after the LayerNorm that consumed both.
  unsigned short* P1 = m->QKV;
  unsigned short* P2 = m->QKV + (size_t)rows * D;
  // MQ_TUNE_VIT_RESID_F32 (precision A/B): proj / fc2 add their f32 accumulators to X in the epilogue instead
  const bool rf32 = g_vit_resid_f32 != 0;
  for (int l = 0; l < m->L; ++l) {
    const Layer& ly = m->layers[l];
    if (l == 0 || rf32)
      K_TRY(mq::layernorm_f32_bf16(m->X, ly.ln1_g, ly.ln1_b, m->Hn, rows, D, 1e-6f, s));
    else
      K_TRY(mq::add_layernorm_f32_bf16(m->X, P1, P2, true, ly.ln1_g, ly.ln1_b, m->Hn, rows, D, 1e-6f, s));
    // qkv written head-major (each head's Q / K / V rows contiguous) for the attention's loads
    g = mq::GemmArgs{m->Hn, ly.wqkv, m->QKV, ly.bqkv, nullptr, rows, 3 * D, D, D, D, 3 * D, 0};
    g.head_dim = g_qkv_head_major ? D / m->H : 0;
    K_TRY(mq::gemm_bf16(g, mq::EPI_BF16, s));
    K_TRY(mq::attention_bf16(m->QKV, m->O, F, T, D, m->H, s, g_qkv_head_major != 0));
    if (rf32) {
      g = mq::GemmArgs{m->O, ly.wproj, m->X, ly.bproj, nullptr, rows, D, D, D, D, D, 0};
      K_TRY(mq::gemm_bf16(g, mq::EPI_RESID_F32, s));
      K_TRY(mq::layernorm_f32_bf16(m->X, ly.ln2_g, ly.ln2_b, m->Hn, rows, D, 1e-6f, s));
    } else {
      g = mq::GemmArgs{m->O, ly.wproj, P1, ly.bproj, nullptr, rows, D, D, D, D, D, 0};
      K_TRY(gemm_plain(g, s));
      K_TRY(mq::add_layernorm_f32_bf16(m->X, P1, nullptr, false, ly.ln2_g, ly.ln2_b, m->Hn, rows, D, 1e-6f, s));
    }
    g = mq::GemmArgs{m->Hn, ly.wfc1, m->G, ly.bfc1, nullptr, rows, FF, D, D, D, FF, 0};
    hipEvent_t e0 = nullptr, e1 = nullptr;
    // live timing of fc1 on every 8th layer (4 launches per ViT-H forward): an event pair still leaves ~4 us of
    // idle GPU on each side of the launch it brackets (0.28 ms per step when all 32 were timed)
    const bool timed = m->timing && ((l & 7) == 7 || (m->L < 8 && l == m->L - 1));
    if (timed) {
      while (m->t_events.size() < m->t_used + 2) {
        // timing only: without the system-scope fence a recorded event writes back and invalidates no cache,
        // which otherwise left a ~6 us gap on each side of every timed launch and started fc1 on cold caches
        hipEvent_t e;
        HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
        m->t_events.push_back(e);
      }
      e0 = m->t_events[m->t_used];
      e1 = m->t_events[m->t_used + 1];
      m->t_used += 2;
      HIP_TRY(hipEventRecord(e0, s));
    }
    K_TRY(mq::gemm_bf16(g, mq::EPI_GELU_BF16, s));
    if (timed) HIP_TRY(hipEventRecord(e1, s));
    g = mq::GemmArgs{m->G, ly.wfc2, rf32 ? (void*)m->X : (void*)P2, ly.bfc2, nullptr, rows, D, FF, FF, FF, D, 0};
    if (rf32)
      K_TRY(mq::gemm_bf16(g, mq::EPI_RESID_F32, s));
    else
      K_TRY(gemm_plain(g, s));
  }
  if (m->L > 0 && !rf32)
    K_TRY(mq::add_layernorm_f32_bf16(m->X, P1, P2, false, m->lnf_g, m->lnf_b, m->Hn, rows, D, 1e-6f, s));
  else
    K_TRY(mq::layernorm_f32_bf16(m->X, m->lnf_g, m->lnf_b, m->Hn, rows, D, 1e-6f, s));
  // head: deconv1 (GEMM + col2im + BN + ReLU)
  unsigned short* cols1 = m->G;
  g = mq::GemmArgs{m->Hn, m->w_dc1, cols1, nullptr, nullptr, rows, 16 * dc, D, D, D, 16 * dc, 0};
  K_TRY(gemm_plain(g, s));
  K_TRY(mq::deconv_col2im_bn_relu(cols1, m->bn1_scale, m->bn1_shift, m->Y1, F, m->gh, m->gw, dc, s));
  const int rows2 = F * 4 * T;
  if (m->dc2_subpixel) {
    // deconv2 + BN + ReLU: four sub-pixel 2x2 convolutions in one implicit GEMM, straight into Y2
    g = mq::GemmArgs{m->Y1, m->w_dc2, m->Y2, m->bn2_shift4, nullptr, rows2, 4 * dc, 4 * dc, dc, 4 * dc, dc, 0};
    g.conv_h = 2 * m->gh;
    g.conv_w = 2 * m->gw;
    g.conv_c = dc;
    K_TRY(mq::deconv_subpixel_bf16(g, mq::EPI_RELU_BF16, s));
  } else {
    g = mq::GemmArgs{m->Y1, m->w_dc2, m->cols2, nullptr, nullptr, rows2, 16 * dc, dc, dc, dc, 16 * dc, 0};
    K_TRY(mq::gemm_bf16(g, mq::EPI_BF16, s));
    K_TRY(mq::deconv_col2im_bn_relu(m->cols2, m->bn2_scale, m->bn2_shift, m->Y2, F, 2 * m->gh, 2 * m->gw, dc, s));
  }
  const int rows3 = F * 16 * T;
  float* hm_dst = flip ? m->hm_all : heatmaps;
  g = mq::GemmArgs{m->Y2, m->w_fin, hm_dst, m->b_fin, nullptr, rows3, m->J, dc, dc, dc, m->J, 16 * T};
  K_TRY(mq::gemm_bf16(g, mq::EPI_NCHW_F32, s));
  if (flip) K_TRY(mq::flip_average(m->hm_all, heatmaps, n, m->J, 4 * m->gh, 4 * m->gw, m->flip_idx, s));
  return 0;
}

int mq_vitpose_forward(mq_vitpose* m, const float* crops, int n, int flip_test, float* heatmaps, void* stream) {
  if (!m || !crops || !heatmaps) return fail("mq_vitpose_forward: null argument");
  if (!m->finalized) return fail("mq_vitpose_forward: model not finalized", -2);
  if (n <= 0) return 0;
  HIP_TRY(hipSetDevice(m->ctx->device));
  hipStream_t s = (hipStream_t)stream;
  const int F = flip_test ? 2 * n : n;
  int rc = ensure_workspace(m, F);
  if (rc) return rc;
  if (!m->use_graph || m->timing) return launch_forward(m, crops, n, flip_test, heatmaps, s);
  if (!m->cap_stream) {
    HIP_TRY(hipStreamCreateWithFlags(&m->cap_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_out, hipEventDisableTiming));
  }
  hipStream_t cs = m->cap_stream;
  if (!m->gexec || m->g_n != n || m->g_flip != flip_test || m->g_in != crops || m->g_out != heatmaps ||
      m->g_gen != g_tuning_gen) {
    if (m->gexec) {
      (void)hipGraphExecDestroy(m->gexec);
      m->gexec = nullptr;
    }
    HIP_TRY(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
    rc = launch_forward(m, crops, n, flip_test, heatmaps, cs);
    hipGraph_t graph = nullptr;
    hipError_t e = hipStreamEndCapture(cs, &graph);
    if (rc) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    if (e != hipSuccess) return fail(std::string("hipStreamEndCapture: ") + hipGetErrorString(e), -5);
    e = hipGraphInstantiate(&m->gexec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return fail(std::string("hipGraphInstantiate: ") + hipGetErrorString(e), -5);
    m->g_n = n;
    m->g_flip = flip_test;
    m->g_gen = g_tuning_gen;
    m->g_in = crops;
    m->g_out = heatmaps;
  }
  HIP_TRY(hipEventRecord(m->ev_in, s));
  HIP_TRY(hipStreamWaitEvent(cs, m->ev_in, 0));
  HIP_TRY(hipGraphLaunch(m->gexec, cs));
  HIP_TRY(hipEventRecord(m->ev_out, cs));
  HIP_TRY(hipStreamWaitEvent(s, m->ev_out, 0));
  return 0;
}

int mq_vitpose_timing(mq_vitpose* m, int enable) {
  if (!m) return fail("mq_vitpose_timing: null model");
  m->timing = enable != 0;
  if (m->timing) m->t_used = 0;
  return 0;
}

int mq_vitpose_timing_result(mq_vitpose* m, double* avg_ms, int* count, int64_t* flops_per_launch) {
  if (!m || !avg_ms || !count) return fail("mq_vitpose_timing_result: null argument");
  double tot = 0.0;
  int cnt = 0;
  for (size_t i = 0; i + 1 < m->t_used; i += 2) {
    HIP_TRY(hipEventSynchronize(m->t_events[i + 1]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, m->t_events[i], m->t_events[i + 1]));
    tot += ms;
    ++cnt;
  }
  *avg_ms = cnt ? tot / cnt : 0.0;
  *count = cnt;
  if (flops_per_launch) *flops_per_launch = (int64_t)2 * (int64_t)(m->g_rows_timed) * m->FF * m->D;
  return 0;
}

int mq_crop_udp(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int height, int width, const float* boxes,
                const int32_t* box_frame, int n, float* crops, float* center, float* scale, void* stream) {
  if (!ctx) return fail("mq_crop_udp: null ctx");
  if (n < 0 || height <= 0 || width <= 0) return fail("mq_crop_udp: bad sizes");
  if (n == 0) return 0;
  if (!frames || !boxes || !box_frame || !crops || !center || !scale) return fail("mq_crop_udp: null buffer");
  HIP_TRY(hipSetDevice(ctx->device));
  K_TRY(mq::crop_udp(frames, frame_stride, height, width, boxes, box_frame, n, crops, center, scale,
                     (hipStream_t)stream));
  return 0;
}

int mq_decode_udp(mq_ctx* ctx, const float* heatmaps, int n, int J, int hm_h, int hm_w, const float* center,
                  const float* scale, double* kp_img, float* score, int32_t* argmax, float* kp_hm, void* stream) {
  if (!ctx) return fail("mq_decode_udp: null ctx");
  if (n < 0 || J <= 0 || hm_h <= 0 || hm_w <= 0) return fail("mq_decode_udp: bad sizes");
  if (n == 0) return 0;
  if (!heatmaps || !center || !scale || !kp_img || !score || !argmax) return fail("mq_decode_udp: null buffer");
  if ((size_t)(hm_h * hm_w + (hm_h + 10) * hm_w) * 4 > 64 * 1024) return fail("mq_decode_udp: heatmap too large");
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->decode_work.ensure((size_t)n * J * hm_h * hm_w * 4)) return fail("decode workspace alloc failed", -5);
  K_TRY(mq::udp_decode(heatmaps, n, J, hm_h, hm_w, center, scale, 192, 256, ctx->decode_work.as<float>(), kp_img,
                       score, argmax, kp_hm, (hipStream_t)stream));
  return 0;
}

int mq_topdown(mq_vitpose* m, const uint8_t* frames, int64_t frame_stride, int height, int width, const float* boxes,
               const int32_t* box_frame, int n, int flip_test, double* kp_img, float* score, int32_t* argmax,
               float* heatmaps, void* stream) {
  if (!m) return fail("mq_topdown: null model");
  if (n <= 0) return 0;
  HIP_TRY(hipSetDevice(m->ctx->device));
  // staging owned by the model (its device): crops, center/scale, heatmaps (if caller passes none).
  // Calls on one model are stream-ordered: the staging is reused by the next call on the model.
  const size_t crop_b = (size_t)n * 3 * m->img_h * m->img_w * 4;
  const size_t cs_b = (size_t)n * 4 * 4;
  const size_t hm_b = (size_t)n * m->J * 16 * m->T * 4;
  if (m->stage.ensure(crop_b + cs_b + hm_b + 1024)) return fail("mq_topdown: scratch alloc failed", -5);
  char* b = m->stage.as<char>();
  float* crops = (float*)b;
  float* center = (float*)(b + crop_b);
  float* scale = center + 2 * n;
  float* hm = heatmaps ? heatmaps : (float*)(b + crop_b + cs_b);
  int rc = mq_crop_udp(m->ctx, frames, frame_stride, height, width, boxes, box_frame, n, crops, center, scale, stream);
  if (rc) return rc;
  rc = mq_vitpose_forward(m, crops, n, flip_test, hm, stream);
  if (rc) return rc;
  return mq_decode_udp(m->ctx, hm, n, m->J, 4 * m->gh, 4 * m->gw, center, scale, kp_img, score, argmax, nullptr,
                       stream);
}

// ----------------------------------------------------------------------------- building blocks
int mq_gemm_bf16(mq_ctx* ctx, const void* A, const void* W, void* C, const float* bias, const float* aux, int M,
                 int N, int K, int lda, int ldw, int ldc, int aux_rows, int epilogue, void* stream) {
  if (!ctx || !A || !W || !C) return fail("mq_gemm_bf16: null argument");
  if (M <= 0 || N <= 0 || K <= 0) return fail("mq_gemm_bf16: bad sizes", -2);
  if (epilogue < 0 || epilogue > 6) return fail("mq_gemm_bf16: bad epilogue", -2);
  if ((epilogue == mq::EPI_POS_F32 || epilogue == mq::EPI_NCHW_F32) && (!aux_rows || (!aux && epilogue == 3)))
    return fail("mq_gemm_bf16: epilogue needs aux", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  mq::GemmArgs g{(const unsigned short*)A, (const unsigned short*)W, C, bias, aux, M, N, K, lda, ldw, ldc, aux_rows};
  int rc = mq::gemm_bf16(g, epilogue, (hipStream_t)stream);
  if (rc) return fail("mq_gemm_bf16: launch failed / unsupported shape (K % 32, lda/ldw % 8)", -6);
  return 0;
}

int mq_gemm_resid_relu_bf16(mq_ctx* ctx, const void* A, const void* W, float* C, const float* bias, uint16_t* out,
                            int M, int N, int K, int lda, int ldw, int ldc, void* stream) {
  if (!ctx || !A || !W || !C || !out) return fail("mq_gemm_resid_relu_bf16: null argument");
  if (M <= 0 || N <= 0 || K <= 0 || K % 64) return fail("mq_gemm_resid_relu_bf16: bad sizes (K % 64 == 0)", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  mq::GemmArgs g{(const unsigned short*)A, (const unsigned short*)W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0};
  g.C2 = out;
  if (mq::gemm_bf16(g, mq::EPI_RESID_RELU, (hipStream_t)stream))
    return fail("mq_gemm_resid_relu_bf16: launch failed / unsupported shape", -6);
  return 0;
}

int mq_id_conv_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch, int k, int stride,
                    int pad, const uint16_t* w, const float* bias, void* out, int cout, int epilogue, void* stream) {
  if (!ctx || !x || !w || !out) return fail("mq_id_conv_bf16: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || ch <= 0 || ch % 64 || k <= 0 || stride <= 0 || pad < 0 || cout <= 0 ||
      cout % 8)
    return fail("mq_id_conv_bf16: bad sizes (ch % 64 == 0, cout % 8 == 0)", -2);
  if (epilogue != mq::EPI_BF16 && epilogue != mq::EPI_F32 && epilogue != mq::EPI_RELU_BF16)
    return fail("mq_id_conv_bf16: epilogue must be 0 (bf16), 4 (f32) or 6 (ReLU bf16)", -2);
  const int oh = (height + 2 * pad - k) / stride + 1, ow = (width + 2 * pad - k) / stride + 1;
  if (oh <= 0 || ow <= 0) return fail("mq_id_conv_bf16: empty output", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  mq::GemmArgs g{(const unsigned short*)x, (const unsigned short*)w, out, bias, nullptr, n_img * oh * ow, cout,
                 k * k * ch, ch, k * k * ch, cout, 0};
  g.conv_h = height;
  g.conv_w = width;
  g.conv_c = ch;
  g.conv_k = k;
  g.conv_s = stride;
  g.conv_p = pad;
  if (mq::conv_small_bf16(g, epilogue, (hipStream_t)stream)) return fail("mq_id_conv_bf16: launch failed", -6);
  return 0;
}

int mq_conv3x3_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch, const uint16_t* w,
                    const float* bias, void* out, int cout, int ldc, int epilogue, void* stream) {
  if (!ctx || !x || !w || !out) return fail("mq_conv3x3_bf16: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || cout <= 0 || ch <= 0 || ch % 64 || ldc < cout)
    return fail("mq_conv3x3_bf16: bad sizes (ch must be a multiple of 64)", -2);
  if (epilogue != mq::EPI_BF16 && epilogue != mq::EPI_F32 && epilogue != mq::EPI_RELU_BF16)
    return fail("mq_conv3x3_bf16: epilogue must be 0 (bf16), 4 (f32) or 6 (ReLU bf16)", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  mq::GemmArgs g{(const unsigned short*)x, (const unsigned short*)w, out, bias, nullptr, n_img * height * width, cout,
                 9 * ch, ch, 9 * ch, ldc, 0};
  g.conv_h = height;
  g.conv_w = width;
  g.conv_c = ch;
  if (mq::conv3x3_bf16(g, epilogue, (hipStream_t)stream)) return fail("mq_conv3x3_bf16: launch failed", -6);
  return 0;
}

int mq_deconv_subpixel_pack(mq_ctx* ctx, const float* w, const float* scale, uint16_t* w_packed, int ch, int cout,
                            void* stream) {
  if (!ctx || !w || !w_packed) return fail("mq_deconv_subpixel_pack: null argument");
  if (ch <= 0 || cout <= 0) return fail("mq_deconv_subpixel_pack: bad sizes", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  K_TRY(mq::deconv_subpixel_pack(w, scale, w_packed, ch, cout, (hipStream_t)stream));
  return 0;
}

int mq_deconv_subpixel_bf16(mq_ctx* ctx, const uint16_t* x, int n_img, int height, int width, int ch,
                            const uint16_t* w_packed, const float* shift4, uint16_t* out, int cout, int relu,
                            void* stream) {
  if (!ctx || !x || !w_packed || !out) return fail("mq_deconv_subpixel_bf16: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || ch <= 0 || ch % 64 || cout <= 0 || cout % 256)
    return fail("mq_deconv_subpixel_bf16: bad sizes (ch % 64 == 0, cout % 256 == 0)", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  mq::GemmArgs g{(const unsigned short*)x, (const unsigned short*)w_packed, out, shift4, nullptr,
                 n_img * height * width, 4 * cout, 4 * ch, ch, 4 * ch, cout, 0};
  g.conv_h = height;
  g.conv_w = width;
  g.conv_c = ch;
  if (mq::deconv_subpixel_bf16(g, relu ? mq::EPI_RELU_BF16 : mq::EPI_BF16, (hipStream_t)stream))
    return fail("mq_deconv_subpixel_bf16: launch failed", -6);
  return 0;
}

int mq_f32_to_bf16(mq_ctx* ctx, const float* src, uint16_t* dst, int64_t count, void* stream) {
  if (!ctx || !src || !dst || count < 0) return fail("mq_f32_to_bf16: bad argument");
  HIP_TRY(hipSetDevice(ctx->device));
  K_TRY(mq::convert_f32_bf16(src, dst, count, (hipStream_t)stream));
  return 0;
}

// ----------------------------------------------------------------------------- detector
static int check_det(mq_ctx* ctx) {
  if (!ctx) return fail("null ctx");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail("hipSetDevice failed", -5);
  return 0;
}

int mq_det_resize_patch(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int n_img, int height, int width,
                        int new_h, int new_w, int pad_h, int pad_w, const int32_t* xofs, const int32_t* xalpha,
                        const int32_t* yofs, const int32_t* yalpha, uint16_t* patches, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!frames || !xofs || !xalpha || !yofs || !yalpha || !patches) return fail("mq_det_resize_patch: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || new_h <= 0 || new_w <= 0 || pad_h < new_h || pad_w < new_w ||
      pad_h % 4 || pad_w % 4)
    return fail("mq_det_resize_patch: bad sizes (padded size must cover the resize and be a multiple of 4)", -2);
  K_TRY(mq::det_resize_patch(frames, frame_stride, n_img, height, width, new_h, new_w, pad_h, pad_w, xofs, xalpha, yofs,
                             yalpha, patches, (hipStream_t)stream));
  return 0;
}

int mq_layernorm(mq_ctx* ctx, const float* x, const float* gamma, const float* beta, void* y, int rows, int dim,
                 float eps, int out_f32, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !gamma || !beta || !y) return fail("mq_layernorm: null argument");
  if (rows < 0 || dim <= 0 || dim % 4 || dim > 3072) return fail("mq_layernorm: dim must be a multiple of 4, <= 3072", -2);
  if (rows == 0) return 0;
  if (out_f32)
    K_TRY(mq::layernorm_f32_f32(x, gamma, beta, (float*)y, rows, dim, eps, (hipStream_t)stream));
  else
    K_TRY(mq::layernorm_f32_bf16(x, gamma, beta, (unsigned short*)y, rows, dim, eps, (hipStream_t)stream));
  return 0;
}

int mq_add_layernorm(mq_ctx* ctx, float* x, const uint16_t* p1, const uint16_t* p2, int store_x, const float* gamma,
                     const float* beta, uint16_t* y, int rows, int dim, float eps, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !p1 || !gamma || !beta || !y) return fail("mq_add_layernorm: null argument");
  if (rows < 0 || dim <= 0 || dim % 4 || dim > 3072)
    return fail("mq_add_layernorm: dim must be a multiple of 4, <= 3072", -2);
  if (rows == 0) return 0;
  K_TRY(mq::add_layernorm_f32_bf16(x, p1, p2, store_x != 0, gamma, beta, y, rows, dim, eps, (hipStream_t)stream));
  return 0;
}

int mq_window_attention(mq_ctx* ctx, const uint16_t* qkv, const float* qkv_bias, const float* rel_table, uint16_t* out,
                        int n_img, int height, int width, int dim, int heads, int shift, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!qkv || !qkv_bias || !rel_table || !out) return fail("mq_window_attention: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || heads <= 0 || dim != heads * 32)
    return fail("mq_window_attention: head_dim must be 32 (dim = 32 * heads)", -2);
  if (shift < 0 || shift >= 7) return fail("mq_window_attention: shift must be in [0, 7)", -2);
  K_TRY(mq::window_attention(qkv, qkv_bias, rel_table, out, n_img, height, width, dim, heads, shift,
                             (hipStream_t)stream));
  return 0;
}

int mq_patch_merge_gather(mq_ctx* ctx, const float* x, int n_img, int height, int width, int dim, float* out,
                          void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !out) return fail("mq_patch_merge_gather: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || dim <= 0) return fail("mq_patch_merge_gather: bad sizes", -2);
  K_TRY(mq::merge_gather(x, n_img, height, width, dim, out, (hipStream_t)stream));
  return 0;
}

int mq_upsample_add(mq_ctx* ctx, float* lo, const float* hi, int n_img, int lo_h, int lo_w, int hi_h, int hi_w, int ch,
                    void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!lo || !hi) return fail("mq_upsample_add: null argument");
  if (n_img <= 0 || lo_h <= 0 || lo_w <= 0 || hi_h <= 0 || hi_w <= 0 || ch <= 0) return fail("mq_upsample_add: bad sizes", -2);
  K_TRY(mq::upsample_add(lo, hi, n_img, lo_h, lo_w, hi_h, hi_w, ch, (hipStream_t)stream));
  return 0;
}

int mq_im2col3x3(mq_ctx* ctx, const float* x, int n_img, int height, int width, int ch, uint16_t* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !out) return fail("mq_im2col3x3: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || ch <= 0 || ch % 4) return fail("mq_im2col3x3: bad sizes", -2);
  K_TRY(mq::im2col3x3(x, n_img, height, width, ch, out, (hipStream_t)stream));
  return 0;
}

int mq_subsample2(mq_ctx* ctx, const float* x, int n_img, int height, int width, int ch, float* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !out) return fail("mq_subsample2: null argument");
  if (n_img <= 0 || height <= 0 || width <= 0 || ch <= 0) return fail("mq_subsample2: bad sizes", -2);
  K_TRY(mq::subsample2(x, n_img, height, width, ch, out, (hipStream_t)stream));
  return 0;
}

int mq_id_crop_resize(mq_ctx* ctx, const uint8_t* frames, int64_t frame_stride, int height, int width,
                      const int32_t* boxes, int n, int out_size, uint8_t* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!frames || !boxes || !out) return fail("mq_id_crop_resize: null argument");
  if (n <= 0 || height <= 0 || width <= 0 || out_size <= 0 || frame_stride < (int64_t)height * width * 3)
    return fail("mq_id_crop_resize: bad sizes", -2);
  K_TRY(mq::id_crop_resize(frames, frame_stride, width, boxes, n, out_size, out, (hipStream_t)stream));
  return 0;
}

int mq_id_preprocess(mq_ctx* ctx, const uint8_t* in, int n, int in_size, int edge, int crop, uint16_t* out,
                     void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!in || !out) return fail("mq_id_preprocess: null argument");
  if (n <= 0 || in_size <= 0 || edge <= 0 || crop <= 0 || crop > edge) return fail("mq_id_preprocess: bad sizes", -2);
  // mmpretrain CenterCrop: y1 = max(0, int(round((h - crop) / 2.)))  (Python round: half to even)
  const double half = (edge - crop) / 2.0;
  const int off = std::max(0, (int)std::nearbyint(half));
  K_TRY(mq::id_edge_crop(in, n, in_size, edge, crop, off, out, (hipStream_t)stream));
  return 0;
}

int mq_id_im2col(mq_ctx* ctx, const uint16_t* x, int n, int h, int w, int c, int kh, int kw, int stride, int pad,
                 int kpad, uint16_t* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !out) return fail("mq_id_im2col: null argument");
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0 || kpad < kh * kw * c ||
      h + 2 * pad < kh || w + 2 * pad < kw)
    return fail("mq_id_im2col: bad sizes", -2);
  K_TRY(mq::im2col_bf16(x, n, h, w, c, kh, kw, stride, pad, kpad, out, (hipStream_t)stream));
  return 0;
}

int mq_id_maxpool(mq_ctx* ctx, const uint16_t* x, int n, int h, int w, int c, uint16_t* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !out) return fail("mq_id_maxpool: null argument");
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0) return fail("mq_id_maxpool: bad sizes", -2);
  K_TRY(mq::maxpool3s2(x, n, h, w, c, out, (hipStream_t)stream));
  return 0;
}

int mq_id_relu_bf16(mq_ctx* ctx, float* x, uint16_t* y, int64_t count, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !y) return fail("mq_id_relu_bf16: null argument");
  if (count <= 0 || count % 4) return fail("mq_id_relu_bf16: count % 4 != 0", -2);
  K_TRY(mq::relu_bf16(x, y, count, (hipStream_t)stream));
  return 0;
}

int mq_id_head(mq_ctx* ctx, const float* x, int n, int hw, int c, const float* fc_w, const float* fc_b, int ncls,
               float* logits, float* probs, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!x || !fc_w || !fc_b || !logits || !probs) return fail("mq_id_head: null argument");
  if (n <= 0 || hw <= 0 || c <= 0 || c > 8192 || ncls <= 0 || ncls > mq::ID_MAX_CLASSES)
    return fail("mq_id_head: bad sizes (c <= 8192, ncls <= 16)", -2);
  K_TRY(mq::gap_fc_softmax(x, n, hw, c, fc_w, fc_b, ncls, logits, probs, (hipStream_t)stream));
  return 0;
}

int mq_nms(mq_ctx* ctx, const float* boxes, const float* scores, const uint8_t* valid, const int8_t* level, int n_img,
           int n_cand, float iou_thr, int max_keep, int32_t* keep, int32_t* n_keep, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!boxes || !scores || !valid || !keep || !n_keep) return fail("mq_nms: null argument");
  if (n_img <= 0 || n_cand <= 0 || n_cand > 8192 || max_keep <= 0) return fail("mq_nms: 1 <= n_cand <= 8192", -2);
  if (ctx->det_ws.ensure(mq::nms_workspace_bytes(n_img, n_cand))) return fail("nms workspace alloc failed", -5);
  K_TRY(mq::nms_batched(boxes, scores, valid, level, n_img, n_cand, iou_thr, max_keep, ctx->det_ws.p, keep, n_keep,
                        (hipStream_t)stream));
  return 0;
}

int mq_rpn_proposals(mq_ctx* ctx, const float* head, int n_img, int n_levels, const int32_t* level_hw,
                     const int32_t* strides, const float* base_anchors, int nms_pre, float img_h, float img_w,
                     float iou_thr, int max_keep, float* proposals, float* scores, int32_t* counts, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!head || !level_hw || !strides || !base_anchors || !proposals || !counts)
    return fail("mq_rpn_proposals: null argument");
  if (n_img <= 0 || n_levels <= 0 || n_levels > 6 || nms_pre <= 0 || max_keep <= 0 || n_img * n_levels > 1024)
    return fail("mq_rpn_proposals: bad sizes", -2);
  mq::DetLevels lv{};
  lv.n = n_levels;
  int rows = 0, cand = 0;
  for (int l = 0; l < n_levels; ++l) {
    lv.h[l] = level_hw[2 * l];
    lv.w[l] = level_hw[2 * l + 1];
    lv.stride[l] = strides[l];
    if (lv.h[l] <= 0 || lv.w[l] <= 0 || lv.stride[l] <= 0) return fail("mq_rpn_proposals: bad level size", -2);
    lv.row_off[l] = rows;
    lv.cand_off[l] = cand;
    rows += lv.h[l] * lv.w[l];
    cand += std::min(lv.h[l] * lv.w[l] * 3, nms_pre);
    for (int a = 0; a < 3; ++a)
      for (int k = 0; k < 4; ++k) lv.base[l][a][k] = base_anchors[(l * 3 + a) * 4 + k];
  }
  lv.cand_total = cand;
  if (cand > 8192) return fail("mq_rpn_proposals: more than 8192 candidates per image", -2);
  int32_t* keep_buf = nullptr;
  const size_t keep_bytes = ((size_t)n_img * max_keep * 4 + 255) & ~(size_t)255;
  const size_t need = mq::rpn_workspace_bytes(n_img, rows, cand, n_levels) + keep_bytes;
  if (ctx->det_ws.ensure(need)) return fail("rpn workspace alloc failed", -5);
  keep_buf = reinterpret_cast<int32_t*>(ctx->det_ws.as<char>() + (need - keep_bytes));
  K_TRY(mq::rpn_proposals(head, lv, n_img, rows, img_h, img_w, iou_thr, max_keep, ctx->det_ws.p, need - keep_bytes,
                          proposals, scores, counts, keep_buf, (hipStream_t)stream));
  return 0;
}

int mq_roi_align(mq_ctx* ctx, const float* p2, const float* p3, const float* p4, const float* p5,
                 const int32_t* level_hw, const int32_t* strides, const float* rois, const int32_t* counts, int n_img,
                 int max_rois, uint16_t* out, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!p2 || !p3 || !p4 || !p5 || !level_hw || !strides || !rois || !counts || !out)
    return fail("mq_roi_align: null argument");
  if (n_img <= 0 || max_rois <= 0) return fail("mq_roi_align: bad sizes", -2);
  mq::DetFeats fs{};
  const float* ps[4] = {p2, p3, p4, p5};
  for (int l = 0; l < 4; ++l) {
    fs.p[l] = ps[l];
    fs.h[l] = level_hw[2 * l];
    fs.w[l] = level_hw[2 * l + 1];
    fs.stride[l] = strides[l];
    if (fs.h[l] <= 0 || fs.w[l] <= 0 || fs.stride[l] <= 0) return fail("mq_roi_align: bad level size", -2);
  }
  K_TRY(mq::roi_align(fs, rois, counts, n_img, max_rois, out, (hipStream_t)stream));
  return 0;
}

int mq_rcnn_post(mq_ctx* ctx, const float* rois, const float* head, const int32_t* counts, int n_img, int max_rois,
                 float img_h, float img_w, float inv_scale_w, float inv_scale_h, float score_thr, float iou_thr,
                 int max_det, float* det_boxes, float* det_scores, int32_t* det_counts, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!rois || !head || !counts || !det_boxes || !det_scores || !det_counts) return fail("mq_rcnn_post: null argument");
  if (n_img <= 0 || max_rois <= 0 || max_rois > 8192 || max_det <= 0) return fail("mq_rcnn_post: bad sizes", -2);
  const size_t keep_bytes = ((size_t)n_img * max_det * 4 + 255) & ~(size_t)255;
  const size_t need = mq::rcnn_workspace_bytes(n_img, max_rois) + keep_bytes;
  if (ctx->det_ws.ensure(need)) return fail("rcnn workspace alloc failed", -5);
  int32_t* keep_buf = reinterpret_cast<int32_t*>(ctx->det_ws.as<char>() + (need - keep_bytes));
  K_TRY(mq::rcnn_post(rois, head, counts, n_img, max_rois, img_h, img_w, inv_scale_w, inv_scale_h, score_thr, iou_thr,
                      max_det, ctx->det_ws.p, det_boxes, det_scores, det_counts, keep_buf, (hipStream_t)stream));
  return 0;
}

int mq_det_topk_boxes(mq_ctx* ctx, const float* det_boxes, const float* det_scores, const int32_t* det_counts,
                      int n_img, int max_det, int k, float score_thr, double min_margin, double max_margin,
                      double desired_ar, float* boxes, float* tight, int32_t* img_of, int32_t* valid, void* stream) {
  if (int rc = check_det(ctx)) return rc;
  if (!det_boxes || !det_scores || !det_counts || !boxes || !tight || !img_of || !valid)
    return fail("mq_det_topk_boxes: null argument");
  if (n_img <= 0 || max_det <= 0 || k <= 0 || k > max_det) return fail("mq_det_topk_boxes: bad sizes", -2);
  if (!(desired_ar > 0) || !(max_margin >= min_margin)) return fail("mq_det_topk_boxes: bad margins", -2);
  K_TRY(mq::det_topk_boxes(det_boxes, det_scores, det_counts, n_img, max_det, k, score_thr, min_margin, max_margin,
                           desired_ar, boxes, tight, img_of, valid, (hipStream_t)stream));
  return 0;
}

// ----------------------------------------------------------------------------- geometry
static int check_geo(mq_ctx* ctx, const void* cams, int C, int n) {
  if (!ctx) return fail("null ctx");
  if (!cams) return fail("null cams");
  if (C <= 0 || C > 16) return fail("n_cams must be in [1, 16]", -2);
  if (n < 0) return fail("negative n", -2);
  if (hipSetDevice(ctx->device) != hipSuccess) return fail("hipSetDevice failed", -5);
  return 0;
}

int mq_omnidir_undistort(mq_ctx* ctx, const double* cams, int C, const double* pts, int n, double* out,
                         void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  K_TRY(mq::omnidir_undistort(cams, C, pts, out, n, (hipStream_t)stream));
  return 0;
}

int mq_omnidir_project(mq_ctx* ctx, const double* cams, int C, const double* p3d, int n, double* out, void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  K_TRY(mq::omnidir_project(cams, C, p3d, out, n, (hipStream_t)stream));
  return 0;
}

int mq_camera_undistort(mq_ctx* ctx, const double* cams, int C, const double* pts, int n, double* out, void* stream) {
  return mq_omnidir_undistort(ctx, cams, C, pts, n, out, stream);
}

int mq_camera_project(mq_ctx* ctx, const double* cams, int C, const double* p3d, int n, double* out, void* stream) {
  return mq_omnidir_project(ctx, cams, C, p3d, n, out, stream);
}

int mq_triangulate_dlt(mq_ctx* ctx, const double* cams, int C, const double* pts, int n, int undistort, double* out,
                       void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  if (undistort && n > 0) {
    // undistort every (camera, point) in parallel first (20 fixed-point iterations each), then the
    // per-point DLT on the undistorted coordinates: the same arithmetic as undistorting inside the DLT
    // kernel, spread over C x n threads instead of n
    if (ctx->dlt_ws.ensure((size_t)C * n * 2 * sizeof(double))) return fail("DLT workspace alloc failed", -5);
    K_TRY(mq::omnidir_undistort(cams, C, pts, ctx->dlt_ws.as<double>(), n, (hipStream_t)stream));
    K_TRY(mq::triangulate_dlt(cams, C, ctx->dlt_ws.as<double>(), n, 0, out, (hipStream_t)stream));
    return 0;
  }
  K_TRY(mq::triangulate_dlt(cams, C, pts, n, undistort, out, (hipStream_t)stream));
  return 0;
}

int mq_reproj_error(mq_ctx* ctx, const double* cams, int C, const double* p3d, const double* p2d, int n, int mean,
                    double* out, void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  K_TRY(mq::reprojection_error(cams, C, p3d, p2d, n, mean, out, (hipStream_t)stream));
  return 0;
}

int mq_triangulate_ransac(mq_ctx* ctx, const double* cams, int C, const double* pts, int n, int min_cams,
                          double threshold, double* p3d, uint8_t* picked, double* p2d, double* err, void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  K_TRY(mq::triangulate_ransac(cams, C, pts, n, min_cams, threshold, p3d, picked, p2d, err, (hipStream_t)stream));
  return 0;
}

int mq_triangulate_pinv(mq_ctx* ctx, const double* cams, int C, const double* und, const uint8_t* use, int n,
                        double* out, void* stream) {
  int rc = check_geo(ctx, cams, C, n);
  if (rc) return rc;
  K_TRY(mq::triangulate_pinv(cams, C, und, use, n, out, (hipStream_t)stream));
  return 0;
}

int mq_geometry_affinity(mq_ctx* ctx, const double* cams, int C, const double* points, const int32_t* cam_of_det,
                         int B, int M, int J, double thr_kp, double* affinity, void* stream) {
  int rc = check_geo(ctx, cams, C, B);
  if (rc) return rc;
  if (!points || !cam_of_det || !affinity) return fail("mq_geometry_affinity: null argument");
  if (M < 0 || J < 0) return fail("mq_geometry_affinity: negative size", -2);
  if ((int64_t)B * M == 0) return 0;
  if ((int64_t)B * M * M > (int64_t)1 << 31 || (int64_t)B * M * J > (int64_t)1 << 28)
    return fail("mq_geometry_affinity: batch too large", -2);
  const size_t rays_b = ((size_t)B * M * J * 6 * 8 + 255) & ~(size_t)255;
  if (ctx->assoc_ws.ensure(rays_b + (size_t)B * M * M * 8 + 256)) return fail("affinity workspace alloc failed", -5);
  double* rays = ctx->assoc_ws.as<double>();
  double* dist = reinterpret_cast<double*>(ctx->assoc_ws.as<char>() + rays_b);
  K_TRY(mq::geometry_affinity(cams, C, points, cam_of_det, B, M, J, thr_kp, rays, dist, affinity, (hipStream_t)stream));
  return 0;
}

int mq_match_svt(mq_ctx* ctx, const double* S, const int32_t* n_det, const int32_t* cam_of_det, int B, int Nmax,
                 double alpha, double lambda, double mu, double tol, int max_iter, int pselect, uint8_t* match,
                 double* x_out, int32_t* iters, void* stream) {
  if (!ctx || !S || !n_det || !cam_of_det || !match || !iters) return fail("mq_match_svt: null argument");
  if (B < 0 || Nmax < 0) return fail("mq_match_svt: negative size", -2);
  if (B == 0 || Nmax == 0) return 0;
  if (Nmax > 64) return fail("mq_match_svt: at most 64 detections per keyframe", -2);
  if ((int64_t)B * Nmax * Nmax > (int64_t)1 << 30) return fail("mq_match_svt: batch too large", -2);
  if (max_iter < 1) return fail("mq_match_svt: max_iter must be >= 1", -2);
  if (!(mu > 0) || !(tol >= 0)) return fail("mq_match_svt: mu must be > 0 and tol >= 0", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->assoc_ws.ensure(mq::match_svt_workspace_bytes(B, Nmax))) return fail("match_svt workspace alloc failed", -5);
  K_TRY(mq::match_svt(S, n_det, cam_of_det, B, Nmax, alpha, lambda, mu, tol, max_iter, pselect, ctx->assoc_ws.p, match,
                      x_out, iters, (hipStream_t)stream));
  return 0;
}

int mq_viterbi_filter(mq_ctx* ctx, const double* kp, int A, int F, int C, int J, double score_threshold, int n_back,
                      double offset_threshold, double* out, void* stream) {
  if (!ctx || !kp || !out) return fail("mq_viterbi_filter: null argument");
  if (A < 0 || F < 0 || C < 0 || J < 0) return fail("mq_viterbi_filter: negative size", -2);
  if (n_back < 1 || n_back > 3) return fail("mq_viterbi_filter: n_back must be in [1, 3]", -2);
  if ((int64_t)A * F * C * J == 0) return 0;
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->scratch.ensure(mq::viterbi_scratch_bytes(A, F, C, J, n_back))) return fail("viterbi scratch alloc failed", -5);
  K_TRY(mq::viterbi_filter(kp, A, F, C, J, score_threshold, n_back, offset_threshold, ctx->scratch.p, out,
                           (hipStream_t)stream));
  return 0;
}

int mq_optim_points(mq_ctx* ctx, const double* cams, int C, const double* p2d, double* x, int B, int F, int J,
                    const int32_t* constraints, int n_strong, int n_weak, const double* scale_smooth_full,
                    double scale_length, double scale_length_weak, double reproj_error_threshold, int reproj_loss,
                    int n_deriv_smooth, int fix_lengths, int max_iter, double ftol, int solver, double* stats,
                    void* stream) {
  if (!ctx || !cams || !p2d || !x || !scale_smooth_full || !stats) return fail("mq_optim_points: null argument");
  if (B < 0 || F < 0 || J < 0 || n_strong < 0 || n_weak < 0) return fail("mq_optim_points: negative size", -2);
  if ((int64_t)B * F * J == 0) return 0;
  if (C < 1 || C > 16) return fail("mq_optim_points: 1 <= cameras <= 16", -2);
  if (J > 32 || n_strong + n_weak > 64) return fail("mq_optim_points: at most 32 joints and 64 constraints", -2);
  if (n_deriv_smooth < 1 || n_deriv_smooth > 3) return fail("mq_optim_points: n_deriv_smooth must be 1..3", -2);
  if (reproj_loss < 0 || reproj_loss > 2) return fail("mq_optim_points: loss must be 0 linear, 1 soft_l1, 2 huber", -2);
  if (!(reproj_error_threshold > 0)) return fail("mq_optim_points: reproj_error_threshold must be > 0", -2);
  if (solver != 0 && solver != 1) return fail("mq_optim_points: solver must be 0 (trf) or 1 (lm)", -2);
  if (max_iter < 0) return fail("mq_optim_points: max_iter must be >= 0", -2);
  if (n_strong + n_weak > 0 && !constraints) return fail("mq_optim_points: null constraints");
  for (int k = 0; k < 2 * (n_strong + n_weak); ++k)
    if (constraints[k] < 0 || constraints[k] >= J) return fail("mq_optim_points: constraint joint out of range", -2);
  HIP_TRY(hipSetDevice(ctx->device));
  const int NL = n_strong + n_weak;
  int rc;
  if (solver == 0) {
    if (ctx->optim_ws.ensure(mq::optim_trf_workspace_bytes(B, F, J, C, NL)))
      return fail("optim workspace alloc failed", -5);
    rc = mq::optim_points_trf(cams, C, p2d, x, B, F, J, constraints, n_strong, n_weak, scale_smooth_full, scale_length,
                              scale_length_weak, reproj_error_threshold, reproj_loss, n_deriv_smooth, fix_lengths,
                              max_iter, ftol, ctx->optim_ws.p, stats, (hipStream_t)stream);
  } else {
    if (ctx->optim_ws.ensure(mq::optim_workspace_bytes(B, F, J, NL))) return fail("optim workspace alloc failed", -5);
    std::vector<double> st4(4 * (size_t)B, 0.0);
    rc = mq::optim_points(cams, C, p2d, x, B, F, J, constraints, n_strong, n_weak, scale_smooth_full, scale_length,
                          scale_length_weak, reproj_error_threshold, reproj_loss, n_deriv_smooth, fix_lengths,
                          max_iter > 0 ? max_iter : 200, ftol, ctx->optim_ws.p, st4.data(), (hipStream_t)stream);
    for (int b = 0; b < B; ++b) {
      for (int i = 0; i < 4; ++i) stats[8 * b + i] = st4[4 * b + i];
      for (int i = 4; i < 8; ++i) stats[8 * b + i] = 0.0;
    }
  }
  if (rc != 0) return fail("mq_optim_points: solver failed (" + std::to_string(rc) + ")", -6);
  return 0;
}

int mq_attention_bf16(mq_ctx* ctx, const uint16_t* qkv, uint16_t* out, int n_img, int tokens, int dim, int heads,
                      void* stream) {
  if (!ctx || !qkv || !out) return fail("mq_attention_bf16: null argument");
  if (n_img <= 0) return 0;
  HIP_TRY(hipSetDevice(ctx->device));
  const int rc = mq::attention_bf16(qkv, out, n_img, tokens, dim, heads, (hipStream_t)stream);
  if (rc != 0) return fail("mq_attention_bf16: unsupported shape (tokens % 32 == 0, <= 192; head dim 64 or 80)", -2);
  return 0;
}

}  // extern "C"

// error reporting for the host-only translation units (optim_host.cpp)
int mq_fail_host(const std::string& msg, int code) { return fail(msg, code); }
