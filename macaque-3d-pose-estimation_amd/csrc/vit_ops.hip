// ViT-side kernels for gfx950: LayerNorm, fused global attention (192 tokens,
// K/V staged whole in LDS), patch im2col (+ flip-test copy), deconv col2im with
// the eval BatchNorm + ReLU fused, and weight packing.
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

// ---------------------------------------------------------------- LayerNorm
// One wave per row: fp32 in, bf16 (GEMM operand) or f32 (residual stream) out.
// NADD > 0: the residual updates of a pre-norm block fused in front of the next LayerNorm -- x += p1 (+= p2),
// the branch outputs in bf16 (bias included) as the proj / fc2 GEMMs write them, added in that order; the
// updated row is written back to x when STORE_X, then normalised.
template <int MAXIT, bool OUT_F32, int NADD, bool STORE_X>
__global__ __launch_bounds__(256) void layernorm_kernel(float* __restrict__ x, const bf16_t* __restrict__ p1,
                                                         const bf16_t* __restrict__ p2, const float* __restrict__ g,
                                                         const float* __restrict__ b, void* __restrict__ yv,
                                                         int rows, int dim, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* xr = x + (size_t)row * dim;
  float4 v[MAXIT], gg[MAXIT], bb[MAXIT];
  uint2 pa[MAXIT], pb[MAXIT];
  // gamma / beta (and the branch outputs) are loaded together with the row (one memory round trip per wave)
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int i = it * 256 + lane * 4;
    pa[it] = pb[it] = make_uint2(0u, 0u);
    if (i < dim) {
      v[it] = *reinterpret_cast<const float4*>(xr + i);
      if constexpr (NADD >= 1) pa[it] = *reinterpret_cast<const uint2*>(p1 + (size_t)row * dim + i);
      if constexpr (NADD >= 2) pb[it] = *reinterpret_cast<const uint2*>(p2 + (size_t)row * dim + i);
      gg[it] = *reinterpret_cast<const float4*>(g + i);
      bb[it] = *reinterpret_cast<const float4*>(b + i);
    } else {
      v[it] = gg[it] = bb[it] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  auto add_bf16x4 = [](float4& a, uint2 q) {
    a.x += __uint_as_float(q.x << 16);
    a.y += __uint_as_float(q.x & 0xffff0000u);
    a.z += __uint_as_float(q.y << 16);
    a.w += __uint_as_float(q.y & 0xffff0000u);
  };
  if constexpr (NADD >= 1) {
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int i = it * 256 + lane * 4;
      if (i < dim) {
        add_bf16x4(v[it], pa[it]);
        if constexpr (NADD >= 2) add_bf16x4(v[it], pb[it]);
        if constexpr (STORE_X) *reinterpret_cast<float4*>(xr + i) = v[it];
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) s += (v[it].x + v[it].y) + (v[it].z + v[it].w);
  const float mean = wave_sum(s) / (float)dim;
  float q = 0.f;
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int i = it * 256 + lane * 4;
    if (i < dim) {
      float a0 = v[it].x - mean, a1 = v[it].y - mean, a2 = v[it].z - mean, a3 = v[it].w - mean;
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)dim + eps);
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int i = it * 256 + lane * 4;
    if (i < dim) {
      const float o0 = (v[it].x - mean) * rstd * gg[it].x + bb[it].x, o1 = (v[it].y - mean) * rstd * gg[it].y + bb[it].y;
      const float o2 = (v[it].z - mean) * rstd * gg[it].z + bb[it].z, o3 = (v[it].w - mean) * rstd * gg[it].w + bb[it].w;
      if constexpr (OUT_F32) {
        *reinterpret_cast<float4*>((float*)yv + (size_t)row * dim + i) = make_float4(o0, o1, o2, o3);
      } else {
        uint2 o;
        o.x = pack_bf16x2(o0, o1);
        o.y = pack_bf16x2(o2, o3);
        *reinterpret_cast<uint2*>((bf16_t*)yv + (size_t)row * dim + i) = o;
      }
    }
  }
}

template <bool OUT_F32, int NADD, bool STORE_X>
static int launch_layernorm(float* x, const bf16_t* p1, const bf16_t* p2, const float* gamma, const float* beta,
                            void* y, int rows, int dim, float eps, hipStream_t s) {
  if (dim % 4 || dim > 3072) return -1;
  dim3 grid((rows + 3) / 4), block(256);
  if (dim <= 512)
    hipLaunchKernelGGL((layernorm_kernel<2, OUT_F32, NADD, STORE_X>), grid, block, 0, s, x, p1, p2, gamma, beta, y,
                       rows, dim, eps);
  else if (dim <= 1280)
    hipLaunchKernelGGL((layernorm_kernel<5, OUT_F32, NADD, STORE_X>), grid, block, 0, s, x, p1, p2, gamma, beta, y,
                       rows, dim, eps);
  else
    hipLaunchKernelGGL((layernorm_kernel<12, OUT_F32, NADD, STORE_X>), grid, block, 0, s, x, p1, p2, gamma, beta, y,
                       rows, dim, eps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int layernorm_f32_bf16(const float* x, const float* gamma, const float* beta, unsigned short* y, int rows, int dim,
                       float eps, hipStream_t s) {
  return launch_layernorm<false, 0, false>(const_cast<float*>(x), nullptr, nullptr, gamma, beta, y, rows, dim, eps, s);
}

int layernorm_f32_f32(const float* x, const float* gamma, const float* beta, float* y, int rows, int dim, float eps,
                      hipStream_t s) {
  return launch_layernorm<true, 0, false>(const_cast<float*>(x), nullptr, nullptr, gamma, beta, y, rows, dim, eps, s);
}

int add_layernorm_f32_bf16(float* x, const unsigned short* p1, const unsigned short* p2, bool store_x,
                           const float* gamma, const float* beta, unsigned short* y, int rows, int dim, float eps,
                           hipStream_t s) {
  const bf16_t* a = reinterpret_cast<const bf16_t*>(p1);
  const bf16_t* b = reinterpret_cast<const bf16_t*>(p2);
  if (!p1) return -1;
  if (b)
    return store_x ? launch_layernorm<false, 2, true>(x, a, b, gamma, beta, y, rows, dim, eps, s)
                   : launch_layernorm<false, 2, false>(x, a, b, gamma, beta, y, rows, dim, eps, s);
  return store_x ? launch_layernorm<false, 1, true>(x, a, nullptr, gamma, beta, y, rows, dim, eps, s)
                 : launch_layernorm<false, 1, false>(x, a, nullptr, gamma, beta, y, rows, dim, eps, s);
}

// ---------------------------------------------------------------- attention
// One workgroup (6 waves) per (image, head); K and V staged whole in LDS by LDS-DMA; each wave owns
// two 16-query blocks (attention2_kernel below).
constexpr int ATT_WAVES = 6;  // 12 query blocks of 16 at T = 192: two per wave
constexpr int ATT_THREADS = 64 * ATT_WAVES;
constexpr int ATT_MAXT = 192;

template <int DH>
struct AttLayout {
  static constexpr int VCH = DH == 64 ? 10 : DH / 8;  // V row stride in 16-B chunks (= 8 * odd dwords mod 64)
  static constexpr int VBYTES = (ATT_MAXT * VCH + 63) / 64 * 1024;
};

// Q / K / V rows of (image, head): row-major QKV (ld = 3 D; sections at columns 0, D, 2 D, the head at
// h DH) or, with nt_hm = images x tokens > 0, the head-major blocks the ViT qkv GEMM writes (GemmArgs
// head_dim): block s H + h of nt_hm x DH, ld = DH -- each head's 192 x 160-B rows contiguous.
template <int DH>
__device__ __forceinline__ int att_bases(const bf16_t* qkv, int D, int H, int h, size_t row0, int nt_hm,
                                         const bf16_t*& qb, const bf16_t*& kb, const bf16_t*& vb) {
  if (nt_hm) {
    qb = qkv + ((size_t)h * nt_hm + row0) * DH;
    kb = qkv + ((size_t)(H + h) * nt_hm + row0) * DH;
    vb = qkv + ((size_t)(2 * H + h) * nt_hm + row0) * DH;
    return DH;
  }
  qb = qkv + row0 * 3 * D + h * DH;
  kb = qb + D;
  vb = kb + D;
  return 3 * D;
}

// XCD-aware (image, head) of a workgroup: blocks b and b + 8 share an XCD (round-robin dispatch), so
// the bijective remap gives every XCD a contiguous range of (image, head) items, all heads of an image on
// one XCD.  A head's Q / K / V rows are 160 B of a 7,680-B QKV row: neighbouring heads share their
// boundary 128-B lines, which then hit in that XCD's L2 instead of being fetched once per XCD.
__device__ __forceinline__ int att_item(int H) {
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// ---------------------------------------------------------------- attention kernel
// One 6-wave workgroup per (image, head), two 16-query blocks per wave, K/V staged whole in LDS by
// LDS-DMA, Q fragments straight to registers:
//   S^T = K Q^T   v_mfma_f32_16x16x32_bf16: ceil(DH/32) k-steps of 32 (the last one half
//                 zero-padded on the Q side when DH % 32 == 16) instead of DH/16 steps of the
//                 half-rate 16x16x16 form.  K image rows of 10 x 16-B chunks (80 d = 160 B, no
//                 pad): the ds_read_b128 lane groups of the A-operand pattern hit 16 distinct
//                 slots, conflict-free.
//   softmax       in registers; row max by 3-input max, sum by plain adds, 2 cross-lane steps.
//   O^T = V^T P^T v_mfma_f32_16x16x32_bf16 with V^T as the A operand (the same ds_read_b64_tr_b16
//                 gather as before) and P as the B operand: the output lands with the query on the
//                 lane and 4 consecutive d per lane, so the 1/l normalisation needs no cross-lane
//                 step and a v_permlane16_swap pairs neighbouring d runs into 16-B row stores.
constexpr int ATT2_KCH = 10;  // K image row stride in 16-B chunks (DH <= 80)

// one 16-B LDS read in inline asm with an immediate offset: the QK^T loop below keeps its own ring of K
// fragments in flight and counts them with explicit lgkmcnt waits (the compiler, left to itself at <= 128
// VGPRs, kept one read ahead of each MFMA)
template <int OFF>
__device__ __forceinline__ bf16x8 att_ds_read16(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
// K fragment of key block tb: row tb * 16 + l16 of the K image = base + tb * 16 rows * KCH * 16 B
__device__ __forceinline__ bf16x8 att_read_kfrag(unsigned base, int tb) {
  constexpr int R = 16 * ATT2_KCH * 16;
  switch (tb) {
    case 0: return att_ds_read16<0>(base);
    case 1: return att_ds_read16<1 * R>(base);
    case 2: return att_ds_read16<2 * R>(base);
    case 3: return att_ds_read16<3 * R>(base);
    case 4: return att_ds_read16<4 * R>(base);
    case 5: return att_ds_read16<5 * R>(base);
    case 6: return att_ds_read16<6 * R>(base);
    case 7: return att_ds_read16<7 * R>(base);
    case 8: return att_ds_read16<8 * R>(base);
    case 9: return att_ds_read16<9 * R>(base);
    case 10: return att_ds_read16<10 * R>(base);
    default: return att_ds_read16<11 * R>(base);
  }
}
template <int N>
__device__ __forceinline__ void att_wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
// a count known after unrolling (the switch folds)
__device__ __forceinline__ void att_wait_lgkm_n(int n) {
  switch (n) {
    case 0: att_wait_lgkm<0>(); break;
    case 1: att_wait_lgkm<1>(); break;
    case 2: att_wait_lgkm<2>(); break;
    case 3: att_wait_lgkm<3>(); break;
    case 4: att_wait_lgkm<4>(); break;
    case 5: att_wait_lgkm<5>(); break;
    case 6: att_wait_lgkm<6>(); break;
    default: att_wait_lgkm<7>(); break;
  }
}

// max of finite floats without the IEEE-mode operand quieting fmaxf carries (v_max3_f32 / v_max_f32 in asm)
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float bfly16_max_raw(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3_raw(__uint_as_float(p[0]), __uint_as_float(p[1]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float bfly32_max_raw(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3_raw(__uint_as_float(p[0]), __uint_as_float(p[1]), __uint_as_float(p[1]));
}

// -DATT_DIAG=<bits> diagnostic builds (tools/gemm_diag.py --attention; never the shipped library, results are
// garbage): 1 no K / V / Q loads; 2 no exponentials (the argument itself); 4 no P V^T MFMAs; 8 no stores; 16 no
// Q K^T MFMAs; 32 no K fragment reads from LDS.  Values a removed part would have produced are laundered through
// an empty asm so the rest stays.
#ifndef ATT_DIAG
#define ATT_DIAG 0
#endif
template <int DH, int TT = 0>
__global__ __launch_bounds__(ATT_THREADS, 4) void attention2_kernel(const bf16_t* __restrict__ qkv,
                                                                     bf16_t* __restrict__ out, int T_rt, int D,
                                                                     int H, float scale_log2, int nt_hm) {
  using L = AttLayout<DH>;
  const int T = TT ? TT : T_rt;
  constexpr int NKS = (DH + 31) / 32;   // 16x16x32 k-steps of QK^T
  constexpr bool HALF = (DH % 32) == 16;  // last k-step carries 16 real d
  constexpr int NDT = DH / 16;          // 16-wide d blocks of O
  constexpr int DCH = DH / 8;           // data chunks per row
  constexpr int KCH = ATT2_KCH;
  constexpr int MAXT = ATT_MAXT;
  constexpr int KBYTES = (MAXT * KCH + 63) / 64 * 1024;
  static_assert(DCH <= KCH, "K image row too short");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Vimg = smem + KBYTES;

  const int item = att_item(H);
  const int img = item / H, h = item % H;
  const size_t row0 = (size_t)img * T;
  const bf16_t *qbase, *kbase, *vbase;
  const int ld = att_bases<DH>(qkv, D, H, h, row0, nt_hm, qbase, kbase, vbase);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int ntb = T / 16;

  const int nk_ins = (ATT_DIAG & 1) ? 0 : (T * KCH + 63) / 64, nv_ins = (ATT_DIAG & 1) ? 0 : (T * L::VCH + 63) / 64;
  for (int ins = wave; ins < nk_ins; ins += ATT_WAVES) {
    const int q = ins * 64 + lane;
    int t = q / KCH, ch = q - (q / KCH) * KCH;
    if (t >= T || ch >= DCH) t = 0, ch = 0;
    __builtin_amdgcn_global_load_lds(MQ_LDS_GLOBAL(kbase + (size_t)t * ld + ch * 8), MQ_LDS_LOCAL(Kimg + ins * 1024),
                                     16, 0, 0);
  }
  for (int ins = wave; ins < nv_ins; ins += ATT_WAVES) {
    const int q = ins * 64 + lane;
    int t = q / L::VCH, ch = q - (q / L::VCH) * L::VCH;
    if (t >= T || ch >= DCH) t = 0, ch = 0;
    __builtin_amdgcn_global_load_lds(MQ_LDS_GLOBAL(vbase + (size_t)t * ld + ch * 8), MQ_LDS_LOCAL(Vimg + ins * 1024),
                                     16, 0, 0);
  }
  // Q^T fragments (B operand: k = d 32 ks + 8 g + j, column = query l16); d >= DH is zero
  bf16x8 qf[2][NKS];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int qb = min(wave + u * ATT_WAVES, ntb - 1);
    const bf16_t* qrow = qbase + (size_t)(qb * 16 + l16) * ld;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (HALF && ks == NKS - 1 && g >= 2)
        qf[u][ks] = bf16x8{};
      else if constexpr ((ATT_DIAG & 1) != 0)
        asm volatile("" : "=v"(qf[u][ks]));
      else
        qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wave >= ntb) return;
  const bool has1 = (TT == MAXT) ? true : (wave + ATT_WAVES < ntb);

  // Per query block u: QK(u) -> softmax(u) -> PV(u), the two blocks one after the other (a
  // software-pipelined order -- QK(1) under softmax(0) -- needs both blocks' scores live: 138 VGPRs,
  // three waves per SIMD, and a second workgroup then only fits a CU on complementary SIMDs; the
  // sequential order stays at <= 128 VGPRs).  K / V fragments are read from LDS once per block.
  f32x4 S[2][MAXT / 16];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int tb = 0; tb < MAXT / 16; ++tb) S[u][tb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // QK^T: the NKS x ntb K fragments (t = ks * ntb + tb) stream through a ring of KR registers, KD reads in
  // flight ahead of the MFMA that uses them (the read of fragment t + KD is issued right after MFMA t - (KR - KD),
  // the last reader of its ring slot); each MFMA waits by a counted lgkmcnt for its own fragment only.  At the
  // full 192 tokens the sequence is static (36 MFMAs); other token counts take the compiler-scheduled loop.
  auto qk = [&](int u) {
    if constexpr (TT == MAXT) {
      constexpr int NTB = MAXT / 16, NF = NKS * NTB, KD = 6, KR = 8;
      unsigned kbase[NKS];
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int chunk = (HALF && ks == NKS - 1) ? 4 * ks + (g & 1) : 4 * ks + g;
        kbase[ks] = (unsigned)(uintptr_t)MQ_LDS_LOCAL(Kimg + l16 * (KCH * 16) + chunk * 16);
      }
      bf16x8 ring[KR];
#pragma unroll
      for (int t = 0; t < KD; ++t) {
        if constexpr ((ATT_DIAG & 32) != 0)
          asm volatile("" : "=v"(ring[t]) : "v"(kbase[t / NTB]));
        else
          ring[t] = att_read_kfrag(kbase[t / NTB], t % NTB);
      }
#pragma unroll
      for (int t = 0; t < NF; ++t) {
        // reads issued after fragment t: min(t + KD, NF) - (t + 1)
        att_wait_lgkm_n(NF - 1 - t < KD - 1 ? NF - 1 - t : KD - 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(ATT_DIAG & 16))
          S[u][t % NTB] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[t % KR], qf[u][t / NTB], S[u][t % NTB], 0, 0, 0);
        else
          asm volatile("" : "+v"(S[u][t % NTB]) : "v"(ring[t % KR]), "v"(qf[u][t / NTB]));
        __builtin_amdgcn_sched_barrier(0);
        if (t + KD < NF) {
          if constexpr ((ATT_DIAG & 32) != 0)
            asm volatile("" : "=v"(ring[(t + KD) % KR]) : "v"(kbase[(t + KD) / NTB]));
          else
            ring[(t + KD) % KR] = att_read_kfrag(kbase[(t + KD) / NTB], (t + KD) % NTB);
        }
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const int chunk = (HALF && ks == NKS - 1) ? 4 * ks + (g & 1) : 4 * ks + g;
        bf16x8 kf[MAXT / 16];
#pragma unroll
        for (int tb = 0; tb < MAXT / 16; ++tb)
          if (tb < ntb) kf[tb] = *reinterpret_cast<const bf16x8*>(Kimg + (tb * 16 + l16) * (KCH * 16) + chunk * 16);
#pragma unroll
        for (int tb = 0; tb < MAXT / 16; ++tb)
          if (tb < ntb) S[u][tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[tb], qf[u][ks], S[u][tb], 0, 0, 0);
      }
    }
  };
  // softmax over the tokens of query l16: registers hold tokens tb*16 + 4 g + e.  The row max and
  // sum run as independent chains so the dependent-latency chain is ntb deep instead of 4 ntb.
  bf16x8 P[2][MAXT / 32];
  float linv[2];
  auto softmax = [&](int u) {
    // row max: four independent chains of v_max3_f32 in inline asm (fmaxf on MFMA results made the compiler
    // quieten every operand first -- one extra v_max_f32 per score in IEEE mode; the scores are finite)
    float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int tb = 0; tb + 1 < MAXT / 16; tb += 2)
      if (tb + 1 < ntb) {
#pragma unroll
        for (int e = 0; e < 4; ++e) m4[e] = max3_raw(m4[e], S[u][tb][e], S[u][tb + 1][e]);
      } else if (tb < ntb) {
#pragma unroll
        for (int e = 0; e < 4; ++e) m4[e] = max3_raw(m4[e], S[u][tb][e], S[u][tb][e]);
      }
    float m = max3_raw(max3_raw(m4[0], m4[1], m4[2]), m4[3], m4[3]);
    // the query's other tokens live in lane groups g ^ 1, g ^ 2: butterflies by permlane swaps (VALU,
    // no LDS round trip as with ds_bpermute)
    m = bfly16_max_raw(m);
    m = bfly32_max_raw(m);
    const float mbu = m * scale_log2;
    // exponent arguments (one packed fma per pair) and the running sums on float pairs
    const f32x2 sc2 = {scale_log2, scale_log2}, mb2 = {-mbu, -mbu};
    f32x2 l2[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
    for (int tb = 0; tb < MAXT / 16; ++tb) {
      if (tb < ntb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 arg = __builtin_elementwise_fma((f32x2){S[u][tb][2 * h], S[u][tb][2 * h + 1]}, sc2, mb2);
#if ATT_DIAG & 2
          const f32x2 pv = arg;
#else
          const f32x2 pv = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
#endif
          S[u][tb][2 * h] = pv.x;
          S[u][tb][2 * h + 1] = pv.y;
          l2[h] += pv;
        }
      }
    }
    float ls = (l2[0].x + l2[1].x) + (l2[0].y + l2[1].y);
    ls = bfly16_sum(ls);
    ls = bfly32_sum(ls);
    linv[u] = 1.0f / ls;
    // B operand of P^T: element j of lane group g = token 32 kst + 16 (j >> 2) + 4 g + (j & 3)
#pragma unroll
    for (int kst = 0; kst < MAXT / 32; ++kst) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        P[u][kst][e] = (__bf16)S[u][2 * kst][e];
        P[u][kst][4 + e] = (__bf16)S[u][2 * kst + 1][e];
      }
    }
  };
  f32x4 O[2][NDT];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) O[u][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // V^T (A operand, row = d, k = the token order of P): transposed read, lane 4q+p of each 16-lane
  // group addresses token row r0+q, columns c0+4p..+3 and receives column c0 + (lane & 15)
  const int trq = l16 >> 2, trp = l16 & 3;
  auto pv = [&](int u) {
#pragma unroll
    for (int kst = 0; kst < MAXT / 32; ++kst) {
      if (kst < T / 32) {
        bf16x8 vb[NDT];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int ra = 2 * kst * 16 + 4 * g + trq;
          const char* pa = Vimg + ra * (L::VCH * 16) + (dt * 16 + 4 * trp) * 2;
          const short4v v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) short4v*)MQ_LDS_LOCAL(pa));
          const short4v v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) short4v*)MQ_LDS_LOCAL(pa + 16 * (L::VCH * 16)));
          const short4v* pv0 = &v0;
          const short4v* pv1 = &v1;
          __builtin_memcpy(&vb[dt], pv0, 8);
          __builtin_memcpy(reinterpret_cast<char*>(&vb[dt]) + 8, pv1, 8);
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
          if constexpr (!(ATT_DIAG & 4))
            O[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb[dt], P[u][kst], O[u][dt], 0, 0, 0);
          else
            asm volatile("" : "+v"(O[u][dt]) : "v"(vb[dt]), "v"(P[u][kst]));
      }
    }
  };
  // O^T C-layout: column = query l16, rows 4 g + e = d within the 16-block dt.  Pairs (dt, dt+1):
  // after v_permlane16_swap even groups hold d 16 dt + 4 g + 0..7, odd groups 16 (dt+1) + 4 (g-1) + 0..7.
  // Block 0 is stored before block 1 runs, so its 20 O registers are free during block 1's QK^T ring.
  const bool odd = g & 1;
  auto store = [&](int u) {
    const int q = (wave + u * ATT_WAVES) * 16 + l16;
    bf16_t* orow = out + (row0 + q) * D + h * DH;
    const float inv = linv[u];
    const f32x2 inv2 = {inv, inv};
#pragma unroll
    for (int dp = 0; dp + 1 < NDT; dp += 2) {
      unsigned pk[2][2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const f32x2 a = (f32x2){O[u][dp + hh][0], O[u][dp + hh][1]} * inv2;
        const f32x2 b = (f32x2){O[u][dp + hh][2], O[u][dp + hh][3]} * inv2;
        pk[hh][0] = pack_bf16x2(a.x, a.y);
        pk[hh][1] = pack_bf16x2(b.x, b.y);
      }
      const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      if constexpr ((ATT_DIAG & 8) != 0)
        asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
      else
        *reinterpret_cast<uint4*>(orow + (dp + (odd ? 1 : 0)) * 16 + 4 * (g - (odd ? 1 : 0))) = o;
    }
    if constexpr (NDT & 1) {
      constexpr int dt = NDT - 1;
      const uint2 o = make_uint2(pack_bf16x2(O[u][dt][0] * inv, O[u][dt][1] * inv),
                                 pack_bf16x2(O[u][dt][2] * inv, O[u][dt][3] * inv));
      if constexpr ((ATT_DIAG & 8) != 0)
        asm volatile("" ::"v"(o.x), "v"(o.y));
      else
        *reinterpret_cast<uint2*>(orow + dt * 16 + 4 * g) = o;
    }
  };
  qk(0);
  softmax(0);
  pv(0);
  store(0);
  if (has1) {
    __builtin_amdgcn_sched_barrier(0);
    qk(1);
    softmax(1);
    pv(1);
    store(1);
  }
}

// MQ_TUNE_ATTN_KRING: 1 (default) = at 192 tokens the static QK^T sequence with the inline-asm K-fragment ring and
// hand-counted lgkmcnt waits; 0 = the compiler-scheduled loop of the generic instantiation (bit-identical,
// tests/test_gpu_attention.py; the fallback should a toolchain change break the ring's register assumptions)
int g_attn_kring = 1;
template <int DH>
static void launch_attention(dim3 grid, dim3 block, hipStream_t s, const unsigned short* qkv, unsigned short* out,
                             int tokens, int dim, int heads, float scale_log2, int nt_hm) {
  constexpr int lds2 = (ATT_MAXT * ATT2_KCH + 63) / 64 * 1024 + AttLayout<DH>::VBYTES;
  if (tokens == ATT_MAXT && g_attn_kring)
    hipLaunchKernelGGL((attention2_kernel<DH, ATT_MAXT>), grid, block, lds2, s, qkv, out, tokens, dim, heads,
                       scale_log2, nt_hm);
  else
    hipLaunchKernelGGL((attention2_kernel<DH, 0>), grid, block, lds2, s, qkv, out, tokens, dim, heads, scale_log2,
                       nt_hm);
}

int attention_bf16(const unsigned short* qkv, unsigned short* out, int n_img, int tokens, int dim, int heads,
                   hipStream_t s, bool head_major) {
  const int dh = dim / heads;
  if (tokens % 32 || tokens > ATT_MAXT || tokens <= 0 || dh * heads != dim) return -1;
  const float scale_log2 = (1.0f / sqrtf((float)dh)) * 1.4426950408889634f;
  dim3 grid(n_img * heads), block(ATT_THREADS);
  if (dh == 80)
    launch_attention<80>(grid, block, s, qkv, out, tokens, dim, heads, scale_log2, head_major ? n_img * tokens : 0);
  else if (dh == 64)
    launch_attention<64>(grid, block, s, qkv, out, tokens, dim, heads, scale_log2, head_major ? n_img * tokens : 0);
  else
    return -2;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---------------------------------------------------------------- patch im2col
// A[(f*T + t)][ci*P*P + ky*P + kx] = crop[f % n][ci][py*P + ky - pad][px*P + kx - pad]
// (zero outside); forwards f >= n read the horizontally flipped crop (flip test).
__global__ void patch_im2col_kernel(const float* __restrict__ crops, bf16_t* __restrict__ A, int n, int copies,
                                    int IH, int IW, int P, int pad, int gh, int gw) {
  const int K = 3 * P * P;
  const int k8 = K / 8;
  const int64_t total = (int64_t)n * copies * gh * gw * k8;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int kc = (int)(idx % k8);
    const int64_t m = idx / k8;
    const int t = (int)(m % (gh * gw));
    const int f = (int)(m / (gh * gw));
    const int src = f % n;
    const bool flip = f >= n;
    const int py = t / gw, px = t % gw;
    const int k0 = kc * 8;
    const int ci = k0 / (P * P);
    const int ky = (k0 / P) % P;
    const int kx0 = k0 % P;
    const int y = py * P + ky - pad;
    const float* plane = crops + ((int64_t)src * 3 + ci) * IH * IW;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int x = px * P + kx0 + e - pad;
      bool ok = (y >= 0) && (y < IH) && (x >= 0) && (x < IW);
      int xs = flip ? (IW - 1 - x) : x;
      v[e] = ok ? plane[(int64_t)y * IW + xs] : 0.f;
    }
    uint4 o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                         pack_bf16x2(v[6], v[7]));
    *reinterpret_cast<uint4*>(A + m * K + k0) = o;
  }
}

int patch_im2col(const float* crops, unsigned short* A, int n_crops, int flip_copies, int img_h, int img_w, int patch,
                 int pad, hipStream_t s) {
  if ((patch * patch) % 8) return -1;
  const int gh = (img_h + 2 * pad - patch) / patch + 1;
  const int gw = (img_w + 2 * pad - patch) / patch + 1;
  const int64_t total = (int64_t)n_crops * flip_copies * gh * gw * (3 * patch * patch / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(patch_im2col_kernel, dim3(blocks), dim3(256), 0, s, crops, A, n_crops, flip_copies, img_h, img_w,
                     patch, pad, gh, gw);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------- deconv col2im
// ConvTranspose2d(k4, s2, p1) as GEMM + gather: cols[(img,iy,ix)][(ky*4+kx)*C + co].
// out[(img,oy,ox)][co] = relu(scale[co] * sum_{valid taps} cols + shift[co]),  NHWC bf16.
__global__ void col2im_bn_relu_kernel(const bf16_t* __restrict__ cols, const float* __restrict__ scale,
                                      const float* __restrict__ shift, bf16_t* __restrict__ out, int n, int IH,
                                      int IW, int C) {
  const int OH = IH * 2, OW = IW * 2;
  const int c8 = C / 8;
  const int64_t total = (int64_t)n * OH * OW * c8;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(idx % c8);
    const int64_t pix = idx / c8;
    const int ox = (int)(pix % OW);
    const int oy = (int)((pix / OW) % OH);
    const int img = (int)(pix / ((int64_t)OW * OH));
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // oy = 2*iy - 1 + ky
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int ky = ((oy + 1) & 1) + 2 * a;
      const int ty = oy + 1 - ky;
      const int iy = ty >> 1;
      if (iy < 0 || iy >= IH) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int kx = ((ox + 1) & 1) + 2 * b;
        const int tx = ox + 1 - kx;
        const int ix = tx >> 1;
        if (ix < 0 || ix >= IW) continue;
        const bf16_t* src = cols + (((int64_t)img * IH + iy) * IW + ix) * (16 * C) + (ky * 4 + kx) * C + cc * 8;
        const uint4 u = *reinterpret_cast<const uint4*>(src);
        const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += bf16_to_f32((bf16_t)(w[e] & 0xffff));
          acc[2 * e + 1] += bf16_to_f32((bf16_t)(w[e] >> 16));
        }
      }
    }
    float r[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      r[e] = fmaxf(acc[e] * scale[c] + shift[c], 0.f);
    }
    uint4 o = make_uint4(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]), pack_bf16x2(r[4], r[5]),
                         pack_bf16x2(r[6], r[7]));
    *reinterpret_cast<uint4*>(out + pix * C + cc * 8) = o;
  }
}

int deconv_col2im_bn_relu(const unsigned short* cols, const float* scale, const float* shift, unsigned short* out,
                          int n_img, int in_h, int in_w, int ch, hipStream_t s) {
  if (ch % 8) return -1;
  const int64_t total = (int64_t)n_img * in_h * 2 * in_w * 2 * (ch / 8);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(col2im_bn_relu_kernel, dim3(blocks), dim3(256), 0, s, cols, scale, shift, out, n_img, in_h, in_w,
                     ch);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------- weight packing
__global__ void f32_to_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = f32_to_bf16(src[i]);
}

int convert_f32_bf16(const float* src, unsigned short* dst, int64_t n, hipStream_t s) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(blocks), dim3(256), 0, s, src, dst, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// torch ConvTranspose2d weight [cin][cout][4][4] -> GEMM rows [(ky*4+kx)*cout + co][cin]
__global__ void deconv_pack_kernel(const float* __restrict__ w, bf16_t* __restrict__ dst, int cin, int cout) {
  const int64_t total = (int64_t)cin * cout * 16;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin);
    const int64_t n = i / cin;
    const int co = (int)(n % cout);
    const int kk = (int)(n / cout);
    dst[i] = f32_to_bf16(w[((int64_t)ci * cout + co) * 16 + kk]);
  }
}

int deconv_weight_pack(const float* w, unsigned short* dst, int cin, int cout, hipStream_t s) {
  const int64_t total = (int64_t)cin * cout * 16;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(deconv_pack_kernel, dim3(blocks), dim3(256), 0, s, w, dst, cin, cout);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// torch ConvTranspose2d(k4, s2, p1) weight [cin][cout][4][4] with the eval-BatchNorm scale folded in ->
// the sub-pixel GEMM operand [(cls * cout + co)][tap * cin + ci].  Output pixel (2y + py, 2x + px) takes
// input (y + dy, x + dx) through kernel tap (ky, kx) exactly when oy = 2 iy - 1 + ky, i.e. for class py
// the taps a = 0, 1: ky = (1 - py) + 2a at dy = py - a (py = 0: ky 1, 3 at dy 0, -1; py = 1: ky 0, 2 at
// dy +1, 0); likewise x.  tap = 2a + b.
__global__ void deconv_subpixel_pack_kernel(const float* __restrict__ w, const float* __restrict__ scale,
                                            bf16_t* __restrict__ dst, int cin, int cout) {
  const int64_t total = (int64_t)16 * cin * cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin);
    const int tap = (int)((i / cin) % 4);
    const int64_t row = i / (4 * (int64_t)cin);
    const int co = (int)(row % cout);
    const int cls = (int)(row / cout);
    const int ky = (1 - (cls >> 1)) + 2 * (tap >> 1), kx = (1 - (cls & 1)) + 2 * (tap & 1);
    const float v = w[((int64_t)ci * cout + co) * 16 + ky * 4 + kx];
    dst[i] = f32_to_bf16(scale ? v * scale[co] : v);
  }
}

int deconv_subpixel_pack(const float* w, const float* scale, unsigned short* dst, int cin, int cout, hipStream_t s) {
  const int64_t total = (int64_t)16 * cin * cout;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(deconv_subpixel_pack_kernel, dim3(blocks), dim3(256), 0, s, w, scale, dst, cin, cout);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mq
