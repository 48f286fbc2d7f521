// bf16 MFMA GEMM for gfx950 with fused epilogues: C[M,N] = A[M,K] * W[N,K]^T.
//
// Both operands are K-contiguous (torch Linear layout), which is the natural
// operand order of v_mfma_f32_16x16x32_bf16: lane l reads 16 contiguous bytes of
// row (l & 15) at k = 8*(l >> 4) for A and of W-row (l & 15) for B.
//
// Block tile (32 WF)^2 x 64, 256 threads = 4 waves (2x2), each wave (16 WF)^2 = WF x WF MFMA tiles:
// WF = 4 gives 128x128 tiles, WF = 2 gives 64x64 tiles for GEMMs too small to fill the CUs with
// 128x128 ones (the ID classifier's stage-3/4 convolutions at a frame's dozen boxes, the detector's
// late Swin stages).  Both accumulate every output in the same order (K ascending, 32 per MFMA), so
// they agree bit for bit.  Tiles are staged HBM -> LDS with global_load_lds_dwordx4 (no VGPR
// round trip) through an NS-slot ring: the DMA of K-step t + NS - 1 is issued before step t's MFMAs,
// and each step waits (counted vmcnt) only for its own stage.  The LDS image is XOR-swizzled on the SOURCE address
// (16-B chunk c of row r lives at slot c ^ ((r >> 1) & 7)); the ds_read_b128
// fragment reads are bank-conflict free under that swizzle.
//
// Blocks are remapped so that consecutive tiles (sharing A row panels) land on
// the same XCD (bijective remap, MI355X has 8 XCDs with private L2s).
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

bool g_gemm_force_small = false;
int g_gemm_tile64 = 1;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int GEMM_THREADS = 256;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// Issue the DMA of one (32 WF)x64 bf16 tile (rows [r0, r0 + 32 WF) of a K-contiguous
// matrix with leading dimension ld, columns [k0, k0+64)) into LDS: WF 8-row groups per wave.
template <int WF>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, int ld, int r0, int rmax, int k0,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < WF; ++i) {
    int rbase = (wave * WF + i) * 8;
    int row = rbase + (lane >> 3);
    int slot = lane & 7;
    int chunk = slot ^ swz(row);
    int grow = r0 + row;
    grow = grow < rmax ? grow : rmax - 1;
    const bf16_t* src = g + (size_t)grow * ld + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(MQ_LDS_GLOBAL(src), MQ_LDS_LOCAL(lds_tile + rbase * 128), 16, 0, 0);
  }
}

// Implicit convolution: the A tile of K-step t is tap t / (C / 64), channels 64 (t % (C / 64)) .. + 63 of
// the tap-shifted input pixels of this tile's output rows; a pixel outside the image gets an offset past
// the buffer end, which the DMA turns into zeros (padding).  cbase / cy / cx: per A slot the row's image
// base offset (elements) and its top-left input coordinate (oy s - p, ox s - p).
template <int WF>
__device__ __forceinline__ void stage_conv_a(__amdgpu_buffer_rsrc_t rsA, const GemmArgs& p, const int (&cbase)[WF],
                                             const int (&cy)[WF], const int (&cx)[WF], int t, char* lds_tile,
                                             int wave, int lane) {
  const int kpt = p.conv_c >> 6;
  const int tap = t / kpt, c0 = (t - tap * kpt) * 64;
  const int ky = tap / p.conv_k, kx = tap - ky * p.conv_k;
#pragma unroll
  for (int i = 0; i < WF; ++i) {
    const int rbase = (wave * WF + i) * 8;
    const int row = rbase + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(row);
    const int iy = cy[i] + ky, ix = cx[i] + kx;
    const bool inside = (unsigned)iy < (unsigned)p.conv_h && (unsigned)ix < (unsigned)p.conv_w;
    const unsigned off = (unsigned)(cbase[i] + (iy * p.conv_w + ix) * p.conv_c + c0 + chunk * 8) * 2u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, MQ_LDS_LOCAL(lds_tile + rbase * 128), 16, inside ? off : 0x80000000u,
                                             0, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 read_frag(const char* lds_tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds_tile + row * 128 + ((chunk ^ swz(row)) << 4));
}

template <int EPI, int WF, bool CONV = false, int NS = 2>
__global__ __launch_bounds__(GEMM_THREADS, 2) void gemm_bf16_kernel(GemmArgs p) {
  constexpr int TM = 32 * WF;                // tile rows = tile columns
  constexpr int TB = TM * BK * 2;            // bytes per operand tile
  constexpr int WT = 16 * WF;                // wave tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the linear block id, then M-fastest tile order
  // inside groups so neighbouring tiles share the W panel in L2.
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tiles_m = (p.M + TM - 1) / TM;
  const int tm = wid % tiles_m;
  const int tn = wid / tiles_m;
  const int m0 = tm * TM, n0 = tn * TM;


  f32x4 acc[WF][WF];
#pragma unroll
  for (int i = 0; i < WF; ++i)
#pragma unroll
    for (int j = 0; j < WF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  // implicit convolution: per A slot (this lane's row of each of the wave's 8-row groups) the output
  // pixel's image base and top-left input coordinate
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, 0x7fffffff, 0x00020000);
  int cbase[WF], cy[WF], cx[WF];
  if constexpr (CONV) {
    const int oh = (p.conv_h + 2 * p.conv_p - p.conv_k) / p.conv_s + 1;
    const int ow = (p.conv_w + 2 * p.conv_p - p.conv_k) / p.conv_s + 1;
#pragma unroll
    for (int i = 0; i < WF; ++i) {
      const int pix = min(m0 + (wave * WF + i) * 8 + (lane >> 3), p.M - 1);
      const int img = pix / (oh * ow), rem = pix - img * (oh * ow);
      const int oy = rem / ow, ox = rem - oy * ow;
      cbase[i] = img * p.conv_h * p.conv_w * p.conv_c;
      cy[i] = oy * p.conv_s - p.conv_p;
      cx[i] = ox * p.conv_s - p.conv_p;
    }
  }
  // K-step t's A and W tiles -> ring slot t % NS (2 WF DMA instructions per wave)
  auto issue = [&](int t) {
    char* st = smem + (t % NS) * 2 * TB;
    if constexpr (CONV)
      stage_conv_a<WF>(rsA, p, cbase, cy, cx, t, st, wave, lane);
    else
      stage_tile<WF>(p.A, p.lda, m0, p.M, t * BK, st, wave, lane);
    stage_tile<WF>(p.W, p.ldw, n0, p.N, t * BK, st + TB, wave, lane);
  };
  // NS-stage ring: K-steps t+1 .. t+NS-2 stay in flight while step t computes.  Each K-step waits for
  // its own stage only (counted vmcnt, this wave's DMAs), then one barrier (every wave's part landed,
  // every wave done reading the slot the next DMA overwrites), then issues stage t+NS-1 into the slot
  // of step t-1.
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s);

  const int frow = lane & 15;
  const int fk = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    if (t + NS - 2 < nk)
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * WF * (NS - 2)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const char* As = smem + (t % NS) * 2 * TB;
    const char* Bs = As + TB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[WF], b[WF];
#pragma unroll
      for (int i = 0; i < WF; ++i) a[i] = read_frag(As, wm * WT + i * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int j = 0; j < WF; ++j) b[j] = read_frag(Bs, wn * WT + j * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < WF; ++i)
#pragma unroll
        for (int j = 0; j < WF; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }

  // Epilogue.  C layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < WF; ++j) {
    const int n = n0 + wn * WT + j * 16 + ccol;
    if (n >= p.N) continue;
    const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < WF; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * WT + i * 16 + crow + e;
        if (m >= p.M) continue;
        float v = acc[i][j][e] + bias;
        if constexpr (EPI == EPI_BF16) {
          *gemm_out_bf16(p, m, n) = f32_to_bf16(v);
        } else if constexpr (EPI == EPI_GELU_BF16) {
          ((bf16_t*)p.C)[(size_t)m * p.ldc + n] = f32_to_bf16(gelu_erf(v));
        } else if constexpr (EPI == EPI_RELU_BF16) {
          ((bf16_t*)p.C)[(size_t)m * p.ldc + n] = f32_to_bf16(fmaxf(v, 0.f));
        } else if constexpr (EPI == EPI_RESID_F32) {
          float* c = (float*)p.C + (size_t)m * p.ldc + n;
          *c = *c + v;
        } else if constexpr (EPI == EPI_RESID_RELU) {
          float* c = (float*)p.C + (size_t)m * p.ldc + n;
          const float o = fmaxf(*c + v, 0.f);
          *c = o;
          ((bf16_t*)p.C2)[(size_t)m * p.ldc + n] = f32_to_bf16(o);
        } else if constexpr (EPI == EPI_POS_F32) {
          ((float*)p.C)[(size_t)m * p.ldc + n] = v + p.aux[(size_t)(m % p.aux_rows) * p.N + n];
        } else if constexpr (EPI == EPI_F32) {
          ((float*)p.C)[(size_t)m * p.ldc + n] = v;
        } else if constexpr (EPI == EPI_NCHW_F32) {
          // row m = image * aux_rows + pixel, col n = channel -> out[image][n][pixel]
          const int img = m / p.aux_rows, pix = m - img * p.aux_rows;
          ((float*)p.C)[((size_t)img * p.N + n) * p.aux_rows + pix] = v;
        }
      }
    }
  }
}

// ============================================================================
// 256x256 tile, BK = 32, 4-stage LDS ring (128 KiB), 512 threads = 8 waves (2 M x 4 N),
// each wave 128 x 64 = 8 x 4 MFMA 16x16x32 tiles.  Every K-step issues the DMA of
// the tile three steps ahead and waits only for the NEXT tile (counted vmcnt +
// raw s_barrier: a __syncthreads() would drain every in-flight DMA).  Arithmetic
// intensity 128 FLOP per staged byte (vs 64 for 128x128), ~3 K-steps (~3k cycles)
// of latency cover.  The MFMA runs "swapped" (D = W * A^T): each lane then holds 4
// consecutive output columns of one row, so the epilogue stores 8 B (bf16) or
// 16 B (f32) per lane instead of scalar 2-byte stores.
// LDS image: 64-byte rows, 16-byte chunk c of row r at slot c ^ ((r >> 1) & 3)
// (ds_read_b128 conflict-free for the 16x16x32 fragment pattern).
// Staging: buffer_load_dwordx4 ... lds with a 32-bit per-lane offset fixed per tile and the
// K advance in soffset.  Each K-step is one basic block with the DMAs and the next stage's
// fragment reads spread between the MFMAs (sched_group_barrier).
// This kernel serves the f32-residual GEMM at short K (proj, K = 1280); gemm_pp.hip serves the rest.
constexpr int B2M = 256, B2N = 256, B2K = 32, B2T = 512, B2NS = 4;
constexpr int B2_OP_BYTES = B2M * B2K * 2;       // 16 KiB per operand per stage
constexpr int B2_STAGE_BYTES = 2 * B2_OP_BYTES;  // 32 KiB
constexpr int B2_LDS = B2NS * B2_STAGE_BYTES;    // 128 KiB

__device__ __forceinline__ int swz2(int row) { return (row >> 1) & 3; }

__device__ __forceinline__ bf16x8 frag256(const char* lds_op, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds_op + row * 64 + ((chunk ^ swz2(row)) << 4));
}

// s_waitcnt vmcnt(N) for any N < 64 (the wait leaves the wave's N youngest VMEM ops in flight)
template <int N_IN_FLIGHT>
__device__ __forceinline__ void wait_vm() {
  static_assert(N_IN_FLIGHT >= 0 && N_IN_FLIGHT < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_IN_FLIGHT) : "memory");
}

// Tile -> (m0, n0): grouped ordering (8 M-tiles per group) so the tiles an XCD works
// on concurrently share A and W panels in its L2.
__device__ __forceinline__ void tile_coords(int wid, int tiles_m, int tiles_n, int& m0, int& n0) {
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tiles_n;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_g = wid - grp * per_group;
  m0 = (first_m + in_g % gsize) * B2M;
  n0 = (in_g / gsize) * B2N;
}

// Persistent: one 512-thread block per CU walks its tiles; the DMA stream and the
// fragment pipeline run straight across tile boundaries (the first stages of the
// next tile are in flight while the current tile's epilogue stores drain).
template <int EPI>
__global__ __launch_bounds__(B2T, 2) void gemm256_kernel(GemmArgs p, int tiles_m, int tiles_n) {
  constexpr int MI = 8;                     // 16-row A fragments per wave
  constexpr int NS = B2NS;
  constexpr int DMA_PER_STAGE = 4;          // per wave: 2 A + 2 W wave-instructions
  constexpr int WROWS = B2M / 2;            // A rows per wave (2 waves along M)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave >> 2, wn = wave & 3;
  const int frow = lane & 15;
  const int fk = lane >> 4;

  // tiles of this XCD = a contiguous range; its blocks take them round-robin
  const int nt = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int nbx = (G - xcd + 7) >> 3;  // blocks on this XCD
  const int xb = bid >> 3;
  const int q = nt >> 3, r = nt & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int len = q + (xcd < r ? 1 : 0);
  const int my_tiles = xb < len ? (len - xb + nbx - 1) / nbx : 0;
  const int nk = p.K / B2K;
  const int total = my_tiles * nk;
  if (total == 0) return;

  // DMA issue cursor: (tile, k) of the next stage to load and this lane's source rows
  // for that tile (recomputed only when the cursor moves to the next tile).  Past the
  // end the cursor stays on the last stage: extra DMAs re-load it into a dead buffer,
  // which keeps every wait count uniform.
  int iss_t = 0, iss_k = 0, iss_slot = 0;
  unsigned va[2], vw[2];
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, (int)((size_t)p.M * p.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, (int)((size_t)p.N * p.ldw * 2), 0x00020000);
  auto set_tile_ptrs = [&](int ti) {
    int m0, n0;
    tile_coords(lo + xb + ti * nbx, tiles_m, tiles_n, m0, n0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (wave * 2 + i) * 16 + (lane >> 2);
      const int chunk = (lane & 3) ^ swz2(row);
      const int ga = min(m0 + row, p.M - 1);
      const int gw = min(n0 + row, p.N - 1);
      va[i] = (unsigned)(((size_t)ga * p.lda + chunk * 8) * 2);
      vw[i] = (unsigned)(((size_t)gw * p.ldw + chunk * 8) * 2);
    }
  };
  set_tile_ptrs(0);
  auto issue_a = [&]() {
    char* sb = smem + iss_slot * B2_STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, MQ_LDS_LOCAL(sb + (wave * 2 + i) * 16 * 64), 16, va[i],
                                               iss_k * B2K * 2, 0, 0);
  };
  auto issue_w = [&]() {
    char* sb = smem + iss_slot * B2_STAGE_BYTES + B2_OP_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, MQ_LDS_LOCAL(sb + (wave * 2 + i) * 16 * 64), 16, vw[i],
                                               iss_k * B2K * 2, 0, 0);
  };
  auto advance = [&]() {
    iss_slot = iss_slot + 1 == NS ? 0 : iss_slot + 1;
    if (iss_k + 1 < nk) {
      ++iss_k;
    } else if (iss_t + 1 < my_tiles) {
      ++iss_t;
      iss_k = 0;
      set_tile_ptrs(iss_t);
    }
  };
  auto stage_ptr = [&](int g) { return smem + (g % NS) * B2_STAGE_BYTES; };

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0 .. NS-2 in flight; stage NS-1 is issued by the first K-step
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) {
    issue_a();
    issue_w();
    advance();
  }
  wait_vm<DMA_PER_STAGE * (NS - 3)>();  // stages 0 and 1 landed (this wave)
  __builtin_amdgcn_s_barrier();

  bf16x8 a[MI], b0[4], b1[4];
  {
    const char* As = stage_ptr(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) b0[j] = frag256(As + B2_OP_BYTES, wn * 64 + j * 16 + frow, fk);
#pragma unroll
    for (int i = 0; i < MI; ++i) a[i] = frag256(As, wm * WROWS + i * 16 + frow, fk);
  }

  auto epilogue = [&](int ti) {
    int m0, n0;
    tile_coords(lo + xb + ti * nbx, tiles_m, tiles_n, m0, n0);
    // lane holds D[n][m] with m = l & 15 (col of D) and n = 4 * (l >> 4) + e
    const int mm = lane & 15;
    const int nn = 4 * (lane >> 4);
    if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
      // pack to bf16, then pair tiles (j, j+1): v_permlane16_swap gives every lane 8
      // consecutive columns (even 16-lane groups: tile j, odd groups: tile j+1) -> one
      // 16-byte store per lane per pair instead of two 8-byte stores.
      const bool odd = (lane >> 4) & 1;
      const int nbase = 4 * (lane >> 4) - (odd ? 4 : 0);
      // all bias loads before the first store: a load behind a store would wait for it
      float4 bias[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + nn;
        bias[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * WROWS + i * 16 + mm;
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
          unsigned pk[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = jp + h;
            float v[4] = {acc[i][j][0] + bias[j].x, acc[i][j][1] + bias[j].y, acc[i][j][2] + bias[j].z,
                          acc[i][j][3] + bias[j].w};
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (EPI == EPI_GELU_BF16) {
              const f32x2 g0 = gelu_sig2((f32x2){v[0], v[1]}), g1 = gelu_sig2((f32x2){v[2], v[3]});
              v[0] = g0.x;
              v[1] = g0.y;
              v[2] = g1.x;
              v[3] = g1.y;
            }
            if constexpr (EPI == EPI_RELU_BF16) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            pk[h][0] = pack_bf16x2(v[0], v[1]);
            pk[h][1] = pack_bf16x2(v[2], v[3]);
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          // even lanes: [own tile j | neighbour's tile j]; odd: [neighbour's j+1 | own j+1]
          const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          const int j = jp + (odd ? 1 : 0);
          const int n = n0 + wn * 64 + j * 16 + nbase;
          if (m < p.M && n < p.N)
            *reinterpret_cast<uint4*>(gemm_out_bf16(p, m, n)) = o;
        }
      }
      return;
    }
    if constexpr (EPI == EPI_RESID_F32) {
      // issue every residual load of the wave's tile first (MI*4 independent 16-B loads in
      // flight), then add and store: one HBM round trip per tile instead of one per fragment
      float4 bias[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + nn;
        bias[j] = (p.bias && n < p.N) ? *reinterpret_cast<const float4*>(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const bool full = (m0 + B2M <= p.M) && (n0 + B2N <= p.N);
      if (full) {
        // CH fragment rows of loads in flight at a time (register budget: the accumulators
        // stay live for the next tile)
        constexpr int CH = MI == 8 ? 1 : 4;
#pragma unroll
        for (int i0 = 0; i0 < MI; i0 += CH) {
          float4 x[CH][4];
#pragma unroll
          for (int c = 0; c < CH; ++c) {
            const int m = m0 + wm * WROWS + (i0 + c) * 16 + mm;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              x[c][j] = *reinterpret_cast<const float4*>((const float*)p.C + (size_t)m * p.ldc + n0 + wn * 64 + j * 16 + nn);
          }
#pragma unroll
          for (int c = 0; c < CH; ++c) {
          const int i = i0 + c;
          const int m = m0 + wm * WROWS + i * 16 + mm;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float4 o = x[c][j];
            o.x += acc[i][j][0] + bias[j].x;
            o.y += acc[i][j][1] + bias[j].y;
            o.z += acc[i][j][2] + bias[j].z;
            o.w += acc[i][j][3] + bias[j].w;
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + n0 + wn * 64 + j * 16 + nn) = o;
          }
          }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * WROWS + i * 16 + mm;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn * 64 + j * 16 + nn;
          if (m < p.M && n < p.N) {
            float4* c = reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + n);
            float4 o = *c;
            o.x += acc[i][j][0] + bias[j].x;
            o.y += acc[i][j][1] + bias[j].y;
            o.z += acc[i][j][2] + bias[j].z;
            o.w += acc[i][j][3] + bias[j].w;
            *c = o;
          }
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * WROWS + i * 16 + mm;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + nn;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m >= p.M || n >= p.N) continue;
        if (p.bias) {
          const float4 bias = *reinterpret_cast<const float4*>(p.bias + n);
          v[0] += bias.x;
          v[1] += bias.y;
          v[2] += bias.z;
          v[3] += bias.w;
        }
        if constexpr (EPI == EPI_POS_F32) {
          const float4 ps = *reinterpret_cast<const float4*>(p.aux + (size_t)(m % p.aux_rows) * p.N + n);
          *reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + n) =
              make_float4(v[0] + ps.x, v[1] + ps.y, v[2] + ps.z, v[3] + ps.w);
        } else if constexpr (EPI == EPI_F32) {
          *reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + n) = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };


  // >= this many VMEM ops of a full tile's epilogue are younger than the DMA of the stage a
  // K-step waits for (bf16: 2 stores per fragment row; f32: 4 stores (+ loads) per row)
  constexpr int EPI_OPS = (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) ? 2 * MI : 4 * MI;
  bool stores_pending = false;
  int kt = 0, ct = 0, cm0 = 0, cn0 = 0;  // K-step within the current tile, tile index, its origin
  auto tile_start = [&]() { tile_coords(lo + xb + ct * nbx, tiles_m, tiles_n, cm0, cn0); };
  tile_start();
  auto end_step = [&]() {
    // stage g+2 landed; g+3 .. g+NS-1 in flight.  Right after a full tile's epilogue its
    // stores sit between those DMAs in the in-order vmcnt queue: let them drain behind
    // this step instead of stalling the MFMAs on them.
    if (stores_pending)
      wait_vm<DMA_PER_STAGE * (NS - 3) + EPI_OPS>();
    else
      wait_vm<DMA_PER_STAGE * (NS - 3)>();
    stores_pending = false;
    __builtin_amdgcn_s_barrier();
    if (++kt == nk) {
      epilogue(ct);
      stores_pending = (cm0 + B2M <= p.M) && (cn0 + B2N <= p.N);
      kt = 0;
      ++ct;
      tile_start();
    }
  };
  // one basic block per K-step body with the DMAs and fragment reads spread between the MFMAs
  auto kstep = [&](int g, bf16x8 (&bc)[4], bf16x8 (&bn)[4]) {
    const char* An = stage_ptr(g + 1);  // past the end: harmless reads of a dead buffer
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI / 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], a[i], acc[i][j], 0, 0, 0);
    issue_a();
#pragma unroll
    for (int j = 0; j < 4; ++j) bn[j] = frag256(An + B2_OP_BYTES, wn * 64 + j * 16 + frow, fk);
#pragma unroll
    for (int i = 0; i < MI / 2; ++i) a[i] = frag256(An, wm * WROWS + i * 16 + frow, fk);
    // first half: 4 MI MFMAs, 2 DMAs, 4 + MI/2 fragment reads
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
    }
#pragma unroll
    for (int t = 0; t < 4 + MI / 2; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x8, 2 * MI - 4 - 4 - MI / 2, 0);
#pragma unroll
    for (int i = MI / 2; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j], a[i], acc[i][j], 0, 0, 0);
    issue_w();
#pragma unroll
    for (int i = MI / 2; i < MI; ++i) a[i] = frag256(An, wm * WROWS + i * 16 + frow, fk);
    // second half: 2 MI MFMAs, 2 DMAs, MI/2 fragment reads
    __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
#pragma unroll
    for (int t = 0; t < MI / 2; ++t) {
      __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x8, MI - 4, 0);
    __builtin_amdgcn_s_setprio(0);
    advance();
    end_step();
  };
  int g = 0;
  for (; g + 1 < total; g += 2) {
    kstep(g, b0, b1);
    kstep(g + 1, b1, b0);
  }
  if (g < total) kstep(g, b0, b1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may outlive the block
}

static int g_num_cus = 0;

template <int EPI>
static void launch256(dim3 grid, hipStream_t stream, const GemmArgs& p, int tiles_m, int tiles_n) {
  static std::atomic<unsigned> attr{0};
  if (first_on_device(attr))
    (void)hipFuncSetAttribute((const void*)gemm256_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, B2_LDS);
  hipLaunchKernelGGL((gemm256_kernel<EPI>), grid, dim3(B2T), B2_LDS, stream, p, tiles_m, tiles_n);
}

static int gemm256(const GemmArgs& p, int epi, hipStream_t stream) {
  if (!g_num_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || !g_num_cus)
      g_num_cus = 256;
  }
  if (gemm_w4_fits(p, epi)) return gemm_w4(p, epi, g_num_cus, stream);
  if (gemm_pingpong_fits(p, epi, g_num_cus)) return gemm_pingpong(p, epi, g_num_cus, stream);
  const int tiles_m = (p.M + B2M - 1) / B2M, tiles_n = (p.N + B2N - 1) / B2N;
  const int tiles = tiles_m * tiles_n;
  dim3 grid(tiles < g_num_cus ? tiles : g_num_cus);
  switch (epi) {
    case EPI_BF16: launch256<EPI_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_GELU_BF16: launch256<EPI_GELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch256<EPI_RELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RESID_F32: launch256<EPI_RESID_F32>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_POS_F32: launch256<EPI_POS_F32>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_F32: launch256<EPI_F32>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

int conv3x3_bf16(const GemmArgs& p, int epi, hipStream_t stream) {
  if (!g_num_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || !g_num_cus)
      g_num_cus = 256;
  }
  return gemm_pingpong_conv(p, epi, g_num_cus, stream);
}

int deconv_subpixel_bf16(const GemmArgs& p, int epi, hipStream_t stream) {
  if (!g_num_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || !g_num_cus)
      g_num_cus = 256;
  }
  return gemm_pingpong_deconv(p, epi, g_num_cus, stream);
}

// 64x64 tiles: a 4-stage ring (64 KiB, still two workgroups per CU) keeps three K-steps of DMA in flight
// under the short per-step MFMA work; 128x128 tiles: double buffered (64 KiB)
template <int WF, bool CONV = false>
static int launch_small(const GemmArgs& p, int epi, hipStream_t stream) {
  constexpr int TM = 32 * WF;
  constexpr int NS = WF == 2 ? 4 : 2;
  const int tiles = ((p.M + TM - 1) / TM) * ((p.N + TM - 1) / TM);
  dim3 grid(tiles), block(GEMM_THREADS);
  const size_t lds = (size_t)NS * 2 * TM * BK * 2;
  if constexpr (CONV) {
    switch (epi) {
      case EPI_BF16: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_BF16, WF, true, NS>), grid, block, lds, stream, p); break;
      case EPI_RELU_BF16:
        hipLaunchKernelGGL((gemm_bf16_kernel<EPI_RELU_BF16, WF, true, NS>), grid, block, lds, stream, p);
        break;
      case EPI_F32: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_F32, WF, true, NS>), grid, block, lds, stream, p); break;
      default: return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -4;
  }
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_BF16, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_GELU_BF16, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_RELU_BF16: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_RELU_BF16, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_RESID_F32: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_RESID_F32, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_POS_F32: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_POS_F32, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_F32: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_F32, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_NCHW_F32: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_NCHW_F32, WF, false, NS>), grid, block, lds, stream, p); break;
    case EPI_RESID_RELU: hipLaunchKernelGGL((gemm_bf16_kernel<EPI_RESID_RELU, WF, false, NS>), grid, block, lds, stream, p); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// small-kernel tile choice: 64x64 when 128x128 tiles cannot occupy every CU once (and K is long enough to
// be worth it), or would leave half of every tile's columns empty (N <= 64: the ID stage-1 convolutions)
static bool use_tile64(const GemmArgs& p) {
  if (!g_num_cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || !g_num_cus)
      g_num_cus = 256;
  }
  const int tiles128 = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  return g_gemm_tile64 && ((tiles128 < g_num_cus && p.K >= 256) || p.N <= 64);
}

int conv_small_bf16(const GemmArgs& p, int epi, hipStream_t stream) {
  if (p.conv_c <= 0 || p.conv_c % 64 || p.conv_k <= 0 || p.conv_s <= 0 || p.conv_p < 0 || p.conv_h <= 0 ||
      p.conv_w <= 0 || p.K != p.conv_k * p.conv_k * p.conv_c || p.ldw % 8 || p.M <= 0 || p.N <= 0)
    return -1;
  const int oh = (p.conv_h + 2 * p.conv_p - p.conv_k) / p.conv_s + 1;
  const int ow = (p.conv_w + 2 * p.conv_p - p.conv_k) / p.conv_s + 1;
  if (oh <= 0 || ow <= 0 || p.M % (oh * ow)) return -1;
  const int64_t in_bytes = (int64_t)(p.M / (oh * ow)) * p.conv_h * p.conv_w * p.conv_c * 2;
  if (in_bytes >= (1ll << 31)) return -1;
  return use_tile64(p) ? launch_small<2, true>(p, epi, stream) : launch_small<4, true>(p, epi, stream);
}

int gemm_bf16(const GemmArgs& p, int epi, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return -1;
  if ((p.lda % 8) || (p.ldw % 8)) return -2;
  if (epi == EPI_RESID_RELU && (!p.C2 || p.K % BK)) return -1;
  if (p.head_dim && (epi != EPI_BF16 || p.head_dim % 8 || p.N % p.head_dim)) return -1;
  // the fused residual + ReLU epilogue exists in the 128x128 / 64x64 kernel only
  bool big = epi != EPI_NCHW_F32 && epi != EPI_RESID_RELU && p.N >= 256 && p.M >= 256 && (p.N % 4) == 0 && (p.K % B2K) == 0 &&
             (p.ldc % 4) == 0 && !g_gemm_force_small;
  // fewer 256x256 tiles than half the CUs (the detector's late-stage Swin GEMMs): the 128x128 kernel
  // puts 4x as many workgroups on the chip
  if (big && (p.K % BK) == 0 && ((p.M + B2M - 1) / B2M) * ((p.N + B2N - 1) / B2N) < 128) big = false;
  if (big) {
    return gemm256(p, epi, stream);
  }
  if (p.K % BK != 0) {
    // K a multiple of 32 but not 64 (Swin stage-1 proj, K = 96): the 256x256x32 kernel clamps its
    // row loads and masks its stores, so small M / N are fine there
    if (p.K % B2K == 0 && epi != EPI_NCHW_F32 && (p.N % 4) == 0 && (p.ldc % 4) == 0) return gemm256(p, epi, stream);
    return -1;
  }
  return use_tile64(p) ? launch_small<2>(p, epi, stream) : launch_small<4>(p, epi, stream);
}


}  // namespace mq
