// Ping-pong bf16 MFMA GEMM for gfx950: C[M,N] = A[M,K] * W[N,K]^T with the fused epilogues of
// gemm_bf16.hip (kernels.hpp GemmEpilogue), for the ViT-H layer GEMMs (qkv, proj, fc1, fc2, deconv).
//
// Tile 256x256, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 block =
// 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (swapped product D = W * A^T, so a lane holds 4
// consecutive output columns of one row).  Persistent: one block per CU walks a contiguous,
// XCD-local range of tiles in grouped order (8 M-tiles per group).
//
// The two wave groups (wm = 0: waves 0-3, wm = 1: waves 4-7; one wave of each on every SIMD) run
// ONE BARRIER APART.  In every barrier-delimited segment one group issues its LDS fragment reads
// and LDS-DMA while the other group runs 16 MFMAs on the same SIMDs, so each SIMD's matrix pipe
// alternates between its two waves instead of both waves waiting on the same reads.  A K-step is
// four phases, one 64x32 quadrant of the wave block each:
//
//   phase  quadrant (m,n)  fragment reads (ds_read_b128)  DMA issued for stage g+1   vmcnt wait retires
//     0        (0,0)       A rows 0-63, W cols 0-31        P0 slots 0,1 + bias        P1(g)
//     1        (0,1)       W cols 32-63                    P0 slots 2,3               P2(g)
//     2        (1,0)       A rows 64-127                   P1 slots 4,5               -
//     3        (1,1)       -                               P2 slots 6,7               P0(g+1), bias
//
// A stage (one BK = 64 slice of the A and W tiles, 64 KiB) is split by the phase that first reads
// it: P0 = A rows {0-63, 128-191} + W rows {0-31, 64-95, 128-159, 192-223}, P1 = the other W
// rows, P2 = the other A rows.  Each wait sits before the barrier one phase ahead of the reads it
// retires; with the groups one barrier apart that barrier is the last one both groups pass before
// either reads.  Two stages (2 x 64 KiB) are enough: a stage buffer is refilled only after its
// last read (phase 2 of the previous K-step).  LDS image: 128-B rows, 16-B chunk c of row r at
// slot c ^ ((r >> 1) & 7) (swizzle applied through the DMA source address; ds_read_b128 of the
// fragment pattern is conflict-free under it).
//
// The bias slice of the current tile (64 floats per wave) also arrives by LDS-DMA (dword form,
// one wave-instruction), once per K-step, so the epilogue issues no global load of its own except
// the residual / pos_embed reads of the f32 epilogues: an ordinary load in the K-loop would make
// the compiler drain every DMA in flight.
//
// Accumulation order per output element is the one of gemm256_kernel (K in ascending 32-deep
// MFMA steps, then + bias, then the epilogue op), so both kernels give bit-identical results.
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

int g_gemm_pingpong = 1;

namespace {

constexpr int PP_BM = 256, PP_BN = 256, PP_BK = 64, PP_T = 512;
constexpr int PP_OP = PP_BM * PP_BK * 2;  // 32 KiB: one operand slice of a stage
constexpr int PP_STAGE = 2 * PP_OP;       // 64 KiB
constexpr int PP_BIAS = 2 * PP_STAGE;     // bias area: 8 waves x 256 B
constexpr int PP_LDS = PP_BIAS + 8 * 256;

__device__ __forceinline__ int pp_swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 pp_frag(const char* op, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(op + row * 128 + ((chunk ^ pp_swz(row)) << 4));
}

template <int N_IN_FLIGHT>
__device__ __forceinline__ void pp_wait_vm() {
  static_assert(N_IN_FLIGHT >= 0 && N_IN_FLIGHT < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_IN_FLIGHT) : "memory");
}

// raw s_barrier (no vmcnt(0) drain, unlike __syncthreads) that the compiler may not move
// memory operations across
__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void pp_tile_coords(int wid, int tiles_m, int tiles_n, int& m0, int& n0) {
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tiles_n;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_g = wid - grp * per_group;
  m0 = (first_m + in_g % gsize) * PP_BM;
  n0 = (in_g / gsize) * PP_BN;
}

// DMA slot i (0..7) of wave w moves the 8-row group starting at this row of its operand.
// Slots 0,1: P0 A rows; 2,3: P0 W rows; 4,5: P1 W rows; 6,7: P2 A rows (16 groups each).
__device__ __forceinline__ int pp_group_row(int w, int i) {
  const int g = w * 2 + (i & 1);
  switch (i >> 1) {
    case 0: return g < 8 ? g * 8 : 128 + (g - 8) * 8;
    case 1: return (g >> 2) * 64 + (g & 3) * 8;
    case 2: return (g >> 2) * 64 + 32 + (g & 3) * 8;
    default: return g < 8 ? 64 + g * 8 : 192 + (g - 8) * 8;
  }
}
__device__ __forceinline__ constexpr bool pp_slot_is_w(int i) { return (i >> 1) == 1 || (i >> 1) == 2; }

// Epilogue of one wave's 128x64 block: acc[i][j] holds C[m0 + wm*128 + i*16 + (l & 15)]
// [n0 + wn*64 + j*16 + 4*(l >> 4) + e].  Zeroes the accumulators for the next tile.
template <int EPI>
__device__ __forceinline__ void pp_epilogue(const GemmArgs& p, f32x4 (&acc)[8][4], const float* bias_lds, int m0,
                                            int n0, int wm, int wn, int lane) {
  const int mm = lane & 15;
  const int nn = 4 * (lane >> 4);
  // The bias slice was LDS-DMA'd and retired by this wave's own counted vmcnt.  Read it in inline asm:
  // a plain LDS read here makes the compiler wait vmcnt(0) for every DMA in flight (it cannot tell the
  // bias slot from the stage buffers the in-flight DMAs write).
  f32x4 bv[4];
  {
    const unsigned addr = (unsigned)(uintptr_t)MQ_LDS_LOCAL(bias_lds + nn);
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
        "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
        : "v"(addr)
        : "memory");
  }
  float4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = make_float4(bv[j][0], bv[j][1], bv[j][2], bv[j][3]);
  const bool full = (m0 + PP_BM <= p.M) && (n0 + PP_BN <= p.N);
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
    // pair fragments (j, j+1): v_permlane16_swap gives every lane 8 consecutive columns -> one
    // 16-byte store per lane per pair
    const bool odd = (lane >> 4) & 1;
    const int nbase = nn - (odd ? 4 : 0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + mm;
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
            const f32x2 g0 = gelu_erf2((f32x2){v[0], v[1]}), g1 = gelu_erf2((f32x2){v[2], v[3]});
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
        const int n = n0 + wn * 64 + (jp + (odd ? 1 : 0)) * 16 + nbase;
        if (full || (m < p.M && n < p.N)) *reinterpret_cast<uint4*>((bf16_t*)p.C + (size_t)m * p.ldc + n) = o;
      }
    }
    return;
  }
  if constexpr (EPI == EPI_RESID_F32) {
    if (full) {
      // four fragment rows (16 independent 16-B loads) in flight per round trip: the A/W
      // fragment registers are dead here and hold them
#pragma unroll
      for (int i0 = 0; i0 < 8; i0 += 4) {
        float4 x[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int m = m0 + wm * 128 + (i0 + c) * 16 + mm;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            x[c][j] = *reinterpret_cast<const float4*>((const float*)p.C + (size_t)m * p.ldc + n0 + wn * 64 + j * 16 + nn);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = i0 + c;
          const int m = m0 + wm * 128 + i * 16 + mm;
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
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wm * 128 + i * 16 + mm;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + nn;
      const float v[4] = {acc[i][j][0] + bias[j].x, acc[i][j][1] + bias[j].y, acc[i][j][2] + bias[j].z,
                          acc[i][j][3] + bias[j].w};
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m >= p.M || n >= p.N) continue;
      float4* c = reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + n);
      if constexpr (EPI == EPI_RESID_F32) {
        float4 o = *c;
        o.x += v[0];
        o.y += v[1];
        o.z += v[2];
        o.w += v[3];
        *c = o;
      } else if constexpr (EPI == EPI_POS_F32) {
        const float4 ps = *reinterpret_cast<const float4*>(p.aux + (size_t)(m % p.aux_rows) * p.N + n);
        *c = make_float4(v[0] + ps.x, v[1] + ps.y, v[2] + ps.z, v[3] + ps.w);
      } else {
        *c = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }
}

template <int EPI, bool CONV = false>
__global__ __launch_bounds__(PP_T, 2) void gemm_pp_kernel(GemmArgs p, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave >> 2, wn = wave & 3;
  const int frow = lane & 15;
  const int fk = lane >> 4;

  // this XCD's tiles = a contiguous range; its blocks take them round-robin
  const int nt = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int nbx = (G - xcd + 7) >> 3;
  const int xb = bid >> 3;
  const int q = nt >> 3, r = nt & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int len = q + (xcd < r ? 1 : 0);
  const int my_tiles = xb < len ? (len - xb + nbx - 1) / nbx : 0;
  const int nk = p.K / PP_BK;
  const int total = my_tiles * nk;
  if (total == 0) return;

  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, (int)((size_t)p.M * p.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, (int)((size_t)p.N * p.ldw * 2), 0x00020000);
  // a null bias is an empty buffer: the DMA then reads zeros
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, 0, p.bias ? p.N * 4 : 0, 0x00020000);

  // DMA issue cursor: (tile, k) of the next stage to load and this lane's source offsets for
  // that tile.  Past the end it stays on the last stage (re-loaded into the idle buffer), which
  // keeps every wait count uniform.
  int iss_t = 0, iss_k = 0;
  unsigned voff[8];
  // implicit convolution: per A slot the output pixel's (y, x) (packed y << 16 | x); voff then holds the
  // element offset of the tap-centre row + this lane's chunk, and the tap shift is added at issue time
  unsigned cyx[8];
  auto set_tile_ptrs = [&](int ti) {
    int m0, n0;
    pp_tile_coords(lo + xb + ti * nbx, tiles_m, tiles_n, m0, n0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = pp_group_row(wave, i) + (lane >> 3);
      const int chunk = (lane & 7) ^ pp_swz(row);
      if (pp_slot_is_w(i)) {
        voff[i] = (unsigned)(((size_t)min(n0 + row, p.N - 1) * p.ldw + chunk * 8) * 2);
      } else if constexpr (CONV) {
        const int pix = min(m0 + row, p.M - 1);
        const int hw = p.conv_h * p.conv_w;
        const int rem = pix - (pix / hw) * hw;
        const int y = rem / p.conv_w;
        cyx[i] = ((unsigned)y << 16) | (unsigned)(rem - y * p.conv_w);
        voff[i] = (unsigned)((size_t)pix * p.conv_c + chunk * 8);
      } else {
        voff[i] = (unsigned)(((size_t)min(m0 + row, p.M - 1) * p.lda + chunk * 8) * 2);
      }
    }
  };
  set_tile_ptrs(0);
  auto issue = [&](int i, int slot) {
    char* dst = smem + slot * PP_STAGE + (pp_slot_is_w(i) ? PP_OP : 0) + pp_group_row(wave, i) * 128;
    if (CONV && !pp_slot_is_w(i)) {
      // K-step iss_k = tap * (C / 64) + c64: the tap's shifted pixel, channels 64 c64 .. + 63; a pixel
      // outside the image gets an offset past the buffer end, which the DMA turns into zeros (padding)
      const int kpt = p.conv_c >> 6;
      const int tap = iss_k / kpt;
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
      const int y = (int)(cyx[i] >> 16) + dy, x = (int)(cyx[i] & 0xffffu) + dx;
      const bool inside = (unsigned)y < (unsigned)p.conv_h && (unsigned)x < (unsigned)p.conv_w;
      const unsigned off = (unsigned)((int)voff[i] + (dy * p.conv_w + dx) * p.conv_c + (iss_k - tap * kpt) * 64);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, MQ_LDS_LOCAL(dst), 16, inside ? off * 2 : 0x80000000u, 0, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(pp_slot_is_w(i) ? rsW : rsA, MQ_LDS_LOCAL(dst), 16, voff[i],
                                               iss_k * PP_BK * 2, 0, 0);
    }
  };
  auto advance = [&]() {
    if (iss_k + 1 < nk) {
      ++iss_k;
    } else if (iss_t + 1 < my_tiles) {
      ++iss_t;
      iss_k = 0;
      set_tile_ptrs(iss_t);
    }
  };

  // compute cursor: tile index, K-step in it, its origin, this wave's bias DMA offset
  int ct = 0, kt = 0, cm0 = 0, cn0 = 0;
  pp_tile_coords(lo + xb, tiles_m, tiles_n, cm0, cn0);
  char* bias_lds = smem + PP_BIAS + wave * 256;
  unsigned bias_off = (unsigned)((cn0 + wn * 64 + lane) * 4);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b0[2][2], b1[2][2];

  auto mfma_quadrant = [&](int qm, int qn, bf16x8 (&bb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j][kk], a[i][kk], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // barrier that opens an MFMA segment: the segment's fragment reads are complete
  auto bar = [&]() { pp_barrier(); };
  auto open_mfma = [&]() {
    bar();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // prologue: stage 0 into buffer 0; P0 (the 4 oldest DMAs) must land before the first reads
#pragma unroll
  for (int i = 0; i < 8; ++i) issue(i, 0);
  advance();
  pp_wait_vm<4>();
  pp_barrier();
  if (wm == 1) pp_barrier();  // stagger: group 1 runs one barrier behind group 0

  // >= this many epilogue stores of a full tile are younger than the DMA the next two waits retire
  constexpr int EPI_OPS = (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) ? 16 : 32;
  bool stores_pending = false;
  for (int g = 0; g < total; ++g) {
    const int slot = g & 1;
    const char* As = smem + slot * PP_STAGE;
    const char* Ws = As + PP_OP;
    // ---- phase 0: quadrant (0,0)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b0[j][kk] = pp_frag(Ws, wn * 64 + j * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i][kk] = pp_frag(As, wm * 128 + i * 16 + frow, kk * 4 + fk);
    }
    issue(0, slot ^ 1);
    issue(1, slot ^ 1);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, MQ_LDS_LOCAL(bias_lds), 4, bias_off, 0, 0, 0);
    if (stores_pending)
      pp_wait_vm<5 + EPI_OPS>();
    else
      pp_wait_vm<5>();
    open_mfma();
    mfma_quadrant(0, 0, b0);
    bar();
    // ---- phase 1: quadrant (0,1)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        b1[j][kk] = pp_frag(Ws, wn * 64 + 32 + j * 16 + frow, kk * 4 + fk);
    issue(2, slot ^ 1);
    issue(3, slot ^ 1);
    if (stores_pending)
      pp_wait_vm<5 + EPI_OPS>();
    else
      pp_wait_vm<5>();
    stores_pending = false;
    open_mfma();
    mfma_quadrant(0, 1, b1);
    bar();
    // ---- phase 2: quadrant (1,0)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i][kk] = pp_frag(As, wm * 128 + 64 + i * 16 + frow, kk * 4 + fk);
    issue(4, slot ^ 1);
    issue(5, slot ^ 1);
    open_mfma();
    mfma_quadrant(1, 0, b0);
    bar();
    // ---- phase 3: quadrant (1,1)
    issue(6, slot ^ 1);
    issue(7, slot ^ 1);
    advance();
    pp_wait_vm<4>();
    open_mfma();
    mfma_quadrant(1, 1, b1);
    bar();
    if (++kt == nk) {
      pp_epilogue<EPI>(p, acc, reinterpret_cast<const float*>(bias_lds), cm0, cn0, wm, wn, lane);
      stores_pending = (cm0 + PP_BM <= p.M) && (cn0 + PP_BN <= p.N);
      kt = 0;
      ++ct;
      if (ct < my_tiles) {
        pp_tile_coords(lo + xb + ct * nbx, tiles_m, tiles_n, cm0, cn0);
        bias_off = (unsigned)((cn0 + wn * 64 + lane) * 4);
      }
    }
  }
  if (wm == 0) pp_barrier();  // balance the stagger
  pp_wait_vm<0>();            // no DMA may outlive the block
}

template <int EPI, bool CONV = false>
void launch_pp(dim3 grid, hipStream_t stream, const GemmArgs& p, int tiles_m, int tiles_n) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              PP_LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, CONV>), grid, dim3(PP_T), PP_LDS, stream, p, tiles_m, tiles_n);
}

}  // namespace

// Implicit-GEMM 3x3 convolution: the ping-pong GEMM with the A tile rows of every K-step gathered from
// the tap's shifted input pixels (replaces an im2col buffer of 9x the input: the FPN / RPN convolutions
// of the detector).  Same accumulation order as im2col + GEMM, so both give the same bits.
int gemm_pingpong_conv(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  if (p.conv_c <= 0 || p.conv_c % PP_BK || p.K != 9 * p.conv_c || p.lda != p.conv_c || p.conv_h <= 0 ||
      p.conv_w <= 0 || p.M % (p.conv_h * p.conv_w) || p.conv_w >= 65536 || p.conv_h >= 65536 ||
      (size_t)p.M * p.lda * 2 >= (1ull << 31) || (size_t)p.N * p.ldw * 2 >= (1ull << 31))
    return -1;
  // the epilogue stores 8 bf16 / 4 f32 columns per lane: whole groups only
  if (epi == EPI_F32 ? (p.N % 4 || p.ldc % 4) : (p.N % 8 || p.ldc % 8)) return -2;
  const int tiles_m = (p.M + PP_BM - 1) / PP_BM, tiles_n = (p.N + PP_BN - 1) / PP_BN;
  const int tiles = tiles_m * tiles_n;
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16, true>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_pp<EPI_RELU_BF16, true>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_F32: launch_pp<EPI_F32, true>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Routing: every 256x256 GEMM with K % 64 == 0, except the f32 residual read-modify-write at short
// K (proj, K = 1280: one tile per CU, 20 K-steps), which goes to the interleaved kernel: it measured
// 8 % faster than the ping-pong there (755 vs 692 TFLOP/s; the residual loads stall both wave
// groups at the tile end).  At K = 5120 (fc2) the ping-pong wins.
bool gemm_pingpong_fits(const GemmArgs& p, int epi) {
  return g_gemm_pingpong && epi != EPI_NCHW_F32 && !(epi == EPI_RESID_F32 && p.K < 2048) && p.K > 0 &&
         p.K % PP_BK == 0 && (size_t)p.M * p.lda * 2 < (1ull << 31) && (size_t)p.N * p.ldw * 2 < (1ull << 31);
}

int gemm_pingpong(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  const int tiles_m = (p.M + PP_BM - 1) / PP_BM, tiles_n = (p.N + PP_BN - 1) / PP_BN;
  const int tiles = tiles_m * tiles_n;
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_GELU_BF16: launch_pp<EPI_GELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_pp<EPI_RELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RESID_F32: launch_pp<EPI_RESID_F32>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_POS_F32: launch_pp<EPI_POS_F32>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_F32: launch_pp<EPI_F32>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace mq
