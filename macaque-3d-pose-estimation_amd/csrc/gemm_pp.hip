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
//
// The tile geometry is a template (PPShape<WMF, WNF>: MFMA fragments per wave in M and N; phase split,
// DMA issue plan and counted waits derived from it); the epilogue is written for WNF = 4 and the library
// instantiates 256 x 256.  A 192 x 320 shape (6 x 5 fragments per wave, 18 / 12 / 18 / 12 MFMAs per
// phase, DMA plan 3 / 2 / 2 / 1, odd-fragment stores, dwordx4 bias DMA) fills whole CU rounds for fc1 /
// qkv / fc2 / proj but measured 1 % slower end to end in the ViT-H forward
// (profiles/r02s3d_vit_probe_wide_tiles.log); its epilogue branches were removed again.
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

int g_gemm_pingpong = 1;

constexpr int PP_BK = 64, PP_T = 512;
constexpr int PP_STAGE = 64 * 1024;   // one BK slice of the A and W tiles (both shapes: (BM + BN) x 128 B)
constexpr int PP_BIAS = 2 * PP_STAGE; // bias area after the 2-stage ring

// Tile geometry: WMF x WNF MFMA fragments (16 x 16) per wave, 8 waves as 2 (M) x 4 (N).
template <int WMF_, int WNF_>
struct PPShape {
  static constexpr int WMF = WMF_, WNF = WNF_;
  static constexpr int QM = WMF / 2;          // fragments per M half (phases 0,1 | 2,3)
  static constexpr int NA = (WNF + 1) / 2;    // fragments of the first N part (phases 0, 2)
  static constexpr int NB = WNF - NA;         // second N part (phases 1, 3)
  static constexpr int BM = 2 * 16 * WMF, BN = 4 * 16 * WNF;
  static constexpr int OPA = BM * PP_BK * 2;  // A slice bytes; the W slice follows it
  // bias slice per wave: 16 WNF = 64 floats, one dword LDS-DMA (256 B)
  static_assert(WNF == 4, "the epilogue's bias read, paired stores and bias DMA are written for 4 fragments");
  static constexpr int BIAS_SLOT = 256;
  static constexpr int LDS = PP_BIAS + 8 * BIAS_SLOT;
  // DMA groups (8 rows x 128 B = one 1-KiB wave instruction) in first-read order: P0 A, P0 W, P1 W, P2 A
  static constexpr int GA0 = BM / 16;         // P0 A groups (M half 0 of both wave groups)
  static constexpr int GW0 = 4 * 2 * NA;      // P0 W groups (N part A of the 4 wave columns)
  static constexpr int GW1 = 4 * 2 * NB;      // P1 W groups
  static constexpr int GA2 = BM / 16;         // P2 A groups
  static_assert(GA0 + GW0 + GW1 + GA2 == 64, "a stage is 64 DMA groups");
  // per-wave DMA instructions per phase
  static constexpr int C0 = WNF == 4 ? 2 : 3, C1 = 2, C2 = 2, C3 = WNF == 4 ? 2 : 1;
  static_assert(C0 + C1 + C2 + C3 == 8, "8 DMA slots per wave");
  static_assert(8 * (C0 + C1) >= GA0 + GW0, "P0 must be issued in phases 0-1");
  static_assert(8 * (C0 + C1 + C2) >= GA0 + GW0 + GW1, "P1 must be issued by phase 2");
  // counted waits (vector memory ops younger than the ones retired): see the kernel
  static constexpr int N0 = C3 + C0 + 1, N1 = C0 + 1 + C1, N3 = C2 + C3;
  // epilogue stores per wave of a full tile (bf16: pairs of fragments as 16-B rows + an 8-B tail)
  static constexpr int STORES_BF16 = WMF * (WNF / 2);
  static constexpr int STORES_F32 = WMF * WNF;
};
using Shape256 = PPShape<8, 4>;

namespace {

__device__ __forceinline__ int pp_swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ bf16x8 pp_frag(const char* op, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(op + row * 128 + ((chunk ^ pp_swz(row)) << 4));
}

// -DPP_DIAG=<bits> diagnostic builds (tools/gemm_diag.py; never the shipped library, results are garbage): take
// parts of the kernel out to see what they cost.  1: no counted vmcnt waits in the K-loop; 2: no LDS-DMA at all (nor
// its waits); 4: no barriers (and no stagger: the wave groups run free); 8: the fragment reads of the first K-step
// only (later K-steps reuse the registers); 16: no epilogue; 32: the bf16 epilogues without their stores; 64: the bf16
// epilogues store every tile into C's first 256 x 256 block; 128: both wave groups run their epilogues in the same
// barrier interval (removed again, in the git history: rejected, r06r); 256: the bf16
// epilogues store each wave's 16 KiB lane-linearly into a fixed region of its own (256 blocks x 128 KiB: only for
// outputs of at least 32 MiB, e.g. fc1, qkv, deconv 1); 512: the bf16 epilogues run all
// their arithmetic first, then issue their 16 stores back to back; 4096: wave group 1 at priority 1 for the whole
// kernel instead of priority 1 around every MFMA segment; 8192: no priority changes; 32768: no lgkmcnt(0) after the
// barrier that opens an MFMA segment (the compiler's own counted waits before each MFMA's operands instead).
#ifndef PP_DIAG
#define PP_DIAG 0
#endif
#define PP_LOOP_WAIT(n)                                   \
  do {                                                    \
    if constexpr (!(PP_DIAG & 3)) pp_wait_vm<n>(); \
  } while (0)

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

template <class S>
__device__ __forceinline__ void pp_tile_coords(int wid, int tiles_m, int tiles_n, int& m0, int& n0) {
#ifndef PP_GROUP_M
#define PP_GROUP_M 8  // (diagnostic builds may set it: tools/gemm_diag.py --group-m)
#endif
  constexpr int GROUP_M = PP_GROUP_M;
  const int per_group = GROUP_M * tiles_n;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_g = wid - grp * per_group;
  m0 = (first_m + in_g % gsize) * S::BM;
  n0 = (in_g / gsize) * S::BN;
}

// DMA group k (0..63, first-read order) -> operand (W?) and first tile row of its 8 rows
template <class S>
__device__ __forceinline__ int pp_group_row(int k, bool& is_w) {
  constexpr int HALF = S::BM / 2;      // rows per wave group
  constexpr int QR = 16 * S::QM;       // rows per M half
  constexpr int WCOL = 16 * S::WNF;    // W rows per wave column
  if (k < S::GA0) {
    is_w = false;
    const int gq = QR / 8;             // groups per (wave group, M half)
    return (k / gq) * HALF + (k % gq) * 8;
  }
  k -= S::GA0;
  if (k < S::GW0) {
    is_w = true;
    const int gq = 2 * S::NA;
    return (k / gq) * WCOL + (k % gq) * 8;
  }
  k -= S::GW0;
  if (k < S::GW1) {
    is_w = true;
    const int gq = 2 * S::NB;
    return (k / gq) * WCOL + 16 * S::NA + (k % gq) * 8;
  }
  k -= S::GW1;
  is_w = false;
  const int gq = QR / 8;
  return (k / gq) * HALF + QR + (k % gq) * 8;
}
// slot i (0..7) of wave w -> its group: phase p's slots of all waves take groups 8 (C0 + .. + C_{p-1})
// + w C_p + (slot within the phase)
template <class S>
__device__ __forceinline__ int pp_slot_group(int w, int i) {
  if (i < S::C0) return w * S::C0 + i;
  i -= S::C0;
  if (i < S::C1) return 8 * S::C0 + w * S::C1 + i;
  i -= S::C1;
  if (i < S::C2) return 8 * (S::C0 + S::C1) + w * S::C2 + i;
  i -= S::C2;
  return 8 * (S::C0 + S::C1 + S::C2) + w * S::C3 + i;
}

// Epilogue of one wave's (16 WMF) x (16 WNF) block: acc[i][j] holds C[m0 + wm*BM/2 + i*16 + (l & 15)]
// [n0 + wn*16*WNF + j*16 + 4*(l >> 4) + e].  Zeroes the accumulators for the next tile.
//
// Sub-pixel deconvolution (DECONV): GEMM row m = input pixel (img, y, x) and column n = class (py, px)
// x C_out + co store to output pixel (img, 2y + py, 2x + px), channel co, of the NHWC (2H, 2W) image.
template <int EPI, class S, bool DECONV = false>
__device__ __forceinline__ void pp_epilogue(const GemmArgs& p, f32x4 (&acc)[S::WMF][S::WNF], const float* bias_lds,
                                            int m0, int n0, int wm, int wn, int lane) {
  constexpr int WMF = S::WMF, WNF = S::WNF;
  const int mm = lane & 15;
  const int nn = 4 * (lane >> 4);
  const int mb = m0 + wm * (S::BM / 2), nb = n0 + wn * 16 * WNF;
  // The bias slice was LDS-DMA'd and retired by this wave's own counted vmcnt.  Read it in inline asm:
  // a plain LDS read here makes the compiler wait vmcnt(0) for every DMA in flight (it cannot tell the
  // bias slot from the stage buffers the in-flight DMAs write).
  f32x4 bv[WNF];
  {
    const unsigned addr = (unsigned)(uintptr_t)MQ_LDS_LOCAL(bias_lds + nn);
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:64\n\tds_read_b128 %2, %4 offset:128\n\t"
        "ds_read_b128 %3, %4 offset:192\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3])
        : "v"(addr)
        : "memory");
  }
  float4 bias[WNF];
#pragma unroll
  for (int j = 0; j < WNF; ++j) bias[j] = make_float4(bv[j][0], bv[j][1], bv[j][2], bv[j][3]);
  const bool full = (m0 + S::BM <= p.M) && (n0 + S::BN <= p.N);
  // C row of GEMM row m, column offset of the tile
  int dc_cls = 0, dc_col = 0;
  if constexpr (DECONV) {
    const int cout = p.N >> 2;
    dc_cls = n0 / cout;
    dc_col = dc_cls * cout;
  }
  auto crow = [&](int m) -> size_t {
    if constexpr (DECONV) {
      const int hw = p.conv_h * p.conv_w;
      const int img = m / hw, rem = m - img * hw;
      const int y = rem / p.conv_w, x = rem - y * p.conv_w;
      return ((size_t)img * 2 * p.conv_h + 2 * y + (dc_cls >> 1)) * (2 * p.conv_w) + 2 * x + (dc_cls & 1);
    } else {
      return (size_t)m;
    }
  };
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
    auto act = [&](int i, int j, float (&v)[4]) {
      v[0] = acc[i][j][0] + bias[j].x;
      v[1] = acc[i][j][1] + bias[j].y;
      v[2] = acc[i][j][2] + bias[j].z;
      v[3] = acc[i][j][3] + bias[j].w;
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
    };
    // pair fragments (j, j+1): v_permlane16_swap gives every lane 8 consecutive columns -> one
    // 16-byte store per lane per pair; an odd last fragment stores its 4 columns (8 B) per lane
    const bool odd = (lane >> 4) & 1;
    const int nbase = nn - (odd ? 4 : 0);
#if PP_DIAG & 512  // all arithmetic first, then the 16 stores back to back
    uint4 ov[WMF][WNF / 2];
#endif
#pragma unroll
    for (int i = 0; i < WMF; ++i) {
      const int m = mb + i * 16 + mm;
      bf16_t* crow_p = (bf16_t*)p.C + crow(m < p.M ? m : 0) * p.ldc - dc_col;
#pragma unroll
      for (int jp = 0; jp + 1 < WNF; jp += 2) {
        unsigned pk[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float v[4];
          act(i, jp + h, v);
          pk[h][0] = pack_bf16x2(v[0], v[1]);
          pk[h][1] = pack_bf16x2(v[2], v[3]);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
        // even lanes: [own tile j | neighbour's tile j]; odd: [neighbour's j+1 | own j+1]
        const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        const int n = nb + (jp + (odd ? 1 : 0)) * 16 + nbase;
#if PP_DIAG & 32  // the epilogue's arithmetic without its stores
        asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
#elif PP_DIAG & 256  // each wave stores its 16 x 1 KiB into a fixed region of its own, lane-linear (whole lines)
        *reinterpret_cast<uint4*>((bf16_t*)p.C + ((size_t)(blockIdx.x * 8 + (threadIdx.x >> 6)) * 16 + i * 2 + (jp >> 1)) * 512 +
                                  lane * 8) = o;
#elif PP_DIAG & 64  // every tile stores into the first 256 x 256 of C (L2-resident lines)
        *reinterpret_cast<uint4*>((bf16_t*)p.C + (size_t)(m & 255) * p.ldc + (n & 255)) = o;
#elif PP_DIAG & 512
        (void)crow_p;
        ov[i][jp >> 1] = o;
#else
        if (full || (m < p.M && n < p.N))
          *reinterpret_cast<uint4*>(EPI == EPI_BF16 && p.head_dim ? gemm_out_bf16(p, m, n) : crow_p + n) = o;
#endif
      }
    }
#if PP_DIAG & 512
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < WMF; ++i) {
      const int m = mb + i * 16 + mm;
      bf16_t* crow_p = (bf16_t*)p.C + crow(m < p.M ? m : 0) * p.ldc - dc_col;
#pragma unroll
      for (int jp = 0; jp + 1 < WNF; jp += 2) {
        const int n = nb + (jp + (odd ? 1 : 0)) * 16 + nbase;
        if (full || (m < p.M && n < p.N))
          *reinterpret_cast<uint4*>(EPI == EPI_BF16 && p.head_dim ? gemm_out_bf16(p, m, n) : crow_p + n) = ov[i][jp >> 1];
      }
    }
#endif
    return;
  }
  if constexpr (EPI == EPI_RESID_F32) {
    if (full) {
      // RG fragment rows (RG x WNF independent 16-B loads) in flight per round trip: the A/W
      // fragment registers are dead here and hold them
      constexpr int RG = 4;
      static_assert(WMF % RG == 0, "row groups");
#pragma unroll
      for (int i0 = 0; i0 < WMF; i0 += RG) {
        float4 x[RG][WNF];
#pragma unroll
        for (int c = 0; c < RG; ++c) {
          const int m = mb + (i0 + c) * 16 + mm;
#pragma unroll
          for (int j = 0; j < WNF; ++j)
            x[c][j] = *reinterpret_cast<const float4*>((const float*)p.C + (size_t)m * p.ldc + nb + j * 16 + nn);
        }
#pragma unroll
        for (int c = 0; c < RG; ++c) {
          const int i = i0 + c;
          const int m = mb + i * 16 + mm;
#pragma unroll
          for (int j = 0; j < WNF; ++j) {
            float4 o = x[c][j];
            o.x += acc[i][j][0] + bias[j].x;
            o.y += acc[i][j][1] + bias[j].y;
            o.z += acc[i][j][2] + bias[j].z;
            o.w += acc[i][j][3] + bias[j].w;
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<float4*>((float*)p.C + (size_t)m * p.ldc + nb + j * 16 + nn) = o;
          }
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < WMF; ++i) {
    const int m = mb + i * 16 + mm;
#pragma unroll
    for (int j = 0; j < WNF; ++j) {
      const int n = nb + j * 16 + nn;
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

// A-operand modes of the kernel
enum PPMode { PP_GEMM = 0, PP_CONV3 = 1, PP_DECONV = 2 };

template <int EPI, int MODE, int WMF_, int WNF_>
__global__ __launch_bounds__(PP_T, 2) void gemm_pp_kernel(GemmArgs p, int tiles_m, int tiles_n) {
  using S = PPShape<WMF_, WNF_>;
  constexpr bool CONV = MODE != PP_GEMM;
  static_assert(!CONV || S::WNF == 4, "implicit convolution: 256 x 256 tiles only");
  static_assert(MODE != PP_DECONV || EPI == EPI_RELU_BF16 || EPI == EPI_BF16, "deconvolution: bf16 NHWC output");
  constexpr int WMF = S::WMF, WNF = S::WNF, QM = S::QM, NA = S::NA, NB = S::NB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm = wave >> 2, wn = wave & 3;
  const int frow = lane & 15;
  const int fk = lane >> 4;
  const int arow = wm * (S::BM / 2);   // this wave's first A row
  const int wcol = wn * 16 * WNF;      // this wave's first W row (output column)

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

  // this wave's 8 DMA slots: operand and first row of each (wave-uniform)
  int grow[8];
  bool gw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) grow[i] = pp_group_row<S>(pp_slot_group<S>(wave, i), gw[i]);

  // DMA issue cursor: (tile, k) of the next stage to load and this lane's source offsets for
  // that tile.  Past the end it stays on the last stage (re-loaded into the idle buffer), which
  // keeps every wait count uniform.
  int iss_t = 0, iss_k = 0;
  unsigned voff[8];
  // implicit convolution: per A slot the output pixel's (y, x) (packed y << 16 | x); voff then holds the
  // element offset of the tap-centre row + this lane's chunk, and the tap shift is added at issue time
  unsigned cyx[8];
  // sub-pixel deconvolution: output parity class (py, px) of the issue tile (N = 4 classes x C_out)
  int iss_py = 0, iss_px = 0;
  auto set_tile_ptrs = [&](int ti) {
    int m0, n0;
    pp_tile_coords<S>(lo + xb + ti * nbx, tiles_m, tiles_n, m0, n0);
    if constexpr (MODE == PP_DECONV) {
      const int cls = n0 / (p.N >> 2);
      iss_py = cls >> 1;
      iss_px = cls & 1;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = grow[i] + (lane >> 3);
      const int chunk = (lane & 7) ^ pp_swz(row);
      if (gw[i]) {
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
  // per slot: its buffer resource and LDS offset, resolved once (no selects in the K-loop)
  __amdgpu_buffer_rsrc_t srs[8];
  int sdst[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    srs[i] = gw[i] ? rsW : rsA;
    sdst[i] = (gw[i] ? S::OPA : 0) + grow[i] * 128;
  }
  auto issue = [&](int i, int slot) {
    if constexpr ((PP_DIAG & 2) != 0) return;
    char* dst = smem + slot * PP_STAGE + sdst[i];
    if (CONV && !gw[i]) {
      // K-step iss_k = tap * (C / 64) + c64: the tap's shifted pixel, channels 64 c64 .. + 63; a pixel
      // outside the image gets an offset past the buffer end, which the DMA turns into zeros (padding).
      // 3x3: tap = (ky, kx), shift (ky - 1, kx - 1).  Sub-pixel deconvolution: tap = (a, b) of the
      // class's 2 x 2 kernel taps, input shift (py - a, px - b) (see deconv_subpixel_pack_kernel).
      const int kpt = p.conv_c >> 6;
      const int tap = iss_k / kpt;
      int dy, dx;
      if constexpr (MODE == PP_DECONV) {
        dy = iss_py - (tap >> 1);
        dx = iss_px - (tap & 1);
      } else {
        dy = tap / 3 - 1;
        dx = tap - (tap / 3) * 3 - 1;
      }
      const int y = (int)(cyx[i] >> 16) + dy, x = (int)(cyx[i] & 0xffffu) + dx;
      const bool inside = (unsigned)y < (unsigned)p.conv_h && (unsigned)x < (unsigned)p.conv_w;
      const unsigned off = (unsigned)((int)voff[i] + (dy * p.conv_w + dx) * p.conv_c + (iss_k - tap * kpt) * 64);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, MQ_LDS_LOCAL(dst), 16, inside ? off * 2 : 0x80000000u, 0, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(srs[i], MQ_LDS_LOCAL(dst), 16, voff[i],
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

  // compute cursor: tile index, K-step in it, its origin, this wave's bias DMA offset (one column per lane)
  int ct = 0, kt = 0, cm0 = 0, cn0 = 0;
  pp_tile_coords<S>(lo + xb, tiles_m, tiles_n, cm0, cn0);
  char* bias_lds = smem + PP_BIAS + wave * S::BIAS_SLOT;
  auto bias_offset = [&](int n0) -> unsigned { return (unsigned)((n0 + wcol + lane) * 4); };
  unsigned bias_off = bias_offset(cn0);
  auto issue_bias = [&]() {
    if constexpr ((PP_DIAG & 2) != 0) return;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, MQ_LDS_LOCAL(bias_lds), 4, bias_off, 0, 0, 0);
  };

  f32x4 acc[WMF][WNF];
#pragma unroll
  for (int i = 0; i < WMF; ++i)
#pragma unroll
    for (int j = 0; j < WNF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[QM][2], b0[NA][2], b1[NB][2];

  auto mfma_quadrant = [&](int qm, auto& bb, int jbase, auto nj) {
    if constexpr (!(PP_DIAG & (4096 | 8192))) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < QM; ++i)
#pragma unroll
        for (int j = 0; j < decltype(nj)::value; ++j)
          acc[qm * QM + i][jbase + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j][kk], a[i][kk], acc[qm * QM + i][jbase + j], 0, 0, 0);
    if constexpr (!(PP_DIAG & (4096 | 8192))) __builtin_amdgcn_s_setprio(0);
  };
  using NAc = std::integral_constant<int, NA>;
  using NBc = std::integral_constant<int, NB>;
  // barrier that opens an MFMA segment: the segment's fragment reads are complete
#ifdef PP_STAMP
  // diagnostic build only (tools/gemm_stamp.py; never the shipped library): s_memtime before and after every barrier of
  // K-steps PP_STAMP_G0..+3 (default 4-7) of block 0, lane 0 of waves 0 and 4 (one wave of each group, the same SIMD), into p.aux
#ifndef PP_STAMP_G0
#define PP_STAMP_G0 4  // first stamped K-step (of the block's walk; 18: across fc1's first tile boundary)
#endif
  int stamp_n = 0, stamp_g = 0;
  auto stamp = [&]() {
    if (blockIdx.x == 0 && lane == 0 && (wave == 0 || wave == 4) && stamp_g >= PP_STAMP_G0 && stamp_g < PP_STAMP_G0 + 4 &&
        p.aux && stamp_n < 64)
      reinterpret_cast<unsigned long long*>(const_cast<float*>(p.aux))[(wave >> 2) * 64 + stamp_n] =
          __builtin_amdgcn_s_memtime();
    ++stamp_n;
  };
  auto bar = [&]() {  // arrival, then release
    stamp();
    pp_barrier();
    stamp();
  };
#else
  auto bar = [&]() {
    if constexpr (!(PP_DIAG & 4)) pp_barrier();
  };
#endif
  auto open_mfma = [&]() {
    bar();
    if constexpr (!(PP_DIAG & 32768)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // prologue: stage 0 into buffer 0; P0 (the slots of phases 0-1) must land before the first reads
#pragma unroll
  for (int i = 0; i < 8; ++i) issue(i, 0);
  advance();
  pp_wait_vm<S::N3>();
  pp_barrier();
  if (!(PP_DIAG & 4) && wm == 1) pp_barrier();  // stagger: group 1 runs one barrier behind group 0
  if constexpr ((PP_DIAG & 4096) != 0)  // static priority for the second-dispatched group instead of per-segment flips
    if (wm == 1) __builtin_amdgcn_s_setprio(1);

  // >= this many epilogue stores of a full tile are younger than the DMA the next two waits retire
  constexpr int EPI_OPS =
      (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) ? S::STORES_BF16 : S::STORES_F32;
  bool stores_pending = false;
  auto epilogue = [&](const char* bl, int m0, int n0) {
    if constexpr (!(PP_DIAG & 16))
      pp_epilogue<EPI, S, MODE == PP_DECONV>(p, acc, reinterpret_cast<const float*>(bl), m0, n0, wm, wn, lane);
  };
  auto tile_full = [&](int m0, int n0) { return !(PP_DIAG & 48) && (m0 + S::BM <= p.M) && (n0 + S::BN <= p.N); };
  for (int g = 0; g < total; ++g) {
#ifdef PP_STAMP
    stamp_g = g;
    if (g == PP_STAMP_G0) stamp_n = 0;
#endif
    const int slot = g & 1;
    const char* As = smem + slot * PP_STAGE;
    const char* Ws = As + S::OPA;
    // ---- phase 0: quadrant (M half 0, N part A)
    auto reads0 = [&]() {
#pragma unroll
      for (int kk = 0; kk < 2 && (!(PP_DIAG & 8) || g == 0); ++kk) {
#pragma unroll
        for (int j = 0; j < NA; ++j)
          b0[j][kk] = pp_frag(Ws, wcol + j * 16 + frow, kk * 4 + fk);
#pragma unroll
        for (int i = 0; i < QM; ++i)
          a[i][kk] = pp_frag(As, arow + i * 16 + frow, kk * 4 + fk);
      }
    };
    reads0();
#pragma unroll
    for (int i = 0; i < S::C0; ++i) issue(i, slot ^ 1);
    issue_bias();
    // retires the DMAs of the previous K-step's phase 2 (younger: its phase 3, this phase + bias)
    if (stores_pending)
      PP_LOOP_WAIT(S::N0 + EPI_OPS);
    else
      PP_LOOP_WAIT(S::N0);
    open_mfma();
    mfma_quadrant(0, b0, 0, NAc{});
    bar();
    // ---- phase 1: quadrant (M half 0, N part B)
#pragma unroll
    for (int kk = 0; kk < 2 && (!(PP_DIAG & 8) || g == 0); ++kk)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        b1[j][kk] = pp_frag(Ws, wcol + 16 * NA + j * 16 + frow, kk * 4 + fk);
#pragma unroll
    for (int i = S::C0; i < S::C0 + S::C1; ++i) issue(i, slot ^ 1);
    // retires the previous K-step's phase-3 DMAs (younger: phase 0 + bias, this phase)
    if (stores_pending)
      PP_LOOP_WAIT(S::N1 + EPI_OPS);
    else
      PP_LOOP_WAIT(S::N1);
    stores_pending = false;
    open_mfma();
    mfma_quadrant(0, b1, NA, NBc{});
    bar();
    // ---- phase 2: quadrant (M half 1, N part A)
#pragma unroll
    for (int kk = 0; kk < 2 && (!(PP_DIAG & 8) || g == 0); ++kk)
#pragma unroll
      for (int i = 0; i < QM; ++i)
        a[i][kk] = pp_frag(As, arow + 16 * QM + i * 16 + frow, kk * 4 + fk);
#pragma unroll
    for (int i = S::C0 + S::C1; i < S::C0 + S::C1 + S::C2; ++i) issue(i, slot ^ 1);
    open_mfma();
    mfma_quadrant(1, b0, 0, NAc{});
    bar();
    // ---- phase 3: quadrant (M half 1, N part B)
#pragma unroll
    for (int i = S::C0 + S::C1 + S::C2; i < 8; ++i) issue(i, slot ^ 1);
    advance();
    PP_LOOP_WAIT(S::N3);  // phases 0-1 of this K-step (P0 of stage g+1) and the bias
    open_mfma();
    mfma_quadrant(1, b1, NA, NBc{});
    bar();
    if (++kt == nk) {
      epilogue(bias_lds, cm0, cn0);
      stores_pending = tile_full(cm0, cn0);
      kt = 0;
      ++ct;
      if (ct < my_tiles) {
        pp_tile_coords<S>(lo + xb + ct * nbx, tiles_m, tiles_n, cm0, cn0);
        bias_off = bias_offset(cn0);
      }
    }
  }
  if constexpr ((PP_DIAG & 16) != 0) {  // keep the accumulators live (a store the host never asks for)
    if (p.M < 0)
#pragma unroll
      for (int i = 0; i < WMF; ++i)
#pragma unroll
        for (int j = 0; j < WNF; ++j) reinterpret_cast<f32x4*>(p.C)[(i * WNF + j) * 512 + threadIdx.x] = acc[i][j];
  }
  if (!(PP_DIAG & 4) && wm == 0) pp_barrier();  // balance the stagger
  pp_wait_vm<0>();            // no DMA may outlive the block
}

template <int EPI, int MODE, class S>
void launch_pp(dim3 grid, hipStream_t stream, const GemmArgs& p, int tiles_m, int tiles_n) {
  static std::atomic<unsigned> attr{0};
  if (first_on_device(attr))
    (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, MODE, S::WMF, S::WNF>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS);
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, MODE, S::WMF, S::WNF>), grid, dim3(PP_T), S::LDS, stream, p, tiles_m, tiles_n);
}

template <class S>
int tiles_of(const GemmArgs& p, int& tm, int& tn) {
  tm = (p.M + S::BM - 1) / S::BM;
  tn = (p.N + S::BN - 1) / S::BN;
  return tm * tn;
}

template <class S>
int launch_shape(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  int tiles_m, tiles_n;
  const int tiles = tiles_of<S>(p, tiles_m, tiles_n);
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_GELU_BF16: launch_pp<EPI_GELU_BF16, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_pp<EPI_RELU_BF16, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RESID_F32: launch_pp<EPI_RESID_F32, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_POS_F32: launch_pp<EPI_POS_F32, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_F32: launch_pp<EPI_F32, PP_GEMM, S>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
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
  int tiles_m, tiles_n;
  const int tiles = tiles_of<Shape256>(p, tiles_m, tiles_n);
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16, PP_CONV3, Shape256>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_pp<EPI_RELU_BF16, PP_CONV3, Shape256>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_F32: launch_pp<EPI_F32, PP_CONV3, Shape256>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// ConvTranspose2d(k4, s2, p1) as four sub-pixel 2x2 convolutions in ONE launch: output parity class
// (py, px) = N tile / C_out, its 2 x 2 taps gathered like the 3x3 implicit convolution, the result
// stored straight into the NHWC (2H, 2W) image (no 16-tap column buffer, no col2im pass).
int gemm_pingpong_deconv(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  const int cout = p.N / 4;
  if (p.conv_c <= 0 || p.conv_c % PP_BK || p.K != 4 * p.conv_c || p.lda != p.conv_c || p.N % 4 ||
      cout % Shape256::BN || p.ldw != p.K || p.ldc != cout || p.conv_h <= 0 || p.conv_w <= 0 ||
      p.M % (p.conv_h * p.conv_w) || p.conv_w >= 65536 || p.conv_h >= 65536 ||
      (size_t)p.M * p.lda * 2 >= (1ull << 31) || (size_t)p.N * p.ldw * 2 >= (1ull << 31))
    return -1;
  int tiles_m, tiles_n;
  const int tiles = tiles_of<Shape256>(p, tiles_m, tiles_n);
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_pp<EPI_BF16, PP_DECONV, Shape256>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_pp<EPI_RELU_BF16, PP_DECONV, Shape256>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

// Routing: every 256x256 GEMM with K % 64 == 0, except the f32 residual read-modify-write at short
// K (proj, K = 1280: one tile per CU, 20 K-steps), which goes to the interleaved kernel: it measured
// 8 % faster than the ping-pong there (755 vs 692 TFLOP/s; the residual loads stall both wave
// groups at the tile end).  At K = 5120 (fc2) the ping-pong wins.
bool gemm_pingpong_fits(const GemmArgs& p, int epi, int num_cus) {
  (void)num_cus;
  return g_gemm_pingpong && epi != EPI_NCHW_F32 && !(epi == EPI_RESID_F32 && p.K < 2048) && p.K > 0 &&
         p.K % PP_BK == 0 && (size_t)p.M * p.lda * 2 < (1ull << 31) && (size_t)p.N * p.ldw * 2 < (1ull << 31);
}

int gemm_pingpong(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  return launch_shape<Shape256>(p, epi, num_cus, stream);
}

}  // namespace mq
