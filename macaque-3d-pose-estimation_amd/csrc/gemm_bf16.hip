// bf16 MFMA GEMM for gfx950 with fused epilogues: C[M,N] = A[M,K] * W[N,K]^T.
//
// Both operands are K-contiguous (torch Linear layout), which is the natural
// operand order of v_mfma_f32_16x16x32_bf16: lane l reads 16 contiguous bytes of
// row (l & 15) at k = 8*(l >> 4) for A and of W-row (l & 15) for B.
//
// Block tile 128x128x64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4 MFMA
// tiles.  Tiles are staged HBM -> LDS with global_load_lds_dwordx4 (no VGPR
// round trip), double buffered: the next K-tile's DMA is issued before the
// current tile's MFMAs.  The LDS image is XOR-swizzled on the SOURCE address
// (16-B chunk c of row r lives at slot c ^ ((r >> 1) & 7)); the ds_read_b128
// fragment reads are bank-conflict free under that swizzle.
//
// Blocks are remapped so that consecutive tiles (sharing A row panels) land on
// the same XCD (bijective remap, MI355X has 8 XCDs with private L2s).
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int GEMM_THREADS = 256;
constexpr int TILE_BYTES = BM * BK * 2;  // 16 KiB per operand tile

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// Issue the DMA of one 128x64 bf16 tile (rows [r0, r0+128) of a K-contiguous
// matrix with leading dimension ld, columns [k0, k0+64)) into LDS.
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ g, int ld, int r0, int rmax, int k0,
                                           char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int rbase = (wave * 4 + i) * 8;
    int row = rbase + (lane >> 3);
    int slot = lane & 7;
    int chunk = slot ^ swz(row);
    int grow = r0 + row;
    grow = grow < rmax ? grow : rmax - 1;
    const bf16_t* src = g + (size_t)grow * ld + k0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(MQ_LDS_GLOBAL(src), MQ_LDS_LOCAL(lds_tile + rbase * 128), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 read_frag(const char* lds_tile, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(lds_tile + row * 128 + ((chunk ^ swz(row)) << 4));
}

template <int EPI>
__global__ __launch_bounds__(GEMM_THREADS, 2) void gemm_bf16_kernel(GemmArgs p) {
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
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tm = wid % tiles_m;
  const int tn = wid / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;


  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  stage_tile(p.A, p.lda, m0, p.M, 0, smem, wave, lane);
  stage_tile(p.W, p.ldw, n0, p.N, 0, smem + TILE_BYTES, wave, lane);
  __syncthreads();

  const int frow = lane & 15;
  const int fk = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * 2 * TILE_BYTES;
      stage_tile(p.A, p.lda, m0, p.M, (t + 1) * BK, nxt, wave, lane);
      stage_tile(p.W, p.ldw, n0, p.N, (t + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
    const char* As = smem + cur * 2 * TILE_BYTES;
    const char* Bs = As + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = read_frag(As, wm * 64 + i * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = read_frag(Bs, wn * 64 + j * 16 + frow, kk * 4 + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue.  C layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
  const int ccol = lane & 15;
  const int crow = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + ccol;
    if (n >= p.N) continue;
    const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 64 + i * 16 + crow + e;
        if (m >= p.M) continue;
        float v = acc[i][j][e] + bias;
        if constexpr (EPI == EPI_BF16) {
          ((bf16_t*)p.C)[(size_t)m * p.ldc + n] = f32_to_bf16(v);
        } else if constexpr (EPI == EPI_GELU_BF16) {
          ((bf16_t*)p.C)[(size_t)m * p.ldc + n] = f32_to_bf16(gelu_erf(v));
        } else if constexpr (EPI == EPI_RESID_F32) {
          float* c = (float*)p.C + (size_t)m * p.ldc + n;
          *c = *c + v;
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

int gemm_bf16(const GemmArgs& p, int epi, hipStream_t stream) {
  if (p.K % BK != 0 || p.M <= 0 || p.N <= 0) return -1;
  if ((p.lda % 8) || (p.ldw % 8)) return -2;
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles), block(GEMM_THREADS);
  const size_t lds = 4 * TILE_BYTES;
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_BF16>, grid, block, lds, stream, p); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_GELU_BF16>, grid, block, lds, stream, p); break;
    case EPI_RESID_F32: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_RESID_F32>, grid, block, lds, stream, p); break;
    case EPI_POS_F32: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_POS_F32>, grid, block, lds, stream, p); break;
    case EPI_F32: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_F32>, grid, block, lds, stream, p); break;
    case EPI_NCHW_F32: hipLaunchKernelGGL(gemm_bf16_kernel<EPI_NCHW_F32>, grid, block, lds, stream, p); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace mq
