// One-wave-per-SIMD bf16 MFMA GEMM for gfx950: C[M,N] = A[M,K] * W[N,K]^T with the bf16 epilogues of
// gemm_pp.hip (bias; bias + GELU; bias + ReLU; head-major qkv store), for the ViT-H layer GEMMs.
//
// Tile 256x256, 256 threads = 4 waves as 2 (M) x 2 (N), ONE wave per SIMD; each wave owns a 128 x 128 block
// = 8 x 8 fragments of v_mfma_f32_16x16x32_bf16 (swapped product D = W * A^T, so a lane holds 4 consecutive
// output columns of one row) in 256 accumulator registers.  Against the ping-pong kernel (8 waves, 128 x 64
// per wave, two waves per SIMD) a wave reads 32 KB of fragments per 128 MFMAs instead of 24 KB per 64, and
// the K loop needs one barrier per 32-deep sub-step instead of eight per 64-deep K-step.
//
// K is walked in 32-deep sub-steps through a 4-slot LDS ring (32 KiB per slot: the A and W tiles' 256 rows
// of 64 B each).  In sub-step s a wave
//   * computes the 64 MFMAs of sub-step s from fragment registers read during sub-step s - 1,
//   * reads the 16 fragments of sub-step s + 1 from slot (s + 1) % 4 into its second register set,
//   * issues the LDS-DMA of sub-step s + 3 into slot (s + 3) % 4 (8 one-KiB pieces per wave: waves 0-1 the
//     A rows, waves 2-3 the W rows),
// interleaved by sched_group_barrier.  At the top of sub-step s one counted vmcnt retires the wave's own DMA
// of slot s + 1 (issued two sub-steps earlier) and one s_barrier publishes everybody's; the same barrier
// proves that every wave has finished reading slot (s - 1) % 4 = (s + 3) % 4 (those fragments fed the
// MFMAs of sub-step s - 1), so the DMA into it may start.  LDS image: 64-B rows, 16-B chunk c of row r at
// c ^ (3 * ((r >> 3) & 1)) (applied through the DMA source address; conflict-free for the fragment reads).
//
// The bias slice of a tile (128 floats per wave) arrives by LDS-DMA right after the previous tile's
// epilogue and is read there in inline asm (a plain LDS read would make the compiler drain every DMA in
// flight).  Accumulation order per output is the ping-pong kernel's (K in ascending 32-deep MFMA steps,
// then + bias, then the epilogue op): both kernels give the same bits.
//
// Persistent: one block per CU walks a contiguous, XCD-local range of tiles in grouped order (8 M-tiles per
// group), as gemm_pp.hip.
#include "common.hpp"
#include "kernels.hpp"

namespace mq {

int g_gemm_w4 = 0;

namespace {

constexpr int W4_T = 256, W4_BK = 32, W4_SLOTS = 4;
constexpr int W4_SLOT = 32 * 1024;          // A 256 rows + W 256 rows of 64 B
constexpr int W4_OPW = 256 * 64;            // the W rows' offset in a slot
constexpr int W4_BIAS = W4_SLOTS * W4_SLOT;  // 4 waves x 128 floats after the ring
constexpr int W4_LDS = W4_BIAS + 4 * 512;
constexpr int W4_DMA = 8;                   // DMA pieces per wave per sub-step
constexpr int W4_STORES = 8 * 4;            // epilogue stores per wave of a full tile (8 row blocks x 4 pairs)
static_assert(W4_DMA + W4_STORES + 2 < 64, "vmcnt is 6 bits");

__device__ __forceinline__ int w4_swz(int row) { return ((row >> 3) & 1) * 3; }

__device__ __forceinline__ bf16x8 w4_frag(const char* op, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(op + row * 64 + ((chunk ^ w4_swz(row)) << 4));
}

template <int N_IN_FLIGHT>
__device__ __forceinline__ void w4_wait_vm() {
  static_assert(N_IN_FLIGHT >= 0 && N_IN_FLIGHT < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_IN_FLIGHT) : "memory");
}

__device__ __forceinline__ void w4_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void w4_tile_coords(int wid, int tiles_m, int tiles_n, int& m0, int& n0) {
  constexpr int GROUP_M = 8;
  const int per_group = GROUP_M * tiles_n;
  const int grp = wid / per_group;
  const int first_m = grp * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int in_g = wid - grp * per_group;
  m0 = (first_m + in_g % gsize) * 256;
  n0 = (in_g / gsize) * 256;
}

// Epilogue of one wave's 128 x 128 block: acc[i][j] holds C[m0 + 128 wm + 16 i + (l & 15)][n0 + 128 wn + 16 j +
// 4 (l >> 4) + e].
template <int EPI>
__device__ __forceinline__ void w4_epilogue(const GemmArgs& p, f32x4 (&acc)[8][8], const float* bias_lds, int m0,
                                            int n0, int wm, int wn, int lane) {
  const int mm = lane & 15;
  const int nn = 4 * (lane >> 4);
  const int mb = m0 + wm * 128, nb = n0 + wn * 128;
  f32x4 bv[8];
  {
    const unsigned addr = (unsigned)(uintptr_t)MQ_LDS_LOCAL(bias_lds + nn);
    asm volatile(
        "ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:64\n\tds_read_b128 %2, %8 offset:128\n\t"
        "ds_read_b128 %3, %8 offset:192\n\tds_read_b128 %4, %8 offset:256\n\tds_read_b128 %5, %8 offset:320\n\t"
        "ds_read_b128 %6, %8 offset:384\n\tds_read_b128 %7, %8 offset:448\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(bv[0]), "=&v"(bv[1]), "=&v"(bv[2]), "=&v"(bv[3]), "=&v"(bv[4]), "=&v"(bv[5]), "=&v"(bv[6]),
          "=&v"(bv[7])
        : "v"(addr)
        : "memory");
  }
  const bool full = (m0 + 256 <= p.M) && (n0 + 256 <= p.N);
  auto act = [&](int i, int j, float (&v)[4]) {
    v[0] = acc[i][j][0] + bv[j][0];
    v[1] = acc[i][j][1] + bv[j][1];
    v[2] = acc[i][j][2] + bv[j][2];
    v[3] = acc[i][j][3] + bv[j][3];
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
  // pairs of fragments (j, j + 1): v_permlane16_swap gives every lane 8 consecutive columns, one 16-B store
  const bool odd = (lane >> 4) & 1;
  const int nbase = nn - (odd ? 4 : 0);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mb + i * 16 + mm;
    bf16_t* crow_p = (bf16_t*)p.C + (size_t)(m < p.M ? m : 0) * p.ldc;
#pragma unroll
    for (int jp = 0; jp < 8; jp += 2) {
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
      const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      const int n = nb + (jp + (odd ? 1 : 0)) * 16 + nbase;
      if (full || (m < p.M && n < p.N))
        *reinterpret_cast<uint4*>(EPI == EPI_BF16 && p.head_dim ? gemm_out_bf16(p, m, n) : crow_p + n) = o;
    }
  }
}

// VS = false: the A / W pieces go global -> LDS by LDS-DMA; VS = true: global -> VGPR (buffer_load_dwordx4) ->
// LDS (ds_write_b128), one sub-step later (a DMA piece's issue costs its wave tens of cycles that no partner wave
// hides here; a plain load and a 16-B LDS store cost a fraction of that).
template <int EPI, bool VS>
__global__ __launch_bounds__(W4_T, 1) void gemm_w4_kernel(GemmArgs p, int tiles_m, int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int frow = lane & 15, fk = lane >> 4;
  const int arow = wm * 128, wcol = wn * 128;

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
  const int nk = p.K / W4_BK;  // even
  if (my_tiles == 0) return;

  const bool dma_w = wave >= 2;  // waves 0-1 load A rows, waves 2-3 W rows (128 rows each)
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, (int)((size_t)p.M * p.lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.W, 0, (int)((size_t)p.N * p.ldw * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.bias, 0, p.bias ? p.N * 4 : 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsD = dma_w ? rsW : rsA;
  const int prow0 = (wave & 1) * 128;                         // first tile row of this wave's pieces
  const int dst0 = (dma_w ? W4_OPW : 0) + prow0 * 64;         // their LDS offset in a slot

  // DMA issue cursor: (tile, sub-step) of the next slot to load and this lane's source offset per piece.  Past
  // the end it stays on the last sub-step (re-loaded into a free slot), which keeps every wait count uniform.
  int iss_t = 0, iss_k = 0;
  unsigned voff[W4_DMA];
  auto set_tile_ptrs = [&](int ti) {
    int m0, n0;
    w4_tile_coords(lo + xb + ti * nbx, tiles_m, tiles_n, m0, n0);
#pragma unroll
    for (int i = 0; i < W4_DMA; ++i) {
      const int row = prow0 + i * 16 + (lane >> 2);
      const int chunk = (lane & 3) ^ w4_swz(row);
      voff[i] = dma_w ? (unsigned)(((size_t)min(n0 + row, p.N - 1) * p.ldw + chunk * 8) * 2)
                      : (unsigned)(((size_t)min(m0 + row, p.M - 1) * p.lda + chunk * 8) * 2);
    }
  };
  set_tile_ptrs(0);
  auto issue = [&](int i, int slot) {
    char* dst = smem + slot * W4_SLOT + dst0 + i * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsD, MQ_LDS_LOCAL(dst), 16, voff[i], iss_k * W4_BK * 2, 0, 0);
  };
  // VS: this lane's 16 B of piece i of the issue cursor's sub-step, into registers; and their LDS store
  uint4 stage[W4_DMA];
  auto load_piece = [&](int i) {
    stage[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsD, voff[i], iss_k * W4_BK * 2, 0));
  };
  auto store_piece = [&](int i, int slot) {
    *reinterpret_cast<uint4*>(smem + slot * W4_SLOT + dst0 + i * 1024 + lane * 16) = stage[i];
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

  // compute cursor
  int cm0 = 0, cn0 = 0;
  w4_tile_coords(lo + xb, tiles_m, tiles_n, cm0, cn0);
  char* bias_lds = smem + W4_BIAS + wave * 512;
  auto issue_bias = [&](int n0) {
    const unsigned off = (unsigned)((n0 + wcol + lane) * 4);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, MQ_LDS_LOCAL(bias_lds), 4, off, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, MQ_LDS_LOCAL(bias_lds + 256), 4, off + 256, 0, 0, 0);
  };

  f32x4 acc[8][8];
  bf16x8 fa[2][8], fb[2][8];

  // prologue: the first tile's bias, then sub-steps 0-2 into slots 0-2; slot 0 must land before the first reads
  issue_bias(cn0);
  if constexpr (VS) {
    // slots 0-2 written here, sub-step 3's pieces left in the stage registers
#pragma unroll
    for (int st = 0; st < 3; ++st) {
#pragma unroll
      for (int i = 0; i < W4_DMA; ++i) load_piece(i);
#pragma unroll
      for (int i = 0; i < W4_DMA; ++i) store_piece(i, st);
      advance();
    }
#pragma unroll
    for (int i = 0; i < W4_DMA; ++i) load_piece(i);
    advance();
    w4_wait_vm<W4_DMA>();  // (the bias DMA)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
#pragma unroll
    for (int st = 0; st < 3; ++st) {
#pragma unroll
      for (int i = 0; i < W4_DMA; ++i) issue(i, st);
      advance();
    }
    w4_wait_vm<2 * W4_DMA>();
  }
  w4_barrier();
#pragma unroll
  for (int i = 0; i < 8; ++i) fa[0][i] = w4_frag(smem, arow + i * 16 + frow, fk);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[0][j] = w4_frag(smem + W4_OPW, wcol + j * 16 + frow, fk);

  // Younger than the DMA a wait retires (issued two sub-steps before): the previous sub-step's 8 pieces, plus,
  // when either of the two sub-steps since then ended a tile, that epilogue's stores (counted for full tiles
  // only: a partial tile's masked stores make the wait stricter, never looser) and the next tile's bias DMA.
  // ext1 applies to the next wait, ext2 to the one after (0: nothing; 1: bias; 2: stores + bias).
  int ext1 = 0, ext2 = 0;
  int g = 0;  // global sub-step index (slot ring position)
  auto substep = [&](auto cur_c) {
    constexpr int cur = decltype(cur_c)::value, nxt = cur ^ 1;
    if constexpr (VS) {
      // this wave's LDS stores of the previous sub-step (slot s + 2) are complete; the barrier publishes them
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      switch (ext1) {
        case 0: w4_wait_vm<W4_DMA>(); break;
        case 1: w4_wait_vm<W4_DMA + 2>(); break;
        default: w4_wait_vm<W4_DMA + W4_STORES + 2>(); break;
      }
      ext1 = ext2;
      ext2 = 0;
    }
    w4_barrier();
    const int s1 = (g + 1) & (W4_SLOTS - 1), s3 = (g + 3) & (W4_SLOTS - 1);
    const char* As = smem + s1 * W4_SLOT;
    const char* Ws = As + W4_OPW;
    // Eight chunks, fenced from each other (sched_barrier): chunk c issues DMA piece c, reads two fragments of
    // sub-step s + 1 (the W fragments in chunks 0-3, the A fragments in 4-7: each is read at least three chunks
    // before its first use) and runs the 8 MFMAs of row block c.
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if constexpr (VS) {
        store_piece(c, s3);  // sub-step s + 3, loaded during sub-step s - 1
        load_piece(c);       // sub-step s + 4
      } else {
        issue(c, s3);
      }
      if (c < 4) {
        fb[nxt][2 * c] = w4_frag(Ws, wcol + 2 * c * 16 + frow, fk);
        fb[nxt][2 * c + 1] = w4_frag(Ws, wcol + (2 * c + 1) * 16 + frow, fk);
      } else {
        fa[nxt][2 * c - 8] = w4_frag(As, arow + (2 * c - 8) * 16 + frow, fk);
        fa[nxt][2 * c - 7] = w4_frag(As, arow + (2 * c - 7) * 16 + frow, fk);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[c][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][j], fa[cur][c], acc[c][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    advance();  // (after the MFMAs: its tile-change branch would split the block the DMAs interleave in)
    ++g;
  };
  // nk is even (K % 64 == 0), so every tile starts on fragment set 0
  for (int ct = 0; ct < my_tiles; ++ct) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; kt += 2) {
      substep(std::integral_constant<int, 0>{});
      substep(std::integral_constant<int, 1>{});
    }
    w4_epilogue<EPI>(p, acc, reinterpret_cast<const float*>(bias_lds), cm0, cn0, wm, wn, lane);
    const bool full = (cm0 + 256 <= p.M) && (cn0 + 256 <= p.N);
    if (ct + 1 < my_tiles) {
      w4_tile_coords(lo + xb + (ct + 1) * nbx, tiles_m, tiles_n, cm0, cn0);
      issue_bias(cn0);
      ext1 = ext2 = full ? 2 : 1;
    }
  }
  w4_wait_vm<0>();  // no DMA may outlive the block
}

template <int EPI, bool VS>
void launch_w4v(dim3 grid, hipStream_t stream, const GemmArgs& p, int tiles_m, int tiles_n) {
  static std::atomic<unsigned> attr{0};
  if (first_on_device(attr))
    (void)hipFuncSetAttribute((const void*)gemm_w4_kernel<EPI, VS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              W4_LDS);
  hipLaunchKernelGGL((gemm_w4_kernel<EPI, VS>), grid, dim3(W4_T), W4_LDS, stream, p, tiles_m, tiles_n);
}
template <int EPI>
void launch_w4(dim3 grid, hipStream_t stream, const GemmArgs& p, int tiles_m, int tiles_n) {
  if (g_gemm_w4 == 2)
    launch_w4v<EPI, true>(grid, stream, p, tiles_m, tiles_n);
  else
    launch_w4v<EPI, false>(grid, stream, p, tiles_m, tiles_n);
}

}  // namespace

bool gemm_w4_fits(const GemmArgs& p, int epi) {
  return g_gemm_w4 && (epi == EPI_BF16 || epi == EPI_GELU_BF16 || epi == EPI_RELU_BF16) && !p.conv_c && !p.C2 &&
         p.K % (2 * W4_BK) == 0 && p.K >= 4 * W4_BK && p.M >= 256 && p.N >= 256 && p.N % 8 == 0 && p.ldc % 8 == 0 &&
         p.lda % 8 == 0 && p.ldw % 8 == 0 && (size_t)p.M * p.lda * 2 < (1ull << 31) &&
         (size_t)p.N * p.ldw * 2 < (1ull << 31);
}

int gemm_w4(const GemmArgs& p, int epi, int num_cus, hipStream_t stream) {
  const int tiles_m = (p.M + 255) / 256, tiles_n = (p.N + 255) / 256;
  const int tiles = tiles_m * tiles_n;
  dim3 grid(tiles < num_cus ? tiles : num_cus);
  switch (epi) {
    case EPI_BF16: launch_w4<EPI_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_GELU_BF16: launch_w4<EPI_GELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    case EPI_RELU_BF16: launch_w4<EPI_RELU_BF16>(grid, stream, p, tiles_m, tiles_n); break;
    default: return -3;
  }
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace mq
