// PROTOTYPE (measurement only, not linked into libmq_hip): the one-wave-per-SIMD GEMM mainloop that
// VERDICT r3 item 2 asks for -- a 128 x 256 workgroup tile, 4 waves (one per SIMD), each wave a 128 x 64
// block (8 x 4 fragments of v_mfma_f32_16x16x32_bf16, the same per-wave block and fragment reads per MFMA
// as the shipped ping-pong kernel), BK = 64, a 3-stage LDS-DMA ring (3 x 48 KiB).  No partner wave on the
// SIMD: each wave issues its own LDS-DMA (12 x 1 KiB per K-step), fragment reads and MFMAs.  A K-step is
// two halves separated by one barrier:
//   half A: 32 MFMAs (k 0-31 of stage g, fragments already in registers) || fragment reads k 32-63 of g
//   wait (own DMAs of stage g+1) ; s_barrier (every wave's DMAs of stage g+1 landed, stage g fully read)
//   half B: 32 MFMAs (k 32-63 of g) || fragment reads k 0-31 of g+1 || LDS-DMA of stage g+3 into g's buffer
// The question it answers: does this mainloop reach the ping-pong's K-step rate?  If it does, the second
// accumulator set (deferred GELU / residual epilogue) is the next step; if not, the design is priced out.
// Epilogue: plain bf16 store of the accumulators (no bias), enough for the mainloop rate.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
#define LDSL(p) ((void __attribute__((address_space(3)))*)(p))

namespace {
constexpr int BM = 128, BN = 256, BK = 64, NT = 256;
constexpr int STAGE = (BM + BN) * 128;   // 48 KiB
constexpr int NST = 3;
constexpr int LDS = NST * STAGE;          // 144 KiB
constexpr int DMA_PER_WAVE = 12;          // (16 A + 32 W groups of 8 rows x 128 B) / 4 waves
constexpr int STORES = 8 * 2;             // bf16 epilogue stores per wave per tile

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }
// fragment reads in inline asm: the compiler's waitcnt pass then leaves the counting to the explicit waits
// (it otherwise drained lgkmcnt(0) before the first MFMA of each half).  Rows i * 16 + frow of an operand
// share one swizzle ((row >> 1) & 7 depends on frow only), so the 8 (4) fragments are one base address plus
// immediate offsets of 2 KiB.
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read16(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
  return v;
}
template <int N>
__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ unsigned pack2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}


// the k-half kk of stage buffer buf: A fragments rows i * 16 + frow, W fragments rows wcol + j * 16 + frow
__device__ __forceinline__ void read_frags(const char* smem, int buf, int kk, int wcol, int frow, int fk,
                                           bf16x8 (&a)[8], bf16x8 (&b)[4]) {
  const int chunk = (kk * 4 + fk) ^ swz(frow);
  const unsigned abase = (unsigned)(uintptr_t)LDSL(smem + buf * STAGE + frow * 128 + chunk * 16);
  const unsigned wbase = abase + BM * 128 + wcol * 128;
  b[0] = ds_read16<0>(wbase);
  b[1] = ds_read16<2048>(wbase);
  b[2] = ds_read16<4096>(wbase);
  b[3] = ds_read16<6144>(wbase);
  a[0] = ds_read16<0>(abase);
  a[1] = ds_read16<2048>(abase);
  a[2] = ds_read16<4096>(abase);
  a[3] = ds_read16<6144>(abase);
  a[4] = ds_read16<8192>(abase);
  a[5] = ds_read16<10240>(abase);
  a[6] = ds_read16<12288>(abase);
  a[7] = ds_read16<14336>(abase);
}

__global__ __launch_bounds__(NT, 1) void gemm_w1_kernel(const unsigned short* A, const unsigned short* W,
                                                        unsigned short* C, int M, int N, int K, int tiles_m,
                                                        int tiles_n) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int frow = lane & 15, fk = lane >> 4;
  const int wcol = wave * 64;
  const int nt = tiles_m * tiles_n;
  const int G = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
  const int nbx = (G - xcd + 7) >> 3, xb = bid >> 3;
  const int q = nt >> 3, r = nt & 7;
  const int lo = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  const int len = q + (xcd < r ? 1 : 0);
  const int my_tiles = xb < len ? (len - xb + nbx - 1) / nbx : 0;
  const int nk = K / BK;
  const int total = my_tiles * nk;
  if (total == 0) return;
  auto coords = [&](int t, int& m0, int& n0) {
    const int wid = lo + xb + t * nbx;
    constexpr int GM = 8;
    const int per = GM * tiles_n, grp = wid / per, fm = grp * GM;
    const int gs = min(tiles_m - fm, GM), in = wid - grp * per;
    m0 = (fm + in % gs) * BM;
    n0 = (in / gs) * BN;
  };
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((size_t)M * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)((size_t)N * K * 2), 0x00020000);
  // this wave's 12 DMA groups: A rows 32 w .. 32 w + 31 (4 groups), W rows 64 w .. 64 w + 63 (8 groups)
  int iss_t = 0, iss_k = 0;
  unsigned voff[DMA_PER_WAVE];
  auto set_tile = [&](int t) {
    int m0, n0;
    coords(t, m0, n0);
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const bool isw = i >= 4;
      const int row = (isw ? 64 * wave + 8 * (i - 4) : 32 * wave + 8 * i) + (lane >> 3);
      const int chunk = (lane & 7) ^ swz(row);
      voff[i] = isw ? (unsigned)(((size_t)min(n0 + row, N - 1) * K + chunk * 8) * 2)
                    : (unsigned)(((size_t)min(m0 + row, M - 1) * K + chunk * 8) * 2);
    }
  };
  auto issue = [&](int i, int buf) {
    const bool isw = i >= 4;
    const int dst = isw ? BM * 128 + (64 * wave + 8 * (i - 4)) * 128 : (32 * wave + 8 * i) * 128;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isw ? rsW : rsA, LDSL(smem + buf * STAGE + dst), 16, voff[i],
                                             iss_k * BK * 2, 0, 0);
  };
  auto advance = [&]() {
    if (iss_k + 1 < nk) {
      ++iss_k;
    } else if (iss_t + 1 < my_tiles) {
      ++iss_t;
      iss_k = 0;
      set_tile(iss_t);
    }
  };
  set_tile(0);
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a0[8], b0[4], a1[8], b1[4];
  // prologue: stages 0, 1, 2 into buffers 0, 1, 2; stage 0 visible, its k 0-31 fragments read
#pragma unroll
  for (int s = 0; s < NST; ++s) {
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) issue(i, s);
    advance();
  }
  wait_vm<2 * DMA_PER_WAVE>();
  barrier();
  read_frags(smem, 0, 0, wcol, frow, fk, a0, b0);
  wait_lgkm<0>();
  __builtin_amdgcn_sched_barrier(0);
  int ct = 0, kt = 0, cm0, cn0;
  coords(0, cm0, cn0);
  bool stores_pending = false;
  for (int g = 0; g < total; ++g) {
    const int buf = g % NST, nbuf = (g + 1) % NST;
    // ---- half A: MFMAs on k 0-31 of stage g, reads of k 32-63 of stage g
    read_frags(smem, buf, 1, wcol, frow, fk, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a0[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    wait_lgkm<0>();  // a1 / b1 (issued 32 MFMAs ago)
    __builtin_amdgcn_sched_barrier(0);
    // stage g + 1 landed (own DMAs: younger = stage g + 2's 12) and, after the barrier, every wave's
    if (stores_pending)
      wait_vm<DMA_PER_WAVE + STORES>();
    else
      wait_vm<DMA_PER_WAVE>();
    stores_pending = false;
    barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- half B: MFMAs on k 32-63 of stage g, reads of k 0-31 of stage g + 1, DMA of stage g + 3 -> buf
    read_frags(smem, nbuf, 0, wcol, frow, fk, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a1[i], acc[i][j], 0, 0, 0);
      if (i < 6) {
        issue(2 * i, buf);
        issue(2 * i + 1, buf);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    wait_lgkm<0>();  // a0 / b0 of stage g + 1
    __builtin_amdgcn_sched_barrier(0);
    advance();
    if (++kt == nk) {
      // plain bf16 epilogue: acc[i][j] = C[m0 + 16 i + frow][n0 + wcol + 16 j + 4 fk + e]; fragment pairs
      // (j, j + 1) through v_permlane16_swap -> one 16-B row store per lane per pair
      const bool odd = fk & 1;
      const int nbase = 4 * fk - (odd ? 4 : 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = cm0 + i * 16 + frow;
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
          unsigned pk[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            pk[h][0] = pack2(acc[i][jp + h][0], acc[i][jp + h][1]);
            pk[h][1] = pack2(acc[i][jp + h][2], acc[i][jp + h][3]);
            acc[i][jp + h] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
          const uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
          const int n = cn0 + wcol + (jp + (odd ? 1 : 0)) * 16 + nbase;
          *reinterpret_cast<uint4*>(C + (size_t)m * N + n) = o;
        }
      }
      stores_pending = true;
      kt = 0;
      if (++ct < my_tiles) coords(ct, cm0, cn0);
    }
  }
  wait_vm<0>();
}
}  // namespace

extern "C" int proto_gemm_w1(const void* A, const void* W, void* C, int M, int N, int K, int num_cus,
                             hipStream_t stream) {
  if (M % BM || N % BN || K % BK || K / BK < 3) return -1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_w1_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  const int tm = M / BM, tn = N / BN;
  const int grid = tm * tn < num_cus ? tm * tn : num_cus;
  hipLaunchKernelGGL(gemm_w1_kernel, dim3(grid), dim3(NT), LDS, stream, (const unsigned short*)A,
                     (const unsigned short*)W, (unsigned short*)C, M, N, K, tm, tn);
  return hipGetLastError() == hipSuccess ? 0 : -4;
}
