// Shared helpers for the MI355X (gfx950 / CDNA4) kernels of libmq_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

// True the first time it is asked for the current device (one bit per device in `seen`): a kernel's function
// attributes (the dynamic-LDS ceiling) are set once per device, also when one process drives several.
inline bool first_on_device(std::atomic<unsigned>& seen) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 32) return true;
  const unsigned bit = 1u << dev;
  return (seen.fetch_or(bit) & bit) == 0;
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short short4v;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef unsigned short bf16_t;  // raw bf16 storage

#define MQ_LDS_GLOBAL(p) ((const void __attribute__((address_space(1)))*)(p))
#define MQ_LDS_LOCAL(p) ((void __attribute__((address_space(3)))*)(p))

__device__ __forceinline__ float bf16_to_f32(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (NaN kept NaN)
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  unsigned u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// two f32 -> packed bf16 pair, round-to-nearest-even: one v_cvt_pk_bf16_f32 on gfx950
// (bit-identical to f32_to_bf16 on every non-NaN input; a NaN stays a NaN)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}

// Exact-erf GELU on two values at once, erfc by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7,
// far below the bf16 rounding of the GEMM output):
//   0.5 x (1 + erf(x / sqrt2)) = max(x, 0) - h,   h = 0.5 |x| erfc(|x| / sqrt2) = |x| P(t) exp(-x^2 / 2)
// with t = 1 / (1 + p |x| / sqrt2) and P = 0.5 * (A&S polynomial in t).  Written on float pairs so the
// polynomial, products and the difference are packed v_pk_*_f32 ops; per pair two v_rcp_f32 and two
// v_exp_f32 (exp2 with the log2(e) factor folded into the constant).  ~8.5 VALU ops per value.
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 ax = __builtin_elementwise_abs(x);
  const f32x2 den = ax * (f32x2){0.23164190f, 0.23164190f} + (f32x2){1.f, 1.f};  // 1 + p |x| / sqrt2
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 poly = t * 0.5307027145f + -0.7265760135f;  // 0.5 * A&S a5, a4
  poly = poly * t + 0.7107068705f;
  poly = poly * t + -0.142248368f;
  poly = poly * t + 0.127414796f;
  poly = poly * t;
  const f32x2 u = (x * x) * -0.72134752044448170368f;  // -x^2 / 2 * log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)};
  const f32x2 h = (ax * poly) * e;
  const f32x2 pos = {fmaxf(x.x, 0.f), fmaxf(x.y, 0.f)};
  return pos - h;
}

// GELU on two values at once as x * sigmoid(g(x)), g(x) = x * P(x^2) with P a degree-6 weighted-minimax
// fit of logit(Phi(x)) / x on [0, 6.5] (|gelu error| <= 8.4e-7 in float32 arithmetic, against <= 5.2e-7
// for the A&S form above; both far below the bf16 rounding of the GEMM output).  P carries the
// -log2(e) factor, so exp2(x P) = exp(-g).  The odd polynomial needs no clamp: P's leading coefficient
// keeps x P monotone in the tails (x P -> -inf for x -> +inf: sigmoid 1; +inf for x -> -inf: exp2 = inf,
// 1 / inf = 0), checked in float32 over |x| <= 60 and for x^2 overflowing.  Per pair 10 packed
// v_pk_*_f32 ops, two v_exp_f32 and two v_rcp_f32 (the A&S form: 12 packed + 4 single + 4).
__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {
  const f32x2 x2 = x * x;
  f32x2 p = x2 * -5.384187762302872e-09f + 3.9220148551066814e-07f;
  p = p * x2 + -1.1564107808226254e-05f;
  p = p * x2 + 0.00016020433395169675f;
  p = p * x2 + 9.275906631955877e-05f;
  p = p * x2 + -0.10483432561159134f;
  p = p * x2 + -2.3022091388702393f;
  const f32x2 u = x * p;
  const f32x2 d = (f32x2){__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)} + 1.0f;
  return x * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// Butterflies across the 16-lane rows of a wave by v_permlane16_swap / v_permlane32_swap (VALU, no
// LDS round trip as with ds_bpermute).  With both operands x, permlane16_swap returns
// {x of rows 0,0,2,2 ; x of rows 1,1,3,3}, permlane32_swap {x of lanes 0-31 twice ; of 32-63 twice},
// so combining the pair gives every lane op(x, x[lane ^ 16]) (resp. ^ 32); a + b == b + a, so the sums
// equal those of a __shfl_xor butterfly bit for bit.
__device__ __forceinline__ float bfly16_max(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float bfly32_max(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}
__device__ __forceinline__ float bfly16_sum(float x) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float bfly32_sum(float x) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}

// Full-wave sum on VALU only (no ds_bpermute LDS round trips): DPP quad_perm xor 1 and xor 2, row_half_mirror
// (quad <-> quad), row_mirror (half-row <-> half-row), then the row butterflies above.  Every lane ends
// with the same value; the pairing is fixed, so the result is deterministic.
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
  int o;
  switch (ctrl_sel) {
    case 0: o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false); break;   // quad [1,0,3,2]
    case 1: o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false); break;   // quad [2,3,0,1]
    case 2: o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false); break;  // row_half_mirror
    default: o = __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false); break; // row_mirror
  }
  return v + __int_as_float(o);
}
__device__ __forceinline__ float wave_sum(float v) {
  v = dpp_add(v, 0);
  v = dpp_add(v, 1);
  v = dpp_add(v, 2);
  v = dpp_add(v, 3);
  return bfly32_sum(bfly16_sum(v));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Camera row layout shared with include/mq_hip.h (24 doubles per camera).  model: 0 omnidir, 1 pinhole
// (k3 = its fifth distortion coefficient), 2 fisheye (k1..k4 in k1, k2, p1, p2); camera.hpp.
struct CamParams {
  double fx, fy, skew, cx, cy, xi, k1, k2, p1, p2;
  double R[9];
  double t[3];
  double model, k3;
};
