// Shared device helpers for the MI355X (gfx950 / CDNA4) super-resolution kernels.
//
// Conventions used by every kernel in this directory:
//   * feature maps are NHWC, element type float (parity mode) or bf16 (train mode),
//     with an explicit pixel stride (`ld`, in elements) so channel slices of a wider
//     buffer (RRDB dense blocks) can be read and written in place;
//   * every global load of activation/weight tiles goes through a buffer resource
//     (V#) whose range check returns zeros for out-of-range offsets: that is how the
//     3x3 zero padding and partial tiles are implemented (no branches in the loaders);
//   * kernels take the caller's hipStream_t and never allocate or synchronise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SR_DEV __device__ __forceinline__

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;

// Offset that is guaranteed to fail the buffer range check (load returns 0).
#define SR_OOB 0x80000000u

SR_DEV float bf16_to_f32(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }
SR_DEV unsigned short f32_to_bf16(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
// one v_cvt_pk_bf16_f32 (the two-scalar form compiled to two conversions, a shift and an OR);
// the same round-to-nearest-even result
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
SR_DEV unsigned pack_bf16x2(float lo, float hi) {
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
// cross-lane sums / maxima over the 16-lane rows (xor 16) and the two wave halves (xor 32) by the
// gfx950 permlane swaps (VALU, no LDS round trip like ds_bpermute); every lane gets the same value
// from the same two operands in the same order
SR_DEV float xsum16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
SR_DEV float xsum32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
SR_DEV float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
SR_DEV float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Element traits: the kernels are written once over "16-byte chunks"; T decides how
// many channels a chunk carries (8 bf16 or 4 f32) and how it converts to f32.
template <typename T> struct Elt;
template <> struct Elt<float> {
  static constexpr int PER16 = 4;  // elements per 16 B chunk
  static constexpr int SIZE = 4;
  SR_DEV static float to_f(float v) { return v; }
  SR_DEV static float from_f(float v) { return v; }
};
template <> struct Elt<unsigned short> {
  static constexpr int PER16 = 8;
  static constexpr int SIZE = 2;
  SR_DEV static float to_f(unsigned short v) { return bf16_to_f32(v); }
  SR_DEV static unsigned short from_f(float v) { return f32_to_bf16(v); }
};
typedef unsigned short bf16_t;

SR_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
SR_DEV u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// One buffer_load_dwordx4 ... lds per call, exactly (inline asm: hipcc cannot split it into
// exec-divergent copies, which would break the hand-counted vmcnt).  M0 is written and
// restored inside the statement (cdna_hip_programming.md §5.7).  `lds` must be wave-uniform.
SR_DEV void glds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  const uint32_t dst = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off), "s"(__builtin_amdgcn_readfirstlane(dst)), "s"(r)
      : "memory");
}

// Fast unsigned division by a runtime constant (Hacker's Delight 10-9, round-up variant,
// exact for every 32-bit numerator). d == 1 is handled by the caller-visible flag.
struct FastDiv {
  uint32_t d, mul, shr;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  if (d <= 1) { f.mul = 0; f.shr = 0; return f; }
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;  // l = ceil(log2 d)
  f.mul = (uint32_t)(((((uint64_t)1 << l) - d) << 32) / d + 1);
  f.shr = l - 1;
  return f;
}
SR_DEV uint32_t fdiv(uint32_t n, FastDiv f) {
  if (f.d == 1) return n;
  uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> 1)) >> f.shr;
}

// XCD-aware, bijective block-id remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (shared L2).
SR_DEV uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  if (nwg < 16) return bid;
  uint32_t q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// erf for the exact-form GELU (nn.GELU default): Abramowitz & Stegun 7.1.26 with the hardware
// reciprocal and exp2, |error| <= 4.7e-7 over all x (GELU <= 2.5e-7 absolute; measured against
// math.erf on [-8, 8]) -- 18 instructions where the library erff takes 38; far below the bf16
// rounding of every GELU output, and below the fp32 parity bar
SR_DEV float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  return copysignf(1.f - p * __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f), x);
}
SR_DEV float gelu_exact(float v) { return 0.5f * v * (1.f + erf_fast(v * 0.70710678118654752f)); }
SR_DEV float gelu_grad(float z) {
  // d/dz [z * Phi(z)] = Phi(z) + z * phi(z); erf_fast's exp(-x^2) at x = z / sqrt(2) is exp(-z^2 / 2),
  // phi's exponential: one v_exp_f32 for both (the GELU' gate of the fc2 dgrad: 71 -> 53 us with
  // no GELU' at all, so its transcendentals are the cost)
  const float x = z * 0.70710678118654752f, ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  const float erf = copysignf(1.f - p * e, x);
  return fmaf(0.5f, erf, 0.5f) + z * 0.39894228040143268f * e;
}

// GELU and GELU' from one erf_fast evaluation: returns gelu(z), dg = gelu'(z) (2 FMAs more than gelu_exact)
SR_DEV float gelu_pair(float z, float& dg) {
  const float x = z * 0.70710678118654752f, ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  const float phi2 = fmaf(0.5f, copysignf(1.f - p * e, x), 0.5f);  // Phi(z)
  dg = fmaf(z * 0.39894228040143268f, e, phi2);
  return z * phi2;
}

// The aux side output of an activation epilogue (sr_conv3x3_desc.aux): GELU' of the pre-activation for
// GELU -- what the backward's gate (gate_mode 1) multiplies by, so the backward evaluates no erf -- and
// the pre-activation value for the other activations; v becomes act(v).
template <int N>
SR_DEV void act_aux_n(float (&v)[N], float (&aux)[N], int act, float slope) {
  if (act == 3) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = gelu_pair(v[j], aux[j]);
    return;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) aux[j] = v[j];
  if (act == 1) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = v[j] > 0.f ? v[j] : 0.f;
  } else if (act == 2) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * slope;
  }
}

SR_DEV float act_apply(float v, int act, float slope) {
  // act: 0 none, 1 relu, 2 leaky relu(slope), 3 GELU (exact erf form, nn.GELU default)
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : v * slope;
  if (act == 3) return gelu_exact(v);
  return v;
}
// the same over 8 values with one (wave-uniform) branch: a per-value switch costs ~4 scalar
// branches per value, exposed when a kernel runs one wave per SIMD
template <int N>
SR_DEV void act_apply_n(float (&v)[N], int act, float slope) {
  if (act == 1) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = v[j] > 0.f ? v[j] : 0.f;
  } else if (act == 2) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * slope;
  } else if (act == 3) {
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = gelu_exact(v[j]);
  }
}
