// Window-attention helpers shared by swin.hip (attention kernels) and swin_fused.hip (the fused
// LayerNorm -> qkv -> window attention -> proj forward).
#pragma once
#include "sr_common.h"

namespace {

SR_DEV int region(int p, int L, int ws, int s) {
  // slices (0, -ws), (-ws, -s), (-s, None) of swinir_arch.py:266-271
  return p < L - ws ? 0 : (p < L - s ? 1 : 2);
}

SR_DEV uint32_t sx_off(int row, int chunk) {  // 16-B chunk (0..3) of a 64-B row
  return (uint32_t)(row * 64 + ((((chunk >> 1) ^ ((row >> 2) & 1))) << 5) + ((chunk & 1) << 4));
}
SR_DEV uint32_t sx_byte(int row, int dim) {  // element dim (multiple of 4) of a 64-B row
  const int b = dim * 2;
  return (uint32_t)(row * 64 + ((((b >> 5) ^ ((row >> 2) & 1))) << 5) + (b & 31));
}
SR_DEV uint32_t st_byte(int row, int col) {  // element col (multiple of 4) of a 128-B dS^T row
  const int b = col * 2;
  return (uint32_t)(row * 128 + ((((b >> 5) ^ ((row >> 1) & 3))) << 5) + (b & 31));
}
SR_DEV s16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}
// A/B fragment for K-step s from a [64][64 B] image: lane (g, tq, tp) reads rows
// 32s + 4g + tq (slots 0..3) and 32s + 16 + 4g + tq (slots 4..7) at elements col0 + 4tp.
SR_DEV s16x8 frag_tr64(const char* img, int s, int g, int tq, int tp, int col0) {
  const s16x4 lo = tr_read(img + sx_byte(32 * s + 4 * g + tq, col0 + 4 * tp));
  const s16x4 hi = tr_read(img + sx_byte(32 * s + 16 + 4 * g + tq, col0 + 4 * tp));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
SR_DEV s16x8 frag_trST(const char* img, int s, int g, int tq, int tp, int col0) {
  const s16x4 lo = tr_read(img + st_byte(32 * s + 4 * g + tq, col0 + 4 * tp));
  const s16x4 hi = tr_read(img + st_byte(32 * s + 16 + 4 * g + tq, col0 + 4 * tp));
  return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// B fragment from C registers of two vertically adjacent 16-row tiles (rows 4g + r)
SR_DEV s16x8 frag_c2(const f32x4& t0, const f32x4& t1) {
  u32x4 u;
  u[0] = pack_bf16x2(t0[0], t0[1]);
  u[1] = pack_bf16x2(t0[2], t0[3]);
  u[2] = pack_bf16x2(t1[0], t1[1]);
  u[3] = pack_bf16x2(t1[2], t1[3]);
  return __builtin_bit_cast(s16x8, u);
}
SR_DEV f32x4 mfma16(const s16x8& a, const s16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
SR_DEV int bin8(int q, int k) { return ((q >> 3) - (k >> 3) + 7) * 15 + ((q & 7) - (k & 7) + 7); }

}  // namespace
