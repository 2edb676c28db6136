// Fused SwinIR attention half-block forward (round 4):
//
//   x2 = x + s1[n] * proj(WindowAttention(qkv(LN1(x))))          (basicsr/archs/swinir_arch.py:283-314,
//                                                                   WindowAttention :144-175)
//
// in ONE kernel, for bf16, window 8, head_dim <= 32 (heads padded to 32), nH * 32 <= 192, Cp <= 192:
// SwinIR-M / -S (embed 180 / 60 .. 192, 6 heads) and the remote-sensing configs.  A 512-thread block
// owns two windows (128 tokens); the token rows are gathered through the cyclic shift and window
// partition (token_pixel), so roll / partition / reverse never materialise.  Per block:
//
//   0. x rows -> LayerNorm (fp32 statistics) -> LDS token tile sX [3][128][128 B] (XOR-swizzled
//      16-B chunks), also stored to ln_out with the row mean / rstd (training: the qkv weight
//      gradient and the LayerNorm backward read them);
//   per head h:
//   A. q/k/v of head h = W_h . sX^T + b (96 x 128, K = Cp): W_h's 96 rows staged in LDS sW (loaded
//      into registers during the previous head, so the L2 round trip hides under its attention and
//      projection); 8 waves = 2 (48 rows) x 4 (32 tokens), v_mfma_f32_16x16x32_bf16.  The results go
//      to LDS (Q, K rows; V in the tr-read image of the attention kernel) and, training, to qkv;
//   B. window attention of head h for both windows: wave = (window, 16-query tile): S^T = K Q^T,
//      relative-position bias + shift mask, softmax over keys (lse stored for the backward),
//      O^T = V^T P^T -- the wattn_fwd_mfma_kernel contractions (swin.hip) on LDS operands; O to LDS
//      and, training, to the attention output `ao` (the proj weight gradient's input);
//   C. x2acc += Wp[:, h*32 .. h*32 + 31] . O_h^T (184(192) x 128, K = 32), accumulated over the
//      heads in registers (wave = 48 output channels x 64 tokens);
//   epilogue: x2 = x + s1[n] * (x2acc + bp), 8-B stores, padded channels stay exactly zero.
//
// HBM per block (training): x read once, ln_out / qkv / ao / x2 written once = 343 MB per SwinIR-M
// layer at B 32 against 540 MB for the three kernels it replaces (LN+qkv lin kernel, attention,
// proj); inference (no saved activations): x read + x2 written, 94 MB.  The backward is unchanged
// (it reads ln_out, qkv, ao, lse exactly as written by the unfused path).
#include "sr_common.h"
#include "sr_internal.h"
#include "swin_common.h"

#include <cstdlib>
#include <type_traits>

namespace {

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
SR_DEV uint2 buf_load8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
// Global stores of the fused kernels go through buffer resources with out-of-range offsets for the
// lanes that must not store, and no branch at all around them (inference: the training outputs'
// resources have size 0, every store drops): on gfx9 stores count in vmcnt, and behind a branch the
// compiler's bookkeeping takes the no-store path's count, so a later load wait drained every store.
SR_DEV float buf_loadf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
SR_DEV void buf_store8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}
SR_DEV void buf_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
SR_DEV void buf_store4f(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

// LayerNorm of a 192-channel token row held by 4 lanes (lane part has the 16-B chunks part, part + 4,
// .., loaded into raw; chunks past KC are zero).  Padded channels of x are exactly zero (the NHWC
// invariant), so the sum needs no mask; the 192 - C zero values add exactly mu^2 each to the squared
// deviations, subtracted once after the row reduction (no per-element select).  Packed fp32 pairs.
SR_DEV f32x2 bf16x2_f(unsigned q) { return f32x2{__uint_as_float(q << 16), __uint_as_float(q & 0xffff0000u)}; }
SR_DEV void ln_row4_stats(const u32x4 (&raw)[6], int C, float eps, float& mu, float& rs) {
  f32x2 sm2 = {0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 6; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) sm2 += bf16x2_f(raw[q][j]);
  float sm = sm2[0] + sm2[1];
  sm += __shfl_xor(sm, 1);
  sm += __shfl_xor(sm, 2);
  mu = sm / C;
  f32x2 sq2 = {0.f, 0.f};
  const f32x2 mu2 = {mu, mu};
#pragma unroll
  for (int q = 0; q < 6; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x2 d = bf16x2_f(raw[q][j]) - mu2;
      sq2 += d * d;
    }
  float sq = sq2[0] + sq2[1];
  sq += __shfl_xor(sq, 1);
  sq += __shfl_xor(sq, 2);
  sq = fmaxf(sq - (float)(192 - C) * mu * mu, 0.f);
  rs = rsqrtf(sq / C + eps);
}
// one normalised chunk (8 channels from c0): o = x A + B with A = rs gamma, B = beta - mu A (gamma /
// beta zero past C, so padded outputs come out exactly 0)
SR_DEV u32x4 ln_chunk(const u32x4& raw, int c0, float mu, float rs, const float* sGB) {
  u32x4 o4;
  const f32x2 mu2 = {mu, mu}, rs2 = {rs, rs};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + 2 * j;
    const f32x2 A = f32x2{sGB[c], sGB[c + 1]} * rs2;
    const f32x2 B = f32x2{sGB[192 + c], sGB[192 + c + 1]} - mu2 * A;
    const f32x2 o = bf16x2_f(raw[j]) * A + B;
    o4[j] = pack_bf16x2(o[0], o[1]);
  }
  return o4;
}

struct SabArgs {
  const bf16_t* x;
  const float* ln_g;
  const float* ln_b;
  const bf16_t* wq;  // qkv GEMM image [3 nH 32][Cp] (row = which * nH * 32 + h * 32 + d)
  const float* bq;   // [3 nH 32]
  const float* table;  // [225][nH]
  const bf16_t* wp;  // proj GEMM image [Cp][nH 32]
  const float* bp;   // [Cp]
  const float* rsc;  // per-image DropPath factor [N] or null
  bf16_t* x2;
  bf16_t* ln_out;  // training outputs (all null for inference)
  float* mean;
  float* rstd;
  bf16_t* qkv;
  bf16_t* ao;
  float* lse;
  int N, H, W, shift, nH, C, Cp, KC;
  int ldq, ldo;
  float eps, scale;
  int nwx, nwin, nwin_total;
  unsigned long long* stamps;  // diagnostics (DBG 32): per-block phase cycles of waves 0 and 4
};

// LDS layout of a block of NW windows (TOK = 64 NW tokens, 256 NW threads).  O_h has its own image
// and the bias table is staged one head column at a time in two slots (head h in slot h & 1; the
// next head's column is loaded at the head's top, with its weights, and written after S1), so a head
// needs two barriers: S1 (Q, K, V of the head in LDS; the weight image and the other table slot free)
// and S2 (O_h in LDS; the next head's weights and table column visible).  Step C of head h and step A
// of head h + 1 then run back to back: A writes Q / K / V, which nobody reads after S2, and C reads O,
// which the next head writes only after its S1.  (Round 4 / early round 5: O_h overlaid Q_h and a
// third barrier per head closed step C.)
template <int NW> struct SabL {
  static constexpr int TOK = 64 * NW, NT = 256 * NW;
  static constexpr int X = 0;                      // [3 cg][TOK rows][128 B]
  static constexpr int W = X + 3 * TOK * 128;      // [3 cg][96 rows][128 B]
  static constexpr int Q = W + 3 * 96 * 128;       // [TOK][64 B]
  static constexpr int K = Q + TOK * 64;
  static constexpr int V = K + TOK * 64;           // [NW windows][64][64 B], sx_byte layout (tr reads)
  static constexpr int O = V + TOK * 64;           // [TOK][64 B]
  static constexpr int TB = O + TOK * 64;          // float [2][256]: bias-table column of head h in slot h & 1
  static constexpr int GB = TB + 2 * 256 * 4;      // float [2][192]: LayerNorm gamma, beta
  static constexpr int BQ = GB + 2 * 192 * 4;      // float [3 nH 32 <= 576]: qkv bias
  static constexpr int BP = BQ + 576 * 4;          // float [192]: proj bias
  static constexpr int LDS = BP + 192 * 4;
  static constexpr int WREG = (96 * 24 + NT - 1) / NT;  // 16-B pieces of W_h (K <= 192) per thread
};
constexpr int SAB_WPIECES = 96 * 24;

// 16-B chunk ch of row r of a [cg][rows][128 B] image (chunk XOR row & 7 within its 128-B group)
SR_DEV uint32_t tile_off(int rows, int r, int ch) {
  return (uint32_t)((ch >> 3) * rows * 128 + r * 128 + (((ch & 7) ^ (r & 7)) << 4));
}
// 16-B chunk c (0..3) of token row t of a [128][64 B] image; rows 4a..4a+3 rotate the chunks by a,
// so 16 consecutive rows reading one chunk hit 16 distinct 4-bank groups
SR_DEV uint32_t qk_off16(int t, int c) { return (uint32_t)(t * 64 + ((c ^ ((t >> 2) & 3)) << 4)); }
SR_DEV uint32_t qk_off(int t, int d) { return qk_off16(t, d >> 3) + (uint32_t)((d & 7) * 2); }

// NW windows per block: 2 (8 waves, one block per CU: 122 KB of LDS).  (One-window blocks, two per
// CU at 77.5 KB, measured the same in round 4 and were removed in round 5.)
// SH: the shifted-window block (the mask arithmetic is compiled only there).
// DBG (timing ablations, wrong results; knob SR_SWIN_ATTN_DBG): 1 no step-A MFMAs, 2 no softmax
// VALU, 4 no step-C MFMAs, 8 no LayerNorm arithmetic, 16 no per-head weight staging; 32: phase stamps
// (s_memtime; results unchanged): per block, waves 0 and 4, the LayerNorm prologue, steps A / B / C
// and the two barrier waits summed over the heads (tools/swin_attn_stamps.py).
// Round 5 (VALU per wave was the bound: ablations put 30-36 us of a 148 us inference launch each in
// the softmax, the LayerNorm and the per-head weight staging): head-invariant addresses hoisted out
// of the head loop (weight pieces: one offset per piece + the head as the buffer soffset; the step-A /
// B store offsets), the softmax in base 2 (table column and scale pre-multiplied by log2 e: one fma
// per score, v_exp_f32 directly), the mask only in shifted blocks.
// Round 6: the prologue's operands in one round trip (s_memtime phase stamps, DBG 32, put the
// LayerNorm prologue at 22 % of the kernel).  Measured and removed (profiles/r06/ab/swin_attn/): the
// per-head weight images double-buffered in LDS and filled by LDS-DMA (no VGPR staging; train
// 142 -> 152..158 us with the wait at S1, 151 -> 150 us waited before S2), static s_setprio 1 for
// waves 4-7 (+-2 us), the last head peeled with the residual loads at its top (inference +4 us),
// and a role-split form (waves 0-3 the qkv projection with W in registers, waves 4-7 softmax / AV /
// proj, a 3-stage pipeline with one barrier per stage: train 144 -> 172 us, inference 115 -> 129 us).
template <int NW, int DBG = 0, bool SH = true>
__global__ __launch_bounds__(256 * NW, 3 - NW) void swin_attn_block_fwd_kernel(SabArgs a) {
  constexpr bool ST = (DBG & 32) != 0;
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tst = 0, t0 = 0, t1 = 0;
  if constexpr (ST) tst = __builtin_readcyclecounter();
  using L = SabL<NW>;
  constexpr int TOK = L::TOK, NT = L::NT;
  __shared__ __attribute__((aligned(16))) char smem[L::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15, tq = (lane >> 2) & 3, tp = lane & 3;
  const int blk = (int)xcd_remap(blockIdx.x, gridDim.x);
  const bool train = a.qkv != nullptr;
  const uint32_t M = (uint32_t)(a.N * a.H * a.W);
  const auto lnr = make_rsrc(a.ln_out, train ? M * a.Cp * 2u : 0u);
  const auto mur = make_rsrc(a.mean, train ? M * 4u : 0u);
  const auto rsr = make_rsrc(a.rstd, train ? M * 4u : 0u);
  const auto qkvr = make_rsrc(a.qkv, train ? M * a.ldq * 2u : 0u);
  const auto aor = make_rsrc(a.ao, train ? M * a.ldo * 2u : 0u);
  const auto lser = make_rsrc(a.lse, train ? (uint32_t)a.nwin_total * a.nH * 64u * 4u : 0u);
  const auto x2r = make_rsrc(a.x2, M * a.Cp * 2u);
  float* sTB = (float*)(smem + L::TB);
  float* sGB = (float*)(smem + L::GB);
  float* sBQ = (float*)(smem + L::BQ);
  float* sBP = (float*)(smem + L::BP);

  // window geometry of the block's windows
  auto win_of = [&](int wi, int& n, int& wy, int& wx) -> bool {
    const int gw = NW * blk + wi;
    n = gw / a.nwin;
    const int win = gw - n * a.nwin;
    wy = win / a.nwx;
    wx = win - wy * a.nwx;
    return gw < a.nwin_total;
  };
  // token t (0..TOK-1) of the block -> pixel row (through the cyclic shift), image; false past the end
  auto tok_pix = [&](int t, int64_t& pix, int& n) -> bool {
    int wy, wx;
    const bool v = win_of(t >> 6, n, wy, wx);
    const int i = t & 63;
    int oy = wy * 8 + (i >> 3) + a.shift, ox = wx * 8 + (i & 7) + a.shift;
    if (oy >= a.H) oy -= a.H;
    if (ox >= a.W) ox -= a.W;
    pix = ((int64_t)n * a.H + oy) * a.W + ox;
    return v;
  };

  // ---- head 0's weights into registers first (their L2 round trip overlaps the LayerNorm)
  // weight loads through buffer resources (out of range -> 0, no branches: the compiler's vmcnt
  // bookkeeping stays exact across them)
  const auto wqr = make_rsrc(a.wq, (uint32_t)((size_t)3 * a.nH * 32 * a.Cp * 2));
  const auto wpr = make_rsrc(a.wp, (uint32_t)((size_t)a.Cp * a.ldo * 2));
  const auto tbr = make_rsrc(a.table, (uint32_t)(225 * a.nH * 4));
  u32x4 wreg[L::WREG];
  // piece p = (row rr of the head's 96, 16-B chunk ch): its global offset at head 0 (the head adds
  // 64 Cp bytes, passed as the buffer soffset) and its LDS offset, computed once
  uint32_t wgo[L::WREG], wlo[L::WREG];
#pragma unroll
  for (int k = 0; k < L::WREG; ++k) {
    const int p = tid + NT * k;
    const int rr = p / 24, ch = p - rr * 24;
    const int grow = (rr >> 5) * a.nH * 32 + (rr & 31);
    wgo[k] = (p < SAB_WPIECES && ch < a.KC) ? (uint32_t)(grow * a.Cp + ch * 8) * 2u : SR_OOB;
    wlo[k] = L::W + tile_off(96, rr, ch);
  }
  auto w_load = [&](int h) {
    const uint32_t so = (uint32_t)(h * 64 * a.Cp);
#pragma unroll
    for (int k = 0; k < L::WREG; ++k)
      wreg[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wqr, wgo[k], so, 0));
  };
  auto w_store = [&]() {
#pragma unroll
    for (int k = 0; k < L::WREG; ++k)
      if (tid + NT * k < SAB_WPIECES) *(u32x4*)(smem + wlo[k]) = wreg[k];
  };
  w_load(0);
  // every small operand (bias table column, qkv / proj biases, LayerNorm gamma / beta) and the token rows
  // are issued together, as unconditional buffer loads (out of range -> 0), before the first global
  // store (on gfx9 vmcnt counts stores too, so a load issued after stores makes its wait drain them):
  // one HBM round trip for the whole prologue.  (Round 5: loads inside `if (tid < ..)` branches made
  // each its own load-wait-write round trip -- the prologue was 22 % of the kernel, DBG 32 stamps.)
  constexpr float LOG2E = 1.4426950408889634f;
  const auto tbl0 = make_rsrc(a.table, (uint32_t)(225 * a.nH * 4));
  const auto bqr = make_rsrc(a.bq, (uint32_t)(3 * a.nH * 32 * 4));
  const auto bpr = make_rsrc(a.bp, (uint32_t)(a.Cp * 4));
  const auto lgr = make_rsrc(a.ln_g, (uint32_t)(a.C * 4));
  const auto lbr = make_rsrc(a.ln_b, (uint32_t)(a.C * 4));
  const auto xin = make_rsrc(a.x, M * a.Cp * 2u);
  constexpr int NBQ = (576 + NT - 1) / NT;
  const float v_tb = buf_loadf(tbl0, tid < 225 ? (uint32_t)(tid * a.nH) * 4u : SR_OOB);
  float v_bq[NBQ];
#pragma unroll
  for (int k = 0; k < NBQ; ++k) v_bq[k] = buf_loadf(bqr, (uint32_t)(tid + NT * k) * 4u);
  const float v_bp = buf_loadf(bpr, (uint32_t)tid * 4u);
  const float v_g = buf_loadf(lgr, (uint32_t)(tid & 255) * 4u), v_b = buf_loadf(lbr, (uint32_t)(tid & 255) * 4u);

  // ---- 0. LayerNorm of the TOK token rows: 4 lanes per row, chunks part, part + 4, ...
  {
    const int r = tid >> 2, part = tid & 3;
    int64_t pr;
    int nr;
    const bool vr = tok_pix(r, pr, nr);
    u32x4 raw[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int ch = part + 4 * q;
      raw[q] = buf_load16(xin, (vr && ch < a.KC) ? (uint32_t)(pr * a.Cp + ch * 8) * 2u : SR_OOB);
    }
    if (tid < 256) sTB[tid] = v_tb * LOG2E;
#pragma unroll
    for (int k = 0; k < NBQ; ++k)
      if (tid + NT * k < 576) sBQ[tid + NT * k] = v_bq[k];
    if (tid < 192) {
      sBP[tid] = v_bp;
      sGB[tid] = v_g;
      sGB[192 + tid] = v_b;
    }
    float mu, rs;
    ln_row4_stats(raw, a.C, a.eps, mu, rs);
    __syncthreads();  // gamma / beta staged
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int ch = part + 4 * q;
      u32x4 o4 = u32x4{0u, 0u, 0u, 0u};
      if (vr && ch < a.KC) {
        if constexpr ((DBG & 8) != 0) o4 = raw[q];
        else o4 = ln_chunk(raw[q], ch * 8, mu, rs, sGB);
      }
      buf_store16(lnr, (vr && ch < a.KC) ? (uint32_t)(pr * a.Cp + ch * 8) * 2u : SR_OOB, o4);
      *(u32x4*)(smem + L::X + tile_off(TOK, r, ch)) = o4;
    }
    buf_store4f(mur, (vr && part == 0) ? (uint32_t)pr * 4u : SR_OOB, mu);
    buf_store4f(rsr, (vr && part == 0) ? (uint32_t)pr * 4u : SR_OOB, rs);
  }
  w_store();
  __syncthreads();
  if constexpr (ST) ph[0] = __builtin_readcyclecounter() - tst;  // LayerNorm prologue

  // per-wave constants
  const int og = w & 1, tg = w >> 1;   // step A: 48 q/k/v rows x 32 tokens
  const int wi = w >> 2, jq = w & 3;   // step B: window, 16-query tile
  const int pog = w & 3, ptg = w >> 2;  // step C: 48 output channels x 64 tokens
  int64_t pixA[2];
  bool vA[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int n_;
    vA[j] = tok_pix(tg * 32 + 16 * j + c16, pixA[j], n_);
  }
  int nB, wyB, wxB;
  const bool vB = win_of(wi, nB, wyB, wxB);
  int64_t pixB;
  {
    int n_;
    tok_pix(wi * 64 + 16 * jq + c16, pixB, n_);
  }
  const int qq = 16 * jq + c16;  // this lane's query (B)
  const int rq = region(wyB * 8 + (qq >> 3), a.H, 8, a.shift) * 3 + region(wxB * 8 + (qq & 7), a.W, 8, a.shift);
  // head-invariant parts of step B, once per block: the shift mask of this lane's 16 keys as bits, and
  // the relative-position index bin8(qq, k) of key k = 16 i + 4 g + r, which is tbase - 30 i - r
  // (k >> 3 = 2 i + (g >> 1), k & 7 = 4 (g & 1) + r), so the table reads take immediate offsets
  // (shifted blocks) the mask of this lane's 16 keys as additive base-2 scores: -100 nats
  float mk[16];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = 16 * i + 4 * g + r;
      mk[4 * i + r] = 0.f;
      if constexpr (SH) {
        const int rk = region(wyB * 8 + (k >> 3), a.H, 8, a.shift) * 3 + region(wxB * 8 + (k & 7), a.W, 8, a.shift);
        if (rk != rq) mk[4 * i + r] = -100.f * LOG2E;
      }
    }
  // head-invariant store offsets (the head adds h * 64 bytes, folded into the per-head base)
  uint32_t qkvo[2], lao;
#pragma unroll
  for (int j = 0; j < 2; ++j) qkvo[j] = vA[j] ? (uint32_t)(pixA[j] * a.ldq) * 2u : SR_OOB;
  lao = vB ? (uint32_t)(pixB * a.ldo) * 2u : SR_OOB;
  const uint32_t lseo = (vB && g == 0) ? (uint32_t)((NW * blk + wi) * a.nH * 64 + qq) * 4u : SR_OOB;
  const float scale2 = a.scale * LOG2E;
  const int tbase = ((qq >> 3) - (g >> 1) + 7) * 15 + (qq & 7) - 4 * (g & 1) + 7;

  f32x4 xacc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) xacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int h = 0; h < a.nH; ++h) {
    if constexpr (ST) t0 = __builtin_readcyclecounter();
    // The head's global loads (projection columns, the next head's weights) are issued here, before
    // its qkv / ao / lse stores; the biases and the table come from LDS (a bias loaded from global
    // after the stores drained all of them, three times per head, in the first version).
    // this head's projection columns (A operand of step C) and the next head's weights, in flight
    u32x4 wpf[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int row = pog * 48 + 16 * i + c16;
      wpf[i] = buf_load16(wpr, row < a.Cp ? (uint32_t)(row * a.ldo + h * 32 + 8 * g) * 2u : SR_OOB);
    }
    if (h + 1 < a.nH && (DBG & 16) == 0) w_load(h + 1);
    const float tbn = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
        tbr, (h + 1 < a.nH && tid < 225) ? (uint32_t)(tid * a.nH + h + 1) * 4u : SR_OOB, 0, 0));  // next column
    __builtin_amdgcn_sched_barrier(0);  // keep these loads here, ahead of the head's stores
    // step B's 16 bias-table values of this lane (+ the shift mask), read now: their LDS latency hides
    // under step A instead of 8 dependent ds_read round trips in the softmax (the column was staged
    // after the previous head's S1 barrier)
    float tbv[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        tbv[4 * i + r] = (sTB + (h & 1) * 256 + tbase - 93)[93 - 30 * i - r];
        if constexpr (SH) tbv[4 * i + r] += mk[4 * i + r];
      }

    // ---- A: q / k / v of head h
    f32x4 acc[3][2];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      const int ch = 4 * kk + g;
      s16x8 af[3], bf[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) af[i] = *(const s16x8*)(smem + L::W + tile_off(96, og * 48 + 16 * i + c16, ch));
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = *(const s16x8*)(smem + L::X + tile_off(TOK, tg * 32 + 16 * j + c16, ch));
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr ((DBG & 1) == 0) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
          else acc[i][j][0] += __builtin_bit_cast(float, (int)(af[i][0] ^ bf[j][1]));
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int oc = og * 48 + 16 * i + 4 * g;  // 4 consecutive rows of q / k / v (one of them)
      const int which = oc >> 5, d = oc & 31;
      const int gr = which * a.nH * 32 + h * 32 + d;
      const f32x4 bias = *(const f32x4*)(sBQ + gr);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int t = tg * 32 + 16 * j + c16;
        uint2 u;
        u.x = pack_bf16x2(acc[i][j][0] + bias[0], acc[i][j][1] + bias[1]);
        u.y = pack_bf16x2(acc[i][j][2] + bias[2], acc[i][j][3] + bias[3]);
        // lane part of the offset in voffset, the head (uniform) as soffset: a lane-varying soffset
        // makes the compiler wrap the store in a waterfall loop
        const uint32_t vo = qkvo[j] == SR_OOB ? SR_OOB : qkvo[j] + (uint32_t)(which * a.nH * 32 + d) * 2u;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, u), qkvr, vo, (uint32_t)h * 64u, 0);
        const uint32_t qk = qk_off(t, d);
        const uint32_t la = which == 0 ? L::Q + qk : which == 1 ? L::K + qk : L::V + (t >> 6) * 4096 + sx_byte(t & 63, d);
        *(uint2*)(smem + la) = u;
      }
    }
    if constexpr (ST) { t1 = __builtin_readcyclecounter(); ph[1] += t1 - t0; }
    __syncthreads();  // S1: Q, K, V of head h in LDS; every wave is past step A (sW) and the top (table slot)
    if constexpr (ST) { t0 = __builtin_readcyclecounter(); ph[2] += t0 - t1; }
    if (h + 1 < a.nH) {
      if constexpr ((DBG & 16) == 0) w_store();
      if (tid < 256) sTB[((h + 1) & 1) * 256 + tid] = tbn * LOG2E;  // (scaled here: a multiply next to the load would wait for it)
    }

    // ---- B: window attention, wave = (window wi, queries 16 jq ..)
    {
      const s16x8 qf = *(const s16x8*)(smem + L::Q + qk_off16(wi * 64 + qq, g));
      f32x4 s[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x8 kf = *(const s16x8*)(smem + L::K + qk_off16(wi * 64 + 16 * i + c16, g));
        s[i] = mfma16(kf, qf, f32x4{0.f, 0.f, 0.f, 0.f});  // S^T[key 16i + 4g + r][query qq]
      }
      float mx = -3.0e38f, inv = 1.f;
      if constexpr ((DBG & 2) == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // key k = 16 i + 4 g + r
          // base 2: scores and table scaled by log2 e (the mask: -100 nats)
          const float v = fmaf(s[i][r], scale2, tbv[4 * i + r]);  // + sTB[bin8(qq, k)] + mask
          s[i][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = xmax32(xmax16(mx));
      float sm = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[i][r] - mx);
          s[i][r] = e;
          sm += e;
        }
      sm = xsum32(xsum16(sm));
      inv = __builtin_amdgcn_rcpf(sm);  // applied to O (8 values per lane) instead of P (16)
      mx = (mx + __log2f(sm)) * 0.6931471805599453f;  // natural-log LSE for the backward
      }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mx), lser, lseo, (uint32_t)h * 256u, 0);
      f32x4 o[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      const char* sVw = smem + L::V + wi * 4096;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const s16x8 pb = frag_c2(s[2 * st], s[2 * st + 1]);
#pragma unroll
        for (int d = 0; d < 2; ++d) o[d] = mfma16(frag_tr64(sVw, st, g, tq, tp, 16 * d), pb, o[d]);
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {  // O^T[dim 16d + 4g + r][query qq]
        uint2 u;
        u.x = pack_bf16x2(o[d][0] * inv, o[d][1] * inv);
        u.y = pack_bf16x2(o[d][2] * inv, o[d][3] * inv);
        const uint32_t vo = lao == SR_OOB ? SR_OOB : lao + (uint32_t)(16 * d + 4 * g) * 2u;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, u), aor, vo, (uint32_t)h * 64u, 0);
        *(uint2*)(smem + L::O + qk_off(wi * 64 + qq, 16 * d + 4 * g)) = u;
      }
    }
    if constexpr (ST) { t1 = __builtin_readcyclecounter(); ph[3] += t1 - t0; }
    __syncthreads();  // S2: O_h in LDS (Q, K, V free); the next head's weights and table column visible
    if constexpr (ST) { t0 = __builtin_readcyclecounter(); ph[4] += t0 - t1; }

    // ---- C: x2acc += Wp[:, head h] . O_h^T
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x8 of = *(const s16x8*)(smem + L::O + qk_off16(ptg * 64 + 16 * j + c16, g));
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if constexpr ((DBG & 4) == 0) xacc[i][j] = mfma16(__builtin_bit_cast(s16x8, wpf[i]), of, xacc[i][j]);
        else xacc[i][j][0] += __builtin_bit_cast(float, (int)(wpf[i][0] ^ (unsigned)of[1]));
      }
    }
    if constexpr (ST) ph[5] += __builtin_readcyclecounter() - t0;
  }

  // ---- epilogue: x2 = x + s1[n] * (proj + bias); all loads before the first store (see above)
  f32x4 biasp[3];
  uint2 xres[3][4];
  float scj[4];
  int64_t pixj[4];
  bool vj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int n;
    vj[j] = tok_pix(ptg * 64 + 16 * j + c16, pixj[j], n);
    scj[j] = (a.rsc && vj[j]) ? a.rsc[n] : 1.f;
  }
  const auto xr = make_rsrc(a.x, (uint32_t)((size_t)a.N * a.H * a.W * a.Cp * 2));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int oc = pog * 48 + 16 * i + 4 * g;
    biasp[i] = oc < a.Cp ? *(const f32x4*)(sBP + oc) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      xres[i][j] = buf_load8(xr, (oc < a.Cp && vj[j]) ? (uint32_t)(pixj[j] * a.Cp + oc) * 2u : SR_OOB);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int oc = pog * 48 + 16 * i + 4 * g;
    const f32x4 bias = biasp[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float sc = scj[j];
      const uint2 xv = xres[i][j];
      uint2 u;
      u.x = pack_bf16x2(bf16_to_f32(xv.x & 0xffff) + sc * (xacc[i][j][0] + bias[0]),
                        bf16_to_f32(xv.x >> 16) + sc * (xacc[i][j][1] + bias[1]));
      u.y = pack_bf16x2(bf16_to_f32(xv.y & 0xffff) + sc * (xacc[i][j][2] + bias[2]),
                        bf16_to_f32(xv.y >> 16) + sc * (xacc[i][j][3] + bias[3]));
      buf_store8(x2r, (oc < a.Cp && vj[j]) ? (uint32_t)(pixj[j] * a.Cp + oc) * 2u : SR_OOB, u);
    }
  }
  if constexpr (ST) {
    // per block, waves 0 and 4: LN prologue, A, S1 wait, B, S2 wait, C (summed over heads), total
    if ((w == 0 || w == 4) && lane == 0) {
      ph[6] = __builtin_readcyclecounter() - tst;
      unsigned long long* st = a.stamps + ((size_t)blockIdx.x * 2 + (w >> 2)) * 8;
#pragma unroll
      for (int k = 0; k < 7; ++k) st[k] = ph[k];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused MLP half of a SwinTransformerBlock (round 4):
//
//   out = x2 + s2[n] * fc2(GELU(fc1(LN2(x2))))          (swinir_arch.py:322-323, Mlp :43-60)
//
// bf16, Cp <= 192, hidden Hp <= 384 (mlp_ratio 2: 360).  A 512-thread block owns 128 consecutive
// token rows: LN2 into an LDS tile (and, training, ln_out / mean / rstd), fc1 with W1 fragments from
// L2 into registers (wave w: hidden tiles w, w + 8, w + 16 over all 128 tokens), bias + exact GELU
// in the epilogue (training: GELU'(z) and h stored, as the lin kernel's aux / output), h into an LDS tile
// that overlays the dead LN tile, then fc2 (wave: 48 output channels x 64 tokens) + bias, DropPath
// row scale and the residual.  HBM (training): x2 read twice, ln_out / z / h / out written once =
// 376 MB per SwinIR-M layer at B 32 against 470 MB for the lin kernel + linear_wk_kernel pair; h is
// never re-read for fc2.
struct SmbArgs {
  const bf16_t* x;   // x2 [M][Cp]
  const float* ln_g;
  const float* ln_b;
  const bf16_t* w1;  // fc1 image [Hp][Cp]
  const float* b1;   // [Hp]
  const bf16_t* w2;  // fc2 image [Cp][Hp]
  const float* b2;   // [Cp]
  const float* rsc;  // [N] or null
  bf16_t* out;
  bf16_t* ln_out;  // training outputs (null for inference)
  float* mean;
  float* rstd;
  bf16_t* z;
  bf16_t* h;
  int M, HW, C, Cp, KC, Hp, HC;  // HC = Hp / 8 (16-B chunks of a hidden row)
  float eps;
};

constexpr int SMB_H = 0;                 // [6 cg][128][128 B]: LN(x2) tile (cg 0..2), then h (cg 0..5)
constexpr int SMB_GB = 6 * 128 * 128;    // float [2][192]
constexpr int SMB_B1 = SMB_GB + 2 * 192 * 4;  // float [384]: fc1 bias
constexpr int SMB_B2 = SMB_B1 + 384 * 4;      // float [192]: fc2 bias
constexpr int SMB_LDS = SMB_B2 + 192 * 4;

__global__ __launch_bounds__(512, 1) void swin_mlp_block_fwd_kernel(SmbArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[SMB_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = (int)xcd_remap(blockIdx.x, gridDim.x) * 128;
  const bool train = a.z != nullptr;
  const uint32_t Mu = (uint32_t)a.M;
  const auto lnr = make_rsrc(a.ln_out, train ? Mu * a.Cp * 2u : 0u);  // size 0: every store drops
  const auto mur = make_rsrc(a.mean, train ? Mu * 4u : 0u);
  const auto rsr = make_rsrc(a.rstd, train ? Mu * 4u : 0u);
  const auto zr = make_rsrc(a.z, train ? Mu * a.Hp * 2u : 0u);
  const auto hr_ = make_rsrc(a.h, train ? Mu * a.Hp * 2u : 0u);
  const auto outr = make_rsrc(a.out, Mu * a.Cp * 2u);
  float* sGB = (float*)(smem + SMB_GB);
  float* sB1 = (float*)(smem + SMB_B1);
  float* sB2 = (float*)(smem + SMB_B2);
  // the small operands, W1's first fragments and the token rows are issued together as unconditional
  // buffer loads (out of range -> 0), before the first global store: one round trip for the prologue
  // (loads inside `if (tid < ..)` branches were each a load-wait-write round trip)
  const float v_b1 = buf_loadf(make_rsrc(a.b1, (uint32_t)(a.Hp * 4)), (uint32_t)tid * 4u);
  const float v_b2 = buf_loadf(make_rsrc(a.b2, (uint32_t)(a.Cp * 4)), (uint32_t)tid * 4u);
  const float v_g = buf_loadf(make_rsrc(a.ln_g, (uint32_t)(a.C * 4)), (uint32_t)(tid & 255) * 4u);
  const float v_b = buf_loadf(make_rsrc(a.ln_b, (uint32_t)(a.C * 4)), (uint32_t)(tid & 255) * 4u);
  // fc1's first two K-steps of W1 fragments, issued before the LayerNorm's stores (on gfx9 vmcnt
  // counts stores too: a load issued after them waits for them)
  const int ntl = (a.Hp + 15) / 16;
  const auto w1r = make_rsrc(a.w1, (uint32_t)((size_t)a.Hp * a.Cp * 2));
  const auto w2r = make_rsrc(a.w2, (uint32_t)((size_t)a.Cp * a.Hp * 2));
  const auto xr = make_rsrc(a.x, (uint32_t)((size_t)a.M * a.Cp * 2));
  auto w1_frag = [&](int i, int kk) -> s16x8 {  // buffer loads: no branches around the MFMAs
    const int row = 16 * (w + 8 * i) + c16, ch = 4 * kk + g;
    const bool v = w + 8 * i < ntl && row < a.Hp && ch < a.KC;
    return __builtin_bit_cast(s16x8, buf_load16(w1r, v ? (uint32_t)(row * a.Cp + ch * 8) * 2u : SR_OOB));
  };
  s16x8 af[2][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    af[0][i] = w1_frag(i, 0);
    af[1][i] = w1_frag(i, 1);
  }
  // ---- LayerNorm of the 128 rows: 4 lanes per row
  {
    const int r = tid >> 2, part = tid & 3, m = m0 + r;
    const bool vr = m < a.M;
    u32x4 raw[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int ch = part + 4 * q;
      raw[q] = buf_load16(xr, (vr && ch < a.KC) ? (uint32_t)(m * a.Cp + ch * 8) * 2u : SR_OOB);
    }
    if (tid < 384) sB1[tid] = v_b1;
    if (tid < 192) {
      sB2[tid] = v_b2;
      sGB[tid] = v_g;
      sGB[192 + tid] = v_b;
    }
    float mu, rs;
    ln_row4_stats(raw, a.C, a.eps, mu, rs);
    __syncthreads();  // gamma / beta staged
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int ch = part + 4 * q;
      u32x4 o4 = u32x4{0u, 0u, 0u, 0u};
      if (vr && ch < a.KC) o4 = ln_chunk(raw[q], ch * 8, mu, rs, sGB);
      buf_store16(lnr, (vr && ch < a.KC) ? (uint32_t)(m * a.Cp + ch * 8) * 2u : SR_OOB, o4);
      *(u32x4*)(smem + SMB_H + tile_off(128, r, ch)) = o4;
    }
    buf_store4f(mur, (vr && part == 0) ? (uint32_t)m * 4u : SR_OOB, mu);
    buf_store4f(rsr, (vr && part == 0) ? (uint32_t)m * 4u : SR_OOB, rs);
  }
  __syncthreads();

  // ---- fc1: hidden tiles t = w, w + 8, w + 16 (< 23) x all 128 tokens; W1 fragments two K-steps ahead
  f32x4 acc[3][8];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the wave's tile count (1..3) as a compile-time constant: a run-time guard per MFMA made the
  // compiler drain every counter before each one
  auto fc1 = [&](auto nt_) {
    constexpr int NT = decltype(nt_)::value;
#pragma unroll
    for (int kk = 0; kk < 6; ++kk) {
      s16x8 an[3];
      if (kk + 2 < 6) {
#pragma unroll
        for (int i = 0; i < NT; ++i) an[i] = w1_frag(i, kk + 2);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch here (the scheduler sinks it to its use)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const s16x8 bf = *(const s16x8*)(smem + SMB_H + tile_off(128, 16 * j + c16, 4 * kk + g));
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i][j] = mfma16(af[kk & 1][i], bf, acc[i][j]);
      }
      if (kk + 2 < 6) {
#pragma unroll
        for (int i = 0; i < NT; ++i) af[kk & 1][i] = an[i];
      }
    }
  };
  if (w + 16 < ntl) fc1(std::integral_constant<int, 3>{});
  else if (w + 8 < ntl) fc1(std::integral_constant<int, 2>{});
  else if (w < ntl) fc1(std::integral_constant<int, 1>{});
  // fc2's first W2 fragments and fc1's biases, before the z / h stores
  const int og = w & 3, tg = w >> 2;
  auto w2_frag = [&](int i, int kk) -> s16x8 {
    const int row = og * 48 + 16 * i + c16, ch = 4 * kk + g;
    const bool v = row < a.Cp && ch < a.HC;
    return __builtin_bit_cast(s16x8, buf_load16(w2r, v ? (uint32_t)(row * a.Hp + ch * 8) * 2u : SR_OOB));
  };
  constexpr int W2LA = 3;  // fc2 K-steps of W2 fragments in flight
  s16x8 bf2[W2LA][3];
#pragma unroll
  for (int u = 0; u < W2LA; ++u)
#pragma unroll
    for (int i = 0; i < 3; ++i) bf2[u][i] = w2_frag(i, u);
  f32x4 bias1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int hr = 16 * (w + 8 * i) + 4 * g;
    bias1[i] = (w + 8 * i < ntl && hr < a.Hp) ? *(const f32x4*)(sB1 + hr) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();  // every wave done with the LN tile: h overwrites it
  // hidden chunks past the last computed tile read as zeros in fc2 (0 x stale LDS could be NaN)
  for (int i = tid; i < 128 * 48; i += 512) {
    const int r = i / 48, ch = i - r * 48;
    if (ch >= 2 * ntl) *(u32x4*)(smem + SMB_H + tile_off(128, r, ch)) = u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (w + 8 * i >= ntl) continue;
    const int hr = 16 * (w + 8 * i) + 4 * g;  // 4 consecutive hidden channels
    const f32x4 bias = bias1[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = 16 * j + c16, m = m0 + t;
      float zv[4], hv[4];  // zv: GELU' of the pre-activation (the aux the fc2 dgrad's gate multiplies by)
#pragma unroll
      for (int r = 0; r < 4; ++r) hv[r] = gelu_pair(hr + r < a.Hp ? acc[i][j][r] + bias[r] : 0.f, zv[r]);
      uint2 uz, uh;
      uz.x = pack_bf16x2(zv[0], zv[1]);
      uz.y = pack_bf16x2(zv[2], zv[3]);
      uh.x = pack_bf16x2(hv[0], hv[1]);
      uh.y = pack_bf16x2(hv[2], hv[3]);
      const uint32_t zo = (m < a.M && hr < a.Hp) ? (uint32_t)(m * a.Hp + hr) * 2u : SR_OOB;
      buf_store8(zr, zo, uz);
      buf_store8(hr_, zo, uh);
      *(uint2*)(smem + SMB_H + tile_off(128, t, hr >> 3) + (hr & 7) * 2) = uh;
    }
  }
  __syncthreads();  // h tile complete

  // ---- fc2: wave = 48 output channels (og) x 64 tokens (tg), K = 384 hidden (zero past Hp)
  f32x4 acc2[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 12; ++kk) {
    s16x8 bn[3];
    if (kk + W2LA < 12) {
#pragma unroll
      for (int i = 0; i < 3; ++i) bn[i] = w2_frag(i, kk + W2LA);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x8 hf = *(const s16x8*)(smem + SMB_H + tile_off(128, tg * 64 + 16 * j + c16, 4 * kk + g));
#pragma unroll
      for (int i = 0; i < 3; ++i) acc2[i][j] = mfma16(bf2[kk % W2LA][i], hf, acc2[i][j]);
    }
    if (kk + W2LA < 12) {
#pragma unroll
      for (int i = 0; i < 3; ++i) bf2[kk % W2LA][i] = bn[i];
    }
  }
  // ---- out = x2 + s2[n] * (fc2 + bias); all loads before the first store
  f32x4 bias2[3];
  uint2 xres[3][4];
  float scj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + tg * 64 + 16 * j + c16;
    scj[j] = (a.rsc && m < a.M) ? a.rsc[m / a.HW] : 1.f;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int oc = og * 48 + 16 * i + 4 * g;
    bias2[i] = oc < a.Cp ? *(const f32x4*)(sB2 + oc) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + tg * 64 + 16 * j + c16;
      xres[i][j] = buf_load8(xr, (oc < a.Cp && m < a.M) ? (uint32_t)(m * a.Cp + oc) * 2u : SR_OOB);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int oc = og * 48 + 16 * i + 4 * g;
    const f32x4 bias = bias2[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + tg * 64 + 16 * j + c16;
      const float sc = scj[j];
      const uint2 xv = xres[i][j];
      uint2 u;
      u.x = pack_bf16x2(bf16_to_f32(xv.x & 0xffff) + sc * (acc2[i][j][0] + bias[0]),
                        bf16_to_f32(xv.x >> 16) + sc * (acc2[i][j][1] + bias[1]));
      u.y = pack_bf16x2(bf16_to_f32(xv.y & 0xffff) + sc * (acc2[i][j][2] + bias[2]),
                        bf16_to_f32(xv.y >> 16) + sc * (acc2[i][j][3] + bias[3]));
      buf_store8(outr, (oc < a.Cp && m < a.M) ? (uint32_t)(m * a.Cp + oc) * 2u : SR_OOB, u);
    }
  }
}


}  // namespace

extern "C" {

int sr_swin_attn_fused_ok(int dtype, int N, int H, int W, int ws, int nH, int hd, int hdp, int C, int Cp) {
  return dtype == SR_BF16 && ws == 8 && hdp == 32 && hd <= 32 && nH >= 1 && nH * 32 <= 192 && Cp % 8 == 0 &&
         Cp <= 192 && C <= Cp && C > 0 && H % 8 == 0 && W % 8 == 0 && N > 0;
}

int sr_swin_attn_fused_fwd(const void* x, const float* ln_g, const float* ln_b, int C, float eps, const void* wqkv,
                           const float* bqkv, const float* bias_table, const void* wproj, const float* bproj,
                           const float* row_scale, int N, int H, int W, int shift, int nH, int Cp, float scale, void* x2,
                           void* ln_out, float* ln_mean, float* ln_rstd, void* qkv, void* attn_out, float* lse,
                           void* stream) {
  if (!x || !ln_g || !ln_b || !wqkv || !bqkv || !bias_table || !wproj || !bproj || !x2)
    return sr_fail(SR_EINVAL, "swin_attn_fused_fwd: null pointer");
  const bool train = qkv != nullptr;
  if (train && (!ln_out || !ln_mean || !ln_rstd || !attn_out || !lse))
    return sr_fail(SR_EINVAL, "swin_attn_fused_fwd: training needs ln_out, mean, rstd, qkv, attn_out and lse");
  if (!sr_swin_attn_fused_ok(SR_BF16, N, H, W, 8, nH, 32, 32, C, Cp) || shift < 0 || shift >= 8)
    return sr_fail(SR_EINVAL, "swin_attn_fused_fwd: bf16, window 8, head dim <= 32, nH * 32 <= 192, Cp <= 192");
  if ((size_t)N * H * W * 3 * nH * 32 * 2 >= 0x80000000ull || (size_t)N * H * W * Cp * 2 >= 0x80000000ull)
    return sr_fail(SR_ETOOBIG, "swin_attn_fused_fwd: qkv map >= 2 GiB (split the batch)");
  SabArgs a{};
  a.x = (const bf16_t*)x; a.ln_g = ln_g; a.ln_b = ln_b; a.wq = (const bf16_t*)wqkv; a.bq = bqkv;
  a.table = bias_table; a.wp = (const bf16_t*)wproj; a.bp = bproj; a.rsc = row_scale;
  a.x2 = (bf16_t*)x2; a.ln_out = (bf16_t*)ln_out; a.mean = ln_mean; a.rstd = ln_rstd;
  a.qkv = (bf16_t*)qkv; a.ao = (bf16_t*)attn_out; a.lse = lse;
  a.N = N; a.H = H; a.W = W; a.shift = shift; a.nH = nH; a.C = C; a.Cp = Cp; a.KC = Cp / 8;
  a.ldq = 3 * nH * 32; a.ldo = nH * 32;
  a.eps = eps; a.scale = scale;
  a.nwx = W / 8; a.nwin = (H / 8) * (W / 8); a.nwin_total = N * a.nwin;
  const dim3 g2((a.nwin_total + 1) / 2);
  hipStream_t s = (hipStream_t)stream;
  const int dbg = sr_knob(K_SWIN_ATTN_DBG);
  if (dbg <= 0) {  // the kernel, specialised for unshifted / shifted blocks
    if (shift) hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 0, true>), g2, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 0, false>), g2, dim3(512), 0, s, a);
    return sr_check(hipGetLastError(), "swin_attn_fused_fwd launch");
  }
  if (dbg == 32) {  // phase stamps (sr_conv3x3_set_stamps buffer: 2 x 8 per block)
    a.stamps = g_sr_stamps;
    if (!a.stamps) return sr_fail(SR_EINVAL, "swin_attn_fused_fwd: SR_SWIN_ATTN_DBG=32 needs sr_conv3x3_set_stamps");
    if (shift) hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 32, true>), g2, dim3(512), 0, s, a);
    else hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 32, false>), g2, dim3(512), 0, s, a);
    return sr_check(hipGetLastError(), "swin_attn_fused_fwd launch");
  }
  switch (dbg) {  // timing ablations (wrong results)
    case 1: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 1>), g2, dim3(512), 0, s, a); break;
    case 2: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 2>), g2, dim3(512), 0, s, a); break;
    case 4: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 4>), g2, dim3(512), 0, s, a); break;
    case 8: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 8>), g2, dim3(512), 0, s, a); break;
    case 16: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 16>), g2, dim3(512), 0, s, a); break;
    case 7: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 7>), g2, dim3(512), 0, s, a); break;
    case 31: hipLaunchKernelGGL((swin_attn_block_fwd_kernel<2, 31>), g2, dim3(512), 0, s, a); break;
    default: return sr_fail(SR_EINVAL, "swin_attn_fused_fwd: unknown SR_SWIN_ATTN_DBG ablation");
  }
  return sr_check(hipGetLastError(), "swin_attn_fused_fwd launch");
}

int sr_swin_mlp_fused_ok(int dtype, int C, int Cp, int Hp) {
  return dtype == SR_BF16 && Cp % 8 == 0 && Cp <= 192 && C > 0 && C <= Cp && Hp % 8 == 0 && Hp > 0 && Hp <= 368;
}

int sr_swin_mlp_fused_fwd(const void* x, const float* ln_g, const float* ln_b, int C, float eps, const void* w1,
                          const float* b1, const void* w2, const float* b2, const float* row_scale, int N, int HW,
                          int Cp, int Hp, void* out, void* ln_out, float* ln_mean, float* ln_rstd, void* z, void* h,
                          void* stream) {
  if (!x || !ln_g || !ln_b || !w1 || !b1 || !w2 || !b2 || !out) return sr_fail(SR_EINVAL, "swin_mlp_fused_fwd: null pointer");
  const bool train = z != nullptr;
  if (train && (!ln_out || !ln_mean || !ln_rstd || !h))
    return sr_fail(SR_EINVAL, "swin_mlp_fused_fwd: training needs ln_out, mean, rstd, z and h");
  if (!sr_swin_mlp_fused_ok(SR_BF16, C, Cp, Hp) || N <= 0 || HW <= 0)
    return sr_fail(SR_EINVAL, "swin_mlp_fused_fwd: bf16, Cp <= 192, hidden <= 368 (multiples of 8)");
  if ((size_t)N * HW * (Cp > Hp ? Cp : Hp) * 2 >= 0x80000000ull)
    return sr_fail(SR_ETOOBIG, "swin_mlp_fused_fwd: token map >= 2 GiB (split the batch)");
  SmbArgs a{};
  a.x = (const bf16_t*)x; a.ln_g = ln_g; a.ln_b = ln_b; a.w1 = (const bf16_t*)w1; a.b1 = b1;
  a.w2 = (const bf16_t*)w2; a.b2 = b2; a.rsc = row_scale; a.out = (bf16_t*)out;
  a.ln_out = (bf16_t*)ln_out; a.mean = ln_mean; a.rstd = ln_rstd; a.z = (bf16_t*)z; a.h = (bf16_t*)h;
  a.M = N * HW; a.HW = HW; a.C = C; a.Cp = Cp; a.KC = Cp / 8; a.Hp = Hp; a.HC = Hp / 8; a.eps = eps;
  const int blocks = (a.M + 127) / 128;
  hipLaunchKernelGGL(swin_mlp_block_fwd_kernel, dim3(blocks), dim3(512), 0, (hipStream_t)stream, a);
  return sr_check(hipGetLastError(), "swin_mlp_fused_fwd launch");
}

}  // extern "C"
