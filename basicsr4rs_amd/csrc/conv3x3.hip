// 3x3 / stride 1 / pad 1 convolution as an im2col-free implicit GEMM on CDNA4 MFMA.
//
// Replaces the cuDNN nn.Conv2d(C, C', 3, 1, 1) calls of the reference SR nets
// (basicsr/archs/arch_util.py:78-79, edsr_arch.py:44-48, rcan_arch.py:40-42,
// rrdbnet_arch.py:21-25): forward, data gradient (same kernel, flipped weights) and
// weight/bias gradient (split-K over pixels, deterministic slab reduction).
//
// GEMM view of the forward: rows m = output pixels (n, y, x) of the NHWC map, columns
// n = output channels, K = (tap, ci) with tap = ky*3 + kx.  The A tile of a K-step is a
// [BM pixels][128 B] slice of the input shifted by the tap (zeros outside the image come
// from the buffer range check), the B tile is [BN][128 B] of the weight rows; both are
// staged through registers into an XOR-swizzled LDS image (conflict-free ds_read_b128,
// tools/lds_banks.py) with one barrier per K-step and a double-buffered image.
// bf16 uses v_mfma_f32_16x16x32_bf16, fp32 (parity mode) v_mfma_f32_16x16x4_f32 on the
// same 16-byte chunk image.  The epilogue stages the fp32 tile through LDS and applies
// bias, activation, ReLU-mask gate, scale, residual, pixel-shuffle / NCHW store with
// 16-byte coalesced stores.
#include <cstdlib>
#include <utility>
#include <type_traits>
#include "sr_common.h"
#include "sr_internal.h"

namespace {

// set by sr_conv3x3_set_variant (tests / A-B timing): 0 auto (phase-interleaved 256x256),
// 1 never a 256x256 kernel, 2 the two-barrier 256x256 kernel (previous schedule)
int g_variant = 0;
#define g_disable_big (g_variant == 1)

struct FwdArgs {
  const void* x;
  const void* w;
  const float* bias;
  const void* gate;
  const void* res;
  const float* aff_scale;
  const float* aff_shift;
  void* y;
  uint32_t x_bytes, w_bytes, g_bytes, r_bytes;
  int N, H, W, M;
  int Cin, ldx, xcoff, in_ps, cpt;  // cpt: 16-byte chunks per tap
  int Cout, Cout_real, ldw, nkc;    // nkc: total K chunks (9*cpt)
  int ldy, ycoff, out_ps, out_nchw;
  int act;
  float slope, alpha;
  int ldg, gcoff;
  float gate_slope;
  int ldr, rcoff;
  float beta;
  const void* res2;
  uint32_t r2_bytes;
  int ldr2, r2coff, rcols;
  float beta2;
  int in_up;  // nearest-neighbour upsample factor folded into the A gather (1 = none)
  int tap0;   // 4 for 1x1 (linear) convs: the single tap is the centre one
  int gate_mode;  // 0: v *= (gate > 0 ? 1 : gate_slope); 1: v *= GELU'(gate); 2: post-residual, gcol0..gcol1
  int gcol0, gcol1;
  void* aux;      // optional store of the pre-activation value (same layout as y)
  float* colsum;  // optional per-(wave, row chunk) column sums of the stored y (see epilogue_tile)
  int tiles_n, tiles;
  FastDiv fd_cpt, fd_W, fd_H, fd_cps;  // fd_cps: divide by C' (channels per shuffle slot)
  FastDiv fd_r;                        // divide by in_ps (1 when none)
  unsigned long long* stamps;  // diagnostics: per-row clock stamps of the band kernel (null = off)
  const float* row_scale;  // optional per-image factor on alpha (SwinIR stochastic depth)
  FastDiv fd_hw;           // divide by H*W (pixel -> image)
  // LayerNorm of the input rows fused into the lin kernel's prologue (sr_linear_ln_fwd)
  const float* ln_g;
  const float* ln_b;
  void* ln_out;  // the normalised rows [M][Cin] (bf16), for the weight gradient and backward
  float* ln_mean;
  float* ln_rstd;
  int ln_C;      // channels normalised (the rest of the Cin padded columns are written as zeros)
  float ln_eps;
  const void* dot;  // band kernel, with colsum: partial sums of y * dot (sr_conv3x3_desc.dot)
  uint32_t d_bytes;
  int ldd, dcoff;
  int cs_band;  // band kernel: colsum / dot partial rows summed over the band's rows (band_cs_rows), 0: per row
  int strip64;  // pph kernel over 64-px column strips of a wider image: 256-row tiles are 4 rows x 64 px
};

// alpha of output row m: a.alpha, times the per-image row_scale when given
SR_DEV float row_alpha(const FwdArgs& a, int m) {
  return a.row_scale ? a.alpha * a.row_scale[fdiv((uint32_t)m, a.fd_hw)] : a.alpha;
}

template <typename T>
SR_DEV void mfma_chunk(const u32x4& a, const u32x4& b, f32x4& acc);

template <>
SR_DEV void mfma_chunk<bf16_t>(const u32x4& a, const u32x4& b, f32x4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a),
                                                __builtin_bit_cast(s16x8, b), acc, 0, 0, 0);
}
template <>
SR_DEV void mfma_chunk<float>(const u32x4& a, const u32x4& b, f32x4& acc) {
  // one 16-byte chunk = 4 consecutive K elements per lane: 4 f32 MFMAs (K=4 each); the
  // lane->k assignment is the same for A and B so the permuted K order sums correctly.
#pragma unroll
  for (int s = 0; s < 4; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[s]), __uint_as_float(b[s]), acc,
                                               0, 0, 0);
}

// Byte offset of chunk c of row r inside a [rows][128 B] swizzled image.
SR_DEV uint32_t swz128(uint32_t r, uint32_t c) { return r * 128u + ((c ^ (r & 7u)) << 4); }

// Fused epilogue over a [ROWS][BN] fp32 tile staged in LDS (row stride CSTR floats):
// bias, activation, gate, alpha, residual, then a plain / pixel-shuffled NHWC store of
// 8-channel (16-byte bf16 / 32-byte f32) groups, or the fp32 NCHW affine store.
template <typename T, int ROWS, int BN, int NT>
SR_DEV void epilogue_tile(const FwdArgs& a, const float* Cs, int CSTR, int m0, int n0, int tid) {
  constexpr int SZ = Elt<T>::SIZE;
  // tile row -> NHWC pixel: m0 + row, or (a.strip64: the pph kernel's column strips, tiles ordered
  // (image, strip, 4-row block)) row r of the 256-row tile is pixel (r / 64, r % 64) of its block
  int sbase = 0;
  if (a.strip64) {
    const int tm = m0 >> 8, tps = a.H >> 2, ns = a.W >> 6;
    const int img = tm / (tps * ns), rem = tm - img * tps * ns, j = rem / tps, yb = rem - j * tps;
    sbase = (img * a.H + yb * 4) * a.W + j * 64;
  }
  auto mpix = [&](int row) -> int {
    if (!a.strip64) return m0 + row;
    const int rr = (m0 & 255) + row;
    return sbase + (rr >> 6) * a.W + (rr & 63);
  };
  if (a.out_nchw) {
    float* y = (float*)a.y;
    const int HW = a.H * a.W;
    for (int idx = tid; idx < ROWS * BN; idx += NT) {
      const int row = idx % ROWS, col = idx / ROWS;
      const int m = mpix(row), n = n0 + col;
      if (m0 + row >= a.M || n >= a.Cout_real) continue;
      float v = Cs[row * CSTR + col] + (a.bias ? a.bias[n] : 0.f);
      v = act_apply(v, a.act, a.slope) * row_alpha(a, m);
      v = v * (a.aff_scale ? a.aff_scale[n] : 1.f) + (a.aff_shift ? a.aff_shift[n] : 0.f);
      const int img = m / HW, pix = m - img * HW;
      y[((size_t)img * a.Cout_real + n) * HW + pix] = v;
    }
    return;
  }
  constexpr int CG = BN / 8;  // 8-channel groups per row
  constexpr int IT = ROWS * CG / NT;  // groups per thread
  static_assert(ROWS * CG % NT == 0, "epilogue tiling");
  constexpr int NV = SZ == 2 ? 1 : 2;  // 16-B loads per 8-channel group
  const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.gate, a.g_bytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res, a.r_bytes);
  const __amdgpu_buffer_rsrc_t rr2 = make_rsrc(a.res2, a.r2_bytes);
  // per batch of IB groups: first issue every gate / residual load (range-checked buffer
  // loads: invalid groups read zeros) so their HBM latency overlaps, then compute + store.
  constexpr int IB = (SZ == 2 ? 4 : 2) < IT ? (SZ == 2 ? 4 : 2) : IT;  // groups per load batch
  static_assert(IT % IB == 0, "epilogue batch");
  // colsum: this thread's 8 channels (cg is fixed: NT % CG == 0) summed over its rows, of the
  // value as stored (bf16-rounded); reduced over the wave's lanes of the same cg below.
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  static_assert(NT % CG == 0 && 64 % CG == 0, "colsum lane map");
#pragma unroll 1
  for (int it0 = 0; it0 < IT; it0 += IB) {
  u32x4 gv[IB][NV], rv1[IB][NV], rv2[IB][NV];
#pragma unroll
  for (int ib = 0; ib < IB; ++ib) {
    const int it = ib;
    const int idx = tid + (it0 + ib) * NT;
    const int row = idx / CG, cg = idx % CG;
    const int m = mpix(row), n = n0 + cg * 8;
    const bool ok = m0 + row < a.M && n < a.Cout;
    const bool okr = ok && n < a.rcols;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (a.gate) {
        const bool gok = ok && (a.gate_mode != 2 || (n >= a.gcol0 && n < a.gcol1));
        gv[it][v] = buf_load16(gr, gok ? (uint32_t)(((size_t)m * a.ldg + a.gcoff + n) * SZ) + 16u * v : SR_OOB);
      }
      if (a.res) rv1[it][v] = buf_load16(rr, okr ? (uint32_t)(((size_t)m * a.ldr + a.rcoff + n) * SZ) + 16u * v : SR_OOB);
      if (a.res2)
        rv2[it][v] = buf_load16(rr2, okr ? (uint32_t)(((size_t)m * a.ldr2 + a.r2coff + n) * SZ) + 16u * v : SR_OOB);
    }
  }
  auto unpack = [&](const u32x4* q, float* o) {
    if constexpr (SZ == 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[2 * j] = bf16_to_f32(q[0][j] & 0xffff);
        o[2 * j + 1] = bf16_to_f32(q[0][j] >> 16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) { o[j] = __uint_as_float(q[0][j]); o[4 + j] = __uint_as_float(q[NV - 1][j]); }
    }
  };
#pragma unroll
  for (int it = 0; it < IB; ++it) {
    const int idx = tid + (it0 + it) * NT;
    const int row = idx / CG, cg = idx % CG;
    const int m = mpix(row), n = n0 + cg * 8;
    if (m0 + row >= a.M || n >= a.Cout) continue;
    float v[8];
    const f32x4 c0 = *(const f32x4*)(Cs + row * CSTR + cg * 8);
    const f32x4 c1 = *(const f32x4*)(Cs + row * CSTR + cg * 8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = c0[j]; v[4 + j] = c1[j]; }
    if (a.bias) {
      const f32x4 b0 = *(const f32x4*)(a.bias + n);
      const f32x4 b1 = *(const f32x4*)(a.bias + n + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] += b0[j]; v[4 + j] += b1[j]; }
    }
    if (a.aux) {  // activation side output (act_aux_n: GELU' for GELU, which the backward's gate reads)
      float ax[8];
      act_aux_n(v, ax, a.act, a.slope);
      const size_t da = (size_t)m * a.ldy + a.ycoff + n;
      if constexpr (SZ == 2) {
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(ax[2 * j], ax[2 * j + 1]);
        *(u32x4*)((bf16_t*)a.aux + da) = o;
      } else {
        *(f32x4*)((float*)a.aux + da) = f32x4{ax[0], ax[1], ax[2], ax[3]};
        *(f32x4*)((float*)a.aux + da + 4) = f32x4{ax[4], ax[5], ax[6], ax[7]};
      }
    } else {
      act_apply_n(v, a.act, a.slope);
    }
    if (a.gate && a.gate_mode != 2) {
      float g[8];
      unpack(gv[it], g);
      if (a.gate_mode == 1) {  // the stored GELU' (the forward's aux)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= g[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= (g[j] > 0.f ? 1.f : a.gate_slope);
      }
    }
    {
      const float al = row_alpha(a, m);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= al;
    }
    if (a.res && n < a.rcols) {
      float rv[8];
      unpack(rv1[it], rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = a.beta * rv[j] + v[j];
    }
    if (a.res2 && n < a.rcols) {
      float rv[8];
      unpack(rv2[it], rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = a.beta2 * rv[j] + v[j];
    }
    if (a.gate && a.gate_mode == 2 && n >= a.gcol0 && n < a.gcol1) {
      float g[8];
      unpack(gv[it], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= (g[j] > 0.f ? 1.f : a.gate_slope);
    }
    size_t dst;  // element offset of the 8-channel group
    if (a.out_ps == 0) {
      dst = (size_t)m * a.ldy + a.ycoff + n;
    } else {
      const int r = a.out_ps;
      const int s = (int)fdiv((uint32_t)n, a.fd_cps);
      const int c = n - s * a.fd_cps.d;
      const int si = s / r, sj = s - (s / r) * r;
      const int xq = (int)fdiv((uint32_t)m, a.fd_W);
      const int xx = m - xq * a.W;  // xq = n*H + y
      dst = ((size_t)(xq * r + si) * (a.W * r) + xx * r + sj) * a.ldy + a.ycoff + c;
    }
    if constexpr (SZ == 2) {
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      *(u32x4*)((bf16_t*)a.y + dst) = o;
      if (a.colsum) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cs[2 * j] += bf16_to_f32(o[j] & 0xffff);
          cs[2 * j + 1] += bf16_to_f32(o[j] >> 16);
        }
      }
    } else {
      *(f32x4*)((float*)a.y + dst) = f32x4{v[0], v[1], v[2], v[3]};
      *(f32x4*)((float*)a.y + dst + 4) = f32x4{v[4], v[5], v[6], v[7]};
      if (a.colsum) {
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] += v[j];
      }
    }
  }
  }
  if (a.colsum) {
    // lanes l, l ^ CG, l ^ 2CG, ... hold the same 8 channels: fixed-order butterfly, then
    // lane cg writes row (m0 / ROWS) * (NT / 64) + wave of the [parts][Cout] partial matrix.
    const int lane = tid & 63;
#pragma unroll
    for (int off = CG; off < 64; off <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) cs[j] += __shfl_xor(cs[j], off, 64);
    const int n = n0 + lane * 8;
    if (lane < CG && n < a.Cout) {
      float* dstp = a.colsum + (size_t)((m0 / ROWS) * (NT / 64) + (tid >> 6)) * a.Cout + n;
      *(f32x4*)dstp = f32x4{cs[0], cs[1], cs[2], cs[3]};
      *(f32x4*)(dstp + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256, 2) void conv3x3_fwd_kernel(FwdArgs a) {
  constexpr int PER = Elt<T>::PER16;
  constexpr int SZ = Elt<T>::SIZE;
  constexpr int MI = BM / WM / 16;
  constexpr int NI = BN / WN / 16;
  constexpr int A_CH = BM * 8 / 256;                     // A chunks per thread
  constexpr int B_CH = (BN * 8 >= 256) ? BN * 8 / 256 : 1;  // B chunks per thread
  constexpr bool B_PART = BN * 8 < 256;                   // only some threads load B
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int CSTR = BN + 4;  // epilogue fp32 row stride (floats)
  constexpr int SMEM = (2 * STAGE > BM * CSTR * 4) ? 2 * STAGE : BM * CSTR * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (int)(tile / a.tiles_n) * BM;
  const int n0 = (int)(tile % a.tiles_n) * BN;

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  // ---- per-thread A rows: pixel coordinates, fixed for the whole K loop ----
  const int cA = tid & 7;
  int ay[A_CH], ax[A_CH], anh[A_CH];  // y, x, n*H (anh < 0: row beyond M)
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int m = m0 + (tid >> 3) + 32 * i;
    if (m < a.M) {
      uint32_t q = fdiv((uint32_t)m, a.fd_W);
      ax[i] = m - (int)q * a.W;
      uint32_t n = fdiv(q, a.fd_H);
      ay[i] = (int)q - (int)n * a.H;
      anh[i] = (int)n * a.H;
    } else {
      ax[i] = 0; ay[i] = -100000; anh[i] = 0;
    }
  }
  const int bRow = tid >> 3;  // B rows bRow + 32*i

  u32x4 ra[A_CH], rb[B_CH];
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.nkc + 7) >> 3;

  auto load = [&](int ks) {
    const int q = ks * 8 + cA;  // this thread's K chunk
    const int tap_i = (int)fdiv((uint32_t)q, a.fd_cpt);
    const int cc = q - tap_i * a.cpt;
    const int tap = tap_i + a.tap0;
    const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
    const bool kval = q < a.nkc;
    const int ch = cc * PER;  // GEMM input channel of the chunk
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int yy = ay[i] + dy, xx = ax[i] + dx;
      const bool v = kval && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      uint32_t off;
      if (a.in_up > 1) {
        const int u = a.in_up;  // source grid is [N, H/u, W/u]
        off = (uint32_t)((((anh[i] / u + yy / u) * (a.W / u) + xx / u) * a.ldx + a.xcoff + ch) * SZ);
      } else if (a.in_ps == 0) {
        off = (uint32_t)((((anh[i] + yy) * a.W + xx) * a.ldx + a.xcoff + ch) * SZ);
      } else {
        const int r = a.in_ps;
        const int s = (int)fdiv((uint32_t)ch, a.fd_cps);
        const int c = ch - s * a.fd_cps.d;
        const int si = s / r, sj = s - (s / r) * r;
        const int Wr = a.W * r;
        off = (uint32_t)((((anh[i] + yy) * r + si) * Wr + xx * r + sj) * a.ldx + a.xcoff + c) * SZ;
      }
      ra[i] = buf_load16(xr, v ? off : SR_OOB);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int row = n0 + bRow + 32 * i;
      const bool v = kval && row < a.Cout && (!B_PART || tid < BN * 8);
      const uint32_t off = (uint32_t)((row * a.ldw + q * PER) * SZ);
      rb[i] = buf_load16(wr, v ? off : SR_OOB);
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * 128;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) *(u32x4*)(As + swz128((tid >> 3) + 32 * i, cA)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i)
      if (!B_PART || tid < BN * 8) *(u32x4*)(Bs + swz128(bRow + 32 * i, cA)) = rb[i];
  };
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const uint32_t c = kk * 4 + (lane >> 4);
      u32x4 fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        fa[i] = *(const u32x4*)(As + swz128(wm * (BM / WM) + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < NI; ++j)
        fb[j] = *(const u32x4*)(Bs + swz128(wn * (BN / WN) + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) mfma_chunk<T>(fa[i], fb[j], acc[i][j]);
    }
  };

  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) load(ks + 1);
    compute(ks & 1);
    if (more) store((ks + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: stage fp32 tile in LDS, then coalesced fused stores ----
  float* Cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * (BM / WM) + i * 16 + (lane >> 4) * 4 + r;
        const int col = wn * (BN / WN) + j * 16 + (lane & 15);
        Cs[row * CSTR + col] = acc[i][j][r];
      }
  __syncthreads();
  epilogue_tile<T, BM, BN, 256>(a, Cs, CSTR, m0, n0, tid);
}

// ------------------------------------------------------------------------------------
// 256 x 256 tile forward / dgrad kernel for bf16 with Cout >= 256 (EDSR-L body and
// upsample convs).  8 waves as 2 (M) x 4 (N), each wave a 128 x 64 output sub-tile
// (8 x 4 v_mfma_f32_16x16x32_bf16 accumulators).  Operands go HBM/L2 -> LDS by LDS-DMA
// (buffer_load_dwordx4 ... lds: no VGPR staging, the range check zero-fills the padding),
// two 64 KB stages in flight, each retired by a counted `s_waitcnt vmcnt` + raw s_barrier
// (cdna_hip_programming.md §5 "Pipelining across barriers").  The DMA image is lane-linear,
// so the XOR swizzle of the ds_read_b128 fragment reads is applied to the per-lane SOURCE
// chunk (rule 21).  Epilogue: the fp32 tile is staged through LDS in two 128-row halves.
// ------------------------------------------------------------------------------------
constexpr int BIG_STAGE = 65536;

__global__ __launch_bounds__(512) void conv3x3_fwd_big_kernel(FwdArgs a) {
  constexpr int MI = 8, NI = 4;
  constexpr int CSTR = 256 + 4;
  constexpr int SMEM = 128 * CSTR * 4;  // epilogue half tile; >= 2 stages of 64 KB
  static_assert(SMEM >= 2 * BIG_STAGE, "LDS too small");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (int)(tile / a.tiles_n) * 256;
  const int n0 = (int)(tile % a.tiles_n) * 256;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  // DMA image rows of this lane: w*32 + j*8 + (lane>>3), j = 0..3; logical 16-B chunk c
  const int c = (lane & 7) ^ (lane >> 3);
  int ay[4], ax[4], anh[4];
  uint32_t boff[4];
  bool bval[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = w * 32 + j * 8 + (lane >> 3);
    const int m = m0 + r;
    if (m < a.M) {
      uint32_t q = fdiv((uint32_t)m, a.fd_W);
      ax[j] = m - (int)q * a.W;
      uint32_t n = fdiv(q, a.fd_H);
      ay[j] = (int)q - (int)n * a.H;
      anh[j] = (int)n * a.H;
    } else {
      ax[j] = 0; ay[j] = -100000; anh[j] = 0;
    }
    const int n = n0 + r;
    bval[j] = n < a.Cout;
    boff[j] = (uint32_t)(n * a.ldw) * 2u + (uint32_t)c * 16u;
  }

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.nkc + 7) >> 3;

  auto issue = [&](int ks, int buf) {
    const int q = ks * 8 + c;
    const int tap_i = (int)fdiv((uint32_t)q, a.fd_cpt);
    const int cc = q - tap_i * a.cpt;
    const int tap = tap_i + a.tap0;
    const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
    const bool kval = q < a.nkc;
    const int ch = cc * 8;
    char* As = smem + buf * BIG_STAGE + w * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int yy = ay[j] + dy, xx = ax[j] + dx;
      const bool v = kval && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      uint32_t off;
      if (a.in_ps == 0) {
        off = (uint32_t)((((anh[j] + yy) * a.W + xx) * a.ldx + a.xcoff + ch) * 2);
      } else {
        const int r = a.in_ps;
        const int s = (int)fdiv((uint32_t)ch, a.fd_cps);
        const int cch = ch - s * a.fd_cps.d;
        const int si = s / r, sj = s - (s / r) * r;
        off = (uint32_t)((((anh[j] + yy) * r + si) * (a.W * r) + xx * r + sj) * a.ldx + a.xcoff + cch) * 2;
      }
      glds16(xr, As + j * 1024, v ? off : SR_OOB);
    }
    char* Bs = smem + buf * BIG_STAGE + 32768 + w * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      glds16(wr, Bs + j * 1024, (kval && bval[j]) ? boff[j] + (uint32_t)ks * 128u : SR_OOB);
  };

  auto compute = [&](int buf) {
    const char* As = smem + buf * BIG_STAGE;
    const char* Bs = As + 32768;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const uint32_t cq = kk * 4 + (lane >> 4);
      u32x4 fa[MI], fb[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *(const u32x4*)(Bs + swz128(wn * 64 + j * 16 + (lane & 15), cq));
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *(const u32x4*)(As + swz128(wm * 128 + i * 16 + (lane & 15), cq));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) mfma_chunk<bf16_t>(fa[i], fb[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    compute(ks & 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + 2 < nk) issue(ks + 2, ks & 1);
  }

  float* Cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
    if (wm == h) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(i * 16 + (lane >> 4) * 4 + r) * CSTR + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    epilogue_tile<bf16_t, 128, 256, 512>(a, Cs, CSTR, m0 + h * 128, n0, tid);
  }
}

// ------------------------------------------------------------------------------------
// 256 x 256 forward / dgrad kernel, phase-interleaved ("ping-pong") schedule.
//
// Same tile, waves, MFMA shape and LDS-DMA staging as conv3x3_fwd_big_kernel, but the
// K-step is cut into 4 phases (cdna_hip_programming.md §5 "256² 8-phase template"):
//   * LDS holds per buffer four 16 KB half-tiles A0 (tile rows 0-127), A1 (128-255),
//     B0 (cols 0-127), B1 (128-255).  Wave (wr = w>>2, wc = w&3) owns rows
//     {h*128 + wr*64 + [0,64)} x cols {g*128 + wc*32 + [0,32)}, h, g in {0, 1}, so its
//     quadrant (h, g) reads exactly half-tiles A_h and B_g.
//   * phase p of K-step t computes quadrant (0,0), (0,1), (1,1), (1,0) (16 MFMAs each)
//     and issues ONE half-tile of step t+1 (2 LDS-DMA per thread) in the order A0, B0, B1,
//     A1; a counted `s_waitcnt vmcnt(4)` keeps two half-tiles in flight across every
//     barrier and retires exactly what the next phase reads.
//   * waves 4-7 run one barrier behind waves 0-3 (stagger), so the two waves sharing a
//     SIMD alternate: one issues its fragment reads and DMA while the other runs MFMAs.
// Reads of a half-tile happen one barrier after the wait that retires it for every wave
// (two barriers for the lagging group); its slot is re-filled >= 4 phases after its last
// read.  Fragments: A 32 VGPR (one half), B 2 x 16 VGPR (both halves), acc 128 VGPR.
// ------------------------------------------------------------------------------------
SR_DEV void pp_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool FAST>
__global__ __launch_bounds__(512) void conv3x3_fwd_pp_kernel(FwdArgs a) {
  constexpr int CSTR = 256 + 4;
  constexpr int SMEM = 128 * CSTR * 4;  // epilogue half tile; >= 2 x 64 KB stages
  static_assert(SMEM >= 2 * BIG_STAGE, "LDS too small");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (int)(tile / a.tiles_n) * 256;
  const int n0 = (int)(tile % a.tiles_n) * 256;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(a.w, a.w_bytes);

  // DMA rows of this lane inside a half-tile: w*16 + j*8 + (lane>>3), j = 0, 1.
  // Index k = h*2 + j (A: tile row h*128 + ...; B: output channel n0 + g*128 + ...).
  // FAST (every 64-deep K-step inside one tap and one shuffle slot, or a 1x1 conv): the A source offset is
  // a per-lane pixel base + a wave-uniform (tap, channel) offset computed on the scalar
  // unit, and the zero padding a per-lane 9-bit mask of valid taps -- the fragment-read /
  // DMA segment of a phase then carries ~3 VALU per DMA instead of the full gather math.
  const int c = (lane & 7) ^ (lane >> 3);  // logical chunk loaded by this lane (row & 7 == lane >> 3)
  const int rps = a.in_ps > 0 ? a.in_ps : 1;
  int ay[4], ax[4], anh[4];
  uint32_t abase[4], amask[4];
  uint32_t boff[4];
  bool bval[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = (k >> 1) * 128 + w * 16 + (k & 1) * 8 + (lane >> 3);
    const int m = m0 + r;
    amask[k] = 0;
    abase[k] = 0;
    if (m < a.M) {
      uint32_t q = fdiv((uint32_t)m, a.fd_W);
      ax[k] = m - (int)q * a.W;
      uint32_t n = fdiv(q, a.fd_H);
      ay[k] = (int)q - (int)n * a.H;
      anh[k] = (int)n * a.H;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = ay[k] + t / 3 - 1, xx = ax[k] + t % 3 - 1;
        if ((unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W) amask[k] |= 1u << t;
      }
      abase[k] = (uint32_t)(((anh[k] + ay[k]) * rps * (a.W * rps) + ax[k] * rps) * a.ldx) * 2u + (uint32_t)c * 16u;
    } else {
      ax[k] = 0; ay[k] = -100000; anh[k] = 0;
    }
    const int n = n0 + r;
    bval[k] = n < a.Cout;
    boff[k] = (uint32_t)(n * a.ldw) * 2u + (uint32_t)c * 16u;
  }

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[h][g][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.nkc + 7) >> 3;
  constexpr uint32_t SLOT_A0 = 0, SLOT_A1 = 16384, SLOT_B0 = 32768, SLOT_B1 = 49152;

  // FAST: wave-uniform state of the K-step whose A half-tiles are issued next (tap,
  // channel offset inside the tap, shuffle slot), advanced once per step on the scalar unit.
  int k_tap = a.tap0, k_chu = 0, k_uoff = 0;
  auto k_eval = [&]() {
    const int dy = k_tap / 3 - 1, dx = k_tap - (k_tap / 3) * 3 - 1;
    if (a.in_ps == 0) {
      k_uoff = ((dy * a.W + dx) * a.ldx + a.xcoff + k_chu) * 2;
    } else {
      const int r = a.in_ps;
      const int sl = (int)fdiv((uint32_t)k_chu, a.fd_cps);
      const int cch = k_chu - sl * a.fd_cps.d;
      const int si = (int)fdiv((uint32_t)sl, a.fd_r), sj = sl - si * r;
      k_uoff = (((dy * r + si) * (a.W * r) + dx * r + sj) * a.ldx + a.xcoff + cch) * 2;
    }
    k_uoff = __builtin_amdgcn_readfirstlane(k_uoff);
  };
  auto k_advance = [&]() {
    k_chu += 64;
    if (k_chu == a.Cin) { k_chu = 0; ++k_tap; }
    k_eval();
  };

  // one A half-tile (h) of K-step ks: 2 DMA per thread (FAST: ks is the step k_* describes)
  auto issue_a = [&](int ks, int h) {
    char* dst = smem + (ks & 1) * BIG_STAGE + (h ? SLOT_A1 : SLOT_A0) + w * 2048;
    if constexpr (FAST) {
      const bool kv = c * 8 < a.Cin - k_chu;  // 1x1 convs: Cin need not fill the last step
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = h * 2 + j;
        glds16(xr, dst + j * 1024, (kv && ((amask[k] >> k_tap) & 1u)) ? abase[k] + (uint32_t)k_uoff : SR_OOB);
      }
    } else {
      const int q = ks * 8 + c;
      const int tap_i = (int)fdiv((uint32_t)q, a.fd_cpt);
      const int cc = q - tap_i * a.cpt;
      const int tap = tap_i + a.tap0;
      const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
      const bool kval = q < a.nkc;
      const int ch = cc * 8;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = h * 2 + j;
        const int yy = ay[k] + dy, xx = ax[k] + dx;
        const bool v = kval && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
        uint32_t off;
        if (a.in_ps == 0) {
          off = (uint32_t)((((anh[k] + yy) * a.W + xx) * a.ldx + a.xcoff + ch) * 2);
        } else {
          const int r = a.in_ps;
          const int sl = (int)fdiv((uint32_t)ch, a.fd_cps);
          const int cch = ch - sl * a.fd_cps.d;
          const int si = sl / r, sj = sl - (sl / r) * r;
          off = (uint32_t)((((anh[k] + yy) * r + si) * (a.W * r) + xx * r + sj) * a.ldx + a.xcoff + cch) * 2;
        }
        glds16(xr, dst + j * 1024, v ? off : SR_OOB);
      }
    }
  };
  auto issue_b = [&](int ks, int g) {
    const bool kval = ks * 8 + c < a.nkc;
    char* dst = smem + (ks & 1) * BIG_STAGE + (g ? SLOT_B1 : SLOT_B0) + w * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = g * 2 + j;
      glds16(wr_, dst + j * 1024, (kval && bval[k]) ? boff[k] + (uint32_t)ks * 128u : SR_OOB);
    }
  };

  u32x4 fa[2][4], fb[2][2][2];  // fa[kk][i] (current A half), fb[g][kk][j]
  auto read_a = [&](int buf, int h) {
    const char* As = smem + buf * BIG_STAGE + (h ? SLOT_A1 : SLOT_A0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[kk][i] = *(const u32x4*)(As + swz128(wr * 64 + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  };
  auto read_b = [&](int buf, int g) {
    const char* Bs = smem + buf * BIG_STAGE + (g ? SLOT_B1 : SLOT_B0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[g][kk][j] = *(const u32x4*)(Bs + swz128(wc * 32 + j * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  };
  auto mma = [&](int h, int g) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma_chunk<bf16_t>(fa[kk][i], fb[g][kk][j], acc[h][g][i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-step 0 fully issued; A0, B0 retired for every wave before the first read
  if constexpr (FAST) k_eval();
  issue_a(0, 0);
  issue_b(0, 0);
  issue_b(0, 1);
  issue_a(0, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  pp_barrier();
  if (wr) pp_barrier();  // stagger: waves 4-7 run one barrier behind

  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const bool more = t + 1 < nk;
    // phase 1: quadrant (0,0); issue A0(t+1); retire B1(t)
    read_a(buf, 0);
    read_b(buf, 0);
    if (more) {
      if constexpr (FAST) k_advance();
      issue_a(t + 1, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    pp_barrier();
    mma(0, 0);
    pp_barrier();
    // phase 2: quadrant (0,1); issue B0(t+1); retire A1(t)
    read_b(buf, 1);
    if (more) {
      issue_b(t + 1, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    mma(0, 1);
    pp_barrier();
    // phase 3: quadrant (1,1); issue B1(t+1)
    read_a(buf, 1);
    if (more) issue_b(t + 1, 1);
    pp_barrier();
    mma(1, 1);
    pp_barrier();
    // phase 4: quadrant (1,0); issue A1(t+1); retire A0(t+1), B0(t+1)
    if (more) {
      issue_a(t + 1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    pp_barrier();
    mma(1, 0);
    pp_barrier();
  }
  if (!wr) pp_barrier();  // balance the stagger

  float* Cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wr * 64 + i * 16 + (lane >> 4) * 4 + r) * CSTR + g * 128 + wc * 32 + j * 16 + (lane & 15)] =
                acc[h][g][i][j][r];
    __syncthreads();
    epilogue_tile<bf16_t, 128, 256, 512>(a, Cs, CSTR, m0 + h * 128, n0, tid);
  }
}

// ------------------------------------------------------------------------------------
// conv3x3_fwd_pph_kernel<R>: the phase-interleaved 256x256 schedule of conv3x3_fwd_pp_kernel
// with the A operand formed from input HALO rows instead of one DMA'd half-tile per tap.
// A 256-pixel tile is R whole image rows of W = 256 / R pixels (R = 4: W 64, R = 2: W 128).
// Per 64-channel chunk the R + 2 rows y0-1 .. y0+R (W + 2 px x 128 B, XOR-swizzled, the
// two border columns zero) are staged in LDS once and all 9 taps read their A fragments
// from them.  The K loop is chunk-major (chunk, tap): per K-step only the two B half-tiles
// (2 x 16 KB) and ONE halo piece per wave are issued, vs. 4 half-tiles in the pp kernel.
// Row slots form a ring: load k = (R+2)*chunk + row goes to slot k mod S, issued once the
// slot's previous row is dead (its last tap row done) and >= 2 K-steps before its first use:
//   R = 4 (S 11, rows of 1 piece per wave): at tap j < 6 of chunk c, row j of chunk c+1;
//   R = 2 (S 5, rows of 2 pieces): taps 0-1 row 3 of chunk c, 2-3 / 4-5 / 6-7 rows 0 / 1 / 2
//   of chunk c+1, tap 8 a dummy.
// Per K-step issue order: B0(t+1) [ph1], B1(t+1) [ph2], halo/dummy piece [ph3]; counted
// waits vmcnt(3) at ph1 (retires B1(t)) and ph4 (retires B0(t+1) and the older halo piece).
// ------------------------------------------------------------------------------------
constexpr int PPH_SLOT0 = 2 * 32768;
template <int R>
struct PphGeom {
  static constexpr int W = 256 / R;
  static constexpr int ROWB = (W + 2) * 128;  // px -1 .. W
  static constexpr int NSLOT = R == 4 ? 11 : 5;
  static constexpr int PIECES = W / 64;  // 1-KB pieces per wave per row
  static constexpr int ZERO = PPH_SLOT0 + NSLOT * ROWB;
  static constexpr int LDS = ZERO + 1024;
  static_assert(LDS <= 160 * 1024, "pph LDS");
};

// P2: the two-interval schedule -- per K-step each wave group runs TWO MFMA intervals of two
// quadrants each (32 MFMAs: (0,0)+(0,1), then (1,1)+(1,0)) instead of four of one, so a K-step
// costs 4 barriers instead of 8.  Reads per group: R1 = A half 0 + both B halves, R2 = A half 1;
// DMA issue: B(t+1) (both halves) in R1 -- its buffer was last read at R1 of step t-1 by both
// groups -- and the halo piece in R2, then a counted vmcnt(1) retires B(t+1) and leaves only this
// step's halo piece in flight (halo pieces retire one step after issue, as before).  Where: the
// leading group (waves 0-3) waits after issuing its second MFMA interval, the lagging group at
// the end of its R2 -- both before the barrier that precedes the leading group's next R1, so
// every wave's pieces have landed when any wave reads them, and the leading group's DMA gets one
// more interval in flight.  Each accumulator's K order is unchanged: bitwise equal to the 4-phase
// form.
// P2 == 2 additionally prefetches the B half-tiles two K-steps ahead: B(t+2) is issued in R2 of
// step t into the buffer step t just read in R1 (both groups' R1 reads complete before the barrier
// that ends R1: lgkmcnt(0)), so a weight tile has ~5 intervals in flight instead of ~3.  Per step
// the issue order is [B(t+2) 4 ops][halo(t) 1 op]; the retire point (as above) waits vmcnt(6),
// which retires B(t+2)'s predecessor B(t+1) and every older halo piece (a halo piece issued at step
// t is then visible from step t+3 on; the ring schedule's first uses are >= 4 steps after issue).
// STRIP (R 4, P2 2): images wider than 64 px (W 256 / 512: EDSR at LR 256) as 64-px column strips,
// tiles ordered (image, strip, 4-row block); each halo row also DMAs its two border columns from the
// neighbouring strips (waves 0 / 1: slot pixels 0..7 and 58..65, the overlap rewriting bytes the row's
// own pieces hold; zeros at the image edges; the other waves a zero dummy, so every halo issue is two
// ops per wave and the retire point counts 8 instead of 6), and the epilogue maps tile rows to pixels
// (FwdArgs.strip64)
template <int R, int P2 = 0, bool STRIP = false>
__global__ __launch_bounds__(512) void conv3x3_fwd_pph_kernel(FwdArgs a) {
  static_assert(!STRIP || (R == 4 && P2 == 2), "pph strips: the R 4 two-interval form");
  using G = PphGeom<R>;
  constexpr int W = G::W, RH = R + 2;
  constexpr int CSTR = 256 + 4;
  constexpr int SMEM = G::LDS > 128 * CSTR * 4 ? G::LDS : 128 * CSTR * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (int)(tile / a.tiles_n) * 256;
  const int n0 = (int)(tile % a.tiles_n) * 256;
  int img, y0, sx0 = 0;  // image, first row, first column of the tile (sx0: STRIP)
  if constexpr (STRIP) {
    const int tm = m0 >> 8, tps = a.H >> 2, ns = a.W >> 6;
    img = tm / (tps * ns);
    const int rem = tm - img * tps * ns, j = rem / tps;
    y0 = (rem - j * tps) * 4;
    sx0 = j * 64;
  } else {
    const int HW = a.H * W;
    img = m0 / HW;
    y0 = (m0 - img * HW) / W;
  }
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr_ = make_rsrc(a.w, a.w_bytes);

  const int c = (lane & 7) ^ (lane >> 3);  // logical 16-B chunk of a B row this lane moves
  const int ch_h = (lane & 7) ^ (((lane >> 3) + 1) & 7);  // halo: slot px index = px + 1
  uint32_t boff[4];
  bool bval[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int n = n0 + (k >> 1) * 128 + w * 16 + (k & 1) * 8 + (lane >> 3);
    bval[k] = n < a.Cout;
    boff[k] = (uint32_t)(n * a.ldw) * 2u + (uint32_t)c * 16u;
  }
  // halo piece p of wave w: pixels 64p + 8w .. +7 of a row.  With in_ps = r (pixel-shuffled
  // input, the upsample convs' dgrads) LR pixel (y, x) of LR channel sl * C' + cch is HR pixel
  // (y r + si, x r + sj) (sl = si r + sj) channel cch: rows r HR rows apart, pixels r apart, and a
  // per-chunk (si, sj, cch) offset instead of cc * 128
  const int rps = a.in_ps > 0 ? a.in_ps : 1;
  const uint32_t hlane = (uint32_t)((sx0 + 8 * w + (lane >> 3)) * rps * a.ldx + a.xcoff) * 2u + (uint32_t)ch_h * 16u;
  const uint32_t rowb = (uint32_t)((STRIP ? a.W : W) * rps * rps * a.ldx) * 2u;
  const uint32_t pieceb = (uint32_t)(64 * rps * a.ldx) * 2u;
  auto chunk_off = [&](int cc) -> uint32_t {
    if (a.in_ps == 0) return (uint32_t)cc * 128u;
    const int c0 = cc * 64;
    const int sl = (int)fdiv((uint32_t)c0, a.fd_cps), cch = c0 - sl * a.fd_cps.d;
    const int si = sl / rps, sj = sl - si * rps;
    return (uint32_t)((si * W * rps + sj) * a.ldx + cch) * 2u;
  };

  if (tid < 64) *(u32x4*)(smem + G::ZERO + tid * 16) = u32x4{0u, 0u, 0u, 0u};
  if (!STRIP && tid < G::NSLOT * 16) {  // border columns (slot px index 0 and W + 1) of every slot
    const int sl = tid >> 4, e = tid & 15;
    *(u32x4*)(smem + PPH_SLOT0 + sl * G::ROWB + (e < 8 ? 0 : (W + 1) * 128) + (e & 7) * 16) =
        u32x4{0u, 0u, 0u, 0u};
  }

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[h][g][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunk = a.Cin >> 6;
  const int nk = nchunk * 9;
  auto issue_dummy = [&]() { glds16(xr, smem + G::ZERO, SR_OOB); };
  auto issue_row = [&](int cc, int rr, int p) {  // piece p of row rr of chunk cc into its slot
    const int y = y0 - 1 + rr;
    const int slot = (RH * cc + rr) % G::NSLOT;
    glds16(xr, smem + PPH_SLOT0 + slot * G::ROWB + 128 + p * 8192 + w * 1024,
           (unsigned)y < (unsigned)a.H
               ? (uint32_t)(img * a.H + y) * rowb + (uint32_t)p * pieceb + hlane + chunk_off(cc)
               : SR_OOB);
    if constexpr (STRIP) {  // the strip's border columns (see the kernel comment)
      if (w < 2) {
        const int q = (w == 0 ? 0 : W - 6) + (lane >> 3);  // slot px index
        const int sx = sx0 + q - 1;
        const int lcb = (lane & 7) ^ (q & 7);
        const bool v = (unsigned)y < (unsigned)a.H && (unsigned)sx < (unsigned)a.W;
        glds16(xr, smem + PPH_SLOT0 + slot * G::ROWB + (w == 0 ? 0 : (W - 6) * 128),
               v ? (uint32_t)(((img * a.H + y) * a.W + sx) * a.ldx + a.xcoff) * 2u + (uint32_t)lcb * 16u + chunk_off(cc)
                 : SR_OOB);
      } else {
        issue_dummy();
      }
    }
  };
  auto issue_halo_dummy = [&]() {  // a halo issue's op count without a row
    issue_dummy();
    if constexpr (STRIP) issue_dummy();
  };
  // the halo piece issued at tap j of chunk cc (ring schedule above)
  auto issue_halo = [&](int cc, int j) {
    if constexpr (R == 4) {
      if (j < 6 && cc + 1 < nchunk) issue_row(cc + 1, j, 0); else issue_halo_dummy();
    } else {
      if (j < 2) issue_row(cc, 3, j);
      else if (j < 8 && cc + 1 < nchunk) issue_row(cc + 1, (j - 2) >> 1, j & 1);
      else issue_halo_dummy();
    }
  };
  // B half g of K-step (chunk kc, tap kt): weight columns kt*Cin + kc*64
  auto issue_b = [&](int buf, int kc, int kt, int g) {
    char* dst = smem + buf * 32768 + g * 16384 + w * 2048;
    const uint32_t kofs = (uint32_t)(kt * a.Cin + kc * 64) * 2u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = g * 2 + j;
      glds16(wr_, dst + j * 1024, bval[k] ? boff[k] + kofs : SR_OOB);
    }
  };
  auto issue_b_dummy = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) issue_dummy();
  };

  u32x4 fa[2][4], fb[2][2][2];
  // A half h of step (cc, ty, tx): the wave's 64 output pixels are row r, columns x0 .. x0+63
  // (R = 4: r = 2h + wr, x0 = 0; R = 2: r = h, x0 = 64 wr); they read halo row r + ty at slot px
  // index x + tx (= px + 1).  Per lane and tx the swizzled offset inside a 16-px group is
  // fixed (16 is a multiple of the 8-row swizzle period): q<tx><kk>, + i * 2048 per group.
  // (named registers, not an array: a runtime-indexed array would live in scratch, and its
  // scratch loads would make the compiler drain vmcnt -- the DMA pipeline -- at every read)
  auto qoff = [&](int tx, int kk) -> uint32_t {
    const uint32_t pxi = (uint32_t)((lane & 15) + tx);
    return pxi * 128u + ((((uint32_t)(kk * 4 + (lane >> 4))) ^ (pxi & 7u)) << 4);
  };
  const uint32_t q00 = qoff(0, 0), q01 = qoff(0, 1), q10 = qoff(1, 0), q11 = qoff(1, 1), q20 = qoff(2, 0),
                 q21 = qoff(2, 1);
  const int xoff = R == 4 ? 0 : wr * 64 * 128;
  auto read_a = [&](int slot, int tx) {
    const char* Rs = smem + PPH_SLOT0 + slot * G::ROWB + xoff;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const uint32_t qa = kk ? q01 : q00, qb = kk ? q11 : q10, qc = kk ? q21 : q20;
      const uint32_t qq = tx == 0 ? qa : (tx == 1 ? qb : qc);
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[kk][i] = *(const u32x4*)(Rs + qq + i * 2048);
    }
  };
  auto read_b = [&](int buf, int g) {
    const char* Bs = smem + buf * 32768 + g * 16384;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        fb[g][kk][j] = *(const u32x4*)(Bs + swz128(wc * 32 + j * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  };
  auto mma = [&](int h, int g) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mfma_chunk<bf16_t>(fa[kk][i], fb[g][kk][j], acc[h][g][i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: the rows chunk 0 needs first (R = 4: all six; R = 2: rows 0-2, row 3 follows
  // at taps 0-1) and both B halves of step 0, all landed
#pragma unroll 1
  for (int rr = 0; rr < (R == 4 ? 6 : 3); ++rr)
#pragma unroll
    for (int p = 0; p < G::PIECES; ++p) issue_row(0, rr, p);
  issue_b(0, 0, 0, 0);
  issue_b(0, 0, 0, 1);
  if constexpr (P2 == 2) {  // B(1) too: the loop issues B(t+2) from step 0 on
    if (nk > 1) { issue_b(1, 0, 1, 0); issue_b(1, 0, 1, 1); }  // step 1 = (chunk 0, tap 1)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr) pp_barrier();  // stagger: waves 4-7 run one barrier behind

  int cc = 0, tap = 0;   // this step
  int ncc = 0, ntap = 1;  // the next step
  int n2cc = 0, n2tap = 2;  // the step after (P2 == 2)
  if (n2tap == 9) { n2tap = 0; ++n2cc; }
#pragma unroll 1
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const bool more = t + 1 < nk;
    const int ty = tap / 3, tx = tap - ty * 3;
    int sa, sb;  // slots of this wave's rows in halves 0 / 1
    if constexpr (R == 4) {
      sa = (RH * cc + ty + wr) % G::NSLOT;
      sb = sa + 2;
    } else {
      sa = (RH * cc + ty) % G::NSLOT;
      sb = sa + 1;
    }
    if (sb >= G::NSLOT) sb -= G::NSLOT;
    if constexpr (P2 == 2) {
      // R1: A half 0, B halves 0 and 1 of this step (their reads complete before the barrier: R2
      // re-fills this buffer with B(t+2))
      read_a(sa, tx);
      read_b(buf, 0);
      read_b(buf, 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      pp_barrier();
      mma(0, 0);
      mma(0, 1);
      pp_barrier();
      // R2: A half 1; issue B(t+2) into this step's buffer, then this step's halo piece; retire B(t+1)
      read_a(sb, tx);
      if (t + 2 < nk) { issue_b(buf, n2cc, n2tap, 0); issue_b(buf, n2cc, n2tap, 1); }
      else { issue_b_dummy(); issue_b_dummy(); }
      issue_halo(cc, tap);
      if constexpr (STRIP) {  // the halo issues are two ops: [halo(t-1) 2][B(t+2) 4][halo(t) 2]
        if (wr) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        if (wr) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      pp_barrier();
      mma(1, 1);
      mma(1, 0);
      if constexpr (STRIP) {
        if (!wr) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        if (!wr) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      }
      pp_barrier();
      cc = ncc;
      tap = ntap;
      if (++ntap == 9) { ntap = 0; ++ncc; }
      if (++n2tap == 9) { n2tap = 0; ++n2cc; }
      continue;
    }
    if constexpr (P2 == 1) {
      // R1: A half 0, B halves 0 and 1 of this step; issue B(t+1) (both halves)
      read_a(sa, tx);
      read_b(buf, 0);
      read_b(buf, 1);
      if (more) { issue_b(buf ^ 1, ncc, ntap, 0); issue_b(buf ^ 1, ncc, ntap, 1); }
      else { issue_b_dummy(); issue_b_dummy(); }
      pp_barrier();
      mma(0, 0);
      mma(0, 1);
      pp_barrier();
      // R2: A half 1; issue this step's halo piece; retire B(t+1)
      read_a(sb, tx);
      issue_halo(cc, tap);
      if (wr) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      pp_barrier();
      mma(1, 1);
      mma(1, 0);
      if (!wr) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      pp_barrier();
      cc = ncc;
      tap = ntap;
      if (++ntap == 9) { ntap = 0; ++ncc; }
      continue;
    }
    // phase 1: quadrant (0,0); issue B0(t+1); retire B1(t)
    read_a(sa, tx);
    read_b(buf, 0);
    if (more) issue_b(buf ^ 1, ncc, ntap, 0); else issue_b_dummy();
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    pp_barrier();
    mma(0, 0);
    pp_barrier();
    // phase 2: quadrant (0,1); issue B1(t+1)
    read_b(buf, 1);
    if (more) issue_b(buf ^ 1, ncc, ntap, 1); else issue_b_dummy();
    pp_barrier();
    mma(0, 1);
    pp_barrier();
    // phase 3: quadrant (1,1); issue this step's halo piece
    read_a(sb, tx);
    issue_halo(cc, tap);
    pp_barrier();
    mma(1, 1);
    pp_barrier();
    // phase 4: quadrant (1,0); retire B0(t+1) (and the older halo piece)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    pp_barrier();
    mma(1, 0);
    pp_barrier();
    cc = ncc;
    tap = ntap;
    if (++ntap == 9) { ntap = 0; ++ncc; }
  }
  if (!wr) pp_barrier();  // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  float* Cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wr * 64 + i * 16 + (lane >> 4) * 4 + r) * CSTR + g * 128 + wc * 32 + j * 16 + (lane & 15)] =
                acc[h][g][i][j][r];
    __syncthreads();
    epilogue_tile<bf16_t, 128, 256, 512>(a, Cs, CSTR, m0 + h * 128, n0, tid);
  }
}

// ------------------------------------------------------------------------------------
// linear_wk_kernel<E>: 1x1 convs streamed over K -- the SwinIR fc2 forward (360 -> 184), the fc1 /
// qkv dgrads (360 / 576 -> 184), and (K <= 192) the fc2 / proj dgrads and proj forward.  A block owns
// 128 tokens x one 192-wide tile of the output channels (Cout <= 576: the tiles of one token tile are
// consecutive blocks, so its token rows are read from L2 by the second) and streams K in 64-wide steps
// through two LDS stages (LDS-DMA of the token tile [128][128 B] and the weight tile [192][128 B], both
// K-contiguous, chunk ^ (row & 7) swizzle; 40 KB a stage, so two blocks share a CU).  C = W . X^T as in
// conv3x3_lin_kernel: the weight rows are permuted on load (32-row group p, tile t, row r -> channel
// 32p + 8(r/4) + 4t + r%4), so a lane ends with 8 consecutive channels of one token and stores them as
// one 16-B vector with the fused epilogue.  4 waves (2 channel x 2 token halves), each 96 channels x
// 64 tokens (6 x 4 accumulator tiles).  (The 64-token lin kernel it replaces on wide K re-read the
// whole weight image per 64 tokens -- 434 MB of L2 reads on the qkv dgrad -- and staged all of K
// before its first MFMA.)
// E: conv3x3_lin_kernel's epilogue codes (bits 0-1 act, 2-3 gate 1 / 2 pre-residual, 4 res, 6 aux, 7
// row scale) for 0 (plain), 8 (GELU' gate: fc2 dgrad), 16 (residual), 67 (GELU + pre-activation aux:
// fc1 forward), 144 (residual + row scale); the bias
// (GEMM column order), alpha and beta always.
// ------------------------------------------------------------------------------------
template <int E>
__global__ __launch_bounds__(256, 2) void linear_wk_kernel(FwdArgs a) {
  constexpr int XI = 128 * 128, WI = 192 * 128, STAGE = XI + WI;
  constexpr int ACT = E & 3, GATE = (E >> 2) & 3;
  constexpr bool RES = (E & 16) != 0, AUX = (E & 64) != 0, RSC = (E & 128) != 0;
  static_assert(GATE != 3 && (E & ~(3 | 12 | 16 | 64 | 128)) == 0, "linear_wk: epilogue subset");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nct = (a.Cout + 191) / 192;  // output-channel tiles (consecutive blocks)
  const int bt = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int tt = bt / nct, ct = bt - tt * nct;
  const int m0 = tt * 128, n0 = ct * 192;
  const int K = a.Cin, nk = (K + 63) >> 6;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(a.w, a.w_bytes);

  // DMA pieces of 64 lanes = 8 rows x 8 chunks: per stage 16 token pieces then 24 weight pieces,
  // wave w taking pieces w, w + 4, ...; lane: row rl of the piece, physical chunk pc = logical lc ^ rl
  const int rl = lane >> 3, lc = (lane & 7) ^ rl;
  int wch[6];  // source weight channel of this lane's row in weight pieces q = 4..9
#pragma unroll
  for (int q = 4; q < 10; ++q) {
    const int row = (w + 4 * q - 16) * 8 + rl;
    const int t = (row >> 4) & 1, r = row & 15;
    wch[q - 4] = n0 + (row >> 5) * 32 + 8 * (r >> 2) + 4 * t + (r & 3);
  }
  auto issue = [&](int ks, int stg) {
    char* st = smem + stg * STAGE;
    const int kc = ks * 8 + lc;
    const bool kv = kc * 8 < K;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = w + 4 * q, m = m0 + p * 8 + rl;
      glds16(xr, st + p * 1024, (kv && m < a.M) ? (uint32_t)((m * a.ldx + a.xcoff + kc * 8) * 2) : SR_OOB);
    }
#pragma unroll
    for (int q = 4; q < 10; ++q) {
      const int p = w + 4 * q - 16, ch = wch[q - 4];
      glds16(wrs, st + XI + p * 1024, (kv && ch < a.Cout) ? (uint32_t)((ch * a.ldw + kc * 8) * 2) : SR_OOB);
    }
  };

  const int c16 = lane & 15, g = lane >> 4;
  f32x4 acc[6][4];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int stg) {
    const char* Xs = smem + stg * STAGE;
    const char* Ws = Xs + XI;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int phys = ((kk * 4 + g) ^ (c16 & 7)) << 4;  // every fragment row has row & 7 == c16 & 7
      u32x4 fa[6], fb[4];
#pragma unroll
      for (int i = 0; i < 6; ++i) fa[i] = *(const u32x4*)(Ws + (wr * 96 + i * 16 + c16) * 128 + phys);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *(const u32x4*)(Xs + (wc * 64 + j * 16 + c16) * 128 + phys);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, fa[i]),
                                                              __builtin_bit_cast(s16x8, fb[j]), acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  issue(0, 0);
  for (int ks = 0; ks < nk; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();  // step ks landed for every wave; step ks - 1's stage is free
    if (ks + 1 < nk) issue(ks + 1, (ks + 1) & 1);
    compute(ks & 1);
  }

  // ---- epilogue: pair P (tiles 2P, 2P + 1) gives channels n = n0 + (3 wr + P) * 32 + 8g .. + 7 of
  // token m0 + 64 wc + 16 j + c16
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res, a.r_bytes);
  const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.gate, a.g_bytes);
  const size_t ybytes = (size_t)a.M * a.ldy * 2;
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(a.y, ybytes < 0x80000000ull ? (uint32_t)ybytes : 0x7fffffffu);
  const __amdgpu_buffer_rsrc_t ar = make_rsrc(a.aux, AUX ? (ybytes < 0x80000000ull ? (uint32_t)ybytes : 0x7fffffffu) : 0u);
  const __amdgpu_buffer_rsrc_t br = make_rsrc(a.bias, a.bias ? (uint32_t)a.Cout * 4u : 0u);
  float alpha_blk = a.alpha;
  if constexpr (RSC) alpha_blk = a.alpha * a.row_scale[fdiv((uint32_t)m0, a.fd_hw)];
  u32x4 rv[3][4], gv[3][4];
  float bv[3][8];
#pragma unroll
  for (int P = 0; P < 3; ++P) {
    const int n = n0 + (3 * wr + P) * 32 + 8 * g;
    const u32x4 b0 = buf_load16(br, (uint32_t)n * 4u), b1 = buf_load16(br, (uint32_t)n * 4u + 16u);
#pragma unroll
    for (int r = 0; r < 4; ++r) { bv[P][r] = __uint_as_float(b0[r]); bv[P][4 + r] = __uint_as_float(b1[r]); }
    if constexpr (GATE != 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wc * 64 + j * 16 + c16;
        gv[P][j] = buf_load16(gr, (n < a.Cout && m < a.M) ? (uint32_t)(((size_t)m * a.ldg + a.gcoff + n) * 2) : SR_OOB);
      }
    }
    if constexpr (RES) {
      const bool rok = n < a.Cout && n < a.rcols;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wc * 64 + j * 16 + c16;
        rv[P][j] = buf_load16(rr, (rok && m < a.M) ? (uint32_t)(((size_t)m * a.ldr + a.rcoff + n) * 2) : SR_OOB);
      }
    }
  }
#pragma unroll
  for (int P = 0; P < 3; ++P) {
    const int n = n0 + (3 * wr + P) * 32 + 8 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wc * 64 + j * 16 + c16;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * P][j][r] + bv[P][r];
        v[4 + r] = acc[2 * P + 1][j][r] + bv[P][4 + r];
      }
      if constexpr (AUX) {  // activation side output (act_aux_n: GELU' for GELU)
        float ax[8];
        act_aux_n(v, ax, ACT, a.slope);
        u32x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = pack_bf16x2(ax[2 * q], ax[2 * q + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(o, ar, (n < a.Cout && m < a.M) ? (uint32_t)(((size_t)m * a.ldy + a.ycoff + n) * 2) : SR_OOB, 0, 0);
      } else if constexpr (ACT == 1) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.f ? v[q] : 0.f;
      } else if constexpr (ACT == 2) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = v[q] > 0.f ? v[q] : v[q] * a.slope;
      } else if constexpr (ACT == 3) {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = gelu_exact(v[q]);
      }
      if constexpr (GATE != 0) {
        float gf[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          gf[2 * q] = bf16_to_f32(gv[P][j][q] & 0xffff);
          gf[2 * q + 1] = bf16_to_f32(gv[P][j][q] >> 16);
        }
        if constexpr (GATE == 1) {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] *= gf[q] > 0.f ? 1.f : a.gate_slope;
        } else {  // the stored GELU' (the forward's aux)
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] *= gf[q];
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] *= alpha_blk;
      if constexpr (RES) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] += a.beta * bf16_to_f32(rv[P][j][q] & 0xffff);
          v[2 * q + 1] += a.beta * bf16_to_f32(rv[P][j][q] >> 16);
        }
      }
      u32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = pack_bf16x2(v[2 * q], v[2 * q + 1]);
      __builtin_amdgcn_raw_buffer_store_b128(o, yr, (n < a.Cout && m < a.M) ? (uint32_t)(((size_t)m * a.ldy + a.ycoff + n) * 2) : SR_OOB, 0, 0);
    }
  }
}

// ------------------------------------------------------------------------------------
// conv3x3_lin_kernel<MT>: 1x1 convs (nn.Linear over NHWC tokens: SwinIR qkv / proj / fc1 /
// fc2 and their dgrads, DCN column GEMMs) with a short K (<= 576).  These GEMMs are
// HBM-bound (AI ~ 100-150 FLOP/B); the 2-D tiled kernels re-read the token rows once per
// N tile and pay a full prologue / epilogue per 2-3 K-steps.  Here a block loads its MT
// token rows x all K ONCE into LDS (LDS-DMA, [K/64][MT][128 B] XOR-swizzled) and then
// sweeps every output channel, 128 per pass (32 per wave): W fragments come from L2
// straight into registers, X^T fragments from LDS, C = W x X^T so each lane ends with 8
// consecutive channels of one token (the W tile rows are permuted on load: tile t row r ->
// channel 8(r/4) + 4t + r%4) and stores 16 B directly, with the fused epilogue (bias,
// activation, pre-activation side output, gate, alpha, residuals) in registers.
// ------------------------------------------------------------------------------------
// E >= 0: the epilogue fixed at compile time (bits 0-1 act, 2-3 gate 0 none / 1 pre-residual
// (g > 0 ? 1 : gate_slope) / 2 pre-residual GELU'(g) / 3 post-residual on gcol0..gcol1, 4 res,
// 5 res2, 6 aux, 7 row_scale, uniform per block: H*W % MT == 0): its operand loads for a pass are
// issued before the pass's MFMAs, so they land under them; E = -1: run-time flags, loads next to
// their use (every combination).
template <int MT, int MAXCG, int NPASS, int E, bool LN = false>
__global__ __launch_bounds__(256, 2) void conv3x3_lin_kernel(FwdArgs a) {
  constexpr int NMT = MT / 16;  // token tiles per wave (every wave covers all MT tokens)
  constexpr bool CE = E >= 0;
  constexpr int ACT = E & 3, GATE = (E >> 2) & 3;
  constexpr bool RES = (E & 16) != 0, RES2 = (E & 32) != 0, AUX = (E & 64) != 0, RSC = (E & 128) != 0;
  __shared__ __attribute__((aligned(16))) char smem[MAXCG * MT * 128];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = (int)xcd_remap(blockIdx.x, gridDim.x) * MT;
  const int K = a.Cin, KC = K >> 3;  // 16-B chunks of a token row
  const int CG = (K + 63) >> 6;      // 128-B chunk groups
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  __shared__ float sgb[LN ? 2 * 192 : 1];  // LN: gamma, beta (channels < 192)
  if constexpr (LN) {
    for (int c = tid; c < 192; c += 256) {
      sgb[c] = c < a.ln_C ? a.ln_g[c] : 0.f;
      sgb[192 + c] = c < a.ln_C ? a.ln_b[c] : 0.f;
    }
  }
  // ---- stage the MT x K token tile: piece p = (chunk group cg, 8-row group rg)
  {
    const int npieces = CG * (MT / 8);
    const int rl = lane >> 3, pc = lane & 7;
    const int lc = pc ^ rl;  // logical chunk this lane fetches (row & 7 == rl)
    for (int p = w; p < npieces; p += 4) {
      const int cg = p / (MT / 8), rg = p - cg * (MT / 8);
      const int row = rg * 8 + rl, m = m0 + row, ch = cg * 8 + lc;
      const bool v = m < a.M && ch < KC;
      glds16(xr, smem + (cg * MT + rg * 8) * 128, v ? (uint32_t)(((size_t)m * a.ldx + a.xcoff + ch * 8) * 2) : SR_OOB);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (LN) {
    // LayerNorm of the staged rows in place (fp32 statistics, two lanes per row over alternate
    // 16-B chunks held in registers: one LDS read per chunk), gamma / beta from LDS, the
    // normalised rows also stored to ln_out with the row mean / rstd: the standalone LN kernel's
    // read of x and this kernel's read of its output become one read
    constexpr int MAXQ = MAXCG * 4;  // chunks per lane (2 lanes per row, MAXCG * 8 chunks)
    const int row = tid >> 1, half = tid & 1, m = m0 + row;
    auto chunk_ptr = [&](int ch) -> u32x4* {
      return (u32x4*)(smem + (ch >> 3) * MT * 128 + row * 128 + (((ch & 7) ^ (row & 7)) << 4));
    };
    u32x4 raw[MAXQ];
    float sm = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int ch = half + 2 * q;
      raw[q] = ch < KC ? *chunk_ptr(ch) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ch * 8 + 2 * j;
        sm += (c < a.ln_C ? bf16_to_f32(raw[q][j] & 0xffff) : 0.f) + (c + 1 < a.ln_C ? bf16_to_f32(raw[q][j] >> 16) : 0.f);
      }
    }
    sm += __shfl_xor(sm, 1);
    const float mu = sm / a.ln_C;
    float sq = 0.f;
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int ch = half + 2 * q;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = ch * 8 + 2 * j;
        const float d0 = c < a.ln_C ? bf16_to_f32(raw[q][j] & 0xffff) - mu : 0.f;
        const float d1 = c + 1 < a.ln_C ? bf16_to_f32(raw[q][j] >> 16) - mu : 0.f;
        sq += d0 * d0 + d1 * d1;
      }
    }
    sq += __shfl_xor(sq, 1);
    const float rs = rsqrtf(sq / a.ln_C + a.ln_eps);
    __syncthreads();  // gamma / beta staged (below the token DMA wait) by every wave
#pragma unroll
    for (int q = 0; q < MAXQ; ++q) {
      const int ch = half + 2 * q;
      if (ch >= KC) break;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = ch * 8 + j;
        const float xv = bf16_to_f32((raw[q][j >> 1] >> (16 * (j & 1))) & 0xffff);
        o[j] = c < a.ln_C ? (xv - mu) * rs * sgb[c] + sgb[192 + c] : 0.f;
      }
      u32x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = pack_bf16x2(o[2 * j], o[2 * j + 1]);
      *chunk_ptr(ch) = r;
      if (m < a.M) *(u32x4*)((bf16_t*)a.ln_out + (size_t)m * K + ch * 8) = r;
    }
    if (half == 0 && m < a.M) {
      a.ln_mean[m] = mu;
      a.ln_rstd[m] = rs;
    }
    __syncthreads();
  }

  const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.gate, a.g_bytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res, a.r_bytes);
  const __amdgpu_buffer_rsrc_t rr2 = make_rsrc(a.res2, a.r2_bytes);
  // output descriptors sized to the output (a lane past it stores at SR_OOB = 2^31, which must
  // fall outside the descriptor to be dropped)
  const size_t ybytes = (size_t)a.M * a.ldy * 2;
  const uint32_t yb = ybytes < 0x80000000ull ? (uint32_t)ybytes : 0x7fffffffu;
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(a.y, yb);
  const __amdgpu_buffer_rsrc_t ar = make_rsrc(a.aux, a.aux ? yb : 0u);
  // compile-time epilogue: the block's row scale (all MT tokens in one image)
  float alpha_blk = a.alpha;
  if constexpr (CE && RSC) alpha_blk = a.alpha * a.row_scale[fdiv((uint32_t)m0, a.fd_hw)];
  const int nkk = (K + 31) >> 5;
  constexpr int npass = NPASS;  // (Cout + 127) / 128, fixed so the pass loop unrolls: the
  // compiler's own vmcnt waits are then exact (a rolled loop waited vmcnt(0) for the W loads,
  // i.e. for the previous pass's output stores too)
  constexpr int MAXKK = MAXCG * 2;
  // W fragments of a whole pass (all K) in registers, the next pass's loads in flight while the
  // current pass computes: an L2 round trip per K-step would otherwise set the pace
  u32x4 wb[MAXKK][2];
  auto wload_pass = [&](int pass) {
    const int r0 = pass * 128 + w * 32 + 8 * (c16 >> 2) + (c16 & 3);
    const bool wv0 = r0 < a.Cout, wv1 = r0 + 4 < a.Cout;
#pragma unroll
    for (int kk = 0; kk < MAXKK; ++kk) {
      const int k = kk * 32 + 8 * g;
      const bool kv = kk < nkk && k < K;
      wb[kk][0] = buf_load16(wr, (wv0 && kv) ? (uint32_t)((r0 * a.ldw + k) * 2) : SR_OOB);
      wb[kk][1] = buf_load16(wr, (wv1 && kv) ? (uint32_t)(((r0 + 4) * a.ldw + k) * 2) : SR_OOB);
    }
  };
  // the bias of every pass up front: a load in the epilogue would queue behind the next pass's
  // W loads (vector memory completes in order), exposing their latency per pass
  // (buffer loads, no branch: a missing bias or channels past Cout read zeros)
  const __amdgpu_buffer_rsrc_t br = make_rsrc(a.bias, a.bias ? (uint32_t)a.Cout * 4u : 0u);
  float bva[NPASS][8];
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) {
    const uint32_t n = (uint32_t)(pass * 128 + w * 32 + 8 * g);
    const u32x4 b0 = buf_load16(br, n * 4u), b1 = buf_load16(br, n * 4u + 16u);
#pragma unroll
    for (int j = 0; j < 4; ++j) { bva[pass][j] = __uint_as_float(b0[j]); bva[pass][4 + j] = __uint_as_float(b1[j]); }
  }
  wload_pass(0);
#pragma unroll
  for (int pass = 0; pass < npass; ++pass) {
    const int nb = pass * 128 + w * 32;  // this wave's 32 channels (tile t row r -> nb + 8(r/4) + 4t + r%4)
    const int n = nb + 8 * g;
    const bool nok = n < a.Cout;
    // compile-time epilogue operands of this pass, issued now so they land under the MFMAs
    // (out-of-range lanes read zeros: buffer offsets past the descriptor)
    u32x4 gv[NMT], rv[NMT], rv2[NMT];
    if constexpr (CE) {
      const bool gok = nok && (GATE != 3 || (n >= a.gcol0 && n < a.gcol1));
      const bool rok = nok && n < a.rcols;
#pragma unroll
      for (int i = 0; i < NMT; ++i) {
        const int m = m0 + i * 16 + c16;
        const bool mok = m < a.M;
        if constexpr (GATE != 0)
          gv[i] = buf_load16(gr, (mok && gok) ? (uint32_t)(((size_t)m * a.ldg + a.gcoff + n) * 2) : SR_OOB);
        if constexpr (RES)
          rv[i] = buf_load16(rr, (mok && rok) ? (uint32_t)(((size_t)m * a.ldr + a.rcoff + n) * 2) : SR_OOB);
        if constexpr (RES2)
          rv2[i] = buf_load16(rr2, (mok && rok) ? (uint32_t)(((size_t)m * a.ldr2 + a.r2coff + n) * 2) : SR_OOB);
      }
    }
    f32x4 acc[NMT][2];
#pragma unroll
    for (int i = 0; i < NMT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < MAXKK; ++kk) {
      // a guarded body, not a break: with MAXKK 12 / 18 (wide K) a break left the loop rolled and
      // the W fragments indexed dynamically (in scratch)
      if (kk < nkk) {
      const int ch = kk * 4 + g;  // logical 16-B chunk of the X^T fragment
      // [cg][row][128 B], physical chunk = logical ^ (row & 7); row & 7 == c16 & 7 for all i
      const char* base = smem + (ch >> 3) * MT * 128 + c16 * 128 + ((((ch & 7) ^ (c16 & 7))) << 4);
      // all NMT fragments of the K step first (in flight together), then the MFMAs
      u32x4 xf[NMT];
#pragma unroll
      for (int i = 0; i < NMT; ++i) xf[i] = *(const u32x4*)(base + i * 16 * 128);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NMT; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, wb[kk][0]),
                                                            __builtin_bit_cast(s16x8, xf[i]), acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, wb[kk][1]),
                                                            __builtin_bit_cast(s16x8, xf[i]), acc[i][1], 0, 0, 0);
      }
      }
    }
    // the next pass's W fragments load while this pass's epilogue runs
    if (pass + 1 < npass) wload_pass(pass + 1);
    // ---- epilogue: lane (g, c16) holds channels nb + 8g .. +7 of token m0 + 16i + c16 and
    // stores them as one 16-B vector (4 lanes cover 64 contiguous bytes of a token row;
    // staging whole rows through LDS measured slower: 78 -> 95 us on the qkv shape)
    const float* bv = bva[pass];
    if constexpr (CE) {
      // branch-free over lanes: stores of out-of-range lanes go past the buffer descriptor
#pragma unroll
      for (int i = 0; i < NMT; ++i) {
        const int m = m0 + i * 16 + c16;
        const bool ok = nok && m < a.M;
        float v[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) { v[r] = acc[i][0][r] + bv[r]; v[4 + r] = acc[i][1][r] + bv[4 + r]; }
        if constexpr (AUX) {  // activation side output (act_aux_n: GELU' for GELU)
          float ax[8];
          act_aux_n(v, ax, ACT, a.slope);
          u32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(ax[2 * j], ax[2 * j + 1]);
          __builtin_amdgcn_raw_buffer_store_b128(o, ar,
                                                 ok ? (uint32_t)(((size_t)m * a.ldy + a.ycoff + n) * 2) : SR_OOB, 0, 0);
        } else if constexpr (ACT == 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : 0.f;
        } else if constexpr (ACT == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.slope;
        } else if constexpr (ACT == 3) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = gelu_exact(v[j]);
        }
        float gf[8];
        if constexpr (GATE != 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            gf[2 * j] = bf16_to_f32(gv[i][j] & 0xffff);
            gf[2 * j + 1] = bf16_to_f32(gv[i][j] >> 16);
          }
        }
        if constexpr (GATE == 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
        } else if constexpr (GATE == 2) {  // the stored GELU' (the forward's aux)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= gf[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= alpha_blk;
        if constexpr (RES) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] += a.beta * bf16_to_f32(rv[i][j] & 0xffff);
            v[2 * j + 1] += a.beta * bf16_to_f32(rv[i][j] >> 16);
          }
        }
        if constexpr (RES2) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[2 * j] += a.beta2 * bf16_to_f32(rv2[i][j] & 0xffff);
            v[2 * j + 1] += a.beta2 * bf16_to_f32(rv2[i][j] >> 16);
          }
        }
        if constexpr (GATE == 3) {
          if (n >= a.gcol0 && n < a.gcol1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
          }
        }
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
        __builtin_amdgcn_raw_buffer_store_b128(o, yr,
                                               ok ? (uint32_t)(((size_t)m * a.ldy + a.ycoff + n) * 2) : SR_OOB, 0, 0);
      }
      continue;
    }
    if (!nok) continue;
#pragma unroll
    for (int i = 0; i < NMT; ++i) {  // fully unrolled: acc must stay register-indexed (no scratch)
      const int m = m0 + i * 16 + c16;
      if (m >= a.M) continue;
      u32x4 gv1, rv1, rv21;
      const bool rok = n < a.rcols;
      if (a.gate) gv1 = buf_load16(gr, (a.gate_mode != 2 || (n >= a.gcol0 && n < a.gcol1))
                                           ? (uint32_t)(((size_t)m * a.ldg + a.gcoff + n) * 2) : SR_OOB);
      if (a.res) rv1 = buf_load16(rr, rok ? (uint32_t)(((size_t)m * a.ldr + a.rcoff + n) * 2) : SR_OOB);
      if (a.res2) rv21 = buf_load16(rr2, rok ? (uint32_t)(((size_t)m * a.ldr2 + a.r2coff + n) * 2) : SR_OOB);
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[r] = acc[i][0][r] + bv[r]; v[4 + r] = acc[i][1][r] + bv[4 + r]; }
      if (a.aux) {  // activation side output (act_aux_n: GELU' for GELU)
        float ax[8];
        act_aux_n(v, ax, a.act, a.slope);
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(ax[2 * j], ax[2 * j + 1]);
        *(u32x4*)((bf16_t*)a.aux + (size_t)m * a.ldy + a.ycoff + n) = o;
      } else {
        act_apply_n(v, a.act, a.slope);
      }
      if (a.gate && a.gate_mode != 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g0 = bf16_to_f32(gv1[j] & 0xffff), g1 = bf16_to_f32(gv1[j] >> 16);
          if (a.gate_mode == 1) {  // the stored GELU'
            v[2 * j] *= g0;
            v[2 * j + 1] *= g1;
          } else {
            v[2 * j] *= g0 > 0.f ? 1.f : a.gate_slope;
            v[2 * j + 1] *= g1 > 0.f ? 1.f : a.gate_slope;
          }
        }
      }
      const float al = row_alpha(a, m);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= al;
      if (a.res) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] += a.beta * bf16_to_f32(rv1[j] & 0xffff);
          v[2 * j + 1] += a.beta * bf16_to_f32(rv1[j] >> 16);
        }
      }
      if (a.res2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] += a.beta2 * bf16_to_f32(rv21[j] & 0xffff);
          v[2 * j + 1] += a.beta2 * bf16_to_f32(rv21[j] >> 16);
        }
      }
      if (a.gate && a.gate_mode == 2 && n >= a.gcol0 && n < a.gcol1) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] *= bf16_to_f32(gv1[j] & 0xffff) > 0.f ? 1.f : a.gate_slope;
          v[2 * j + 1] *= bf16_to_f32(gv1[j] >> 16) > 0.f ? 1.f : a.gate_slope;
        }
      }
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      *(u32x4*)((bf16_t*)a.y + (size_t)m * a.ldy + a.ycoff + n) = o;
    }
  }
}

// ------------------------------------------------------------------------------------
// Forward / dgrad for narrow convs (Cout <= 64: RCAN / RRDB / SRResNet bodies at W 64 or
// 128).  A block computes 256 consecutive output pixels = R = 256 / W full rows of one image
// x all Cout channels.  Per 64-channel input chunk it stages the halo rows y0-1 .. y0+R,
// cols -1 .. W of that image once in LDS by LDS-DMA (XOR-swizzled 128-B rows, zero padding
// from the range check) and forms all nine taps from it: the A fragment of tap (ty, tx) is
// the row set shifted by ty*(W+2)+tx -- x is read from L2 once per chunk instead of once per
// tap.  Each wave owns CW co tiles x PT pixel tiles and keeps its weights in registers one
// kernel row (3 taps) at a time, the next row in flight, so the weight bytes cross L2 once
// per wave and chunk, not once per tap and pixel tile.  The fp32 tile goes
// through the shared fused epilogue (bias, activation, gate, residuals, pixel shuffle).
// ------------------------------------------------------------------------------------
// DIRECT (CO_T 4, plain store, no colsum): C = W x X^T with the two co tiles of a wave
// row-permuted (tile c row r -> channel 8(r/4) + 4c + r%4), so each lane ends with 8
// consecutive channels of one pixel and the fused epilogue stores 16 B from registers -- no
// LDS staging round trip (which cost ~1/3 of the kernel at nf 64).
template <int CO_T, bool W256 = false, bool DIRECT = false, int HALF = 0>
__global__ __launch_bounds__(256, HALF ? 3 : 2) void conv3x3_fwd_halo_kernel(FwdArgs a) {
  static_assert(!DIRECT || CO_T == 4, "direct epilogue: two co tiles per wave");
  constexpr int BN = CO_T * 16;
  constexpr int CSTR = BN + 4;
  constexpr int CW = CO_T >= 4 ? CO_T / 2 : 1;  // co tiles per wave
  constexpr int WC = CO_T / CW;                  // waves along co
  constexpr int WP = 4 / WC;                     // waves along pixels
  constexpr int PT = 16 / WP;                    // 16-pixel tiles per wave
  // >= (R+2)*(W+2) rounded up to 8: 400 (W 64), 520 (W 128), 776 (W 256: HR-resolution conv_last)
  constexpr int HROWS = W256 ? 776 : 528;
  constexpr int SMEM_H = HROWS * (HALF ? 64 : 128);
  constexpr int SMEM_E = 128 * CSTR * 4;
  constexpr int SMEM = SMEM_H > SMEM_E ? SMEM_H : SMEM_E;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = w % WC, wp = w / WC;
  const int g = lane >> 4, c16 = lane & 15;
  const uint32_t tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (int)tile * 256;
  const int n0 = blockIdx.y * BN;  // co tile (Cout > 64: one block row per 64 output channels)
  const int W = a.W, H = a.H;
  const int WPAD = W + 2;
  const int R = 256 / W;
  const int HR = (R + 2) * WPAD;
  const int q0 = m0 / W;  // n*H + y0
  const int n = q0 / H, y0 = q0 - n * H;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);

  int hb[PT];  // halo row of pixel 16*(PT*wp+i) + c16 at tap (0, 0)
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int q = 16 * (PT * wp + i) + c16;
    const int rr = q / W;
    hb[i] = rr * WPAD + (q - rr * W);
  }
  f32x4 acc[PT][CW];
#pragma unroll
  for (int i = 0; i < PT; ++i)
#pragma unroll
    for (int c = 0; c < CW; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lc8 = (lane & 7) ^ (lane >> 3);  // logical 16-B chunk of this lane's DMA slot
  constexpr int CCH = HALF ? 32 : 64;        // channels per chunk
  const int nch = (a.Cin + CCH - 1) / CCH;
  const int ninstr = HALF ? (HR + 15) >> 4 : (HR + 7) >> 3;
  const int rps = a.in_ps > 0 ? a.in_ps : 1;
  for (int ch = 0; ch < nch; ++ch) {
    const int ci0 = ch * CCH;
    if (ch) __syncthreads();  // every wave is done with the previous chunk's halo
    // in_ps = r (pixel-shuffled input: the upsample convs' dgrads): LR channel sl * C' + c of LR pixel
    // (y, x) is channel c of HR pixel (y r + si, x r + sj); a 64-channel chunk lies in one slot
    int si = 0, sj = 0, cch0 = ci0;
    if (a.in_ps > 0) {
      const int sl = (int)fdiv((uint32_t)ci0, a.fd_cps);
      si = sl / rps;
      sj = sl - si * rps;
      cch0 = ci0 - sl * a.fd_cps.d;
    }
    // the chunk's upper 32 channels exist (not for Cin 32: RRDB dense dgrads).  A runtime flag
    // even for Cin 64: measured 2-3 % faster on RCAN / RRDB than the constant-folded form
    const bool khi = !HALF && ci0 + 32 < a.Cin;
    for (int k = w; k < ninstr; k += 4) {
      // HALF: 64-B rows, 4 lanes per row, chunk swizzled by (row >> 2) & 3
      const int hr = HALF ? 16 * k + (lane >> 2) : 8 * k + (lane >> 3);
      const int lc = HALF ? (lane & 3) ^ ((hr >> 2) & 3) : lc8;
      const bool cv = ci0 + lc * 8 < a.Cin;
      const int hy = hr / WPAD, hx = hr - hy * WPAD;
      const int yy = y0 - 1 + hy, xx = hx - 1;
      const bool v = cv && hr < HR && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const int pix = a.in_ps > 0 ? ((n * H + yy) * rps + si) * (W * rps) + xx * rps + sj : (n * H + yy) * W + xx;
      const uint32_t off = (uint32_t)((pix * a.ldx + a.xcoff + cch0 + lc * 8) * 2);
      glds16(xr, smem + k * 1024, v ? off : SR_OOB);
    }
    // this wave's weights, one kernel row (3 taps x 2 K halves x CW co tiles) at a time, the
    // next row loaded while the current one computes; row 0 overlaps the halo DMA
    u32x4 bw[2][3][2][CW];
    auto load_row = [&](int ty, u32x4 (&dst)[3][2][CW]) {
#pragma unroll
      for (int tx = 0; tx < 3; ++tx)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int c = 0; c < CW; ++c) {
            const int co = DIRECT ? n0 + wc * CW * 16 + 8 * (c16 >> 2) + 4 * c + (c16 & 3)
                                  : n0 + (wc * CW + c) * 16 + c16;
            const int ci = ci0 + kk * 32 + 8 * g;
            const int tap = ty * 3 + tx;
            const bool v = co < a.Cout && ci < a.Cin;
            if (kk == 0 || khi)
              dst[tx][kk][c] = buf_load16(wr, v ? (uint32_t)((co * a.ldw + tap * a.Cin + ci) * 2) : SR_OOB);
          }
    };
    load_row(0, bw[0]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // opaque 0: keeps the 9*2*PT fragment addresses from being hoisted out of the chunk loop
    // as loop invariants (they would pin ~144 VGPRs); recomputing them is ~4 VALU each
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int ty = 0; ty < 3; ++ty) {
      if (ty < 2) load_row(ty + 1, bw[(ty + 1) & 1]);
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
        const int toff = ty * WPAD + tx;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          if (kk == 1 && !khi) continue;
#pragma unroll
          for (int i = 0; i < PT; ++i) {
            const uint32_t hrow = hb[i] + z + toff;
            const u32x4 fa = *(const u32x4*)(smem + (HALF ? hrow * 64u + ((g ^ ((hrow >> 2) & 3u)) << 4)
                                                          : swz128(hrow, kk * 4 + g)));
#pragma unroll
            for (int c = 0; c < CW; ++c) {
              if constexpr (DIRECT)
                mfma_chunk<bf16_t>(bw[ty & 1][tx][kk][c], fa, acc[i][c]);
              else
                mfma_chunk<bf16_t>(fa, bw[ty & 1][tx][kk][c], acc[i][c]);
            }
          }
        }
      }
    }
  }

  if constexpr (DIRECT) {
    // lane (g, c16): channels n0 + 32 wc + 8g .. +7 of pixel m0 + 16 (PT wp + i) + c16
    const int nn = n0 + wc * 32 + 8 * g;
    if (nn >= a.Cout) return;
    const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.gate, a.g_bytes);
    const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res, a.r_bytes);
    const __amdgpu_buffer_rsrc_t rr2 = make_rsrc(a.res2, a.r2_bytes);
    float bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bv[j] = 0.f;
    if (a.bias) {
      const f32x4 b0 = *(const f32x4*)(a.bias + nn), b1 = *(const f32x4*)(a.bias + nn + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { bv[j] = b0[j]; bv[4 + j] = b1[j]; }
    }
    const bool gok = a.gate_mode != 2 || (nn >= a.gcol0 && nn < a.gcol1);
    const bool rok = nn < a.rcols;
    auto unpack8 = [](const u32x4& q, float* o) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[2 * j] = bf16_to_f32(q[j] & 0xffff);
        o[2 * j + 1] = bf16_to_f32(q[j] >> 16);
      }
    };
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int m = m0 + 16 * (PT * wp + i) + c16;
      if (m >= a.M) continue;
      u32x4 gv, rv, rv2;
      if (a.gate) gv = buf_load16(gr, gok ? (uint32_t)(((size_t)m * a.ldg + a.gcoff + nn) * 2) : SR_OOB);
      if (a.res) rv = buf_load16(rr, rok ? (uint32_t)(((size_t)m * a.ldr + a.rcoff + nn) * 2) : SR_OOB);
      if (a.res2) rv2 = buf_load16(rr2, rok ? (uint32_t)(((size_t)m * a.ldr2 + a.r2coff + nn) * 2) : SR_OOB);
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[r] = acc[i][0][r] + bv[r]; v[4 + r] = acc[i][1][r] + bv[4 + r]; }
      if (a.aux) {  // activation side output (act_aux_n: GELU' for GELU)
        float ax[8];
        act_aux_n(v, ax, a.act, a.slope);
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(ax[2 * j], ax[2 * j + 1]);
        *(u32x4*)((bf16_t*)a.aux + (size_t)m * a.ldy + a.ycoff + nn) = o;
      } else {
        act_apply_n(v, a.act, a.slope);
      }
      float gf[8];
      if (a.gate) unpack8(gv, gf);
      if (a.gate && a.gate_mode == 1) {  // the stored GELU'
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gf[j];
      } else if (a.gate && a.gate_mode == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
      }
      const float al = row_alpha(a, m);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= al;
      if (a.res && rok) {
        float rf[8];
        unpack8(rv, rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a.beta * rf[j] + v[j];
      }
      if (a.res2 && rok) {
        float rf[8];
        unpack8(rv2, rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = a.beta2 * rf[j] + v[j];
      }
      if (a.gate && a.gate_mode == 2 && gok) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
      }
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      *(u32x4*)((bf16_t*)a.y + (size_t)m * a.ldy + a.ycoff + nn) = o;
    }
    return;
  }
  float* Cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int row = 16 * (PT * wp + i) - 128 * h;  // pixel tile origin inside half h
      if (row >= 0 && row < 128) {
#pragma unroll
        for (int c = 0; c < CW; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(row + 4 * g + r) * CSTR + (wc * CW + c) * 16 + c16] = acc[i][c][r];
      }
    }
    __syncthreads();
    epilogue_tile<bf16_t, 128, BN, 256>(a, Cs, CSTR, m0 + h * 128, n0, tid);
  }
}

// ------------------------------------------------------------------------------------
// Narrow-conv forward / dgrad, row-streaming persistent form (bf16 3x3, Cin 32 or 64,
// Cout 32 or 64, W 64 or 128: RCAN / SRResNet bodies, RRDB conv1 and dgrads into 64 ch).
//
// The tile kernel above loads a halo, computes and stores in one pass per block, so with one
// wave of blocks the chip runs the three phases one after the other (RCAN conv at B 32:
// 24 us, of which 8 us store tail and ~5 us load burst; the MFMA work is ~4.6 us per SIMD).
// Here a block owns a band of consecutive output rows (one row = W pixels of one image; the
// NHWC rows of all images are one contiguous sequence) and streams it: input rows live in an
// (LA + 2)-slot LDS ring (slot = global row % S, W + 2 swizzled 128-B pixel rows, zero border
// columns written once); row s + LA is DMA'd while row s is computed, the residual / gate
// operands of row s are DMA'd into per-wave staging before its MFMAs (each lane reads back its
// own 16 B), and its stores drain while later rows compute.  Rows outside an image (the 3x3
// zero padding in y) are never read: the taps that would read them are skipped (wave-uniform
// test per row).  Each wave keeps ALL its weights (32 output channels x 9 taps x Cin) in
// registers for the whole band, loaded once.
// MFMA as the DIRECT halo epilogue: C = W x X^T with row-permuted weight tiles, so each lane
// ends with 8 consecutive channels of one pixel and stores 16 B; colsum (RCAN avg-pool)
// partial rows per (image row, pixel wave).
// vmcnt bookkeeping per wave: per row [NG staging pieces] [PPW row pieces] .. MFMAs ..
// vmcnt(PPW) (staging landed) [PT stores] [NC colsum stores]; before row s the count of vector
// memory ops younger than row s + 1's pieces is known in closed form (prologue rows, then the
// steady state (PT + NC) + (LA - 2) * ops-per-row) and waited with a run-time vmcnt.
// ------------------------------------------------------------------------------------
// s_waitcnt vmcnt(n) for a run-time n (wave-uniform): the immediate is chosen by a binary
// search over 0..63 (6 scalar branches; a linear compare chain cost ~40 cycles per step at one
// wave per SIMD); n > 63 waits for vmcnt(63), which only waits longer.
template <int LO, int HI>
SR_DEV void vm_wait_bs(int n) {
  if constexpr (LO == HI) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LO) : "memory");
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (n <= MID) vm_wait_bs<LO, MID>(n);
    else vm_wait_bs<MID + 1, HI>(n);
  }
}
SR_DEV void vm_wait_dyn(int n) { vm_wait_bs<0, 63>(n < 0 ? 0 : (n > 63 ? 63 : n)); }

// E (the epilogue, fixed at compile time: at one wave per SIMD every run-time branch of a
// per-row epilogue is exposed): bits 0-1 act, 2-3 gate (0 none, 1 pre-residual (g > 0 ? 1 :
// gate_slope), 2 pre-residual GELU'(g), 3 post-residual (g > 0 ? 1 : gate_slope) on output
// channels gcol0..gcol1), 4 res, 5 res2, 6 aux, 7 colsum, 8 row_scale, 9 dot (with 7: the partial
// sums are of y * dot, the dot operand staged like the residuals).
// blocks per CU the band kernel is built for: two for the W 64 forms whose ring + staging fit
// 80 KB of LDS and 256 registers (no second staging operand), one otherwise.  And (round 6) the RCAB
// conv1 dgrad with the dot epilogue (656: residual + dot staging, 82 KB): not for a second band block
// but so that it shares a CU with a side-stream ring wgrad block (78 KB) as the plain residual form
// does -- at one block per CU (the weight image beside the ring, 154 KB) it held whole CUs against the
// side stream and RCAN ran 35.6 vs 33.6 ms
constexpr int band_occ(int W, int E) {
  return W == 64 && (E == 0 || E == 1 || E == 2 || E == 4 || E == 16 || E == 128 || E == 656) ? 2 : 1;
}
// NWV: waves per block, 4 (one per SIMD) or 8 (two per SIMD, each with half the row's pixel
// tiles, so one wave's epilogue and LDS waits overlap the other's MFMAs; the ring and the weight
// image shared).  8 at W 128: RRDB 63.8 -> 61.0 ms; at W 64 (one pixel tile per wave) RCAN
// 33.8 -> 37.0 ms, so 4 there.
template <int CO, int W, int LA, int KH, int E, int NWV = 4>
__global__ __launch_bounds__(NWV * 64, NWV == 8 ? 2 : band_occ(W, E)) void conv3x3_fwd_band_kernel(FwdArgs a) {
  constexpr int ACT = E & 3, GATE = (E >> 2) & 3;
  constexpr bool RES = (E & 16) != 0, RES2 = (E & 32) != 0, AUX = (E & 64) != 0, CS = (E & 128) != 0,
                 RSC = (E & 256) != 0, DOT = (E & 512) != 0, STRIP = (E & 1024) != 0;
  static_assert(!DOT || CS, "band: dot partials need colsum");
  static_assert(!STRIP || (!CS && !RSC), "band: column strips carry no per-image epilogue");
  constexpr int IR = GATE ? 1 : 0, IR2 = IR + (RES ? 1 : 0), ID = IR2 + (RES2 ? 1 : 0), NSTG = ID + (DOT ? 1 : 0);
  static_assert(NWV == 4 || (NWV == 8 && W / 16 / (8 / (CO / 32)) >= 1), "band: a pixel tile per wave");
  constexpr int WC = CO / 32;       // waves along output channels (32 each = 2 co tiles)
  constexpr int WP = NWV / WC;      // waves along the row's pixels
  constexpr int PT = W / 16 / WP;   // 16-pixel tiles per wave
  constexpr int WPAD = W + 2;
  constexpr int SLOT = WPAD * 128;
  constexpr int S = LA + 2;         // ring slots: rows s-1 .. s+1 read, s+2 .. s+LA in flight
  constexpr int PPW = W / 8 / NWV;  // 1-KB DMA pieces per wave per row
  constexpr int NG = NSTG * PT;     // staging pieces per wave per row (gate / res / res2)
  constexpr int NC = (CS ? 2 : 0) + (AUX ? PT : 0);  // stores after the PT output stores
  constexpr int PPWX = PPW + (STRIP ? 1 : 0);  // + the strip's border piece (or a dummy) per wave
  constexpr int KROW = NG + PPWX + PT + NC;           // vector memory ops per wave per row
  // per-wave staging (none for the wide strip forms without epilogue operands, CO > 64: their LDS is
  // the weight image's)
  constexpr int EPI = (NSTG ? NSTG : (CO > 64 ? 0 : 1)) * PT * 1024;
  constexpr int CIN = 32 * KH;
  constexpr int WROW = 9 * CIN * 2;  // bytes of one output channel's weights [tap][ci]
  constexpr int WBYTES = CO * WROW;
  constexpr int RING = (S + 1) * SLOT + NWV * EPI;
  // ring + one all-zero slot (the rows above / below an image read it, so the MFMA sequence has
  // no branches) + staging; the weight image after them where both fit (WSEP: the ring prologue
  // is issued before the weights are waited for; only forms built for one block per CU: the extra
  // LDS would cost the W 64 forms their second block and RCAN 2.7 ms), else in the same space
  // before the ring starts
  constexpr bool WSEP = band_occ(W, E) == 1 && RING + WBYTES <= 160 * 1024;
  __shared__ __attribute__((aligned(16))) char smem[WSEP ? RING + WBYTES : (RING > WBYTES ? RING : WBYTES)];
  char* const wimg = smem + (WSEP ? RING : 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = w % WC, wp = w / WC;
  const int g = lane >> 4, c16 = lane & 15;
  const int H = a.H;
  // STRIP (E bit 10): the image is a.W = strips x W pixels wide and each band row is one W-px column
  // strip of an image row, strip rows ordered (image, strip, y) so a band streams down a strip; the
  // strip's two border columns are real pixels of its neighbours (one extra 1-KB piece per row from
  // waves 0 / 1, a zero dummy from the others), and with in_up = 2 the pieces gather the nearest
  // upsample of a half-size input
  const int strips = STRIP ? a.W / W : 1;
  const int HS = H * strips;
  const int T = a.N * HS;  // output rows (strip rows)
  struct RowG { size_t base; int y, irow, x0; };  // first pixel, y, image row n*H + y, strip x origin
  auto row_geom = [&](int q) -> RowG {
    if constexpr (!STRIP) {
      return RowG{(size_t)q * W, q % H, q, 0};
    } else {
      const int nq = q / HS, rem = q - nq * HS, j = rem / H, y = rem - j * H;
      return RowG{(size_t)(nq * H + y) * a.W + j * W, y, nq * H + y, j * W};
    }
  };
  const int upsh = STRIP && a.in_up == 2 ? 1 : 0;
  // input offset (bytes, chunk lc) of pixel sx of image row irow (STRIP)
  auto src_off = [&](int irow, int sx, int lc) -> uint32_t {
    const size_t px = (size_t)(irow >> upsh) * (a.W >> upsh) + (sx >> upsh);
    return (uint32_t)((px * a.ldx + a.xcoff + lc * 8) * 2);
  };
#ifdef SR_BAND_STAMPS
  const unsigned long long t_start = __builtin_readcyclecounter();
  unsigned long long ph[4] = {0ull, 0ull, 0ull, 0ull};  // row wait / barrier / MFMA / epilogue
#endif
  const int G = gridDim.x;
  const int bb = blockIdx.x;
  const int s0 = (int)((int64_t)bb * T / G), s1 = (int)((int64_t)(bb + 1) * T / G);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.gate, a.g_bytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.res, a.r_bytes);
  const __amdgpu_buffer_rsrc_t rr2 = make_rsrc(a.res2, a.r2_bytes);
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(a.dot, a.d_bytes);

  // weights: one coalesced LDS-DMA image [co][tap][ci] (1 KB contiguous per wave instruction),
  // then each wave reads its MFMA fragments from it: co = wc*32 + 8*(c16>>2) + 4*c + (c16&3)
  // (DIRECT row permutation), K chunk kk*32 + 8*g of every tap
  for (int p = w; p < WBYTES / 1024; p += NWV) {
    const int e = p * 1024 + lane * 16;
    const int co = e / WROW, off = e - co * WROW;
    if constexpr (STRIP) {  // Cin may be 8 / 16 / 24 below CIN (the RRDBNet conv_last dgrad): zero-padded per tap
      const int tap = off / (CIN * 2), cib = off - tap * (CIN * 2);
      glds16(wr, wimg + p * 1024, cib < a.Cin * 2 ? (uint32_t)(co * a.ldw * 2 + tap * a.Cin * 2 + cib) : SR_OOB);
    } else {
      glds16(wr, wimg + p * 1024, (uint32_t)(co * a.ldw * 2 + off));
    }
  }
  const int nn = wc * 32 + 8 * g;  // this lane's 8 output channels
  float bv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bv[j] = 0.f;
  if (a.bias) {
    const f32x4 b0 = *(const f32x4*)(a.bias + nn), b1 = *(const f32x4*)(a.bias + nn + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { bv[j] = b0[j]; bv[4 + j] = b1[j]; }
  }
  float rsv = a.alpha;  // RSC: alpha * row_scale of image s0 / H + lane (a band spans < 64 images)
  if constexpr (RSC) {
    const int ni = s0 / H + lane;
    rsv = ni < a.N ? a.alpha * a.row_scale[ni] : 0.f;
  }
  u32x4 bw[9][2][2];
  auto read_weights = [&]() {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int co = wc * 32 + 8 * (c16 >> 2) + 4 * c + (c16 & 3);
          bw[tap][kk][c] = kk < KH ? *(const u32x4*)(wimg + co * WROW + (tap * CIN + kk * 32 + 8 * g) * 2)
                                   : u32x4{0u, 0u, 0u, 0u};
        }
    // every fragment in registers (and the compiler knows it) before the ring overwrites the image
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int c = 0; c < 2; ++c) asm volatile("" ::"v"(bw[tap][kk][c]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  auto zero_borders = [&]() {  // pixel rows 0 and W + 1 of every slot (STRIP: DMA'd per row), and the zero slot S
    for (int i = tid; i < (STRIP ? 0 : S * 2 * 8); i += NWV * 64) {
      const int sl = i >> 4, side = (i >> 3) & 1, ch = i & 7;
      *(u32x4*)(smem + sl * SLOT + (side ? (W + 1) * 128 : 0) + ch * 16) = u32x4{0u, 0u, 0u, 0u};
    }
    for (int i = tid; i < SLOT / 16; i += NWV * 64) *(u32x4*)(smem + S * SLOT + i * 16) = u32x4{0u, 0u, 0u, 0u};
  };
  if constexpr (!WSEP) {
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(bv[j]));
    asm volatile("" ::"v"(rsv));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    read_weights();
    __syncthreads();
    zero_borders();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    zero_borders();  // disjoint from the weight image and from the pixel rows the prologue DMAs
  }
#ifdef SR_BAND_STAMPS
  const unsigned long long t_loaded = __builtin_readcyclecounter();
#endif

  // DMA of global row q (pixels 1..W of slot q % S); rows outside [0, T) read zeros
  const int lc_lane = lane & 7;
  auto issue_row = [&](int q) {
    char* slot = smem + (q % S) * SLOT;
    const bool qv = q >= 0 && q < T;
    RowG rg{};
    if constexpr (STRIP) rg = row_geom(q);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int k = w * PPW + j;            // piece: pixel rows 1 + 8k .. 8 + 8k
      const int px = 1 + 8 * k + (lane >> 3);
      const int lc = lc_lane ^ (px & 7);    // logical 16-B chunk landing in physical slot lane & 7
      const bool v = qv && lc * 8 < a.Cin;
      uint32_t off;
      if constexpr (STRIP) off = src_off(rg.irow, rg.x0 + px - 1, lc);
      else off = (uint32_t)((((size_t)q * W + (px - 1)) * a.ldx + a.xcoff + lc * 8) * 2);
      glds16(xr, slot + (1 + 8 * k) * 128, v ? off : SR_OOB);
    }
    if constexpr (STRIP) {
      // wave 0: slot pixels 0..7 (the left border, 1..7 again as piece 0 has them), wave 1: W-6..W+1
      // (W+1 the right border): a rewrite of the same bytes is harmless.  The image's outer columns
      // load as zeros (OOB).  Other waves: one zero dummy into the zero slot (uniform vmcnt counts).
      if (w < 2) {
        const int pb = w == 0 ? 0 : W - 6;
        const int px = pb + (lane >> 3);
        const int lc = lc_lane ^ (px & 7);
        const int sx = rg.x0 + px - 1;
        const bool v = qv && (unsigned)sx < (unsigned)a.W && lc * 8 < a.Cin;
        glds16(xr, slot + pb * 128, v ? src_off(rg.irow, sx, lc) : SR_OOB);
      } else {
        glds16(xr, smem + S * SLOT, SR_OOB);
      }
    }
  };
  const bool gok = GATE != 3 || (nn >= a.gcol0 && nn < a.gcol1);
  const bool rok = nn < a.rcols;
  auto unpack8 = [](const u32x4& q, float* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = bf16_to_f32(q[j] & 0xffff);
      o[2 * j + 1] = bf16_to_f32(q[j] >> 16);
    }
  };
  char* epi = smem + (S + 1) * SLOT + w * EPI;
  // gate / res / res2 of this wave's pixels of output row q into its staging buffer (NG ops)
  auto issue_staging = [&](int q) {
    const bool qv = q < T;
    const size_t mb = row_geom(q).base;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const size_t m = mb + wp * PT * 16 + i * 16 + c16;
      if constexpr (GATE != 0)
        glds16(gr, epi + i * 1024, qv && gok ? (uint32_t)((m * a.ldg + a.gcoff + nn) * 2) : SR_OOB);
      if constexpr (RES)
        glds16(rr, epi + (IR * PT + i) * 1024, qv && rok ? (uint32_t)((m * a.ldr + a.rcoff + nn) * 2) : SR_OOB);
      if constexpr (RES2)
        glds16(rr2, epi + (IR2 * PT + i) * 1024, qv && rok ? (uint32_t)((m * a.ldr2 + a.r2coff + nn) * 2) : SR_OOB);
      if constexpr (DOT)
        glds16(dr, epi + (ID * PT + i) * 1024, qv ? (uint32_t)((m * a.ldd + a.dcoff + nn) * 2) : SR_OOB);
    }
  };
  // prologue: rows s0 - 1 .. s0 + LA - 1 (s0 - 1 first: the oldest), then row s0's staging
  if (s0 < s1) {
    for (int q = s0 - 1; q < s0 + LA; ++q) issue_row(q);
    issue_staging(s0);
  }
  if constexpr (WSEP) {
    // this wave's weight pieces landed (older than the (LA + 1) * PPW + NG prologue ops just
    // issued), then every wave's; the zeros visible to every wave
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(bv[j]));
    asm volatile("" ::"v"(rsv));
    vm_wait_dyn(s0 < s1 ? (LA + 1) * PPWX + NG : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    read_weights();
  }
  const int n0 = s0 / H;
  float cst[8];  // band-reduced channel sums (a.cs_band)
#pragma unroll
  for (int j = 0; j < 8; ++j) cst[j] = 0.f;

  // Per row, in issue order: [MFMAs] [epilogue] [staging of row s + 1: NG] [pieces of row
  // s + LA: PPW] [stores: PT + NC].  Vector memory ops complete in issue order, so a wait for
  // one op is a wait for every older one: the row pieces and the staging are issued after the
  // epilogue, so neither wait below ever covers the stores or the DMA of the row just issued.
#pragma unroll 1
  for (int s = s0; s < s1; ++s) {
#ifdef SR_BAND_STAMPS
    const unsigned long long t0 = __builtin_readcyclecounter();
#endif
    // rows <= s + 1 landed: the ops issued after row s + 1's pieces may stay in flight
    if (s + 1 >= s0 + LA) {
      constexpr int STEADY = (PT + NC) + (LA - 2) * KROW;
      static_assert(STEADY <= 63, "band: too many vector memory ops in flight for vmcnt");
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEADY) : "memory");
    } else {
      vm_wait_dyn((s0 + LA - 2 - s) * PPWX + NG + (s - s0) * KROW);
    }
#ifdef SR_BAND_STAMPS
    const unsigned long long t1 = __builtin_readcyclecounter();
#endif
    // every wave's pieces of row s + 1 are in LDS, and every wave is done with row s - 2,
    // whose slot row s + LA reuses (S = LA + 2)
    pp_barrier();
#ifdef SR_BAND_STAMPS
    const unsigned long long t2 = __builtin_readcyclecounter();
#endif
    const RowG rgs = row_geom(s);
    const int n_img = STRIP ? 0 : s / H, y = rgs.y;

    f32x4 acc[PT][2];
#pragma unroll
    for (int i = 0; i < PT; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int sl1 = s % S;
    const int sl0 = y == 0 ? S : (sl1 == 0 ? S - 1 : sl1 - 1);      // zero slot above an image
    const int sl2 = y == H - 1 ? S : (sl1 == S - 1 ? 0 : sl1 + 1);  // ... and below it
    const char* srows[3] = {smem + sl0 * SLOT, smem + sl1 * SLOT, smem + sl2 * SLOT};
    // K steps (tap, K half) in order.  Fragment reads run FD - 1 K steps ahead of the MFMAs.  They
    // are inline-asm ds_reads with hand-counted lgkmcnt waits that pass the fragments through (so
    // no MFMA can be scheduled before its wait): the compiler otherwise sinks every read to just
    // before its use and exposes the full LDS latency per 2 MFMAs (one wave per SIMD has nothing
    // else to run).
    constexpr int NK = 9 * KH;
    constexpr int FD = PT >= 8 ? 2 : 5;  // 8 pixel tiles (CO 256 over 8 waves): 2 K steps of fragments
    u32x4 fa[FD][PT];
    uint32_t rbase[3];
#pragma unroll
    for (int ty = 0; ty < 3; ++ty)
      rbase[ty] = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)srows[ty];
    auto read_k = [&](int k, u32x4 (&dst)[PT]) {
      const int tap = k / KH, kk = k % KH, ty = tap / 3, tx = tap % 3;
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const uint32_t ad = rbase[ty] + swz128(wp * PT * 16 + i * 16 + c16 + tx, kk * 4 + g);
        asm volatile("ds_read_b128 %0, %1" : "=v"(dst[i]) : "v"(ad));
      }
    };
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < FD - 1; ++k) read_k(k, fa[k]);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if (k + FD - 1 < NK) read_k(k + FD - 1, fa[(k + FD - 1) % FD]);
      const int ahead = (NK - 1 - k < FD - 1 ? NK - 1 - k : FD - 1) * PT;  // reads issued after step k's
      u32x4* f = fa[k % FD];
      if constexpr (PT == 1) {
        switch (ahead) {
          case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0])); break;
          case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(f[0])); break;
          case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f[0])); break;
          case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(f[0])); break;
          default: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0])); break;
        }
      } else if constexpr (PT == 2) {
        switch (ahead) {
          case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1])); break;
          case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f[0]), "+v"(f[1])); break;
          case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1])); break;
          case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(f[0]), "+v"(f[1])); break;
          default: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1])); break;
        }
      } else if constexpr (PT == 8) {
        if (ahead == 0)
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]),
                       "+v"(f[6]), "+v"(f[7]));
        else
          asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]),
                       "+v"(f[6]), "+v"(f[7]));
      } else {
        switch (ahead) {
          case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])); break;
          case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])); break;
          case 8: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])); break;
          case 12: asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])); break;
          default: asm volatile("s_waitcnt lgkmcnt(15)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3])); break;
        }
      }
      const int tap = k / KH, kk = k % KH;
#pragma unroll
      for (int i = 0; i < PT; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c) mfma_chunk<bf16_t>(bw[tap][kk][c], f[i], acc[i][c]);
    }
    // The compiler interleaves the epilogue's accumulator reads with the last MFMAs and, on a
    // branchy path, once left too few wait states between the final MFMA and the read of its
    // result (acc[PT-1][1][3] came out stale).  Fence the MFMA block and pad it.
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#ifdef SR_BAND_STAMPS
    const unsigned long long t3 = __builtin_readcyclecounter();
#endif

    // this row's staging landed (issued before row s + LA - 1's pieces and row s - 1's stores)
    if constexpr (NG > 0) {
      if (s == s0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPWX + PT + NC) : "memory");
    }
    float rs = a.alpha;
    if constexpr (RSC) rs = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, rsv), n_img - n0));
    float cs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cs[j] = 0.f;
    u32x4 ov[PT], avx[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) { v[r] = acc[i][0][r] + bv[r]; v[4 + r] = acc[i][1][r] + bv[4 + r]; }
      if constexpr (AUX) {  // activation side output (act_aux_n: GELU' for GELU)
        float ax[8];
        act_aux_n(v, ax, ACT, a.slope);
#pragma unroll
        for (int j = 0; j < 4; ++j) avx[i][j] = pack_bf16x2(ax[2 * j], ax[2 * j + 1]);
      } else if constexpr (ACT == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : 0.f;
      } else if constexpr (ACT == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = v[j] > 0.f ? v[j] : v[j] * a.slope;
      } else if constexpr (ACT == 3) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = gelu_exact(v[j]);
      }
      float gf[8];
      if constexpr (GATE != 0) unpack8(*(const u32x4*)(epi + i * 1024 + lane * 16), gf);
      if constexpr (GATE == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
      } else if constexpr (GATE == 2) {  // the stored GELU'
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= gf[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= rs;
      if constexpr (RES) {
        float rf[8];
        unpack8(*(const u32x4*)(epi + (IR * PT + i) * 1024 + lane * 16), rf);
        if (rok) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = a.beta * rf[j] + v[j];
        }
      }
      if constexpr (RES2) {
        float rf[8];
        unpack8(*(const u32x4*)(epi + (IR2 * PT + i) * 1024 + lane * 16), rf);
        if (rok) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = a.beta2 * rf[j] + v[j];
        }
      }
      if constexpr (GATE == 3) {
        if (gok) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] *= gf[j] > 0.f ? 1.f : a.gate_slope;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ov[i][j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      if constexpr (CS && DOT) {  // y as stored times the dot operand
        float df[8];
        unpack8(*(const u32x4*)(epi + (ID * PT + i) * 1024 + lane * 16), df);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cs[2 * j] += bf16_to_f32(ov[i][j] & 0xffff) * df[2 * j];
          cs[2 * j + 1] += bf16_to_f32(ov[i][j] >> 16) * df[2 * j + 1];
        }
      } else if constexpr (CS) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          cs[2 * j] += bf16_to_f32(ov[i][j] & 0xffff);
          cs[2 * j + 1] += bf16_to_f32(ov[i][j] >> 16);
        }
      }
    }
    if constexpr (NG > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read before refill
    issue_staging(s + 1);
    issue_row(s + LA);
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const size_t m = rgs.base + wp * PT * 16 + i * 16 + c16;
      *(u32x4*)((bf16_t*)a.y + m * a.ldy + a.ycoff + nn) = ov[i];
    }
    if constexpr (AUX) {
#pragma unroll
      for (int i = 0; i < PT; ++i) {
        const size_t m = rgs.base + wp * PT * 16 + i * 16 + c16;
        *(u32x4*)((bf16_t*)a.aux + m * a.ldy + a.ycoff + nn) = avx[i];
      }
    }
    if constexpr (CS) {
      // the 16 lanes of a g group hold the same 8 channels: fixed-order butterfly, then lane
      // c16 == 0 writes partial row s * WP + wp (P = H * WP rows per image) -- or, band-reduced
      // (a.cs_band: every band is a.cs_band rows of one image), the running sum over the band's rows
      // so far to partial row bb * WP + wp, so the last row's store leaves the band's sum
      // (P = H / cs_band * WP rows per image; same-address stores of one wave land in order)
      // Band-reduced: each lane keeps its own sums over the band's rows and the butterfly runs once, at
      // the band's last row (it costs ~1300 cycles per row at one wave per SIMD: 32 cross-lane moves in
      // 4 dependent rounds); the rows before store the lane's unreduced running sum to the same
      // address, which the last row's store overwrites (the two stores per row keep the vmcnt counts)
      if (a.cs_band) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { cst[j] += cs[j]; cs[j] = cst[j]; }
        if (s + 1 == s1) {
#pragma unroll
          for (int off = 1; off < 16; off <<= 1)
#pragma unroll
            for (int j = 0; j < 8; ++j) cs[j] += __shfl_xor(cs[j], off, 64);
        }
      } else {
#pragma unroll
        for (int off = 1; off < 16; off <<= 1)
#pragma unroll
          for (int j = 0; j < 8; ++j) cs[j] += __shfl_xor(cs[j], off, 64);
      }
      float* dstp = a.colsum + ((size_t)(a.cs_band ? bb : s) * WP + wp) * a.Cout + nn;
      // exactly two vector store instructions per wave (lanes masked): counted in NC
      if (c16 == 0) *(f32x4*)dstp = f32x4{cs[0], cs[1], cs[2], cs[3]};
      if (c16 == 0) *(f32x4*)(dstp + 4) = f32x4{cs[4], cs[5], cs[6], cs[7]};
    }
#ifdef SR_BAND_STAMPS
    const unsigned long long t4 = __builtin_readcyclecounter();
    ph[0] += t1 - t0; ph[1] += t2 - t1; ph[2] += t3 - t2; ph[3] += t4 - t3;
#endif
  }
#ifdef SR_BAND_STAMPS
  if (a.stamps && tid == 0) {
    unsigned long long* st = a.stamps + (size_t)blockIdx.x * 16;
    st[0] = t_start; st[1] = t_loaded; st[2] = __builtin_readcyclecounter(); st[3] = s1 - s0;
    st[4] = ph[0]; st[5] = ph[1]; st[6] = ph[2]; st[7] = ph[3];
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing row pieces (zeros past T) land before exit
}

// ------------------------------------------------------------------------------------
// HR tail convs (conv_last: Cout <= 16, NCHW fp32 store, W >= 256, Cin 64..256): row streaming
// over 32-px column strips.  A block owns (image, strip, band of RB rows); per output row ONE new
// input row (34 px x Cin, per 64-ch chunk a [40 px][128 B] swizzled image) is DMA'd into a ring
// of LA + 2 slots, LA rows ahead, so x crosses HBM ~once (the one-row halo tiles read it three
// times).  The waves split K by 64-channel chunk (NW = Cin / 64 chunks; with fewer chunks they
// split the two 16-px tiles), keep their chunk's weights in registers, and combine their partial
// sums through LDS; the fused tail epilogue (bias, activation, alpha, NCHW affine) stores 4
// consecutive pixels of one channel per lane.
// ------------------------------------------------------------------------------------
template <int NW>
__global__ __launch_bounds__(256, 1) void conv3x3_fwd_tail_kernel(FwdArgs a) {
  constexpr int LA = 3, S = LA + 2;
  constexpr int CHB = 40 * 128;         // one 64-ch chunk of a ring row (34 px used)
  constexpr int SLOT = NW * CHB;
  constexpr int PPR = NW * 5;           // 1-KB pieces per row
  constexpr int PPW = (PPR + 3) / 4;    // per wave (padded with dummies: uniform vmcnt counts)
  constexpr int G = 4 / NW;             // wave groups over the two px tiles
  constexpr int NT = G == 1 ? 2 : 1;    // px tiles per wave
  constexpr int PART = 4 * NT * 64 * 16;  // one partial-sum buffer
  __shared__ __attribute__((aligned(16))) char smem[S * SLOT + 2 * PART + 1024];
  char* part = smem + S * SLOT;
  char* dummy = part + 2 * PART;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c16 = lane & 15;
  const int H = a.H, W = a.W;
  const int strips = W >> 5, RB = a.tiles;
  const int bands = (H + RB - 1) / RB;
  int b = (int)blockIdx.x;
  const int band = b % bands; b /= bands;
  const int strip = b % strips;
  const int n = b / strips;
  const int x0 = strip * 32, y0 = band * RB, y1 = min(H, y0 + RB);
  const int chunk = w % NW, grp = w / NW;
  const bool mma_on = G < 4 || grp < 2;  // Cin 64: waves 2, 3 only move data
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, a.w_bytes);
  const int STO = w < 2 ? 1 : 0;        // waves 0, 1 store one vector per row (tiles 0, 1)

  // this wave's weights: co = c16, K chunk kk*32 + 8g of its 64-ch chunk, all taps
  u32x4 bw[9][2];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ci = chunk * 64 + kk * 32 + 8 * g;
      bw[tap][kk] = buf_load16(wr, c16 < a.Cout ? (uint32_t)((c16 * a.ldw + tap * a.Cin + ci) * 2) : SR_OOB);
    }
  // the epilogue's per-channel constants (loads here, not in the row loop: they would count in
  // the row loop's vmcnt bookkeeping)
  const int co = c16;
  const bool cok = co < a.Cout_real;
  const float ebias = (a.bias && cok) ? a.bias[co] : 0.f;
  const float escale = (a.aff_scale && cok) ? a.aff_scale[co] : 1.f;
  const float eshift = (a.aff_shift && cok) ? a.aff_shift[co] : 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) asm volatile("" ::"v"(bw[tap][kk]));
  asm volatile("" ::"v"(ebias), "v"(escale), "v"(eshift));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // DMA of input row yy (outside [0, H): zeros) into its ring slot: piece p = (chunk p / 5,
  // px rows 8 (p % 5) ..); physical 16-B slot lane & 7 of px row r holds logical chunk
  // (lane & 7) ^ (r & 7)
  auto issue_row = [&](int yy) {
    char* slot = smem + ((yy - (y0 - 1)) % S) * SLOT;
    const bool yv = (unsigned)yy < (unsigned)H;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int p = w + 4 * j;
      const int c = p / 5, q = p - c * 5;
      const int px = 8 * q + (lane >> 3);
      const int lc = (lane & 7) ^ (px & 7);
      const int xx = x0 - 1 + px;
      const bool v = p < PPR && yv && px < 34 && (unsigned)xx < (unsigned)W;
      const uint32_t off = (uint32_t)(((((size_t)n * H + yy) * W + xx) * a.ldx + a.xcoff + c * 64 + lc * 8) * 2);
      glds16(xr, p < PPR ? slot + c * CHB + q * 1024 : dummy, v ? off : SR_OOB);
    }
  };
  for (int yy = y0 - 1; yy < y0 + LA; ++yy) issue_row(yy);

#pragma unroll 1
  for (int y = y0; y < y1; ++y) {
    const int s = y - y0;
    // rows <= y + 1 landed (ops issued after row y + 1's pieces may stay in flight)
    if (s + 1 >= LA) {
      if (STO) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(1 + (LA - 2) * (PPW + 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LA - 2) * PPW) : "memory");
    } else {
      vm_wait_dyn((LA - 2 - s) * PPW + s * (PPW + STO));  // issued after row y + 1: rows y + 2 .. y0 + LA, stores
    }
    __syncthreads();
    issue_row(y + LA);  // its slot held row y - 2, done by every wave (barrier above)
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (mma_on) {
#pragma unroll
      for (int ty = 0; ty < 3; ++ty) {
        const char* row = smem + ((y - 1 + ty - (y0 - 1)) % S) * SLOT + chunk * CHB;
#pragma unroll
        for (int tx = 0; tx < 3; ++tx)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const int tile = G == 1 ? t : grp;
              const u32x4 fa = *(const u32x4*)(row + swz128(tile * 16 + c16 + tx, kk * 4 + g));
              mfma_chunk<bf16_t>(fa, bw[ty * 3 + tx][kk], acc[t]);
            }
      }
    }
    f32x4* pb = (f32x4*)(part + (s & 1) * PART);
#pragma unroll
    for (int t = 0; t < NT; ++t) pb[(w * NT + t) * 64 + lane] = acc[t];
    __syncthreads();
    if (tid < 128) {  // (tile, lane): px tile * 16 + 4g + r, channel c16
      const int t = tid >> 6;
      f32x4 v;
      if constexpr (G == 1) v = pb[(0 * 2 + t) * 64 + lane] + pb[(1 * 2 + t) * 64 + lane] +
                                pb[(2 * 2 + t) * 64 + lane] + pb[(3 * 2 + t) * 64 + lane];
      else if constexpr (G == 2) v = pb[(t * 2 + 0) * 64 + lane] + pb[(t * 2 + 1) * 64 + lane];
      else v = pb[t * 64 + lane];
      if (cok) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = act_apply(v[r] + ebias, a.act, a.slope) * a.alpha * escale + eshift;
        float* yp = (float*)a.y + (((size_t)n * a.Cout_real + co) * H + y) * W + x0 + t * 16 + 4 * g;
        *(f32x4*)yp = f32x4{o[0], o[1], o[2], o[3]};
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // trailing row pieces land before exit
}

// ------------------------------------------------------------------------------------
// Weight gradient.  GEMM per tap: C[co][ci] = sum_p dy[p][co] * x[p + tap][ci] over a
// K-range of pixels (split-K).  LDS images are [pixels][cols] (rows = K); MFMA operands
// need 8 consecutive K per lane, read with ds_read_b64_tr_b16 (bf16) or ds_read_b32
// (f32).  Partial tiles go to an fp32 slab ws[split][tap][co][ci]; blocks of the centre
// tap and first ci tile also emit the bias-gradient partial sums.
// ------------------------------------------------------------------------------------
struct WgArgs {
  const void* dy;
  const void* x;
  float* ws;    // [S][9][Cout][Cin]
  float* wsb;   // [S][Cout]
  uint32_t dy_bytes, x_bytes;
  int N, H, W, M;
  int Cin, ldx, xcoff;
  int Cout, ldy, ycoff, out_ps;
  int in_up;  // nearest upsample factor of the x gather (1 = none)
  int taps, tap0;  // 9 / 0 for 3x3, 1 / 4 for 1x1 (linear)
  int tiles_co, tiles_ci, splits, kper;  // kper: pixels per split (multiple of KSTEP)
  int bias_group;  // pp kernel: > 0 = the bias-role blocks come after all tile blocks, each doing this many splits
  int bias_fused;  // pp kernel: no bias-role blocks; the centre-tap, first-ci-tile blocks sum dy as well
  FastDiv fd_W, fd_H, fd_cps;
  unsigned long long* stamps;  // diagnostics (SR_BAND_STAMPS builds): per-block phase cycles
};

// 32-byte-block XOR swizzle for the [K rows][256 B] tr-read image (tools/lds_banks.py):
// the 8 rows a 32-lane half reads ({0..3, 8..11} + base) land on 8 distinct blocks.
SR_DEV uint32_t swz_tr(uint32_t row, uint32_t byte_in_row, uint32_t row_bytes) {
  const uint32_t f = (row & 3u) | (((row >> 3) & 1u) << 2);
  const uint32_t blk = (byte_in_row >> 5) ^ (f & ((row_bytes >> 5) - 1));
  return row * row_bytes + (blk << 5) + (byte_in_row & 31u);
}

template <typename T, int BMW, int BNW, int WM, int WN>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_kernel(WgArgs a) {
  constexpr int PER = Elt<T>::PER16;
  constexpr int SZ = Elt<T>::SIZE;
  constexpr bool BF = (SZ == 2);
  constexpr int KSTEP = BF ? 64 : 32;  // pixels per K-step
  constexpr int MI = BMW / WM / 16;
  constexpr int NI = BNW / WN / 16;
  constexpr int ARB = BMW * SZ;  // bytes per A row (one pixel's co tile)
  constexpr int BRB = BNW * SZ;
  constexpr int ACPR = ARB / 16, BCPR = BRB / 16;  // chunks per row
  constexpr int ACH = KSTEP * ACPR, BCH = KSTEP * BCPR;  // chunks per tile
  constexpr int A_PT = (ACH + 255) / 256, B_PT = (BCH + 255) / 256;
  constexpr int STAGE = KSTEP * (ARB + BRB);
  constexpr int SMEM = 2 * STAGE > 256 * 8 * 4 ? 2 * STAGE : 256 * 8 * 4;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // block -> (split, tap, co tile, ci tile); splits outermost so concurrent blocks share
  // the same pixel range (dy / x rows re-read from L2).
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int per_split = a.taps * a.tiles_co * a.tiles_ci;
  const int split = (int)b / per_split;
  int rem = (int)b - split * per_split;
  const int tap = rem / (a.tiles_co * a.tiles_ci);
  rem -= tap * a.tiles_co * a.tiles_ci;
  const int co0 = (rem / a.tiles_ci) * BMW;
  const int ci0 = (rem % a.tiles_ci) * BNW;
  const int etap = tap + a.tap0;
  const int dy_ = etap / 3 - 1, dx_ = etap % 3 - 1;
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const bool do_bias = (etap == 4) && (ci0 == 0) && a.wsb != nullptr;

  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);

  u32x4 ra[A_PT], rb[B_PT];
  float bacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto pix_decomp = [&](int p, int& nh, int& y, int& x) {
    uint32_t q = fdiv((uint32_t)p, a.fd_W);
    x = p - (int)q * a.W;
    uint32_t n = fdiv(q, a.fd_H);
    y = (int)q - (int)n * a.H;
    nh = (int)n * a.H;
  };

  auto load = [&](int p0) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int c = tid + 256 * i;
      const int row = c / ACPR, cc = c % ACPR;
      const int p = p0 + row;
      const int co = co0 + cc * PER;
      bool v = (c < ACH) && p < p_end && co < a.Cout;
      uint32_t off = SR_OOB;
      if (v) {
        if (a.out_ps == 0) {
          off = (uint32_t)(((size_t)p * a.ldy + a.ycoff + co) * SZ);
        } else {
          int nh, y, x;
          pix_decomp(p, nh, y, x);
          const int r = a.out_ps;
          const int s = (int)fdiv((uint32_t)co, a.fd_cps);
          const int cch = co - s * a.fd_cps.d;
          const int si = s / r, sj = s - (s / r) * r;
          off = (uint32_t)((((size_t)((nh + y) * r + si) * (a.W * r) + x * r + sj) * a.ldy + a.ycoff + cch) * SZ);
        }
      }
      ra[i] = buf_load16(dyr, off);
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int c = tid + 256 * i;
      const int row = c / BCPR, cc = c % BCPR;
      const int p = p0 + row;
      const int ci = ci0 + cc * PER;
      bool v = (c < BCH) && p < p_end && ci < a.Cin;
      uint32_t off = SR_OOB;
      if (v) {
        int nh, y, x;
        pix_decomp(p, nh, y, x);
        const int yy = y + dy_, xx = x + dx_;
        if ((unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W) {
          const int u = a.in_up;
          off = (uint32_t)(((size_t)((nh / u + yy / u) * (a.W / u) + xx / u) * a.ldx + a.xcoff + ci) * SZ);
        }
      }
      rb[i] = buf_load16(xr, off);
    }
  };
  auto bias_accum = [&]() {
    // every A chunk a thread loads covers the same 8 (or 4) channels across K-steps
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      if (BF) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bacc[2 * j] += bf16_to_f32(ra[i][j] & 0xffff);
          bacc[2 * j + 1] += bf16_to_f32(ra[i][j] >> 16);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) bacc[j] += __uint_as_float(ra[i][j]);
      }
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + KSTEP * ARB;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int c = tid + 256 * i;
      if (c < ACH) {
        const int row = c / ACPR, cc = c % ACPR;
        const uint32_t o = BF ? swz_tr(row, cc * 16, ARB) : (uint32_t)(row * ARB + cc * 16);
        *(u32x4*)(As + o) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int c = tid + 256 * i;
      if (c < BCH) {
        const int row = c / BCPR, cc = c % BCPR;
        const uint32_t o = BF ? swz_tr(row, cc * 16, BRB) : (uint32_t)(row * BRB + cc * 16);
        *(u32x4*)(Bs + o) = rb[i];
      }
    }
  };
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + KSTEP * ARB;
    if constexpr (BF) {
      const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        s16x8 fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int col = wm * (BMW / WM) + i * 16 + 4 * p;  // co column of this lane's address
          const int r0 = kk * 32 + 8 * g + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(As + swz_tr(r0, col * 2, ARB)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(As + swz_tr(r0 + 4, col * 2, ARB)));
          fa[i] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int col = wn * (BNW / WN) + j * 16 + 4 * p;
          const int r0 = kk * 32 + 8 * g + q;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Bs + swz_tr(r0, col * 2, BRB)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(Bs + swz_tr(r0 + 4, col * 2, BRB)));
          fb[j] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    } else {
      const int k = lane >> 4, c16 = lane & 15;
#pragma unroll 4
      for (int ks = 0; ks < KSTEP; ks += 4) {
        float fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i)
          fa[i] = *(const float*)(As + (ks + k) * ARB + (wm * (BMW / WM) + i * 16 + c16) * 4);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          fb[j] = *(const float*)(Bs + (ks + k) * BRB + (wn * (BNW / WN) + j * 16 + c16) * 4);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  const int nk = (p_end - p_begin + KSTEP - 1) / KSTEP;
  if (nk > 0) {
    load(p_begin);
    if (do_bias) bias_accum();
    store(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) load(p_begin + (ks + 1) * KSTEP);
    compute(ks & 1);
    if (more) {
      if (do_bias) bias_accum();
      store((ks + 1) & 1);
    }
    __syncthreads();
  }

  // partial tile -> slab ws[split][tap][co][ci]; C/D layout: row = co, col = ci
  float* ws = a.ws + ((size_t)split * a.taps + tap) * a.Cout * a.Cin;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * (BMW / WM) + i * 16 + (lane >> 4) * 4 + r;
        const int ci = ci0 + wn * (BNW / WN) + j * 16 + (lane & 15);
        if (co < a.Cout && ci < a.Cin) ws[(size_t)co * a.Cin + ci] = acc[i][j][r];
      }

  if (do_bias) {
    float* red = (float*)smem;  // [256][8]
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bacc[j];
    __syncthreads();
    if (tid < BMW) {
      const int cc = tid / PER, j = tid % PER;
      float s = 0.f;
      // threads whose A chunks are chunk cc of a row: tid' with (tid' + 256 i) % ACPR == cc
      for (int t2 = 0; t2 < 256; ++t2)
        if ((t2 % ACPR) == cc && t2 < ACH) s += red[t2 * 8 + j];
      if (co0 + tid < a.Cout) a.wsb[(size_t)split * a.Cout + co0 + tid] = s;
    }
  }
}

// ------------------------------------------------------------------------------------
// 256 (co) x 256 (ci) weight-gradient tile per tap for bf16, Cout >= 256 and Cin >= 256.
// Same LDS-DMA pipeline as conv3x3_fwd_big_kernel: the [64 pixels][256 ch] images of dy and
// of the tap-shifted x arrive by buffer_load ... lds (two 64 KB stages, counted vmcnt, raw
// barriers); MFMA operands need 8 consecutive pixels per lane and are read transposed
// with ds_read_b64_tr_b16 from 32-byte-block XOR-swizzled 512-byte rows (the swizzle is
// applied to the per-lane DMA source chunk).  The bias gradient of the centre-tap blocks
// is one extra MFMA per A fragment against an all-ones B operand (dy^T . 1).
// ------------------------------------------------------------------------------------
SR_DEV uint32_t swz512(uint32_t row, uint32_t byte_in_row) {
  const uint32_t f = (row & 3u) | (((row >> 3) & 1u) << 2);
  return row * 512u + ((((byte_in_row >> 5) ^ f)) << 5) + (byte_in_row & 31u);
}

// Bias-gradient role of the wgrad launch: the [64 pixels][256 co] dy image of each K-step
// (same LDS-DMA pipeline, A operand only) times an all-ones B operand on MFMA.
SR_DEV void wgrad_bias_role(const WgArgs& a, char* smem, int split, int co0) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  constexpr int STAGE = 2 * 64 * 512;
  int lc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int R = 8 * w + 2 * j + (lane >> 5);
    const int f = (R & 3) | (((R >> 3) & 1) << 2);
    lc[j] = ((((lane & 31) >> 1) ^ f) << 1) | (lane & 1);
  }
  auto issue = [&](int p0, int buf) {
    char* As = smem + buf * STAGE + w * 4096;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int R = 8 * w + 2 * j + (lane >> 5);
      const int p = p0 + R;
      const bool pv = p < p_end;
      const int pc = pv ? p : 0;
      const int co = co0 + lc[j] * 8;
      uint32_t off;
      if (a.out_ps == 0) {
        off = (uint32_t)((pc * a.ldy + a.ycoff + co) * 2);
      } else {
        uint32_t q = fdiv((uint32_t)pc, a.fd_W);
        const int x = pc - (int)q * a.W;
        const int r = a.out_ps;
        const int s = (int)fdiv((uint32_t)co, a.fd_cps);
        const int cch = co - s * a.fd_cps.d;
        const int si = s / r, sj = s - (s / r) * r;
        off = (uint32_t)((((int)q * r + si) * (a.W * r) + x * r + sj) * a.ldy + a.ycoff + cch) * 2;
      }
      glds16(dyr, As + j * 1024, (pv && co < a.Cout) ? off : SR_OOB);
    }
  };
  const s16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const int nk = (p_end - p_begin + 63) / 64;
  if (nk > 0) issue(p_begin, 0);
  if (nk > 1) issue(p_begin + 64, 1);
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* As = smem + (ks & 1) * STAGE;
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = kk * 32 + 8 * g + q;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = w * 32 + i * 16 + 4 * pp;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + swz512(r0, col * 2)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + swz512(r0 + 4, col * 2)));
        const s16x8 fa = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, ones, accb[i], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + 2 < nk) issue(p_begin + (ks + 2) * 64, ks & 1);
  }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + w * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (co < a.Cout) a.wsb[(size_t)split * a.Cout + co] = accb[i][r];
      }
  }
}

__global__ __launch_bounds__(512) void conv3x3_wgrad_big_kernel(WgArgs a) {
  constexpr int MI = 8, NI = 4;
  constexpr int STAGE = 2 * 64 * 512;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  // block -> (split, role): roles 0 .. 9*tco*tci-1 are (tap, co tile, ci tile) GEMM tiles,
  // the last tco roles (present only when db is wanted) are bias-gradient blocks.
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.taps * a.tiles_co * a.tiles_ci;
  const int per_split = ntile + (a.wsb ? a.tiles_co : 0);
  const int split = (int)b / per_split;
  int rem = (int)b - split * per_split;
  if (rem >= ntile) {
    wgrad_bias_role(a, smem, split, (rem - ntile) * 256);
    return;
  }
  const int tap = rem / (a.tiles_co * a.tiles_ci);
  rem -= tap * a.tiles_co * a.tiles_ci;
  const int co0 = (rem / a.tiles_ci) * 256;
  const int ci0 = (rem % a.tiles_ci) * 256;
  const int etap = tap + a.tap0;
  const int dy_ = etap / 3 - 1, dx_ = etap % 3 - 1;
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);

  // DMA rows of this lane: R_j = 8w + 2j + (lane >> 5); logical 16-B chunk lc_j (source swizzle)
  int lc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int R = 8 * w + 2 * j + (lane >> 5);
    const int f = (R & 3) | (((R >> 3) & 1) << 2);
    lc[j] = ((((lane & 31) >> 1) ^ f) << 1) | (lane & 1);
  }

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int p0, int buf) {
    char* As = smem + buf * STAGE + w * 4096;
    char* Bs = As + 32768;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int R = 8 * w + 2 * j + (lane >> 5);
      const int p = p0 + R;
      const bool pv = p < p_end;
      const int pc = pv ? p : 0;
      uint32_t q = fdiv((uint32_t)pc, a.fd_W);
      const int x = pc - (int)q * a.W;
      uint32_t n = fdiv(q, a.fd_H);
      const int y = (int)q - (int)n * a.H;
      const int co = co0 + lc[j] * 8;
      uint32_t offa;
      if (a.out_ps == 0) {
        offa = (uint32_t)((pc * a.ldy + a.ycoff + co) * 2);
      } else {
        const int r = a.out_ps;
        const int s = (int)fdiv((uint32_t)co, a.fd_cps);
        const int cch = co - s * a.fd_cps.d;
        const int si = s / r, sj = s - (s / r) * r;
        offa = (uint32_t)((((int)q * r + si) * (a.W * r) + x * r + sj) * a.ldy + a.ycoff + cch) * 2;
      }
      glds16(dyr, As + j * 1024, (pv && co < a.Cout) ? offa : SR_OOB);
      const int yy = y + dy_, xx = x + dx_;
      const int ci = ci0 + lc[j] * 8;
      const bool bv = pv && ci < a.Cin && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      const uint32_t offb = (uint32_t)((((int)q + dy_) * a.W + xx) * a.ldx + a.xcoff + ci) * 2;
      glds16(xr, Bs + j * 1024, bv ? offb : SR_OOB);
    }
  };

  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + 32768;
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = kk * 32 + 8 * g + q;
      s16x8 fa[MI], fb[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int col = wn * 64 + j * 16 + 4 * pp;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + swz512(r0, col * 2)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(Bs + swz512(r0 + 4, col * 2)));
        fb[j] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int col = wm * 128 + i * 16 + 4 * pp;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + swz512(r0, col * 2)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s16x4*)(As + swz512(r0 + 4, col * 2)));
        fa[i] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  };

  const int nk = (p_end - p_begin + 63) / 64;
  if (nk > 0) issue(p_begin, 0);
  if (nk > 1) issue(p_begin + 64, 1);
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    compute(ks & 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ks + 2 < nk) issue(p_begin + (ks + 2) * 64, ks & 1);
  }

  float* ws = a.ws + ((size_t)split * a.taps + tap) * a.Cout * a.Cin;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
        const int ci = ci0 + wn * 64 + j * 16 + (lane & 15);
        if (co < a.Cout && ci < a.Cin) ws[(size_t)co * a.Cin + ci] = acc[i][j][r];
      }
}

// ------------------------------------------------------------------------------------
// Weight gradient, phase-interleaved 256x256 (co x ci) tile: the schedule of
// conv3x3_fwd_pp_kernel applied to the per-tap GEMM over pixels.  Half-tiles are
// [64 pixels][128 channels] images (256-B rows, 32-B-block swizzle, ds_read_b64_tr_b16
// operand reads): A_h = dy channels co0 + h*128.., B_g = x channels ci0 + g*128.. at the
// tap-shifted pixel.  Needs W % 64 == 0 (a 64-pixel K-step is one image-row segment, so
// the tap's zero padding is a wave-uniform row test plus a per-lane column test and every
// source offset is a scalar per-step base + a per-lane constant) and Cout, Cin (and the
// shuffle slot width) multiples of 128.  Output: fp32 slab tile staged through LDS and
// written with 16-B row-contiguous stores.
// ------------------------------------------------------------------------------------
// P2: the two-interval schedule of conv3x3_fwd_pph_kernel<.., P2> -- R1 reads A half 0 and both B
// halves and issues all four half-tiles of step t+1 (their buffer was last read at R2 of step t-1
// by both groups), two quadrants per MFMA interval, R2 reads A half 1; the leading group retires
// step t+1's DMAs after issuing its second MFMA interval, the lagging group at the end of its R2.
template <bool P2 = false>
__global__ __launch_bounds__(512) void conv3x3_wgrad_pp_kernel(WgArgs a) {
  constexpr int STAGE = 65536;
  constexpr int CSTR = 256 + 4;
  constexpr int SMEM = 128 * CSTR * 4;
  static_assert(SMEM >= 2 * STAGE, "LDS too small");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.taps * a.tiles_co * a.tiles_ci;
  int split, rem;
  if (a.bias_group > 0) {
    // tile blocks first; the bias-role blocks (light: dy only) each take bias_group splits, so
    // fewer CUs sit on them and the tile blocks get more splits (shorter K ranges)
    if ((int)b >= a.splits * ntile) {
      const int bb = (int)b - a.splits * ntile;
      const int grp = bb / a.tiles_co, co_t = bb - grp * a.tiles_co;
      const int s1 = min(a.splits, (grp + 1) * a.bias_group);
      for (int sp = grp * a.bias_group; sp < s1; ++sp) {
        if (sp > grp * a.bias_group) __syncthreads();  // the previous split's LDS stages are free
        wgrad_bias_role(a, smem, sp, co_t * 256);
      }
      return;
    }
    split = (int)b / ntile;
    rem = (int)b - split * ntile;
  } else {
    const int per_split = ntile + (a.wsb && !a.bias_fused ? a.tiles_co : 0);
    split = (int)b / per_split;
    rem = (int)b - split * per_split;
    if (rem >= ntile) {
      wgrad_bias_role(a, smem, split, (rem - ntile) * 256);
      return;
    }
  }
  const int tap = rem / (a.tiles_co * a.tiles_ci);
  rem -= tap * a.tiles_co * a.tiles_ci;
  const int co0 = (rem / a.tiles_ci) * 256;
  const int ci0 = (rem % a.tiles_ci) * 256;
  const int etap = tap + a.tap0;
  const int dy_ = etap / 3 - 1, dx_ = etap % 3 - 1;
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const int rps = a.out_ps > 0 ? a.out_ps : 1;

  // DMA rows of this lane: R_j = 8w + 4j + (lane >> 4), 16-B slot lane & 15 holding the
  // logical chunk lc_j of the swizzled 256-B row.
  int Rj[2];
  uint32_t la[2], lb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int R = 8 * w + 4 * j + (lane >> 4);
    const int f = (R & 3) | (((R >> 3) & 1) << 2);
    const int sl = lane & 15;
    const int lc = (((sl >> 1) ^ f) << 1) | (sl & 1);
    Rj[j] = R;
    la[j] = (uint32_t)(R * rps * a.ldy) * 2u + (uint32_t)lc * 16u;
    lb[j] = (uint32_t)(R * a.ldx) * 2u + (uint32_t)lc * 16u;
  }

  // scalar state of the K-step being issued
  int s_ua0 = 0, s_ua1 = 0, s_ub = 0, s_x0 = 0, s_left = 0, s_yv = 0;
  auto k_eval = [&](int ks) {
    const int p0s = p_begin + ks * 64;
    const int q = (int)fdiv((uint32_t)p0s, a.fd_W);
    const int x0 = p0s - q * a.W;
    const int n = (int)fdiv((uint32_t)q, a.fd_H);
    const int y = q - n * a.H;
    int ua[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int cu = co0 + h * 128;
      if (a.out_ps == 0) {
        ua[h] = (p0s * a.ldy + a.ycoff + cu) * 2;
      } else {
        const int r = a.out_ps;
        const int sl = (int)fdiv((uint32_t)cu, a.fd_cps);
        const int cch = cu - sl * a.fd_cps.d;
        const int si = sl / r, sj = sl - si * r;
        ua[h] = (((q * r + si) * (a.W * r) + x0 * r + sj) * a.ldy + a.ycoff + cch) * 2;
      }
    }
    s_ua0 = __builtin_amdgcn_readfirstlane(ua[0]);
    s_ua1 = __builtin_amdgcn_readfirstlane(ua[1]);
    s_ub = __builtin_amdgcn_readfirstlane((((q + dy_) * a.W + x0 + dx_) * a.ldx + a.xcoff + ci0) * 2);
    s_x0 = __builtin_amdgcn_readfirstlane(x0 + dx_);
    s_left = __builtin_amdgcn_readfirstlane(p_end - p0s);
    s_yv = __builtin_amdgcn_readfirstlane((unsigned)(y + dy_) < (unsigned)a.H ? 1 : 0);
  };
  constexpr uint32_t SLOT_A0 = 0, SLOT_A1 = 16384, SLOT_B0 = 32768, SLOT_B1 = 49152;
  auto issue_a = [&](int ks, int h) {
    char* dst = smem + (ks & 1) * STAGE + (h ? SLOT_A1 : SLOT_A0) + w * 2048;
    const uint32_t ua = (uint32_t)(h ? s_ua1 : s_ua0);
#pragma unroll
    for (int j = 0; j < 2; ++j) glds16(dyr, dst + j * 1024, Rj[j] < s_left ? ua + la[j] : SR_OOB);
  };
  auto issue_b = [&](int ks, int g) {
    char* dst = smem + (ks & 1) * STAGE + (g ? SLOT_B1 : SLOT_B0) + w * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool v = s_yv && Rj[j] < s_left && (unsigned)(s_x0 + Rj[j]) < (unsigned)a.W;
      glds16(xr, dst + j * 1024, v ? (uint32_t)s_ub + (uint32_t)g * 256u + lb[j] : SR_OOB);
    }
  };

  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  s16x8 fa[2][4], fb[2][2][2];  // fa[kk][i] (current A half), fb[g][kk][j]
  auto tr8 = [&](const char* base, int r0, int col) -> s16x8 {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(base + swz_tr(r0, col * 2, 256)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(base + swz_tr(r0 + 4, col * 2, 256)));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto read_a = [&](int buf, int h) {
    const char* As = smem + buf * STAGE + (h ? SLOT_A1 : SLOT_A0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[kk][i] = tr8(As, kk * 32 + 8 * tg + tq, wr * 64 + i * 16 + 4 * tp);
  };
  auto read_b = [&](int buf, int g) {
    const char* Bs = smem + buf * STAGE + (g ? SLOT_B1 : SLOT_B0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[g][kk][j] = tr8(Bs, kk * 32 + 8 * tg + tq, wc * 32 + j * 16 + 4 * tp);
  };
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[h][g][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused bias (a.bias_fused): the centre-tap blocks of the first ci tile also sum dy over their
  // pixels -- wave (wr, wc) takes A row block i = wc of each half against a ones operand
  const bool bias_here = a.bias_fused && a.wsb && tap == a.taps / 2 && ci0 == 0;
  const s16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  auto mma = [&](int h, int g) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[h][g][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[g][kk][j], acc[h][g][i][j], 0, 0, 0);
    if (g == 0 && bias_here) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (wc == 0) accb[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][0], ones, accb[h], 0, 0, 0);
        else if (wc == 1) accb[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][1], ones, accb[h], 0, 0, 0);
        else if (wc == 2) accb[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][2], ones, accb[h], 0, 0, 0);
        else accb[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][3], ones, accb[h], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = (p_end - p_begin + 63) / 64;  // >= 1 (every split owns >= 1 pixel)
  k_eval(0);
  issue_a(0, 0);
  issue_b(0, 0);
  issue_b(0, 1);
  issue_a(0, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  pp_barrier();
  if (wr) pp_barrier();
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const bool more = t + 1 < nk;
    if constexpr (P2) {
      // step 0's four half-tiles were retired by the prologue's vmcnt(4) only partly: drain once
      if (t == 0) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); pp_barrier(); pp_barrier(); }
      read_a(buf, 0);
      read_b(buf, 0);
      read_b(buf, 1);
      if (more) {
        k_eval(t + 1);
        issue_a(t + 1, 0);
        issue_b(t + 1, 0);
        issue_b(t + 1, 1);
        issue_a(t + 1, 1);
      }
      pp_barrier();
      mma(0, 0);
      mma(0, 1);
      pp_barrier();
      read_a(buf, 1);
      // A half 1 is read here and re-filled at the other group's next R1 (one interval later):
      // these reads complete before the barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (wr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();
      mma(1, 1);
      mma(1, 0);
      if (!wr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      pp_barrier();
      continue;
    }
    read_a(buf, 0);
    read_b(buf, 0);
    if (more) {
      k_eval(t + 1);
      issue_a(t + 1, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    pp_barrier();
    mma(0, 0);
    pp_barrier();
    read_b(buf, 1);
    if (more) {
      issue_b(t + 1, 0);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    pp_barrier();
    mma(0, 1);
    pp_barrier();
    read_a(buf, 1);
    if (more) issue_b(t + 1, 1);
    pp_barrier();
    mma(1, 1);
    pp_barrier();
    if (more) {
      issue_a(t + 1, 1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    pp_barrier();
    mma(1, 0);
    pp_barrier();
  }
  if (!wr) pp_barrier();

  if (bias_here && (lane & 15) == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + h * 128 + wr * 64 + wc * 16 + (lane >> 4) * 4 + r;
        if (co < a.Cout) a.wsb[(size_t)split * a.Cout + co] = accb[h][r];
      }
  }
  float* ws = a.ws + ((size_t)split * a.taps + tap) * a.Cout * a.Cin;
  float* Cs = (float*)smem;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Cs[(wr * 64 + i * 16 + (lane >> 4) * 4 + r) * CSTR + g * 128 + wc * 32 + j * 16 + (lane & 15)] =
                acc[h][g][i][j][r];
    __syncthreads();
    for (int idx = tid; idx < 128 * 64; idx += 512) {
      const int row = idx >> 6, c4 = (idx & 63) * 4;
      const int co = co0 + h * 128 + row, ci = ci0 + c4;
      if (co < a.Cout && ci < a.Cin)
        *(f32x4*)(ws + (size_t)co * a.Cin + ci) = *(const f32x4*)(Cs + row * CSTR + c4);
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient of a 1x1 conv (the SwinIR linears: dW[co][ci] = sum_t dy[t][co] x[t][ci] over
// the tokens t, db[co] = sum_t dy[t][co]), bf16.  A block owns a 192 (co) x 192 (ci) tile over a
// token K-range (split-K): SwinIR-M's 576 / 184 / 360 / 192 channel counts are 3 / 1 / 2 / 1 such
// tiles (4-7 % padding, against 28-50 % in 256x256 tiles).  A 64-token K-step is six [64 tok][64 ch]
// LDS images (128-B rows; 32-B blocks XOR-swizzled by row bits 1 and 3, so the 8 rows a 32-lane
// half reads with ds_read_b64_tr_b16 land on 8 distinct bank groups): dy co sub-tiles 0-2, then x ci
// sub-tiles 0-2, DMA'd straight to LDS (wave w: rows 8w .. 8w + 7 of each, the swizzle applied to
// the lane's source channels).  Three stages, two steps in flight, one barrier per step.  8 waves
// (2 co x 4 ci), each 96 co x 48 ci (6 x 3 accumulator tiles).  Blocks of the first ci tile also
// sum dy against a ones operand for the bias (wave (wr, wc): co fragments wc and wc + 4).  Output:
// the pp kernel's fp32 slab ws[split][Cout][Cin] and bias slab (same reduce).
// ------------------------------------------------------------------------------------
SR_DEV uint32_t swz_tr128(uint32_t row, uint32_t byte_in_row) {
  const uint32_t g = ((row >> 1) & 1u) | (((row >> 3) & 1u) << 1);
  return row * 128u + ((((byte_in_row >> 5) ^ g) & 3u) << 5) + (byte_in_row & 31u);
}

__global__ __launch_bounds__(512) void linear_wgrad_kernel(WgArgs a) {
  constexpr int IMG = 8192;       // [64 tok][64 ch] bf16
  constexpr int STAGE = 6 * IMG;  // 48 KB
  constexpr int NST = 3;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.tiles_co * a.tiles_ci;
  const int split = (int)b / ntile;
  const int rem = (int)b - split * ntile;
  const int cot = rem / a.tiles_ci, cit = rem - cot * a.tiles_ci;
  const int co0 = cot * 192, ci0 = cit * 192;
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const int nk = (p_end - p_begin + 63) / 64;
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);

  // DMA lane geometry: image row drow, physical 16-B slot lane & 7 = logical 32-B block
  // ((lane & 7) >> 1) ^ g(drow), half lane & 1
  const int drow = 8 * w + (lane >> 3);
  const int gsw = ((drow >> 1) & 1) | (((drow >> 3) & 1) << 1);
  const int lch = ((((lane & 7) >> 1) ^ gsw) << 4) + (lane & 1) * 8;
  uint32_t offy[3], offx[3];
  bool vy[3], vx[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int co = co0 + i * 64 + lch, ci = ci0 + i * 64 + lch;
    vy[i] = co < a.Cout;
    vx[i] = ci < a.Cin;
    offy[i] = (uint32_t)((drow * a.ldy + a.ycoff + co) * 2);
    offx[i] = (uint32_t)((drow * a.ldx + a.xcoff + ci) * 2);
  }
  auto issue = [&](int ks, int stg) {
    const int p0 = p_begin + ks * 64;
    char* st = smem + stg * STAGE + w * 1024;
    const bool tv = p0 + drow < p_end;
    const uint32_t by = (uint32_t)p0 * (uint32_t)a.ldy * 2u, bx = (uint32_t)p0 * (uint32_t)a.ldx * 2u;
#pragma unroll
    for (int i = 0; i < 3; ++i) glds16(dyr, st + i * IMG, tv && vy[i] ? by + offy[i] : SR_OOB);
#pragma unroll
    for (int i = 0; i < 3; ++i) glds16(xr, st + (3 + i) * IMG, tv && vx[i] ? bx + offx[i] : SR_OOB);
  };

  const int tg = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  auto tr8 = [&](const char* img, int r0, int col) -> s16x8 {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + swz_tr128(r0, col * 2)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + swz_tr128(r0 + 4, col * 2)));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  f32x4 acc[6][3];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bool bias_here = a.wsb != nullptr && cit == 0;
  const s16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

  auto compute = [&](int stg) {
    const char* st = smem + stg * STAGE;
    s16x8 fa[2][6], fb[2][3];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = kk * 32 + 8 * tg + tq;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int c = wr * 96 + i * 16;
        fa[kk][i] = tr8(st + (c >> 6) * IMG, r0, (c & 63) + 4 * tp);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int c = wc * 48 + j * 16;
        fb[kk][j] = tr8(st + (3 + (c >> 6)) * IMG, r0, (c & 63) + 4 * tp);
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
      if (bias_here) {
        // co fragments wc and wc + 4 of this wave's row block (wave-uniform branches: no indexed
        // fragment array, which would go to scratch)
        if (wc == 0) {
          accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][0], ones, accb[0], 0, 0, 0);
          accb[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][4], ones, accb[1], 0, 0, 0);
        } else if (wc == 1) {
          accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][1], ones, accb[0], 0, 0, 0);
          accb[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][5], ones, accb[1], 0, 0, 0);
        } else if (wc == 2) {
          accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][2], ones, accb[0], 0, 0, 0);
        } else {
          accb[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][3], ones, accb[0], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  if (nk > 0) issue(0, 0);
  if (nk > 1) issue(1, 1);
  int stg = 0;
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk)
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();  // step t landed for every wave; every wave finished reading step t - 1's stage
    if (t + 2 < nk) issue(t + 2, stg == 0 ? 2 : stg - 1);
    compute(stg);
    stg = stg == 2 ? 0 : stg + 1;
  }

  float* ws = a.ws + (size_t)split * a.Cout * a.Cin;
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wr * 96 + i * 16 + (lane >> 4) * 4 + r;
        const int ci = ci0 + wc * 48 + j * 16 + (lane & 15);
        if (co < a.Cout && ci < a.Cin) ws[(size_t)co * a.Cin + ci] = acc[i][j][r];
      }
  if (bias_here && (lane & 15) == 0) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = k == 0 ? wc : wc + 4;
      if (i < 6) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wr * 96 + i * 16 + (lane >> 4) * 4 + r;
          if (co < a.Cout) a.wsb[(size_t)split * a.Cout + co] = accb[k][r];
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient for narrow convs (Cout <= 64: RCAN / RRDB / SRResNet bodies; or 64-channel output
// tiles of a wider conv, wg_ring_wide), all nine taps in one block, whole image rows per split
// (W % 64 == 0).  The block walks each 64-px column segment of its rows top to bottom, so a K-step
// loads ONE new x halo row (66 px of a 16-ci tile per wave) into a ring and dy[64 px][Cout] once;
// rows above / below an image read a zero slot (x read ~once per pass instead of ~3x).  Every tap's
// GEMM is formed from LDS.  Wave w owns ci tile w (16 channels) x all co tiles x 9 taps (36 * CO_T
// accumulator tiles, pinned to AGPRs); operands by ds_read_b64_tr_b16.  LDS images are
// [tile][row][32 B] with row r stored at r ^ ((r >> 3) & 1) << 2: the rows a 32-lane half reads
// ({b..b+3} u {b+8..b+11}, any base b) hit distinct 32-B bank slots.  Both images are filled by
// LDS-DMA, two steps in flight.  Nearest-neighbour input upsampling (in_up 2, RRDBNet conv_up*) is
// folded into the halo gather; pixel-shuffled dy (the wide form) into the dy gather.  The first
// step of a segment loads its three rows itself, after the previous segment's last step (its slots
// may still be read), so a block has nseg - 1 one-step bubbles.
// (Round 4's variants -- two row groups or two co groups per 8-wave block, co split over blocks,
// early DMA issue, deeper pipelines -- all measured slower and were removed in round 5.)
//
// Output: the block's [tap][ci][co] partial sums (co fastest: a lane's 4 accumulator rows are 4
// consecutive co, one 16-B store per (tap, co tile)) into slab row `split` of [S][9][Cin][Cout].
// (Round 5 tried an in-kernel reduce: write-through slab rows, a ticket per group of G splits, the
// last arriver summing the group's rows in split order into a level-2 slab for the standalone reduce.
// Measured in the step it lost badly -- RCAN 38.1 -> 51.0 / 60.6 ms at G 2 / 4, RRDB 67.3 -> 77.6 /
// 80.7 ms: each group's tail reads (G - 1) x 147 KB at a few GB/s per block while the chip-wide reduce
// it replaces reads the whole slab in ~11 us -- and it was removed)
// ------------------------------------------------------------------------------------
SR_DEV int hrow(int r) { return r ^ (((r >> 3) & 1) << 2); }

template <int CO_T>
__global__ __launch_bounds__(256, 1) void conv3x3_wgrad_ring_kernel(WgArgs a) {
  constexpr int D = 2;              // steps in flight
  constexpr int LA = 3;             // fragment reads ahead of the MFMA group that needs them
  constexpr int RS = 3 * 1024;      // one halo row of one 16-ci tile: 96 rows x 32 B (66 used)
  constexpr int RSL = D + 2;        // ring slots: rows q-1 .. q+1 read, D - 1 in flight (+1 being issued)
  constexpr int RING = (RSL + 1) * RS;  // + the zero slot, per ci tile
  constexpr int DYB = CO_T * 2048;  // dy image: CO_T tiles x 64 rows x 32 B
  constexpr int DYS = DYB + 1024;   // + 1 KB target for padding DMAs
  constexpr int DYI = (CO_T * 2 + 3) / 4;  // dy DMAs per wave
  __shared__ __attribute__((aligned(16))) char smem[4 * RING + D * DYS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  // block = (split, co tile, ci chunk), ci fastest: the tiles of one split (the same x / dy rows)
  // are consecutive, so xcd_remap keeps them on one XCD's L2
  const int per_split = a.tiles_ci * a.tiles_co;
  const int split = (int)b / per_split;
  const int rem_ = (int)b - split * per_split;
  const int cot = rem_ / a.tiles_ci;
  const int chunk = rem_ - cot * a.tiles_ci;
  const int ci0 = chunk * 64;
  const int co0 = cot * (CO_T * 16);
  // out_ps: the co tile lies in one shuffle slot (C' a multiple of the tile width, checked on the host)
  const int ps_sl = a.out_ps > 0 ? (int)fdiv((uint32_t)co0, a.fd_cps) : 0;
  const int ps_si = a.out_ps > 0 ? ps_sl / a.out_ps : 0, ps_sj = a.out_ps > 0 ? ps_sl - ps_si * a.out_ps : 0;
  const int rows_total = a.N * a.H;
  const int rps = a.kper / a.W;  // image rows per split
  const int r0 = split * rps, r1 = min(rows_total, r0 + rps);
  const int nrows = r1 - r0, nseg = a.W >> 6, nk = nrows * nseg;
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const int sh = a.in_up > 1 ? 1 : 0;  // in_up is 1 or 2 here
  const int Hs = a.H >> sh, Ws = a.W >> sh;
  char* ring = smem + w * RING;
  char* dys = smem + 4 * RING;
  auto slot = [](int q) { return (q + RSL) % RSL; };  // q >= -1

  // this lane's halo pixels of its 3 DMAs per row: physical row 32i + (lane >> 1) holds pixel
  // hrow(.) (x0 - 1 + that), channel half lane & 1
  int hpx[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int hr = hrow(32 * i + (lane >> 1));
    hpx[i] = hr < 66 ? hr : -100000;
  }
  const int cil = ci0 + w * 16 + (lane & 1) * 8;
  const bool civ = cil < a.Cin;
  for (int i = lane; i < RS / 16; i += 64) *(u32x4*)(ring + RSL * RS + i * 16) = u32x4{0u, 0u, 0u, 0u};

  f32x4 acc[9][CO_T], accb[CO_T];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < CO_T; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < CO_T; ++c) accb[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.wsb != nullptr && chunk == 0 && w == 0;

  // x halo row q (global image row; outside [0, rows_total) -> zeros), column segment seg
  auto issue_row = [&](int q, int seg) {
    const bool qv = q >= 0 && q < rows_total;
    const int n = qv ? (int)fdiv((uint32_t)q, a.fd_H) : 0;
    const int yy = q - n * a.H;
    char* dst = ring + slot(q) * RS;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int xx = seg * 64 - 1 + hpx[i];
      const bool v = qv && civ && (unsigned)xx < (unsigned)a.W;
      const uint32_t off = (uint32_t)((((n * Hs + (yy >> sh)) * Ws + (xx >> sh)) * a.ldx + a.xcoff + cil) * 2);
      glds16(xr, dst + i * 1024, v ? off : SR_OOB);
    }
  };
  // step j = (segment j / nrows, row r0 + j % nrows); the first step of a segment loads its
  // three rows and is issued after the previous segment's last step (whose slots it reuses)
  auto first = [&](int j) { return j % nrows == 0; };
  auto nops = [&](int j) { return DYI + (first(j) ? 9 : 3); };
  auto issue_iter = [&](int j) { const int f = j - j % nrows - 1, e = j - D; return f > e ? f : e; };
  auto issue = [&](int j) {
    const int seg = j / nrows, q = r0 + (j - seg * nrows);
    if (first(j)) {
      issue_row(q - 1, seg);
      issue_row(q, seg);
    }
    issue_row(q + 1, seg);
    const int p0s = q * a.W + seg * 64;
    char* st = dys + (j % D) * DYS;
#pragma unroll
    for (int i = 0; i < DYI; ++i) {
      const int k = w + 4 * i;  // dy DMA index: co tile k >> 1, rows 32 (k & 1) ..
      char* dst = st + DYB;
      uint32_t off = SR_OOB;
      if (k < CO_T * 2) {
        const int pr = hrow((k & 1) * 32 + (lane >> 1));
        const int co = co0 + (k >> 1) * 16 + (lane & 1) * 8;
        dst = st + k * 1024;
        if (co < a.Cout) {
          if (a.out_ps == 0) {
            off = (uint32_t)(((p0s + pr) * a.ldy + a.ycoff + co) * 2);
          } else {  // pixel-shuffled dy: GEMM column sl * C' + c of LR pixel (q, x) = HR pixel (q r + si, x r + sj), channel c
            const int r = a.out_ps;
            const int hp = (q * r + ps_si) * (a.W * r) + (seg * 64 + pr) * r + ps_sj;
            off = (uint32_t)((hp * a.ldy + a.ycoff + co - ps_sl * a.fd_cps.d) * 2);
          }
        }
      }
      glds16(dyr, dst, off);
    }
  };

  const int g = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  auto tr2 = [&](const char* img, int r0_) -> s16x8 {  // rows r0 + tq (K 0..3), r0 + 4 + tq (K 4..7)
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + hrow(r0_ + tq) * 32 + tp * 8));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + hrow(r0_ + 4 + tq) * 32 + tp * 8));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  const s16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
  auto compute = [&](int j) {
    const int q = r0 + j % nrows;
    const int y = q - (int)fdiv((uint32_t)q, a.fd_H) * a.H;
    const char* rows3[3] = {ring + (y == 0 ? RSL : slot(q - 1)) * RS, ring + slot(q) * RS,
                            ring + (y == a.H - 1 ? RSL : slot(q + 1)) * RS};
    const char* ds = dys + (j % D) * DYS;
    // Fragment reads (per K half: this wave's dy tiles, then the 9 taps' x tiles) run LA reads
    // ahead of the MFMA group (one tap x CO_T co tiles) that needs them, in program order fixed by
    // scheduling barriers (the compiler otherwise sinks each read to just before its MFMAs); at
    // most ~2 (LA + 1) reads are in flight, within what lgkmcnt counts, so its waits stay exact.
    constexpr int NR = CO_T + 9;
    s16x8 fr[2 * NR];
    auto rd = [&](int r) {
      const int kk = r / NR, i = r - kk * NR;
      fr[r] = i < CO_T ? tr2(ds + i * 2048, kk * 32 + 8 * g) : tr2(rows3[(i - CO_T) / 3], ((i - CO_T) % 3) + kk * 32 + 8 * g);
    };
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int need = kk * NR + CO_T + t;
        // reads not yet issued up to need + LA (the previous group issued up to its need + LA)
        const int lo = (kk == 0 && t == 0) ? 0 : (t > 0 ? need + LA : NR + LA);
#pragma unroll
        for (int r = 0; r < 2 * NR; ++r)
          if (r >= lo && r <= need + LA) rd(r);
        // accumulators pinned to AGPRs (inline asm): with this many of them the compiler
        // otherwise moves every one between AGPRs and VGPRs once per step
#pragma unroll
        for (int c = 0; c < CO_T; ++c)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[t][c]) : "v"(fr[kk * NR + c]), "v"(fr[need]));
        __builtin_amdgcn_sched_barrier(0);
      }
      if (do_bias) {  // builtin: the compiler pads the VALU write of `ones` before its read
#pragma unroll
        for (int c = 0; c < CO_T; ++c) accb[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[kk * NR + c], ones, accb[c], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  __syncthreads();  // zero slots written
  int next = 0;  // steps issued so far, in step order (issue_iter is non-decreasing)
  while (next < nk && issue_iter(next) < 0) issue(next++);
  for (int ks = 0; ks < nk; ++ks) {
    // step ks's DMAs landed; the steps issued after it may stay in flight
    if (next == ks + D && (ks + 1) % nrows != 0 && (ks + 1) / nrows == (next - 1) / nrows) {
      // steady state: the D - 1 steps after ks, none of them a segment's first
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * (DYI + 3)) : "memory");
    } else {
      int younger = 0;
      for (int j = ks + 1; j < next; ++j) younger += nops(j);
      vm_wait_dyn(younger);
    }
    __builtin_amdgcn_s_barrier();
    compute(ks);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    while (next < nk && issue_iter(next) <= ks) issue(next++);
  }

  // the last MFMAs' results are read below (inline-asm MFMAs: the hazard wait is ours)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  const int c16 = lane & 15;
  const int ci = ci0 + w * 16 + c16;
  // slab row `split`; the standalone reduce sums the S rows
  if (ci < a.Cin) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float* ws = a.ws + (((size_t)split * 9 + t) * a.Cin + ci) * a.Cout;
#pragma unroll
      for (int c = 0; c < CO_T; ++c) {
        const int co = co0 + c * 16 + g * 4;
        if (co < a.Cout) *(f32x4*)(ws + co) = acc[t][c];
      }
    }
  }
  if (do_bias && c16 == 0) {
#pragma unroll
    for (int c = 0; c < CO_T; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + c * 16 + g * 4 + r;
        if (co < a.Cout) a.wsb[(size_t)split * a.Cout + co] = accb[c][r];
      }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient over one kernel ROW of taps (round 6): bf16 3x3, Cout % 256 == 0, Cin % 128 == 0,
// W % 64 == 0, no upsample; pixel-shuffled dy with C' % 256 == 0 (the EDSR-L body and upsample convs).  A pp-kernel block is one tap of
// a 256 x 256 (co x ci) tile: each K-step DMAs the dy tile AND a tap-shifted x tile (64 KB per 4.2 M
// MACs) and its 8 waves of 128 x 64 read 192 KB of fragments.  Here a block owns the three taps
// (ky, 0..2) of a 256 x 128 tile: a K-step (64 pixels of one image row) DMAs the dy tile (32 KB) and
// ONE x halo row of 66 pixels (16.5 KB), and the three taps' B operands are that row read at row
// offsets 0 / 1 / 2: 48.5 KB per 6.3 M MACs.  4 waves, one per SIMD; wave (wr, wc) = 128 co x 64 ci x
// 3 taps, 384 accumulator registers (taps 0 / 1 pinned to AGPRs, tap 2 in VGPRs); an A fragment feeds
// 12 MFMAs and a B fragment 8 (40 KB of fragment reads per wave and step for 1.6 M MACs).  Three LDS
// stages; one barrier per step, placed before the step's last MFMA group, after which the next step's
// first fragment reads run under that group.  Operand images as the ring kernel's: [16-channel tile]
// [row][32 B] with rows permuted by hrow (conflict-free tr reads at any row offset); the halo row's 66
// rows arrive as three 32-row pieces, the third (rows 34..65) rewriting 30 rows of the second with the
// same bytes.  Image edges and rows outside the image read zeros (out-of-range buffer offsets).  Bias:
// bias-role blocks after the tile blocks, each summing dy over bias_group splits.  Output: the pp
// kernel's [S][9][Cout][Cin] slab (same reduce), staged through LDS for 16-B row stores.
// ------------------------------------------------------------------------------------
// Compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N - 1 (fully unrolled by construction;
// a #pragma unroll loop this large exceeds the unroller's threshold and its arrays go to scratch).
template <typename F, int... I>
SR_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
SR_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
constexpr int row3_need(int gi) { return (gi / 12) * 20 + 8 + gi % 12; }  // last fragment read group gi uses

__global__ __launch_bounds__(256, 1) void conv3x3_wgrad_row3_kernel(WgArgs a) {
  constexpr int LA = 1;  // fragment reads one MFMA group ahead (two: the same time, 4 more VGPRs)
  constexpr int DYT = 2048;      // one 16-co tile of dy: 64 rows x 32 B
  constexpr int XT = 66 * 32;    // one 16-ci tile of the halo row: 66 rows x 32 B
  constexpr int DYB = 16 * DYT;  // 256 co
  constexpr int STG = DYB + 8 * XT;
  constexpr int NOPS = 14;       // LDS-DMAs per wave and K-step: 8 dy + 6 x
  __shared__ __attribute__((aligned(16))) char smem[3 * STG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = 3 * a.tiles_co * a.tiles_ci;
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, a.dy_bytes);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, a.x_bytes);
  const int g = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;

  // pixel-shuffled dy (out_ps r, the upsample convs): a 256-co tile lies in ONE shuffle slot sl
  // (C' % 256 == 0, checked on the host), so GEMM column co0 + c of LR pixel (q, x) is channel
  // co0 - sl C' + c of HR pixel (q r + sl / r, x r + sl % r): LR pixels r HR pixels apart
  const int rps = a.out_ps > 0 ? a.out_ps : 1;
  auto dy_base = [&](int p0s, int co0) -> int {  // byte offset of (first pixel of the K-step, co0)
    if (a.out_ps == 0) return (p0s * a.ldy + a.ycoff + co0) * 2;
    const int q = (int)fdiv((uint32_t)p0s, a.fd_W), x0 = p0s - q * a.W;
    const int sl = (int)fdiv((uint32_t)co0, a.fd_cps), si = sl / rps, sj = sl - si * rps;
    return (((q * rps + si) * (a.W * rps) + x0 * rps + sj) * a.ldy + a.ycoff + co0 - sl * (int)a.fd_cps.d) * 2;
  };
  // dy pieces of this wave: k = w + 4 i -> co tile k >> 1, physical rows 32 (k & 1) + (lane >> 1)
  uint32_t dyl[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k = w + 4 * i;
    const int pr = hrow((k & 1) * 32 + (lane >> 1));
    dyl[i] = (uint32_t)((pr * rps * a.ldy + (k >> 1) * 16 + (lane & 1) * 8) * 2);
  }
  auto issue_dy = [&](char* st, int s_dyb) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = w + 4 * i;
      glds16(dyr, st + (k >> 1) * DYT + (k & 1) * 1024, (uint32_t)s_dyb + dyl[i]);
    }
  };
  auto tr2 = [&](const char* img, int r0_) -> s16x8 {  // rows r0 + tq (K 0..3), r0 + 4 + tq (K 4..7)
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + hrow(r0_ + tq) * 32 + tp * 8));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + hrow(r0_ + 4 + tq) * 32 + tp * 8));
    return s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  if ((int)b >= a.splits * ntile) {
    // bias role: dy column sums of one 256-co tile over bias_group splits (dy images only, two stages)
    const int bb = (int)b - a.splits * ntile;
    const int grp = bb / a.tiles_co, co0 = (bb - grp * a.tiles_co) * 256;
    const s16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
    const int s1 = min(a.splits, (grp + 1) * a.bias_group);
    for (int sp = grp * a.bias_group; sp < s1; ++sp) {
      const int p_begin = sp * a.kper, p_end = min(a.M, p_begin + a.kper);
      const int nk = (p_end - p_begin) >> 6;
      auto base = [&](int ks) { return __builtin_amdgcn_readfirstlane(dy_base(p_begin + ks * 64, co0)); };
      f32x4 accb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      __syncthreads();  // the previous split's stage reads are done
      if (nk > 0) issue_dy(smem, base(0));
      if (nk > 1) issue_dy(smem + STG, base(1));
      for (int ks = 0; ks < nk; ++ks) {
        if (ks + 1 < nk)
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const char* st = smem + (ks & 1) * STG;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tr2(st + (w * 4 + i) * DYT, kk * 32 + 8 * g), ones, accb[i], 0, 0, 0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ks + 2 < nk) issue_dy(smem + (ks & 1) * STG, base(ks + 2));
      }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int co = co0 + (w * 4 + i) * 16 + g * 4 + r;
            if (co < a.Cout) a.wsb[(size_t)sp * a.Cout + co] = accb[i][r];
          }
      }
    }
    return;
  }

  const int split = (int)b / ntile;
  int rem = (int)b - split * ntile;
  const int ky = rem / (a.tiles_co * a.tiles_ci);
  rem -= ky * a.tiles_co * a.tiles_ci;
  const int co0 = (rem / a.tiles_ci) * 256;
  const int ci0 = (rem % a.tiles_ci) * 128;
  const int dy_ = ky - 1;
  const int p_begin = split * a.kper;
  const int p_end = min(a.M, p_begin + a.kper);
  const int nk = (p_end - p_begin) >> 6;  // >= 1: whole 64-pixel steps (M, kper multiples of 64)

  // x pieces of this wave: k = w + 4 i (i < 6) -> ci tile k / 3, piece k % 3 at physical row 0 / 32 / 34;
  // lane: physical row base + (lane >> 1) = logical halo row (pixel x0 - 1 + row) hrow(.), channel half lane & 1
  uint32_t xl[6];
  int xlr[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int k = w + 4 * i, t = k / 3, pc = k - 3 * t;
    const int lr = hrow((pc == 0 ? 0 : (pc == 1 ? 32 : 34)) + (lane >> 1));
    xlr[i] = lr;
    xl[i] = (uint32_t)((lr * a.ldx + t * 16 + (lane & 1) * 8) * 2);
  }
  // scalar state of a K-step's DMAs (k_eval), then its 14 pieces (piece < 8: dy, else x)
  int s_dyb = 0, s_xb = 0, s_xm1 = 0, s_yv = 0;
  auto k_eval = [&](int ks) {
    const int p0s = p_begin + ks * 64;
    const int q = (int)fdiv((uint32_t)p0s, a.fd_W);
    const int x0 = p0s - q * a.W;
    const int n = (int)fdiv((uint32_t)q, a.fd_H);
    const int y = q - n * a.H;
    s_dyb = __builtin_amdgcn_readfirstlane(dy_base(p0s, co0));
    s_xb = __builtin_amdgcn_readfirstlane((((q + dy_) * a.W + x0 - 1) * a.ldx + a.xcoff + ci0) * 2);
    s_xm1 = __builtin_amdgcn_readfirstlane(x0 - 1);
    s_yv = __builtin_amdgcn_readfirstlane((unsigned)(y + dy_) < (unsigned)a.H ? 1 : 0);
  };
  auto piece = [&](char* st, int pi) {  // pi: compile-time after unrolling
    if (pi < 8) {
      const int k = w + 4 * pi;
      glds16(dyr, st + (k >> 1) * DYT + (k & 1) * 1024, (uint32_t)s_dyb + dyl[pi]);
    } else {
      const int i = pi - 8, k = w + 4 * i, t = k / 3, pc = k - 3 * t;
      const bool v = s_yv && (unsigned)(s_xm1 + xlr[i]) < (unsigned)a.W;
      glds16(xr, st + DYB + t * XT + (pc == 0 ? 0 : (pc == 1 ? 32 : 34)) * 32, v ? (uint32_t)(s_xb + (int)xl[i]) : SR_OOB);
    }
  };
  auto issue = [&](int ks, char* st) {
    k_eval(ks);
#pragma unroll
    for (int pi = 0; pi < NOPS; ++pi) piece(st, pi);
  };

  f32x4 acc0[8][4], acc1[8][4], acc2[8][4];  // taps kx 0 / 1 (AGPRs), 2 (VGPRs); [co tile][ci tile]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc0[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  // a step's fragment reads: r = 20 kk + i, i < 8: A (dy) co tile wr * 8 + i; 8 <= i < 20: B, tap
  // kx = (i - 8) >> 2, ci tile wc * 4 + ((i - 8) & 3) (the halo row at row offset kx)
  s16x8 fa[2][8], fb[2][12];
  auto rd = [&](const char* st, auto R) {
    constexpr int r = R, kk = r / 20, i = r - kk * 20;
    if constexpr (i < 8) {
      fa[kk][i] = tr2(st + (wr * 8 + i) * DYT, kk * 32 + 8 * g);
    } else {
      constexpr int c = i - 8;
      fb[kk][c] = tr2(st + DYB + (wc * 4 + (c & 3)) * XT, kk * 32 + 8 * g + (c >> 2));
    }
  };
  // MFMA group gi (24 per step): kk = gi / 12, B fragment c = gi % 12 against the 8 A fragments
  auto group = [&acc0, &acc1, &acc2, &fa, &fb](auto GI) {  // (explicit: if constexpr branches)
    constexpr int gi = GI, kk = gi / 12, c = gi % 12, kx = c >> 2, j = c & 3;
    (void)acc0, (void)acc1, (void)acc2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (kx == 0)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc0[i][j]) : "v"(fa[kk][i]), "v"(fb[kk][c]));
      else if constexpr (kx == 1)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc1[i][j]) : "v"(fa[kk][i]), "v"(fb[kk][c]));
      else
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc2[i][j]) : "v"(fa[kk][i]), "v"(fb[kk][c]));
    }
  };
  // read stream position x (group x's last read): x < 24 this step, x >= 24 the next step's
  constexpr auto rpos = [](int x) { return x < 24 ? row3_need(x) : 40 + row3_need(x - 24); };
  constexpr int GB = 24 - LA;  // the group before which the barrier runs (its reads reach the next step)

  issue(0, smem);
  if (nk > 1) issue(1, smem + STG);
  if (nk > 2) issue(2, smem + 2 * STG);
  vm_wait_dyn(NOPS * (min(nk, 3) - 1));
  __builtin_amdgcn_s_barrier();
  static_for<rpos(LA - 1) + 1>([&](auto R) { rd(smem, R); });
  int stc = 0;  // stage of step t
  for (int t = 0; t < nk; ++t) {
    const int stn = stc == 2 ? 0 : stc + 1;
    const char* cur = smem + stc * STG;
    const char* nxt = smem + stn * STG;
    const bool more = t + 1 < nk;
    static_for<24>([&](auto GI) {
      constexpr int gi = GI;
      // this step's reads up to group gi + LA's
      static_for<40>([&](auto R) {
        if constexpr (R > rpos(gi + LA - 1) && R <= rpos(gi + LA) && R < 40) rd(cur, R);
      });
      if constexpr (gi == GB) {
        if (more) {
          // every read of step t is issued: once they completed and step t + 1 landed (in every wave),
          // step t's stage takes step t + 3's DMAs and step t + 1's first reads run under these groups
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (t + 2 < nk)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NOPS) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          if (t + 3 < nk) issue(t + 3, smem + stc * STG);
        }
      }
      if constexpr (gi >= GB) {
        if (more) {
          static_for<40>([&](auto R) {
            if constexpr (R + 40 > rpos(gi + LA - 1) && R + 40 <= rpos(gi + LA)) rd(nxt, R);
          });
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      group(GI);
      __builtin_amdgcn_sched_barrier(0);
    });
    stc = stn;
  }

  // the last MFMAs' results are read below (inline-asm MFMAs: the hazard wait is ours)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // slab: 4-B stores straight from the accumulators (16 lanes: 64 contiguous bytes).  (Staged through
  // LDS for 16-B row stores, as the pp kernel does, it measured slower: 165-173 vs 163-170 us.)
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    float* ws = a.ws + ((size_t)split * 9 + ky * 3 + kx) * a.Cout * a.Cin;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = kx == 0 ? acc0[i][j] : (kx == 1 ? acc1[i][j] : acc2[i][j]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ws[(size_t)(co0 + wr * 128 + i * 16 + g * 4 + r) * a.Cin + ci0 + wc * 64 + j * 16 + (lane & 15)] = v[r];
      }
  }
}

// dw[co][ci][ky][kx] = scale * sum_s ws[s][tap][co'][ci], co' = GEMM column of co (out_ps
// permutation); one thread per (co, ci): slab reads coalesced along ci, 9 taps per thread.
__global__ void wgrad_reduce_kernel(const float* ws, const float* wsb, float* dw, float* db, int S,
                                    int Cout, int Cin, int Cout_real, int Cin_real, int out_ps, int taps,
                                    const int* co_map, const int* ci_map, float scale, int accumulate) {
  const int64_t total = (int64_t)Cout_real * Cin_real;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1;
  const int cps = Cout_real / r2;  // C' (channels after shuffle)
  if (i < total) {
    const int ci = (int)(i % Cin_real);
    const int co = (int)(i / Cin_real);
    const int cop = co_map ? co_map[co] : (out_ps > 0 ? (co % r2) * cps + co / r2 : co);  // GEMM column
    const int cip = ci_map ? ci_map[ci] : ci;                                                // GEMM k channel
    const size_t stride = (size_t)taps * Cout * Cin;
    float s[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) s[t] = 0.f;
    for (int k = 0; k < S; ++k) {
      const float* src = ws + k * stride + (size_t)cop * Cin + cip;
#pragma unroll
      for (int t = 0; t < 9; ++t)
        if (t < taps) s[t] += src[(size_t)t * Cout * Cin];
    }
    float* d = dw + i * taps;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if (t < taps) d[t] = s[t] * scale + (accumulate ? d[t] : 0.f);
  }
  if (db && i < Cout_real) {
    const int co = (int)i;
    const int cop = co_map ? co_map[co] : (out_ps > 0 ? (co % r2) * cps + co / r2 : co);
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += wsb[(size_t)k * Cout + cop];
    db[co] = s * scale + (accumulate ? db[co] : 0.f);
  }
}

// Slab reduction for the RGB head conv (Cin_real <= 8, not a multiple of 4): wgrad_reduce_kernel
// gives each (co, ci) pair ONE thread that walks all S slabs (RRDB conv_first: 192 threads x
// S 1024 = 1.28 ms).  Here one block per output channel: 256 threads split the slabs, each
// keeps 9 x Cin_real (+ bias) partial sums, then a fixed-order LDS tree -- deterministic.
__global__ __launch_bounds__(256) void wgrad_reduce_narrow_kernel(const float* ws, const float* wsb, float* dw,
                                                                  float* db, int S, int Cout, int Cin, int Cin_real,
                                                                  int out_ps, int taps, const int* co_map,
                                                                  const int* ci_map, float scale, int accumulate) {
  constexpr int NV = 9 * 8 + 1;
  __shared__ float red[NV][256];
  const int co = blockIdx.x, t = threadIdx.x;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1;
  const int cps = (int)gridDim.x / r2;
  const int cop = co_map ? co_map[co] : (out_ps > 0 ? (co % r2) * cps + co / r2 : co);
  int cip[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) cip[c] = c < Cin_real ? (ci_map ? ci_map[c] : c) : 0;
  float s[9][8], sb = 0.f;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int c = 0; c < 8; ++c) s[tp][c] = 0.f;
  const size_t stride = (size_t)taps * Cout * Cin, tstride = (size_t)Cout * Cin;
  for (int k = t; k < S; k += 256) {
    const float* src = ws + k * stride + (size_t)cop * Cin;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (tp < taps && c < Cin_real) s[tp][c] += src[tp * tstride + cip[c]];
    if (db) sb += wsb[(size_t)k * Cout + cop];
  }
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int c = 0; c < 8; ++c) red[tp * 8 + c][t] = s[tp][c];
  red[NV - 1][t] = sb;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w)
      for (int v = 0; v < NV; ++v) red[v][t] += red[v][t + w];
    __syncthreads();
  }
  if (t < 9 * 8) {
    const int tp = t >> 3, c = t & 7;
    if (tp < taps && c < Cin_real) {
      float* d = dw + ((size_t)co * Cin_real + c) * taps + tp;
      *d = red[t][0] * scale + (accumulate ? *d : 0.f);
    }
  } else if (t == NV - 1 && db) {
    db[co] = red[t][0] * scale + (accumulate ? db[co] : 0.f);
  }
}

// Slab reduction, one kernel for both slab layouts (TR false: [S][taps][Cout][Cin], groups (tap,
// co, 4 ci); TR true: the row-streaming wgrad's [S][taps][Cin][Cout], groups (tap, ci, 4 co)), no
// gathered loads (ci_map with TR false / co_map with TR true go to the kernels below).  A block
// of nw waves holds GPW groups x P = nw * 64 / GPW split phases: lane -> (phase, group), one 16-B
// load per split, GPW * 16 B contiguous per phase and wave instruction, phases k = ph (mod P)
// with 4 independent loads in flight, then a fixed-order LDS combine -- deterministic.  The host
// sizes P to ~8 slabs per thread and GPW so that the grid covers the chip (RCAN: S 256 over 9216
// groups = 288 blocks of 32 groups x 32 phases instead of 144 of 64 x 16).
// CIG (TR false with a ci_map, the SwinIR proj / dense linears over padded head channels): groups run
// over the GEMM columns (16-B loads, no gather) and each sum is stored at its parameter column, through
// the GEMM -> parameter inverse of ci_map built in LDS (-1: a padding column, dropped).  (The gathered
// wgrad_reduce4_kernel it replaces read 36 MB in 60 us in the SwinIR step.)
template <int GPW, bool TR, bool CIG = false>
__global__ __launch_bounds__(1024) void wgrad_reduce_g_kernel(const float* ws, const float* wsb, float* dw, float* db,
                                                              int S, int Cout, int Cin, int Cout_real, int Cin_real,
                                                              int out_ps, int taps, const int* co_map,
                                                              const int* ci_map, float scale, int wblocks,
                                                              int accumulate) {
  extern __shared__ f32x4 red[];  // nw * 64 entries (dynamic: a 4-wave block needs 4 KB, so it can
                                  // share a CU with the 158 KB pph kernel when it runs on a side stream)
  const int nw = (int)(blockDim.x >> 6);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1;
  const int cps = Cout_real / r2;
  if ((int)blockIdx.x >= wblocks) {  // bias: 64 co per block, nw phases
    const int c = ((int)blockIdx.x - wblocks) * 64 + lane;
    float sb = 0.f;
    if (c < Cout_real) {
      const int cop = co_map ? co_map[c] : (out_ps > 0 ? (c % r2) * cps + c / r2 : c);
      for (int k = wv; k < S; k += nw) sb += wsb[(size_t)k * Cout + cop];
    }
    red[wv * 64 + lane] = f32x4{sb, 0.f, 0.f, 0.f};
    __syncthreads();
    if (wv == 0 && c < Cout_real) {
      float sm = red[lane][0];
      for (int k = 1; k < nw; ++k) sm += red[k * 64 + lane][0];
      db[c] = sm * scale + (accumulate ? db[c] : 0.f);
    }
    return;
  }
  const int P = nw * (64 / GPW);
  const int ph = wv * (64 / GPW) + lane / GPW, gl = lane % GPW;
  const int64_t i = (int64_t)blockIdx.x * GPW + gl;
  const int c4n = TR ? (Cout_real + 3) >> 2 : (CIG ? Cin >> 2 : Cin_real >> 2);
  [[maybe_unused]] int* inv = nullptr;
  if constexpr (CIG) {
    __shared__ int inv_s[1024];  // GEMM column -> parameter column (Cin <= 1024, checked on the host)
    inv = inv_s;
    for (int k = threadIdx.x; k < Cin; k += blockDim.x) inv_s[k] = -1;
    __syncthreads();
    for (int c = threadIdx.x; c < Cin_real; c += blockDim.x) inv_s[ci_map[c]] = c;
    __syncthreads();
  }
  const int rows = TR ? Cin_real : Cout_real;
  const int64_t total = (int64_t)taps * rows * c4n;
  int q4 = 0, rw = 0, tap = 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    q4 = (int)(i % c4n);
    const int64_t t2 = i / c4n;
    rw = (int)(t2 % rows);
    tap = (int)(t2 / rows);
    int rp;
    if (TR) rp = ci_map ? ci_map[rw] : rw;
    else rp = co_map ? co_map[rw] : (out_ps > 0 ? (rw % r2) * cps + rw / r2 : rw);
    const size_t stride = (size_t)taps * Cout * Cin;
    const float* src = ws + ((size_t)tap * (TR ? Cin : Cout) + rp) * (TR ? Cout : Cin) + q4 * 4;
    // 8 independent 16-B loads in flight, and the < 8 left over issued together too (clamped to a
    // valid split, zeroed after the load: no branch, so no load waits for the one before it -- the
    // round-5 form ran its remainder one dependent iteration at a time, e.g. 2-3 of the 6-7 loads per
    // lane at the EDSR body wgrad's 26 splits)
    int k = ph;
    for (; k + 7 * P < S; k += 8 * P) {
      f32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = *(const f32x4*)(src + (size_t)(k + j * P) * stride);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j];
    }
    if (k < S) {
      f32x4 v[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int kj = k + j * P < S ? k + j * P : S - 1;
        v[j] = *(const f32x4*)(src + (size_t)kj * stride);
      }
#pragma unroll
      for (int j = 0; j < 7; ++j)
        if (k + j * P < S) acc += v[j];
    }
  }
  red[ph * GPW + gl] = acc;
  __syncthreads();
  if (ph == 0 && i < total) {
    f32x4 sm = red[gl];
    for (int k = 1; k < P; ++k) sm += red[k * GPW + gl];
    if (TR) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = q4 * 4 + e;
        if (co < Cout_real) {
          float* d = dw + ((size_t)co * Cin_real + rw) * taps + tap;
          *d = sm[e] * scale + (accumulate ? *d : 0.f);
        }
      }
    } else if constexpr (CIG) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int pc = inv[q4 * 4 + e];
        if (pc >= 0) {
          float* d = dw + ((size_t)rw * Cin_real + pc) * taps + tap;
          *d = sm[e] * scale + (accumulate ? *d : 0.f);
        }
      }
    } else {
      float* d = dw + ((size_t)rw * Cin_real + q4 * 4) * taps + tap;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[(size_t)e * taps] = sm[e] * scale + (accumulate ? d[(size_t)e * taps] : 0.f);
    }
  }
}

// Slab reduction for Cin_real % 4 == 0 (16-B loads, or gathered through ci_map): 64 (tap, co, 4 ci) groups per
// 1024-thread block; the 16 waves take splits k = wave (mod 16) with independent 16-B loads
// (coalesced along ci), then a fixed-order LDS combine -- deterministic, and S / 16 loads
// per thread instead of S.  The last ceil(Cout_real / 64) blocks sum the bias slab the same
// way (one co per lane).
__global__ __launch_bounds__(1024) void wgrad_reduce4_kernel(const float* ws, const float* wsb, float* dw, float* db,
                                                             int S, int Cout, int Cin, int Cout_real, int Cin_real,
                                                             int out_ps, int taps, const int* co_map,
                                                             const int* ci_map, float scale, int wblocks,
                                                             int accumulate) {
  __shared__ f32x4 red[16][64];
  const int t = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1;
  const int cps = Cout_real / r2;
  if ((int)blockIdx.x >= wblocks) {  // bias
    const int c = ((int)blockIdx.x - wblocks) * 64 + t;
    float sb = 0.f;
    if (c < Cout_real) {
      const int cop = co_map ? co_map[c] : (out_ps > 0 ? (c % r2) * cps + c / r2 : c);
      for (int k = wv; k < S; k += 16) sb += wsb[(size_t)k * Cout + cop];
    }
    red[wv][t] = f32x4{sb, 0.f, 0.f, 0.f};
    __syncthreads();
    if (wv == 0 && c < Cout_real) {
      float sm = red[0][t][0];
#pragma unroll
      for (int k = 1; k < 16; ++k) sm += red[k][t][0];
      db[c] = sm * scale + (accumulate ? db[c] : 0.f);
    }
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * 64 + t;
  const int c4n = Cin_real >> 2;
  const int64_t total = (int64_t)taps * Cout_real * c4n;
  int co = 0, ci4 = 0, tap = 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    ci4 = (int)(i % c4n);
    const int64_t t2 = i / c4n;
    co = (int)(t2 % Cout_real);
    tap = (int)(t2 / Cout_real);
    const int cop = co_map ? co_map[co] : (out_ps > 0 ? (co % r2) * cps + co / r2 : co);
    const size_t stride = (size_t)taps * Cout * Cin;
    const float* row = ws + ((size_t)tap * Cout + cop) * Cin;
    if (ci_map) {  // GEMM channels of the 4 parameter channels (padded heads): gathered loads
      int cip[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) cip[e] = ci_map[ci4 * 4 + e];
      for (int k = wv; k < S; k += 16) {
        const float* sk = row + (size_t)k * stride;
        acc += f32x4{sk[cip[0]], sk[cip[1]], sk[cip[2]], sk[cip[3]]};
      }
    } else {
      const float* src = row + ci4 * 4;
      int k = wv;
      for (; k + 48 < S; k += 64) {
        const f32x4 v0 = *(const f32x4*)(src + (size_t)k * stride);
        const f32x4 v1 = *(const f32x4*)(src + (size_t)(k + 16) * stride);
        const f32x4 v2 = *(const f32x4*)(src + (size_t)(k + 32) * stride);
        const f32x4 v3 = *(const f32x4*)(src + (size_t)(k + 48) * stride);
        acc += v0; acc += v1; acc += v2; acc += v3;
      }
      for (; k < S; k += 16) acc += *(const f32x4*)(src + (size_t)k * stride);
    }
  }
  red[wv][t] = acc;
  __syncthreads();
  if (wv == 0 && i < total) {
    f32x4 sm = red[0][t];
#pragma unroll
    for (int k = 1; k < 16; ++k) sm += red[k][t];
    float* d = dw + ((size_t)co * Cin_real + ci4 * 4) * taps + tap;
#pragma unroll
    for (int e = 0; e < 4; ++e) d[(size_t)e * taps] = sm[e] * scale + (accumulate ? d[(size_t)e * taps] : 0.f);
  }
}

// Slab reduction for the row-streaming wgrad's [S][taps][Cin][Cout] slab: 64 (tap, ci, 4 co)
// groups per 1024-thread block, 16-B loads coalesced along co, the 16 waves take splits
// k = wave (mod 16), fixed-order LDS combine (deterministic); bias blocks as wgrad_reduce4_kernel.
__global__ __launch_bounds__(1024) void wgrad_reduce_tr_kernel(const float* ws, const float* wsb, float* dw, float* db,
                                                               int S, int Cout, int Cin, int Cout_real, int Cin_real,
                                                               int taps, const int* co_map, const int* ci_map,
                                                               float scale, int wblocks, int accumulate, int out_ps) {
  __shared__ f32x4 red[16][64];
  const int t = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1, cps = Cout_real / r2;
  // GEMM column of parameter output channel c (co_map, or the PixelShuffle order: slot c % r^2)
  auto gcol = [&](int c) { return co_map ? co_map[c] : (out_ps > 0 ? (c % r2) * cps + c / r2 : c); };
  if ((int)blockIdx.x >= wblocks) {  // bias
    const int c = ((int)blockIdx.x - wblocks) * 64 + t;
    float sb = 0.f;
    if (c < Cout_real) {
      const int cop = gcol(c);
      for (int k = wv; k < S; k += 16) sb += wsb[(size_t)k * Cout + cop];
    }
    red[wv][t] = f32x4{sb, 0.f, 0.f, 0.f};
    __syncthreads();
    if (wv == 0 && c < Cout_real) {
      float sm = red[0][t][0];
#pragma unroll
      for (int k = 1; k < 16; ++k) sm += red[k][t][0];
      db[c] = sm * scale + (accumulate ? db[c] : 0.f);
    }
    return;
  }
  const int64_t i = (int64_t)blockIdx.x * 64 + t;
  const int c4n = (Cout_real + 3) >> 2;
  const int64_t total = (int64_t)taps * Cin_real * c4n;
  int co4 = 0, ci = 0, tap = 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (i < total) {
    co4 = (int)(i % c4n);
    const int64_t t2 = i / c4n;
    ci = (int)(t2 % Cin_real);
    tap = (int)(t2 / Cin_real);
    const int cip = ci_map ? ci_map[ci] : ci;
    const size_t stride = (size_t)taps * Cin * Cout;
    const float* row = ws + ((size_t)tap * Cin + cip) * Cout;
    if (co_map || out_ps > 0) {  // GEMM columns of the 4 parameter channels: gathered loads
      int cop[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) cop[e] = co4 * 4 + e < Cout_real ? gcol(co4 * 4 + e) : 0;
      for (int k = wv; k < S; k += 16) {
        const float* sk = row + (size_t)k * stride;
        acc += f32x4{sk[cop[0]], sk[cop[1]], sk[cop[2]], sk[cop[3]]};
      }
    } else {
      const float* src = row + co4 * 4;
      int k = wv;
      for (; k + 48 < S; k += 64) {
        const f32x4 v0 = *(const f32x4*)(src + (size_t)k * stride);
        const f32x4 v1 = *(const f32x4*)(src + (size_t)(k + 16) * stride);
        const f32x4 v2 = *(const f32x4*)(src + (size_t)(k + 32) * stride);
        const f32x4 v3 = *(const f32x4*)(src + (size_t)(k + 48) * stride);
        acc += v0; acc += v1; acc += v2; acc += v3;
      }
      for (; k < S; k += 16) acc += *(const f32x4*)(src + (size_t)k * stride);
    }
  }
  red[wv][t] = acc;
  __syncthreads();
  if (wv == 0 && i < total) {
    f32x4 sm = red[0][t];
#pragma unroll
    for (int k = 1; k < 16; ++k) sm += red[k][t];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co4 * 4 + e;
      if (co < Cout_real) {
        float* d = dw + ((size_t)co * Cin_real + ci) * taps + tap;
        *d = sm[e] * scale + (accumulate ? *d : 0.f);
      }
    }
  }
}

// One element (n, ci, tap) of the padded GEMM images of a conv / linear weight (and, for i <
// Cout, its bias entry): wf [Cout][taps*Cin] forward rows, wd [Cin][taps*Cout] the flipped
// transposed dgrad rows; row_map / col_map (or the PixelShuffle permutation) give the source
// output / input channel of each padded row / column (-1: zero padding).
template <typename T>
SR_DEV void prep_elem(const float* w, const float* bias, int Cout_real, int Cin_real, int Cout, int Cin, int out_ps,
                      int taps, const int* row_map, const int* col_map, T* wf, T* wd, float* bias_g, int64_t i) {
  const int64_t total = (int64_t)Cout * Cin * taps;
  const int r2 = out_ps > 0 ? out_ps * out_ps : 1;
  const int cps = Cout_real / r2;
  auto row_of = [&](int n) -> int {
    if (row_map) return row_map[n];
    if (n >= Cout_real) return -1;
    return out_ps > 0 ? (n % cps) * r2 + n / cps : n;
  };
  if (i < total) {
    const int tap = (int)(i % taps);
    const int ci = (int)((i / taps) % Cin);
    const int n = (int)(i / ((int64_t)taps * Cin));
    const int co = row_of(n);
    const int cs = col_map ? col_map[ci] : (ci < Cin_real ? ci : -1);
    float v = 0.f;
    if (co >= 0 && cs >= 0) v = w[((size_t)co * Cin_real + cs) * taps + tap];
    if (wf) wf[(size_t)n * taps * Cin + (size_t)tap * Cin + ci] = Elt<T>::from_f(v);
    if (wd) wd[(size_t)ci * taps * Cout + (size_t)(taps - 1 - tap) * Cout + n] = Elt<T>::from_f(v);
  }
  if (bias_g && i < Cout) {
    const int n = (int)i;
    const int co = row_of(n);
    bias_g[n] = (co >= 0 && bias) ? bias[co] : 0.f;
  }
}

template <typename T>
__global__ void prep_kernel(const float* w, const float* bias, int Cout_real, int Cin_real, int Cout, int Cin,
                            int out_ps, int taps, const int* row_map, const int* col_map, T* wf, T* wd,
                            float* bias_g) {
  prep_elem<T>(w, bias, Cout_real, Cin_real, Cout, Cin, out_ps, taps, row_map, col_map, wf, wd, bias_g,
               (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// All of a net's cached GEMM images in one launch (after an optimizer step): block b belongs
// to the item whose [block_start[k], block_start[k+1]) range holds it, and owns a 32 (GEMM row n)
// x 32 (channel ci) tile of it, all taps.  The tile is read coalesced along (ci, tap) -- the
// fp32 [Cout][Cin][taps] layout -- into LDS, then written as 64-B runs along ci (wf rows) and
// along n (wd rows), instead of one scattered 2-B store per element per image.
constexpr int PREP_T = 32;
template <typename T>
__global__ __launch_bounds__(256) void prep_batch_kernel(const sr_prep_item* __restrict__ items,
                                                         const int* __restrict__ block_start, int n) {
  __shared__ float tile[PREP_T][9][PREP_T + 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  int lo = 0, hi = n - 1;  // last k with block_start[k] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (block_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const sr_prep_item it = items[lo];
  const int taps = it.ksize == 1 ? 1 : 9;
  const int tci = (it.Cin + PREP_T - 1) / PREP_T;
  const int t = b - block_start[lo];
  const int n0 = (t / tci) * PREP_T, c0 = (t % tci) * PREP_T;
  const int r2 = it.out_ps > 0 ? it.out_ps * it.out_ps : 1;
  const int cps = it.Cout_real / r2;
  auto row_of = [&](int nn) -> int {
    if (it.row_map) return it.row_map[nn];
    if (nn >= it.Cout_real) return -1;
    return it.out_ps > 0 ? (nn % cps) * r2 + nn / cps : nn;
  };
  const int per = PREP_T * taps;  // elements per GEMM row of the tile
  for (int idx = tid; idx < PREP_T * per; idx += 256) {
    const int nl = idx / per, rem = idx - nl * per;
    const int cil = rem / taps, tap = rem - cil * taps;
    const int nn = n0 + nl, ci = c0 + cil;
    float v = 0.f;
    if (nn < it.Cout && ci < it.Cin) {
      const int co = row_of(nn);
      const int cs = it.col_map ? it.col_map[ci] : (ci < it.Cin_real ? ci : -1);
      if (co >= 0 && cs >= 0) v = it.w[((size_t)co * it.Cin_real + cs) * taps + tap];
    }
    tile[nl][tap][cil] = v;
  }
  if (it.bias_g && c0 == 0 && tid < PREP_T) {
    const int nn = n0 + tid;
    if (nn < it.Cout) {
      const int co = row_of(nn);
      it.bias_g[nn] = (co >= 0 && it.bias) ? it.bias[co] : 0.f;
    }
  }
  __syncthreads();
  T* wf = (T*)it.wf;
  T* wd = (T*)it.wd;
  if (Elt<T>::SIZE == 2 && it.Cin % 8 == 0 && it.Cout % 8 == 0) {
    // bf16: 8 consecutive GEMM-row elements per thread, one 16-B store (with Cin and Cout multiples of
    // 8 and the tile origins of 32, an 8-run lies wholly inside or outside the image; a pixel-shuffled
    // conv's Cout -- 27 at x3 -- takes the element loop below); the 2-B stores of that loop ran at
    // ~1.5 TB/s (EDSR: 227 us per step)
    constexpr int G8 = PREP_T / 8;
    for (int g = tid; g < PREP_T * taps * G8; g += 256) {
      const int a0 = g / (taps * G8), r = g - a0 * (taps * G8);
      const int tap = r / G8, e8 = (r - tap * G8) * 8;
      if (wf) {  // wf[n][tap][ci]: n = n0 + a0, ci = c0 + e8 ..
        const int nn = n0 + a0, ci = c0 + e8;
        if (nn < it.Cout && ci < it.Cin) {
          u32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(tile[a0][tap][e8 + 2 * j], tile[a0][tap][e8 + 2 * j + 1]);
          *(u32x4*)(wf + (size_t)nn * taps * it.Cin + (size_t)tap * it.Cin + ci) = o;
        }
      }
      if (wd) {  // wd[ci][taps - 1 - tap][n]: ci = c0 + a0, n = n0 + e8 ..
        const int ci = c0 + a0, nn = n0 + e8;
        if (nn < it.Cout && ci < it.Cin) {
          u32x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(tile[e8 + 2 * j][tap][a0], tile[e8 + 2 * j + 1][tap][a0]);
          *(u32x4*)(wd + (size_t)ci * taps * it.Cout + (size_t)(taps - 1 - tap) * it.Cout + nn) = o;
        }
      }
    }
    return;
  }
  for (int idx = tid; idx < PREP_T * per; idx += 256) {
    if (wf) {  // wf[n][tap][ci]: runs along ci
      const int nl = idx / per, rem = idx - nl * per;
      const int tap = rem / PREP_T, cil = rem - tap * PREP_T;
      const int nn = n0 + nl, ci = c0 + cil;
      if (nn < it.Cout && ci < it.Cin) wf[(size_t)nn * taps * it.Cin + (size_t)tap * it.Cin + ci] = Elt<T>::from_f(tile[nl][tap][cil]);
    }
    if (wd) {  // wd[ci][taps - 1 - tap][n]: runs along n
      const int cil = idx / per, rem = idx - cil * per;
      const int tap = rem / PREP_T, nl = rem - tap * PREP_T;
      const int nn = n0 + nl, ci = c0 + cil;
      if (nn < it.Cout && ci < it.Cin)
        wd[(size_t)ci * taps * it.Cout + (size_t)(taps - 1 - tap) * it.Cout + nn] = Elt<T>::from_f(tile[nl][tap][cil]);
    }
  }
}

template <typename T, int BM, int BN, int WM, int WN>
hipError_t launch_fwd(const FwdArgs& a0, hipStream_t s) {
  FwdArgs a = a0;
  const int tm = (a.M + BM - 1) / BM;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  a.tiles = tm * a.tiles_n;
  hipLaunchKernelGGL((conv3x3_fwd_kernel<T, BM, BN, WM, WN>), dim3(a.tiles), dim3(256), 0, s, a);
  return hipGetLastError();
}

// pph over 64-px column strips (STRIP): bf16, W a multiple of 64 above 128 (EDSR at LR 256: the body
// convs and their dgrads), H a multiple of 4, no pixel-shuffled input, no channel sums.  Variant 77:
// the pp kernel for them (A/B, tests).
bool fwd_use_pph_strip(const FwdArgs& a) {
  return g_variant != 2 && g_variant != 24 && g_variant != 77 && a.W > 128 && a.W % 64 == 0 && a.H % 4 == 0 &&
         a.Cin % 64 == 0 && a.in_ps == 0 && a.in_up == 1 && a.tap0 == 0 && !a.colsum;
}
// Halo variant of the 256x256 kernel: whole-row tiles of W = 64 / 128 images, 64-channel chunks.
bool fwd_use_pph(const FwdArgs& a) {
  return g_variant != 2 && g_variant != 24 &&
         ((a.W == 64 && a.H % 4 == 0) || (a.W == 128 && a.H % 2 == 0)) && a.Cin % 64 == 0 &&
         (a.in_ps == 0 || (a.fd_cps.d % 64 == 0 && g_variant != 50)) && a.in_up == 1 && a.tap0 == 0;
}

hipError_t launch_fwd_big(const FwdArgs& a0, hipStream_t s) {
  FwdArgs a = a0;
  const int tm = (a.M + 255) / 256;
  a.tiles_n = (a.Cout + 255) / 256;
  a.tiles = tm * a.tiles_n;
  if (g_variant == 2)
    hipLaunchKernelGGL(conv3x3_fwd_big_kernel, dim3(a.tiles), dim3(512), 0, s, a);
  else if (fwd_use_pph_strip(a)) {
    a.strip64 = 1;
    hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<4, 2, true>), dim3(a.tiles), dim3(512), 0, s, a);
  } else if (fwd_use_pph(a) && a.W == 128 && g_variant != 59)
    if (g_variant == 61) hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<2, 1>), dim3(a.tiles), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<2, 2>), dim3(a.tiles), dim3(512), 0, s, a);
  else if (fwd_use_pph(a) && a.W == 128)
    hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<2, 0>), dim3(a.tiles), dim3(512), 0, s, a);
  else if (g_variant != 59 && fwd_use_pph(a))
    if (g_variant == 61) hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<4, 1>), dim3(a.tiles), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<4, 2>), dim3(a.tiles), dim3(512), 0, s, a);
  else if (fwd_use_pph(a))
    hipLaunchKernelGGL((conv3x3_fwd_pph_kernel<4, 0>), dim3(a.tiles), dim3(512), 0, s, a);
  else if ((a.Cin % 64 == 0 || a.tap0 == 4) && (a.in_ps == 0 || a.fd_cps.d % 64 == 0))
    hipLaunchKernelGGL(conv3x3_fwd_pp_kernel<true>, dim3(a.tiles), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL(conv3x3_fwd_pp_kernel<false>, dim3(a.tiles), dim3(512), 0, s, a);
  return hipGetLastError();
}

// Narrow-conv halo kernel: bf16 3x3, W 64 or 128, whole-row 256-pixel tiles; Cout <= 64 in one
// block column, Cout 65..255 (RRDB dense-block dgrads) in 64-channel block columns.  (Round 4's
// one-row tiles for the wide W-256 convs measured slower than the pp / tile kernels and were removed
// in round 5: EDSR conv_last dgrad 1390 vs 550 us, profiles/r04/halo256/.)
bool fwd_use_halo(const FwdArgs& a, bool bf) {
  // pixel-shuffled input (the upsample convs' dgrads into 64 channels) when each 64-channel chunk lies
  // in one shuffle slot; variant 68: the tile kernel for those (A/B)
  const bool ps_ok = a.in_ps > 0 && a.fd_cps.d % 64 == 0 && a.W != 256 && g_variant != 68;
  if (!bf || a.in_up != 1 || (a.in_ps != 0 && !ps_ok) || a.tap0 != 0 || g_variant == 1) return false;
  if (a.W == 256)  // HR-resolution tail convs (conv_last, Cout <= 16, NCHW store): one row per tile
    return a.Cout <= 16 && g_variant != 29;
  return !a.out_nchw && a.Cout < 256 && (a.W == 64 || a.W == 128) && a.H % (256 / a.W) == 0;
}

hipError_t launch_fwd_halo(const FwdArgs& a0, hipStream_t s) {
  FwdArgs a = a0;
  a.tiles_n = (a.Cout + 63) / 64;
  a.tiles = a.M / 256;
  const int ct = (a.Cout + 15) / 16;
  const dim3 grid(a.tiles, a.tiles_n);
  if (a.W == 256) hipLaunchKernelGGL((conv3x3_fwd_halo_kernel<1, true>), grid, dim3(256), 0, s, a);
  else if (ct == 1) hipLaunchKernelGGL(conv3x3_fwd_halo_kernel<1>, grid, dim3(256), 0, s, a);
  else if (ct == 2 && a.in_ps == 0)
    hipLaunchKernelGGL((conv3x3_fwd_halo_kernel<2, false, false, 3>), grid, dim3(256), 0, s, a);
  else if (ct == 2) hipLaunchKernelGGL(conv3x3_fwd_halo_kernel<2>, grid, dim3(256), 0, s, a);
  else if (!a.colsum && !a.out_nchw && a.out_ps == 0)
    hipLaunchKernelGGL((conv3x3_fwd_halo_kernel<4, false, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv3x3_fwd_halo_kernel<4>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// Kernel family sr_conv3x3_fwd launches for a call (dispatch, kernel names and the
// epilogue geometry behind colsum all follow this one choice).
enum FwdKind { FK_HALO, FK_BIG, FK_256_16, FK_256_32, FK_128_64, FK_128_128, FK_LIN, FK_BAND, FK_TAIL, FK_BANDS };
// row-streaming narrow conv: bf16 3x3, Cin 32 / 64, Cout 32 / 64 exactly, W 64 / 128, plain or
// channel-slice NHWC in and out (variant 34: the tile kernel instead, for A/B)
// the band kernel's compile-time epilogue code (see conv3x3_fwd_band_kernel) for these arguments,
// -1 when it is not one of the instantiated ones
int band_epi(const FwdArgs& a, int grid) {
  int gate = 0;
  if (a.gate) gate = a.gate_mode == 2 ? 3 : (a.gate_mode == 1 ? 2 : 1);
  const int e = a.act | (gate << 2) | (a.res ? 16 : 0) | (a.res2 ? 32 : 0) | (a.aux ? 64 : 0) |
                (a.colsum || a.dot ? 128 : 0) | (a.row_scale ? 256 : 0) | (a.dot ? 512 : 0);  // dot implies colsum
  if (a.row_scale) {  // the images of one band fit one wave's lanes
    const int rows = (a.N * a.H + grid - 1) / grid;
    if ((rows + a.H - 1) / a.H + 1 > 64) return -1;
  }
  switch (e) {
    case 0: case 1: case 2: case 4: case 16: case 20: case 28: case 48: case 72: case 128: case 304: return e;
    case 656: return a.Cin == 64 && a.Cout == 64 ? e : -1;  // RCAB conv1 dgrad + the CA dot partials
    default: return -1;
  }
}
bool fwd_use_band(const FwdArgs& a, bool bf) {
  if (!(bf && a.tap0 == 0 && a.in_up == 1 && a.in_ps == 0 && !a.out_nchw && a.out_ps == 0 &&
        (a.W == 64 || a.W == 128) && (a.Cin == 32 || a.Cin == 64) && (a.Cout == 32 || a.Cout == 64) &&
        a.Cout_real == a.Cout && g_variant != 1 && g_variant != 34))  // 34: the tile kernel (A/B, tests)
    return false;
  const int rows = a.N * a.H, gmax = g_variant == 35 ? 64 : 256;
  return band_epi(a, rows < gmax ? rows : gmax) >= 0;
}
// 64-channel-output convs on images wider than 128 px (W 256 / 512: the RRDBNet HR convs conv_up1 /
// conv_up2 / conv_hr, their dgrads and conv_last's dgrad from its 8 padded output channels), and W 128
// with the nearest x2 upsample folded in, as band launches over 128-px column strips (STRIP: E bit
// 10): Cin 64 with a plain, ReLU, LeakyReLU or lrelu-gate epilogue, Cin 8..32 plain or gated.
// Variant 76: the generic tile kernel for them (A/B, tests).
bool fwd_use_band_strip(const FwdArgs& a, bool bf) {
  if (!(bf && a.tap0 == 0 && (a.in_up == 1 || a.in_up == 2) && a.in_ps == 0 && !a.out_nchw && a.out_ps == 0 &&
        a.W % 128 == 0 && (a.W > 128 || a.in_up == 2) && (a.Cin == 64 || (a.Cin <= 32 && a.Cin % 8 == 0)) &&
        (a.Cout == 64 || (a.Cin <= 32 && (a.Cout == 128 || a.Cout == 256))) && a.Cout_real == a.Cout &&
        !a.colsum && !a.dot && !a.row_scale && !a.res2 && !a.aux && g_variant != 1 && g_variant != 34 &&
        g_variant != 76))
    return false;
  const int e = band_epi(a, 256);
  if (a.Cout > 64) return e == 0;  // 8-channel input into 128 / 256 (EDSR's conv_last dgrad): one launch
  return a.Cin == 64 ? (e == 0 || e == 1 || e == 2 || e == 4) : (e == 0 || e == 4);
}
// the same from a narrow input (Cin 8..32) into 192 output channels (or 128 / 256 with an epilogue
// operand): 64-channel output-column slices, the narrow input re-read per slice.  (EDSR's conv_last
// dgrad, 8 -> 256 at HR, ran as four slices at 99 us each -- 2.7 TB/s, bound by the per-row latency of
// a band that stores 128 B per pixel -- and is now one CO 256 launch.)
bool fwd_use_band_strip_sliced(const FwdArgs& a, bool bf) {
  if (!(a.Cout > 64 && a.Cout <= 256 && a.Cout % 64 == 0 && a.Cin <= 32) || fwd_use_band_strip(a, bf)) return false;
  FwdArgs b = a;
  b.Cout = b.Cout_real = 64;
  return fwd_use_band_strip(b, bf);
}
// wider outputs (RRDB dense-block dgrads: Cout 96..192 from a 32- or 64-channel input) as
// band launches over 64-channel output column slices: the narrow input is re-read per slice
bool fwd_use_band_sliced(const FwdArgs& a, bool bf) {
  if (!(bf && a.tap0 == 0 && a.in_up == 1 && a.in_ps == 0 && !a.out_nchw && a.out_ps == 0 &&
        (a.W == 64 || a.W == 128) && (a.Cin == 32 || a.Cin == 64) && a.Cout > 64 && a.Cout < 256 &&
        a.Cout % 32 == 0 && a.Cout_real == a.Cout && !a.colsum && g_variant != 1 && g_variant != 34))
    return false;
  const int rows = a.N * a.H, gmax = g_variant == 35 ? 64 : 256;
  return band_epi(a, rows < gmax ? rows : gmax) >= 0;
}
// the lin kernel's compile-time epilogue code for these arguments (see conv3x3_lin_kernel), -1
// for the run-time-flag form; instantiated: plain (qkv fwd, proj dgrad), GELU' gate (fc2
// dgrad), residual (proj fwd), GELU + pre-activation (fc1 fwd), residual + row scale (proj
// fwd with stochastic depth)
int lin_epi(const FwdArgs& a) {
  int gate = 0;
  if (a.gate) gate = a.gate_mode == 2 ? 3 : (a.gate_mode == 1 ? 2 : 1);
  const int e = a.act | (gate << 2) | (a.res ? 16 : 0) | (a.res2 ? 32 : 0) | (a.aux ? 64 : 0) |
                (a.row_scale ? 128 : 0);
  if (a.row_scale && (a.H * a.W) % 128) return -1;  // row scale uniform per 128-token block
  if ((size_t)a.M * a.ldy * 2 >= 0x80000000ull) return -1;  // buffer-store offsets are 31-bit
  switch (e) {
    case 0: case 8: case 16: case 67: case 144: return e;
    default: return -1;
  }
}
// short-K 1x1 convs (linears): token tile staged once, all output channels swept.  K <= 192 on
// 128-token tiles; 192 < K <= 576 (SwinIR fc2 fwd 360 -> 184, fc1 / qkv dgrads 360 / 576 -> 184) on
// 64-token tiles, Cout <= 384 (variant 55: those on the 256x256 pp kernel instead, for A/B)
bool fwd_use_lin(const FwdArgs& a, bool bf) {
  if (!(bf && a.tap0 == 4 && !a.out_nchw && a.out_ps == 0 && a.in_ps == 0 && a.in_up == 1 && g_variant != 1))
    return false;
  if (a.Cin <= 192) return a.Cout <= 640;
  return a.Cin <= 576 && a.Cout <= 384 && g_variant != 55;
}
// linear_wk_kernel for the linears with K > SR_LWK_MINK (default 0: all; 192: only the wide-K ones,
// which the 64-token lin kernel took), K <= 576, 96 < Cout <= 576 and a plain / GELU' gate / GELU +
// pre-activation / residual / residual + row-scale epilogue; knob SR_LWK=0 or variant 64: the lin kernel (A/B, tests)
bool lin_use_wk(const FwdArgs& a) {
  const int mink = sr_knob(K_LWK) == 0 ? (1 << 30) : (sr_knob(K_LWK_MINK) > 0 ? sr_knob(K_LWK_MINK) : 0);
  if (g_variant == 64 || a.Cin <= mink || a.Cin > 576 || a.Cout > 576 || a.Cout <= 96) return false;
  const int e = lin_epi(a);
  return e == 0 || e == 8 || e == 16 || e == 67 || e == 144;
}
// HR tail convs: Cout <= 16 with the NCHW fp32 store, W >= 256 (32-px strips), Cin 64 / 128 / 256
bool fwd_use_tail(const FwdArgs& a, bool bf) {
  return bf && a.tap0 == 0 && a.in_up == 1 && a.in_ps == 0 && a.out_ps == 0 && a.out_nchw && a.Cout <= 16 &&
         a.W >= 256 && a.W % 32 == 0 && (a.Cin == 64 || a.Cin == 128 || a.Cin == 256) && !a.gate && !a.res && !a.res2 &&
         !a.aux && !a.colsum && !a.row_scale && g_variant != 1 && g_variant != 29;
}
FwdKind fwd_kind(const FwdArgs& a, bool bf) {
  if (fwd_use_tail(a, bf)) return FK_TAIL;
  if (fwd_use_lin(a, bf)) return FK_LIN;
  if (fwd_use_band(a, bf) || fwd_use_band_strip(a, bf)) return FK_BAND;
  if (fwd_use_band_sliced(a, bf) || fwd_use_band_strip_sliced(a, bf)) return FK_BANDS;
  // 128 < Cout < 256 from Cin >= 128, K a multiple of 64 (SwinIR-M's 180 -> 180 convs with the GEMM K padded
  // to 192 on the host, ops/conv.py _kpad): the halo-row 256x256 kernel with a partial output tile rather
  // than the 64-channel halo kernel (variant 79: the halo kernel, A/B and tests)
  if (bf && a.Cout > 128 && a.Cout < 256 && a.Cin >= 128 && !a.out_nchw && a.out_ps == 0 && !a.colsum &&
      !a.dot && fwd_use_pph(a) && !g_disable_big && g_variant != 79)
    return FK_BIG;
  if (fwd_use_halo(a, bf)) return FK_HALO;
  // 1x1 convs with K > 192 (SwinIR fc2 fwd, qkv / fc1 dgrads: K 368 / 576 -> 184) on the 256x256
  // kernel with a partial N tile: x read once (vs twice by 128x128 tiles); 68 -> 57 us and 82 -> 65 us
  const bool lin_big = a.tap0 == 4 && a.Cin > 192 && a.Cout >= 128;
  if (bf && !a.out_nchw && (a.Cout >= 256 || lin_big) && a.in_up == 1 && !g_disable_big) return FK_BIG;
  if (a.out_nchw || a.Cout <= 16) return FK_256_16;
  if (a.Cout <= 32) return FK_256_32;
  if (a.Cout <= 64) return FK_128_64;
  return FK_128_128;
}
// Rows per epilogue chunk and threads per block of each family: colsum has
// M / rows * threads / 64 partial rows.
void fwd_epi_geom(FwdKind k, int* rows, int* nt) {
  *rows = (k == FK_256_16 || k == FK_256_32) ? 256 : 128;
  *nt = k == FK_BIG ? 512 : 256;
}

// waves per band block: 8 at W 128, 4 at W 64.  With channel sums
// at Cout 32, 4: the partial rows per image (H x pixel waves) then match the tile and halo
// epilogues' (H W / 128 x 4), so the count does not depend on which of them a call lands on.
// Band-reduced channel sums: when the band grid splits the rows evenly and a band never crosses an
// image (rows per band divides H), each band leaves one partial row per pixel wave instead of one per
// row -- RCAN B 32: 16 instead of 128 partial rows per image, the count the standalone partials pass
// (sr_channel_partials) gives, so the channel-attention kernels that sum them stage 8x less.  Returns
// the rows per band, 0 when the sums stay per row.  Variant 37: per-row sums (tests).
int band_grid(const FwdArgs& a) {
  const int rows = a.N * a.H, gmax = g_variant == 35 ? 64 : 256;
  return rows < gmax ? rows : gmax;
}
int band_cs_rows(const FwdArgs& a) {
  const int T = a.N * a.H, G = band_grid(a);
  if (g_variant == 37 || T % G || a.H % (T / G) || T / G < 2) return 0;
  return T / G;
}
int band_nwv(const FwdArgs& a) {
  return a.W == 128 && !(a.Cout == 32 && (a.colsum || a.dot)) ? 8 : 4;
}
hipError_t launch_band8(const FwdArgs& a, hipStream_t s) {
  const int rows = a.N * a.H;
  FwdArgs ab = a;
  ab.stamps = g_sr_stamps;
  ab.cs_band = a.colsum ? band_cs_rows(a) : 0;
  const int gmax = g_variant == 35 ? 64 : 256;
  const dim3 grid(rows < gmax ? rows : gmax);
  const int e = band_epi(a, grid.x);
#define SR_BAND_E(CO_, W_, LA_, KH_, E_) \
  case E_: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<CO_, W_, LA_, KH_, E_, 8>), grid, dim3(512), 0, s, ab); break;
#define SR_BAND(CO_, W_, LA_, KH_) \
  if (a.Cout == CO_ && a.W == W_ && a.Cin == 32 * KH_) { \
switch (e) { \
  SR_BAND_E(CO_, W_, LA_, KH_, 0) SR_BAND_E(CO_, W_, LA_, KH_, 1) SR_BAND_E(CO_, W_, LA_, KH_, 2) \
  SR_BAND_E(CO_, W_, LA_, KH_, 4) SR_BAND_E(CO_, W_, LA_, KH_, 16) SR_BAND_E(CO_, W_, LA_, KH_, 20) \
  SR_BAND_E(CO_, W_, LA_, KH_, 28) \
  SR_BAND_E(CO_, W_, LA_, KH_, 48) SR_BAND_E(CO_, W_, LA_, KH_, 72) SR_BAND_E(CO_, W_, LA_, KH_, 128) \
  SR_BAND_E(CO_, W_, LA_, KH_, 304) \
  default: return hipErrorInvalidValue; \
} \
return hipGetLastError(); \
  }
  if (e == 656) {  // instantiated for the RCAN shapes only
    hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 656, 8>), grid, dim3(512), 0, s, ab);
    return hipGetLastError();
  }
  SR_BAND(64, 128, 3, 2) SR_BAND(64, 128, 3, 1) SR_BAND(32, 128, 4, 2) SR_BAND(32, 128, 4, 1)
#undef SR_BAND
#undef SR_BAND_E
  return hipErrorInvalidValue;
}
hipError_t launch_band_strip(const FwdArgs& a, hipStream_t s) {
  const int rows = a.N * a.H * (a.W / 128);
  FwdArgs ab = a;
  ab.stamps = g_sr_stamps;
  const int gmax = g_variant == 35 ? 64 : 256;  // 35: long bands crossing strips and images (tests)
  const dim3 grid(rows < gmax ? rows : gmax);
  if (a.Cin <= 32 && a.Cout > 64) {  // plain epilogue only (fwd_use_band_strip)
    if (a.Cout == 256) hipLaunchKernelGGL((conv3x3_fwd_band_kernel<256, 128, 3, 1, 1024, 8>), grid, dim3(512), 0, s, ab);
    else hipLaunchKernelGGL((conv3x3_fwd_band_kernel<128, 128, 3, 1, 1024, 8>), grid, dim3(512), 0, s, ab);
    return hipGetLastError();
  }
  if (a.Cin <= 32) {
    switch (band_epi(a, grid.x)) {
      case 0: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 1, 1024, 8>), grid, dim3(512), 0, s, ab); break;
      case 4: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 1, 1028, 8>), grid, dim3(512), 0, s, ab); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  switch (band_epi(a, grid.x)) {
    case 0: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 1024, 8>), grid, dim3(512), 0, s, ab); break;
    case 1: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 1025, 8>), grid, dim3(512), 0, s, ab); break;
    case 2: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 1026, 8>), grid, dim3(512), 0, s, ab); break;
    case 4: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 1028, 8>), grid, dim3(512), 0, s, ab); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
hipError_t launch_band(const FwdArgs& a, hipStream_t s) {
  if (a.W > 128 || a.in_up != 1) return launch_band_strip(a, s);
  if (band_nwv(a) == 8) return launch_band8(a, s);
  // one block per CU (one wave per SIMD: the weights live in registers); variant 35 forces 64 blocks
  // (long bands: ring wrap-around and image crossings inside a band, for tests).  (Two bands per CU
  // for the band_occ forms measured faster alone but slower in the RCAN step beside the side-stream
  // weight gradients; the switch was removed in round 5.)
  const int rows = a.N * a.H;
  const int gmax = g_variant == 35 ? 64 : 256;
  FwdArgs ab = a;
  ab.stamps = g_sr_stamps;
  ab.cs_band = a.colsum ? band_cs_rows(a) : 0;
  const dim3 grid(rows < gmax ? rows : gmax);
  const int e = band_epi(a, grid.x);
  if (e == 656) {  // instantiated for the RCAN shapes only
    if (a.W == 64) hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 64, 5, 2, 656>), grid, dim3(256), 0, s, ab);
    else hipLaunchKernelGGL((conv3x3_fwd_band_kernel<64, 128, 3, 2, 656>), grid, dim3(256), 0, s, ab);
    return hipGetLastError();
  }
#define SR_BAND_E(CO_, W_, LA_, KH_, E_) \
  case E_: hipLaunchKernelGGL((conv3x3_fwd_band_kernel<CO_, W_, LA_, KH_, E_>), grid, dim3(256), 0, s, ab); break;
#define SR_BAND(CO_, W_, LA_, KH_) \
  if (a.Cout == CO_ && a.W == W_ && a.Cin == 32 * KH_) { \
switch (e) { \
  SR_BAND_E(CO_, W_, LA_, KH_, 0) SR_BAND_E(CO_, W_, LA_, KH_, 1) SR_BAND_E(CO_, W_, LA_, KH_, 2) \
  SR_BAND_E(CO_, W_, LA_, KH_, 4) SR_BAND_E(CO_, W_, LA_, KH_, 16) SR_BAND_E(CO_, W_, LA_, KH_, 20) \
  SR_BAND_E(CO_, W_, LA_, KH_, 28) \
  SR_BAND_E(CO_, W_, LA_, KH_, 48) SR_BAND_E(CO_, W_, LA_, KH_, 72) SR_BAND_E(CO_, W_, LA_, KH_, 128) \
  SR_BAND_E(CO_, W_, LA_, KH_, 304) \
  default: return hipErrorInvalidValue; \
} \
return hipGetLastError(); \
  }
  SR_BAND(64, 64, 5, 2) SR_BAND(64, 64, 5, 1) SR_BAND(32, 64, 5, 2) SR_BAND(32, 64, 5, 1)
  SR_BAND(64, 128, 3, 2) SR_BAND(64, 128, 3, 1) SR_BAND(32, 128, 4, 2) SR_BAND(32, 128, 4, 1)
#undef SR_BAND
#undef SR_BAND_E
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t dispatch_fwd(const FwdArgs& a, hipStream_t s) {
  switch (fwd_kind(a, sizeof(T) == 2)) {
case FK_LIN: {
  FwdArgs b = a;
  const int e = lin_epi(a);
  if (lin_use_wk(a)) {  // 128-token x 192-channel tiles, K streamed
    const dim3 grid(((a.M + 127) / 128) * ((a.Cout + 191) / 192));
    if (e == 0) hipLaunchKernelGGL(linear_wk_kernel<0>, grid, dim3(256), 0, s, b);
    else if (e == 8) hipLaunchKernelGGL(linear_wk_kernel<8>, grid, dim3(256), 0, s, b);
    else if (e == 67) hipLaunchKernelGGL(linear_wk_kernel<67>, grid, dim3(256), 0, s, b);
    else if (e == 16) hipLaunchKernelGGL(linear_wk_kernel<16>, grid, dim3(256), 0, s, b);
    else hipLaunchKernelGGL(linear_wk_kernel<144>, grid, dim3(256), 0, s, b);
    return hipGetLastError();
  }
  if (a.Cin > 192) {  // wide K: 64-token tiles, the whole K (<= 384 / 576) staged
    b.tiles = (a.M + 63) / 64;
#define SR_LINW_E(CG_, NP_, E_) \
  case E_: hipLaunchKernelGGL((conv3x3_lin_kernel<64, CG_, NP_, E_>), dim3(b.tiles), dim3(256), 0, s, b); break;
#define SR_LINW(CG_, NP_) \
  case NP_: \
switch (e) { \
  SR_LINW_E(CG_, NP_, 0) SR_LINW_E(CG_, NP_, 16) SR_LINW_E(CG_, NP_, 144) \
  default: hipLaunchKernelGGL((conv3x3_lin_kernel<64, CG_, NP_, -1>), dim3(b.tiles), dim3(256), 0, s, b); \
} \
break;
    if (a.Cin <= 384) {
      switch ((a.Cout + 127) / 128) { SR_LINW(6, 1) SR_LINW(6, 2) SR_LINW(6, 3) default: return hipErrorInvalidValue; }
    } else {
      switch ((a.Cout + 127) / 128) { SR_LINW(9, 1) SR_LINW(9, 2) SR_LINW(9, 3) default: return hipErrorInvalidValue; }
    }
#undef SR_LINW
#undef SR_LINW_E
    return hipGetLastError();
  }
  b.tiles = (a.M + 127) / 128;
#define SR_LIN_E(NP_, E_) \
  case E_: hipLaunchKernelGGL((conv3x3_lin_kernel<128, 3, NP_, E_>), dim3(b.tiles), dim3(256), 0, s, b); break;
#define SR_LIN(NP_) \
  case NP_: \
switch (e) { \
  SR_LIN_E(NP_, 0) SR_LIN_E(NP_, 8) SR_LIN_E(NP_, 16) SR_LIN_E(NP_, 67) SR_LIN_E(NP_, 144) \
  default: hipLaunchKernelGGL((conv3x3_lin_kernel<128, 3, NP_, -1>), dim3(b.tiles), dim3(256), 0, s, b); \
} \
break;
  switch ((a.Cout + 127) / 128) {
    SR_LIN(1) SR_LIN(2) SR_LIN(3) SR_LIN(4) SR_LIN(5)
    default: return hipErrorInvalidValue;
  }
#undef SR_LIN
#undef SR_LIN_E
  return hipGetLastError();
}
case FK_BAND: return launch_band(a, s);
case FK_BANDS: {
  // 64-channel output column slices (the last may be 32 wide), each a band launch with the
  // weight rows, bias, output / residual / gate columns and the gate / residual column
  // ranges shifted to the slice
  for (int n0 = 0; n0 < a.Cout; n0 += 64) {
    FwdArgs b = a;
    const int cw = a.Cout - n0 < 64 ? a.Cout - n0 : 64;
    b.Cout = b.Cout_real = cw;
    b.w = (const bf16_t*)a.w + (size_t)n0 * a.ldw;
    b.w_bytes = a.w_bytes - (uint32_t)((size_t)n0 * a.ldw * 2);
    if (a.bias) b.bias = a.bias + n0;
    b.ycoff = a.ycoff + n0;
    b.gcoff = a.gcoff + n0;
    b.rcoff = a.rcoff + n0;
    b.r2coff = a.r2coff + n0;
    b.gcol0 = a.gcol0 - n0;
    b.gcol1 = a.gcol1 - n0;
    b.rcols = a.rcols - n0;
    const hipError_t e = launch_band(b, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
case FK_TAIL: {
  FwdArgs b = a;
  b.tiles = a.H < 32 ? a.H : 32;  // rows per band
  const dim3 grid((unsigned)(a.N * (a.W / 32) * ((a.H + b.tiles - 1) / b.tiles)));
  switch (a.Cin / 64) {
    case 1: hipLaunchKernelGGL(conv3x3_fwd_tail_kernel<1>, grid, dim3(256), 0, s, b); break;
    case 2: hipLaunchKernelGGL(conv3x3_fwd_tail_kernel<2>, grid, dim3(256), 0, s, b); break;
    case 3: return hipErrorInvalidValue;
    default: hipLaunchKernelGGL(conv3x3_fwd_tail_kernel<4>, grid, dim3(256), 0, s, b); break;
  }
  return hipGetLastError();
}
case FK_HALO: return launch_fwd_halo(a, s);
case FK_BIG: return launch_fwd_big(a, s);
case FK_256_16: return launch_fwd<T, 256, 16, 4, 1>(a, s);
case FK_256_32: return launch_fwd<T, 256, 32, 4, 1>(a, s);
case FK_128_64: return launch_fwd<T, 128, 64, 2, 2>(a, s);
default: return launch_fwd<T, 128, 128, 2, 2>(a, s);
  }
}

inline int tile_for(int c) { return c <= 16 ? 16 : c <= 32 ? 32 : c <= 64 ? 64 : 128; }
// wgrad tile (co x ci): grow the larger side until 4 waves each own a 16x16 sub-tile.
inline void wg_tiles(int cout, int cin, int* bm, int* bn) {
  int m = tile_for(cout), n = tile_for(cin);
  while ((m / 16) * (n / 16) < 4) {
    if (m <= n) n *= 2; else m *= 2;
  }
  *bm = m;
  *bn = n;
}

// Wave grid (WM x WN = 4) for a BMW x BNW wgrad tile: every wave needs >= one 16x16 tile.
constexpr int wg_wm(int bm, int bn) {
  return (bm >= 32 && bn >= 32) ? 2 : (bm >= 64 ? 4 : 1);
}

template <typename T, int BMW, int BNW>
hipError_t launch_wg(WgArgs a, hipStream_t s) {
  constexpr int WM = wg_wm(BMW, BNW);
  constexpr int WN = 4 / WM;
  static_assert(BMW / WM >= 16 && BNW / WN >= 16, "wgrad tile too small for 4 waves");
  a.tiles_co = (a.Cout + BMW - 1) / BMW;
  a.tiles_ci = (a.Cin + BNW - 1) / BNW;
  const int blocks = a.splits * a.taps * a.tiles_co * a.tiles_ci;
  hipLaunchKernelGGL((conv3x3_wgrad_kernel<T, BMW, BNW, WM, WN>), dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename T>
hipError_t dispatch_wg(const WgArgs& a, hipStream_t s) {
  int bm, bn;
  wg_tiles(a.Cout, a.Cin, &bm, &bn);
#define SR_WG(X, Y) \
  if (bm == X && bn == Y) return launch_wg<T, X, Y>(a, s);
  SR_WG(128, 128) SR_WG(128, 64) SR_WG(64, 128) SR_WG(64, 64) SR_WG(128, 32) SR_WG(32, 128)
  SR_WG(128, 16) SR_WG(16, 128) SR_WG(64, 32) SR_WG(32, 64) SR_WG(64, 16) SR_WG(16, 64)
  SR_WG(32, 32)
#undef SR_WG
  return hipErrorInvalidValue;
}

// Weight gradients with >= 128 channels each side that are not multiples of 128 (SwinIR linears
// 184 / 368 / 576, its 184-channel 3x3 convs): the 256x256 phase-interleaved kernel with partial
// tiles (columns past Cout / Cin read neighbouring data that only feeds the discarded rows /
// columns of the tile) -- far fewer operand re-reads than 128x128 tiles.
bool wg_use_pp_partial(const sr_conv3x3_wgrad_desc* d) {
  return d->dtype == SR_BF16 && d->Cout >= 128 && d->Cin >= 128 && d->W % 64 == 0 &&
         d->in_up <= 1 && d->out_ps == 0 && !g_disable_big && g_variant != 2 && g_variant != 28;
}

bool wg_use_big(const sr_conv3x3_wgrad_desc* d) {
  return (d->dtype == SR_BF16 && d->Cout >= 256 && d->Cin >= 256 && d->in_up <= 1 && !g_disable_big) ||
         wg_use_pp_partial(d);
}

// Phase-interleaved wgrad kernel: W a multiple of 64, channel counts (and the pixel-shuffle
// slot width) multiples of 128.
bool wg_use_pp(const sr_conv3x3_wgrad_desc* d) {
  if (!wg_use_big(d) || g_variant == 2) return false;
  if (wg_use_pp_partial(d)) return true;
  const int cps = d->out_ps > 0 ? d->Cout / (d->out_ps * d->out_ps) : 128;
  return d->W % 64 == 0 && d->Cout % 128 == 0 && d->Cin % 128 == 0 && cps % 128 == 0;
}

// Splits per bias-role block of the pp kernel (0: one bias block per split, interleaved with the
// tile blocks).  The bias role reads dy only, so a third of the CUs' worth of bias blocks can take
// three splits each and the tile blocks get more, shorter splits (EDSR-L body wgrad, 247 blocks:
// 176 -> 170 us).  3x3 convs only (the SwinIR linears' slabs are HBM traffic: more splits cost
// there).  (Groups of 2 and the interleaved layout were variants 51 / 53 until round 6.)
int wg_bias_group(const sr_conv3x3_wgrad_desc* d) {
  if (d->ksize == 1 || !wg_use_pp(d)) return 0;
  return 3;
}

// The pp kernel's bias gradient inside its centre-tap blocks: no bias-role blocks, so one 256-block
// wave holds floor(256 / tiles) splits.  Taken for Cout > 256 (the EDSR upsample convs, 36 tiles:
// 6 -> 7 splits, 677 -> 650 us at 64^2, 2614 -> 2517 us at 128^2); at one co tile the centre-tap
// blocks' extra MFMAs cost more than the split gained (EDSR body 170 -> 177 us, SwinIR 3x3 161 ->
// 173 us), so those keep the grouped bias blocks.
bool wg_bias_fused(const sr_conv3x3_wgrad_desc* d) {
  if (d->ksize == 1 || !wg_use_pp(d)) return false;
  return d->Cout > 256;
}

// Row-streaming wgrad over 64-channel output tiles of a wider conv (Cout above 64, the last tile
// partial): a block is (split, co tile, 64-ci chunk); at 80 KB of LDS two blocks share a CU, so the
// plan targets 512 blocks.  Taken where the 256x256 pp kernel is not at home -- channel counts that
// are not multiples of 128 (SwinIR's 184-channel convs: 164 -> 116 us at B 32, 64^2) or Cin < 128
// (the head convs); on the EDSR-L body shape it ties the pp kernel (193 vs 189 us; 256 blocks 256 us,
// 3 / 4 steps in flight 250-280 us: LDS for one block per CU), which stays there.
// knob SR_RING_WIDE: 0 = off, > 0 = on for every Cout > 64 shape with that block target (A/B);
// variant 62: on everywhere (parity tests).
int ring_wide_env() {
  const int x = sr_knob(K_RING_WIDE);
  return x >= -1 && x <= 4096 ? x : -1;
}
int ring_wide_target() {
  if (g_variant == 62) return 512;
  const int v = ring_wide_env();
  return v < 0 ? 512 : v;
}
bool wg_ring_wide(const sr_conv3x3_wgrad_desc* d) {
  if (ring_wide_target() <= 0 || g_variant == 1 || d->dtype != SR_BF16 || d->ksize == 1 || d->Cout <= 64 ||
      d->W % 64 || d->in_up > 2)
    return false;
  const bool ps_off = sr_knob(K_RING_PS) == 0;
  if (d->out_ps > 0 && (d->in_up > 1 || (d->Cout / (d->out_ps * d->out_ps)) % 64 != 0 || g_variant == 67 || ps_off))
    return false;  // pixel-shuffled dy: each 64-wide co tile inside one shuffle slot; variant 67 / knob SR_RING_PS=0: off (A/B)
  if (g_variant == 62 || ring_wide_env() > 0) return true;
  return d->Cout % 128 != 0 || d->Cin % 128 != 0;
}
// Kernel-row wgrad (conv3x3_wgrad_row3_kernel): bf16 3x3, Cout % 256, Cin % 128, W % 64, no upsample,
// pixel-shuffled dy when a 256-co tile lies in one shuffle slot (the EDSR-L body and upsample convs).  Knob SR_WG_ROW3=0 or variant 78: the pp kernel (A/B, parity
// cross-check); SR_WG_ROW3=k > 0: bias-role blocks of k splits (default 2).
int wg_row3_bg() {
  const int k = sr_knob(K_WG_ROW3);
  return k > 0 && k <= 64 ? k : 2;
}
bool wg_use_row3(const sr_conv3x3_wgrad_desc* d) {
  if (sr_knob(K_WG_ROW3) == 0 || g_variant == 1 || g_variant == 2 || g_variant == 28 || g_variant == 62 ||
      g_variant == 78)
    return false;
  const bool ps_ok = d->out_ps == 0 || (d->Cout / (d->out_ps * d->out_ps)) % 256 == 0;  // a co tile in one slot
  return d->dtype == SR_BF16 && d->ksize != 1 && d->Cout % 256 == 0 && d->Cin % 128 == 0 && d->W % 64 == 0 &&
         ps_ok && d->in_up <= 1 && ring_wide_env() <= 0;
}
// 1x1 weight gradient on linear_wgrad_kernel (192x192 tiles): bf16 dense token rows, no pixel
// shuffle / upsample.  Knob SR_LWG=0 or variant 63: off (the pp kernel, A/B and tests).
bool wg_use_lin(const sr_conv3x3_wgrad_desc* d) {
  const bool off = sr_knob(K_LWG) == 0;
  return !off && g_variant != 63 && g_variant != 1 && d->dtype == SR_BF16 && d->ksize == 1 && d->in_up <= 1 &&
         d->out_ps == 0 && d->Cout >= 64 && d->Cin >= 64;
}
// Block target of its split plan: 128 (half the chip: it runs on the weight-gradient side stream beside
// the main stream, and half the splits halve its slab; SwinIR 35.74 -> 34.71 ms against 256, 160 / 96 / 64
// slower, round 5), or knob SR_LWG_T (A/B)
int lin_wg_target() {
  const int x = sr_knob(K_LWG_T);
  return x >= 16 && x <= 4096 ? x : 128;
}
// Row-streaming wgrad (conv3x3_wgrad_ring_kernel): bf16 3x3, Cout <= 64, W % 64 == 0, nearest upsample
// <= 2 (or over 64-channel output tiles, wg_ring_wide).
bool wg_use_halo(const sr_conv3x3_wgrad_desc* d) {
  if (wg_ring_wide(d)) return true;
  return d->dtype == SR_BF16 && d->ksize != 1 && d->Cout <= 64 && d->W % 64 == 0 && d->in_up <= 2 && d->out_ps == 0 &&
         g_variant != 1;
}

// Block target of the narrow ring wgrad split plan: 512, or knob SR_RING_SPLITS (A/B sweeps)
int ring_split_target() {
  const int x = sr_knob(K_RING_SPLITS);
  return x >= 16 && x <= 4096 ? x : 512;
}
// 16-channel co tiles per wave of the ring wgrad and its output-channel tiles
int ring_ct(const sr_conv3x3_wgrad_desc* d) { return wg_ring_wide(d) ? 4 : (d->Cout + 15) / 16; }
int ring_tiles_co(const sr_conv3x3_wgrad_desc* d) { return wg_ring_wide(d) ? (d->Cout + 63) / 64 : 1; }

// Split-K factor: enough blocks to cover the chip (~1 round of 256 one-per-CU blocks for the
// 256x256 kernel, ~2 rounds for the small ones), pixels per split a multiple of 64.
void wgrad_plan(const sr_conv3x3_wgrad_desc* d, int* splits, int* kper) {
  const int M = d->N * d->H * d->W;
  int bm, bn, target;
  int extra = 0;  // bias-role blocks per split (big kernel)
  if (wg_use_halo(d)) {
    // ~2 blocks per CU, but at least 8 K-steps per block (the slab costs 8 B per tap-MAC row)
    // (A/B on RCAN / RRDB: twice or half as many splits are 6-12 % slower per step)
    const int chunks = (d->Cin + 63) / 64;
    int S = (wg_ring_wide(d) ? ring_wide_target() : ring_split_target()) / (chunks * ring_tiles_co(d));
    const int maxS = M / 512 > 1 ? M / 512 : 1;
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    // whole image rows per split
    const int rows = d->N * d->H;
    const int rps = (rows + S - 1) / S;
    *splits = (rows + rps - 1) / rps;
    *kper = rps * d->W;
    return;
  }
  if (wg_use_lin(d)) {
    const int tiles = ((d->Cout + 191) / 192) * ((d->Cin + 191) / 192);
    int S = lin_wg_target() / tiles;
    const int maxS = (M + 63) / 64;
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    int kp = (M + S - 1) / S;
    kp = (kp + 63) / 64 * 64;
    *splits = (M + kp - 1) / kp;
    *kper = kp;
    return;
  }
  if (wg_use_row3(d)) {  // one 256-block wave: S x 3 x tiles tile blocks + the bias-role blocks
    const int bg = wg_row3_bg(), tco = d->Cout / 256;
    const int ntile = 3 * tco * (d->Cin / 128);
    int S = (int)(256.0 / (ntile + (double)tco / bg));
    while (S > 1 && S * ntile + (S + bg - 1) / bg * tco > 256) --S;
    const int maxS = M / 64;
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    int kp = (M + S - 1) / S;
    kp = (kp + 63) / 64 * 64;
    *splits = (M + kp - 1) / kp;
    *kper = kp;
    return;
  }
  if (wg_bias_fused(d)) {
    const int ntile = 9 * ((d->Cout + 255) / 256) * ((d->Cin + 255) / 256);
    int S = 256 / ntile;
    const int maxS = (M + 255) / 256;
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    int kp = (M + S - 1) / S;
    kp = (kp + 63) / 64 * 64;
    *splits = (M + kp - 1) / kp;
    *kper = kp;
    return;
  }
  if (wg_bias_group(d) > 0) {  // pp kernel, bias-role blocks grouped (see conv3x3_wgrad_pp_kernel)
    const int bg = wg_bias_group(d), tco = (d->Cout + 255) / 256;
    const int ntile = 9 * tco * ((d->Cin + 255) / 256);
    int S = (int)(256.0 / (ntile + (double)tco / bg));
    while (S > 1 && S * ntile + (S + bg - 1) / bg * tco > 256) --S;
    const int maxS = (M + 255) / 256;
    if (S > maxS) S = maxS;
    if (S < 1) S = 1;
    int kp = (M + S - 1) / S;
    kp = (kp + 63) / 64 * 64;
    *splits = (M + kp - 1) / kp;
    *kper = kp;
    return;
  }
  if (wg_use_big(d)) {
    bm = bn = 256;
    target = 256;  // (512: 40.2 -> 41.7 ms EDSR step, round 2)
    extra = (d->Cout + 255) / 256;
  } else {
    wg_tiles(d->Cout, d->Cin, &bm, &bn);
    target = 1024;
  }
  const int taps = d->ksize == 1 ? 1 : 9;
  const int tiles = taps * ((d->Cout + bm - 1) / bm) * ((d->Cin + bn - 1) / bn) + extra;
  int S = extra ? target / tiles : (target + tiles / 2) / tiles;
  const int maxS = (M + 255) / 256;  // at least 256 pixels per split
  if (S > maxS) S = maxS;
  if (S < 1) S = 1;
  int kp = (M + S - 1) / S;
  kp = (kp + 63) / 64 * 64;
  S = (M + kp - 1) / kp;
  *splits = S;
  *kper = kp;
}

// Shape / flag fields of FwdArgs from a descriptor (no pointers; validated by the caller).
FwdArgs fwd_shape(const sr_conv3x3_desc* d) {
  const int SZ = d->dtype == SR_BF16 ? 2 : 4;
  const int PER = 16 / SZ;
  const int taps = d->ksize == 1 ? 1 : 9;
  FwdArgs a{};
  a.N = d->N; a.H = d->H; a.W = d->W; a.M = d->N * d->H * d->W;
  a.Cin = d->Cin; a.ldx = d->ldx; a.xcoff = d->xcoff; a.in_ps = d->in_ps;
  a.cpt = d->Cin / PER; a.nkc = taps * a.cpt;
  a.tap0 = taps == 1 ? 4 : 0;
  a.gate_mode = d->gate_mode;
  a.gcol0 = d->gcol0; a.gcol1 = d->gcol1;
  a.Cout = d->Cout; a.Cout_real = d->Cout_real > 0 ? d->Cout_real : d->Cout; a.ldw = d->ldw;
  a.ldy = d->ldy; a.ycoff = d->ycoff; a.out_ps = d->out_ps; a.out_nchw = d->out_nchw;
  a.act = d->act; a.slope = d->slope; a.alpha = d->alpha;
  a.ldg = d->ldg; a.gcoff = d->gcoff; a.gate_slope = d->gate_slope;
  a.ldr = d->ldr; a.rcoff = d->rcoff; a.beta = d->beta;
  a.ldr2 = d->ldr2; a.r2coff = d->r2coff; a.beta2 = d->beta2;
  a.rcols = d->rcols > 0 ? d->rcols : d->Cout;
  a.in_up = d->in_up > 1 ? d->in_up : 1;
  a.fd_cpt = make_fastdiv(a.cpt > 0 ? a.cpt : 1);
  a.fd_W = make_fastdiv(d->W > 0 ? d->W : 1);
  a.fd_H = make_fastdiv(d->H > 0 ? d->H : 1);
  int cps = 1;
  if (d->in_ps > 0) cps = d->Cin / (d->in_ps * d->in_ps);
  if (d->out_ps > 0) cps = d->Cout / (d->out_ps * d->out_ps);
  a.fd_cps = make_fastdiv(cps > 0 ? cps : 1);
  a.fd_r = make_fastdiv(d->in_ps > 0 ? d->in_ps : 1);
  a.row_scale = d->row_scale;
  a.fd_hw = make_fastdiv(d->H * d->W > 0 ? d->H * d->W : 1);
  a.dot = d->dot; a.ldd = d->ldd; a.dcoff = d->dcoff;
  if (d->dot) {  // the dot epilogue comes with a residual: the pointer-free kind / parts / name queries
    static const char one = 1;  // see the launch's epilogue code (sr_conv3x3_fwd sets the real res)
    a.res = &one;
  }
  return a;
}

// Partial rows per image of the colsum output, or 0 when the call cannot produce it.
int colsum_parts(const sr_conv3x3_desc* d, const FwdArgs& a0) {
  static float one;
  FwdArgs a = a0;
  a.colsum = &one;  // the kernel choice of a call that asks for the sums
  if (d->out_ps || d->out_nchw || fwd_kind(a, d->dtype == SR_BF16) == FK_LIN) return 0;
  if (fwd_kind(a, d->dtype == SR_BF16) == FK_BAND) {  // (rows or bands) x pixel waves
    const int rpb = band_cs_rows(a);
    return (rpb ? d->H / rpb : d->H) * (band_nwv(a) / (d->Cout / 32));
  }
  int rows, nt;
  fwd_epi_geom(fwd_kind(a, d->dtype == SR_BF16), &rows, &nt);
  const int HW = d->H * d->W;
  if (HW % rows) return 0;
  return HW / rows * (nt / 64);
}
}  // namespace

extern "C" {

int sr_conv3x3_fwd(const sr_conv3x3_desc* d, const void* x, const void* w, const float* bias,
                   const void* gate, const void* res, const void* res2, const float* aff_scale,
                   const float* aff_shift, void* y, void* aux, float* colsum, void* stream) {
  if (!d || !x || !w || !y) return sr_fail(SR_EINVAL, "conv3x3_fwd: null pointer");
  const int SZ = d->dtype == SR_BF16 ? 2 : 4;
  const int PER = 16 / SZ;
  if (d->Cin % 8 || d->ldx % PER || d->xcoff % PER || (!d->out_nchw && (d->Cout % 8)))
    return sr_fail(SR_EINVAL, "conv3x3_fwd: Cin/Cout/ld/coff must be multiples of 8 (pad channels)");
  const int taps = d->ksize == 1 ? 1 : 9;
  if (d->ksize != 0 && d->ksize != 1 && d->ksize != 3) return sr_fail(SR_EINVAL, "conv3x3_fwd: ksize must be 1 or 3");
  if (d->ldw < taps * d->Cin) return sr_fail(SR_EINVAL, "conv3x3_fwd: ldw < taps*Cin");
  if (aux && (d->out_ps || d->out_nchw)) return sr_fail(SR_EINVAL, "conv3x3_fwd: aux needs plain store");
  if ((gate || res || res2) && d->out_ps) return sr_fail(SR_EINVAL, "conv3x3_fwd: gate/res need plain store");
  const int up = d->in_up > 1 ? d->in_up : 1;
  if (up > 1 && (d->in_ps > 0 || d->H % up || d->W % up))
    return sr_fail(SR_EINVAL, "conv3x3_fwd: in_up needs H, W divisible by it and no in_ps");
  if (d->in_ps > 0 && d->out_ps > 0) return sr_fail(SR_EINVAL, "conv3x3_fwd: in_ps and out_ps exclusive");
  if (d->in_ps > 0 && (d->Cin / (d->in_ps * d->in_ps)) % PER)
    return sr_fail(SR_EINVAL, "conv3x3_fwd: shuffled channel count must be a multiple of 8");
  if (d->out_ps > 0 && (d->Cout / (d->out_ps * d->out_ps)) % PER)
    return sr_fail(SR_EINVAL, "conv3x3_fwd: shuffled channel count must be a multiple of 8");
  FwdArgs a = fwd_shape(d);
  if (colsum && colsum_parts(d, a) == 0)
    return sr_fail(SR_EINVAL, "conv3x3_fwd: colsum needs a plain store and H*W a multiple of the epilogue rows");
  const int M = a.M;
  const int r_in = d->in_ps > 0 ? d->in_ps : 1;
  const size_t xb = (size_t)M * r_in * r_in * (size_t)d->ldx * SZ / ((size_t)up * up);
  const size_t wb = (size_t)d->Cout * d->ldw * SZ;
  if (xb >= 0x80000000ull || wb >= 0x80000000ull)
    return sr_fail(SR_ETOOBIG, "conv3x3_fwd: tensor >= 2 GiB (split the batch)");
  a.x = x; a.w = w; a.bias = bias; a.gate = gate; a.res = res; a.res2 = res2;
  a.aff_scale = aff_scale; a.aff_shift = aff_shift; a.y = y; a.aux = aux; a.colsum = colsum;
  if (d->dot) {  // with every operand pointer set: the band kernel's epilogue code decides
    if (!colsum || !res || d->dtype != SR_BF16 || fwd_kind(a, true) != FK_BAND || d->ldd % 8 || d->dcoff % 8)
      return sr_fail(SR_EINVAL, "conv3x3_fwd: dot partials need colsum on the band kernel (bf16, 64 -> 64 ch)");
    const size_t db = (size_t)d->N * d->H * d->W * d->ldd * 2;
    if (db >= 0x80000000ull) return sr_fail(SR_ETOOBIG, "conv3x3_fwd: dot operand >= 2 GiB");
    a.d_bytes = (uint32_t)db;
  }
  a.x_bytes = (uint32_t)xb; a.w_bytes = (uint32_t)wb;
  a.g_bytes = gate ? (uint32_t)((size_t)M * d->ldg * SZ) : 0;
  a.r_bytes = res ? (uint32_t)((size_t)M * d->ldr * SZ) : 0;
  a.r2_bytes = res2 ? (uint32_t)((size_t)M * d->ldr2 * SZ) : 0;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = d->dtype == SR_BF16 ? dispatch_fwd<bf16_t>(a, s) : dispatch_fwd<float>(a, s);
  return sr_check(e, "conv3x3_fwd launch");
}

int sr_linear_ln_fwd(const sr_conv3x3_desc* d, const void* x, const float* ln_gamma, const float* ln_beta, int ln_C,
                     float eps, void* ln_out, float* ln_mean, float* ln_rstd, const void* w, const float* bias, void* y,
                     void* aux, void* stream) {
  if (!d || !x || !ln_gamma || !ln_beta || !ln_out || !ln_mean || !ln_rstd || !w || !y)
    return sr_fail(SR_EINVAL, "linear_ln_fwd: null pointer");
  if (d->dtype != SR_BF16 || d->ksize != 1 || d->Cin % 8 || d->Cout % 8 || d->ldx != d->Cin || d->xcoff != 0 ||
      ln_C <= 0 || ln_C > d->Cin || d->ldw < d->Cin)
    return sr_fail(SR_EINVAL, "linear_ln_fwd: bf16 1x1 conv over dense rows (ldx == Cin) with ln_C <= Cin");
  FwdArgs a = fwd_shape(d);
  if (!fwd_use_lin(a, true) || a.Cin > 192)
    return sr_fail(SR_EINVAL, "linear_ln_fwd: shape not on the lin kernel (Cin <= 192, Cout <= 640)");
  a.aux = aux;
  const int e = lin_epi(a);
  if (e != 0 && e != 67) return sr_fail(SR_EINVAL, "linear_ln_fwd: epilogue must be plain or GELU + pre-activation aux");
  const size_t xb = (size_t)a.M * d->ldx * 2, wb = (size_t)d->Cout * d->ldw * 2;
  if (xb >= 0x80000000ull || wb >= 0x80000000ull) return sr_fail(SR_ETOOBIG, "linear_ln_fwd: tensor >= 2 GiB");
  a.x = x; a.w = w; a.bias = bias; a.y = y;
  a.x_bytes = (uint32_t)xb; a.w_bytes = (uint32_t)wb;
  a.ln_g = ln_gamma; a.ln_b = ln_beta; a.ln_out = ln_out; a.ln_mean = ln_mean; a.ln_rstd = ln_rstd;
  a.ln_C = ln_C; a.ln_eps = eps;
  a.tiles = (a.M + 127) / 128;
  hipStream_t s = (hipStream_t)stream;
#define SR_LNL(NP_)                                                                                       \
  case NP_:                                                                                               \
    if (e == 0) hipLaunchKernelGGL((conv3x3_lin_kernel<128, 3, NP_, 0, true>), dim3(a.tiles), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((conv3x3_lin_kernel<128, 3, NP_, 67, true>), dim3(a.tiles), dim3(256), 0, s, a); \
    break;
  switch ((a.Cout + 127) / 128) {
    SR_LNL(1) SR_LNL(2) SR_LNL(3) SR_LNL(4) SR_LNL(5)
    default: return sr_fail(SR_EINVAL, "linear_ln_fwd: Cout > 640");
  }
#undef SR_LNL
  return sr_check(hipGetLastError(), "linear_ln_fwd launch");
}

// 1 when sr_conv3x3_fwd can fuse the dot partials (d->dot) into this conv with a residual operand:
// the band kernel's residual + colsum + dot epilogue (RCAB conv1 dgrad shapes).
int sr_conv3x3_fwd_dot_ok(const sr_conv3x3_desc* d) {
  if (!d || d->N <= 0 || d->H <= 0 || d->W <= 0 || d->dtype != SR_BF16) return 0;
  FwdArgs a = fwd_shape(d);
  static const char one = 1;
  a.res = &one;
  a.dot = &one;
  a.colsum = (float*)&one;
  sr_conv3x3_desc dd = *d;
  dd.dot = &one;
  return fwd_kind(a, true) == FK_BAND && colsum_parts(&dd, a) > 0 ? 1 : 0;
}

int sr_conv3x3_fwd_colsum_parts(const sr_conv3x3_desc* d) {
  if (!d || d->N <= 0 || d->H <= 0 || d->W <= 0) return 0;
  return colsum_parts(d, fwd_shape(d));
}

// Name of the kernel instantiation sr_conv3x3_fwd / sr_conv3x3_wgrad will launch for a
// descriptor (bench.py traces and rocprof summaries are matched on these names).
const char* sr_conv3x3_fwd_kernel_name(const sr_conv3x3_desc* d) {
  const bool bf = d->dtype == SR_BF16;
  switch (fwd_kind(fwd_shape(d), bf)) {
    case FK_LIN: return lin_use_wk(fwd_shape(d)) ? "linear_wk_kernel" : "conv3x3_lin_kernel";
    case FK_HALO: return "conv3x3_fwd_halo_kernel";
    case FK_BAND: return "conv3x3_fwd_band_kernel";
    case FK_TAIL: return "conv3x3_fwd_tail_kernel";
    case FK_BANDS: return "conv3x3_fwd_band_kernel";
    case FK_BIG: {
      if (g_variant == 2) return "conv3x3_fwd_big_kernel";
      return fwd_use_pph(fwd_shape(d)) || fwd_use_pph_strip(fwd_shape(d)) ? "conv3x3_fwd_pph_kernel" : "conv3x3_fwd_pp_kernel";
    }
    case FK_256_16: return bf ? "conv3x3_fwd_kernel<bf16,256,16>" : "conv3x3_fwd_kernel<f32,256,16>";
    case FK_256_32: return bf ? "conv3x3_fwd_kernel<bf16,256,32>" : "conv3x3_fwd_kernel<f32,256,32>";
    case FK_128_64: return bf ? "conv3x3_fwd_kernel<bf16,128,64>" : "conv3x3_fwd_kernel<f32,128,64>";
    default: return bf ? "conv3x3_fwd_kernel<bf16,128,128>" : "conv3x3_fwd_kernel<f32,128,128>";
  }
}

int sr_conv3x3_fwd_launches(const sr_conv3x3_desc* d) {
  if (!d) return 0;
  const FwdArgs a = fwd_shape(d);
  return fwd_kind(a, d->dtype == SR_BF16) == FK_BANDS ? (a.Cout + 63) / 64 : 1;
}

const char* sr_conv3x3_wgrad_kernel_name(const sr_conv3x3_wgrad_desc* d) {
  if (wg_use_halo(d)) return "conv3x3_wgrad_ring_kernel";
  if (wg_use_lin(d)) return "linear_wgrad_kernel";
  if (wg_use_row3(d)) return "conv3x3_wgrad_row3_kernel";
  if (wg_use_pp(d)) return "conv3x3_wgrad_pp_kernel";
  if (wg_use_big(d)) return "conv3x3_wgrad_big_kernel";
  return d->dtype == SR_BF16 ? "conv3x3_wgrad_kernel<bf16>" : "conv3x3_wgrad_kernel<f32>";
}

// Kernel-variant switch for the parity tests' cross-checks: 0 = automatic, 1 = never a 256x256 kernel,
// 2 = the two-barrier 256x256 kernels; the others each route one family to the kernel it replaced
// (24, 28, 29, 33, 34, 35, 36, 37, 50, 55, 59, 61, 62, 63, 64, 67, 68, 76, 77, 78, 79: see their sites above).  The
// measured-slower paths and the timing ablations were removed in round 6 (git history).
int sr_conv3x3_set_variant(int variant) {
  static const int kValid[] = {0, 1, 2, 24, 28, 29, 33, 34, 35, 36, 37, 50, 55, 59, 61, 62, 63, 64, 67, 68, 76, 77, 78, 79};
  bool ok = false;
  for (int v : kValid) ok = ok || v == variant;
  if (!ok) return sr_fail(SR_EINVAL, "conv3x3_set_variant: not a parity cross-check variant");
  g_variant = variant;
  return SR_OK;
}

int sr_conv3x3_get_variant(void) { return g_variant; }

// Diagnostics: the band kernel writes 16 clock values per block (wave 0: start, weights loaded,
// end, rows, cycles summed over rows in the row wait / barrier / MFMA / epilogue phases, then
// LDS zeroed, weight loads issued) into buf while it is set; null turns it off.
int sr_conv3x3_set_stamps(void* buf) {
  g_sr_stamps = (unsigned long long*)buf;
  return SR_OK;
}

size_t sr_conv3x3_wgrad_workspace(const sr_conv3x3_wgrad_desc* d) {
  int S, kp;
  wgrad_plan(d, &S, &kp);
  const int taps = d->ksize == 1 ? 1 : 9;
  return ((size_t)S * taps * d->Cout * d->Cin + (size_t)S * d->Cout) * sizeof(float) + 256;
}

}  // extern "C"

namespace {
// The slab reduce of a sr_conv3x3_wgrad call (S splits of its plan, slab ws, bias slab wsb)
int wgrad_reduce_launch(const sr_conv3x3_wgrad_desc* d, int S, int taps, const float* ws, const float* wsb, float* dw,
                        float* db, const int* co_map, const int* ci_map, hipStream_t s) {
  const int acc1 = d->accumulate & 1;
  const int Cout_real = d->Cout_real > 0 ? d->Cout_real : d->Cout;
  const int Cin_real = d->Cin_real > 0 ? d->Cin_real : d->Cin;
  const int64_t total = (int64_t)Cout_real * Cin_real;
  const int64_t work = total > Cout_real ? total : Cout_real;
  const bool tr = wg_use_halo(d);
  // (the row-streaming slab keeps wgrad_reduce_tr_kernel: 32-group blocks measured slower on RCAN / RRDB)
  const bool cig = !tr && ci_map && d->Cin % 4 == 0 && d->Cin <= 1024;  // ci gather on the output side
  if (!tr && ((Cin_real % 4 == 0 && !ci_map) || cig)) {
    // split phases P ~ S / 8 (pow2 <= 32), group width GPW so that the grid covers the chip
    const int64_t groups = tr ? (int64_t)taps * Cin_real * ((Cout_real + 3) / 4)
                              : (int64_t)taps * Cout_real * ((cig ? d->Cin : Cin_real) / 4);
    int P = 1;
    while (P * 8 < S && P < 32) P <<= 1;
    int gpw = 64;
    while (gpw > 16 && P * gpw / 64 > 16) gpw >>= 1;  // <= 16 waves
    while (gpw > 16 && (groups + gpw - 1) / gpw < 256 && P * gpw / 64 >= 2) gpw >>= 1;
    const int nw = P * gpw / 64 > 0 ? P * gpw / 64 : 1;
    const int wblocks = (int)((groups + gpw - 1) / gpw);
    const int bblocks = db ? (Cout_real + 63) / 64 : 0;
    const dim3 grid((unsigned)(wblocks + bblocks)), blk((unsigned)(nw * 64));
#define SR_RG(G, T, ...)                                                                                        \
  hipLaunchKernelGGL((wgrad_reduce_g_kernel<G, T, ##__VA_ARGS__>), grid, blk, (size_t)nw * 64 * 16, s, (const float*)ws, (const float*)wsb, dw, db, \
                     S, d->Cout, d->Cin, Cout_real, Cin_real, d->out_ps, taps, co_map, ci_map, d->scale, wblocks,  \
                     acc1)
    if (tr) { if (gpw == 64) SR_RG(64, true); else if (gpw == 32) SR_RG(32, true); else SR_RG(16, true); }
    else if (cig) { if (gpw == 64) SR_RG(64, false, true); else if (gpw == 32) SR_RG(32, false, true); else SR_RG(16, false, true); }
    else { if (gpw == 64) SR_RG(64, false); else if (gpw == 32) SR_RG(32, false); else SR_RG(16, false); }
#undef SR_RG
  } else if (tr) {
    const int64_t work4 = (int64_t)taps * Cin_real * ((Cout_real + 3) / 4);
    const int wblocks = (int)((work4 + 63) / 64);
    const int bblocks = db ? (Cout_real + 63) / 64 : 0;
    hipLaunchKernelGGL(wgrad_reduce_tr_kernel, dim3((unsigned)(wblocks + bblocks)), dim3(1024), 0, s,
                       (const float*)ws, (const float*)wsb, dw, db, S, d->Cout, d->Cin, Cout_real, Cin_real, taps,
                       co_map, ci_map, d->scale, wblocks, acc1, d->out_ps);
  } else if (Cin_real % 4 == 0) {
    const int64_t work4 = (int64_t)taps * Cout_real * (Cin_real / 4);
    const int wblocks = (int)((work4 + 63) / 64);
    const int bblocks = db ? (Cout_real + 63) / 64 : 0;
    hipLaunchKernelGGL(wgrad_reduce4_kernel, dim3((unsigned)(wblocks + bblocks)), dim3(1024), 0, s, (const float*)ws,
                       (const float*)wsb, dw, db, S, d->Cout, d->Cin, Cout_real, Cin_real, d->out_ps, taps, co_map,
                       ci_map, d->scale, wblocks, acc1);
  } else if (Cin_real <= 8 && g_variant != 33) {
    hipLaunchKernelGGL(wgrad_reduce_narrow_kernel, dim3((unsigned)Cout_real), dim3(256), 0, s, (const float*)ws,
                       (const float*)wsb, dw, db, S, d->Cout, d->Cin, Cin_real, d->out_ps, taps, co_map, ci_map,
                       d->scale, acc1);
  } else {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s,
                       (const float*)ws, (const float*)wsb, dw, db, S, d->Cout, d->Cin, Cout_real,
                       Cin_real, d->out_ps, taps, co_map, ci_map, d->scale, acc1);
  }
  return sr_check(hipGetLastError(), "conv3x3_wgrad reduce launch");
}
}  // namespace

extern "C" {

int sr_conv3x3_wgrad(const sr_conv3x3_wgrad_desc* d, const void* dy, const void* x, void* workspace,
                     size_t ws_bytes, float* dw, float* db, const int* co_map, const int* ci_map, void* stream) {
  if (!d || !dy || !x || !workspace || !dw) return sr_fail(SR_EINVAL, "conv3x3_wgrad: null pointer");
  const int SZ = d->dtype == SR_BF16 ? 2 : 4;
  const int PER = 16 / SZ;
  if (d->Cin % 8 || d->Cout % 8 || d->ldx % PER || d->ldy % PER || d->xcoff % PER || d->ycoff % PER)
    return sr_fail(SR_EINVAL, "conv3x3_wgrad: channel counts / strides must be multiples of 8");
  if (ws_bytes < sr_conv3x3_wgrad_workspace(d)) return sr_fail(SR_EINVAL, "conv3x3_wgrad: workspace too small");
  const int M = d->N * d->H * d->W;
  const int r = d->out_ps > 0 ? d->out_ps : 1;
  const int up = d->in_up > 1 ? d->in_up : 1;
  if (up > 1 && (d->H % up || d->W % up)) return sr_fail(SR_EINVAL, "conv3x3_wgrad: H, W must divide by in_up");
  const size_t xb = (size_t)M * d->ldx * SZ / ((size_t)up * up);
  const size_t dyb2 = (size_t)M * r * r * (size_t)d->ldy * SZ;
  if (xb >= 0x80000000ull || dyb2 >= 0x80000000ull)
    return sr_fail(SR_ETOOBIG, "conv3x3_wgrad: tensor >= 2 GiB (split the batch)");
  WgArgs a{};
  a.dy = dy; a.x = x;
  int S, kp;
  wgrad_plan(d, &S, &kp);
  a.ws = (float*)workspace;
  const int taps = d->ksize == 1 ? 1 : 9;
  a.taps = taps;
  a.tap0 = taps == 1 ? 4 : 0;
  a.wsb = db ? a.ws + (size_t)S * taps * d->Cout * d->Cin : nullptr;
  a.dy_bytes = (uint32_t)dyb2; a.x_bytes = (uint32_t)xb;
  a.N = d->N; a.H = d->H; a.W = d->W; a.M = M;
  a.Cin = d->Cin; a.ldx = d->ldx; a.xcoff = d->xcoff;
  a.Cout = d->Cout; a.ldy = d->ldy; a.ycoff = d->ycoff; a.out_ps = d->out_ps;
  a.in_up = up;
  a.splits = S; a.kper = kp;
  a.fd_W = make_fastdiv(d->W); a.fd_H = make_fastdiv(d->H);
  int cps = d->out_ps > 0 ? d->Cout / (d->out_ps * d->out_ps) : 1;
  if (d->out_ps > 0 && cps % PER)
    return sr_fail(SR_EINVAL, "conv3x3_wgrad: shuffled channel count must be a multiple of 8");
  a.fd_cps = make_fastdiv(cps);
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  a.stamps = g_sr_stamps;
  if (wg_use_halo(d)) {
    a.tiles_co = ring_tiles_co(d);
    a.tiles_ci = (a.Cin + 63) / 64;
    const int ct = ring_ct(d);
    const dim3 grid(S * a.tiles_ci * a.tiles_co);
    if (ct == 1) hipLaunchKernelGGL(conv3x3_wgrad_ring_kernel<1>, grid, dim3(256), 0, s, a);
    else if (ct == 2) hipLaunchKernelGGL(conv3x3_wgrad_ring_kernel<2>, grid, dim3(256), 0, s, a);
    else if (ct == 3) hipLaunchKernelGGL(conv3x3_wgrad_ring_kernel<3>, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(conv3x3_wgrad_ring_kernel<4>, grid, dim3(256), 0, s, a);
    e = hipGetLastError();
  } else if (wg_use_lin(d)) {
    a.tiles_co = (a.Cout + 191) / 192;
    a.tiles_ci = (a.Cin + 191) / 192;
    hipLaunchKernelGGL(linear_wgrad_kernel, dim3(S * a.tiles_co * a.tiles_ci), dim3(512), 0, s, a);
    e = hipGetLastError();
  } else if (wg_use_row3(d)) {
    a.tiles_co = a.Cout / 256;
    a.tiles_ci = a.Cin / 128;
    a.bias_group = wg_row3_bg();
    const int nb = S * 3 * a.tiles_co * a.tiles_ci + (a.wsb ? (S + a.bias_group - 1) / a.bias_group * a.tiles_co : 0);
    hipLaunchKernelGGL(conv3x3_wgrad_row3_kernel, dim3(nb), dim3(256), 0, s, a);
    e = hipGetLastError();
  } else if (wg_use_big(d)) {
    a.tiles_co = (a.Cout + 255) / 256;
    a.tiles_ci = (a.Cin + 255) / 256;
    const int per_split = taps * a.tiles_co * a.tiles_ci + (a.wsb ? a.tiles_co : 0);
    a.bias_group = wg_bias_group(d);
    a.bias_fused = wg_bias_fused(d) ? 1 : 0;
    if (a.bias_fused) {
      a.bias_group = 0;
      if (g_variant != 59)
        hipLaunchKernelGGL((conv3x3_wgrad_pp_kernel<true>), dim3(S * taps * a.tiles_co * a.tiles_ci), dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL(conv3x3_wgrad_pp_kernel<false>, dim3(S * taps * a.tiles_co * a.tiles_ci), dim3(512), 0, s, a);
    } else if (a.bias_group > 0) {
      const int nb = S * taps * a.tiles_co * a.tiles_ci + (a.wsb ? (S + a.bias_group - 1) / a.bias_group * a.tiles_co : 0);
      if (g_variant != 59) hipLaunchKernelGGL((conv3x3_wgrad_pp_kernel<true>), dim3(nb), dim3(512), 0, s, a);
      else hipLaunchKernelGGL(conv3x3_wgrad_pp_kernel<false>, dim3(nb), dim3(512), 0, s, a);
    } else if (wg_use_pp(d) && g_variant != 59)
      hipLaunchKernelGGL((conv3x3_wgrad_pp_kernel<true>), dim3(S * per_split), dim3(512), 0, s, a);
    else if (wg_use_pp(d))
      hipLaunchKernelGGL(conv3x3_wgrad_pp_kernel<false>, dim3(S * per_split), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL(conv3x3_wgrad_big_kernel, dim3(S * per_split), dim3(512), 0, s, a);
    e = hipGetLastError();
  } else {
    e = d->dtype == SR_BF16 ? dispatch_wg<bf16_t>(a, s) : dispatch_wg<float>(a, s);
  }
  if (e != hipSuccess) return sr_check(e, "conv3x3_wgrad launch");
  if (d->accumulate & 2) return SR_OK;  // bit 1: slab only (sr_conv3x3_wgrad_reduce later, e.g. on another stream)
  return wgrad_reduce_launch(d, S, taps, a.ws, a.wsb, dw, db, co_map, ci_map, s);
}

int sr_conv3x3_wgrad_reduce(const sr_conv3x3_wgrad_desc* d, void* workspace, size_t ws_bytes, float* dw, float* db,
                            const int* co_map, const int* ci_map, void* stream) {
  if (!d || !workspace || !dw) return sr_fail(SR_EINVAL, "conv3x3_wgrad_reduce: null pointer");
  if (ws_bytes < sr_conv3x3_wgrad_workspace(d)) return sr_fail(SR_EINVAL, "conv3x3_wgrad_reduce: workspace too small");
  int S, kp;
  wgrad_plan(d, &S, &kp);
  const int taps = d->ksize == 1 ? 1 : 9;
  float* ws = (float*)workspace;
  float* wsb = db ? ws + (size_t)S * taps * d->Cout * d->Cin : nullptr;
  return wgrad_reduce_launch(d, S, taps, ws, wsb, dw, db, co_map, ci_map, (hipStream_t)stream);
}

int sr_conv_prep_mapped(int dtype, int ksize, const float* w, const float* bias, int Cout_real, int Cin_real,
                        int Cout, int Cin, int out_ps, const int* row_map, const int* col_map, void* wf, void* wd,
                        float* bias_g, void* stream) {
  if (!w) return sr_fail(SR_EINVAL, "conv_prep: null weight");
  if (ksize != 1 && ksize != 3) return sr_fail(SR_EINVAL, "conv_prep: ksize must be 1 or 3");
  if ((!row_map && Cout < Cout_real) || (!col_map && Cin < Cin_real)) return sr_fail(SR_EINVAL, "conv_prep: padded < real");
  if (out_ps > 0 && (Cout_real % (out_ps * out_ps) || Cout != Cout_real || row_map))
    return sr_fail(SR_EINVAL, "conv_prep: shuffled conv needs Cout == Cout_real divisible by r^2");
  const int taps = ksize == 1 ? 1 : 9;
  const int64_t total = (int64_t)Cout * Cin * taps;
  const int64_t work = total > Cout ? total : Cout;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(prep_kernel<bf16_t>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, w, bias, Cout_real,
                       Cin_real, Cout, Cin, out_ps, taps, row_map, col_map, (bf16_t*)wf, (bf16_t*)wd, bias_g);
  else
    hipLaunchKernelGGL(prep_kernel<float>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, w, bias, Cout_real,
                       Cin_real, Cout, Cin, out_ps, taps, row_map, col_map, (float*)wf, (float*)wd, bias_g);
  return sr_check(hipGetLastError(), "conv_prep launch");
}

int sr_conv_prep_blocks(const sr_prep_item* it) {
  return ((it->Cout + PREP_T - 1) / PREP_T) * ((it->Cin + PREP_T - 1) / PREP_T);
}

int sr_conv_prep_batch(int dtype, const sr_prep_item* items, const int* block_start, int n, int total_blocks,
                       void* stream) {
  if (!items || !block_start || n <= 0 || total_blocks <= 0) return sr_fail(SR_EINVAL, "conv_prep_batch: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(prep_batch_kernel<bf16_t>, dim3(total_blocks), dim3(256), 0, s, items, block_start, n);
  else
    hipLaunchKernelGGL(prep_batch_kernel<float>, dim3(total_blocks), dim3(256), 0, s, items, block_start, n);
  return sr_check(hipGetLastError(), "conv_prep_batch launch");
}

int sr_conv3x3_prep(int dtype, const float* w, const float* bias, int Cout_real, int Cin_real, int Cout, int Cin,
                    int out_ps, void* wf, void* wd, float* bias_g, void* stream) {
  return sr_conv_prep_mapped(dtype, 3, w, bias, Cout_real, Cin_real, Cout, Cin, out_ps, nullptr, nullptr, wf, wd,
                             bias_g, stream);
}

}  // extern "C"
