// SwinIR token-side kernels: LayerNorm and fused (shifted) window attention.
//
//   sr_layernorm_fwd / _bwd : nn.LayerNorm(C) over the channel rows of an NHWC token map
//       (PatchEmbed norm, SwinTransformerBlock norm1/norm2, final norm:
//       basicsr/archs/swinir_arch.py:240, 251, 600-604, 846), eps 1e-5, fp32 statistics.
//   sr_window_attn_fwd / _bwd : WindowAttention (swinir_arch.py:144-175) including the block's
//       cyclic shift and window partition/reverse (:288-314) — the qkv rows are GATHERED by
//       (window, token) -> pixel index ((wy*ws + i/ws + s) mod H, (wx*ws + i%ws + s) mod W), so
//       torch.roll / window_partition / window_reverse never materialise; the shift mask
//       (:262-281, -100 between different regions) is computed from region ids on the fly;
//       the relative-position bias (:119-133, 157-160) is gathered from the [(2ws-1)^2, nH] table.
//
// qkv layout: per token row, [3][nH][hdp] with hdp >= head_dim (zero padded, 16-B aligned
// heads); out layout [nH][hdp].  bf16 with window 8 and hdp 32 (SwinIR-M/S/light) runs the
// MFMA kernels; other shapes and the fp32 parity mode run the fp32-FMA kernels (one wave per
// (image, window, head) unit, lane = query token).
#include <cstdlib>

#include "sr_common.h"
#include "sr_internal.h"
#include "swin_common.h"

namespace {

template <typename T>
SR_DEV float ld_elt(const T* p) {
  return Elt<T>::to_f(*p);
}

// ---------------------------------------------------------------- LayerNorm
// One wave per row; lane l holds channels l, l+64, l+128, ... (coalesced across the wave).
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, int ldx, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, int64_t M, int C, int Cp,
                                                     float eps, T* __restrict__ y, int ldy,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int MAXE = 8;  // C <= 512
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += nw) {
    const T* xr = x + row * ldx;
    float v[MAXE];
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int c = lane + 64 * e;
      v[e] = c < C ? ld_elt(xr + c) : 0.f;
      s += v[e];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    const float mu = s / C;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int c = lane + 64 * e;
      const float d = c < C ? v[e] - mu : 0.f;
      q += d * d;
    }
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
    const float rs = rsqrtf(q / C + eps);
    T* yr = y + row * ldy;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int c = lane + 64 * e;
      if (c < C) yr[c] = Elt<T>::from_f((v[e] - mu) * rs * gamma[c] + beta[c]);
      else if (c < Cp) yr[c] = Elt<T>::from_f(0.f);
    }
    if (lane == 0) {
      mean_out[row] = mu;
      rstd_out[row] = rs;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; out = dx (+ res).
// dgamma/dbeta partials per wave -> partial[wave][2][C].
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, int lddy, const T* __restrict__ x,
                                                     int ldx, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                     int64_t M, int C, int Cp, const T* __restrict__ res, int ldr,
                                                     T* __restrict__ dx, int lddx, float* __restrict__ partial) {
  constexpr int MAXE = 8;
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  float dg[MAXE], db[MAXE];
#pragma unroll
  for (int e = 0; e < MAXE; ++e) dg[e] = db[e] = 0.f;
  for (int64_t row = gw; row < M; row += nw) {
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXE], g[MAXE];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int c = lane + 64 * e;
      if (c < C) {
        const float d = ld_elt(dy + row * lddy + c);
        xh[e] = (ld_elt(x + row * ldx + c) - mu) * rs;
        g[e] = d * gamma[c];
        dg[e] += d * xh[e];
        db[e] += d;
      } else {
        xh[e] = g[e] = 0.f;
      }
      s1 += g[e];
      s2 += g[e] * xh[e];
    }
    for (int o = 32; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o);
      s2 += __shfl_xor(s2, o);
    }
    s1 /= C;
    s2 /= C;
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
      const int c = lane + 64 * e;
      if (c < C) {
        float v = rs * (g[e] - s1 - xh[e] * s2);
        if (res) v += ld_elt(res + row * ldr + c);
        dx[row * lddx + c] = Elt<T>::from_f(v);
      } else if (c < Cp) {
        dx[row * lddx + c] = Elt<T>::from_f(0.f);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int c = lane + 64 * e;
    if (c < C) {
      partial[(gw * 2 + 0) * C + c] = dg[e];
      partial[(gw * 2 + 1) * C + c] = db[e];
    }
  }
}

__global__ void ln_bwd_reduce(const float* __restrict__ partial, int nw, int C, float* __restrict__ dgamma,
                              float* __restrict__ dbeta, int acc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * C) return;
  const int which = i / C, c = i % C;
  float s = 0.f;
  for (int w = 0; w < nw; ++w) s += partial[((size_t)w * 2 + which) * C + c];
  float* o = which ? dbeta : dgamma;
  o[c] = (acc ? o[c] : 0.f) + s;
}

// Vectorised bf16 LayerNorm for padded widths Cp <= 256 (SwinIR embed 60..180): half a
// wave per row, lane hl = lane & 31 holds channels 8*hl .. 8*hl+7 (one 16-B load), so a
// wave covers 2 rows per iteration; statistics by 32-lane butterflies.
SR_DEV float hsum32(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

SR_DEV void unpack8(const u32x4& q, float* o) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[2 * j] = bf16_to_f32(q[j] & 0xffff);
    o[2 * j + 1] = bf16_to_f32(q[j] >> 16);
  }
}

SR_DEV u32x4 pack8(const float* v) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
  return o;
}

__global__ __launch_bounds__(256) void ln_fwd8_kernel(const bf16_t* __restrict__ x, int ldx, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, int64_t M, int C, int Cp, float eps,
                                                      bf16_t* __restrict__ y, int ldy, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int c0 = hl * 8;
  float gm[8], bt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gm[j] = c0 + j < C ? gamma[c0 + j] : 0.f;
    bt[j] = c0 + j < C ? beta[c0 + j] : 0.f;
  }
  // RU rows per half-wave per iteration, all loads issued before any reduction: one 16-B load
  // per lane in flight left the kernel at ~2.8 TB/s (too few bytes in flight per CU)
  constexpr int RU = 4;
  const int64_t nrw = (int64_t)gridDim.x * 8;
  for (int64_t r0 = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); r0 < M; r0 += RU * nrw) {
    u32x4 raw[RU];  // packed until use: 4 VGPRs per row in flight instead of 8
#pragma unroll
    for (int k = 0; k < RU; ++k) {
      const int64_t row = r0 + k * nrw;
      raw[k] = (c0 < Cp && row < M) ? *(const u32x4*)(x + row * ldx + c0) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < RU; ++k) {
      const int64_t row = r0 + k * nrw;
      float v[1][8];
      unpack8(raw[k], v[0]);
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c0 + j >= C) v[0][j] = 0.f;
        sm += v[0][j];
      }
      const float mu = hsum32(sm) / C;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = c0 + j < C ? v[0][j] - mu : 0.f;
        q += d * d;
      }
      const float rs = rsqrtf(hsum32(q) / C + eps);
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = c0 + j < C ? (v[0][j] - mu) * rs * gm[j] + bt[j] : 0.f;
      if (row < M) {
        if (c0 < Cp) *(u32x4*)(y + row * ldy + c0) = pack8(o);
        if (hl == 0) {
          mean_out[row] = mu;
          rstd_out[row] = rs;
        }
      }
    }
  }
}

// Backward, same mapping; per-block dgamma / dbeta partials (LDS-combined over the block's
// SLOTS row slots) -> partial[block][2][C], summed by ln_bwd_reduce8.
template <int SLOTS>
__global__ __launch_bounds__(SLOTS * 32) void ln_bwd8_kernel(const bf16_t* __restrict__ dy, int lddy, const bf16_t* __restrict__ x,
                                                      int ldx, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                      int64_t M, int C, int Cp, const bf16_t* __restrict__ res, int ldr,
                                                      bf16_t* __restrict__ dx, int lddx, float* __restrict__ partial,
                                                      const float* __restrict__ rscale, int HW, bf16_t* __restrict__ dxs) {
  __shared__ float red[SLOTS][2][256];
  const int lane = threadIdx.x & 63, hl = lane & 31, slot = threadIdx.x >> 5;
  const int c0 = hl * 8;
  float gm[8], dg[8], db[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gm[j] = c0 + j < C ? gamma[c0 + j] : 0.f;
    dg[j] = db[j] = 0.f;
  }
  const int64_t nrw = (int64_t)gridDim.x * SLOTS;
  for (int64_t row = (int64_t)blockIdx.x * SLOTS + slot; row < M; row += nrw) {
    const float mu = mean[row], rs = rstd[row];
    float d[8], xv[8], rv[8];
    if (c0 < Cp) {
      unpack8(*(const u32x4*)(dy + row * lddy + c0), d);
      unpack8(*(const u32x4*)(x + row * ldx + c0), xv);
      if (res) unpack8(*(const u32x4*)(res + row * ldr + c0), rv);
    }
    float xh[8], g[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c0 + j < C) {
        xh[j] = (xv[j] - mu) * rs;
        g[j] = d[j] * gm[j];
        dg[j] += d[j] * xh[j];
        db[j] += d[j];
      } else {
        xh[j] = g[j] = 0.f;
      }
      s1 += g[j];
      s2 += g[j] * xh[j];
    }
    s1 = hsum32(s1) / C;
    s2 = hsum32(s2) / C;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = c0 + j < C ? rs * (g[j] - s1 - xh[j] * s2) : 0.f;
      if (res && c0 + j < C) o[j] += rv[j];
    }
    if (c0 < Cp) {
      *(u32x4*)(dx + row * lddx + c0) = pack8(o);
      if (dxs) {  // also dx * rscale[image] (a stochastic-depth branch gradient), same layout
        const float sc = rscale[row / HW];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= sc;
        *(u32x4*)(dxs + row * lddx + c0) = pack8(o);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[slot][0][c0 + j] = dg[j];
    red[slot][1][c0 + j] = db[j];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * C; i += SLOTS * 32) {
    const int which = i / C, c = i - which * C;
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) sm += red[k][which][c];
    partial[((size_t)blockIdx.x * 2 + which) * C + c] = sm;
  }
}

// dgamma / dbeta = sum over nb block partials: 16 columns per 1024-thread block (23 blocks at
// C 180 instead of 6 with 64 columns), 64 row lanes per column each summing rows r, r + 64, ...
// with up to 8 independent loads in flight, then a fixed-order LDS tree -- deterministic.
__global__ __launch_bounds__(1024) void ln_bwd_reduce8(const float* __restrict__ partial, int nb, int C,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta, int acc) {
  __shared__ float red[64][17];
  const int cl = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  const bool ok = col < 2 * C;
  const int which = ok ? col / C : 0, c = ok ? col - which * C : 0;
  float sm[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) sm[u] = 0.f;
  if (ok) {
    for (int b0 = r; b0 < nb; b0 += 64 * 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int b = b0 + u * 64;
        if (b < nb) sm[u] += partial[((size_t)b * 2 + which) * C + c];
      }
    }
  }
  red[r][cl] = ((sm[0] + sm[1]) + (sm[2] + sm[3])) + ((sm[4] + sm[5]) + (sm[6] + sm[7]));
  __syncthreads();
  for (int w = 32; w > 0; w >>= 1) {
    if (r < w) red[r][cl] += red[r + w][cl];
    __syncthreads();
  }
  if (r == 0 && ok) {
    float* o = which ? dbeta : dgamma;
    o[c] = (acc ? o[c] : 0.f) + red[0][cl];
  }
}

// ---------------------------------------------------------------- window attention
struct AttnArgs {
  const void* qkv;
  const void* out;   // forward output (backward only)
  const void* dout;  // (backward only)
  void* y;           // forward: out; backward: dqkv
  float* lse;        // [units][T]
  const float* bias_table;
  float* dbias_part;  // [units][nbins] (backward)
  int ldq, ldo;
  int N, H, W, ws, shift, nH, hd, hdp;
  float scale;
  int nwx, nwin, units, T, nbins;
};

SR_DEV void unit_decode(const AttnArgs& a, int unit, int& n, int& wy, int& wx, int& h) {
  h = unit % a.nH;
  const int t = unit / a.nH;
  const int win = t % a.nwin;
  n = t / a.nwin;
  wy = win / a.nwx;
  wx = win % a.nwx;
}

SR_DEV int64_t token_pixel(const AttnArgs& a, int n, int wy, int wx, int i) {
  const int sy = wy * a.ws + i / a.ws, sx = wx * a.ws + i % a.ws;  // position in the shifted image
  int oy = sy + a.shift, ox = sx + a.shift;                          // torch.roll(-s): shifted[p] = x[p + s]
  if (oy >= a.H) oy -= a.H;
  if (ox >= a.W) ox -= a.W;
  return ((int64_t)n * a.H + oy) * a.W + ox;
}

SR_DEV int token_region(const AttnArgs& a, int wy, int wx, int i) {
  if (a.shift == 0) return 0;
  return region(wy * a.ws + i / a.ws, a.H, a.ws, a.shift) * 3 + region(wx * a.ws + i % a.ws, a.W, a.ws, a.shift);
}

SR_DEV int rel_bin(const AttnArgs& a, int i, int j) {
  const int dy = i / a.ws - j / a.ws + a.ws - 1;
  const int dx = i % a.ws - j % a.ws + a.ws - 1;
  return dy * (2 * a.ws - 1) + dx;
}

constexpr int TMAX = 64, DMAX = 32, DSTR = 33;

// One wave per unit; lane i = query token i of the window.
template <typename T>
__global__ __launch_bounds__(64) void wattn_fwd_kernel(AttnArgs a) {
  __shared__ float sK[TMAX * DSTR], sV[TMAX * DSTR];
  __shared__ int sR[TMAX];
  const int unit = blockIdx.x;
  const int i = threadIdx.x;
  int n, wy, wx, h;
  unit_decode(a, unit, n, wy, wx, h);
  const bool act = i < a.T;
  const T* qkv = (const T*)a.qkv;
  float q[DMAX];
  int64_t pi = 0;
  if (act) {
    pi = token_pixel(a, n, wy, wx, i);
    const T* row = qkv + pi * a.ldq;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      const bool dv = d < a.hd;
      q[d] = dv ? ld_elt(row + h * a.hdp + d) : 0.f;
      sK[i * DSTR + d] = dv ? ld_elt(row + (a.nH + h) * a.hdp + d) : 0.f;
      sV[i * DSTR + d] = dv ? ld_elt(row + (2 * a.nH + h) * a.hdp + d) : 0.f;
    }
    sR[i] = token_region(a, wy, wx, i);
  }
  __syncthreads();
  float srow[TMAX];
  float mx = -3.0e38f;
  if (act) {
    const int ri = sR[i];
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      float s = -3.0e38f;
      if (j < a.T) {
        float dot = 0.f;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) dot += q[d] * sK[j * DSTR + d];
        s = dot * a.scale + a.bias_table[rel_bin(a, i, j) * a.nH + h];
        if (a.shift && sR[j] != ri) s += -100.f;
      }
      srow[j] = s;
      mx = fmaxf(mx, s);
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      const float e = j < a.T ? __expf(srow[j] - mx) : 0.f;
      srow[j] = e;
      sum += e;
    }
    const float inv = 1.f / sum;
    float o[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) o[d] = 0.f;
#pragma unroll
    for (int j = 0; j < TMAX; ++j) {
      if (j < a.T) {
        const float p = srow[j] * inv;
#pragma unroll
        for (int d = 0; d < DMAX; ++d) o[d] += p * sV[j * DSTR + d];
      }
    }
    T* orow = (T*)a.y + pi * a.ldo + h * a.hdp;
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      if (d < a.hdp) orow[d] = Elt<T>::from_f(d < a.hd ? o[d] : 0.f);
    a.lse[(int64_t)unit * a.T + i] = mx + __logf(sum);
  }
}

// Backward: recompute P from lse; dV_j = sum_i P_ij dO_i, dP_ij = dO_i . V_j,
// dS = P (dP - D_i), dQ_i = scale sum_j dS_ij K_j, dK_j = scale sum_i dS_ij Q_i,
// dbias[bin(i,j)] += dS_ij.  One wave per unit; P and dS staged in LDS.
template <typename T>
__global__ __launch_bounds__(64) void wattn_bwd_kernel(AttnArgs a) {
  __shared__ float sQ[TMAX * DSTR], sK[TMAX * DSTR], sV[TMAX * DSTR], sdO[TMAX * DSTR];
  __shared__ float sP[TMAX * (TMAX + 1)], sdS[TMAX * (TMAX + 1)];
  __shared__ float sBin[(2 * 8 - 1) * (2 * 8 - 1)];
  __shared__ int sR[TMAX];
  const int unit = blockIdx.x;
  const int i = threadIdx.x;
  int n, wy, wx, h;
  unit_decode(a, unit, n, wy, wx, h);
  const bool act = i < a.T;
  const T* qkv = (const T*)a.qkv;
  int64_t pi = 0;
  float D = 0.f;
  for (int b = i; b < a.nbins; b += 64) sBin[b] = 0.f;
  if (act) {
    pi = token_pixel(a, n, wy, wx, i);
    const T* row = qkv + pi * a.ldq;
    const T* orow = (const T*)a.out + pi * a.ldo + h * a.hdp;
    const T* drow = (const T*)a.dout + pi * a.ldo + h * a.hdp;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      const bool dv = d < a.hd;
      sQ[i * DSTR + d] = dv ? ld_elt(row + h * a.hdp + d) : 0.f;
      sK[i * DSTR + d] = dv ? ld_elt(row + (a.nH + h) * a.hdp + d) : 0.f;
      sV[i * DSTR + d] = dv ? ld_elt(row + (2 * a.nH + h) * a.hdp + d) : 0.f;
      const float dov = dv ? ld_elt(drow + d) : 0.f;
      sdO[i * DSTR + d] = dov;
      D += dov * (dv ? ld_elt(orow + d) : 0.f);
    }
    sR[i] = token_region(a, wy, wx, i);
  }
  __syncthreads();
  if (act) {
    const float lse = a.lse[(int64_t)unit * a.T + i];
    const int ri = sR[i];
    for (int j = 0; j < a.T; ++j) {
      float dot = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        dot += sQ[i * DSTR + d] * sK[j * DSTR + d];
        dp += sdO[i * DSTR + d] * sV[j * DSTR + d];
      }
      float s = dot * a.scale + a.bias_table[rel_bin(a, i, j) * a.nH + h];
      if (a.shift && sR[j] != ri) s += -100.f;
      const float p = __expf(s - lse);
      const float ds = p * (dp - D);
      sP[i * (TMAX + 1) + j] = p;
      sdS[i * (TMAX + 1) + j] = ds;
      atomicAdd(&sBin[rel_bin(a, i, j)], ds);
    }
  }
  __syncthreads();
  if (act) {
    // lane i now plays key/value token j = i for dK_j, dV_j; and query i for dQ_i
    float dq[DMAX], dk[DMAX], dv[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) dq[d] = dk[d] = dv[d] = 0.f;
    for (int t = 0; t < a.T; ++t) {
      const float dsi = sdS[i * (TMAX + 1) + t];  // dS[i][t]
      const float dsj = sdS[t * (TMAX + 1) + i];  // dS[t][i]
      const float pj = sP[t * (TMAX + 1) + i];    // P[t][i]
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        dq[d] += dsi * sK[t * DSTR + d];
        dk[d] += dsj * sQ[t * DSTR + d];
        dv[d] += pj * sdO[t * DSTR + d];
      }
    }
    T* grow = (T*)a.y + pi * a.ldq;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if (d < a.hdp) {
        const bool valid = d < a.hd;
        grow[h * a.hdp + d] = Elt<T>::from_f(valid ? dq[d] * a.scale : 0.f);
        grow[(a.nH + h) * a.hdp + d] = Elt<T>::from_f(valid ? dk[d] * a.scale : 0.f);
        grow[(2 * a.nH + h) * a.hdp + d] = Elt<T>::from_f(valid ? dv[d] : 0.f);
      }
    }
  }
  __syncthreads();
  for (int b = i; b < a.nbins; b += 64) a.dbias_part[(int64_t)unit * a.nbins + b] = sBin[b];
}


// ---------------------------------------------------------------- MFMA window attention
// bf16, window 8 (64 tokens), heads padded to hdp = 32: one wave per (image, window, head)
// unit; every contraction is a v_mfma_f32_16x16x32_bf16 with a 16-row tile per lane group.
//   fragment layouts (16x16x32): A/B lane l holds row l&15, K = 8*(l>>4) .. +7; C lane l
//   holds rows 4*(l>>4) + r (r = 0..3) of column l&15.
//   forward : S^T = K Q^T (A = K rows, B = Q rows, both straight 16-B loads of the qkv
//             rows), softmax over keys per query column (lane-local + 2 butterflies),
//             O^T = V^T P^T with B = P^T taken from the C registers (K-slot order
//             {32s+4g+r, 32s+16+4g+r}) and A = V^T by ds_read_b64_tr_b16 from an LDS copy of V
//             read in the same key order.
//   backward: S = Q K^T, dP = dO V^T (direct loads), P from lse, dS = P (dP - D);
//             dV^T = dO^T P, dK^T = Q^T dS (B from registers, A tr-read), dQ^T = K^T dS^T
//             (dS^T staged in LDS as bf16, tr-read); dbias by LDS float adds.
// LDS images: [64 rows][64 B] with the 32-B half swapped on (row >> 2) & 1, and dS^T
// [64][128 B] with 32-B blocks XORed by (row >> 1) & 3: conflict-free tr reads.

__global__ __launch_bounds__(64) void wattn_fwd_mfma_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(16))) char sV[64 * 64];
  __shared__ float sT[225];
  // XCD-aware: the heads of one window (which share the qkv rows' cache lines) run on one XCD
  const int unit = (int)xcd_remap(blockIdx.x, gridDim.x), lane = threadIdx.x;
  const int g = lane >> 4, c = lane & 15, tq = (lane >> 2) & 3, tp = lane & 3;
  int n, wy, wx, h;
  unit_decode(a, unit, n, wy, wx, h);
  const bf16_t* qkv = (const bf16_t*)a.qkv;
  int64_t pix[4];
  s16x8 qf[4], kf[4];
  u32x4 vf[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pix[i] = token_pixel(a, n, wy, wx, 16 * i + c);
    const bf16_t* row = qkv + pix[i] * a.ldq + g * 8;
    qf[i] = __builtin_bit_cast(s16x8, *(const u32x4*)(row + h * 32));
    kf[i] = __builtin_bit_cast(s16x8, *(const u32x4*)(row + (a.nH + h) * 32));
    vf[i] = *(const u32x4*)(row + (2 * a.nH + h) * 32);
  }
  float tv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) tv[k] = lane + 64 * k < 225 ? a.bias_table[(lane + 64 * k) * a.nH + h] : 0.f;
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (lane + 64 * k < 225) sT[lane + 64 * k] = tv[k];
#pragma unroll
  for (int i = 0; i < 4; ++i) *(u32x4*)(sV + sx_off(16 * i + c, g)) = vf[i];
  __syncthreads();

  f32x4 acc[4][4];  // S^T[key 16i + 4g + r][query 16j + c]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(kf[i], qf[j], f32x4{0.f, 0.f, 0.f, 0.f});

  // element (key 16i + 4g + r, query 16j + c) has bin bb(g, c) + 30 (j - i) - r: 28 distinct
  // biases per lane, read once
  const int bb = ((c >> 3) - (g >> 1) + 7) * 15 + (c & 7) - 4 * (g & 1) + 7;
  float bt[7][4];
#pragma unroll
  for (int d = 0; d < 7; ++d)
#pragma unroll
    for (int r = 0; r < 4; ++r) bt[d][r] = sT[bb + 30 * (d - 3) - r];
  int rk[4][4], rq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rq[i] = region(wy * 8 + 2 * i + (c >> 3), a.H, 8, a.shift) * 3 + region(wx * 8 + (c & 7), a.W, 8, a.shift);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      rk[i][r] = region(wy * 8 + 2 * i + (g >> 1), a.H, 8, a.shift) * 3 + region(wx * 8 + 4 * (g & 1) + r, a.W, 8, a.shift);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qq = 16 * j + c;
    float mx = -3.0e38f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] * a.scale + bt[j - i + 3][r];
        if (a.shift && rk[i][r] != rq[j]) v -= 100.f;
        acc[i][j][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = __expf(acc[i][j][r] - mx);
        acc[i][j][r] = e;
        sm += e;
      }
    sm += __shfl_xor(sm, 16);
    sm += __shfl_xor(sm, 32);
    const float inv = 1.f / sm;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] *= inv;
    if (g == 0) a.lse[(int64_t)unit * 64 + qq] = mx + __logf(sm);
  }

  f32x4 o[2][4];
#pragma unroll
  for (int d = 0; d < 2; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) o[d][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    s16x8 vt[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) vt[d] = frag_tr64(sV, s, g, tq, tp, 16 * d);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x8 pb = frag_c2(acc[2 * s][j], acc[2 * s + 1][j]);
#pragma unroll
      for (int d = 0; d < 2; ++d) o[d][j] = mfma16(vt[d], pb, o[d][j]);
    }
  }
  bf16_t* out = (bf16_t*)a.y;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      uint2 w2;
      w2.x = pack_bf16x2(o[d][j][0], o[d][j][1]);
      w2.y = pack_bf16x2(o[d][j][2], o[d][j][3]);
      *(uint2*)(out + pix[j] * a.ldo + h * 32 + 16 * d + 4 * g) = w2;
    }
}

// Element (query 16i + 4g + r, key 16j + c) of a C tile has relative-position bin
// base(g, c) + 30 (i - j) + r (bin8), so a lane touches 28 distinct bins: their biases are
// read once and their dS contributions pre-summed in registers before the LDS adds.
constexpr int ATT_UPW = 4;  // windows per backward wave
constexpr int ATT_SLOTS_LANE = 28, ATT_SLOTS = 64 * ATT_SLOTS_LANE;  // per-lane bias-gradient slots
SR_DEV int bin_base_qk(int g, int c) { return ((g >> 1) - (c >> 3) + 7) * 15 + 4 * (g & 1) - (c & 7) + 7; }

// Window-attention backward at two waves per SIMD (round 4; round 2's kernel held a whole window's
// S / dP tiles, the next window's loads and the bias column in 466 registers at one wave per SIMD,
// so nothing hid its dependent load -> MFMA -> exp -> MFMA chain; it was removed in round 5 with its
// LDS-atomic bias-gradient form and the 1 / 2 windows-per-wave forms, all measured slower).  Here the queries go in two halves of 32 (the K-step of the dV / dK contractions): per
// half, S and dP for its two 16-query tiles (64 registers), P and dS, the dV^T / dK^T MFMAs, then
// dS^T of the half into a [64 keys][32 queries] LDS image and dQ of those 32 queries at once; K rows
// and Q / dO rows come from the LDS images instead of registers, the bias column from LDS per use.
// 16.2 KB of LDS and <= 256 registers: two 1-wave blocks per SIMD, one's loads under the other's
// math.  Per element the same arithmetic in the same order as round 2's kernel (bit-identical dQ / dK / dV).
template <int UPW>
__global__ __launch_bounds__(64, 2) void wattn_bwd_mfma2_kernel(AttnArgs a) {
  // [0, 4K) K image, [4K, 8K) Q, [8K, 12K) dO, [12K, 16K) dS^T of one query half
  __shared__ __attribute__((aligned(16))) char smem[4 * 4096];
  __shared__ __attribute__((aligned(16))) float sT[228], sD[64], sL[64];
  char* sK = smem;
  char* sQ = smem + 4096;
  char* sdO = smem + 8192;
  char* sdS = smem + 12288;
  const int lane = threadIdx.x;
  const int g = lane >> 4, c = lane & 15, tq = (lane >> 2) & 3, tp = lane & 3;
  const int part = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int h = part % a.nH;
  const int win0 = (part / a.nH) * UPW;
  const int bb = bin_base_qk(g, c);
  float dbs[7][4];
#pragma unroll
  for (int d = 0; d < 7; ++d)
#pragma unroll
    for (int r = 0; r < 4; ++r) dbs[d][r] = 0.f;
  const bf16_t* qkv = (const bf16_t*)a.qkv;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (lane + 64 * k < 225) sT[lane + 64 * k] = a.bias_table[(lane + 64 * k) * a.nH + h];
  for (int uw = 0; uw < UPW; ++uw) {
    const int wg = win0 + uw;
    if (wg >= a.N * a.nwin) break;
    const int unit = wg * a.nH + h;
    const int n = wg / a.nwin, win = wg - n * a.nwin;
    const int wy = win / a.nwx, wx = win - (win / a.nwx) * a.nwx;
    int64_t pix[4];
    s16x8 vf[4];
    {
      u32x4 qu[4], ku[4], vu[4], du[4], ou[4];
      f32x4 l4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pix[i] = token_pixel(a, n, wy, wx, 16 * i + c);
        const bf16_t* row = qkv + pix[i] * a.ldq + g * 8;
        qu[i] = *(const u32x4*)(row + h * 32);
        ku[i] = *(const u32x4*)(row + (a.nH + h) * 32);
        vu[i] = *(const u32x4*)(row + (2 * a.nH + h) * 32);
        const int64_t orow = pix[i] * a.ldo + h * 32 + g * 8;
        du[i] = *(const u32x4*)((const bf16_t*)a.dout + orow);
        ou[i] = *(const u32x4*)((const bf16_t*)a.out + orow);
        l4[i] = *(const f32x4*)(a.lse + (int64_t)unit * 64 + 16 * i + 4 * g);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        vf[i] = __builtin_bit_cast(s16x8, vu[i]);
        *(u32x4*)(sQ + sx_off(16 * i + c, g)) = qu[i];
        *(u32x4*)(sK + sx_off(16 * i + c, g)) = ku[i];
        *(u32x4*)(sdO + sx_off(16 * i + c, g)) = du[i];
        float t = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          t += bf16_to_f32(du[i][e] & 0xffff) * bf16_to_f32(ou[i][e] & 0xffff) +
               bf16_to_f32(du[i][e] >> 16) * bf16_to_f32(ou[i][e] >> 16);
        t += __shfl_xor(t, 16);
        t += __shfl_xor(t, 32);
        if (g == 0) sD[16 * i + c] = t;
        if (c == 0) *(f32x4*)(sL + 16 * i + 4 * g) = l4[i];
      }
    }
    __syncthreads();
    int rk[4];  // shift-mask region of key 16j + c
#pragma unroll
    for (int j = 0; j < 4; ++j)
      rk[j] = region(wy * 8 + 2 * j + (c >> 3), a.H, 8, a.shift) * 3 + region(wx * 8 + (c & 7), a.W, 8, a.shift);
    f32x4 dv[2][4], dk[2][4];
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j) dv[d][j] = dk[d][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16_t* gq = (bf16_t*)a.y;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      // S = Q K^T and dP = dO V^T for queries 16i + 4g + r (i = 2s, 2s + 1), keys 16j + c
      f32x4 pa[2][4], ds[2][4];
      {
        s16x8 kf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) kf[j] = __builtin_bit_cast(s16x8, *(const u32x4*)(sK + sx_off(16 * j + c, g)));
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
          const int i = 2 * s + ii;
          const s16x8 qf = __builtin_bit_cast(s16x8, *(const u32x4*)(sQ + sx_off(16 * i + c, g)));
          const s16x8 df = __builtin_bit_cast(s16x8, *(const u32x4*)(sdO + sx_off(16 * i + c, g)));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pa[ii][j] = mfma16(qf, kf[j], f32x4{0.f, 0.f, 0.f, 0.f});
            ds[ii][j] = mfma16(df, vf[j], f32x4{0.f, 0.f, 0.f, 0.f});
          }
        }
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii) {
        const int i = 2 * s + ii;
        const f32x4 lc = *(const f32x4*)(sL + 16 * i + 4 * g);
        const f32x4 Dq = *(const f32x4*)(sD + 16 * i + 4 * g);
        int rq[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rq[r] = region(wy * 8 + 2 * i + (g >> 1), a.H, 8, a.shift) * 3 + region(wx * 8 + 4 * (g & 1) + r, a.W, 8, a.shift);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = pa[ii][j][r] * a.scale + sT[bb + 30 * (i - j) + r];
            if (a.shift && rq[r] != rk[j]) v -= 100.f;
            const float p = __expf(v - lc[r]);
            const float dsv = p * (ds[ii][j][r] - Dq[r]);
            pa[ii][j][r] = p;
            ds[ii][j][r] = dsv;
            dbs[i - j + 3][r] += dsv;
          }
      }
      // dV^T += dO^T P and dK^T += Q^T dS over this half's 32 queries: [dim 16d + 4g + r][key 16j + c]
      {
        s16x8 at[2], qt[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          at[d] = frag_tr64(sdO, s, g, tq, tp, 16 * d);
          qt[d] = frag_tr64(sQ, s, g, tq, tp, 16 * d);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const s16x8 pb = frag_c2(pa[0][j], pa[1][j]);
          const s16x8 sb = frag_c2(ds[0][j], ds[1][j]);
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            dv[d][j] = mfma16(at[d], pb, dv[d][j]);
            dk[d][j] = mfma16(qt[d], sb, dk[d][j]);
          }
        }
      }
      // dS^T of this half: [key 16j + c][query 16 ii + 4g .. + 3] (bf16, as the one-wave kernel)
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint2 w2;
          w2.x = pack_bf16x2(ds[ii][j][0], ds[ii][j][1]);
          w2.y = pack_bf16x2(ds[ii][j][2], ds[ii][j][3]);
          *(uint2*)(sdS + sx_byte(16 * j + c, 16 * ii + 4 * g)) = w2;
        }
      __syncthreads();
      // dQ^T = K^T dS^T for queries 32s + 16jj + c: [dim 16d + 4g + r], keys in two K-steps
      f32x4 dq[2][2];
#pragma unroll
      for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) dq[d][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s16x8 kt[2];
#pragma unroll
        for (int d = 0; d < 2; ++d) kt[d] = frag_tr64(sK, ks, g, tq, tp, 16 * d);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const s16x8 sb = frag_tr64(sdS, ks, g, tq, tp, 16 * jj);
#pragma unroll
          for (int d = 0; d < 2; ++d) dq[d][jj] = mfma16(kt[d], sb, dq[d][jj]);
        }
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        bf16_t* row = gq + pix[2 * s + jj] * a.ldq + 4 * g;
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          uint2 w;
          w.x = pack_bf16x2(dq[d][jj][0] * a.scale, dq[d][jj][1] * a.scale);
          w.y = pack_bf16x2(dq[d][jj][2] * a.scale, dq[d][jj][3] * a.scale);
          *(uint2*)(row + h * 32 + 16 * d) = w;
        }
      }
      __syncthreads();  // dS^T image read: free for the next half
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16_t* row = gq + pix[j] * a.ldq + 4 * g;
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        uint2 w;
        w.x = pack_bf16x2(dk[d][j][0] * a.scale, dk[d][j][1] * a.scale);
        w.y = pack_bf16x2(dk[d][j][2] * a.scale, dk[d][j][3] * a.scale);
        *(uint2*)(row + (a.nH + h) * 32 + 16 * d) = w;
        w.x = pack_bf16x2(dv[d][j][0], dv[d][j][1]);
        w.y = pack_bf16x2(dv[d][j][2], dv[d][j][3]);
        *(uint2*)(row + (2 * a.nH + h) * 32 + 16 * d) = w;
      }
    }
    __syncthreads();  // LDS images free for the next window
  }
  // the lane's 28 pre-summed bias gradients as they are (one 1792-float slot row per wave, folded
  // into the 225 bins by wattn_dbias_slots / _fold in a fixed order): gfx950's fp32 LDS atomics
  // cost more than the rest of a wave's tail
  f32x4* dst = (f32x4*)(a.dbias_part + ((int64_t)part * 64 + lane) * ATT_SLOTS_LANE);
#pragma unroll
  for (int d = 0; d < 7; ++d) dst[d] = f32x4{dbs[d][0], dbs[d][1], dbs[d][2], dbs[d][3]};
}

// slot rows, folded into the table gradient in two fixed-order stages (deterministic):
// stage 1 (wattn_dbias_slots): block = (head, 256-slot chunk, quarter of the head's rows); a lane
// sums 4 consecutive slots with 16-B loads over rows j = q + 4 (wave + 16 k) of the head (4 loads in
// flight), the 16 waves combine through LDS in a fixed order -> slots[q][h][1792];
// stage 2 (wattn_dbias_fold): one block per head stages the head's slot row (4 quarters summed) in
// LDS and thread b folds bin b's candidate slots (d, r, gh, g1) in a fixed order.  (Round 4 ran
// stage 2 as nH blocks of branchy scalar loops over global memory: 70 us per call; a wave per
// (head, bin) gathering from global memory: 27 us.)
constexpr int DB_Q = 4;  // quarters of each head's rows in stage 1
__global__ __launch_bounds__(1024) void wattn_dbias_slots(const float* __restrict__ part, int parts, int nH,
                                                          float* __restrict__ slots) {
  __shared__ f32x4 red[16][64];
  constexpr int NCH = ATT_SLOTS / 256;  // 7 chunks of 256 slots
  const int b = blockIdx.x;
  const int q = b % DB_Q, ch = (b / DB_Q) % NCH, h = b / (DB_Q * NCH);
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sl = ch * 256 + 4 * l;
  const int rows = parts / nH;  // rows of head h: p = h + nH j
  f32x4 sm = {0.f, 0.f, 0.f, 0.f};
  int j = q + DB_Q * wv;
  constexpr int STEP = DB_Q * 16;
  for (; j + 3 * STEP < rows; j += 4 * STEP) {
    const f32x4 v0 = *(const f32x4*)(part + (int64_t)(h + nH * j) * ATT_SLOTS + sl);
    const f32x4 v1 = *(const f32x4*)(part + (int64_t)(h + nH * (j + STEP)) * ATT_SLOTS + sl);
    const f32x4 v2 = *(const f32x4*)(part + (int64_t)(h + nH * (j + 2 * STEP)) * ATT_SLOTS + sl);
    const f32x4 v3 = *(const f32x4*)(part + (int64_t)(h + nH * (j + 3 * STEP)) * ATT_SLOTS + sl);
    sm += v0; sm += v1; sm += v2; sm += v3;
  }
  for (; j < rows; j += STEP) sm += *(const f32x4*)(part + (int64_t)(h + nH * j) * ATT_SLOTS + sl);
  red[wv][l] = sm;
  __syncthreads();
  if (wv == 0) {
    f32x4 t = red[0][l];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][l];
    *(f32x4*)(slots + ((int64_t)q * nH + h) * ATT_SLOTS + sl) = t;
  }
}
// bin b's candidate slots (d, r, gh, g1) in the fold order, as a compile-time CSR table: every one of
// the 1792 slots of a row feeds exactly one of the 225 bins (1 .. 16 each).  (The fold used to test
// all 112 candidates per bin at run time, integer divisions included: 23 us per call in the step.)
struct alignas(16) DbiasTab {
  short idx[ATT_SLOTS];  // first: 16-B aligned for the staging loads
  short start[226];
};
constexpr DbiasTab make_dbias_tab() {
  DbiasTab t{};
  int n = 0;
  for (int b = 0; b < 225; ++b) {
    t.start[b] = (short)n;
    for (int e = 0; e < 112; ++e) {
      const int d = e >> 4, r = (e >> 2) & 3, gh = (e >> 1) & 1, g1 = e & 1;
      const int qq = b - 30 * (d - 3) - r;  // bin_base_qk of the contributing lanes
      if (qq < 0 || qq >= 225) continue;
      const int dyp = qq / 15, dxp = qq - 15 * dyp;  // (g >> 1) - (c >> 3) + 7, 4 (g & 1) - (c & 7) + 7
      const int chh = gh - (dyp - 7), c7 = 4 * g1 - (dxp - 7);
      if (dyp < 6 || dyp > 8 || dxp > 11 || chh < 0 || chh > 1 || c7 < 0 || c7 > 7) continue;
      t.idx[n++] = (short)(((2 * gh + g1) * 16 + 8 * chh + c7) * ATT_SLOTS_LANE + 4 * d + r);
    }
  }
  t.start[225] = (short)n;
  return t;
}
constexpr DbiasTab kDbiasTabHost = make_dbias_tab();
static_assert(kDbiasTabHost.start[225] == ATT_SLOTS, "every slot feeds one bin");
__constant__ DbiasTab kDbiasTab = make_dbias_tab();

__global__ __launch_bounds__(256) void wattn_dbias_fold(const float* __restrict__ slots, int nH,
                                                        float* __restrict__ dbias, int acc) {
  // one block per head: the head's 4 quarter rows summed into an LDS slot row with coalesced 16-B
  // loads (scattered 4-B global reads of other XCDs' freshly written lines were the cost: 27 us in
  // the step), the bin table staged beside it; then thread b sums bin b's slots in a fixed order
  __shared__ f32x4 sl4[ATT_SLOTS / 4];
  __shared__ __attribute__((aligned(16))) short sidx[ATT_SLOTS];
  __shared__ short sst[226];
  const int h = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < ATT_SLOTS / 4; i += 256) {
    f32x4 v = ((const f32x4*)(slots + (int64_t)h * ATT_SLOTS))[i];
#pragma unroll
    for (int q = 1; q < DB_Q; ++q) v += ((const f32x4*)(slots + ((int64_t)q * nH + h) * ATT_SLOTS))[i];
    sl4[i] = v;
  }
  for (int i = t; i < ATT_SLOTS / 8; i += 256) ((u32x4*)sidx)[i] = ((const u32x4*)kDbiasTab.idx)[i];
  if (t < 226) sst[t] = kDbiasTab.start[t];
  __syncthreads();
  const float* sl = (const float*)sl4;
  const int b = t;
  if (b >= 225) return;
  float s = 0.f;
  for (int i = sst[b], e = sst[b + 1]; i < e; ++i) s += sl[sidx[i]];
  dbias[b * nH + h] = (acc ? dbias[b * nH + h] : 0.f) + s;
}

__global__ void wattn_dbias_reduce2(const float* __restrict__ part, int units, int nH, int nbins,
                                    float* __restrict__ dbias, int acc);
// the table gradient from the partial rows: parts > 0 rows of nbins, parts < 0 -parts slot rows
// (stage-1 sums after them in the workspace)
void dbias_reduce(const float* ws, int parts, int nH, int nbins, float* dbias, int acc, hipStream_t s) {
  if (parts > 0) {
    hipLaunchKernelGGL(wattn_dbias_reduce2, dim3(nH * ((nbins + 63) / 64)), dim3(1024), 0, s, ws, parts, nH, nbins,
                       dbias, acc);
    return;
  }
  float* slots = const_cast<float*>(ws) + (int64_t)(-parts) * ATT_SLOTS;
  hipLaunchKernelGGL(wattn_dbias_slots, dim3(nH * (ATT_SLOTS / 256) * DB_Q), dim3(1024), 0, s, ws, -parts, nH, slots);
  hipLaunchKernelGGL(wattn_dbias_fold, dim3(nH), dim3(256), 0, s, (const float*)slots, nH, dbias, acc);
}

bool attn_mfma_ok(const AttnArgs& a, int dtype) {
  return dtype == SR_BF16 && a.ws == 8 && a.hdp == 32 && a.ldq % 8 == 0 && a.ldo % 8 == 0;
}

// dbias[bin][h] = sum over the units of head h of dbias_part[unit][bin]: one block per
// (head, 64-bin chunk), 16 waves split the units (coalesced 64-bin rows), LDS combine.
__global__ __launch_bounds__(1024) void wattn_dbias_reduce2(const float* __restrict__ part, int units, int nH, int nbins,
                                                            float* __restrict__ dbias, int acc) {
  __shared__ float red[16][64];
  const int h = blockIdx.x % nH, chunk = blockIdx.x / nH;
  const int bin = chunk * 64 + (threadIdx.x & 63), wv = threadIdx.x >> 6;
  float sm = 0.f;
  if (bin < nbins)
    for (int u = h + wv * nH; u < units; u += 16 * nH) sm += part[(int64_t)u * nbins + bin];
  red[wv][threadIdx.x & 63] = sm;
  __syncthreads();
  if (wv == 0 && bin < nbins) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][threadIdx.x];
    dbias[bin * nH + h] = (acc ? dbias[bin * nH + h] : 0.f) + t;
  }
}

bool attn_setup(AttnArgs& a, int N, int H, int W, int ws, int shift, int nH, int hd, int hdp, float scale) {
  if (ws < 1 || ws > 8 || hd > DMAX || hd > hdp || H % ws || W % ws || shift < 0 || shift >= ws) return false;
  a.N = N; a.H = H; a.W = W; a.ws = ws; a.shift = shift; a.nH = nH; a.hd = hd; a.hdp = hdp; a.scale = scale;
  a.nwx = W / ws;
  a.nwin = (H / ws) * (W / ws);
  a.units = N * a.nwin * nH;
  a.T = ws * ws;
  a.nbins = (2 * ws - 1) * (2 * ws - 1);
  return true;
}

}  // namespace

namespace {
constexpr int LN_BWD_BLOCKS = 512;
bool ln_vec8(int Cp, int ld1, int ld2) { return Cp <= 256 && Cp % 8 == 0 && ld1 % 8 == 0 && ld2 % 8 == 0; }
}  // namespace

// Absolute position embedding (swinir_arch.py:789-791, :879-880): y[n][p][c] = x[n][p][c] + pos[p][c]
// over dense token rows [N][P][Cp] (padded channels c >= C copied), and its parameter gradient
// dpos[p][c] (+)= sum_n dy[n][p][c] (fixed order over n: deterministic).
template <typename T>
__global__ void add_pos_kernel(const T* __restrict__ x, const float* __restrict__ pos, int64_t total, int P, int C,
                               int Cp, T* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const int p = (int)((i / Cp) % P);
    float v = Elt<T>::to_f(x[i]);
    if (c < C) v += pos[(int64_t)p * C + c];
    y[i] = Elt<T>::from_f(v);
  }
}

template <typename T>
__global__ void pos_grad_kernel(const T* __restrict__ dy, int N, int P, int C, int Cp, float* __restrict__ dpos,
                                int accumulate) {
  const int64_t total = (int64_t)P * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i / C), c = (int)(i - (int64_t)p * C);
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc += Elt<T>::to_f(dy[((int64_t)n * P + p) * Cp + c]);
    dpos[i] = accumulate ? dpos[i] + acc : acc;
  }
}

extern "C" {

int sr_layernorm_fwd(int dtype, const void* x, int ldx, const float* gamma, const float* beta, int64_t M, int C, int Cp,
                     float eps, void* y, int ldy, float* mean, float* rstd, void* stream) {
  if (!x || !gamma || !beta || !y || !mean || !rstd || C > 512 || Cp < C) return sr_fail(SR_EINVAL, "layernorm_fwd: bad arguments");
  const unsigned grid = (unsigned)((M + 3) / 4 < 16384 ? (M + 3) / 4 : 16384);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16 && ln_vec8(Cp, ldx, ldy)) {
    const unsigned g8 = (unsigned)((M + 7) / 8 < 4096 ? (M + 7) / 8 : 4096);
    hipLaunchKernelGGL(ln_fwd8_kernel, dim3(g8), dim3(256), 0, s, (const bf16_t*)x, ldx, gamma, beta, M, C, Cp, eps,
                       (bf16_t*)y, ldy, mean, rstd);
  } else if (dtype == SR_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, ldx, gamma, beta, M, C, Cp,
                       eps, (bf16_t*)y, ldy, mean, rstd);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)x, ldx, gamma, beta, M, C, Cp,
                       eps, (float*)y, ldy, mean, rstd);
  return sr_check(hipGetLastError(), "layernorm_fwd launch");
}

// dgamma / dbeta partial rows sr_layernorm_bwd leaves in the workspace on its vectorised path
// (bf16, Cp <= 256), 0 when that path does not apply (the reduce then always runs inside)
int sr_layernorm_bwd_parts(int dtype, int64_t M, int Cp, int ldx, int lddx, int lddy, int ldr) {
  if (!(dtype == SR_BF16 && ln_vec8(Cp, ldx, lddx) && lddy % 8 == 0 && ldr % 8 == 0)) return 0;
  return (int)((M + 15) / 16 < LN_BWD_BLOCKS ? (M + 15) / 16 : LN_BWD_BLOCKS);
}

int sr_layernorm_bwd_reduce(const float* workspace, int nparts, int C, float* dgamma, float* dbeta, int accumulate,
                            void* stream) {
  if (!workspace || !dgamma || !dbeta || nparts <= 0 || C <= 0 || C > 512)
    return sr_fail(SR_EINVAL, "layernorm_bwd_reduce: bad arguments");
  hipLaunchKernelGGL(ln_bwd_reduce8, dim3((2 * C + 15) / 16), dim3(1024), 0, (hipStream_t)stream, workspace, nparts, C,
                     dgamma, dbeta, accumulate & 1);
  return sr_check(hipGetLastError(), "layernorm_bwd_reduce launch");
}

size_t sr_layernorm_bwd_workspace(int64_t M, int C) {
  (void)M;
  return (size_t)2048 * 4 * 2 * C * sizeof(float);
}

}  // extern "C"

namespace {
int ln_bwd_impl(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* mean, const float* rstd,
                const float* gamma, int64_t M, int C, int Cp, const void* res, int ldr, void* dx, int lddx,
                float* dgamma, float* dbeta, void* workspace, size_t ws_bytes, int accumulate, void* stream,
                const float* rscale, int HW, void* dx_scaled) {
  if (!dy || !x || !mean || !rstd || !gamma || !dx || !dgamma || !dbeta || C > 512)
    return sr_fail(SR_EINVAL, "layernorm_bwd: bad arguments");
  if (ws_bytes < sr_layernorm_bwd_workspace(M, C)) return sr_fail(SR_EINVAL, "layernorm_bwd: workspace too small");
  const unsigned grid = (unsigned)((M + 3) / 4 < 2048 ? (M + 3) / 4 : 2048);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16 && ln_vec8(Cp, ldx, lddx) && lddy % 8 == 0 && (!res || ldr % 8 == 0)) {
    // 16 row slots (512 threads) per block: twice the waves in flight of 8 slots for the same
    // number of dgamma / dbeta partials (more blocks instead moves the cost into the reduce)
    const unsigned g8 = (unsigned)((M + 15) / 16 < LN_BWD_BLOCKS ? (M + 15) / 16 : LN_BWD_BLOCKS);
    hipLaunchKernelGGL(ln_bwd8_kernel<16>, dim3(g8), dim3(512), 0, s, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, mean,
                       rstd, gamma, M, C, Cp, (const bf16_t*)res, ldr, (bf16_t*)dx, lddx, (float*)workspace, rscale, HW,
                       (bf16_t*)dx_scaled);
    if (!(accumulate & 2))  // bit 1: partials only (sr_layernorm_bwd_reduce later, e.g. on another stream)
      hipLaunchKernelGGL(ln_bwd_reduce8, dim3((2 * C + 15) / 16), dim3(1024), 0, s, (const float*)workspace, (int)g8, C,
                         dgamma, dbeta, accumulate & 1);
    return sr_check(hipGetLastError(), "layernorm_bwd launch");
  }
  if (dx_scaled) return sr_fail(SR_EINVAL, "layernorm_bwd_scaled: bf16, Cp <= 256, 16-B aligned rows only");
  accumulate &= 1;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx,
                       mean, rstd, gamma, M, C, Cp, (const bf16_t*)res, ldr, (bf16_t*)dx, lddx, (float*)workspace);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)dy, lddy, (const float*)x, ldx,
                       mean, rstd, gamma, M, C, Cp, (const float*)res, ldr, (float*)dx, lddx, (float*)workspace);
  hipLaunchKernelGGL(ln_bwd_reduce, dim3((2 * C + 255) / 256), dim3(256), 0, s, (const float*)workspace, (int)grid * 4,
                     C, dgamma, dbeta, accumulate);
  return sr_check(hipGetLastError(), "layernorm_bwd launch");
}
}  // namespace

extern "C" {

int sr_layernorm_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* mean, const float* rstd,
                     const float* gamma, int64_t M, int C, int Cp, const void* res, int ldr, void* dx, int lddx,
                     float* dgamma, float* dbeta, void* workspace, size_t ws_bytes, int accumulate, void* stream) {
  return ln_bwd_impl(dtype, dy, lddy, x, ldx, mean, rstd, gamma, M, C, Cp, res, ldr, dx, lddx, dgamma, dbeta, workspace,
                     ws_bytes, accumulate, stream, nullptr, 1, nullptr);
}

int sr_layernorm_bwd_scaled(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* mean,
                            const float* rstd, const float* gamma, int64_t M, int C, int Cp, const void* res, int ldr,
                            void* dx, int lddx, float* dgamma, float* dbeta, void* workspace, size_t ws_bytes,
                            int accumulate, const float* row_scale, int HW, void* dx_scaled, void* stream) {
  if (!row_scale || !dx_scaled || HW <= 0 || M % HW) return sr_fail(SR_EINVAL, "layernorm_bwd_scaled: bad row scale");
  return ln_bwd_impl(dtype, dy, lddy, x, ldx, mean, rstd, gamma, M, C, Cp, res, ldr, dx, lddx, dgamma, dbeta, workspace,
                     ws_bytes, accumulate, stream, row_scale, HW, dx_scaled);
}

int sr_window_attn_fwd(int dtype, const void* qkv, int ldq, int N, int H, int W, int ws, int shift, int nH, int hd,
                       int hdp, float scale, const float* bias_table, void* out, int ldo, float* lse, void* stream) {
  AttnArgs a{};
  if (!qkv || !bias_table || !out || !lse || !attn_setup(a, N, H, W, ws, shift, nH, hd, hdp, scale))
    return sr_fail(SR_EINVAL, "window_attn_fwd: bad arguments (ws <= 8, head_dim <= 32, H/W divisible by ws)");
  a.qkv = qkv; a.y = out; a.lse = lse; a.bias_table = bias_table; a.ldq = ldq; a.ldo = ldo;
  hipStream_t s = (hipStream_t)stream;
  if (attn_mfma_ok(a, dtype))
    hipLaunchKernelGGL(wattn_fwd_mfma_kernel, dim3(a.units), dim3(64), 0, s, a);
  else if (dtype == SR_BF16)
    hipLaunchKernelGGL(wattn_fwd_kernel<bf16_t>, dim3(a.units), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(wattn_fwd_kernel<float>, dim3(a.units), dim3(64), 0, s, a);
  return sr_check(hipGetLastError(), "window_attn_fwd launch");
}

size_t sr_window_attn_bwd_workspace(int N, int H, int W, int ws, int nH) {
  const int nb = (2 * ws - 1) * (2 * ws - 1);
  const size_t units = (size_t)N * (H / ws) * (W / ws) * nH;
  // slot rows at 1 window per wave + the quarter sums of wattn_dbias_slots
  const size_t rows = units * nb, slots = ws == 8 ? (units + (size_t)DB_Q * nH) * ATT_SLOTS : 0;
  return (rows > slots ? rows : slots) * sizeof(float);
}

int sr_window_attn_bwd(int dtype, const void* qkv, int ldq, const void* out, const void* dout, int ldo, const float* lse,
                       int N, int H, int W, int ws, int shift, int nH, int hd, int hdp, float scale,
                       const float* bias_table, void* dqkv, float* dbias_table, void* workspace, size_t ws_bytes,
                       int accumulate, void* stream) {
  AttnArgs a{};
  if (!qkv || !out || !dout || !lse || !bias_table || !dqkv || !dbias_table ||
      !attn_setup(a, N, H, W, ws, shift, nH, hd, hdp, scale))
    return sr_fail(SR_EINVAL, "window_attn_bwd: bad arguments");
  if (ws_bytes < sr_window_attn_bwd_workspace(N, H, W, ws, nH)) return sr_fail(SR_EINVAL, "window_attn_bwd: workspace");
  a.qkv = qkv; a.out = out; a.dout = dout; a.y = dqkv; a.lse = (float*)lse; a.bias_table = bias_table;
  a.dbias_part = (float*)workspace; a.ldq = ldq; a.ldo = ldo;
  hipStream_t s = (hipStream_t)stream;
  int parts = a.units;  // dbias partial rows, interleaved by head (row % nH == head)
  bool slot_rows = false;
  if (attn_mfma_ok(a, dtype)) {
    parts = nH * ((N * a.nwin + ATT_UPW - 1) / ATT_UPW);
    slot_rows = true;
    hipLaunchKernelGGL((wattn_bwd_mfma2_kernel<ATT_UPW>), dim3(parts), dim3(64), 0, s, a);
  } else if (dtype == SR_BF16) {
    hipLaunchKernelGGL(wattn_bwd_kernel<bf16_t>, dim3(a.units), dim3(64), 0, s, a);
  } else {
    hipLaunchKernelGGL(wattn_bwd_kernel<float>, dim3(a.units), dim3(64), 0, s, a);
  }
  if (!(accumulate & 2))  // bit 1: partials only (sr_window_attn_dbias_reduce later)
    dbias_reduce((const float*)workspace, slot_rows ? -parts : parts, nH, a.nbins, dbias_table, accumulate & 1, s);
  return sr_check(hipGetLastError(), "window_attn_bwd launch");
}

// relative-bias gradient partial rows sr_window_attn_bwd leaves in its workspace
int sr_window_attn_bwd_parts(int dtype, int N, int H, int W, int ws, int nH, int hd, int hdp, int ldq, int ldo) {
  AttnArgs a{};
  if (!attn_setup(a, N, H, W, ws, 0, nH, hd, hdp, 1.f)) return 0;
  a.ldq = ldq; a.ldo = ldo;
  if (!attn_mfma_ok(a, dtype)) return a.units;
  const int parts = nH * ((N * a.nwin + ATT_UPW - 1) / ATT_UPW);
  return -parts;  // negative: slot rows (see sr_hip.h)
}

int sr_window_attn_dbias_reduce(const float* workspace, int parts, int nH, int ws, float* dbias_table, int accumulate,
                                void* stream) {
  const int nbins = (2 * ws - 1) * (2 * ws - 1);
  if (!workspace || !dbias_table || parts == 0 || nH <= 0 || ws <= 0 || (parts < 0 && ws != 8))
    return sr_fail(SR_EINVAL, "window_attn_dbias_reduce: bad arguments");
  dbias_reduce(workspace, parts, nH, nbins, dbias_table, accumulate & 1, (hipStream_t)stream);
  return sr_check(hipGetLastError(), "window_attn_dbias_reduce launch");
}

int sr_add_pos_embed(int dtype, const void* x, int N, int P, int C, int Cp, const float* pos, void* y, void* stream) {
  if (!x || !pos || !y || N <= 0 || P <= 0 || C <= 0 || Cp < C) return sr_fail(SR_EINVAL, "add_pos_embed: bad arguments");
  const int64_t total = (int64_t)N * P * Cp;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(add_pos_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)x, pos, total, P, C,
                       Cp, (bf16_t*)y);
  else
    hipLaunchKernelGGL(add_pos_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)x, pos, total, P, C,
                       Cp, (float*)y);
  return sr_check(hipGetLastError(), "add_pos_embed launch");
}

int sr_pos_embed_grad(int dtype, const void* dy, int N, int P, int C, int Cp, float* dpos, int accumulate, void* stream) {
  if (!dy || !dpos || N <= 0 || P <= 0 || C <= 0 || Cp < C) return sr_fail(SR_EINVAL, "pos_embed_grad: bad arguments");
  const int64_t total = (int64_t)P * C;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(pos_grad_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)dy, N, P, C, Cp,
                       dpos, accumulate);
  else
    hipLaunchKernelGGL(pos_grad_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)dy, N, P, C, Cp,
                       dpos, accumulate);
  return sr_check(hipGetLastError(), "pos_embed_grad launch");
}

}  // extern "C"
