// Deformable convolution (DCNv1 / DCNv2) sampling kernels for gfx950.
//
// The reference (basicsr/ops/dcn/src/deform_conv_cuda.cpp:490-685, kernels
// deform_conv_cuda_kernel.cu:571-770) loops over the batch: per image it builds an fp32
// column matrix [C*K, Ho*Wo] with one thread per (c, pixel), runs a serial addmm, and in
// backward scatters with atomics and re-reads the columns once per offset channel.
//
// Here the deformable part is reduced to two batched HBM-bound passes around MFMA GEMMs
// (the GEMMs are the 1x1 path of conv3x3.hip):
//   sr_dcn_im2col : cols[p][g][tap][ci] = mask * bilinear(x, p + tap + offset), all images
//                   in one launch, pixel-major rows so the GEMM reads them as a K-contiguous
//                   operand; x is NHWC so each bilinear corner is a 16-byte channel vector.
//   sr_dcn_col2im : the reference's backward scatters as two passes over dcols:
//                   dcn_coord_grad_kernel (col2im_coord: offset and mask gradients, one
//                   item per (pixel, tap, deformable group) reducing over the group's
//                   channels in registers, no atomics) and dcn_grad_x_kernel (col2im:
//                   bilinear scatter accumulated in an LDS image of the output tile's input
//                   footprint, flushed with channel-contiguous atomics).
//   sr_dcn_fwd_fused : (bf16, C = 64, Cout <= 64) the sampling and the GEMM in one kernel,
//                   the column tile built in LDS per tap (dcn_fwd_mfma_kernel).
// Offsets and masks are staged through LDS per pixel tile so their NCHW reads and writes
// stay coalesced while the item loop runs deformable-group-fastest (adjacent lanes touch
// adjacent channel vectors of the same pixel).
#include "sr_common.h"
#include "sr_internal.h"

#include <cstdlib>

namespace {

struct DcnArgs {
  int N, C, H, W, Cp, Ho, Wo;
  int kh, kw, sh, sw, ph, pw, dh, dw;
  int G, DG, cg, cgp, cpg;  // conv groups, deformable groups, channels per conv group (+pad), per deform group
  int K, L, TP;             // taps, column row length (G*K*cgp), pixels per tile
};

template <typename T, int V> struct Vec;
template <> struct Vec<bf16_t, 8> {
  SR_DEV static void load(const bf16_t* p, float* f) {
    const u32x4 u = *(const u32x4*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(u[i] << 16);
      f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
  SR_DEV static void store(bf16_t* p, const float* f) {
    u32x4 u;
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
    *(u32x4*)p = u;
  }
};
template <> struct Vec<float, 4> {
  SR_DEV static void load(const float* p, float* f) {
    const f32x4 v = *(const f32x4*)p;
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = v[i];
  }
  SR_DEV static void store(float* p, const float* f) { *(f32x4*)p = f32x4{f[0], f[1], f[2], f[3]}; }
};
template <typename T> struct Vec<T, 1> {
  SR_DEV static void load(const T* p, float* f) { f[0] = Elt<T>::to_f(*p); }
  SR_DEV static void store(T* p, const float* f) { *p = Elt<T>::from_f(f[0]); }
};

// Bilinear sampling geometry of one (pixel, tap): the reference's validity rule
// (h > -1 && w > -1 && h < H && w < W, deform_conv_cuda_kernel.cu:619) and corner rules
// (dmcn_im2col_bilinear, :468-498).  Corner offsets are pixel indices within the image,
// -1 where the corner lies outside.
struct Sample {
  bool valid;
  float lh, lw, hh, hw;
  int o1, o2, o3, o4;
};

SR_DEV Sample make_sample(float h, float w, int H, int W) {
  Sample s;
  s.valid = (h > -1.f && w > -1.f && h < (float)H && w < (float)W);
  s.o1 = s.o2 = s.o3 = s.o4 = -1;
  s.lh = s.lw = s.hh = s.hw = 0.f;
  if (!s.valid) return s;
  const float fh = floorf(h), fw = floorf(w);
  const int hl = (int)fh, wl = (int)fw, hh_ = hl + 1, wh = wl + 1;
  s.lh = h - fh;
  s.lw = w - fw;
  s.hh = 1.f - s.lh;
  s.hw = 1.f - s.lw;
  if (hl >= 0 && wl >= 0) s.o1 = hl * W + wl;
  if (hl >= 0 && wh <= W - 1) s.o2 = hl * W + wh;
  if (hh_ <= H - 1 && wl >= 0) s.o3 = hh_ * W + wl;
  if (hh_ <= H - 1 && wh <= W - 1) s.o4 = hh_ * W + wh;
  return s;
}

// LDS tile of offsets ([DG*2K][TP]) followed by masks ([DG*K][TP]) for pixels
// [p0, p0+np) of image n; missing mask (DCNv1) reads as 1.
SR_DEV void load_tile(float* s_off, float* s_msk, const float* off, const float* msk, const DcnArgs& a, int n,
                      int p0, int np) {
  const int64_t HWo = (int64_t)a.Ho * a.Wo;
  const int noff = a.DG * 2 * a.K, nm = a.DG * a.K;
  for (int i = threadIdx.x; i < (noff + nm) * a.TP; i += blockDim.x) {
    const int ch = i / a.TP, px = i - ch * a.TP;
    float v = 0.f;
    if (px < np) {
      if (ch < noff) v = off[((int64_t)n * noff + ch) * HWo + p0 + px];
      else v = msk ? msk[((int64_t)n * nm + ch - noff) * HWo + p0 + px] : 1.f;
    }
    if (ch < noff) s_off[ch * a.TP + px] = v;
    else s_msk[(ch - noff) * a.TP + px] = v;
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(256) dcn_im2col_kernel(DcnArgs a, const T* __restrict__ x,
                                                         const float* __restrict__ off, const float* __restrict__ msk,
                                                         T* __restrict__ cols) {
  extern __shared__ float s_lds[];
  float* s_off = s_lds;
  float* s_msk = s_lds + a.DG * 2 * a.K * a.TP;
  const int HWo = a.Ho * a.Wo;
  const int tiles = (HWo + a.TP - 1) / a.TP;
  const int n = blockIdx.x / tiles, p0 = (blockIdx.x - n * tiles) * a.TP;
  const int np = min(a.TP, HWo - p0);
  load_tile(s_off, s_msk, off, msk, a, n, p0, np);
  __syncthreads();
  const T* xim = x + (int64_t)n * a.H * a.W * a.Cp;
  const int items = np * a.K * a.DG;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int dgi = it % a.DG, t2 = it / a.DG, tap = t2 % a.K, px = t2 / a.K;
    const int p = p0 + px, ho = p / a.Wo, wo = p - ho * a.Wo;
    const int i = tap / a.kw, j = tap - i * a.kw;
    const float oh = s_off[(dgi * 2 * a.K + 2 * tap) * a.TP + px];
    const float ow = s_off[(dgi * 2 * a.K + 2 * tap + 1) * a.TP + px];
    const float m = s_msk[(dgi * a.K + tap) * a.TP + px];
    const float h = (float)(ho * a.sh - a.ph + i * a.dh) + oh;
    const float w = (float)(wo * a.sw - a.pw + j * a.dw) + ow;
    const Sample s = make_sample(h, w, a.H, a.W);
    const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
    T* row = cols + ((int64_t)n * HWo + p) * a.L;
    for (int c = dgi * a.cpg; c < (dgi + 1) * a.cpg; c += V) {
      float v1[V], v2[V], v3[V], v4[V], r[V];
#pragma unroll
      for (int e = 0; e < V; ++e) v1[e] = v2[e] = v3[e] = v4[e] = 0.f;
      if (s.o1 >= 0) Vec<T, V>::load(xim + (int64_t)s.o1 * a.Cp + c, v1);
      if (s.o2 >= 0) Vec<T, V>::load(xim + (int64_t)s.o2 * a.Cp + c, v2);
      if (s.o3 >= 0) Vec<T, V>::load(xim + (int64_t)s.o3 * a.Cp + c, v3);
      if (s.o4 >= 0) Vec<T, V>::load(xim + (int64_t)s.o4 * a.Cp + c, v4);
#pragma unroll
      for (int e = 0; e < V; ++e) r[e] = (w1 * v1[e] + w2 * v2[e] + w3 * v3[e] + w4 * v4[e]) * m;
      const int g = c / a.cg, ci = c - g * a.cg;
      Vec<T, V>::store(row + (g * a.K + tap) * a.cgp + ci, r);
    }
  }
  if (a.cgp != a.cg) {  // zero the per-group channel padding of the column rows
    const int padc = a.cgp - a.cg, per = a.G * a.K * padc;
    for (int it = threadIdx.x; it < np * per; it += blockDim.x) {
      const int px = it / per, r = it - px * per, gt = r / padc, ci = a.cg + r - gt * padc;
      cols[((int64_t)n * HWo + p0 + px) * a.L + gt * a.cgp + ci] = Elt<T>::from_f(0.f);
    }
  }
}

// Offset / mask gradients (col2im_coord, deform_conv_cuda_kernel.cu:696-770): one item
// per (pixel, tap, deformable group) walks the group's channels once and reduces in
// registers; results replace the item's own LDS words and are stored coalesced.
template <typename T, int V>
__global__ void __launch_bounds__(256) dcn_coord_grad_kernel(DcnArgs a, const T* __restrict__ dcols,
                                                             const T* __restrict__ x, const float* __restrict__ off,
                                                             const float* __restrict__ msk, float* __restrict__ goff,
                                                             float* __restrict__ gmsk, unsigned* __restrict__ amax) {
  extern __shared__ float s_lds[];
  float* s_off = s_lds;
  float* s_msk = s_lds + a.DG * 2 * a.K * a.TP;
  const int HWo = a.Ho * a.Wo;
  const int tiles = (HWo + a.TP - 1) / a.TP;
  const int n = blockIdx.x / tiles, p0 = (blockIdx.x - n * tiles) * a.TP;
  const int np = min(a.TP, HWo - p0);
  load_tile(s_off, s_msk, off, msk, a, n, p0, np);
  __syncthreads();
  const T* xim = x + (int64_t)n * a.H * a.W * a.Cp;
  const int items = np * a.K * a.DG;
  float vmax = 0.f;  // max |mask * dcols| over the samples this block scatters (grad_x scale)
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int dgi = it % a.DG, t2 = it / a.DG, tap = t2 % a.K, px = t2 / a.K;
    const int p = p0 + px, ho = p / a.Wo, wo = p - ho * a.Wo;
    const int i = tap / a.kw, j = tap - i * a.kw;
    float* ph = &s_off[(dgi * 2 * a.K + 2 * tap) * a.TP + px];
    float* pw = &s_off[(dgi * 2 * a.K + 2 * tap + 1) * a.TP + px];
    float* pm = &s_msk[(dgi * a.K + tap) * a.TP + px];
    const float m = *pm;
    const float h = (float)(ho * a.sh - a.ph + i * a.dh) + *ph;
    const float w = (float)(wo * a.sw - a.pw + j * a.dw) + *pw;
    const Sample s = make_sample(h, w, a.H, a.W);
    float acc_h = 0.f, acc_w = 0.f, acc_m = 0.f;
    if (s.valid) {
      const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
      const T* row = dcols + ((int64_t)n * HWo + p) * a.L;
      for (int c = dgi * a.cpg; c < (dgi + 1) * a.cpg; c += V) {
        float v1[V], v2[V], v3[V], v4[V], dc[V];
#pragma unroll
        for (int e = 0; e < V; ++e) v1[e] = v2[e] = v3[e] = v4[e] = 0.f;
        const int g = c / a.cg, ci = c - g * a.cg;
        Vec<T, V>::load(row + (g * a.K + tap) * a.cgp + ci, dc);
        if (s.o1 >= 0) Vec<T, V>::load(xim + (int64_t)s.o1 * a.Cp + c, v1);
        if (s.o2 >= 0) Vec<T, V>::load(xim + (int64_t)s.o2 * a.Cp + c, v2);
        if (s.o3 >= 0) Vec<T, V>::load(xim + (int64_t)s.o3 * a.Cp + c, v3);
        if (s.o4 >= 0) Vec<T, V>::load(xim + (int64_t)s.o4 * a.Cp + c, v4);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          // d bilinear / d h and d w (dmcn_get_coordinate_weight, :527-569) and the
          // un-masked sample for the mask gradient
          const float wh = -s.hw * v1[e] - s.lw * v2[e] + s.hw * v3[e] + s.lw * v4[e];
          const float ww = -s.hh * v1[e] + s.hh * v2[e] - s.lh * v3[e] + s.lh * v4[e];
          acc_h += wh * dc[e] * m;
          acc_w += ww * dc[e] * m;
          acc_m += dc[e] * (w1 * v1[e] + w2 * v2[e] + w3 * v3[e] + w4 * v4[e]);
          vmax = fmaxf(vmax, fabsf(dc[e] * m));
          if (!(fabsf(dc[e] * m) <= 3.0e38f)) vmax = __builtin_inff();  // NaN / inf: grad_x falls back
        }
      }
    }
    // each item owns exactly the LDS words it read: overwrite them with its gradients
    *ph = acc_h;
    *pw = acc_w;
    *pm = acc_m;
  }
  // block max -> per-image max (non-negative floats order like their bit patterns)
  for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
  if ((threadIdx.x & 63) == 0 && vmax > 0.f) atomicMax(amax + n, __float_as_uint(vmax));
  __syncthreads();
  const int noff = a.DG * 2 * a.K, nm = a.DG * a.K;
  for (int q = threadIdx.x; q < (noff + nm) * a.TP; q += blockDim.x) {
    const int ch = q / a.TP, px = q - ch * a.TP;
    if (px >= np) continue;
    if (ch < noff) goff[((int64_t)n * noff + ch) * HWo + p0 + px] = s_off[ch * a.TP + px];
    else if (gmsk) gmsk[((int64_t)n * nm + ch - noff) * HWo + p0 + px] = s_msk[(ch - noff) * a.TP + px];
  }
}

// grad_x (col2im, :636-694): scatter mask * dcols to the four bilinear corners.  The
// workgroup owns a 2-D output tile; every corner that falls into the tile's input
// footprint (+ a halo of R pixels for the offsets) accumulates in an LDS image of CPP
// channels, and the footprint is flushed once per channel pass with channel-contiguous
// (coalesced) global fp32 atomics.  Corners outside the footprint (offsets larger than the
// halo) go straight to global atomics, so the result never depends on the offset range.
//
// LDS accumulation is int64 fixed point (ds_add_u64): fp32 LDS atomics run at ~1/25 of
// the integer rate on gfx950 (tools/lds_atomic_bench.hip, tools/atomic_bench2.hip).  The
// per-image scale 2^e puts max |mask * dcols| (from the coordinate kernel) below 2^48, so a
// cell sum of <= 2^14 contributions cannot overflow and the in-block sum is exact to
// 2^-48 of the largest term (finer than fp32 accumulation) and order independent.
// Non-finite gradients (max = inf) use direct fp32 atomics to propagate NaN / inf.
struct XGeom {
  int TT, R, RH, RW, CPP;  // output tile edge, halo, footprint rows / cols, channels per pass
};

template <typename T, int V>
__global__ void __launch_bounds__(256) dcn_grad_x_kernel(DcnArgs a, XGeom xg, const T* __restrict__ dcols,
                                                         const float* __restrict__ off, const float* __restrict__ msk,
                                                         const unsigned* __restrict__ amax, float* __restrict__ gx) {
  extern __shared__ unsigned long long s_acc[];  // [RH*RW][CPP+1]
  const int HWo = a.Ho * a.Wo;
  const int tw = (a.Wo + xg.TT - 1) / xg.TT, th = (a.Ho + xg.TT - 1) / xg.TT;
  const int n = blockIdx.x / (tw * th), t = blockIdx.x - n * (tw * th);
  const float mx = __uint_as_float(amax[n]);
  if (mx == 0.f) return;  // nothing of this image is scattered (uniform per block)
  const bool direct = !(mx <= 3.0e38f);
  int ex = 0;
  frexpf(direct ? 1.f : mx, &ex);
  const int e = min(127, 48 - ex);
  const float sc = ldexpf(1.f, e), isc = ldexpf(1.f, -e);
  const int ho0 = (t / tw) * xg.TT, wo0 = (t - (t / tw) * tw) * xg.TT;
  const int ry0 = ho0 * a.sh - a.ph - xg.R, rx0 = wo0 * a.sw - a.pw - xg.R;
  const int RP = xg.RH * xg.RW, ST = xg.CPP + 1;
  const int npx = xg.TT * xg.TT, nvec = xg.CPP / V;
  float* gim = gx + (int64_t)n * a.H * a.W * a.Cp;
  for (int c0 = 0; c0 < a.C; c0 += xg.CPP) {
    for (int i = threadIdx.x; i < RP * ST; i += blockDim.x) s_acc[i] = 0ull;
    __syncthreads();
    const int items = npx * nvec * a.K;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
      const int px = it % npx, r = it / npx, cv = r % nvec, tap = r / nvec;
      const int ho = ho0 + px / xg.TT, wo = wo0 + px % xg.TT;
      const int c = c0 + cv * V;
      if (ho >= a.Ho || wo >= a.Wo || c >= a.C) continue;
      const int p = ho * a.Wo + wo;
      const int dgi = c / a.cpg, g = c / a.cg, ci = c - g * a.cg;
      const int i = tap / a.kw, j = tap - i * a.kw;
      const float oh = off[(((int64_t)n * a.DG + dgi) * 2 * a.K + 2 * tap) * HWo + p];
      const float ow = off[(((int64_t)n * a.DG + dgi) * 2 * a.K + 2 * tap + 1) * HWo + p];
      const float m = msk ? msk[(((int64_t)n * a.DG + dgi) * a.K + tap) * HWo + p] : 1.f;
      const float h = (float)(ho * a.sh - a.ph + i * a.dh) + oh;
      const float w = (float)(wo * a.sw - a.pw + j * a.dw) + ow;
      const Sample s = make_sample(h, w, a.H, a.W);
      if (!s.valid) continue;
      float dc[V];
      Vec<T, V>::load(dcols + ((int64_t)n * HWo + p) * a.L + (g * a.K + tap) * a.cgp + ci, dc);
      const int hl = (int)floorf(h), wl = (int)floorf(w);
      const float wt[4] = {s.hh * s.hw, s.hh * s.lw, s.lh * s.hw, s.lh * s.lw};
      const int oo[4] = {s.o1, s.o2, s.o3, s.o4};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (oo[q] < 0) continue;
        const int ly = hl + (q >> 1) - ry0, lx = wl + (q & 1) - rx0;
        if (!direct && ly >= 0 && ly < xg.RH && lx >= 0 && lx < xg.RW) {
          unsigned long long* dst = s_acc + (ly * xg.RW + lx) * ST + cv * V;
#pragma unroll
          for (int e2 = 0; e2 < V; ++e2)
            atomicAdd(dst + e2, (unsigned long long)__float2ll_rn(wt[q] * (dc[e2] * m) * sc));
        } else {
          float* dst = gim + (int64_t)oo[q] * a.Cp + c;
#pragma unroll
          for (int e2 = 0; e2 < V; ++e2) unsafeAtomicAdd(dst + e2, wt[q] * (dc[e2] * m));
        }
      }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < RP * xg.CPP; i += blockDim.x) {
      const int pix = i / xg.CPP, ch = i - pix * xg.CPP;
      const int yy = ry0 + pix / xg.RW, xx = rx0 + pix % xg.RW;
      if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W || c0 + ch >= a.C) continue;
      const long long v = (long long)s_acc[pix * ST + ch];
      if (v != 0) unsafeAtomicAdd(gim + ((int64_t)yy * a.W + xx) * a.Cp + c0 + ch, (float)v * isc);
    }
    __syncthreads();
  }
}

// Fused deformable forward (bf16, one conv group, C = cgp = Cp = 64, Cout <= 64): the column
// matrix never reaches HBM.  A block owns DF_TP consecutive output pixels of one image and
// every output channel; per tap it gathers the DF_TP x 64 modulated samples (the im2col item
// math above, same expression, so the rows equal sr_dcn_im2col's) straight into an LDS tile
// and multiplies it by the tap's 64 x 64 weight slice on v_mfma_f32_16x16x32_bf16 (B fragments
// from L2 into registers, issued before the gather so they land under it).  Thread t keeps one
// pixel (t % DF_TP) for all taps and 4 of its 8 channel vectors, so the offset / mask reads of a
// wave are 64 consecutive floats of one NCHW plane.  This global-gather form runs for
// x_blocked = 1: x as channel-vector planes [N][8][H][W][8] (pixel stride 16 B, vector stride
// H*W*16 B), so the corners a wave gathers for one vector of 64 neighbouring pixels share cache
// lines (on NHWC every lane hit its own 128-B line: 504 us on the C5 shape, 373 us blocked).  NHWC
// x (what the op passes) takes dcn_fwd_win_kernel below, which gathers from an LDS window (160 us).  LDS rows are padded to 144 B: the 16 rows
// one A-fragment read touches start on 16 distinct 4-bank groups.  Epilogue: bias, bf16
// rounding (the unfused path stores its GEMM output as bf16), fp32 NCHW store of 4 consecutive
// pixels per lane.  cols (optional) receives the column rows for the backward's weight
// gradient.  Replaces im2col + 1x1 GEMM + NHWC->NCHW of the unfused path; the reference's
// per-image modulated_deformable_im2col_cuda + addmm (deform_conv_cuda.cpp:560-590).
constexpr int DF_TP = 128, DF_RS = 72;  // pixels per block; LDS row stride in bf16 (144 B)

SR_DEV void mfma_bf16(const u32x4& a, const u32x4& b, f32x4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a), __builtin_bit_cast(s16x8, b), acc, 0,
                                                0, 0);
}

__global__ void __launch_bounds__(256) dcn_fwd_mfma_kernel(DcnArgs a, const bf16_t* __restrict__ x,
                                                           const float* __restrict__ off,
                                                           const float* __restrict__ msk,
                                                           const bf16_t* __restrict__ wf, int ldw, int wrows,
                                                           int cout, const float* __restrict__ bias,
                                                           float* __restrict__ y, bf16_t* __restrict__ cols,
                                                           uint32_t pxb, uint32_t vb) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[DF_TP * DF_RS];
  const int HWo = a.Ho * a.Wo;
  const int tiles = (HWo + DF_TP - 1) / DF_TP;
  const int n = blockIdx.x / tiles, p0 = (blockIdx.x - n * tiles) * DF_TP;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int px = tid & (DF_TP - 1), v0 = tid >> 7;  // pixel; first channel vector (then +2, +4, +6)
  const int p = p0 + px;
  const bool pv = p < HWo;
  const int ho = pv ? p / a.Wo : 0, wo = pv ? p - ho * a.Wo : 0;
  const float hb = (float)(ho * a.sh - a.ph), wb = (float)(wo * a.sw - a.pw);
  const int64_t HWo64 = HWo;
  const auto xr = make_rsrc(x + (int64_t)n * a.H * a.W * a.Cp, (uint32_t)((size_t)a.H * a.W * a.Cp * 2));
  const auto wr = make_rsrc(wf, (uint32_t)((size_t)wrows * ldw * 2));
  const float* offn = off + (int64_t)n * a.DG * 2 * a.K * HWo64 + p;
  const float* mskn = msk ? msk + (int64_t)n * a.DG * a.K * HWo64 + p : nullptr;
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < a.K; ++k) {
    // this tap's B fragments: B[k = ci][col = co] = wf[co][k*64 + ci]
    u32x4 bq[4][2];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bq[cb][kk] = buf_load16(wr, (uint32_t)(((16 * cb + (lane & 15)) * ldw + k * 64 + 32 * kk + 8 * (lane >> 4)) * 2));
    const int ti = k / a.kw, tj = k - ti * a.kw;
    const float hk = hb + (float)(ti * a.dh), wk = wb + (float)(tj * a.dw);
    float wt[4][4], mm[4];
    uint32_t co[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int v = v0 + 2 * j, dgi = v * 8 / a.cpg;
      float oh = 0.f, ow = 0.f, m = 0.f;
      if (pv) {
        oh = offn[(int64_t)(dgi * 2 * a.K + 2 * k) * HWo64];
        ow = offn[(int64_t)(dgi * 2 * a.K + 2 * k + 1) * HWo64];
        m = mskn ? mskn[(int64_t)(dgi * a.K + k) * HWo64] : 1.f;
      }
      const Sample s = make_sample(hk + oh, wk + ow, a.H, a.W);
      const bool ok = pv && s.valid;
      wt[j][0] = s.hh * s.hw; wt[j][1] = s.hh * s.lw; wt[j][2] = s.lh * s.hw; wt[j][3] = s.lh * s.lw;
      mm[j] = m;
      const uint32_t cb16 = (uint32_t)v * vb;
      co[j][0] = ok && s.o1 >= 0 ? (uint32_t)s.o1 * pxb + cb16 : SR_OOB;
      co[j][1] = ok && s.o2 >= 0 ? (uint32_t)s.o2 * pxb + cb16 : SR_OOB;
      co[j][2] = ok && s.o3 >= 0 ? (uint32_t)s.o3 * pxb + cb16 : SR_OOB;
      co[j][3] = ok && s.o4 >= 0 ? (uint32_t)s.o4 * pxb + cb16 : SR_OOB;
    }
    u32x4 cv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) cv[j][q] = buf_load16(xr, co[j][q]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v1[8], v2[8], v3[8], v4[8], r[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v1[2 * e] = __uint_as_float(cv[j][0][e] << 16); v1[2 * e + 1] = __uint_as_float(cv[j][0][e] & 0xffff0000u);
        v2[2 * e] = __uint_as_float(cv[j][1][e] << 16); v2[2 * e + 1] = __uint_as_float(cv[j][1][e] & 0xffff0000u);
        v3[2 * e] = __uint_as_float(cv[j][2][e] << 16); v3[2 * e + 1] = __uint_as_float(cv[j][2][e] & 0xffff0000u);
        v4[2 * e] = __uint_as_float(cv[j][3][e] << 16); v4[2 * e + 1] = __uint_as_float(cv[j][3][e] & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e)
        r[e] = (wt[j][0] * v1[e] + wt[j][1] * v2[e] + wt[j][2] * v3[e] + wt[j][3] * v4[e]) * mm[j];
      u32x4 u;
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = pack_bf16x2(r[2 * e], r[2 * e + 1]);
      const int v = v0 + 2 * j;
      *(u32x4*)&sA[px * DF_RS + v * 8] = u;
      if (cols && pv) *(u32x4*)(cols + ((int64_t)n * HWo64 + p) * a.L + k * 64 + v * 8) = u;
    }
    __syncthreads();
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const u32x4 af = *(const u32x4*)&sA[(32 * wv + 16 * rb + (lane & 15)) * DF_RS + 32 * kk + 8 * (lane >> 4)];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) mfma_bf16(af, bq[cb][kk], acc[rb][cb]);
      }
    __syncthreads();
  }
  const bool vec4 = (HWo & 3) == 0;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int c = 16 * cb + (lane & 15);
    if (c >= cout) continue;
    const float b = bias ? bias[c] : 0.f;
    float* yc = y + ((int64_t)n * cout + c) * HWo64;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int pr = p0 + 32 * wv + 16 * rb + 4 * (lane >> 4);
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = bf16_to_f32(f32_to_bf16(acc[rb][cb][i] + b));
      if (vec4 && pr + 3 < HWo) {
        *(f32x4*)(yc + pr) = f32x4{o[0], o[1], o[2], o[3]};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (pr + i < HWo) yc[pr + i] = o[i];
      }
    }
  }
}

int make_args(const sr_dcn_desc* d, DcnArgs& a) {
  if (!d) return sr_fail(SR_EINVAL, "dcn: null descriptor");
  a.N = d->N; a.C = d->C; a.H = d->H; a.W = d->W; a.Cp = d->Cp; a.Ho = d->Ho; a.Wo = d->Wo;
  a.kh = d->kh; a.kw = d->kw; a.sh = d->stride_h; a.sw = d->stride_w; a.ph = d->pad_h; a.pw = d->pad_w;
  a.dh = d->dil_h; a.dw = d->dil_w; a.G = d->groups; a.DG = d->deformable_groups; a.cgp = d->cgp;
  if (a.N <= 0 || a.C <= 0 || a.H <= 0 || a.W <= 0 || a.Ho <= 0 || a.Wo <= 0 || a.kh <= 0 || a.kw <= 0 ||
      a.sh <= 0 || a.sw <= 0 || a.dh <= 0 || a.dw <= 0 || a.ph < 0 || a.pw < 0)
    return sr_fail(SR_EINVAL, "dcn: non-positive size");
  if (a.G <= 0 || a.DG <= 0 || a.C % a.G || a.C % a.DG)
    return sr_fail(SR_EINVAL, "dcn: channels must be divisible by groups and deformable_groups");
  if (a.Cp < a.C || a.Cp % 8) return sr_fail(SR_EINVAL, "dcn: Cp must be >= C and a multiple of 8");
  a.cg = a.C / a.G;
  a.cpg = a.C / a.DG;
  if (a.cgp < a.cg || a.cgp % 8) return sr_fail(SR_EINVAL, "dcn: cgp must be >= C/groups and a multiple of 8");
  if (a.Ho != (a.H + 2 * a.ph - (a.dh * (a.kh - 1) + 1)) / a.sh + 1 ||
      a.Wo != (a.W + 2 * a.pw - (a.dw * (a.kw - 1) + 1)) / a.sw + 1)
    return sr_fail(SR_EINVAL, "dcn: output size does not match the convolution geometry");
  a.K = a.kh * a.kw;
  a.L = a.G * a.K * a.cgp;
  // pixel tile: offsets + masks of every deformable group in LDS (<= 64 KB)
  a.TP = 64;
  while (a.TP > 16 && (size_t)a.DG * 3 * a.K * a.TP * 4 > 32768) a.TP >>= 1;
  while (a.TP > 1 && (size_t)a.DG * 3 * a.K * a.TP * 4 > 65536) a.TP >>= 1;
  if ((size_t)a.DG * 3 * a.K * a.TP * 4 > 65536) return sr_fail(SR_EINVAL, "dcn: too many deformable groups x taps");
  return SR_OK;
}

// vector width: 16-byte channel vectors when every group boundary is vector aligned
template <typename T> int vec_width(const DcnArgs& a) {
  const int v = Elt<T>::PER16;
  return (a.cpg % v == 0 && a.cg % v == 0) ? v : 1;
}

template <typename T>
int launch_im2col(const DcnArgs& a, const void* x, const float* off, const float* msk, void* cols, hipStream_t s) {
  const int tiles = (a.Ho * a.Wo + a.TP - 1) / a.TP;
  const dim3 grid((unsigned)(a.N * tiles));
  const size_t lds = (size_t)a.DG * 3 * a.K * a.TP * 4;
  if (vec_width<T>(a) > 1)
    hipLaunchKernelGGL((dcn_im2col_kernel<T, Elt<T>::PER16>), grid, dim3(256), lds, s, a, (const T*)x, off, msk,
                       (T*)cols);
  else
    hipLaunchKernelGGL((dcn_im2col_kernel<T, 1>), grid, dim3(256), lds, s, a, (const T*)x, off, msk, (T*)cols);
  return sr_check(hipGetLastError(), "dcn_im2col launch");
}

XGeom grad_x_geom(const DcnArgs& a) {
  // largest (tile, halo) whose LDS footprint fits 64 KB; halo 0 still covers the
  // undeformed footprint, anything outside goes to global atomics
  static const int cfg[][2] = {{16, 4}, {16, 2}, {8, 4}, {8, 2}, {8, 0}, {4, 0}};
  // channels per pass: 8, or knob SR_DCN_CPP = 16 / 32 (A/B: fewer passes over dcols, a larger LDS image)
  const int cpp = sr_knob(K_DCN_CPP) == 16 || sr_knob(K_DCN_CPP) == 32 ? sr_knob(K_DCN_CPP) : 8;
  XGeom g;
  g.CPP = cpp;
  const size_t lim = cpp == 8 ? 65536 : 160 * 1024;
  for (const auto& c : cfg) {
    g.TT = c[0];
    g.R = c[1];
    g.RH = (g.TT - 1) * a.sh + (a.kh - 1) * a.dh + 2 * g.R + 2;
    g.RW = (g.TT - 1) * a.sw + (a.kw - 1) * a.dw + 2 * g.R + 2;
    if ((size_t)g.RH * g.RW * (g.CPP + 1) * 8 <= lim) return g;
  }
  g.CPP = 8;
  g.TT = 4; g.R = 0; g.RH = g.RW = 1;  // degenerate footprint: everything through global atomics
  return g;
}

template <typename T>
int launch_col2im(const DcnArgs& a, const void* dcols, const void* x, const float* off, const float* msk, float* gx,
                  float* goff, float* gmsk, unsigned* amax, hipStream_t s, bool coord = true) {
  const int tiles = (a.Ho * a.Wo + a.TP - 1) / a.TP;
  const size_t lds = (size_t)a.DG * 3 * a.K * a.TP * 4;
  const bool vec = vec_width<T>(a) > 1;
  if (!coord) {  // the coordinate pass (and amax) ran already (dcn_coord_win_kernel)
  } else if (vec)
    hipLaunchKernelGGL((dcn_coord_grad_kernel<T, Elt<T>::PER16>), dim3((unsigned)(a.N * tiles)), dim3(256), lds, s, a,
                       (const T*)dcols, (const T*)x, off, msk, goff, gmsk, amax);
  else
    hipLaunchKernelGGL((dcn_coord_grad_kernel<T, 1>), dim3((unsigned)(a.N * tiles)), dim3(256), lds, s, a,
                       (const T*)dcols, (const T*)x, off, msk, goff, gmsk, amax);
  if (coord && hipGetLastError() != hipSuccess) return sr_fail(SR_ELAUNCH, "dcn_coord_grad launch");
  const XGeom xg = grad_x_geom(a);
  const int xt = ((a.Ho + xg.TT - 1) / xg.TT) * ((a.Wo + xg.TT - 1) / xg.TT);
  const size_t xlds = (size_t)xg.RH * xg.RW * (xg.CPP + 1) * 8;
  if (xlds > 65536) {
    const hipError_t e1 = vec ? hipFuncSetAttribute((const void*)dcn_grad_x_kernel<T, Elt<T>::PER16>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)xlds)
                              : hipFuncSetAttribute((const void*)dcn_grad_x_kernel<T, 1>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)xlds);
    if (e1 != hipSuccess) return sr_fail(SR_ELAUNCH, "dcn_col2im: LDS attribute");
  }
  if (vec)
    hipLaunchKernelGGL((dcn_grad_x_kernel<T, Elt<T>::PER16>), dim3((unsigned)(a.N * xt)), dim3(256), xlds, s, a, xg,
                       (const T*)dcols, off, msk, amax, gx);
  else
    hipLaunchKernelGGL((dcn_grad_x_kernel<T, 1>), dim3((unsigned)(a.N * xt)), dim3(256), xlds, s, a, xg,
                       (const T*)dcols, off, msk, amax, gx);
  return sr_check(hipGetLastError(), "dcn_col2im launch");
}

// Windowed form of the fused forward (x NHWC): the block's output tile is 8 x 16 pixels, and
// the x window it can sample (its receptive field grown by R pixels on each side for the
// offsets; 15 x 23 pixels x 64 channels = 44 KB at 3x3, stride 1, R 2) is staged in LDS once,
// coalesced.  The per-tap gathers then read LDS; a sample whose 2 x 2 corners leave the window
// (|offset| > R) reads them from global memory, so the result never depends on the offset
// range.  The window holds pixel pix's channel vector v in slot v ^ (pix & 7): the vectors of 16
// different pixels land on 16 distinct 4-bank groups.  Offsets and masks of tap k + 1 are loaded
// while tap k gathers.  Tiles of one image are remapped onto one XCD (shared L2 for the window
// rows of neighbouring tiles).  Sample math, A tile, MFMA and epilogue as dcn_fwd_mfma_kernel.
constexpr int DW_TH = 8, DW_TW = 16, DW_NT = 512;

__global__ void __launch_bounds__(DW_NT, 4) dcn_fwd_win_kernel(DcnArgs a, const bf16_t* __restrict__ x,
                                                               const float* __restrict__ off,
                                                               const float* __restrict__ msk,
                                                               const bf16_t* __restrict__ wf, int ldw, int wrows,
                                                               int cout, const float* __restrict__ bias,
                                                               float* __restrict__ y, bf16_t* __restrict__ cols,
                                                               int R, int WH, int WW, int dbg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  bf16_t* sA = (bf16_t*)s_raw;                           // [DF_TP][DF_RS]
  bf16_t* sB = sA + DF_TP * DF_RS;                       // [64 co][DF_RS]: this tap's weight slice
  unsigned char* sX = (unsigned char*)(sB + 64 * DF_RS);  // [WH * WW][8 slots][16 B]
  const int HWo = a.Ho * a.Wo;
  const int64_t HWo64 = HWo;
  const int tw = (a.Wo + DW_TW - 1) / DW_TW, th = (a.Ho + DW_TH - 1) / DW_TH;
  const int bid = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / (tw * th), t = bid - n * (tw * th);
  const int ho0 = (t / tw) * DW_TH, wo0 = (t - (t / tw) * tw) * DW_TW;
  const int y0 = ho0 * a.sh - a.ph - R, x0 = wo0 * a.sw - a.pw - R;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;  // 8 waves
  const int px = tid & (DF_TP - 1), v0 = tid >> 7;              // pixel; channel vectors v0 and v0 + 4
  const int ho = ho0 + (px >> 4), wo = wo0 + (px & 15);
  const bool pv = ho < a.Ho && wo < a.Wo;
  const int p = pv ? ho * a.Wo + wo : 0;
  const float hb = (float)(ho * a.sh - a.ph), wb = (float)(wo * a.sw - a.pw);
  const uint32_t pxb = (uint32_t)a.Cp * 2u;
  const auto xr = make_rsrc(x + (int64_t)n * a.H * a.W * a.Cp, (uint32_t)((size_t)a.H * a.W * a.Cp * 2));
  const auto wr = make_rsrc(wf, (uint32_t)((size_t)wrows * ldw * 2));
  // stage the window: 4 loads in flight per thread, then their stores
  const int nwin = (dbg & 8) ? 0 : WH * WW * 8;
  for (int b0 = 0; b0 < nwin; b0 += 4 * DW_NT) {
    u32x4 val[4];
    int dst[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = b0 + u * DW_NT + tid;
      const int pix = i >> 3, v = i & 7;
      const int wy = pix / WW, wx = pix - wy * WW;
      const int yy = y0 + wy, xx = x0 + wx;
      const bool in = i < nwin && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      val[u] = buf_load16(xr, in ? (uint32_t)(yy * a.W + xx) * pxb + (uint32_t)v * 16u : SR_OOB);
      dst[u] = i < nwin ? pix * 128 + ((v ^ (pix & 7)) << 4) : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (dst[u] >= 0) *(u32x4*)(sX + dst[u]) = val[u];
  }
  const float* offn = off + (int64_t)n * a.DG * 2 * a.K * HWo64 + p;
  const float* mskn = msk ? msk + (int64_t)n * a.DG * a.K * HWo64 + p : nullptr;
  const int dg0 = v0 * 8 / a.cpg, dg1 = (v0 + 4) * 8 / a.cpg;
  float om[2][3];
  auto load_om = [&](int k, float (&o)[2][3]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int dgi = j ? dg1 : dg0;
      if (dbg & 2) {
        o[j][0] = 0.3f; o[j][1] = -0.2f; o[j][2] = 0.5f;
        continue;
      }
      o[j][0] = pv ? offn[(int64_t)(dgi * 2 * a.K + 2 * k) * HWo64] : 0.f;
      o[j][1] = pv ? offn[(int64_t)(dgi * 2 * a.K + 2 * k + 1) * HWo64] : 0.f;
      o[j][2] = pv ? (mskn ? mskn[(int64_t)(dgi * a.K + k) * HWo64] : 1.f) : 0.f;
    }
  };
  load_om(0, om);
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // window staged
  for (int k = 0; k < a.K; ++k) {
    // this tap's 64 x 64 weight slice, one 16-B piece per thread, written to LDS after the gather
    // (every wave reading its B fragments from L2 moved 8x the bytes: 1.2 GB per C5 call)
    const u32x4 wpiece = buf_load16(wr, (uint32_t)(((tid >> 3) * ldw + k * 64 + (tid & 7) * 8) * 2));
    float omn[2][3];
    if (k + 1 < a.K) load_om(k + 1, omn);
    const int ti = k / a.kw, tj = k - ti * a.kw;
    const float hk = hb + (float)(ti * a.dh), wk = wb + (float)(tj * a.dw);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int v = v0 + 4 * j;
      const float h = hk + om[j][0], w = wk + om[j][1];
      const Sample s = make_sample(h, w, a.H, a.W);
      const bool ok = pv && s.valid;
      const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
      const int hl = ok ? (int)floorf(h) : 0, wl = ok ? (int)floorf(w) : 0;
      const int ly = hl - y0, lx = wl - x0;
      u32x4 cv[4];
      if ((dbg & 1) || (ok && ly >= 0 && ly + 1 < WH && lx >= 0 && lx + 1 < WW)) {
        const int q0 = (dbg & 1) ? ((ly & 7) * WW + (lx & 15)) : ly * WW + lx;
        const int qs[4] = {q0, q0 + 1, q0 + WW, q0 + WW + 1};
#pragma unroll
        for (int q = 0; q < 4; ++q) cv[q] = *(const u32x4*)(sX + qs[q] * 128 + ((v ^ (qs[q] & 7)) << 4));
      } else {
        const uint32_t cb16 = (uint32_t)v * 16u;
        cv[0] = buf_load16(xr, ok && s.o1 >= 0 ? (uint32_t)s.o1 * pxb + cb16 : SR_OOB);
        cv[1] = buf_load16(xr, ok && s.o2 >= 0 ? (uint32_t)s.o2 * pxb + cb16 : SR_OOB);
        cv[2] = buf_load16(xr, ok && s.o3 >= 0 ? (uint32_t)s.o3 * pxb + cb16 : SR_OOB);
        cv[3] = buf_load16(xr, ok && s.o4 >= 0 ? (uint32_t)s.o4 * pxb + cb16 : SR_OOB);
      }
      u32x4 u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float r2[2];
#pragma unroll
        for (int hi = 0; hi < 2; ++hi) {
          const auto f = [&](uint32_t w32) { return __uint_as_float(hi ? (w32 & 0xffff0000u) : (w32 << 16)); };
          r2[hi] = (w1 * f(cv[0][e]) + w2 * f(cv[1][e]) + w3 * f(cv[2][e]) + w4 * f(cv[3][e])) * om[j][2];
        }
        u[e] = pack_bf16x2(r2[0], r2[1]);
      }
      *(u32x4*)&sA[px * DF_RS + v * 8] = u;
      if (cols && pv) *(u32x4*)(cols + ((int64_t)n * HWo64 + p) * a.L + k * 64 + v * 8) = u;
    }
    *(u32x4*)&sB[(tid >> 3) * DF_RS + (tid & 7) * 8] = wpiece;
    __syncthreads();
    if (!(dbg & 4)) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const u32x4 af = *(const u32x4*)&sA[(16 * wv + (lane & 15)) * DF_RS + 32 * kk + 8 * (lane >> 4)];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          // B[k = ci][col = co] = wf[co][k*64 + ci]
          const u32x4 bf = *(const u32x4*)&sB[(16 * cb + (lane & 15)) * DF_RS + 32 * kk + 8 * (lane >> 4)];
          mfma_bf16(af, bf, acc[cb]);
        }
      }
    }
    __syncthreads();
    if (k + 1 < a.K) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 3; ++e) om[j][e] = omn[j][e];
    }
  }
  const bool vec4 = (a.Wo & 3) == 0;
  const int oh = ho0 + wv, ow = wo0 + 4 * (lane >> 4);
  if (oh >= a.Ho) return;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int c = 16 * cb + (lane & 15);
    if (c >= cout) continue;
    const float b = bias ? bias[c] : 0.f;
    float* yc = y + ((int64_t)n * cout + c) * HWo64 + oh * a.Wo;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = bf16_to_f32(f32_to_bf16(acc[cb][i] + b));
    if (vec4 && ow + 3 < a.Wo) {
      *(f32x4*)(yc + ow) = f32x4{o[0], o[1], o[2], o[3]};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ow + i < a.Wo) yc[ow + i] = o[i];
    }
  }
}

// Ablation mask of dcn_fwd_win_kernel (SR_DCN_DBG, read per call; tools/dcn_ablate.py): 1 no global
// fallback, 2 constant offsets (no offset / mask reads), 4 no MFMA, 8 no window staging.  Results are
// wrong under any of them; 0 (unset) is the kernel.
int dcn_dbg() { return sr_knob(K_DCN_DBG) > 0 ? sr_knob(K_DCN_DBG) : 0; }

// Window geometry of dcn_fwd_win_kernel: the largest R <= 2 whose LDS (A tile + window) fits 64 KB.
bool win_geom(const DcnArgs& a, int* R, int* WH, int* WW, size_t* lds) {
  const int rk = sr_knob(K_DCN_R);
  const int r0 = rk >= 0 && rk <= 6 ? rk : 2;
  for (int r = r0; r >= 0; --r) {
    const int wh = (DW_TH - 1) * a.sh + (a.kh - 1) * a.dh + 2 + 2 * r;
    const int ww = (DW_TW - 1) * a.sw + (a.kw - 1) * a.dw + 2 + 2 * r;
    const size_t l = (size_t)(DF_TP + 64) * DF_RS * 2 + (size_t)wh * ww * 128;
    if (l <= 160 * 1024) {
      *R = r; *WH = wh; *WW = ww; *lds = l;
      return true;
    }
  }
  return false;
}

// Shapes the fused forward takes (see dcn_fwd_mfma_kernel); SR_DCN_FUSED=0 turns it off (A/B).
bool dcn_fused_ok(const sr_dcn_desc* d, const DcnArgs& a, int cout) {
  const bool off = sr_knob(K_DCN_FUSED) == 0;
  return !off && d->dtype == SR_BF16 && a.G == 1 && a.C == 64 && a.Cp == 64 && a.cgp == 64 && cout >= 1 &&
         cout <= 64 && a.cpg % 8 == 0 && (size_t)a.H * a.W * a.Cp * 2 < 0x80000000ull;
}

// Offset / mask gradients with the forward's LDS x window (bf16, one conv group, C = 64): the
// block owns an 8 x 16 output tile and stages its x window once (as dcn_fwd_win_kernel); per tap
// it stages the tap's offsets and masks for the tile in LDS (coalesced 16-pixel row segments),
// then item (pixel, channel vector v) reads its 16-B dcols piece (8 consecutive lanes = one
// pixel's 128-B row), its four corners from the window (global memory past it), and sums
// d bilinear / d h, / d w and the un-masked sample against dcols over its 8 channels; lanes of one
// deformable group combine by xor-shuffles and the group's first lane writes the three results
// over the LDS words it read, which are then stored coalesced.  Per-image max |mask * dcols| for
// the scatter's fixed-point scale as dcn_coord_grad_kernel.  Same math as that kernel (the
// reference's col2im_coord, deform_conv_cuda_kernel.cu:696-770); the channel sums run 8 per lane
// then across lanes.
__global__ void __launch_bounds__(DW_NT, 2) dcn_coord_win_kernel(DcnArgs a, const bf16_t* __restrict__ dcols,
                                                                 const bf16_t* __restrict__ x,
                                                                 const float* __restrict__ off,
                                                                 const float* __restrict__ msk,
                                                                 float* __restrict__ goff, float* __restrict__ gmsk,
                                                                 unsigned* __restrict__ amax, int R, int WH, int WW) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  float* sO = (float*)s_raw;                                  // [3 * DG][DF_TP]: dh, dw per group, then masks
  unsigned char* sX = s_raw + (size_t)3 * a.DG * DF_TP * 4;  // [WH * WW][8 slots][16 B]
  const int HWo = a.Ho * a.Wo;
  const int64_t HWo64 = HWo;
  const int tw = (a.Wo + DW_TW - 1) / DW_TW, th = (a.Ho + DW_TH - 1) / DW_TH;
  const int bid = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / (tw * th), t = bid - n * (tw * th);
  const int ho0 = (t / tw) * DW_TH, wo0 = (t - (t / tw) * tw) * DW_TW;
  const int y0 = ho0 * a.sh - a.ph - R, x0 = wo0 * a.sw - a.pw - R;
  const int tid = threadIdx.x;
  const int v = tid & 7, pxl = tid >> 3;  // channel vector; pixel (and pixel + 64)
  const uint32_t pxb = (uint32_t)a.Cp * 2u;
  const auto xr = make_rsrc(x + (int64_t)n * a.H * a.W * a.Cp, (uint32_t)((size_t)a.H * a.W * a.Cp * 2));
  const int nwin = WH * WW * 8;
  for (int b0 = 0; b0 < nwin; b0 += 4 * DW_NT) {
    u32x4 val[4];
    int dst[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = b0 + u * DW_NT + tid;
      const int pix = i >> 3, vv = i & 7;
      const int wy = pix / WW, wx = pix - wy * WW;
      const int yy = y0 + wy, xx = x0 + wx;
      const bool in = i < nwin && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      val[u] = buf_load16(xr, in ? (uint32_t)(yy * a.W + xx) * pxb + (uint32_t)vv * 16u : SR_OOB);
      dst[u] = i < nwin ? pix * 128 + ((vv ^ (pix & 7)) << 4) : -1;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (dst[u] >= 0) *(u32x4*)(sX + dst[u]) = val[u];
  }
  const int gl = a.cpg / 8;             // lanes per deformable group (1, 2, 4 or 8)
  const int dgi = v * 8 / a.cpg;
  const int nrow = 3 * a.DG;            // staged rows per tap
  const int64_t obase = (int64_t)n * a.DG * 2 * a.K * HWo64, mbase = (int64_t)n * a.DG * a.K * HWo64;
  float vmax = 0.f;
  for (int k = 0; k < a.K; ++k) {
    // stage this tap's offsets and masks: row r < 2*DG is (group r/2, component r%2), then masks
    // (loading the next tap's a tap ahead in registers measured slower: 445 vs 421 us)
    for (int i = tid; i < nrow * DF_TP; i += DW_NT) {
      const int r = i / DF_TP, q = i - r * DF_TP;
      const int ho = ho0 + (q >> 4), wo = wo0 + (q & 15);
      float val = 0.f;
      if (ho < a.Ho && wo < a.Wo) {
        const int64_t pp = (int64_t)ho * a.Wo + wo;
        if (r < 2 * a.DG) val = off[obase + (int64_t)((r >> 1) * 2 * a.K + 2 * k + (r & 1)) * HWo64 + pp];
        else val = msk ? msk[mbase + (int64_t)((r - 2 * a.DG) * a.K + k) * HWo64 + pp] : 1.f;
      }
      sO[i] = val;
    }
    __syncthreads();
    const int ti = k / a.kw, tj = k - ti * a.kw;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = pxl + 64 * j;
      const int ho = ho0 + (px >> 4), wo = wo0 + (px & 15);
      const bool pv = ho < a.Ho && wo < a.Wo;
      const int p = pv ? ho * a.Wo + wo : 0;
      u32x4 dcu = u32x4{0u, 0u, 0u, 0u};
      if (pv) dcu = *(const u32x4*)(dcols + ((int64_t)n * HWo64 + p) * a.L + k * 64 + v * 8);
      float* ph = &sO[(2 * dgi) * DF_TP + px];
      float* pw = &sO[(2 * dgi + 1) * DF_TP + px];
      float* pm = &sO[(2 * a.DG + dgi) * DF_TP + px];
      const float m = *pm;
      const float h = (float)(ho * a.sh - a.ph + ti * a.dh) + *ph;
      const float w = (float)(wo * a.sw - a.pw + tj * a.dw) + *pw;
      const Sample s = make_sample(h, w, a.H, a.W);
      const bool ok = pv && s.valid;
      float acc_h = 0.f, acc_w = 0.f, acc_m = 0.f;
      if (ok) {
        const int ly = (int)floorf(h) - y0, lx = (int)floorf(w) - x0;
        u32x4 cv[4];
        if (ly >= 0 && ly + 1 < WH && lx >= 0 && lx + 1 < WW) {
          const int q0 = ly * WW + lx;
          const int qs[4] = {q0, q0 + 1, q0 + WW, q0 + WW + 1};
#pragma unroll
          for (int q = 0; q < 4; ++q) cv[q] = *(const u32x4*)(sX + qs[q] * 128 + ((v ^ (qs[q] & 7)) << 4));
        } else {
          const uint32_t cb16 = (uint32_t)v * 16u;
          cv[0] = buf_load16(xr, s.o1 >= 0 ? (uint32_t)s.o1 * pxb + cb16 : SR_OOB);
          cv[1] = buf_load16(xr, s.o2 >= 0 ? (uint32_t)s.o2 * pxb + cb16 : SR_OOB);
          cv[2] = buf_load16(xr, s.o3 >= 0 ? (uint32_t)s.o3 * pxb + cb16 : SR_OOB);
          cv[3] = buf_load16(xr, s.o4 >= 0 ? (uint32_t)s.o4 * pxb + cb16 : SR_OOB);
        }
        const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const auto f = [&](uint32_t w32) { return __uint_as_float((e & 1) ? (w32 & 0xffff0000u) : (w32 << 16)); };
          const float v1 = f(cv[0][e >> 1]), v2 = f(cv[1][e >> 1]), v3 = f(cv[2][e >> 1]), v4 = f(cv[3][e >> 1]);
          const float dc = f(dcu[e >> 1]);
          const float wh = -s.hw * v1 - s.lw * v2 + s.hw * v3 + s.lw * v4;
          const float ww = -s.hh * v1 + s.hh * v2 - s.lh * v3 + s.lh * v4;
          acc_h += wh * dc * m;
          acc_w += ww * dc * m;
          acc_m += dc * (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
          vmax = fmaxf(vmax, fabsf(dc * m));
          if (!(fabsf(dc * m) <= 3.0e38f)) vmax = __builtin_inff();
        }
      }
      // combine the group's lanes (consecutive: v is the lane's low 3 bits)
      for (int o = 1; o < gl; o <<= 1) {
        acc_h += __shfl_xor(acc_h, o);
        acc_w += __shfl_xor(acc_w, o);
        acc_m += __shfl_xor(acc_m, o);
      }
      __builtin_amdgcn_wave_barrier();
      if ((v & (gl - 1)) == 0) {  // every lane of the group has read these words (same wave)
        *ph = acc_h;
        *pw = acc_w;
        *pm = acc_m;
      }
    }
    __syncthreads();
    for (int i = tid; i < nrow * DF_TP; i += DW_NT) {
      const int r = i / DF_TP, q = i - r * DF_TP;
      const int ho = ho0 + (q >> 4), wo = wo0 + (q & 15);
      if (ho >= a.Ho || wo >= a.Wo) continue;
      const int64_t pp = (int64_t)ho * a.Wo + wo;
      if (r < 2 * a.DG) goff[obase + (int64_t)((r >> 1) * 2 * a.K + 2 * k + (r & 1)) * HWo64 + pp] = sO[i];
      else if (gmsk) gmsk[mbase + (int64_t)((r - 2 * a.DG) * a.K + k) * HWo64 + pp] = sO[i];
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
  if ((tid & 63) == 0 && vmax > 0.f) atomicMax(amax + n, __float_as_uint(vmax));
}

// dcn_coord_win_kernel's shapes (as the fused forward's, any Cout) and window (R <= 2, LDS <= 80 KB
// so two blocks share a CU); SR_DCN_COORD_WIN=0 keeps dcn_coord_grad_kernel (A/B).
bool coord_win_ok(const sr_dcn_desc* d, const DcnArgs& a) {
  const bool off = sr_knob(K_DCN_COORD_WIN) == 0;
  return !off && d->dtype == SR_BF16 && a.G == 1 && a.C == 64 && a.Cp == 64 && a.cgp == 64 && a.cpg % 8 == 0 &&
         (size_t)a.H * a.W * a.Cp * 2 < 0x80000000ull;
}
bool coord_win_geom(const DcnArgs& a, int* R, int* WH, int* WW, size_t* lds) {
  for (int r = 2; r >= 0; --r) {
    const int wh = (DW_TH - 1) * a.sh + (a.kh - 1) * a.dh + 2 + 2 * r;
    const int ww = (DW_TW - 1) * a.sw + (a.kw - 1) * a.dw + 2 + 2 * r;
    const size_t l = (size_t)3 * a.DG * DF_TP * 4 + (size_t)wh * ww * 128;
    if (l <= 80 * 1024) {
      *R = r; *WH = wh; *WW = ww; *lds = l;
      return true;
    }
  }
  return false;
}

// ---------------------------------------------------------------------------------------------
// Fused backward (round 4; bf16, one conv group, C = 64, Cout <= 64): the column gradient
// dcols = dy . W (the reference's per-image addmm into columns, deform_conv_cuda.cpp:640-660) is
// never stored.  Both kernels form each tap's dcols tile on MFMA from the dy tile, transposed:
// dcols^T[ci][px] = sum_co wd[k*64 + ci][co] * dy[px][co] (v_mfma_f32_16x16x32_bf16 with the
// weight rows as A and a pixel row of dy as B), rounded to bf16 as the dcols path's GEMM stores it,
// so both paths sample the same values.
//   dcn_coord_dy8_kernel : offset / mask gradients (col2im_coord, deform_conv_cuda_kernel.cu:696-770)
//                          on dcn_coord_win_kernel's 8 x 16 tile and x window, the tap's 64 x 64 weight
//                          slice double-buffered in LDS; per-image max |mask * dcols|.
//   dcn_gradx_dy8_kernel : the bilinear scatter (col2im, :635-693) into the fixed-point LDS image of a
//                          16 x 16 tile's footprint, 16 channels per pass (one MFMA tile), weight
//                          fragments from L2 a tap ahead, offsets / masks a tap ahead.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// 4 bf16 channels [c, c + 4) of pixel q of the LDS window (slot layout of dcn_fwd_win_kernel)
SR_DEV u32x2 win_read4(const unsigned char* sX, int q, int c) {
  return *(const u32x2*)(sX + q * 128 + (((c >> 3) ^ (q & 7)) << 4) + ((c >> 2) & 1) * 8);
}
SR_DEV u32x2 glb_read4(__amdgpu_buffer_rsrc_t xr, int o, uint32_t pxb, int c) {
  const u32x4 v = buf_load16(xr, o >= 0 ? (uint32_t)o * pxb + (uint32_t)(c >> 3) * 16u : SR_OOB);
  return (c & 4) ? u32x2{v[2], v[3]} : u32x2{v[0], v[1]};
}
SR_DEV float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
SR_DEV float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
SR_DEV float bf16_round(float v) { return bf16_to_f32(f32_to_bf16(v)); }

constexpr int DX_TT = 16, DX_CPP = 16, DX_ST = DX_CPP + 1;  // tile edge, channels per pass, LDS pixel stride
constexpr int GX_PD = 1;  // taps of operands in flight in the scatter kernel (3: 394 vs 354 us)

// Eight-channel lane layout.  The MFMA leaves a lane 4 channels (16 cb + 4 (lane >> 4) .. + 3) of ONE
// pixel (lane & 15) per 16-channel tile; a bilinear sample (offset / mask reads, corner geometry) for
// 4 channels measured 438 us for the coordinate kernel (SQ: half the wave time waiting, VALU-heavy).
// With two pixel tiles per wave (tile rows 2 w and 2 w + 1) a lane swaps with lane ^ 16 the row it does
// not keep: afterwards lane (g, pl) holds channels 16 cb + 8 (g >> 1) .. + 7 of pixel pl of row g & 1 --
// one 16-B channel vector, one sample per deformable-group vector (308 us).
SR_DEV void own8(const f32x4& a0, const f32x4& a1, int g, float (&o)[8]) {
  const bool odd = g & 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float recv = __shfl_xor(odd ? a0[i] : a1[i], 16);  // the partner's values of my row
    const float mine = odd ? a1[i] : a0[i];
    o[i] = bf16_round(odd ? recv : mine);
    o[4 + i] = bf16_round(odd ? mine : recv);
  }
}

constexpr int DC8_NT = 256;  // 4 waves: an 8 x 16 tile, two rows per wave

// Offsets / masks read per lane a tap ahead (16 consecutive pixels of one plane per 16 lanes) and the
// gradients stored per lane, so no offset staging and ONE barrier per tap (the weight slices are
// double-buffered in LDS).  gxz (optional): the NCHW grad_x of the call, zeroed by the blocks after
// their last tap (the scatter kernel that follows accumulates into it).
__global__ void __launch_bounds__(DC8_NT, 2) dcn_coord_dy8_kernel(DcnArgs a, const bf16_t* __restrict__ dy, int ldy,
                                                                 const bf16_t* __restrict__ wd, int ldw, int cop,
                                                                 const bf16_t* __restrict__ x,
                                                                 const float* __restrict__ off,
                                                                 const float* __restrict__ msk,
                                                                 float* __restrict__ goff, float* __restrict__ gmsk,
                                                                 unsigned* __restrict__ amax, int R, int WH, int WW,
                                                                 float* __restrict__ gxz, int64_t gxn4) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
  bf16_t* sW = (bf16_t*)s_raw;                                 // [2][64 ci][DF_RS]: wd rows of taps k, k + 1
  unsigned char* sX = s_raw + 2 * 64 * DF_RS * 2;             // [WH * WW][8 slots][16 B]
  const int HWo = a.Ho * a.Wo;
  const int64_t HWo64 = HWo;
  const int tw = (a.Wo + DW_TW - 1) / DW_TW, th = (a.Ho + DW_TH - 1) / DW_TH;
  const int bid = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / (tw * th), t = bid - n * (tw * th);
  const int ho0 = (t / tw) * DW_TH, wo0 = (t - (t / tw) * tw) * DW_TW;
  const int y0 = ho0 * a.sh - a.ph - R, x0 = wo0 * a.sw - a.pw - R;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4, pl = lane & 15;
  const int ho = ho0 + 2 * wv + (g & 1), wo = wo0 + pl;  // this lane's pixel
  const bool pv = ho < a.Ho && wo < a.Wo;
  const int p = pv ? ho * a.Wo + wo : 0;
  const uint32_t pxb = (uint32_t)a.Cp * 2u;
  const auto xr = make_rsrc(x + (int64_t)n * a.H * a.W * a.Cp, (uint32_t)((size_t)a.H * a.W * a.Cp * 2));
  const auto dyr = make_rsrc(dy + (int64_t)n * HWo64 * ldy, (uint32_t)((size_t)HWo * ldy * 2));
  const auto wr = make_rsrc(wd, (uint32_t)((size_t)a.K * 64 * ldw * 2));
  u32x4 dyf[2][2];  // B fragments of both rows
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int hu = ho0 + 2 * wv + uu;
    const bool v = hu < a.Ho && wo < a.Wo;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int co = 32 * kk + 8 * g;
      dyf[uu][kk] = buf_load16(dyr, v && co < cop ? (uint32_t)((hu * a.Wo + wo) * ldy + co) * 2u : SR_OOB);
    }
  }
  auto wload = [&](int k, u32x4 (&wp)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = tid + DC8_NT * j, row = q >> 3, pc = q & 7;
      wp[j] = buf_load16(wr, 8 * pc < cop ? (uint32_t)((k * 64 + row) * ldw + 8 * pc) * 2u : SR_OOB);
    }
  };
  auto wstore = [&](int buf, const u32x4 (&wp)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = tid + DC8_NT * j, row = q >> 3, pc = q & 7;
      *(u32x4*)&sW[(buf * 64 + row) * DF_RS + 8 * pc] = wp[j];
    }
  };
  const int64_t obase = (int64_t)n * a.DG * 2 * a.K * HWo64, mbase = (int64_t)n * a.DG * a.K * HWo64;
  int dgc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) dgc[cb] = (16 * cb + 8 * (g >> 1)) / a.cpg;
  auto load_om = [&](int k, float (&o)[4][3]) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int dgi = dgc[cb];
      o[cb][0] = pv ? off[obase + (int64_t)(dgi * 2 * a.K + 2 * k) * HWo64 + p] : 0.f;
      o[cb][1] = pv ? off[obase + (int64_t)(dgi * 2 * a.K + 2 * k + 1) * HWo64 + p] : 0.f;
      o[cb][2] = pv ? (msk ? msk[mbase + (int64_t)(dgi * a.K + k) * HWo64 + p] : 1.f) : 0.f;
    }
  };
  u32x4 wp[2];
  wload(0, wp);
  float om[4][3], om1[4][3];  // taps k and k + 1 (the loads run two taps ahead)
  load_om(0, om);
  if (a.K > 1) load_om(1, om1);
  const int nwin = WH * WW * 8;
  for (int b0 = 0; b0 < nwin; b0 += 4 * DC8_NT) {
    u32x4 val[4];
    int dst[4];
#pragma unroll
    for (int uq = 0; uq < 4; ++uq) {
      const int i = b0 + uq * DC8_NT + tid;
      const int pix = i >> 3, vv = i & 7;
      const int wy = pix / WW, wx = pix - wy * WW;
      const int yy = y0 + wy, xx = x0 + wx;
      const bool in = i < nwin && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W;
      val[uq] = buf_load16(xr, in ? (uint32_t)(yy * a.W + xx) * pxb + (uint32_t)vv * 16u : SR_OOB);
      dst[uq] = i < nwin ? pix * 128 + ((vv ^ (pix & 7)) << 4) : -1;
    }
#pragma unroll
    for (int uq = 0; uq < 4; ++uq)
      if (dst[uq] >= 0) *(u32x4*)(sX + dst[uq]) = val[uq];
  }
  wstore(0, wp);
  if (a.K > 1) wload(1, wp);
  __syncthreads();
  float vmax = 0.f;
  const int gv = a.cpg / 8;  // channel vectors per deformable group
  for (int k = 0; k < a.K; ++k) {
    float omn[4][3];
    if (k + 2 < a.K) load_om(k + 2, omn);
    f32x4 acc[2][4];
#pragma unroll
    for (int uu = 0; uu < 2; ++uu)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[uu][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* sWk = sW + (k & 1) * 64 * DF_RS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const u32x4 af = *(const u32x4*)&sWk[(16 * cb + pl) * DF_RS + 32 * kk + 8 * g];
        mfma_bf16(af, dyf[0][kk], acc[0][cb]);
        mfma_bf16(af, dyf[1][kk], acc[1][cb]);
      }
    if (k + 1 < a.K) {  // the other buffer's last readers (tap k - 1) are past this tap's barrier
      wstore((k + 1) & 1, wp);
      if (k + 2 < a.K) wload(k + 2, wp);
    }
    const int ti = k / a.kw, tj = k - ti * a.kw;
    const float hk = (float)(ho * a.sh - a.ph + ti * a.dh), wk = (float)(wo * a.sw - a.pw + tj * a.dw);
    float rh[4], rw[4], rm[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float dc[8];
      own8(acc[0][cb], acc[1][cb], g, dc);
      const int v = 2 * cb + (g >> 1);
      const float m = om[cb][2];
      const float h = hk + om[cb][0], w = wk + om[cb][1];
      const Sample s = make_sample(h, w, a.H, a.W);
      float ah = 0.f, aw = 0.f, am = 0.f;
      if (pv && s.valid) {
        const int ly = (int)floorf(h) - y0, lx = (int)floorf(w) - x0;
        u32x4 cv[4];
        if (ly >= 0 && ly + 1 < WH && lx >= 0 && lx + 1 < WW) {
          const int q0 = ly * WW + lx;
          const int qs[4] = {q0, q0 + 1, q0 + WW, q0 + WW + 1};
#pragma unroll
          for (int q = 0; q < 4; ++q) cv[q] = *(const u32x4*)(sX + qs[q] * 128 + ((v ^ (qs[q] & 7)) << 4));
        } else {
          const uint32_t cb16 = (uint32_t)v * 16u;
          cv[0] = buf_load16(xr, s.o1 >= 0 ? (uint32_t)s.o1 * pxb + cb16 : SR_OOB);
          cv[1] = buf_load16(xr, s.o2 >= 0 ? (uint32_t)s.o2 * pxb + cb16 : SR_OOB);
          cv[2] = buf_load16(xr, s.o3 >= 0 ? (uint32_t)s.o3 * pxb + cb16 : SR_OOB);
          cv[3] = buf_load16(xr, s.o4 >= 0 ? (uint32_t)s.o4 * pxb + cb16 : SR_OOB);
        }
        const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const auto f = [&](uint32_t w32) { return __uint_as_float((e & 1) ? (w32 & 0xffff0000u) : (w32 << 16)); };
          const float v1 = f(cv[0][e >> 1]), v2 = f(cv[1][e >> 1]), v3 = f(cv[2][e >> 1]), v4 = f(cv[3][e >> 1]);
          const float wh = -s.hw * v1 - s.lw * v2 + s.hw * v3 + s.lw * v4;
          const float ww = -s.hh * v1 + s.hh * v2 - s.lh * v3 + s.lh * v4;
          ah += wh * dc[e] * m;
          aw += ww * dc[e] * m;
          am += dc[e] * (w1 * v1 + w2 * v2 + w3 * v3 + w4 * v4);
          vmax = fmaxf(vmax, fabsf(dc[e] * m));
          if (!(fabsf(dc[e] * m) <= 3.0e38f)) vmax = __builtin_inff();
        }
      }
      rh[cb] = ah; rw[cb] = aw; rm[cb] = am;
    }
    // a group's vectors: cb pairs (cpg 32) or all four (cpg 64) of the lane, then the lanes ^ 32
    if (gv >= 4) {
      rh[0] += rh[1]; rw[0] += rw[1]; rm[0] += rm[1];
      rh[2] += rh[3]; rw[2] += rw[3]; rm[2] += rm[3];
    }
    if (gv >= 8) { rh[0] += rh[2]; rw[0] += rw[2]; rm[0] += rm[2]; }
    if (gv >= 2) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        rh[cb] += __shfl_xor(rh[cb], 32); rw[cb] += __shfl_xor(rw[cb], 32); rm[cb] += __shfl_xor(rm[cb], 32);
      }
    }
    if (pv) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int v = 2 * cb + (g >> 1);
        if (v % gv == 0) {  // the lane holding the group's first vector
          const int dgi = dgc[cb];
          goff[obase + (int64_t)(dgi * 2 * a.K + 2 * k) * HWo64 + p] = rh[cb];
          goff[obase + (int64_t)(dgi * 2 * a.K + 2 * k + 1) * HWo64 + p] = rw[cb];
          if (gmsk) gmsk[mbase + (int64_t)(dgi * a.K + k) * HWo64 + p] = rm[cb];
        }
      }
    }
    __syncthreads();  // the next tap's weight slice is in LDS
    if (k + 1 < a.K) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int e = 0; e < 3; ++e) {
          om[cb][e] = om1[cb][e];
          om1[cb][e] = omn[cb][e];
        }
    }
  }
  for (int o = 32; o > 0; o >>= 1) vmax = fmaxf(vmax, __shfl_xor(vmax, o));
  if (lane == 0 && vmax > 0.f) atomicMax(amax + n, __float_as_uint(vmax));
  for (int64_t i = (int64_t)blockIdx.x * DC8_NT + tid; i < gxn4; i += (int64_t)gridDim.x * DC8_NT)
    ((f32x4*)gxz)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// The scatter kernel.  FXB 64: the int64 fixed-point LDS image of the
// round-3 kernel (scale 2^(48 - e) for a per-image max |mask * dcols| below 2^e); FXB 32: int32 fixed
// point, scale 2^(18 - e): a cell sums at most 16 x 16 pixels x 9 taps < 2^12 contributions of at
// most 2^18 each, so it cannot overflow; the quantum is 2^-18 of the image's max |mask * dcols| (the
// dcols themselves carry bf16 rounding, 2^-9 of each value).  The float -> int64 conversion is ~12 VALU
// instructions per corner and channel, the int32 one two -- the kernel is VALU-bound on them -- and
// the int32 image is half the LDS (a wider halo fits).  fp32 LDS atomics are ~25x slower on gfx950.
// NCHW: grad_x as fp32 [N][C][H][W] (the op's output layout: no NHWC -> NCHW pass), else NHWC
// [N][H][W][Cp]; the flush then walks pixels fastest, so the atomics of a wave are row-contiguous.
// OCC: 8-wave blocks per CU the registers are budgeted for (launch bounds count waves per SIMD; at 3
// the int32 kernel spills 22 VGPRs and ran 1.10 vs 1.01 ms for the C5 op fwd + bwd)
template <int FXB, bool NCHW, int OCC = 2>
__global__ void __launch_bounds__(DW_NT, 2 * OCC) dcn_gradx_dy8_kernel(DcnArgs a, int R, int RH, int RW,
                                                                 const bf16_t* __restrict__ dy, int ldy,
                                                                 const bf16_t* __restrict__ wd, int ldw, int cop,
                                                                 const float* __restrict__ off,
                                                                 const float* __restrict__ msk,
                                                                 const unsigned* __restrict__ amax,
                                                                 float* __restrict__ gx) {
  extern __shared__ unsigned long long s_acc[];  // [RH * RW][DX_ST]: u64 (FXB 64) or u32
  unsigned* s_acc32 = (unsigned*)s_acc;
  const int HWo = a.Ho * a.Wo;
  const int64_t HWo64 = HWo;
  const int tw = (a.Wo + DX_TT - 1) / DX_TT, th = (a.Ho + DX_TT - 1) / DX_TT;
  const int bid = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / (tw * th), t = bid - n * (tw * th);
  const float mx = __uint_as_float(amax[n]);
  if (mx == 0.f) return;  // nothing of this image is scattered (uniform per block)
  const bool direct = !(mx <= 3.0e38f);
  int ex = 0;
  frexpf(direct ? 1.f : mx, &ex);
  const int e = min(127, (FXB == 64 ? 48 : 18) - ex);
  const float sc = ldexpf(1.f, e), isc = ldexpf(1.f, -e);
  const int ho0 = (t / tw) * DX_TT, wo0 = (t - (t / tw) * tw) * DX_TT;
  const int ry0 = ho0 * a.sh - a.ph - R, rx0 = wo0 * a.sw - a.pw - R;
  const int RP = RH * RW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, g = lane >> 4, pl = lane & 15;
  const int64_t HW64 = (int64_t)a.H * a.W;
  float* gim = gx + (int64_t)n * HW64 * (NCHW ? a.C : a.Cp);
  // element (pixel o, channel c) of this image's grad_x, and the step between channels
  auto gaddr = [&](int64_t o, int c) { return NCHW ? gim + c * HW64 + o : gim + o * a.Cp + c; };
  const int64_t cstep = NCHW ? HW64 : 1;
  const auto dyr = make_rsrc(dy + (int64_t)n * HWo64 * ldy, (uint32_t)((size_t)HWo * ldy * 2));
  const auto wr = make_rsrc(wd, (uint32_t)((size_t)a.K * 64 * ldw * 2));
  const int ho = ho0 + 2 * wv + (g & 1), wo = wo0 + pl;  // this lane's pixel
  const bool pv = ho < a.Ho && wo < a.Wo;
  const int p = pv ? ho * a.Wo + wo : 0;
  u32x4 dyf[2][2];
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int hu = ho0 + 2 * wv + uu;
    const bool v = hu < a.Ho && wo < a.Wo;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int co = 32 * kk + 8 * g;
      dyf[uu][kk] = buf_load16(dyr, v && co < cop ? (uint32_t)((hu * a.Wo + wo) * ldy + co) * 2u : SR_OOB);
    }
  }
  const float* offn = off + (int64_t)n * a.DG * 2 * a.K * HWo64;
  const float* mskn = msk ? msk + (int64_t)n * a.DG * a.K * HWo64 : nullptr;
  for (int c0 = 0; c0 < a.C; c0 += DX_CPP) {
    const int c = c0 + 8 * (g >> 1), dgi = c / a.cpg;  // this lane's 8 channels
    auto load_w = [&](int k, u32x4 (&wa)[2]) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int co = 32 * kk + 8 * g;
        wa[kk] = buf_load16(wr, co < cop ? (uint32_t)((k * 64 + c0 + pl) * ldw + co) * 2u : SR_OOB);
      }
    };
    auto load_om = [&](int k, float (&o)[3]) {
      o[0] = pv ? offn[(int64_t)(dgi * 2 * a.K + 2 * k) * HWo64 + p] : 0.f;
      o[1] = pv ? offn[(int64_t)(dgi * 2 * a.K + 2 * k + 1) * HWo64 + p] : 0.f;
      o[2] = pv ? (mskn ? mskn[(int64_t)(dgi * a.K + k) * HWo64 + p] : 1.f) : 0.f;
    };
    // operands GX_PD taps ahead (a tap's work is ~0.3 us per wave, an HBM load several times that):
    // slot d holds tap k + d; the slots shift down one per tap (register moves)
    u32x4 wa[GX_PD][2];
    float om[GX_PD][3];
#pragma unroll
    for (int d = 0; d < GX_PD; ++d)
      if (d < a.K) {
        load_w(d, wa[d]);
        load_om(d, om[d]);
      }
    for (int i = tid; i < RP * DX_ST; i += DW_NT) {
      if (FXB == 64) s_acc[i] = 0ull;
      else s_acc32[i] = 0u;
    }
    __syncthreads();
    for (int k = 0; k < a.K; ++k) {
      u32x4 wn[2];
      float omn[3];
      if (k + GX_PD < a.K) {
        load_w(k + GX_PD, wn);
        load_om(k + GX_PD, omn);
      }
      f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      mfma_bf16(wa[0][0], dyf[0][0], acc0);
      mfma_bf16(wa[0][1], dyf[0][1], acc0);
      mfma_bf16(wa[0][0], dyf[1][0], acc1);
      mfma_bf16(wa[0][1], dyf[1][1], acc1);
      float dm[8];
      own8(acc0, acc1, g, dm);
      const int ti = k / a.kw, tj = k - ti * a.kw;
      const float h = (float)(ho * a.sh - a.ph + ti * a.dh) + om[0][0];
      const float w = (float)(wo * a.sw - a.pw + tj * a.dw) + om[0][1];
      const Sample s = make_sample(h, w, a.H, a.W);
      if (pv && s.valid) {
#pragma unroll
        for (int e2 = 0; e2 < 8; ++e2) dm[e2] *= om[0][2];
        const int hl = (int)floorf(h), wl = (int)floorf(w);
        const float wt[4] = {s.hh * s.hw, s.hh * s.lw, s.lh * s.hw, s.lh * s.lw};
        const int oo[4] = {s.o1, s.o2, s.o3, s.o4};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (oo[q] < 0) continue;
          const int ly = hl + (q >> 1) - ry0, lx = wl + (q & 1) - rx0;
          if (!direct && ly >= 0 && ly < RH && lx >= 0 && lx < RW) {
            const int base = (ly * RW + lx) * DX_ST + 8 * (g >> 1);
#pragma unroll
            for (int e2 = 0; e2 < 8; ++e2) {
              if (FXB == 64) atomicAdd(s_acc + base + e2, (unsigned long long)__float2ll_rn(wt[q] * dm[e2] * sc));
              else atomicAdd(s_acc32 + base + e2, (unsigned)__float2int_rn(wt[q] * dm[e2] * sc));
            }
          } else {
            float* dst = gaddr(oo[q], c);
#pragma unroll
            for (int e2 = 0; e2 < 8; ++e2) unsafeAtomicAdd(dst + e2 * cstep, wt[q] * dm[e2]);
          }
        }
      }
#pragma unroll
      for (int d = 0; d + 1 < GX_PD; ++d) {
        wa[d][0] = wa[d + 1][0]; wa[d][1] = wa[d + 1][1];
        om[d][0] = om[d + 1][0]; om[d][1] = om[d + 1][1]; om[d][2] = om[d + 1][2];
      }
      wa[GX_PD - 1][0] = wn[0]; wa[GX_PD - 1][1] = wn[1];
      om[GX_PD - 1][0] = omn[0]; om[GX_PD - 1][1] = omn[1]; om[GX_PD - 1][2] = omn[2];
    }
    __syncthreads();
    for (int i = tid; i < RP * DX_CPP; i += DW_NT) {
      const int ch = NCHW ? i / RP : i % DX_CPP, pix = NCHW ? i - ch * RP : i / DX_CPP;
      const int yy = ry0 + pix / RW, xx = rx0 + pix % RW;
      if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W) continue;
      const float v = FXB == 64 ? (float)(long long)s_acc[pix * DX_ST + ch] * isc : (float)(int)s_acc32[pix * DX_ST + ch] * isc;
      if (v != 0.f) unsafeAtomicAdd(gaddr((int64_t)yy * a.W + xx, c0 + ch), v);
    }
    __syncthreads();
  }
}

// Shapes and geometry of the fused backward: coord_win's shapes with Cout <= 64; the coordinate
// kernel's LDS (offset tile + weight slice + window, R <= 2) and the scatter image (R <= 2) each
// within 80 KB, two blocks per CU.  (The op layer's SR_DCN_BWD_FUSED=0 keeps the dcols path.)
struct BwdGeom {
  int R1, WH, WW, R2, RH, RW;
  size_t lds1, lds2;
  int fx;  // fixed-point bits of the scatter image (64 / 32)
};
// Scatter image (A/B): knob SR_DCN_GX_FX=64 the int64 fixed-point image, else int32
int gx_fx_env() { return sr_knob(K_DCN_GX_FX) == 64 ? 64 : 32; }

bool bwd_fused_geom(const sr_dcn_desc* d, const DcnArgs& a, int cop, BwdGeom* bg) {
  if (!coord_win_ok(d, a) || cop < 8 || cop > 64 || cop % 8) return false;
  bg->fx = gx_fx_env();
  bool ok1 = false, ok2 = false;
  for (int r = 2; r >= 0 && !ok1; --r) {
    const int wh = (DW_TH - 1) * a.sh + (a.kh - 1) * a.dh + 2 + 2 * r;
    const int ww = (DW_TW - 1) * a.sw + (a.kw - 1) * a.dw + 2 + 2 * r;
    const size_t l = (size_t)2 * 64 * DF_RS * 2 + (size_t)wh * ww * 128;
    if (l <= 80 * 1024) { bg->R1 = r; bg->WH = wh; bg->WW = ww; bg->lds1 = l; ok1 = true; }
  }
  const size_t esz = bg->fx == 64 ? 8 : 4;
  const size_t lim2 = 80 * 1024;
  for (int r = bg->fx == 64 ? 2 : 4; r >= 0 && !ok2; --r) {
    const int rh = (DX_TT - 1) * a.sh + (a.kh - 1) * a.dh + 2 * r + 2;
    const int rw = (DX_TT - 1) * a.sw + (a.kw - 1) * a.dw + 2 * r + 2;
    const size_t l = (size_t)rh * rw * DX_ST * esz;
    if (l <= lim2) { bg->R2 = r; bg->RH = rh; bg->RW = rw; bg->lds2 = l; ok2 = true; }
  }
  return ok1 && ok2;
}

}  // namespace

extern "C" {

int sr_dcn_fwd_fused_ok(const sr_dcn_desc* d, int cout) {
  DcnArgs a;
  if (make_args(d, a) != SR_OK) return 0;
  return dcn_fused_ok(d, a, cout) ? 1 : 0;
}

int sr_dcn_fwd_fused(const sr_dcn_desc* d, const void* x, int x_blocked, const float* offset, const float* mask,
                     const void* wf, int ldw, int wrows, int cout, const float* bias, float* y, void* cols,
                     void* stream) {
  DcnArgs a;
  int rc = make_args(d, a);
  if (rc) return rc;
  if (!dcn_fused_ok(d, a, cout)) return sr_fail(SR_EINVAL, "dcn_fwd_fused: unsupported shape (query sr_dcn_fwd_fused_ok)");
  if (!x || !offset || !wf || !y) return sr_fail(SR_EINVAL, "dcn_fwd_fused: null pointer");
  if (ldw < a.K * 64 || wrows < cout || (size_t)wrows * ldw * 2 >= 0x80000000ull)
    return sr_fail(SR_EINVAL, "dcn_fwd_fused: weight image must be [>= cout][>= K*64] bf16");
  int R, WH, WW;
  size_t lds;
  if (!x_blocked && win_geom(a, &R, &WH, &WW, &lds)) {
    const int wt = ((a.Ho + DW_TH - 1) / DW_TH) * ((a.Wo + DW_TW - 1) / DW_TW);
    if (lds > 65536 &&
        hipFuncSetAttribute((const void*)dcn_fwd_win_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
            hipSuccess)
      return sr_fail(SR_ELAUNCH, "dcn_fwd_fused: LDS attribute");
    hipLaunchKernelGGL(dcn_fwd_win_kernel, dim3((unsigned)(a.N * wt)), dim3(DW_NT), lds, (hipStream_t)stream, a,
                       (const bf16_t*)x, offset, mask, (const bf16_t*)wf, ldw, wrows, cout, bias, y, (bf16_t*)cols,
                       R, WH, WW, dcn_dbg());
    return sr_check(hipGetLastError(), "dcn_fwd_fused launch");
  }
  const int tiles = (a.Ho * a.Wo + DF_TP - 1) / DF_TP;
  hipLaunchKernelGGL(dcn_fwd_mfma_kernel, dim3((unsigned)(a.N * tiles)), dim3(256), 0, (hipStream_t)stream, a,
                     (const bf16_t*)x, offset, mask, (const bf16_t*)wf, ldw, wrows, cout, bias, y, (bf16_t*)cols,
                     x_blocked ? 16u : 128u, x_blocked ? (uint32_t)(a.H * a.W * 16) : 16u);
  return sr_check(hipGetLastError(), "dcn_fwd_fused launch");
}

int sr_dcn_im2col(const sr_dcn_desc* d, const void* x, const float* offset, const float* mask, void* cols,
                  void* stream) {
  DcnArgs a;
  int rc = make_args(d, a);
  if (rc) return rc;
  if (!x || !offset || !cols) return sr_fail(SR_EINVAL, "dcn_im2col: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (d->dtype == SR_BF16) return launch_im2col<bf16_t>(a, x, offset, mask, cols, s);
  if (d->dtype == SR_F32) return launch_im2col<float>(a, x, offset, mask, cols, s);
  return sr_fail(SR_EINVAL, "dcn_im2col: bad dtype");
}

int sr_dcn_bwd_fused_ok(const sr_dcn_desc* d, int cout_p) {
  DcnArgs a;
  BwdGeom bg;
  if (make_args(d, a) != SR_OK) return 0;
  return bwd_fused_geom(d, a, cout_p, &bg) ? 1 : 0;
}

int sr_dcn_bwd_fused(const sr_dcn_desc* d, const void* dy, int ldy, const void* wd, int ldw, int cout_p, const void* x,
                     const float* offset, const float* mask, float* grad_x, int grad_x_nchw, float* grad_offset,
                     float* grad_mask, void* workspace, size_t ws_bytes, void* stream) {
  DcnArgs a;
  int rc = make_args(d, a);
  if (rc) return rc;
  BwdGeom bg;
  if (!bwd_fused_geom(d, a, cout_p, &bg))
    return sr_fail(SR_EINVAL, "dcn_bwd_fused: unsupported shape (query sr_dcn_bwd_fused_ok)");
  if (!dy || !wd || !x || !offset || !grad_x || !grad_offset) return sr_fail(SR_EINVAL, "dcn_bwd_fused: null pointer");
  if (grad_mask && !mask) return sr_fail(SR_EINVAL, "dcn_bwd_fused: grad_mask needs mask");
  if (ldy < cout_p || ldy % 8 || ldw < cout_p || ldw % 8)
    return sr_fail(SR_EINVAL, "dcn_bwd_fused: dy / weight image strides must be >= cout_p and multiples of 8");
  if ((size_t)a.Ho * a.Wo * ldy * 2 >= 0x80000000ull || (size_t)a.K * 64 * ldw * 2 >= 0x80000000ull)
    return sr_fail(SR_ETOOBIG, "dcn_bwd_fused: tensor >= 2 GiB per image");
  if (!workspace || ws_bytes < sr_dcn_col2im_workspace(d)) return sr_fail(SR_EINVAL, "dcn_bwd_fused: workspace too small");
  unsigned* amax = (unsigned*)workspace;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(amax, 0, (size_t)a.N * sizeof(unsigned), s) != hipSuccess)
    return sr_fail(SR_ELAUNCH, "dcn_bwd_fused: memset failed");
  const bool nchw = grad_x_nchw != 0;
  const void* k2 = bg.fx == 64 ? (nchw ? (const void*)dcn_gradx_dy8_kernel<64, true> : (const void*)dcn_gradx_dy8_kernel<64, false>)
                               : (nchw ? (const void*)dcn_gradx_dy8_kernel<32, true> : (const void*)dcn_gradx_dy8_kernel<32, false>);
  if (bg.lds1 > 65536 && hipFuncSetAttribute((const void*)dcn_coord_dy8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)bg.lds1) != hipSuccess)
    return sr_fail(SR_ELAUNCH, "dcn_bwd_fused: LDS attribute");
  if (bg.lds2 > 65536 && hipFuncSetAttribute(k2, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bg.lds2) != hipSuccess)
    return sr_fail(SR_ELAUNCH, "dcn_bwd_fused: LDS attribute");
  // NCHW grad_x is written in full: the coordinate kernel zeroes it (C H W a multiple of 4: C = 64)
  const int64_t gxn4 = nchw ? (int64_t)a.N * a.C * a.H * a.W / 4 : 0;
  const int wt = ((a.Ho + DW_TH - 1) / DW_TH) * ((a.Wo + DW_TW - 1) / DW_TW);
  hipLaunchKernelGGL(dcn_coord_dy8_kernel, dim3((unsigned)(a.N * wt)), dim3(DC8_NT), bg.lds1, s, a, (const bf16_t*)dy,
                     ldy, (const bf16_t*)wd, ldw, cout_p, (const bf16_t*)x, offset, mask, grad_offset, grad_mask, amax,
                     bg.R1, bg.WH, bg.WW, nchw ? grad_x : nullptr, gxn4);
  if (hipGetLastError() != hipSuccess) return sr_fail(SR_ELAUNCH, "dcn_coord_dy8 launch");
  const int xt = ((a.Ho + DX_TT - 1) / DX_TT) * ((a.Wo + DX_TT - 1) / DX_TT);
  const dim3 xg((unsigned)(a.N * xt));
#define SR_GX(FXB, NC, OC)                                                                                    \
  hipLaunchKernelGGL((dcn_gradx_dy8_kernel<FXB, NC, OC>), xg, dim3(DW_NT), bg.lds2, s, a, bg.R2, bg.RH, bg.RW, \
                     (const bf16_t*)dy, ldy, (const bf16_t*)wd, ldw, cout_p, offset, mask, (const unsigned*)amax, \
                     grad_x)
  if (bg.fx == 64) { if (nchw) SR_GX(64, true, 2); else SR_GX(64, false, 2); }
  else { if (nchw) SR_GX(32, true, 2); else SR_GX(32, false, 2); }
#undef SR_GX
  return sr_check(hipGetLastError(), "dcn_gradx_dy8 launch");
}

size_t sr_dcn_col2im_workspace(const sr_dcn_desc* d) { return d ? (size_t)d->N * sizeof(unsigned) : 0; }

int sr_dcn_col2im(const sr_dcn_desc* d, const void* dcols, const void* x, const float* offset, const float* mask,
                  float* grad_x, float* grad_offset, float* grad_mask, void* workspace, size_t ws_bytes,
                  void* stream) {
  DcnArgs a;
  int rc = make_args(d, a);
  if (rc) return rc;
  if (!dcols || !x || !offset || !grad_x || !grad_offset) return sr_fail(SR_EINVAL, "dcn_col2im: null pointer");
  if (!workspace || ws_bytes < sr_dcn_col2im_workspace(d)) return sr_fail(SR_EINVAL, "dcn_col2im: workspace too small");
  unsigned* amax = (unsigned*)workspace;
  if (grad_mask && !mask) return sr_fail(SR_EINVAL, "dcn_col2im: grad_mask needs mask");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(amax, 0, (size_t)a.N * sizeof(unsigned), s) != hipSuccess)
    return sr_fail(SR_ELAUNCH, "dcn_col2im: memset failed");
  if (d->dtype == SR_BF16) {
    int R, WH, WW;
    size_t lds;
    if (coord_win_ok(d, a) && coord_win_geom(a, &R, &WH, &WW, &lds)) {
      const int wt = ((a.Ho + DW_TH - 1) / DW_TH) * ((a.Wo + DW_TW - 1) / DW_TW);
      if (lds > 65536 &&
          hipFuncSetAttribute((const void*)dcn_coord_win_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds) != hipSuccess)
        return sr_fail(SR_ELAUNCH, "dcn_col2im: LDS attribute");
      hipLaunchKernelGGL(dcn_coord_win_kernel, dim3((unsigned)(a.N * wt)), dim3(DW_NT), lds, s, a,
                         (const bf16_t*)dcols, (const bf16_t*)x, offset, mask, grad_offset, grad_mask, amax, R, WH,
                         WW);
      if (hipGetLastError() != hipSuccess) return sr_fail(SR_ELAUNCH, "dcn_coord_win launch");
      return launch_col2im<bf16_t>(a, dcols, x, offset, mask, grad_x, grad_offset, grad_mask, amax, s, false);
    }
    return launch_col2im<bf16_t>(a, dcols, x, offset, mask, grad_x, grad_offset, grad_mask, amax, s);
  }
  if (d->dtype == SR_F32)
    return launch_col2im<float>(a, dcols, x, offset, mask, grad_x, grad_offset, grad_mask, amax, s);
  return sr_fail(SR_EINVAL, "dcn_col2im: bad dtype");
}

}  // extern "C"
