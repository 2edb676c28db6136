// HBM-bound block kernels around the convs of MSRResNet, RCAN and RRDBNet.
//
//   sr_bilinear_up_add   MSRResNet global skip: out += F.interpolate(x, scale, 'bilinear',
//                        align_corners=False) (basicsr/archs/srresnet_arch.py:64-65)
//   sr_channel_reduce    per-(n, c) sum / dot over pixels of NHWC maps (deterministic two-pass):
//                        RCAN ChannelAttention AdaptiveAvgPool2d(1) (rcan_arch.py:19) and its
//                        backward reduction
//   sr_channel_partials  the first pass alone (consumers sum the per-chunk partials)
//   sr_ca_mlp_fwd/_bwd   the 1x1 conv -> ReLU -> 1x1 conv -> Sigmoid squeeze MLP (rcan_arch.py:19-20),
//                        summing partial pools (conv colsum / channel partials) on the way in
//   sr_nc_affine         out = beta x + alpha u s[n, c] + gamma t[n, c] (RCAB tail and its du)
//   sr_ca_fwd_apply      squeeze MLP + RCAB tail y = x + rs * u * s in one launch (rcan_arch.py:22-24, 44-46)
//   sr_ca_bwd_apply      squeeze-MLP backward + du = rs * dout * s + dpool / HW in one launch
//   sr_ca_param_grad     the squeeze convs' parameter gradients (off the critical path)
//   sr_act_backward_nhwc strided (channel-slice) ReLU/LeakyReLU backward (RRDB dense slices)
//   sr_nearest_up_backward  sum of each 2x2 (s x s) block: backward of F.interpolate(
//                        scale_factor=s, mode='nearest') (rrdbnet_arch.py:116-117); _gate: times the
//                        LeakyReLU derivative of the upsampled map (conv_up1 / conv_up2 activations)
//   sr_copy_channels     strided channel-slice copy (RRDB dense buffers)
#include "sr_common.h"
#include "sr_internal.h"

namespace {

__global__ void bilinear_up_add_kernel(const float* __restrict__ x, int N, int C, int H, int W, int s,
                                       const float* __restrict__ base, float* __restrict__ y) {
  const int Ho = H * s, Wo = W * s;
  const int64_t total = (int64_t)N * C * Ho * Wo;
  const float inv = 1.f / (float)s;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (int64_t)gridDim.x * blockDim.x) {
    const int ox = (int)(o % Wo);
    const int oy = (int)((o / Wo) % Ho);
    const int64_t nc = o / ((int64_t)Wo * Ho);
    // PyTorch area_pixel_compute_source_index, align_corners=False, scale = 1/s
    float sy = ((float)oy + 0.5f) * inv - 0.5f;
    float sx = ((float)ox + 0.5f) * inv - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    sx = sx < 0.f ? 0.f : sx;
    const int y0 = (int)sy, x0 = (int)sx;
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
    const float ly1 = sy - (float)y0, lx1 = sx - (float)x0;
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
    const float* p = x + nc * H * W;
    const float v = ly0 * (lx0 * p[y0 * W + x0] + lx1 * p[y0 * W + x1]) +
                    ly1 * (lx0 * p[y1 * W + x0] + lx1 * p[y1 * W + x1]);
    y[o] = base[o] + v;
  }
}

// partial[n][chunk][c] = sum over the chunk's pixels of a[n,p,c] (* b[n,p,c]); threads: 8-channel
// groups x pixel lanes; one block per (chunk, n).
constexpr int RED_CHUNK = 256;  // pixels per block

template <typename T>
__global__ void channel_reduce_partial(const T* __restrict__ a, int lda, int acoff, const T* __restrict__ b, int ldb,
                                       int bcoff, int HW, int C, float* __restrict__ partial) {
  constexpr int PER = Elt<T>::PER16;
  __shared__ float red[256 * 8];
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int groups = C / 8;
  const int lanes = 256 / groups;  // pixel lanes
  const int tid = threadIdx.x;
  const int g = tid % groups, pl = tid / groups;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (PER == 8) {
    // bf16: 8 pixels' loads in flight per iteration (one load pair per round trip left the
    // kernel latency-bound: RCAN 13 us for 34 MB; 4 in flight: 11.6 us)
    if (pl < lanes) {
      const int p0 = chunk * RED_CHUNK, p1 = min(HW, p0 + RED_CHUNK);
      for (int p = p0 + pl; p < p1; p += 8 * lanes) {
        u32x4 va[8], vb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {  // unconditional (clamped) loads, masked after: no branch per load
          const int pu = p + u * lanes;
          const size_t pix = (size_t)n * HW + (pu < p1 ? pu : p);
          va[u] = *(const u32x4*)(a + pix * lda + acoff + g * 8);
          vb[u] = b ? *(const u32x4*)(b + pix * ldb + bcoff + g * 8) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (p + u * lanes >= p1) va[u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float a0 = bf16_to_f32(va[u][k] & 0xffff), a1 = bf16_to_f32(va[u][k] >> 16);
            if (b) { a0 *= bf16_to_f32(vb[u][k] & 0xffff); a1 *= bf16_to_f32(vb[u][k] >> 16); }
            acc[2 * k] += a0;
            acc[2 * k + 1] += a1;
          }
      }
    }
  } else if (pl < lanes) {
    const int p0 = chunk * RED_CHUNK, p1 = min(HW, p0 + RED_CHUNK);
    for (int p = p0 + pl; p < p1; p += lanes) {
      const size_t pix = (size_t)n * HW + p;
      const T* pa = a + pix * lda + acoff + g * 8;
      const T* pb = b ? b + pix * ldb + bcoff + g * 8 : nullptr;
#pragma unroll
      for (int h = 0; h < 8 / PER; ++h) {
        const u32x4 va = *(const u32x4*)(pa + h * PER);
        u32x4 vb;
        if (pb) vb = *(const u32x4*)(pb + h * PER);
        if constexpr (PER == 8) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float a0 = bf16_to_f32(va[k] & 0xffff), a1 = bf16_to_f32(va[k] >> 16);
            if (pb) { a0 *= bf16_to_f32(vb[k] & 0xffff); a1 *= bf16_to_f32(vb[k] >> 16); }
            acc[2 * k] += a0;
            acc[2 * k + 1] += a1;
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float a0 = __uint_as_float(va[k]);
            if (pb) a0 *= __uint_as_float(vb[k]);
            acc[h * 4 + k] += a0;
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[tid * 8 + k] = acc[k];
  __syncthreads();
  if (tid < C) {
    const int gg = tid / 8, k = tid % 8;
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += red[(l * groups + gg) * 8 + k];
    partial[((size_t)n * nchunk + chunk) * C + tid] = s;
  }
}

__global__ void channel_reduce_final(const float* __restrict__ partial, int N, int nchunk, int C, float scale,
                                     float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int k = 0; k < nchunk; ++k) s += partial[((size_t)n * nchunk + k) * C + c];
  out[i] = s * scale;
}

// sum over p = p0, p0 + G, ... < P of base[p * ld], fixed order, 8 loads in flight per batch
SR_DEV float strided_sum(const float* __restrict__ base, int p0, int P, int G, int ld) {
  float acc = 0.f;
  int p = p0;
  for (; p + 7 * G < P; p += 8 * G) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = base[(size_t)(p + k * G) * ld];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  for (; p < P; p += G) acc += base[(size_t)p * ld];
  return acc;
}

// pool[n][c] = scale * sum_p parts[n*P + p][c] (fixed order: G partial sums per channel, then
// their sum), h = relu(W1 pool + b1) [N,Cr], s = sigmoid(W2 h + b2); W1 [Cr][C], W2 [C][Cr].
__global__ __launch_bounds__(1024) void ca_mlp_fwd_kernel(const float* __restrict__ parts, int P, float scale, const float* __restrict__ w1,
                                  const float* __restrict__ b1, const float* __restrict__ w2,
                                  const float* __restrict__ b2, int C, int Cr, float* __restrict__ pool,
                                  float* __restrict__ h, float* __restrict__ s) {
  extern __shared__ float sh[];  // red [max(nt, C)] | pl [C] | hr [Cr]
  const int n = blockIdx.x, nt = blockDim.x;
  const int G = C < nt ? nt / C : 1;
  float* red = sh;
  float* pl = sh + (C > nt ? C : nt);
  float* hr = pl + C;
  const float* pn = parts + (size_t)n * P * C;
  for (int i = threadIdx.x; i < C * G; i += nt) {
    const int c = i % C, g = i / C;
    red[g * C + c] = strided_sum(pn + c, g, P, G, C);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += nt) {
    float acc = 0.f;
    for (int g = 0; g < G; ++g) acc += red[g * C + c];
    acc *= scale;
    pl[c] = acc;
    pool[n * C + c] = acc;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < Cr; r += nt) {
    float acc = b1 ? b1[r] : 0.f;
    for (int c = 0; c < C; ++c) acc += w1[r * C + c] * pl[c];
    acc = acc > 0.f ? acc : 0.f;
    hr[r] = acc;
    h[n * Cr + r] = acc;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += nt) {
    float acc = b2 ? b2[c] : 0.f;
    for (int r = 0; r < Cr; ++r) acc += w2[c * Cr + r] * hr[r];
    s[n * C + c] = 1.f / (1.f + expf(-acc));
  }
}

// Backward of the squeeze MLP for the whole batch (one 1024-thread block, everything staged
// in LDS): ds[n][c] = scale * sum_p parts[n*P + p][c] = d loss / d s.  accumulate: the
// parameter gradients are added to dw1/db1/dw2/db2 (gradient views of the optimizer).
constexpr int CA_MAXNC = 8192, CA_MAXNR = 1024;
__global__ __launch_bounds__(1024) void ca_mlp_bwd_kernel(const float* __restrict__ parts, int P, float scale,
                                                          const float* __restrict__ s, const float* __restrict__ h,
                                                          const float* __restrict__ pool, const float* __restrict__ w1,
                                                          const float* __restrict__ w2, int N, int C, int Cr,
                                                          float* __restrict__ dpool, float* __restrict__ dw1,
                                                          float* __restrict__ db1, float* __restrict__ dw2,
                                                          float* __restrict__ db2, int accumulate) {
  __shared__ float dz2[CA_MAXNC], pl[CA_MAXNC], dz1[CA_MAXNR], hh[CA_MAXNR], W1[CA_MAXNR], W2[CA_MAXNR];
  const int t = threadIdx.x, nt = blockDim.x;
  for (int i = t; i < N * C; i += nt) {
    const int n = i / C, c = i - n * C;
    const float ds = strided_sum(parts + (size_t)n * P * C + c, 0, P, 1, C);
    const float si = s[i];
    dz2[i] = ds * scale * si * (1.f - si);
    pl[i] = pool[i];
  }
  for (int i = t; i < N * Cr; i += nt) hh[i] = h[i];
  for (int i = t; i < C * Cr; i += nt) {
    W1[i] = w1[i];  // [Cr][C]
    W2[i] = w2[i];  // [C][Cr]
  }
  __syncthreads();
  for (int i = t; i < N * Cr; i += nt) {
    const int n = i / Cr, r = i - n * Cr;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc += W2[c * Cr + r] * dz2[n * C + c];
    dz1[i] = hh[i] > 0.f ? acc : 0.f;
  }
  __syncthreads();
  for (int i = t; i < C * Cr; i += nt) {
    const int c = i / Cr, r = i - c * Cr;
    float a2 = 0.f, a1 = 0.f;
    for (int n = 0; n < N; ++n) {
      a2 += dz2[n * C + c] * hh[n * Cr + r];
      a1 += dz1[n * Cr + r] * pl[n * C + c];
    }
    dw2[i] = (accumulate ? dw2[i] : 0.f) + a2;                  // [C][Cr]
    dw1[r * C + c] = (accumulate ? dw1[r * C + c] : 0.f) + a1;  // [Cr][C]
  }
  for (int c = t; c < C; c += nt) {
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc += dz2[n * C + c];
    if (db2) db2[c] = (accumulate ? db2[c] : 0.f) + acc;
  }
  for (int r = t; r < Cr; r += nt) {
    float acc = 0.f;
    for (int n = 0; n < N; ++n) acc += dz1[n * Cr + r];
    if (db1) db1[r] = (accumulate ? db1[r] : 0.f) + acc;
  }
  for (int i = t; i < N * C; i += nt) {
    const int n = i / C, c = i - n * C;
    float acc = 0.f;
    for (int r = 0; r < Cr; ++r) acc += W1[r * C + c] * dz1[n * Cr + r];
    dpool[i] = acc;
  }
}

// ---- Fused channel-attention apply kernels (RCAB, rcan_arch.py:8-24, :44-46) -------------------
// The squeeze MLP of one image is a few hundred FLOPs; as its own launch it is a dependent,
// latency-bound kernel (ca_mlp_fwd 5 us, ca_mlp_bwd 17.6 us on one block) ahead of an elementwise
// pass over the image (nc_affine 8.5 us, HBM-bound).  Here every block of the elementwise pass
// recomputes its image's MLP from the partial sums (fixed summation order, so every block gets
// bit-identical s / dpool) and applies it to its pixel range.  The block issues the loads of the MLP
// operands first (partial rows straight into registers, weights staged in LDS) and then its map
// vectors (CA_VPT 16-B vectors per thread per map): loads retire in order, so the MLP waits for its
// own operands only and its chain runs while the map traffic is in flight.  The chain is kept short:
// the partial rows are summed by 16 row groups per channel quad in parallel, the C-long dot products
// of the 1x1 convs are wave reductions (one output per wave, C % 64 == 0; a per-thread loop
// otherwise), so a block spends ~1 us in it instead of ~5 us of serial LDS loops (RCAN x4 B 32:
// ca_fwd_apply 14.9 us, ca_bwd_apply 9.7 us with the serial chain).  Block 0 of each image also
// writes the MLP state the backward / the parameter gradients need.  Grid (K, N), 256 threads,
// C % 8 == 0, C <= CA_FMAXC, Cr <= CA_FMAXR, C * Cr <= CA_FMAXW, P * C <= CA_FMAXP.
constexpr int CA_FMAXC = 256, CA_FMAXR = 64, CA_FMAXW = 2048, CA_FMAXP = 8192, CA_FNT = 256, CA_VPT = 8;
constexpr int CA_RPT = CA_FMAXP / 4 / CA_FNT;  // partial-row vectors per thread (8)

// Staging into LDS with every load of the thread issued before the first LDS store (a load/store
// loop waits one global-memory round trip per iteration: 17 iterations made ca_param_grad 9 us).
// Up to U floats per thread; the caller guarantees n <= U * CA_FNT.  Loads are unconditional
// (clamped): a branch around a load makes the compiler drain every load in flight at the join.
template <int U>
SR_DEV void ca_stage_f1(const float* __restrict__ src, int n, float* __restrict__ dst) {
  float v[U];
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int i = threadIdx.x + j * CA_FNT;
    v[j] = src[i < n ? i : 0];
  }
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int i = threadIdx.x + j * CA_FNT;
    if (i < n) dst[i] = v[j];
  }
}

// the same in two halves, so that other loads can be issued in between: ca_fetch_f1 loads U floats
// per thread into registers, ca_put_f1 stores all of them to an LDS array of U * CA_FNT floats
// (slots past n hold clamped copies nobody reads)
template <int U>
SR_DEV void ca_fetch_f1(const float* __restrict__ src, int n, float (&v)[U]) {
#pragma unroll
  for (int j = 0; j < U; ++j) {
    const int i = threadIdx.x + j * CA_FNT;
    v[j] = src[i < n ? i : 0];
  }
}
template <int U>
SR_DEV void ca_put_f1(float* __restrict__ dst, const float (&v)[U]) {
#pragma unroll
  for (int j = 0; j < U; ++j) dst[threadIdx.x + j * CA_FNT] = v[j];
}

// this thread's map vectors of pixels [p0, p1) of image n: vector i = p0 * cv + t + j * CA_FNT
template <typename T>
SR_DEV void ca_load_vec(const T* __restrict__ m, size_t base, int i0, int i1, u32x4 (&v)[CA_VPT]) {
#pragma unroll
  for (int j = 0; j < CA_VPT; ++j) {
    const int i = i0 + threadIdx.x + j * CA_FNT;
    v[j] = ((const u32x4*)m)[base + (i < i1 ? i : i0)];  // unconditional (clamped) load: no branch per load
  }
}

// The partial rows [P][C] of one image, thread (q, g) = (t % C4, t / C4): channel quad q, rows
// g, g + RG, ... (RG = CA_FNT / C4 row groups; the host checks P <= CA_RPT * RG, which P * C <= CA_FMAXP
// implies when C4 divides CA_FNT).  ca_rows_issue loads them, ca_rows_sum adds them in
// row order and then the RG group sums in group order into out[c] (LDS), times scale.
SR_DEV void ca_rows_issue(const float* __restrict__ pn, int P, int C, f32x4 (&v)[CA_RPT]) {
  const int C4 = C >> 2, RG = CA_FNT / C4, t = threadIdx.x;
  const int q = t % C4, g = t / C4 < RG ? t / C4 : 0;
#pragma unroll
  for (int j = 0; j < CA_RPT; ++j) {
    const int p = g + j * RG;
    v[j] = ((const f32x4*)pn)[(size_t)(p < P ? p : 0) * C4 + q];  // clamped, masked in ca_rows_sum
  }
}

SR_DEV void ca_rows_sum(const f32x4 (&v)[CA_RPT], int P, int C, f32x4* __restrict__ red, float scale,
                        float* __restrict__ out) {
  const int C4 = C >> 2, RG = CA_FNT / C4, t = threadIdx.x;
  const int g = t / C4;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc = z;
#pragma unroll
  for (int j = 0; j < CA_RPT; ++j) acc += (g < RG && g + j * RG < P) ? v[j] : z;
  red[t] = acc;  // = red[g * C4 + q]; the slots past RG * C4 are never read (unconditional: a branch
                 // here lets the compiler sink the row loads behind the map loads)
  __syncthreads();
  for (int c = t; c < C; c += CA_FNT) {
    const float* rf = (const float*)red;
    float s = 0.f;
    for (int k = 0; k < RG; ++k) s += rf[k * C + c];
    out[c] = s * scale;
  }
}

// sum over the 64 lanes of a wave (every lane gets the same, fixed-order result)
SR_DEV float ca_wave_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
  return xsum32(xsum16(v));
}

// y = x + alpha * u * s[n, c] over pixels [k * ppb, (k + 1) * ppb) of image n
template <typename T>
__global__ __launch_bounds__(256) void ca_fwd_apply_kernel(const float* __restrict__ parts, int P, float scale,
                                                           const float* __restrict__ w1, const float* __restrict__ b1,
                                                           const float* __restrict__ w2, const float* __restrict__ b2,
                                                           const T* __restrict__ x, const T* __restrict__ u, int HW,
                                                           int C, int Cr, int ppb, float alpha, T* __restrict__ y,
                                                           float* __restrict__ pool, float* __restrict__ h,
                                                           float* __restrict__ s) {
  constexpr int PER = Elt<T>::PER16;
  __shared__ f32x4 red[CA_FNT];
  __shared__ float W1[CA_FMAXW], W2[CA_FMAXW], B1[CA_FNT], B2[CA_FNT], pl[CA_FMAXC], hr[CA_FMAXR], sl[CA_FMAXC];
  const int n = blockIdx.y, k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int cv = C / PER;
  const int i0 = k * ppb * cv, i1 = min(HW, (k + 1) * ppb) * cv;
  const size_t base = ((size_t)n * HW) * cv;
  const float* pn = parts + (size_t)n * P * C;
  // the MLP operands first, then the map vectors (loads retire in order)
  f32x4 rv[CA_RPT];
  float w1v[CA_FMAXW / CA_FNT], w2v[CA_FMAXW / CA_FNT], b1v[1], b2v[1];
  ca_rows_issue(pn, P, C, rv);
  ca_fetch_f1(w1, C * Cr, w1v);
  ca_fetch_f1(w2, C * Cr, w2v);
  ca_fetch_f1(b1 ? b1 : w1, b1 ? Cr : 1, b1v);
  ca_fetch_f1(b2 ? b2 : w2, b2 ? C : 1, b2v);
  __builtin_amdgcn_sched_barrier(0);  // issue order: MLP operands, then the maps (loads retire in order)
  u32x4 vx[CA_VPT], vu[CA_VPT];
  ca_load_vec(x, base, i0, i1, vx);
  ca_load_vec(u, base, i0, i1, vu);
  __builtin_amdgcn_sched_barrier(0);  // the map loads stay ahead of the first wait on the MLP operands
  ca_put_f1(W1, w1v);
  ca_put_f1(W2, w2v);
  b1v[0] = b1 ? b1v[0] : 0.f;
  b2v[0] = b2 ? b2v[0] : 0.f;
  ca_put_f1(B1, b1v);
  ca_put_f1(B2, b2v);
  ca_rows_sum(rv, P, C, red, scale, pl);
  __syncthreads();
  if (C % 64 == 0) {  // h[r] = relu(b1 + W1[r] . pool): one wave per output
    for (int r = wv; r < Cr; r += CA_FNT / 64) {
      float acc = 0.f;
      for (int c = lane; c < C; c += 64) acc += W1[r * C + c] * pl[c];
      acc = ca_wave_sum(acc) + B1[r];
      if (lane == 0) hr[r] = acc > 0.f ? acc : 0.f;
    }
  } else {
    for (int r = t; r < Cr; r += CA_FNT) {
      float acc = 0.f;
      for (int c = 0; c < C; ++c) acc += W1[r * C + c] * pl[c];
      acc += B1[r];
      hr[r] = acc > 0.f ? acc : 0.f;
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += CA_FNT) {
    float acc = B2[c];
    for (int r = 0; r < Cr; ++r) acc += W2[c * Cr + r] * hr[r];
    sl[c] = 1.f / (1.f + expf(-acc));
  }
  __syncthreads();
  if (k == 0) {
    for (int c = t; c < C; c += CA_FNT) { pool[n * C + c] = pl[c]; s[n * C + c] = sl[c]; }
    for (int r = t; r < Cr; r += CA_FNT) h[n * Cr + r] = hr[r];
  }
#pragma unroll
  for (int j = 0; j < CA_VPT; ++j) {
    const int i = i0 + t + j * CA_FNT;
    if (i >= i1) break;
    const int c0 = (i % cv) * PER;
    u32x4 o;
    if constexpr (PER == 8) {
      const f32x4 s0 = *(const f32x4*)(sl + c0), s1 = *(const f32x4*)(sl + c0 + 4);
      const float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float u0 = bf16_to_f32(vu[j][q] & 0xffff), u1 = bf16_to_f32(vu[j][q] >> 16);
        const float x0 = bf16_to_f32(vx[j][q] & 0xffff), x1 = bf16_to_f32(vx[j][q] >> 16);
        o[q] = pack_bf16x2(x0 + alpha * u0 * sv[2 * q], x1 + alpha * u1 * sv[2 * q + 1]);
      }
    } else {
      const f32x4 s0 = *(const f32x4*)(sl + c0);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o[q] = __float_as_uint(__uint_as_float(vx[j][q]) + alpha * __uint_as_float(vu[j][q]) * s0[q]);
    }
    ((u32x4*)y)[base + i] = o;
  }
}

// du = alpha * dy * s[n, c] + dpool[n, c] / HW, with ds = alpha * sum_p parts (dL/ds), dz2 = ds s (1 - s),
// dz1 = relu'(h) (W2^T dz2), dpool = W1^T dz1 recomputed per block
template <typename T>
__global__ __launch_bounds__(256) void ca_bwd_apply_kernel(const float* __restrict__ parts, int P, float alpha,
                                                           const float* __restrict__ s, const float* __restrict__ h,
                                                           const float* __restrict__ w1, const float* __restrict__ w2,
                                                           const T* __restrict__ dy, int HW, int C, int Cr, int ppb,
                                                           T* __restrict__ du, float* __restrict__ dz2_out,
                                                           float* __restrict__ dz1_out) {
  constexpr int PER = Elt<T>::PER16;
  __shared__ f32x4 red[CA_FNT];
  __shared__ float W1[CA_FMAXW], W2[CA_FMAXW], sl[CA_FNT], hh[CA_FNT], ds[CA_FMAXC], dz2[CA_FMAXC],
      dz1[CA_FMAXR], tp[CA_FMAXC];
  const int n = blockIdx.y, k = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int cv = C / PER;
  const int i0 = k * ppb * cv, i1 = min(HW, (k + 1) * ppb) * cv;
  const size_t base = ((size_t)n * HW) * cv;
  const float* pn = parts + (size_t)n * P * C;
  // the MLP operands first, then the map vectors (loads retire in order)
  f32x4 rv[CA_RPT];
  float w1v[CA_FMAXW / CA_FNT], w2v[CA_FMAXW / CA_FNT], sv1[1], hv1[1];
  ca_rows_issue(pn, P, C, rv);
  ca_fetch_f1(w1, C * Cr, w1v);
  ca_fetch_f1(w2, C * Cr, w2v);
  ca_fetch_f1(s + n * C, C, sv1);
  ca_fetch_f1(h + n * Cr, Cr, hv1);
  __builtin_amdgcn_sched_barrier(0);  // issue order: MLP operands, then the map (loads retire in order)
  u32x4 vd[CA_VPT];
  ca_load_vec(dy, base, i0, i1, vd);
  __builtin_amdgcn_sched_barrier(0);  // the map loads stay ahead of the first wait on the MLP operands
  ca_put_f1(W1, w1v);
  ca_put_f1(W2, w2v);
  ca_put_f1(sl, sv1);
  ca_put_f1(hh, hv1);
  ca_rows_sum(rv, P, C, red, alpha, ds);
  __syncthreads();
  for (int c = t; c < C; c += CA_FNT) {
    const float si = sl[c];
    dz2[c] = ds[c] * si * (1.f - si);
  }
  __syncthreads();
  if (C % 64 == 0) {  // dz1[r] = relu'(h) W2[:, r] . dz2: one wave per output
    for (int r = wv; r < Cr; r += CA_FNT / 64) {
      float acc = 0.f;
      for (int c = lane; c < C; c += 64) acc += W2[c * Cr + r] * dz2[c];
      acc = ca_wave_sum(acc);
      if (lane == 0) dz1[r] = hh[r] > 0.f ? acc : 0.f;
    }
  } else {
    for (int r = t; r < Cr; r += CA_FNT) {
      float acc = 0.f;
      for (int c = 0; c < C; ++c) acc += W2[c * Cr + r] * dz2[c];
      dz1[r] = hh[r] > 0.f ? acc : 0.f;
    }
  }
  __syncthreads();
  const float inv_hw = 1.f / (float)HW;
  for (int c = t; c < C; c += CA_FNT) {
    float acc = 0.f;
    for (int r = 0; r < Cr; ++r) acc += W1[r * C + c] * dz1[r];
    tp[c] = inv_hw * acc;
  }
  if (k == 0) {
    for (int c = t; c < C; c += CA_FNT) dz2_out[n * C + c] = dz2[c];
    for (int r = t; r < Cr; r += CA_FNT) dz1_out[n * Cr + r] = dz1[r];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < CA_VPT; ++j) {
    const int i = i0 + t + j * CA_FNT;
    if (i >= i1) break;
    const int c0 = (i % cv) * PER;
    u32x4 o;
    if constexpr (PER == 8) {
      const f32x4 s0 = *(const f32x4*)(sl + c0), s1 = *(const f32x4*)(sl + c0 + 4);
      const f32x4 t0 = *(const f32x4*)(tp + c0), t1 = *(const f32x4*)(tp + c0 + 4);
      const float sv[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float tv[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float d0 = bf16_to_f32(vd[j][q] & 0xffff), d1 = bf16_to_f32(vd[j][q] >> 16);
        o[q] = pack_bf16x2(alpha * d0 * sv[2 * q] + tv[2 * q], alpha * d1 * sv[2 * q + 1] + tv[2 * q + 1]);
      }
    } else {
      const f32x4 s0 = *(const f32x4*)(sl + c0), t0 = *(const f32x4*)(tp + c0);
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = __float_as_uint(alpha * __uint_as_float(vd[j][q]) * s0[q] + t0[q]);
    }
    ((u32x4*)du)[base + i] = o;
  }
}

// squeeze-conv parameter gradients from the per-image dz2 / dz1 (same loop order as ca_mlp_bwd_kernel);
// one block, the operands staged in LDS first (the per-n loop over global memory was a 25 us
// latency chain), the n loops in batches of 8 independent LDS loads
__global__ __launch_bounds__(256) void ca_param_grad_kernel(const float* __restrict__ dz2, const float* __restrict__ dz1,
                                                            const float* __restrict__ h, const float* __restrict__ pool,
                                                            int N, int C, int Cr, float* __restrict__ dw1,
                                                            float* __restrict__ db1, float* __restrict__ dw2,
                                                            float* __restrict__ db2, int accumulate) {
  extern __shared__ float sm[];  // dz2 [N*C] | pool [N*C] | dz1 [N*Cr] | h [N*Cr]
  float* Z2 = sm;
  float* PL = Z2 + N * C;
  float* Z1 = PL + N * C;
  float* HH = Z1 + N * Cr;
  const int t = threadIdx.x;
  ca_stage_f1<16>(dz2, N * C, Z2);
  ca_stage_f1<16>(pool, N * C, PL);
  ca_stage_f1<4>(dz1, N * Cr, Z1);
  ca_stage_f1<4>(h, N * Cr, HH);
  __syncthreads();
  for (int i = t; i < C * Cr; i += CA_FNT) {
    const int c = i / Cr, r = i - c * Cr;
    float a2 = 0.f, a1 = 0.f;
    int n = 0;
    for (; n + 7 < N; n += 8) {
      float z2[8], hv[8], z1[8], pv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        z2[q] = Z2[(n + q) * C + c];
        hv[q] = HH[(n + q) * Cr + r];
        z1[q] = Z1[(n + q) * Cr + r];
        pv[q] = PL[(n + q) * C + c];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a2 += z2[q] * hv[q];
        a1 += z1[q] * pv[q];
      }
    }
    for (; n < N; ++n) {
      a2 += Z2[n * C + c] * HH[n * Cr + r];
      a1 += Z1[n * Cr + r] * PL[n * C + c];
    }
    dw2[i] = (accumulate ? dw2[i] : 0.f) + a2;
    dw1[r * C + c] = (accumulate ? dw1[r * C + c] : 0.f) + a1;
  }
  for (int c = t; c < C; c += CA_FNT) {
    if (db2) db2[c] = (accumulate ? db2[c] : 0.f) + strided_sum(Z2 + c, 0, N, 1, C);
  }
  for (int r = t; r < Cr; r += CA_FNT) {
    if (db1) db1[r] = (accumulate ? db1[r] : 0.f) + strided_sum(Z1 + r, 0, N, 1, Cr);
  }
}

// out = beta * x + alpha * u * s[n,c] + gamma * t[n,c]   (all NHWC with the same C, dense)
// RCAB forward: beta 1, alpha rs, s = sigmoid, t = null.  RCAB du: x = null, u = dout,
// alpha = rs, s = sigmoid, gamma = 1/HW, t = dpool.
template <typename T>
__global__ void nc_affine_kernel(const T* __restrict__ x, const T* __restrict__ u, const float* __restrict__ s,
                                 const float* __restrict__ t, uint32_t nv, FastDiv fd_cv, FastDiv fd_hwcv, int C,
                                 float beta, float alpha, float gamma, T* __restrict__ out) {
  constexpr int PER = Elt<T>::PER16;
  // 32-bit indexing (checked on the host); one 16-byte vector = PER consecutive channels
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) {
    const uint32_t q = fdiv(i, fd_cv);
    const int c0 = (int)(i - q * fd_cv.d) * PER;
    const int n = (int)fdiv(i, fd_hwcv);
    const u32x4 vu = ((const u32x4*)u)[i];
    u32x4 vx = {0, 0, 0, 0};
    if (x) vx = ((const u32x4*)x)[i];
    float sv[PER], tv[PER];
    const float* sp = s + n * C + c0;
#pragma unroll
    for (int k = 0; k < PER; k += 4) {
      const f32x4 q4 = *(const f32x4*)(sp + k);
#pragma unroll
      for (int j = 0; j < 4; ++j) sv[k + j] = q4[j];
    }
    if (t) {
      const float* tp = t + n * C + c0;
#pragma unroll
      for (int k = 0; k < PER; k += 4) {
        const f32x4 q4 = *(const f32x4*)(tp + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) tv[k + j] = gamma * q4[j];
      }
    } else {
#pragma unroll
      for (int k = 0; k < PER; ++k) tv[k] = 0.f;
    }
    u32x4 o;
    if constexpr (PER == 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float u0 = bf16_to_f32(vu[k] & 0xffff), u1 = bf16_to_f32(vu[k] >> 16);
        const float x0 = bf16_to_f32(vx[k] & 0xffff), x1 = bf16_to_f32(vx[k] >> 16);
        o[k] = pack_bf16x2(beta * x0 + alpha * u0 * sv[2 * k] + tv[2 * k],
                           beta * x1 + alpha * u1 * sv[2 * k + 1] + tv[2 * k + 1]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = __float_as_uint(beta * __uint_as_float(vx[k]) + alpha * __uint_as_float(vu[k]) * sv[k] + tv[k]);
    }
    ((u32x4*)out)[i] = o;
  }
}

template <typename T>
__global__ void act_backward_nhwc_kernel(const T* __restrict__ dy, int ldd, int dcoff, const T* __restrict__ y, int ldy,
                                         int ycoff, T* __restrict__ out, int ldo, int ocoff, int64_t P, int C, float neg,
                                         float alpha) {
  constexpr int PER = Elt<T>::PER16;
  const int groups = C / PER;
  const int64_t nv = P * groups;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / groups;
    const int g = (int)(i % groups);
    const u32x4 d = *(const u32x4*)(dy + p * ldd + dcoff + g * PER);
    const u32x4 yy = *(const u32x4*)(y + p * ldy + ycoff + g * PER);
    u32x4 o;
    if constexpr (PER == 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = bf16_to_f32(d[k] & 0xffff), d1 = bf16_to_f32(d[k] >> 16);
        const float y0 = bf16_to_f32(yy[k] & 0xffff), y1 = bf16_to_f32(yy[k] >> 16);
        o[k] = pack_bf16x2(alpha * d0 * (y0 > 0.f ? 1.f : neg), alpha * d1 * (y1 > 0.f ? 1.f : neg));
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = __float_as_uint(alpha * __uint_as_float(d[k]) * (__uint_as_float(yy[k]) > 0.f ? 1.f : neg));
    }
    *(u32x4*)(out + p * ldo + ocoff + g * PER) = o;
  }
}

// out[n,y,x,c] (+)= sum_{i,j<s} d[n, y*s+i, x*s+j, c]; with a gate (the LR map the upsample read, itself
// a LeakyReLU / ReLU output): out = that sum * (gate > 0 ? 1 : slope), the activation backward of the
// conv that produced the gate fused in (RRDBNet HR tail, ops/conv.py conv_chain)
template <typename T>
__global__ void nearest_up_backward_kernel(const T* __restrict__ d, int ldd, int N, int H, int W, int C, int s,
                                           const T* __restrict__ gate, int ldg, float slope, T* __restrict__ out,
                                           int ldo, int accumulate) {
  constexpr int PER = Elt<T>::PER16;
  const int groups = C / PER;
  const int64_t nv = (int64_t)N * H * W * groups;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(i % groups);
    const int64_t p = i / groups;
    const int x = (int)(p % W);
    const int y = (int)((p / W) % H);
    const int64_t n = p / ((int64_t)W * H);
    float acc[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) acc[k] = 0.f;
    for (int a = 0; a < s; ++a)
      for (int b = 0; b < s; ++b) {
        const u32x4 v = *(const u32x4*)(d + ((n * H * s + y * s + a) * (int64_t)W * s + x * s + b) * ldd + g * PER);
        if constexpr (PER == 8) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[2 * k] += bf16_to_f32(v[k] & 0xffff);
            acc[2 * k + 1] += bf16_to_f32(v[k] >> 16);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] += __uint_as_float(v[k]);
        }
      }
    if (gate) {
      const u32x4 v = *(const u32x4*)(gate + p * ldg + g * PER);
      if constexpr (PER == 8) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] *= bf16_to_f32(v[k] & 0xffff) > 0.f ? 1.f : slope;
          acc[2 * k + 1] *= bf16_to_f32(v[k] >> 16) > 0.f ? 1.f : slope;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] *= __uint_as_float(v[k]) > 0.f ? 1.f : slope;
      }
    }
    T* dst = out + p * ldo + g * PER;
    if (accumulate) {
      const u32x4 v = *(const u32x4*)dst;
      if constexpr (PER == 8) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += bf16_to_f32(v[k] & 0xffff);
          acc[2 * k + 1] += bf16_to_f32(v[k] >> 16);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += __uint_as_float(v[k]);
      }
    }
    u32x4 o;
    if constexpr (PER == 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = pack_bf16x2(acc[2 * k], acc[2 * k + 1]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(acc[k]);
    }
    *(u32x4*)dst = o;
  }
}

template <typename T>
__global__ void copy_channels_kernel(const T* __restrict__ src, int lds_, int scoff, T* __restrict__ dst, int ldd,
                                     int dcoff, int64_t P, int C) {
  constexpr int PER = Elt<T>::PER16;
  const int groups = C / PER;
  const int64_t nv = P * groups;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / groups;
    const int g = (int)(i % groups);
    *(u32x4*)(dst + p * ldd + dcoff + g * PER) = *(const u32x4*)(src + p * lds_ + scoff + g * PER);
  }
}

inline unsigned grid_for(int64_t n, int64_t cap = 8192) {
  int64_t g = (n + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int sr_bilinear_up_add(const float* x, int N, int C, int H, int W, int s, const float* base, float* y,
                       void* stream) {
  if (!x || !base || !y || s < 1) return sr_fail(SR_EINVAL, "bilinear_up_add: bad arguments");
  const int64_t total = (int64_t)N * C * H * s * W * s;
  hipLaunchKernelGGL(bilinear_up_add_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, x, N, C, H, W,
                     s, base, y);
  return sr_check(hipGetLastError(), "bilinear_up_add launch");
}

size_t sr_channel_reduce_workspace(int N, int HW, int C) {
  return (size_t)N * ((HW + RED_CHUNK - 1) / RED_CHUNK) * C * sizeof(float);
}

int sr_channel_reduce(int dtype, const void* a, int lda, int acoff, const void* b, int ldb, int bcoff, int N, int HW,
                      int C, float scale, float* out, void* workspace, size_t ws_bytes, void* stream) {
  if (!a || !out || !workspace || C % 8 || C > 2048 || C / 8 > 256)
    return sr_fail(SR_EINVAL, "channel_reduce: bad arguments (C multiple of 8, <= 2048)");
  if (ws_bytes < sr_channel_reduce_workspace(N, HW, C)) return sr_fail(SR_EINVAL, "channel_reduce: workspace too small");
  const int nchunk = (HW + RED_CHUNK - 1) / RED_CHUNK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(channel_reduce_partial<bf16_t>, dim3(nchunk, N), dim3(256), 0, s, (const bf16_t*)a, lda, acoff,
                       (const bf16_t*)b, ldb, bcoff, HW, C, (float*)workspace);
  else
    hipLaunchKernelGGL(channel_reduce_partial<float>, dim3(nchunk, N), dim3(256), 0, s, (const float*)a, lda, acoff,
                       (const float*)b, ldb, bcoff, HW, C, (float*)workspace);
  hipLaunchKernelGGL(channel_reduce_final, dim3((N * C + 255) / 256), dim3(256), 0, s, (const float*)workspace, N,
                     nchunk, C, scale, out);
  return sr_check(hipGetLastError(), "channel_reduce launch");
}

int sr_channel_partials_count(int HW) { return (HW + RED_CHUNK - 1) / RED_CHUNK; }

int sr_channel_partials(int dtype, const void* a, int lda, int acoff, const void* b, int ldb, int bcoff, int N,
                        int HW, int C, float* parts, void* stream) {
  if (!a || !parts || C % 8 || C > 2048 || N <= 0 || HW <= 0)
    return sr_fail(SR_EINVAL, "channel_partials: bad arguments (C multiple of 8, <= 2048)");
  const int nchunk = sr_channel_partials_count(HW);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(channel_reduce_partial<bf16_t>, dim3(nchunk, N), dim3(256), 0, s, (const bf16_t*)a, lda, acoff,
                       (const bf16_t*)b, ldb, bcoff, HW, C, parts);
  else
    hipLaunchKernelGGL(channel_reduce_partial<float>, dim3(nchunk, N), dim3(256), 0, s, (const float*)a, lda, acoff,
                       (const float*)b, ldb, bcoff, HW, C, parts);
  return sr_check(hipGetLastError(), "channel_partials launch");
}

int sr_ca_mlp_fwd(const float* parts, int P, float scale, const float* w1, const float* b1, const float* w2,
                  const float* b2, int N, int C, int Cr, float* pool, float* h, float* s_out, void* stream) {
  if (!parts || P < 1 || !w1 || !w2 || !pool || !h || !s_out || C < 1 || Cr < 1)
    return sr_fail(SR_EINVAL, "ca_mlp_fwd: bad arguments");
  const int nt = 1024;
  const size_t smem = ((C > nt ? C : nt) + C + Cr) * sizeof(float);
  if (smem > 64 * 1024) return sr_fail(SR_EINVAL, "ca_mlp_fwd: C too large");
  hipLaunchKernelGGL(ca_mlp_fwd_kernel, dim3(N), dim3(nt), smem, (hipStream_t)stream, parts, P, scale, w1, b1, w2, b2,
                     C, Cr, pool, h, s_out);
  return sr_check(hipGetLastError(), "ca_mlp_fwd launch");
}

int sr_ca_mlp_bwd(const float* parts, int P, float scale, const float* s, const float* h, const float* pool,
                  const float* w1, const float* w2, int N, int C, int Cr, float* dpool, float* dw1, float* db1,
                  float* dw2, float* db2, int accumulate, void* stream) {
  if (!parts || P < 1 || !s || !h || !pool || !w1 || !w2 || !dpool || !dw1 || !dw2)
    return sr_fail(SR_EINVAL, "ca_mlp_bwd: bad arguments");
  if (N * C > CA_MAXNC || N * Cr > CA_MAXNR || C * Cr > CA_MAXNR)
    return sr_fail(SR_EINVAL, "ca_mlp_bwd: N*C <= 8192, N*Cr and C*Cr <= 1024 (split the batch)");
  hipLaunchKernelGGL(ca_mlp_bwd_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, parts, P, scale, s, h, pool, w1,
                     w2, N, C, Cr, dpool, dw1, db1, dw2, db2, accumulate);
  return sr_check(hipGetLastError(), "ca_mlp_bwd launch");
}

// pixels per block of the fused CA kernels: CA_VPT 16-B vectors per thread
static int ca_ppb(int HW, int C, int PER) {
  int ppb = CA_FNT * CA_VPT * PER / C;
  return ppb > HW ? HW : ppb;
}

static bool ca_shapes_ok(int C, int Cr, int P) {
  return C % 8 == 0 && C <= CA_FMAXC && Cr >= 1 && Cr <= CA_FMAXR && C * Cr <= CA_FMAXW && P >= 1 &&
         (int64_t)P * C <= CA_FMAXP && P <= CA_RPT * (CA_FNT / (C / 4));
}

int sr_ca_fwd_apply(int dtype, const float* parts, int P, float scale, const float* w1, const float* b1,
                    const float* w2, const float* b2, const void* x, const void* u, int N, int HW, int C, int Cr,
                    float alpha, void* y, float* pool, float* h, float* s_out, void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!parts || !w1 || !w2 || !x || !u || !y || !pool || !h || !s_out || N < 1 || HW < 1 || !ca_shapes_ok(C, Cr, P) ||
      !aligned16(x) || !aligned16(u) || !aligned16(y) || !aligned16(parts))
    return sr_fail(SR_EINVAL, "ca_fwd_apply: bad arguments (C % 8 == 0, C <= 256, Cr <= 64, C*Cr <= 2048, P*C <= 8192, "
                              "16-B aligned maps and partial rows)");
  if ((int64_t)N * HW * C / PER >= 0x7fffffffll) return sr_fail(SR_ETOOBIG, "ca_fwd_apply: tensor too large");
  const int ppb = ca_ppb(HW, C, PER);
  const dim3 grid((unsigned)((HW + ppb - 1) / ppb), (unsigned)N);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(ca_fwd_apply_kernel<bf16_t>, grid, dim3(CA_FNT), 0, st, parts, P, scale, w1, b1, w2, b2,
                       (const bf16_t*)x, (const bf16_t*)u, HW, C, Cr, ppb, alpha, (bf16_t*)y, pool, h, s_out);
  else
    hipLaunchKernelGGL(ca_fwd_apply_kernel<float>, grid, dim3(CA_FNT), 0, st, parts, P, scale, w1, b1, w2, b2,
                       (const float*)x, (const float*)u, HW, C, Cr, ppb, alpha, (float*)y, pool, h, s_out);
  return sr_check(hipGetLastError(), "ca_fwd_apply launch");
}

int sr_ca_bwd_apply(int dtype, const float* parts, int P, float alpha, const float* s, const float* h, const float* w1,
                    const float* w2, const void* dy, int N, int HW, int C, int Cr, void* du, float* dz2, float* dz1,
                    void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!parts || !s || !h || !w1 || !w2 || !dy || !du || !dz2 || !dz1 || N < 1 || HW < 1 || !ca_shapes_ok(C, Cr, P) ||
      !aligned16(dy) || !aligned16(du) || !aligned16(parts))
    return sr_fail(SR_EINVAL, "ca_bwd_apply: bad arguments (C % 8 == 0, C <= 256, Cr <= 64, C*Cr <= 2048, P*C <= 8192, "
                              "16-B aligned maps and partial rows)");
  if ((int64_t)N * HW * C / PER >= 0x7fffffffll) return sr_fail(SR_ETOOBIG, "ca_bwd_apply: tensor too large");
  const int ppb = ca_ppb(HW, C, PER);
  const dim3 grid((unsigned)((HW + ppb - 1) / ppb), (unsigned)N);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(ca_bwd_apply_kernel<bf16_t>, grid, dim3(CA_FNT), 0, st, parts, P, alpha, s, h, w1, w2,
                       (const bf16_t*)dy, HW, C, Cr, ppb, (bf16_t*)du, dz2, dz1);
  else
    hipLaunchKernelGGL(ca_bwd_apply_kernel<float>, grid, dim3(CA_FNT), 0, st, parts, P, alpha, s, h, w1, w2,
                       (const float*)dy, HW, C, Cr, ppb, (float*)du, dz2, dz1);
  return sr_check(hipGetLastError(), "ca_bwd_apply launch");
}

int sr_ca_param_grad(const float* dz2, const float* dz1, const float* h, const float* pool, int N, int C, int Cr,
                     float* dw1, float* db1, float* dw2, float* db2, int accumulate, void* stream) {
  if (!dz2 || !dz1 || !h || !pool || !dw1 || !dw2 || N < 1 || C < 1 || Cr < 1)
    return sr_fail(SR_EINVAL, "ca_param_grad: bad arguments");
  const size_t smem = (size_t)N * (C + Cr) * 2 * sizeof(float);
  if (N * C > 16 * CA_FNT || N * Cr > 4 * CA_FNT)
    return sr_fail(SR_EINVAL, "ca_param_grad: N * C <= 4096 and N * Cr <= 1024 (split the batch)");
  hipLaunchKernelGGL(ca_param_grad_kernel, dim3(1), dim3(CA_FNT), smem, (hipStream_t)stream, dz2, dz1, h, pool, N, C,
                     Cr, dw1, db1, dw2, db2, accumulate);
  return sr_check(hipGetLastError(), "ca_param_grad launch");
}

int sr_nc_affine(int dtype, const void* x, const void* u, const float* s, const float* t, int N, int HW, int C,
                 float beta, float alpha, float gamma, void* out, void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!u || !s || !out || C % PER || !aligned16(u) || !aligned16(out) || (x && !aligned16(x)) || !aligned16(s) ||
      (t && !aligned16(t)))
    return sr_fail(SR_EINVAL, "nc_affine: bad arguments");
  const int64_t nv = (int64_t)N * HW * C / PER;
  if (nv >= 0x7fffffffll) return sr_fail(SR_ETOOBIG, "nc_affine: tensor too large (split the batch)");
  const FastDiv fcv = make_fastdiv(C / PER), fhw = make_fastdiv((uint32_t)HW * (C / PER));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(nc_affine_kernel<bf16_t>, dim3(grid_for(nv)), dim3(256), 0, st, (const bf16_t*)x,
                       (const bf16_t*)u, s, t, (uint32_t)nv, fcv, fhw, C, beta, alpha, gamma, (bf16_t*)out);
  else
    hipLaunchKernelGGL(nc_affine_kernel<float>, dim3(grid_for(nv)), dim3(256), 0, st, (const float*)x, (const float*)u,
                       s, t, (uint32_t)nv, fcv, fhw, C, beta, alpha, gamma, (float*)out);
  return sr_check(hipGetLastError(), "nc_affine launch");
}

int sr_act_backward_nhwc(int dtype, int64_t P, int C, const void* dy, int ldd, int dcoff, const void* y, int ldy,
                         int ycoff, void* out, int ldo, int ocoff, int act, float slope, float alpha, void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!dy || !y || !out || C % PER || ldd % PER || ldy % PER || ldo % PER || dcoff % PER || ycoff % PER || ocoff % PER)
    return sr_fail(SR_EINVAL, "act_backward_nhwc: bad arguments (16-byte aligned channel slices)");
  const float neg = act == SR_ACT_LRELU ? slope : (act == SR_ACT_RELU ? 0.f : 1.f);
  const int64_t nv = P * (C / PER);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(act_backward_nhwc_kernel<bf16_t>, dim3(grid_for(nv)), dim3(256), 0, st, (const bf16_t*)dy, ldd,
                       dcoff, (const bf16_t*)y, ldy, ycoff, (bf16_t*)out, ldo, ocoff, P, C, neg, alpha);
  else
    hipLaunchKernelGGL(act_backward_nhwc_kernel<float>, dim3(grid_for(nv)), dim3(256), 0, st, (const float*)dy, ldd,
                       dcoff, (const float*)y, ldy, ycoff, (float*)out, ldo, ocoff, P, C, neg, alpha);
  return sr_check(hipGetLastError(), "act_backward_nhwc launch");
}

int sr_nearest_up_backward_gate(int dtype, const void* d, int ldd, int N, int H, int W, int C, int s, const void* gate,
                                int ldg, float slope, void* out, int ldo, int accumulate, void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!d || !out || C % PER || ldd % PER || ldo % PER || s < 1 || (gate && (ldg % PER || ldg < C)))
    return sr_fail(SR_EINVAL, "nearest_up_backward: bad arguments");
  const int64_t nv = (int64_t)N * H * W * (C / PER);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(nearest_up_backward_kernel<bf16_t>, dim3(grid_for(nv)), dim3(256), 0, st, (const bf16_t*)d, ldd,
                       N, H, W, C, s, (const bf16_t*)gate, ldg, slope, (bf16_t*)out, ldo, accumulate);
  else
    hipLaunchKernelGGL(nearest_up_backward_kernel<float>, dim3(grid_for(nv)), dim3(256), 0, st, (const float*)d, ldd, N,
                       H, W, C, s, (const float*)gate, ldg, slope, (float*)out, ldo, accumulate);
  return sr_check(hipGetLastError(), "nearest_up_backward launch");
}

int sr_nearest_up_backward(int dtype, const void* d, int ldd, int N, int H, int W, int C, int s, void* out, int ldo,
                           int accumulate, void* stream) {
  return sr_nearest_up_backward_gate(dtype, d, ldd, N, H, W, C, s, nullptr, 0, 1.f, out, ldo, accumulate, stream);
}

int sr_copy_channels(int dtype, const void* src, int lds_, int scoff, void* dst, int ldd, int dcoff, int64_t P, int C,
                     void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!src || !dst || C % PER || lds_ % PER || ldd % PER || scoff % PER || dcoff % PER)
    return sr_fail(SR_EINVAL, "copy_channels: bad arguments");
  const int64_t nv = P * (C / PER);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(copy_channels_kernel<bf16_t>, dim3(grid_for(nv)), dim3(256), 0, st, (const bf16_t*)src, lds_,
                       scoff, (bf16_t*)dst, ldd, dcoff, P, C);
  else
    hipLaunchKernelGGL(copy_channels_kernel<float>, dim3(grid_for(nv)), dim3(256), 0, st, (const float*)src, lds_,
                       scoff, (float*)dst, ldd, dcoff, P, C);
  return sr_check(hipGetLastError(), "copy_channels launch");
}

}  // extern "C"
