// HBM-bound layout, loss and optimizer kernels of the SR train step.
//
//   sr_nchw_to_nhwc / sr_nhwc_to_nchw : network head/tail boundary (NCHW fp32 API of the
//       reference nets, NHWC inside), fused with the EDSR/RCAN mean shift
//       (basicsr/archs/edsr_arch.py:51-59).
//   sr_pixel_shuffle_nchw             : nn.PixelShuffle / pixel_unshuffle on NCHW
//       (basicsr/archs/arch_util.py:136-139, 217-234), bit-exact index map.
//   sr_l1_loss                        : L1Loss (basicsr/losses/basic_loss.py:27-52) fused
//       with its gradient; deterministic two-pass reduction.
//   sr_adam_ema                       : torch.optim.Adam step + model EMA
//       (basicsr/models/base_model.py:75-82) on the flat fp32 parameter vector.
#include "sr_common.h"
#include "sr_internal.h"

namespace {

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int H, int W, int Cp,
                                    const float* shift, const float* scale, T* __restrict__ y) {
  // one thread per output pixel: reads C strided floats (coalesced across threads along W)
  const int64_t HW = (int64_t)H * W;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N * HW) return;
  const int64_t n = p / HW, hw = p - n * HW;
  T* dst = y + p * Cp;
  for (int c = 0; c < Cp; ++c) {
    float v = 0.f;
    if (c < C) {
      v = x[(n * C + c) * HW + hw];
      v = (v - (shift ? shift[c] : 0.f)) * (scale ? scale[c] : 1.f);
    }
    dst[c] = Elt<T>::from_f(v);
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ x, int N, int H, int W, int ld, int coff, int C,
                                    const float* scale, const float* shift, float* __restrict__ y) {
  const int64_t HW = (int64_t)H * W;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N * HW) return;
  const int64_t n = p / HW, hw = p - n * HW;
  const T* src = x + p * ld + coff;
  for (int c = 0; c < C; ++c) {
    float v = Elt<T>::to_f(src[c]);
    y[(n * C + c) * HW + hw] = v * (scale ? scale[c] : 1.f) + (shift ? shift[c] : 0.f);
  }
}

// Wide-channel variants (feature maps, C >= 16): a 64-pixel x 32-channel tile is
// transposed through LDS so both the NCHW side (pixels contiguous) and the NHWC side
// (channels contiguous) are accessed with unit stride; the per-pixel kernels above are
// kept for the 3-channel image boundary where a tile would be mostly padding.
template <typename T>
__global__ void __launch_bounds__(256) nchw_to_nhwc_tiled_kernel(const float* __restrict__ x, int C, int64_t HW,
                                                                 int Cp, const float* shift, const float* scale,
                                                                 T* __restrict__ y) {
  __shared__ float t[32][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64, n = blockIdx.z;
  const int c0 = blockIdx.y * 32;
  for (int i = threadIdx.x; i < 32 * 64; i += 256) {
    const int c = i >> 6, p = i & 63;
    float v = 0.f;
    if (c0 + c < C && p0 + p < HW) {
      v = x[(n * C + c0 + c) * HW + p0 + p];
      v = (v - (shift ? shift[c0 + c] : 0.f)) * (scale ? scale[c0 + c] : 1.f);
    }
    t[c][p] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 32; i += 256) {
    const int p = i >> 5, c = i & 31;
    if (p0 + p < HW && c0 + c < Cp) y[(n * HW + p0 + p) * Cp + c0 + c] = Elt<T>::from_f(t[c][p]);
  }
}

// Vector form (HW % 4 == 0, Cp % 8 == 0, 16-B aligned maps: the DCN operands, x / dy at C 64):
// a 64-channel x 64-pixel tile, read as float4 along the pixels and written as 8-channel (16 B of
// bf16, 32 B of fp32) vectors per pixel; the scalar tile above moved 4 B in / 2 B out per lane.
// The same arithmetic per element ((x - shift) * scale, one rounding), so the same output bits.
template <typename T>
__global__ void __launch_bounds__(256) nchw_to_nhwc_vec_kernel(const float* __restrict__ x, int C, int64_t HW,
                                                               int Cp, const float* shift, const float* scale,
                                                               T* __restrict__ y) {
  __shared__ float t[64][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64, n = blockIdx.z;
  const int c0 = blockIdx.y * 64;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int c = i >> 4, p = (i & 15) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 + c < C && p0 + p < HW) {
      v = *(const float4*)(x + (n * C + c0 + c) * HW + p0 + p);
      const float sh = shift ? shift[c0 + c] : 0.f, sc = scale ? scale[c0 + c] : 1.f;
      v.x = (v.x - sh) * sc;
      v.y = (v.y - sh) * sc;
      v.z = (v.z - sh) * sc;
      v.w = (v.w - sh) * sc;
    }
    t[c][p] = v.x;
    t[c][p + 1] = v.y;
    t[c][p + 2] = v.z;
    t[c][p + 3] = v.w;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int p = i >> 3, cg = (i & 7) * 8;
    if (p0 + p >= HW || c0 + cg >= Cp) continue;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = t[cg + j][p];
    T* dst = y + (n * HW + p0 + p) * Cp + c0 + cg;
    if constexpr (sizeof(T) == 2) {
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
      *(u32x4*)dst = o;
    } else {
      *(float4*)dst = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(dst + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) nhwc_to_nchw_tiled_kernel(const T* __restrict__ x, int64_t HW, int ld,
                                                                 int coff, int C, const float* scale,
                                                                 const float* shift, float* __restrict__ y) {
  __shared__ float t[32][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64, n = blockIdx.z;
  const int c0 = blockIdx.y * 32;
  for (int i = threadIdx.x; i < 64 * 32; i += 256) {
    const int p = i >> 5, c = i & 31;
    float v = 0.f;
    if (p0 + p < HW && c0 + c < C) v = Elt<T>::to_f(x[(n * HW + p0 + p) * ld + coff + c0 + c]);
    t[c][p] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * 64; i += 256) {
    const int c = i >> 6, p = i & 63;
    if (c0 + c < C && p0 + p < HW)
      y[(n * C + c0 + c) * HW + p0 + p] = t[c][p] * (scale ? scale[c0 + c] : 1.f) + (shift ? shift[c0 + c] : 0.f);
  }
}

// out[n, c, h*r+i, w*r+j] = in[n, c*r*r + i*r + j, h, w]   (r > 0, shuffle)
// out[n, c*s*s + i*s + j, h, w] = in[n, c, h*s+i, w*s+j]   (r = -s, unshuffle)
template <typename T>
__global__ void pixel_shuffle_kernel(const T* __restrict__ x, int N, int C, int H, int W, int r,
                                     T* __restrict__ y) {
  const int64_t total = (int64_t)N * C * H * W;
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
       o += (int64_t)gridDim.x * blockDim.x) {
    if (r > 0) {
      const int Co = C / (r * r), Ho = H * r, Wo = W * r;
      int64_t t = o;
      const int xo = (int)(t % Wo); t /= Wo;
      const int yo = (int)(t % Ho); t /= Ho;
      const int c = (int)(t % Co); const int64_t n = t / Co;
      const int i = yo % r, j = xo % r;
      y[o] = x[((n * C + c * r * r + i * r + j) * H + yo / r) * W + xo / r];
    } else {
      const int s = -r;
      const int Co = C * s * s, Ho = H / s, Wo = W / s;
      int64_t t = o;
      const int xo = (int)(t % Wo); t /= Wo;
      const int yo = (int)(t % Ho); t /= Ho;
      const int co = (int)(t % Co); const int64_t n = t / Co;
      const int c = co / (s * s), i = (co / s) % s, j = co % s;
      y[o] = x[((n * C + c) * H + yo * s + i) * W + xo * s + j];
    }
  }
}

constexpr int L1_BLOCKS = 1024;

__global__ void l1_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                  float gscale, float* __restrict__ grad, float* __restrict__ partial) {
  __shared__ float red[256];
  float s = 0.f;
  const int64_t n4 = n / 4;
  const f32x4* a4 = (const f32x4*)a;
  const f32x4* b4 = (const f32x4*)b;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 d = a4[i] - b4[i];
    f32x4 g;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s += fabsf(d[k]);
      g[k] = d[k] > 0.f ? gscale : (d[k] < 0.f ? -gscale : 0.f);
    }
    if (grad) ((f32x4*)grad)[i] = g;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d = a[i] - b[i];
    s += fabsf(d);
    if (grad) grad[i] = d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void l1_final_kernel(const float* __restrict__ partial, int nb, float scale, float* loss) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (float)(red[0] * (double)scale);
}

__global__ void adam_ema_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, float* __restrict__ ema, int64_t n, float lr,
                                float beta1, float beta2, float eps, float bc1, float bc2, float decay,
                                float gscale) {
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    float mi = m[i], vi = v[i];
    mi = mi + (1.f - beta1) * (gi - mi);          // exp_avg.lerp_(grad, 1 - beta1)
    vi = vi * beta2 + (1.f - beta2) * gi * gi;    // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vi) / bc2s + eps;
    const float pi = p[i] - step_size * (mi / denom);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (ema) ema[i] = ema[i] * decay + pi * (1.f - decay);
  }
}

// Same update with the step-dependent scalars read from device memory, so one launch can be
// captured in a HIP graph and replayed: hyper = {step, lr, grad_scale}; adam_step_kernel
// increments step (one thread) ahead of the update.
__global__ void adam_step_kernel(float* hyper) {
  if (threadIdx.x == 0 && blockIdx.x == 0) hyper[0] += 1.f;
}

__global__ void adam_ema_dev_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                    float* __restrict__ v, float* __restrict__ ema, int64_t n,
                                    const float* __restrict__ hyper, float beta1, float beta2, float eps,
                                    float decay) {
  const float step = hyper[0], lr = hyper[1], gscale = hyper[2];
  const float bc1 = 1.f - powf(beta1, step), bc2 = 1.f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    float mi = m[i], vi = v[i];
    mi = mi + (1.f - beta1) * (gi - mi);
    vi = vi * beta2 + (1.f - beta2) * gi * gi;
    const float denom = sqrtf(vi) / bc2s + eps;
    const float pi = p[i] - step_size * (mi / denom);
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
    if (ema) ema[i] = ema[i] * decay + pi * (1.f - decay);
  }
}

// dz = alpha * dy * (y > 0 ? 1 : neg) with neg = 0 (ReLU) or slope (LeakyReLU); the sign of the
// activation output equals the sign of its input for both.  8 bf16 / 4 f32 per 16-byte access.
template <typename T>
__global__ void act_backward_kernel(const T* __restrict__ dy, const T* __restrict__ y, int64_t n, float neg,
                                    float alpha, T* __restrict__ out) {
  constexpr int PER = Elt<T>::PER16;
  const int64_t nv = n / PER;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    const u32x4 d = ((const u32x4*)dy)[i], yy = ((const u32x4*)y)[i];
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
      for (int k = 0; k < 4; ++k) {
        const float d0 = __uint_as_float(d[k]), y0 = __uint_as_float(yy[k]);
        o[k] = __float_as_uint(alpha * d0 * (y0 > 0.f ? 1.f : neg));
      }
    }
    ((u32x4*)out)[i] = o;
  }
  for (int64_t i = nv * PER + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d0 = Elt<T>::to_f(dy[i]), y0 = Elt<T>::to_f(y[i]);
    out[i] = Elt<T>::from_f(alpha * d0 * (y0 > 0.f ? 1.f : neg));
  }
}

// out[m][c] = x[m][c] * scale[m / HW] on a dense [M][C] map (C a multiple of the 16-B chunk):
// the per-sample factor of SwinIR stochastic depth applied to a residual-branch gradient.
template <typename T>
__global__ void row_scale_kernel(const T* __restrict__ x, const float* __restrict__ scale, uint32_t nv,
                                 FastDiv fd_vpr, FastDiv fd_hw, T* __restrict__ out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) {
    const float f = scale[fdiv(fdiv(i, fd_vpr), fd_hw)];
    const u32x4 d = ((const u32x4*)x)[i];
    u32x4 o;
    if constexpr (Elt<T>::PER16 == 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = pack_bf16x2(f * bf16_to_f32(d[k] & 0xffff), f * bf16_to_f32(d[k] >> 16));
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = __float_as_uint(f * __uint_as_float(d[k]));
    }
    ((u32x4*)out)[i] = o;
  }
}

inline unsigned grid_for(int64_t n, int64_t cap = 4096) {
  int64_t g = (n + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace

extern "C" {

int sr_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, int Cp, const float* shift,
                    const float* scale, void* y, void* stream) {
  if (!x || !y || Cp < C) return sr_fail(SR_EINVAL, "nchw_to_nhwc: bad arguments");
  const int64_t P = (int64_t)N * H * W;
  hipStream_t s = (hipStream_t)stream;
  const int64_t HW = (int64_t)H * W;
  if (C >= 16 && N <= 65535 && HW % 4 == 0 && Cp % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((Cp + 63) / 64), (unsigned)N);
    if (dtype == SR_BF16)
      hipLaunchKernelGGL(nchw_to_nhwc_vec_kernel<bf16_t>, grid, dim3(256), 0, s, x, C, HW, Cp, shift, scale,
                         (bf16_t*)y);
    else
      hipLaunchKernelGGL(nchw_to_nhwc_vec_kernel<float>, grid, dim3(256), 0, s, x, C, HW, Cp, shift, scale,
                         (float*)y);
    return sr_check(hipGetLastError(), "nchw_to_nhwc launch");
  }
  if (C >= 16 && N <= 65535) {
    const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((Cp + 31) / 32), (unsigned)N);
    if (dtype == SR_BF16)
      hipLaunchKernelGGL(nchw_to_nhwc_tiled_kernel<bf16_t>, grid, dim3(256), 0, s, x, C, HW, Cp, shift, scale,
                         (bf16_t*)y);
    else
      hipLaunchKernelGGL(nchw_to_nhwc_tiled_kernel<float>, grid, dim3(256), 0, s, x, C, HW, Cp, shift, scale,
                         (float*)y);
    return sr_check(hipGetLastError(), "nchw_to_nhwc launch");
  }
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, x,
                       N, C, H, W, Cp, shift, scale, (bf16_t*)y);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, x, N,
                       C, H, W, Cp, shift, scale, (float*)y);
  return sr_check(hipGetLastError(), "nchw_to_nhwc launch");
}

int sr_nhwc_to_nchw(int dtype, const void* x, int N, int H, int W, int ld, int coff, int C,
                    const float* scale, const float* shift, float* y, void* stream) {
  if (!x || !y || ld < coff + C) return sr_fail(SR_EINVAL, "nhwc_to_nchw: bad arguments");
  const int64_t P = (int64_t)N * H * W;
  hipStream_t s = (hipStream_t)stream;
  if (C >= 16 && N <= 65535) {
    const int64_t HW = (int64_t)H * W;
    const dim3 grid((unsigned)((HW + 63) / 64), (unsigned)((C + 31) / 32), (unsigned)N);
    if (dtype == SR_BF16)
      hipLaunchKernelGGL(nhwc_to_nchw_tiled_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, HW, ld, coff,
                         C, scale, shift, y);
    else
      hipLaunchKernelGGL(nhwc_to_nchw_tiled_kernel<float>, grid, dim3(256), 0, s, (const float*)x, HW, ld, coff, C,
                         scale, shift, y);
    return sr_check(hipGetLastError(), "nhwc_to_nchw launch");
  }
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16_t>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s,
                       (const bf16_t*)x, N, H, W, ld, coff, C, scale, shift, y);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s,
                       (const float*)x, N, H, W, ld, coff, C, scale, shift, y);
  return sr_check(hipGetLastError(), "nhwc_to_nchw launch");
}

int sr_pixel_shuffle_nchw(int dtype, const void* x, int N, int C, int H, int W, int r, void* y,
                          void* stream) {
  if (!x || !y || r == 0) return sr_fail(SR_EINVAL, "pixel_shuffle: bad arguments");
  if (r > 0 && C % (r * r)) return sr_fail(SR_EINVAL, "pixel_shuffle: C not divisible by r^2");
  if (r < 0 && (H % (-r) || W % (-r))) return sr_fail(SR_EINVAL, "pixel_unshuffle: H/W not divisible by s");
  const int64_t total = (int64_t)N * C * H * W;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(pixel_shuffle_kernel<bf16_t>, dim3(grid_for(total, 8192)), dim3(256), 0, s,
                       (const bf16_t*)x, N, C, H, W, r, (bf16_t*)y);
  else
    hipLaunchKernelGGL(pixel_shuffle_kernel<float>, dim3(grid_for(total, 8192)), dim3(256), 0, s,
                       (const float*)x, N, C, H, W, r, (float*)y);
  return sr_check(hipGetLastError(), "pixel_shuffle launch");
}

size_t sr_l1_loss_workspace(int64_t n) {
  (void)n;
  return L1_BLOCKS * sizeof(float);
}

int sr_l1_loss(const float* pred, const float* gt, int64_t n, float weight, int mean, float* loss,
               float* grad, void* workspace, size_t ws_bytes, void* stream) {
  if (!pred || !gt || !loss || !workspace || n <= 0) return sr_fail(SR_EINVAL, "l1_loss: bad arguments");
  if (ws_bytes < sr_l1_loss_workspace(n)) return sr_fail(SR_EINVAL, "l1_loss: workspace too small");
  if (((uintptr_t)pred | (uintptr_t)gt | (uintptr_t)grad) & 15)
    return sr_fail(SR_EINVAL, "l1_loss: tensors must be 16-byte aligned");
  const float norm = mean ? (float)n : 1.f;
  const unsigned nb = grid_for(n / 4 + 1, L1_BLOCKS);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(l1_partial_kernel, dim3(nb), dim3(256), 0, s, pred, gt, n, weight / norm, grad,
                     (float*)workspace);
  hipLaunchKernelGGL(l1_final_kernel, dim3(1), dim3(256), 0, s, (const float*)workspace, (int)nb,
                     weight / norm, loss);
  return sr_check(hipGetLastError(), "l1_loss launch");
}

int sr_adam_ema(float* p, const float* g, float* m, float* v, float* ema, int64_t n, float lr, float beta1,
                float beta2, float eps, float bc1, float bc2, float ema_decay, float grad_scale, void* stream) {
  if (!p || !g || !m || !v || n <= 0) return sr_fail(SR_EINVAL, "adam_ema: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_ema_kernel, dim3(grid_for(n, 8192)), dim3(256), 0, s, p, g, m, v, ema, n, lr,
                     beta1, beta2, eps, bc1, bc2, ema_decay, grad_scale);
  return sr_check(hipGetLastError(), "adam_ema launch");
}

int sr_adam_ema_dev(float* p, const float* g, float* m, float* v, float* ema, int64_t n, float* hyper, float beta1,
                    float beta2, float eps, float ema_decay, void* stream) {
  if (!p || !g || !m || !v || !hyper || n <= 0) return sr_fail(SR_EINVAL, "adam_ema_dev: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_step_kernel, dim3(1), dim3(64), 0, s, hyper);
  hipLaunchKernelGGL(adam_ema_dev_kernel, dim3(grid_for(n, 8192)), dim3(256), 0, s, p, g, m, v, ema, n, hyper, beta1,
                     beta2, eps, ema_decay);
  return sr_check(hipGetLastError(), "adam_ema_dev launch");
}

int sr_act_backward(int dtype, const void* dy, const void* y, int64_t n, int act, float slope, float alpha,
                    void* out, void* stream) {
  if (!dy || !y || !out || n < 0) return sr_fail(SR_EINVAL, "act_backward: bad arguments");
  if (((uintptr_t)dy | (uintptr_t)y | (uintptr_t)out) & 15)
    return sr_fail(SR_EINVAL, "act_backward: tensors must be 16-byte aligned");
  const float neg = act == SR_ACT_LRELU ? slope : (act == SR_ACT_RELU ? 0.f : 1.f);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(act_backward_kernel<bf16_t>, dim3(grid_for(n / 8 + 1, 8192)), dim3(256), 0, s,
                       (const bf16_t*)dy, (const bf16_t*)y, n, neg, alpha, (bf16_t*)out);
  else
    hipLaunchKernelGGL(act_backward_kernel<float>, dim3(grid_for(n / 4 + 1, 8192)), dim3(256), 0, s,
                       (const float*)dy, (const float*)y, n, neg, alpha, (float*)out);
  return sr_check(hipGetLastError(), "act_backward launch");
}

int sr_row_scale(int dtype, const void* x, int64_t M, int C, int HW, const float* scale, void* out, void* stream) {
  const int PER = dtype == SR_BF16 ? 8 : 4;
  if (!x || !scale || !out || M < 0 || C <= 0 || HW <= 0 || C % PER || M % HW)
    return sr_fail(SR_EINVAL, "row_scale: bad arguments (C must be a multiple of the 16-B chunk, M of HW)");
  if (((uintptr_t)x | (uintptr_t)out) & 15) return sr_fail(SR_EINVAL, "row_scale: tensors must be 16-byte aligned");
  const int64_t nv = M * C / PER;
  if (nv >= 0x80000000ll) return sr_fail(SR_ETOOBIG, "row_scale: tensor too large");
  if (nv == 0) return SR_OK;
  hipStream_t s = (hipStream_t)stream;
  const FastDiv fv = make_fastdiv((uint32_t)(C / PER)), fh = make_fastdiv((uint32_t)HW);
  if (dtype == SR_BF16)
    hipLaunchKernelGGL(row_scale_kernel<bf16_t>, dim3(grid_for(nv, 8192)), dim3(256), 0, s, (const bf16_t*)x, scale,
                       (uint32_t)nv, fv, fh, (bf16_t*)out);
  else
    hipLaunchKernelGGL(row_scale_kernel<float>, dim3(grid_for(nv, 8192)), dim3(256), 0, s, (const float*)x, scale,
                       (uint32_t)nv, fv, fh, (float*)out);
  return sr_check(hipGetLastError(), "row_scale launch");
}

}  // extern "C"
