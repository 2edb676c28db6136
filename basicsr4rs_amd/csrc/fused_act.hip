// fused_bias_act (StyleGAN2 FusedLeakyReLU) for gfx950.
//
//   sr_fused_bias_act : the reference op (basicsr/ops/fused_act/src/fused_bias_act_kernel.cu,
//       fused_bias_act_op): y = scale * act(x + b[(i / step_b) % size_b]) for act 1
//       (linear) / 3 (leaky relu with `alpha`), grad 0 (value), 1 (first derivative, gated
//       by `ref` > 0) or 2 (second derivative = 0).  16-byte vectors whenever a vector
//       never straddles a bias-channel boundary.
//   sr_fused_lrelu_bwd : FusedLeakyReLUFunctionBackward.forward (fused_act.py:30-44) as one
//       pass: dx = fused_bias_act(dy, -, out, 3, 1) and grad_bias = dx summed over every
//       dim but 1, with a deterministic two-level reduction (no atomics).
#include "sr_common.h"
#include "sr_internal.h"
#include <algorithm>

namespace {

SR_DEV float fba(float x, float ref, int mode, float alpha, float scale) {
  float y;
  switch (mode) {
    default:
    case 10: y = x; break;
    case 11: y = x; break;
    case 12: y = 0.f; break;
    case 30: y = (x > 0.f) ? x : x * alpha; break;
    case 31: y = (ref > 0.f) ? x : x * alpha; break;
    case 32: y = 0.f; break;
  }
  return y * scale;
}

template <typename T, int V>
__global__ void __launch_bounds__(256) fused_bias_act_kernel(const T* __restrict__ x, const T* __restrict__ b,
                                                             const T* __restrict__ ref, T* __restrict__ out,
                                                             int64_t nvec, FastDiv fstep, int size_b, int mode,
                                                             float alpha, float scale) {
  for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i0 = v * V;
    float bias = 0.f;
    if (b) {
      // size_x < 2^31 is enforced by the host (the reference indexes with int)
      const uint32_t q = fdiv((uint32_t)i0, fstep);
      bias = Elt<T>::to_f(b[q % (uint32_t)size_b]);
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float xv = Elt<T>::to_f(x[i0 + e]) + bias;
      const float rv = ref ? Elt<T>::to_f(ref[i0 + e]) : 0.f;
      out[i0 + e] = Elt<T>::from_f(fba(xv, rv, mode, alpha, scale));
    }
  }
}

// Layout [R][C][S]: block (c, part) handles rows [r0, r1) of channel c, S contiguous values
// each; dx written, the block's partial bias gradient stored in ws[c * parts + part].
template <typename T>
__global__ void __launch_bounds__(256) lrelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ out,
                                                        T* __restrict__ dx, int R, int C, int64_t S, int parts,
                                                        float alpha, float scale, float* __restrict__ ws) {
  const int c = blockIdx.x / parts, part = blockIdx.x - c * parts;
  const int r0 = (int)((int64_t)R * part / parts), r1 = (int)((int64_t)R * (part + 1) / parts);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r) {
    const int64_t base = ((int64_t)r * C + c) * S;
    for (int64_t s = threadIdx.x; s < S; s += blockDim.x) {
      const int64_t i = base + s;
      const float g = fba(Elt<T>::to_f(dy[i]), Elt<T>::to_f(out[i]), 31, alpha, scale);
      const T gq = Elt<T>::from_f(g);
      dx[i] = gq;
      acc += Elt<T>::to_f(gq);
    }
  }
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) ws[blockIdx.x] = red[0];
}

// Small-S variant (S < 64, e.g. [N, C] EqualLinear outputs): one thread per (c, part),
// adjacent threads own adjacent channels so row reads stay contiguous.
template <typename T>
__global__ void __launch_bounds__(256) lrelu_bwd_small_kernel(const T* __restrict__ dy, const T* __restrict__ out,
                                                              T* __restrict__ dx, int R, int C, int64_t S, int parts,
                                                              float alpha, float scale, float* __restrict__ ws) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)C * parts) return;
  const int part = (int)(t / C), c = (int)(t - (int64_t)part * C);
  const int r0 = (int)((int64_t)R * part / parts), r1 = (int)((int64_t)R * (part + 1) / parts);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r)
    for (int64_t s = 0; s < S; ++s) {
      const int64_t i = ((int64_t)r * C + c) * S + s;
      const float g = fba(Elt<T>::to_f(dy[i]), Elt<T>::to_f(out[i]), 31, alpha, scale);
      const T gq = Elt<T>::from_f(g);
      dx[i] = gq;
      acc += Elt<T>::to_f(gq);
    }
  ws[(int64_t)c * parts + part] = acc;
}

__global__ void bias_reduce_kernel(const float* __restrict__ ws, int C, int parts, float* __restrict__ db) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < parts; ++p) s += ws[(int64_t)c * parts + p];
  db[c] = s;
}

int bwd_parts(int R, int C, int64_t S) {
  if (S < 64) return std::max(1, std::min(R, (1 << 16) / std::max(C, 1)));
  const int64_t per_c = (int64_t)R * S;
  int parts = (int)std::max<int64_t>(1, std::min<int64_t>(R, (2048 + C - 1) / C));
  while (parts > 1 && per_c / parts < 4096) parts >>= 1;
  return parts;
}

template <typename T>
int launch_fba(const void* x, const void* b, const void* ref, void* out, int64_t n, int step_b, int size_b, int mode,
               float alpha, float scale, hipStream_t s) {
  const FastDiv f = make_fastdiv((uint32_t)step_b);
  constexpr int V = Elt<T>::PER16;
  const bool vec = (n % V == 0) && (!b || step_b % V == 0);
  const int64_t nv = vec ? n / V : n;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nv + 255) / 256, 8192));
  if (vec)
    hipLaunchKernelGGL((fused_bias_act_kernel<T, V>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)b,
                       (const T*)ref, (T*)out, nv, f, size_b, mode, alpha, scale);
  else
    hipLaunchKernelGGL((fused_bias_act_kernel<T, 1>), dim3(grid), dim3(256), 0, s, (const T*)x, (const T*)b,
                       (const T*)ref, (T*)out, nv, f, size_b, mode, alpha, scale);
  return sr_check(hipGetLastError(), "fused_bias_act launch");
}

template <typename T>
int launch_bwd(const void* dy, const void* out, void* dx, float* db, int R, int C, int64_t S, float alpha, float scale,
               float* ws, hipStream_t s) {
  const int parts = bwd_parts(R, C, S);
  if (S < 64) {
    const int64_t th = (int64_t)C * parts;
    hipLaunchKernelGGL((lrelu_bwd_small_kernel<T>), dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s,
                       (const T*)dy, (const T*)out, (T*)dx, R, C, S, parts, alpha, scale, ws);
  } else {
    hipLaunchKernelGGL((lrelu_bwd_kernel<T>), dim3((unsigned)(C * parts)), dim3(256), 0, s, (const T*)dy,
                       (const T*)out, (T*)dx, R, C, S, parts, alpha, scale, ws);
  }
  if (db) hipLaunchKernelGGL(bias_reduce_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, C, parts, db);
  return sr_check(hipGetLastError(), "fused_lrelu_bwd launch");
}

}  // namespace

extern "C" {

int sr_fused_bias_act(int dtype, const void* x, const void* bias, const void* ref, void* out, int64_t size_x,
                      int step_b, int size_b, int act, int grad, float alpha, float scale, void* stream) {
  if (!x || !out) return sr_fail(SR_EINVAL, "fused_bias_act: null pointer");
  if (size_x < 0 || size_x >= (int64_t)1 << 31) return sr_fail(SR_EINVAL, "fused_bias_act: size out of int range");
  if (bias && (size_b <= 0 || step_b <= 0)) return sr_fail(SR_EINVAL, "fused_bias_act: bad bias geometry");
  if (size_x == 0) return SR_OK;
  const int mode = act * 10 + grad;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_F32) return launch_fba<float>(x, bias, ref, out, size_x, step_b, size_b, mode, alpha, scale, s);
  if (dtype == SR_BF16) return launch_fba<bf16_t>(x, bias, ref, out, size_x, step_b, size_b, mode, alpha, scale, s);
  return sr_fail(SR_EINVAL, "fused_bias_act: bad dtype");
}

size_t sr_fused_lrelu_bwd_workspace(int R, int C, int64_t S) {
  return (size_t)C * bwd_parts(R, C, S) * sizeof(float);
}

int sr_fused_lrelu_bwd(int dtype, const void* dy, const void* out, void* dx, float* grad_bias, int R, int C,
                       int64_t S, float alpha, float scale, void* workspace, size_t ws_bytes, void* stream) {
  if (!dy || !out || !dx) return sr_fail(SR_EINVAL, "fused_lrelu_bwd: null pointer");
  if (R <= 0 || C <= 0 || S <= 0) return sr_fail(SR_EINVAL, "fused_lrelu_bwd: empty tensor");
  if (ws_bytes < sr_fused_lrelu_bwd_workspace(R, C, S) || !workspace)
    return sr_fail(SR_EINVAL, "fused_lrelu_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_F32) return launch_bwd<float>(dy, out, dx, grad_bias, R, C, S, alpha, scale, (float*)workspace, s);
  if (dtype == SR_BF16) return launch_bwd<bf16_t>(dy, out, dx, grad_bias, R, C, S, alpha, scale, (float*)workspace, s);
  return sr_fail(SR_EINVAL, "fused_lrelu_bwd: bad dtype");
}

}  // extern "C"
