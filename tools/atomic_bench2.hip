// Microbenchmark: LDS integer atomics and global fp32 atomics (coalesced vs scattered) on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ void __launch_bounds__(256) lds_k(unsigned long long* out, int iters) {
  __shared__ unsigned long long acc64[8192];
  unsigned* acc32 = (unsigned*)acc64;
  for (int i = threadIdx.x; i < 8192; i += 256) acc64[i] = 0;
  __syncthreads();
  const int idx = threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) atomicAdd(&acc32[(idx * 17 + it) & 16383], (unsigned)it);
    else atomicAdd(&acc64[(idx * 17 + it) & 8191], (unsigned long long)it);
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = acc64[threadIdx.x];
}

template <int MODE>
__global__ void __launch_bounds__(256) glb_k(float* buf, int iters, int n) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    int64_t a;
    if (MODE == 0) a = (t + (int64_t)it * 65536 * 4) % n;              // coalesced, 64 consecutive floats / wave
    else a = ((t * 2654435761ull) + it * 97ull) % (unsigned long long)n;  // scattered
    unsafeAtomicAdd(buf + a, 1.0f);
  }
}

int main() {
  unsigned long long* out;
  float* buf;
  const int n = 64 << 20;
  hipMalloc(&out, 2048 * 256 * 8);
  hipMalloc(&buf, (size_t)n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float ms;
  for (int m = 0; m < 2; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(lds_k<0>, dim3(2048), dim3(256), 0, 0, out, 4096);
      else hipLaunchKernelGGL(lds_k<1>, dim3(2048), dim3(256), 0, 0, out, 4096);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("lds %s  %.3f ms  %.2f lane-ops/clk/CU\n", m ? "u64" : "u32", ms,
           2048.0 * 256 * 4096 / (ms * 1e-3) / 256 / 2.4e9);
  }
  for (int m = 0; m < 2; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(glb_k<0>, dim3(4096), dim3(256), 0, 0, buf, 64, n);
      else hipLaunchKernelGGL(glb_k<1>, dim3(4096), dim3(256), 0, 0, buf, 64, n);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    hipEventElapsedTime(&ms, a, b);
    printf("global f32 %s  %.3f ms  %.2f G lane-atomics/s\n", m ? "scattered" : "coalesced", ms,
           4096.0 * 256 * 64 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
