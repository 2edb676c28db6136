// Microbenchmark: ds_add_f32 throughput on gfx950 for several lane->address patterns.
// build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_bench.hip -o /tmp/ldsab
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int MODE>
__global__ void __launch_bounds__(256) k(float* out, int iters, int stride) {
  __shared__ float acc[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float v = 1.0f + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
    int addr;
    if (MODE == 0) addr = (wave * 64 + lane) & 16383;                     // consecutive
    else if (MODE == 1) addr = (wave * 1024 + lane * stride + it) & 16383;  // strided
    else addr = wave * 4;                                                  // all lanes same address
    if (MODE == 3) { acc[addr] += v; } else { atomicAdd(&acc[addr], v); }
    v += 1.f;
  }
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = acc[threadIdx.x];
}

int main() {
  float* out;
  hipMalloc(&out, 1024 * 256 * 4 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 4096, blocks = 2048;
  const char* names[] = {"consecutive", "stride17", "stride16", "same-addr", "plain add (non-atomic)"};
  for (int m = 0; m < 5; ++m) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(a);
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 17);
      if (m == 2) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 16);
      if (m == 3) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
      if (m == 4) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
      hipEventRecord(b);
      hipEventSynchronize(b);
    }
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)blocks * 256 * iters;
    printf("%-24s %8.3f ms  %.2f lane-atomics/clk/CU (256 CUs, 2.4 GHz)\n", names[m], ms,
           lane_ops / (ms * 1e-3) / 256 / 2.4e9);
  }
  return 0;
}
