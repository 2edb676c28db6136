// Microbenchmark: cycles per v_mfma_f32_16x16x32_bf16 at one wave per SIMD, 36 independent
// AGPR accumulators (the row-streaming wgrad's inner form), random bf16 operands.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

template <int NACC>
__global__ __launch_bounds__(256, 1) void k(const s16x8* in, float* out, unsigned long long* cyc, int iters) {
  const int tid = threadIdx.x;
  s16x8 a = in[tid], b = in[(tid + 64) & 255];
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i]) : "v"(a), "v"(b));
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const unsigned long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  s16x8* in; float* out; unsigned long long* cyc;
  (void)hipMalloc(&in, 256 * sizeof(s16x8)); (void)hipMalloc(&out, 1024 * 256 * 4); (void)hipMalloc(&cyc, 1024 * 8);
  std::vector<short> h(256 * 8);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (short)(0x3f00 + (i * 37 % 200));
  hipMemcpy(in, h.data(), h.size() * 2, hipMemcpyHostToDevice);
  const int iters = 2000;
  for (int grid : {256, 1024}) {
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k<36>, dim3(grid), dim3(256), 0, 0, in, out, cyc, iters);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<36>, dim3(grid), dim3(256), 0, 0, in, out, cyc, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(256);
    hipMemcpy(c.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : c) avg += v; avg /= 256;
    const double n = 36.0 * iters;
    const double fl = 2.0 * 16 * 16 * 32 * n * 4 * grid;  // 4 waves per block
    printf("grid %d: %.2f cyc/mfma (s_memtime), kernel %.3f ms, %.1f TF/s, implied clock %.2f GHz\n", grid, avg / n, ms,
           fl / ms / 1e9, avg / (ms * 1e-3) / 1e9 * (grid > 256 ? 256.0 / grid : 1.0));
  }
  return 0;
}
