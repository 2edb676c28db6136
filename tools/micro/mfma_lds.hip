// Microbenchmark: cycles per v_mfma_f32_16x16x32_bf16 at one wave per SIMD (4 waves / block,
// 256 blocks) with LDS fragment reads interleaved: none / ds_read_b64_tr_b16 / ds_read_b128,
// reads feeding the next round's operands (so they must land), 36 AGPR accumulators.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 65536 / 4; i += 256) ((int*)lds)[i] = 0x3f003f00 + (i & 255);
  __syncthreads();
  s16x8 fa[4], fb[9];
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[i] = *(const s16x8*)(lds + (i * 1024 + lane * 16));
#pragma unroll
  for (int i = 0; i < 9; ++i) fb[i] = *(const s16x8*)(lds + (8192 + i * 1024 + lane * 16));
  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[t][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* base = lds + (tid >> 6) * 16384;
  s16x8 fn[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) fn[i] = fb[i];
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (MODE == 1) {  // 2 tr reads per tap group (as the wgrad: 26 per 36 MFMAs ~ 1.44 ops/group)
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + ((t * 64 + lane) & 511) * 32));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + ((t * 64 + lane + 8) & 511) * 32));
          fb[t] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else if (MODE == 2) {
          fb[t] = *(const s16x8*)(base + ((t * 64 + lane) & 1023) * 16);
        }
        if (MODE >= 3) {  // tr read for group t + LA (LA = MODE - 2 groups ahead, ring of 9)
          constexpr int LA = MODE - 2;
          const int tn = (t + LA) % 9;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + ((tn * 64 + lane) & 511) * 32));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s16x4*)(base + ((tn * 64 + lane + 8) & 511) * 32));
          fn[tn] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[t][c]) : "v"(fa[c]), "v"(MODE >= 3 ? fn[t] : fb[t]));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  const unsigned long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) s += acc[t][c][0] + acc[t][c][3];
  out[blockIdx.x * 256 + tid] = s;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(float* out, unsigned long long* cyc) {
  const int iters = 200;
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
  hipDeviceSynchronize();
  std::vector<unsigned long long> c(256);
  (void)hipMemcpy(c.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : c) avg += v;
  avg /= 256;
  printf("mode %d: %.2f cyc/mfma\n", MODE, avg / (72.0 * iters));
}

int main() {
  float* out; unsigned long long* cyc;
  (void)hipMalloc(&out, 256 * 256 * 4); (void)hipMalloc(&cyc, 256 * 8);
  run<0>(out, cyc); run<1>(out, cyc); run<2>(out, cyc); run<3>(out, cyc); run<5>(out, cyc); run<8>(out, cyc);
  return 0;
}
