// tools/ubench_exec.hip -- does a wave64 VALU instruction cost less when one
// 32-lane half of EXEC is zero?  Times a chain of independent v_fma_f32 with
// EXEC = all 64 lanes, lanes 0-31, lanes 0-15, one lane.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void k(float *out, int iters, float b, float c, int active) {
  const int lane = threadIdx.x & 63;
  float a[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) a[q] = lane * 1e-3f + q;
  if (lane < active) {
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int q = 0; q < 8; ++q) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[q]) : "v"(b), "v"(c));
    }
  }
  float s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += a[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 20000;
  float *out;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int acts[] = {64, 32, 16, 1, 33};
  for (int rep = 0; rep < 2; ++rep)
    for (int act : acts) {
      hipEventRecord(e0);
      k<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f, act);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) std::printf("active lanes %2d: %8.3f ms  (%.3f ns per wave-instr per SIMD)\n", act, ms,
                           ms * 1e6 / ((double)blocks * 4 / 1024 * iters * 8));
    }
  return 0;
}
