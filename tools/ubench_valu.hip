// tools/ubench_valu.hip -- measures the fp32 VALU issue rates the scan kernel
// depends on: v_fma_f32 vs v_pk_fma_f32 (VGPR operands, and one SGPR-pair
// operand as the scan uses), at full occupancy.  Prints TFLOP/s per variant.
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__global__ __launch_bounds__(256) void k_fma(float *out, int iters, float b, float c) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(c));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk(float *out, int iters, float b, float c) {
  f2 a[8];
  f2 bb = {b, b}, cc = {c, c};
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = f2{threadIdx.x * 1e-3f + k, (float)k};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[k]) : "v"(bb), "v"(cc));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pk_s(float *out, int iters, f2 bb, float c) {
  f2 a[8];
  f2 cc = {c, c};
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = f2{threadIdx.x * 1e-3f + k, (float)k};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[k]) : "s"(bb), "v"(cc));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma_s(float *out, int iters, float b, float c) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[k]) : "s"(b), "v"(c));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// packed fp16 FMA (2 halves per lane): is it issued at the v_fma_f32 rate?
__global__ __launch_bounds__(256) void k_pk16(float *out, int iters, float b, float c) {
  h2 a[8];
  h2 bb = {(_Float16)b, (_Float16)b}, cc = {(_Float16)c, (_Float16)c};
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = h2{(_Float16)(threadIdx.x * 1e-3f + k), (_Float16)k};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f16 %0, %1, %2, %0" : "+v"(a[k]) : "v"(bb), "v"(cc));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += (float)a[k].x + (float)a[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_max3_f32 (the slab test's reduction)
__global__ __launch_bounds__(256) void k_max3(float *out, int iters, float b, float c) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(c));
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 20000;
  float *out;
  CHK(hipMalloc(&out, sizeof(float) * blocks * threads));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const double lanes = (double)blocks * threads;
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < 6; ++v) {
      CHK(hipEventRecord(e0));
      if (v == 0) k_fma<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      if (v == 1) k_fma_s<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      if (v == 2) k_pk<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      if (v == 3) k_pk_s<<<blocks, threads>>>(out, iters, f2{0.999f, 0.998f}, 1e-3f);
      if (v == 4) k_pk16<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      if (v == 5) k_max3<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double fl = lanes * iters * 8 * 2 * (v >= 2 && v <= 4 ? 2 : 1);
      const double instr = lanes / 64 * iters * 8;
      const char *nm[] = {"v_fma_f32 (vgpr)", "v_fma_f32 (sgpr)", "v_pk_fma_f32 (vgpr)", "v_pk_fma_f32 (sgpr pair)",
                          "v_pk_fma_f16 (vgpr)", "v_max3_f32 (2 flop/lane)"};
      if (rep == 1)
        std::printf("%-26s %8.3f ms  %7.1f TFLOP/s  %6.3f wave-instr/clk/CU @2.4GHz\n", nm[v], ms,
                    fl / ms / 1e9, instr / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
