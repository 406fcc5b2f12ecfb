// Exhaustive check of the hardware square root (v_sqrt_f32) against the
// correctly rounded one, over every positive normal fp32 input, and the same
// for v_rsq_f32 against round(1/sqrt(x)) -- is the 10-instruction sqrt_k
// correction ever needed?   hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float hw_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }

// correctly rounded sqrt of a positive normal float via fp64 (exact: a double
// holds sqrt(x) to 53 bits, and the 24-bit rounding of that is never a double
// rounding tie for fp32 inputs)
__device__ __forceinline__ float cr_sqrt(float x) { return (float)__builtin_sqrt((double)x); }

__global__ void check(uint32_t lo, uint32_t hi, unsigned long long *bad, uint32_t *first) {
  unsigned long long nb = 0;
  uint32_t f = 0xffffffffu;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)b);
    const float a = hw_sqrt(x), c = cr_sqrt(x);
    if (__float_as_uint(a) != __float_as_uint(c)) {
      ++nb;
      if ((uint32_t)b < f) f = (uint32_t)b;
    }
  }
  atomicAdd(bad, nb);
  atomicMin(first, f);
}

int main() {
  unsigned long long *bad;
  uint32_t *first;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 4);
  // ranges: all positive normals; and the kernel's clamped domain [2^-96, +inf)
  const uint32_t ranges[][2] = {{0x00800000u, 0x7f800000u}, {0x0f800000u, 0x7f800000u}, {0x3f800000u, 0x40800000u}};
  for (auto &r : ranges) {
    hipMemset(bad, 0, 8);
    hipMemset(first, 0xff, 4);
    check<<<8192, 256>>>(r[0], r[1], bad, first);
    unsigned long long hb;
    uint32_t hf;
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
    float fx;
    memcpy(&fx, &hf, 4);
    printf("v_sqrt_f32 vs correctly rounded, inputs [0x%08x, 0x%08x): %llu mismatches (first 0x%08x = %.9g)\n", r[0],
           r[1], hb, hf, hb ? fx : 0.0f);
  }
  return 0;
}
