// tools/ubench_sqrt2.hip -- cheaper correctly rounded fp32 square roots for the
// candidate roots?  Exhaustive check, over every
// non-negative finite fp32 input, of two candidates against the correctly
// rounded sqrt, then their issue cost at full occupancy:
//   f64:   (float) v_sqrt_f64((double) x)          (3 VALU)
//   rsqnr: y = v_rsq_f32(x); s = x y; s + (x - s^2) y/2   (5 VALU, x > 0 only)
//   cur:   v_sqrt_f32 + the two-residual correction (the kernel's sqrt before round 2's end, 9 VALU)
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_sqrt2 tools/ubench_sqrt2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float m_f64(float x) { return (float)__builtin_amdgcn_sqrt((double)x); }
__device__ __forceinline__ float m_rsqnr(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y, hy = 0.5f * y;
  const float r = fmaf(-s, s, x);
  return fmaf(r, hy, s);
}
__device__ __forceinline__ float m_cur(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const uint32_t b = __float_as_uint(s);
  const float sd = __uint_as_float(b - 1u), su = __uint_as_float(b + 1u);
  const float rd = fmaf(-sd, s, x), ru = fmaf(-su, s, x);
  float o = rd <= 0.0f ? sd : s;
  return ru > 0.0f ? su : o;
}
// correctly rounded: the fp64 sqrt (OCML, correctly rounded) of an fp32 is
// never a double-rounding tie for fp32
__device__ __forceinline__ float cr_sqrt(float x) { return (float)__builtin_sqrt((double)x); }

template <int M>
__device__ __forceinline__ float meth(float x) {
  return M == 0 ? m_f64(x) : M == 1 ? m_rsqnr(x) : m_cur(x);
}

template <int M>
__global__ void check(uint32_t lo, uint32_t hi, unsigned long long *bad, uint32_t *first) {
  unsigned long long nb = 0;
  uint32_t f = 0xffffffffu;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)b);
    if (__float_as_uint(meth<M>(x)) != __float_as_uint(cr_sqrt(x))) {
      ++nb;
      if ((uint32_t)b < f) f = (uint32_t)b;
    }
  }
  atomicAdd(bad, nb);
  atomicMin(first, f);
}

template <int M>
__global__ __launch_bounds__(256) void rate(float *out, int iters, float b) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 1.0f + threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = meth<M>(a[k]) + b;  // +b keeps the chain and the value in range
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  unsigned long long *bad;
  uint32_t *first;
  float *out;
  hipMalloc(&bad, 8);
  hipMalloc(&first, 4);
  const int blocks = 256 * 8 * 4, threads = 256, iters = 2000;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  const char *names[] = {"f64", "rsqnr", "cur"};
  const uint32_t ranges[][2] = {{0x00000000u, 0x7f800000u}, {0x00800000u, 0x7f800000u}, {0x0f800000u, 0x7f800000u}};
  for (int m = 0; m < 3; ++m) {
    for (auto &r : ranges) {
      hipMemset(bad, 0, 8);
      hipMemset(first, 0xff, 4);
      if (m == 0) check<0><<<8192, 256>>>(r[0], r[1], bad, first);
      if (m == 1) check<1><<<8192, 256>>>(r[0], r[1], bad, first);
      if (m == 2) check<2><<<8192, 256>>>(r[0], r[1], bad, first);
      unsigned long long hb;
      uint32_t hf;
      hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
      hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
      float fx;
      memcpy(&fx, &hf, 4);
      printf("%-6s inputs [0x%08x, 0x%08x): %llu mismatches (first 0x%08x = %.9g)\n", names[m], r[0], r[1], hb,
             hf, hb ? fx : 0.0f);
    }
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    for (int m = 0; m < 3; ++m) {
      hipEventRecord(e0);
      if (m == 0) rate<0><<<blocks, threads>>>(out, iters, 1e-3f);
      if (m == 1) rate<1><<<blocks, threads>>>(out, iters, 1e-3f);
      if (m == 2) rate<2><<<blocks, threads>>>(out, iters, 1e-3f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double wave_ops = (double)blocks * threads / 64 * iters * 8;
      if (rep == 1) printf("%-6s %8.3f ms  %.3f ns per wave sqrt per SIMD\n", names[m], ms, ms * 1e6 / (wave_ops / 1024));
    }
  }
  return 0;
}
