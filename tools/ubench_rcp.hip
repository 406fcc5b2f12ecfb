// tools/ubench_rcp.hip -- is v_rcp_f32 + one Newton step, r + r (1 - q r), the
// correctly rounded reciprocal of every fp32 q?  Exhaustive over all 2^32 bit
// patterns (NaNs skipped) against the IEEE division 1.0f / q, then the issue
// cost of both forms (the refined root's second root).
//   hipcc --offload-arch=gfx950 -O3 -o rcpcheck tools/ubench_rcp.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ float rcp_nr(float q) {
  const float r = __builtin_amdgcn_rcpf(q);
  return fmaf(fmaf(-q, r, 1.0f), r, r);
}

__global__ void check(uint64_t lo, uint64_t hi, unsigned long long *bad, uint32_t *first,
                      unsigned long long *bad_normal) {
  unsigned long long nb = 0, nn = 0;
  uint32_t f = 0xffffffffu;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const float q = __uint_as_float((uint32_t)b);
    if (q != q) continue;
    const float a = rcp_nr(q);
    const float c = 1.0f / q;
    if (__float_as_uint(a) != __float_as_uint(c)) {
      ++nb;
      const uint32_t e = ((uint32_t)b >> 23) & 0xffu;
      if (e >= 1 && e <= 252) ++nn;  // normal q whose reciprocal is normal too
      if ((uint32_t)b < f) f = (uint32_t)b;
    }
  }
  atomicAdd(bad, nb);
  atomicAdd(bad_normal, nn);
  atomicMin(first, f);
}

template <int M>
__global__ __launch_bounds__(256) void rate(float *out, int iters, float b) {
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 1.5f + threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (M == 0 ? rcp_nr(a[k]) : 1.0f / a[k]) + b;
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  unsigned long long *bad, *badn;
  uint32_t *first;
  float *out;
  const int blocks = 256 * 8 * 4, threads = 256, iters = 2000;
  if (hipMalloc(&bad, 8) || hipMalloc(&badn, 8) || hipMalloc(&first, 4) ||
      hipMalloc(&out, sizeof(float) * blocks * threads))
    return 1;
  const uint64_t ranges[][2] = {{0x00000000ull, 0x80000000ull}, {0x80000000ull, 0x100000000ull}};
  for (auto &r : ranges) {
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(badn, 0, 8);
    (void)hipMemset(first, 0xff, 4);
    check<<<8192, 256>>>(r[0], r[1], bad, first, badn);
    unsigned long long hb, hn;
    uint32_t hf;
    if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost) || hipMemcpy(&hn, badn, 8, hipMemcpyDeviceToHost) ||
        hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost))
      return 1;
    float fx;
    memcpy(&fx, &hf, 4);
    printf("rcp+Newton vs 1.0f/q, q bits [0x%09llx, 0x%09llx): %llu mismatches, %llu with q and 1/q normal "
           "(first 0x%08x = %.9g)\n", (unsigned long long)r[0], (unsigned long long)r[1], hb, hn, hf,
           hb ? fx : 0.0f);
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char *names[] = {"rcp+Newton", "1.0f/q (IEEE)"};
  for (int rep = 0; rep < 2; ++rep) {
    for (int m = 0; m < 2; ++m) {
      (void)hipEventRecord(e0);
      if (m == 0) rate<0><<<blocks, threads>>>(out, iters, 1e-3f);
      if (m == 1) rate<1><<<blocks, threads>>>(out, iters, 1e-3f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double wave_ops = (double)blocks * threads / 64 * iters * 8;
      if (rep == 1) printf("%-14s %8.3f ms  %.3f ns per wave op per SIMD\n", names[m], ms, ms * 1e6 / (wave_ops / 1024));
    }
  }
  return 0;
}
