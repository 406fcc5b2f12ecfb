// tools/ubench_rates.hip -- issue rate of single VALU instructions on gfx950 at
// full occupancy (8 independent chains per lane, 8 waves per SIMD).  Prints
// wave-instructions per clock per CU at 2.4 GHz (4 SIMDs: 4.0 would be one
// instruction per SIMD per clock).  Used to choose the slab test's instruction
// mix.
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_rates tools/ubench_rates.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define KERN(name, T, INIT, ASM, CONS)                                                \
  __global__ __launch_bounds__(256) void name(float *out, int iters, float b, float c) { \
    T a[8];                                                                           \
    T bb = INIT(b), cc = INIT(c);                                                     \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) a[k] = INIT(threadIdx.x * 1e-3f + k); \
    for (int i = 0; i < iters; ++i) {                                                 \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ASM : "+v"(a[k]) : CONS(bb), "v"(cc)); \
    }                                                                                 \
    float s = 0;                                                                      \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) s += sum(a[k]);                     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                   \
  }

__device__ __forceinline__ float sum(float x) { return x; }
__device__ __forceinline__ float sum(f2 x) { return x.x + x.y; }
__device__ __forceinline__ float sum(int x) { return (float)x; }
#define F1(x) (float)(x)
#define F2(x) f2{(float)(x), (float)(x)}
#define I1(x) (int)(x)
#define V(x) "v"(x)
#define S(x) "s"(x)

KERN(k_fma, float, F1, "v_fma_f32 %0, %1, %2, %0", V)
KERN(k_fma_s, float, F1, "v_fma_f32 %0, %1, %2, %0", S)
KERN(k_fmac, float, F1, "v_fmac_f32 %0, %1, %2", V)
KERN(k_add, float, F1, "v_add_f32 %0, %1, %0", V)
KERN(k_mul, float, F1, "v_mul_f32 %0, %1, %0", V)
KERN(k_sub_s, float, F1, "v_sub_f32 %0, %1, %0", S)
KERN(k_max, float, F1, "v_max_f32 %0, %1, %0", V)
KERN(k_max_s, float, F1, "v_max_f32 %0, %1, %0", S)
KERN(k_max3, float, F1, "v_max3_f32 %0, %1, %2, %0", V)
KERN(k_med3, float, F1, "v_med3_f32 %0, %1, %2, %0", V)
KERN(k_pkfma, f2, F2, "v_pk_fma_f32 %0, %1, %2, %0", V)
KERN(k_pkfma_s, f2, F2, "v_pk_fma_f32 %0, %1, %2, %0", S)
KERN(k_pkmul, f2, F2, "v_pk_mul_f32 %0, %1, %0", V)
KERN(k_pkadd, f2, F2, "v_pk_add_f32 %0, %1, %0", V)
KERN(k_addu, int, I1, "v_add_u32 %0, %1, %0", V)
KERN(k_xor, int, I1, "v_xor_b32 %0, %1, %0", V)
KERN(k_mullo, int, I1, "v_mul_lo_u32 %0, %1, %0", V)
KERN(k_cndmask, float, F1, "v_cmp_lt_f32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %2, vcc", V)
KERN(k_sqrt, float, F1, "v_sqrt_f32 %0, %0", V)
KERN(k_and, int, I1, "v_and_b32 %0, %1, %0", V)
KERN(k_lshr, int, I1, "v_lshrrev_b32 %0, %1, %0", V)
KERN(k_ashr, int, I1, "v_ashrrev_i32 %0, %1, %0", V)
KERN(k_bfi, int, I1, "v_bfi_b32 %0, %1, %2, %0", V)
KERN(k_add3, int, I1, "v_add3_u32 %0, %1, %2, %0", V)
KERN(k_lshladd, int, I1, "v_lshl_add_u32 %0, %0, 1, %1", V)
KERN(k_madu24, int, I1, "v_mad_u32_u24 %0, %1, %2, %0", V)
KERN(k_subf, float, F1, "v_sub_f32 %0, %1, %0", V)
KERN(k_fmak, float, F1, "v_fmaak_f32 %0, %1, %0, 0x3f000000", V)
KERN(k_cvt, float, F1, "v_cvt_f32_u32 %0, %0", V)
// v_cmp alone (writes an SGPR pair) and v_cndmask alone (reads one)
__global__ __launch_bounds__(256) void k_cmp(float *out, int iters, float b, float c) {
  float a[8];
  unsigned long long m = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
    _Pragma("unroll") for (int k = 0; k < 8; ++k) {
      unsigned long long r;
      asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(r) : "v"(a[k]), "v"(b));
      m ^= r;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(m & 1) + a[0];
}
__global__ __launch_bounds__(256) void k_cnd(float *out, int iters, float b, float c) {
  float a[8];
  const unsigned long long m = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
  _Pragma("unroll") for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  for (int i = 0; i < iters; ++i) {
    _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(c), "s"(m));
  }
  float s = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
// v_mad_u64_u32 (the compiler's choice for pcg4d's x += y * w): 64-bit accumulators
__global__ __launch_bounds__(256) void k_mad64(float *out, int iters, float b, float c) {
  unsigned long long a[8];
  unsigned bb = (unsigned)(b * 1e6f);
  _Pragma("unroll") for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 7u + k;
  for (int i = 0; i < iters; ++i) {
    _Pragma("unroll") for (int k = 0; k < 8; ++k) {
      unsigned long long cy;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[k]), "=s"(cy) : "v"((unsigned)a[k]), "v"(bb));
    }
  }
  float s = 0;
  _Pragma("unroll") for (int k = 0; k < 8; ++k) s += (float)(unsigned)a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
KERN(k_rcp, float, F1, "v_rcp_f32 %0, %0", V)

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

typedef void (*kfn)(float *, int, float, float);

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 10000;
  float *out;
  CHK(hipMalloc(&out, sizeof(float) * blocks * threads));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  struct {
    kfn f;
    const char *name;
    int ninstr;  // instructions per asm statement
  } ks[] = {{k_fma, "v_fma_f32 (vgpr)", 1},       {k_fma_s, "v_fma_f32 (sgpr src)", 1},
            {k_fmac, "v_fmac_f32 (VOP2)", 1},     {k_add, "v_add_f32", 1},
            {k_mul, "v_mul_f32", 1},              {k_sub_s, "v_sub_f32 (sgpr src)", 1},
            {k_max, "v_max_f32", 1},              {k_max_s, "v_max_f32 (sgpr src)", 1},
            {k_max3, "v_max3_f32", 1},            {k_med3, "v_med3_f32", 1},
            {k_pkfma, "v_pk_fma_f32", 1},         {k_pkfma_s, "v_pk_fma_f32 (sgpr pair)", 1},
            {k_pkmul, "v_pk_mul_f32", 1},         {k_pkadd, "v_pk_add_f32", 1},
            {k_addu, "v_add_u32", 1},             {k_xor, "v_xor_b32", 1},
            {k_mullo, "v_mul_lo_u32", 1},         {k_cndmask, "v_cmp_lt_f32 + v_cndmask", 2},
            {k_sqrt, "v_sqrt_f32", 1},            {k_rcp, "v_rcp_f32", 1},
            {k_and, "v_and_b32", 1},              {k_lshr, "v_lshrrev_b32", 1},
            {k_ashr, "v_ashrrev_i32", 1},         {k_bfi, "v_bfi_b32", 1},
            {k_add3, "v_add3_u32", 1},            {k_lshladd, "v_lshl_add_u32", 1},
            {k_madu24, "v_mad_u32_u24", 1},       {k_subf, "v_sub_f32 (vgpr)", 1},
            {k_fmak, "v_fmaak_f32 (literal)", 1}, {k_cvt, "v_cvt_f32_u32", 1},
            {k_cmp, "v_cmp_lt_f32 (vcc only)", 1}, {k_cnd, "v_cndmask_b32 (vcc)", 1},
            {k_mad64, "v_mad_u64_u32", 1}};
  const int nk = sizeof(ks) / sizeof(ks[0]);
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < nk; ++v) {
      CHK(hipEventRecord(e0));
      ks[v].f<<<blocks, threads>>>(out, iters, 0.999f, 1e-3f);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      const double instr = (double)blocks * threads / 64 * iters * 8 * ks[v].ninstr;
      if (rep == 1)
        std::printf("%-28s %8.3f ms  %6.3f wave-instr/clk/CU @2.4GHz\n", ks[v].name, ms,
                    instr / (ms * 1e-3) / 256 / 2.4e9);
    }
  }
  return 0;
}
