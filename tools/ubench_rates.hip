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
            {k_sqrt, "v_sqrt_f32", 1},            {k_rcp, "v_rcp_f32", 1}};
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
