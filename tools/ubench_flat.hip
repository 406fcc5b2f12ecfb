// tools/ubench_flat.hip -- latency of one dependent 16-byte load per lane, by
// path: ds_read_b128 (LDS), global_load_dwordx4 hitting the L1, and
// flat_load_dwordx4 through a generic pointer into LDS or into global memory
// (could C4's hot items be read through one flat load whose lanes
// point into LDS or global memory?).  One block of 64 lanes per CU-wide
// launch, every lane chasing its own random cycle through a 1 024-entry table
// (16 KiB: LDS-resident, and L1-resident after one lap).  Also a mixed case:
// a flat load where `cold` of 64 lanes read global memory.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_flat tools/ubench_flat.hip && /tmp/ubench_flat
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int kN = 1024;  // uint4 entries (16 KiB: fits the L1)
constexpr int kSteps = 4096;

// the next index sits in .x; .y/.z/.w are payload
template <int MODE>
__global__ __launch_bounds__(64) void chase(const uint4 *__restrict__ gtab, int cold, uint32_t zero,
                                            unsigned long long *cycles, uint32_t *sink) {
  __shared__ uint4 s_tab[kN];
  for (int i = threadIdx.x; i < kN; i += 64) s_tab[i] = gtab[i];
  __syncthreads();
  uint32_t idx = (threadIdx.x * 61u) & (kN - 1);
  // warm the L1 with one lap over the global table
  uint32_t w = idx;
  for (int i = 0; i < kN / 64; ++i) w = gtab[w].x;
  // generic pointers whose address space the compiler cannot see
  const uint4 *lds_gen = (const uint4 *)s_tab;
  const uint4 *glb_gen = gtab;
  asm volatile("" : "+v"(lds_gen), "+v"(glb_gen));
  const bool lane_cold = (int)threadIdx.x < cold;
  const uint4 *mixed = lane_cold ? glb_gen : lds_gen;
  uint32_t acc = w & 1u;
  const unsigned long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < kSteps; ++i) {
    uint4 v;
    if (MODE == 0) v = s_tab[idx + acc];                    // ds_read_b128
    else if (MODE == 1) v = gtab[idx + acc];                // global_load_dwordx4 (L1)
    else if (MODE == 2) v = lds_gen[idx + acc];             // flat -> LDS
    else if (MODE == 3) v = glb_gen[idx + acc];             // flat -> global
    else v = mixed[idx + acc];                              // flat, `cold` lanes global
    idx = v.x;
    acc = (v.y ^ v.z ^ v.w) & zero;  // keeps the 16-byte load whole; adds 0 (zero = 0 at run time)
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = idx + acc;
}

template <int MODE>
double run(const uint4 *d_tab, int cold, unsigned long long *d_cyc, uint32_t *d_sink, int blocks) {
  chase<MODE><<<blocks, 64>>>(d_tab, cold, 0u, d_cyc, d_sink);
  std::vector<unsigned long long> c(blocks);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  (void)hipMemcpy(c.data(), d_cyc, 8 * blocks, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto x : c) s += (double)x;
  return s / blocks / kSteps;
}

int main() {
  // a random single cycle over kN entries
  std::vector<uint32_t> perm(kN);
  for (int i = 0; i < kN; ++i) perm[i] = i;
  uint64_t r = 88172645463325252ull;
  for (int i = kN - 1; i > 0; --i) {
    r ^= r << 13; r ^= r >> 7; r ^= r << 17;
    const int j = (int)(r % (uint64_t)(i + 1));
    std::swap(perm[i], perm[j]);
  }
  std::vector<uint4> tab(kN);
  for (int i = 0; i < kN; ++i) tab[perm[i]] = make_uint4(perm[(i + 1) % kN], i, 2 * i, 3 * i);
  uint4 *d_tab;
  unsigned long long *d_cyc;
  uint32_t *d_sink;
  const int blocks = 256;  // one wave per CU
  if (hipMalloc(&d_tab, sizeof(uint4) * kN) || hipMalloc(&d_cyc, 8 * blocks) ||
      hipMalloc(&d_sink, 4 * 64 * blocks))
    return 1;
  (void)hipMemcpy(d_tab, tab.data(), sizeof(uint4) * kN, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) {
    printf("{\"rep\": %d, \"cycles_per_dependent_load\": {\"ds_read_b128\": %.1f, \"global_load_L1\": %.1f, "
           "\"flat_to_lds\": %.1f, \"flat_to_global\": %.1f",
           rep, run<0>(d_tab, 0, d_cyc, d_sink, blocks), run<1>(d_tab, 0, d_cyc, d_sink, blocks),
           run<2>(d_tab, 0, d_cyc, d_sink, blocks), run<3>(d_tab, 0, d_cyc, d_sink, blocks));
    for (int cold : {0, 1, 8, 64}) printf(", \"flat_mixed_cold%d\": %.1f", cold, run<4>(d_tab, cold, d_cyc, d_sink, blocks));
    printf("}}\n");
  }
  return 0;
}
