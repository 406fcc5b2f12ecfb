// rt_sched.hip -- the pilot schedule's block ordering, on the device.
//
// RT_FLAG_PILOT_SCHEDULE (include/rt.h): a 4-spp pilot of the
// instrumented kernel stores every tile's segment count; the blocks of the
// real render are then launched most expensive first (longest-processing-time
// first), the `units` waves of one tile group adjacent.  This file turns the
// tile costs into that launch order without leaving the stream: a per-block
// sum, a stable radix sort by decreasing cost (hipcub, so equal costs keep
// block order -- what std::stable_sort did on the host in round 1) and the
// expansion by units.  Temporaries are stream-ordered allocations, so
// rt_render_async stays asynchronous on the first render of a geometry too.
// Kept apart from rt_kernel.hip so that the hipcub instantiations do not slow
// down rebuilding the render kernel.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>

namespace {

constexpr int kWavesPerBlock = 4;  // = rtk::kWavesPerBlock (rt_layout.h)

__global__ __launch_bounds__(256) void block_costs(const uint32_t *__restrict__ tile_cost, uint32_t blocks,
                                                   uint32_t *__restrict__ cost, uint32_t *__restrict__ idx) {
  const uint32_t b = blockIdx.x * 256u + threadIdx.x;
  if (b >= blocks) return;
  uint32_t s = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) s += tile_cost[(size_t)b * kWavesPerBlock + w];
  cost[b] = s;
  idx[b] = b;
}

__global__ __launch_bounds__(256) void expand_units(const uint32_t *__restrict__ sorted, uint32_t blocks,
                                                    uint32_t units, uint32_t *__restrict__ order) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= (uint64_t)blocks * units) return;
  const uint32_t k = (uint32_t)(i / units), u = (uint32_t)(i % units);
  order[i] = sorted[k] * units + u;
}

}  // namespace

// order[i * units + u] = sorted_block[i] * units + u, sorted by decreasing
// cost (ties: lower block first).  tile_cost holds blocks * kWavesPerBlock
// entries; order holds blocks * units.  Everything is enqueued on st.
extern "C" hipError_t rt_internal_block_order(const uint32_t *tile_cost, uint32_t blocks, uint32_t units,
                                              uint32_t *order, hipStream_t st) {
  if (!blocks || !units) return hipSuccess;
  uint32_t *buf = nullptr;  // cost, idx, cost_sorted, idx_sorted
  hipError_t e = hipMallocAsync((void **)&buf, 4 * (size_t)blocks * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  uint32_t *cost = buf, *idx = buf + blocks, *cost_s = buf + 2 * (size_t)blocks, *idx_s = buf + 3 * (size_t)blocks;
  block_costs<<<(blocks + 255) / 256, 256, 0, st>>>(tile_cost, blocks, cost, idx);
  e = hipGetLastError();
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  if (e == hipSuccess)
    e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp_bytes, cost, cost_s, idx, idx_s, (int)blocks, 0,
                                                     32, st);
  if (e == hipSuccess) e = hipMallocAsync(&tmp, tmp_bytes ? tmp_bytes : 4, st);
  if (e == hipSuccess)
    e = hipcub::DeviceRadixSort::SortPairsDescending(tmp, tmp_bytes, cost, cost_s, idx, idx_s, (int)blocks, 0, 32,
                                                     st);
  if (e == hipSuccess) {
    const uint64_t n = (uint64_t)blocks * units;
    expand_units<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(idx_s, blocks, units, order);
    e = hipGetLastError();
  }
  if (tmp) (void)hipFreeAsync(tmp, st);
  (void)hipFreeAsync(buf, st);
  return e;
}
