// rt_layout.h -- internal to librtow: the device-side data layout shared by
// the render kernel (rt_kernel.hip), the acceleration-structure builder
// (rt_accel.cpp) and the C ABI (rt_api.cpp), and the kernel launch interface
// between them.  Not installed; the public interface is include/rt.h.
//
// Layout in HBM: sphere records as SoA pairs for the scan and
// the BVH leaves, 32-B BVH nodes in 8 DFS orders, 48-B shading records, the
// layer grid (u32 cells + 16-B items), the caller's frame tile (W x rows x 3
// fp32 sums, row 0 = top) and 8 x 32 u64 counters.
#ifndef RTOW_RT_LAYOUT_H
#define RTOW_RT_LAYOUT_H

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "rt_internal.h"

namespace rtk {

constexpr int kTile = 8;           // 8x8 pixels per wave
constexpr int kWavesPerBlock = 4;  // 256 threads
constexpr int kBlock = 64 * kWavesPerBlock;
constexpr int kSpherePad = 8;      // scan unroll granularity
// auto rt_params.units without the pilot schedule: below kSplitTiles tiles
// (86 016: 10.5 waves per wave slot of the chip at 256 CUs x 4 SIMDs x 8) a
// tile's samples are split over kUnits waves; above it a wave traces all of
// them.  Measured on the headline frame before the sample pool (round 1,
// tools/rank_times.py): 1 GPU (129 600 tiles) 302 ms unsplit vs
// 310 / 314 with units 2 / 4; a 1/2 share (64 800 tiles) 175 ms unsplit vs
// 158 split, a 1/8 share 103 vs 42.
constexpr long long kSplitTiles = 12LL * 256 * 4 * 7;
// With the pilot schedule (RT_FLAG_PILOT_SCHEDULE) the expensive tiles start
// first, and with the sample pool a wave has no tail of its own, so the split
// only needs ~16 waves per wave slot (8192 slots): units = round(131072 /
// tiles), at most 8.  Measured with even sample shares (tools/rank_times.py
// --pilot, tools/units_frame.py --pilot; profiles/r02zd_units_even_split.log):
// the whole 4K frame (129 600 tiles) 142.8 ms unsplit; a 1/2 share 73.2 / 71.6
// ms at units 1 / 2; a 1/4 share 39.2 / 36.7 / 36.0 at 1 / 2 / 4; a 1/8 share
// 38.0 / 19.5 / 18.7 / 18.5 at 1 / 2 / 4 / 8; C1 (1080p, 100 spp, 32 400
// tiles) 8.5 / 8.0 / 7.9 / 8.2 ms at 1 / 2 / 3 / 4.
constexpr long long kPilotTilesPerUnit = 16LL * 256 * 4 * 8;
constexpr int kUnits = 8;  // without the pilot
// the per-wave stats counters are spread over 32 slots of 8 (by block index)
// and summed on the host: ~10^5 waves adding to one address serialise at the
// end of short launches (1/8 shares: 17.47 vs 17.57 ms slowest rank,
// profiles/r02zl_ab_counter_slots.log)
constexpr int kCounterSlots = 32;
// Bounded launches (failure detection): a render is split into
// launches of about this many samples at most (RT_OPT_LAUNCH_SAMPLES
// overrides).  2^35 (round 5; 2^32 before) keeps the headline frame (4.15e9
// samples, ~0.12 s) and a C3 rank share in one launch and cuts a C4 rank
// share (6.7e10) into 2 sample ranges of 1 000 spp (~1.2 s each): a wave's
// longer sample pool idles fewer lanes at its tail, C4's share 2.40 -> 2.36 s
// and C3's whole frame 921 -> 911 ms against 2^32.  When
// sample ranges alone would leave fewer than kMinPoolSpp samples per pixel
// per wave, the work entries are split into strided ranges as well and the
// samples into chunks of ~kPoolSpp (rt_api.cpp plan_launches).  At most
// kMaxLaunches launches per render.
constexpr double kLaunchSamples = 34359738368.0;
constexpr double kMinPoolSpp = 100.0;
constexpr double kPoolSpp = 250.0;
constexpr long long kMaxLaunches = 65536;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// scan record for two consecutive spheres i, i+1 (32 B): every field is a
// pair so that one s_load_dwordx8 yields ready-made SGPR pairs
struct __attribute__((aligned(32))) pair_geom {
  f2 cx, cy, cz, ks;  // ks = |C|^2 - r^2
};

// BVH node for the wave-uniform, stackless traversal (RT_FLAG_ACCEL_BVH): DFS
// pre-order, one padded AABB per node, `skip` = next node when the subtree is
// not entered.  32 B = one s_load_dwordx8; the (lo, hi) pairs feed
// v_pk_fma_f32 like the sphere records do.
struct __attribute__((aligned(32))) bvh_node {
  f2 bx, by, bz;  // (lo, hi) per axis; layer mode: bx = (centre x, centre z),
                  // by = (half-width x, half-width z), bz unused (bvh_builder::to_centre_form)
  int32_t skip;
  uint32_t leaf;  // 0: internal (first child = this + 1); else (1 + first pair) | kTwoPairs
};
constexpr int kLeafPairs = 2;            // leaves hold up to 4 spheres: 1 or 2 scan pairs
constexpr uint32_t kTwoPairs = 1u << 31;  // leaf flag: 3-4 spheres (else 1-2, one pair)

// per-sphere shading record, fetched once per segment for the closest sphere
struct __attribute__((aligned(16))) shade_rec {
  float cx, cy, cz, inv_r;
  float ar, ag, ab, param;  // albedo (1,1,1 for dielectrics); fuzz | ior
  uint32_t kind;
  float radius, ks;
  float inv_param;          // 1/ior (dielectric)
  float r0;                 // Schlick r0 = ((1-ior)/(1+ior))^2 (dielectric)
  uint32_t sealed;          // 1: a lambertian ball no other ball overlaps (rt_accel.cpp sealed_spheres)
  float pad1, pad2;
};

// Where the layer grid lives during a launch (rt_context_set_option
// RT_OPT_GRID_PLACEMENT; the image is the same for every placement):
//   kGridGlobal: cells and items read from global memory (L1 / L2);
//   kGridLds:    the block copies items and u16 cell starts into LDS (the
//                final scene: ~900 items, 16 KB);
//   kGridCells:  only the u16 cell starts in LDS, items from global memory
//                (large scenes: C4's ~22 000 items do not fit, its cells do
//                at a coarser cell size).
enum { kGridGlobal = 0, kGridLds = 1, kGridCells = 2 };

struct kparams {
  rt_camera cam;
  int width, height, spp, max_depth;
  int row_block, band_stride, band_offset, local_rows;
  int tiles_x, n_pad, n_nodes;
  float oref2;  // BVH padding assumes |ray origin|^2 <= oref2 (else the wave scans)
  // layer mode (bvh_builder::split_layer): the BVH holds only the spheres of
  // one thin y-layer, whose slab interval the walk computes once per ray;
  // the few other spheres are n_extra_pairs scan pairs from extra_pair0 on
  f2 layer;
  int layer_mode, extra_pair0, n_extra_pairs;
  float layer_cy;
  uint32_t seed32, flags;
  float inv_wm1, inv_hm1;  // 1/(W-1), 1/(H-1) rounded once (cpu camera model)
  // exact division by the width: W = wodd << wshift, wodd * winv == 1 (mod 2^32)
  uint32_t wshift, winv;
  // this launch's samples [s_lo, s_lo + s_cnt) of every pixel, split over
  // `units` waves per tile: block b traces samples [s_lo + u s_cnt / units,
  // s_lo + (u + 1) s_cnt / units), u = b % units
  int units, s_lo, s_cnt;
  // this launch's work entries: blockIdx.x * block_stride + block_base
  // indexes block_order (or is the entry itself), entries [0, blocks * units)
  // 0: the wave stores its tile's pixels as floats (one launch, one unit);
  // 1: it adds its integer sums into the frame with atomics (several units or
  // launches per tile; finish_sums converts at the end)
  int sum_atomic;
  // fixed-point pixel sums: a sample adds q(v 2^F) to
  // its pixel's uint32 sum; the frame holds sum 2^-F.  F = 31 - floor(log2
  // spp); q truncates, or, when dither != 0 (F < 20: spp >= 4096), rounds
  // stochastically (unbiased for every spp)
  float qscale, qinv;  // 2^F, 2^-F
  int dither, block_base;
  int block_stride;
  // WIDE renders (a scene albedo above 1): 64-bit sums, a sample's radiance
  // clamped at vcap (rt_api.cpp sum_format)
  float vcap;
  // device buffers (rt_context; out = the caller's frame tile)
  const struct pair_geom *scan_geom;  // brute-force order
  const struct pair_geom *geom;       // BVH leaf order
  const struct bvh_node *nodes;       // 8 DFS orders of n_nodes
  const int *orig;                    // BVH slot -> original index
  const struct shade_rec *shade;
  float *out;
  unsigned long long *counters;
  // block schedule (nullptr = launch order): block_order[blockIdx] is the
  // block of work to run, most expensive first (rt_context tile-cost pilot)
  const uint32_t *block_order;
  uint32_t *tile_cost;  // pilot renders: segments traced per tile
  // layer grid (layer mode, bvh_builder::build_grid): x-z cells over the
  // layer spheres; cell = (first item << 4) | item count, row-major [nz][nx];
  // item = (cx, cz, ks, original index bits).  nullptr: walk the layer BVH.
  const uint32_t *grid_cells;
  const f4 *grid_items;
  float grid_x0, grid_z0;  // corner of cell (0, 0), a ring cell
  float grid_xi, grid_zi;  // inner box (the listed region): [xi, x1] x [zi, z1]
  float grid_x1, grid_z1, grid_g, grid_invg;
  int grid_nx, grid_nz;    // cells including the ring
  // LDS-resident grid: kGridLds copies the items (16 B) and then n_cells + 1
  // u16 item-start LDS addresses (cell i's items are [start_i, start_{i+1}));
  // kGridCells copies n_cells + 1 u16 item-start INDICES only
  int grid_n_items, grid_n_cells;
  // layer mode: the extras' first scan pair and its slots' original indices
  // (geom + extra_pair0, orig + 2 extra_pair0), resolved on the host so the
  // kernel does no 64-bit index arithmetic per step
  const struct pair_geom *extra_geom;
  const int *extra_orig;
};

// LDS bytes of the grid copy of one block
__host__ __device__ constexpr size_t grid_lds_bytes(int placement, long long n_items, long long n_cells) {
  return placement == kGridLds ? (size_t)n_items * 16u + ((size_t)(n_cells + 1) * 2u + 15u) / 16u * 16u
         : placement == kGridCells ? ((size_t)(n_cells + 1) * 2u + 15u) / 16u * 16u
                                   : 0u;
}
// LDS budget of the grid copy: with render_kernel's static LDS (the tiles'
// pixel sums and row indices) a 256-thread block stays within 20 KB, so 8
// blocks (8 waves per SIMD) still fit in the CU's 160 KB
constexpr size_t kStaticLds = 3 * kBlock * 4 + kWavesPerBlock * kTile * 8;  // sums + row table (pixel base, valid columns)
constexpr size_t kGridLdsMax = 160 * 1024 / 8 - kStaticLds;
// WIDE builds hold 64-bit pixel sums: 3 KB more static LDS
constexpr size_t kGridLdsMaxWide = kGridLdsMax - 3 * kBlock * 4;

// ---- launch interface (defined in rt_kernel.hip) ----
// render_kernel variant bits
enum {
  kVarOpen = 1,       // RT_FLAG_OPEN_INTERVAL
  kVarMetalUnit = 2,  // RT_FLAG_METAL_UNIT_VECTOR
  kVarBvh = 4,        // RT_FLAG_ACCEL_BVH
  kVarStats = 8,      // RT_FLAG_COUNT_WORK (and the pilot)
  kVarGrid = 16,      // the layer-grid walk (with kVarBvh on a layer scene)
  kVarPlaceShift = 5, // bits 5-6: the grid placement (kGridGlobal / kGridLds / kGridCells)
  kVarWide = 128      // 64-bit pixel sums (a scene albedo above 1)
};
hipError_t launch_render(int variant, unsigned blocks, size_t lds_bytes, hipStream_t st, const kparams &kp);
hipError_t launch_finish_sums(uint32_t *frame, uint64_t n, float qinv, hipStream_t st);
hipError_t launch_finish_sums_wide(const uint64_t *sums, float *frame, uint64_t n, float qinv, hipStream_t st);
hipError_t launch_tonemap(bool fp32, const float *sums, uint64_t n, int spp, const void *thresholds,
                          uint8_t *out, hipStream_t st);
hipError_t launch_kat(int kind, const double *in, int n, double *out);
hipError_t upload_turn_table();

}  // namespace rtk

#endif  // RTOW_RT_LAYOUT_H
