// rt_render.hip -- the MI355X (gfx950) render kernel and the device half of
// the C ABI in include/rt.h.
//
// Replaces render<<<>>> (src/gpu/camera.h:169-195) and, inside it, get_ray
// (camera.h:153-167 / src/cpu/camera.h:28-34), ray_color (src/cpu/main.cc:12-30,
// iterative as in src/gpu/camera.h:112-138), hittable_list::hit / sphere::hit
// (src/cpu/hittable_list.h:28-43, src/cpu/sphere.h:24-51) and the three
// material::scatter functions (src/cpu/material.h:15-88).
//
// Design (DESIGN.md "Kernel"):
//  * one lane per pixel, one wave64 per 8x8 pixel tile, 4 waves per block;
//  * the lane loops over ITS pixel's spp samples and regenerates a camera ray
//    as soon as a path ends ("path regeneration"), so every bounce iteration
//    of the wave does useful work on every lane until that lane's pixel is
//    finished; the wave exits on __ballot(alive) == 0;
//  * closest hit: a wave-uniform, stackless BVH walk (in the
//    final scene a tree over the thin layer of small spheres, 3.2) or the
//    brute-force scan; node and sphere records are scalar (SMEM) loads into
//    SGPRs that feed v_pk_fma_f32 directly -- no LDS traffic, no per-lane
//    divergence; the square root and the interval test run only in the
//    branch where some lane's discriminant is non-negative;
//  * 8 waves per SIMD: kernel parameters are re-read from the kernarg segment
//    where they are used and per-lane coordinates recomputed, so nothing
//    rarely used stays in registers across the bounce loop;
//  * counter-based RNG (pcg4d keyed by pixel, sample, bounce slot, seed):
//    no per-pixel state, results independent of launch geometry and of the
//    number of GPUs;
//  * fp32 with explicit fmaf and -ffp-contract=off: the kernel is bit-exact
//    with the CPU restatement in oracle/rt_oracle.cc (kernel mode).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "rt.h"
#include "rt_turn_table.h"

extern "C" void rt_internal_set_hip_error(int e);
extern "C" hipError_t rt_internal_block_order(const uint32_t *tile_cost, uint32_t blocks, uint32_t units,
                                              uint32_t *order, hipStream_t st);

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

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// STATS builds: the grid walk's box_hits counts wave-level DDA iterations, or
// with RT_COUNT_ITEMS=1 wave-level item iterations, =2 wave-level item
// iterations that run the root sequence (tools/grid_wave_counts.py)
#ifndef RT_COUNT_ITEMS
#define RT_COUNT_ITEMS 0
#endif

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

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
  float pad0, pad1, pad2;
};

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
  // the split of a tile's samples over waves: block b traces samples
  // [u spp / units, (u + 1) spp / units) of its tiles, u = b % units
  int units, pad_u;
  // fixed-point pixel sums: a sample adds trunc(v 2^F)
  // to its pixel's uint32 sum; the frame holds sum 2^-F
  float qscale, qinv;  // 2^F, 2^-F with F = 31 - floor(log2(spp))
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
  // LDS-resident grid (render_kernel<..., GLDS>): the block copies the items
  // (16 B) and then n_cells + 1 u16 item-start addresses (cell i's items are
  // [start_i, start_{i+1})) into dynamic LDS at launch
  int grid_n_items, grid_n_cells;
};

// the dynamic LDS of the GLDS builds: grid items, then the u16 cells
extern __shared__ f4 s_grid_dyn[];
typedef const __attribute__((address_space(3))) f4 lds_f4;
__host__ __device__ constexpr size_t grid_lds_bytes(int n_items, int n_cells) {
  return (size_t)n_items * 16u + ((size_t)(n_cells + 1) * 2u + 15u) / 16u * 16u;
}
// LDS budget of the grid copy: with render_kernel's static LDS (the tiles'
// pixel sums and row indices) a 256-thread block stays within 20 KB, so 8
// blocks (8 waves per SIMD) still fit in the CU's 160 KB
constexpr size_t kStaticLds = 3 * kBlock * 4 + kWavesPerBlock * kTile * 4;
constexpr size_t kGridLdsMax = 160 * 1024 / 8 - kStaticLds;

// The kernel arguments, re-read from the kernarg segment (constant address
// space: scalar loads that hit the scalar cache) at the rare places that need
// camera constants, instead of holding them in SGPRs for the whole kernel.
// The empty asm hides the pointer's invariance so the compiler cannot hoist
// the loads back to the kernel entry; the word-wise copy keeps the address
// space (unused words are dead).
typedef const uint32_t __attribute__((address_space(4))) kword_c;
// Scene data are read-only for the whole launch: read through the constant
// address space, uniform addresses become scalar (SMEM) loads into SGPRs.
#define RT_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const RT_CONST T *as_const(const T *p) {
  return (const RT_CONST T *)p;
}
// per-lane buffers (shading records, frame, counters) in the global
// address space: global_load/store rather than flat (no lgkmcnt coupling)
#define RT_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ RT_GLOBAL T *as_global(T *p) {
  return (RT_GLOBAL T *)p;
}
// a whole record from the constant address space (one s_load_dwordxN when uniform)
template <class T>
__device__ __forceinline__ T cload_g(const RT_GLOBAL T *p) {
  static_assert(sizeof(T) % 16 == 0, "16-byte records");
  typedef uint32_t quad __attribute__((ext_vector_type(4)));
  struct { quad q[sizeof(T) / 16]; } w;
#pragma unroll
  for (unsigned i = 0; i < sizeof(T) / 16; ++i) w.q[i] = ((const RT_GLOBAL quad *)p)[i];
  return __builtin_bit_cast(T, w);
}
template <class T>
__device__ __forceinline__ T cload(const RT_CONST T *p) {
  static_assert(sizeof(T) % 4 == 0, "dword records");
  typedef uint32_t words __attribute__((ext_vector_type(sizeof(T) / 4)));
  return __builtin_bit_cast(T, *(const RT_CONST words *)p);
}
__device__ __forceinline__ kparams kernargs() {
  kword_c *q = (kword_c *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  kparams r;
  uint32_t *w = reinterpret_cast<uint32_t *>(&r);
#pragma unroll
  for (unsigned i = 0; i < sizeof(kparams) / 4; ++i) w[i] = q[i];
  return r;
}

// ---------------------------------------------------------------- RNG ----
// pcg4d (Jarzynski & Olano, "Hash Functions for GPU Rendering", JCGT 2020):
// a 4-D -> 4-D counter hash; one call gives the 4 uniforms a bounce needs.
// The second and third inputs (sample index, bounce slot) are < 2^24
// (params_ok bounds spp and max_depth), as is the LCG multiplier: their
// products take the full-rate 24-bit multiply (v_mul_u32_u24, the same low
// 32 bits) instead of the quarter-rate v_mul_lo_u32.
__device__ __forceinline__ uint4 pcg4d(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t x = a * 1664525u + 1013904223u;
  uint32_t y = __umul24(b, 1664525u) + 1013904223u;
  uint32_t z = __umul24(c, 1664525u) + 1013904223u;
  uint32_t w = d * 1664525u + 1013904223u;
  x += y * w; y += z * x; z += x * y; w += y * z;
  x ^= x >> 16; y ^= y >> 16; z ^= z >> 16; w ^= w >> 16;
  x += y * w; y += z * x; z += x * y; w += y * z;
  return make_uint4(x, y, z, w);
}

__device__ __forceinline__ float unif(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

// sqrtf(max(x, 2^-96)), correctly rounded: y = v_rsq_f32(x), s = x y, then one
// Newton step on the product, s + (x - s^2) y/2.  Equal to the correctly
// rounded sqrt for every fp32 in [2^-96, +inf) (checked exhaustively on the
// GPU: tools/ubench_sqrt2.hip, profiles/r02zh_ubench_sqrt2.log); below 2^-96
// it is not (NaN at 0), and the clamp keeps those out.  5 VALU + the clamp,
// against 9 for v_sqrt_f32 with LLVM's two-residual correction, at 2.3x its
// issue rate.  No call site can tell the clamp from sqrtf (arguments are 0 or
// >> 2^-96, and a root 2^-48 instead of 0 rounds away against any t >=
// 0.001); the host restatement applies the same clamp.
__device__ __forceinline__ float sqrt_k(float x) {
  x = fmaxf(x, 0x1p-96f);
  const float y = __builtin_amdgcn_rsqf(x);
  const float s = x * y, hy = 0.5f * y;
  return fmaf(fmaf(-s, s, x), hy, s);
}

// sin/cos of 2 pi u, u in [0, 1): the table's (cos, sin) of 2 pi i / 1024 for
// i = floor(1024 u) (include/rt_turn_table.h: fp64 Taylor, rounded once; the
// oracle builds the same table), rotated by the remainder d = frac(1024 u) 2
// pi / 1024 < 0.0062 with cos d = 1 - d^2/2, sin d = d (1 - d^2/6) (truncation
// < 1e-10).  13 VALU and one 8-byte load instead of a quadrant-reduced Taylor
// pair (~26 VALU): 142.0 -> 139.9 ms.
constexpr int kTurnTab = RT_TURN_TABLE;
__device__ f2 g_turn_tab[kTurnTab];
__device__ __forceinline__ void sincos_turn(float u, float &s, float &c) {
  const float t = u * (float)kTurnTab;
  const float fl = floorf(t);
  const f2 sc = as_global(g_turn_tab)[(int)fl];
  const float d = (t - fl) * (6.28318530717958648f / (float)kTurnTab);
  const float x2 = d * d;
  const float cd = fmaf(x2, -0.5f, 1.0f);
  const float sd = d * fmaf(x2, -0.166666667f, 1.0f);
  c = fmaf(sc.x, cd, -(sc.y * sd));
  s = fmaf(sc.y, cd, sc.x * sd);
}

// Radius of a uniform point in the unit ball (the radius law of
// random_in_unit_sphere's rejection loop, vec3.h:105-112: CDF r^3): the largest of three independent uniforms, from the step hash's
// z and w draws and its unused low bytes of x, y, z (unif() takes the top 24
// bits).  One v_max3 instead of a cube root.
__device__ __forceinline__ float ball_radius(const uint4 r) {
  const uint32_t lo = ((r.x & 0xffu) << 24) | ((r.y & 0xffu) << 16) | ((r.z & 0xffu) << 8);
  return fmaxf(fmaxf(unif(r.z), unif(r.w)), unif(lo));
}

// (rho cos 2 pi u, rho sin 2 pi u), rho = sqrt_k(a): the polar draw of both
//  * the uniform direction on the unit sphere (z = 1 - 2 u1, a = 1 - z^2,
//    u = u2; replaces the rejection loop of random_unit_vector,
//    src/cpu/vec3.h:105-114, equal in distribution), and
//  * camera_ray's lens-disk sample (a = u3, u = u4).
// The render loop runs it once per lane and step for whichever of the two the
// lane needs (a wave whose lanes both bounce and start new paths would
// otherwise run it twice).
__device__ __forceinline__ void polar(float a, float u, float &x, float &y) {
  const float rho = sqrt_k(a);
  float s, c;
  sincos_turn(u, s, c);
  x = rho * c;
  y = rho * s;
}

// x * 1/|x| with 1/|x| from an integer-seeded inverse square root and three
// Newton steps y <- y (3/2 - (l2/2) y^2): plain fp32 mul/fma, so the host
// restatement reproduces it bit for bit, and ~12 VALU instead of a correctly
// rounded sqrt followed by a correctly rounded division (~28).  |result| is 1
// within a few ulp; l2 is never 0 or inf here ("Kernel").
__device__ __forceinline__ void normalize3(float &x, float &y, float &z) {
  const float l2 = fmaf(z, z, fmaf(y, y, x * x));
  float r = __uint_as_float(0x5f375a86u - (__float_as_uint(l2) >> 1));
  const float h = 0.5f * l2;
#pragma unroll
  for (int k = 0; k < 3; ++k) r = r * fmaf(-h, r * r, 1.5f);
  x *= r;
  y *= r;
  z *= r;
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
  return fmaf(az, bz, fmaf(ay, by, ax * bx));
}

// reflect(v, n) = v - 2 dot(v, n) n (src/cpu/vec3.h:122-124), dn = dot(v, n)
__device__ __forceinline__ void reflect3(float vx, float vy, float vz, float nx, float ny, float nz, float dn,
                                         float &rx, float &ry, float &rz) {
  const float k2 = -2.0f * dn;
  rx = fmaf(k2, nx, vx);
  ry = fmaf(k2, ny, vy);
  rz = fmaf(k2, nz, vz);
}

// refract(uv, n, ratio) (src/cpu/vec3.h:126-131) with cos_t = fminf(-dot(uv, n), 1):
// perp = ratio (uv + cos_t n), parallel = -sqrt(|1 - |perp|^2|) n
__device__ __forceinline__ void refract3(float vx, float vy, float vz, float nx, float ny, float nz, float cos_t,
                                         float ratio, float &sx, float &sy, float &sz) {
  const float qx = ratio * fmaf(cos_t, nx, vx);
  const float qy = ratio * fmaf(cos_t, ny, vy);
  const float qz = ratio * fmaf(cos_t, nz, vz);
  const float m = -sqrt_k(fabsf(1.0f - dot3(qx, qy, qz, qx, qy, qz)));
  sx = fmaf(m, nx, qx);
  sy = fmaf(m, ny, qy);
  sz = fmaf(m, nz, qz);
}

// Schlick's reflectance (src/cpu/material.h:82-87), r0 = ((1 - ref_idx) / (1 +
// ref_idx))^2 precomputed in fp64 (the same for ior and 1 / ior)
__device__ __forceinline__ float schlick(float cosine, float r0) {
  const float x = 1.0f - cosine;
  const float x2 = x * x;
  return fmaf(1.0f - r0, x2 * x2 * x, r0);
}

// camera ray for (pixel, sample): get_ray, src/cpu/camera.h:28-34 (model CPU)
// or src/gpu/camera.h:153-167 (model GPU), from r = pcg4d(pix, sample, 0,
// seed32) and the lens sample (ddx, ddy) = polar(unif(r.z), unif(r.w)) (used
// only when the camera has a lens); the direction is left unnormalised
__device__ __forceinline__ void camera_dir(const kparams &p, const uint4 r, float ddx, float ddy,
                                           int col, int grow, float &ox, float &oy, float &oz,
                                           float &dx, float &dy, float &dz) {
  float u1 = unif(r.x), u2 = unif(r.y);
  float fs, ft;
  if (p.cam.model == RT_CAMERA_CPU) {
    int j = p.height - 1 - grow;
    fs = ((float)col + u1) * p.inv_wm1;
    ft = ((float)j + u2) * p.inv_hm1;
  } else {
    fs = (float)col + (u1 - 0.5f);
    ft = (float)grow + (u2 - 0.5f);
  }
  float tx = fmaf(ft, p.cam.vert[0], fmaf(fs, p.cam.horiz[0], p.cam.corner[0]));
  float ty = fmaf(ft, p.cam.vert[1], fmaf(fs, p.cam.horiz[1], p.cam.corner[1]));
  float tz = fmaf(ft, p.cam.vert[2], fmaf(fs, p.cam.horiz[2], p.cam.corner[2]));
  ox = p.cam.eye[0];
  oy = p.cam.eye[1];
  oz = p.cam.eye[2];
  if (p.cam.has_lens) {
    ox = fmaf(ddy, p.cam.lens_v[0], fmaf(ddx, p.cam.lens_u[0], ox));
    oy = fmaf(ddy, p.cam.lens_v[1], fmaf(ddx, p.cam.lens_u[1], oy));
    oz = fmaf(ddy, p.cam.lens_v[2], fmaf(ddx, p.cam.lens_u[2], oz));
  }
  dx = tx - ox;
  dy = ty - oy;
  dz = tz - oz;
}

// the whole camera ray for r = pcg4d(pix, sample, 0, seed32)
__device__ __forceinline__ void camera_ray(const kparams &p, const uint4 r, int col, int grow,
                                           float &ox, float &oy, float &oz,
                                           float &dx, float &dy, float &dz) {
  float ddx = 0.0f, ddy = 0.0f;
  if (p.cam.has_lens) polar(unif(r.z), unif(r.w), ddx, ddy);
  camera_dir(p, r, ddx, ddy, col, grow, ox, oy, oz, dx, dy, dz);
  normalize3(dx, dy, dz);
}

template <bool OPEN>
__device__ __forceinline__ bool in_range(float t, float tmin, float tmax) {
  if (OPEN) return (t > tmin) & (t < tmax);   // interval::surrounds
  return (t >= tmin) & (t <= tmax);           // src/cpu/sphere.h:38-42
}

// This lane's index in its wave, recomputed where it is needed (volatile: not
// hoisted, so it is not held in a VGPR through the bounce loop).
__device__ __forceinline__ int lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// running closest hit of one lane (hittable_list::hit's closest_so_far/rec),
// kept as the 64-bit key the candidate rule orders by: (tmax bits, tie2 | near).
// tmax >= t_min > 0 (or +inf: no hit), so its bits order like its value; tie2
// = 2 (0x7fffffff - index) for the closed interval (ties to the larger index)
// or 2 index for the open one (ties to the smaller); near: the winner was taken
// at its entering root.  One 64-bit compare decides "closer, ties by index"
// (same sphere twice: equal keys, no update).
struct hit_state {
  float tmax;
  uint32_t lo;  // tie2 | near; 0xffffffff with tmax = +inf: no hit
};
template <bool OPEN>
__device__ __forceinline__ uint32_t tie2_of(uint32_t idx) {
  return OPEN ? idx << 1 : (0x7fffffffu - idx) << 1;
}
template <bool OPEN>
__device__ __forceinline__ int best_of(const hit_state &hs) {
  if (hs.tmax == __builtin_huge_valf()) return -1;
  return (int)(OPEN ? hs.lo >> 1 : 0x7fffffffu - (hs.lo >> 1));
}
__device__ __forceinline__ int near_of(const hit_state &hs) { return (int)(hs.lo & 1u); }
__device__ __forceinline__ hit_state no_hit() { return hit_state{__builtin_huge_valf(), 0xffffffffu}; }

// closest-hit candidate update (sphere.h:34-44 with a = |d|^2 = 1).  The root
// a sphere offers is t0 if t0 is past t_min, else t1; it wins if it is closer
// than tmax, ties going to the LAST index for src/cpu's closed interval and to
// the FIRST for src/gpu's open one.  This makes the result independent of the
// order spheres are visited in: brute-force scan and BVH traversal agree bit
// for bit.
// tie2 = tie2_of<OPEN>(index).
template <bool OPEN>
__device__ __forceinline__ void candidate(bool c, float h, float disc, uint32_t tie2, hit_state &hs) {
  if (c) {
    const float sq = sqrt_k(disc);
    const float t0 = h - sq, t1 = h + sq;
    const bool use0 = OPEN ? (t0 > 0.001f) : (t0 >= 0.001f);
    const float root = use0 ? t0 : t1;
    // root >= t_min  <=>  t1 >= t_min (t1 >= t0; with use0, t0 >= t_min)
    const bool above = OPEN ? (t1 > 0.001f) : (t1 >= 0.001f);
    const uint32_t lo = tie2 + (use0 ? 1u : 0u);
    const uint64_t key = ((uint64_t)__float_as_uint(root) << 32) | lo;
    const uint64_t cur = ((uint64_t)__float_as_uint(hs.tmax) << 32) | hs.lo;
    if (above & (key < cur)) {
      hs.tmax = root;
      hs.lo = lo;
    }
  }
}

// per-segment ray constants of the expanded quadratic, splatted for packed math
struct ray_pre {
  f2 dx, dy, dz, nk1, o2, ox2, oy2, oz2;
};

// Test NP consecutive sphere pairs (wave-uniform address -> SGPRs).  Per pair:
// 7 v_pk_fma_f32 + 2 v_cmp; one scalar OR of the ballots decides whether any
// lane needs the sqrt / interval work.  orig maps slots to original indices
// (BVH order); nullptr = identity (brute-force order).
// The dot products take the y term first, h = fma(cz,dz, fma(cx,dx, fma(cy,dy, nk1)))
// (DESIGN.md 2).  NOY: every sphere has the BVH layer's centre y, and r.nk1 /
// r.o2 already hold fma(cy, dy, nk1) / fma(cy, -2 oy, o2) -- the same bits with
// 5 instead of 7 v_pk_fma_f32 per pair.
template <bool OPEN, int NP, bool STATS, bool NOY = false>
__device__ __forceinline__ void scan_pairs(const RT_CONST pair_geom *__restrict__ g, int slot0,
                                           const RT_CONST int *__restrict__ orig, const ray_pre &r,
                                           hit_state &hs, uint32_t &roots) {
  pair_geom q[NP];
  f2 h[NP], e[NP];
  bool c[2 * NP];
  uint64_t any = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    q[j] = cload(g + j);
    const f2 hy = NOY ? r.nk1 : fma2(q[j].cy, r.dy, r.nk1);
    const f2 gy = NOY ? r.o2 : fma2(q[j].cy, r.oy2, r.o2);
    h[j] = fma2(q[j].cz, r.dz, fma2(q[j].cx, r.dx, hy));
    const f2 gg = fma2(q[j].cz, r.oz2, fma2(q[j].cx, r.ox2, gy));
    e[j] = fma2(h[j], h[j], -gg);
    // discriminant >= 0  <=>  e >= ks  (exact for finite floats)
    c[2 * j] = e[j].x >= q[j].ks.x;
    c[2 * j + 1] = e[j].y >= q[j].ks.y;
  }
#pragma unroll
  for (int j = 0; j < 2 * NP; ++j) any |= __builtin_amdgcn_ballot_w64(c[j]);
  if (any) {  // wave-uniform: the rare path where some line meets a sphere
    if (STATS) {
#pragma unroll
      for (int j = 0; j < 2 * NP; ++j) roots += __builtin_amdgcn_ballot_w64(c[j]) != 0 ? 1u : 0u;
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int s0 = slot0 + 2 * j;
      const int i0 = orig ? orig[s0] : s0;
      const int i1 = orig ? orig[s0 + 1] : s0 + 1;
      candidate<OPEN>(c[2 * j], h[j].x, e[j].x - q[j].ks.x, tie2_of<OPEN>((uint32_t)i0), hs);
      candidate<OPEN>(c[2 * j + 1], h[j].y, e[j].y - q[j].ks.y, tie2_of<OPEN>((uint32_t)i1), hs);
    }
  }
}

// scan_pairs in plain fp32, one sphere at a time: the same fma per sphere as
// one half of the packed form (the same bits), without splatting the ray terms
// into VGPR pairs and without moving the second SGPR operand of every
// v_pk_fma_f32 into a VGPR first (the grid build's extras: 4 spheres a step)
template <bool OPEN, int NP, bool STATS>
__device__ __forceinline__ void scan_pairs_scalar(const RT_CONST pair_geom *__restrict__ g, int slot0,
                                                  const RT_CONST int *__restrict__ orig, const ray_pre &r,
                                                  hit_state &hs, uint32_t &roots) {
  float h[2 * NP], e[2 * NP], ks[2 * NP];
  bool c[2 * NP];
  uint64_t any = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const pair_geom q = cload(g + j);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float cx = s ? q.cx.y : q.cx.x, cy = s ? q.cy.y : q.cy.x, cz = s ? q.cz.y : q.cz.x;
      const float hy = fmaf(cy, r.dy.x, r.nk1.x);
      const float gy = fmaf(cy, r.oy2.x, r.o2.x);
      const float hh = fmaf(cz, r.dz.x, fmaf(cx, r.dx.x, hy));
      const float gg = fmaf(cz, r.oz2.x, fmaf(cx, r.ox2.x, gy));
      const float ee = fmaf(hh, hh, -gg);
      h[2 * j + s] = hh;
      e[2 * j + s] = ee;
      ks[2 * j + s] = s ? q.ks.y : q.ks.x;
      c[2 * j + s] = ee >= ks[2 * j + s];
    }
  }
#pragma unroll
  for (int j = 0; j < 2 * NP; ++j) any |= __builtin_amdgcn_ballot_w64(c[j]);
  if (any) {
    if (STATS) {
#pragma unroll
      for (int j = 0; j < 2 * NP; ++j) roots += __builtin_amdgcn_ballot_w64(c[j]) != 0 ? 1u : 0u;
    }
#pragma unroll
    for (int j = 0; j < 2 * NP; ++j) {
      const int i0 = orig ? orig[slot0 + j] : slot0 + j;
      candidate<OPEN>(c[j], h[j], e[j] - ks[j], tie2_of<OPEN>((uint32_t)i0), hs);
    }
  }
}

// Well-conditioned recomputation of the winning sphere's chosen root.  The
// scan's expanded quadratic is cheap but, in fp32, near a small sphere's
// silhouette its root is off by ~1e-4 along the normal: hit points land
// inside the sphere and grazing scattered rays get trapped (measured +1.2 %
// segments vs src/cpu at C0).  Per winner, once per segment:
//   c    = |oc|^2 - r^2  (centered)  or  g + ks (expanded, exact for the
//          r = 1000 ground where |C|^2 - r^2 = 0), whichever has the smaller
//          intermediate magnitude;
//   disc = r^2 - |oc - b d|^2 (perpendicular form)  or  b^2 - c;
//   roots q = -(b + sign(b) sqrt(disc)) and c RN(1/q)  (no cancellation).
// RN(1/q) is rcp_k: v_rcp_f32 and one Newton step, r + r (1 - q r), equal to
// 1.0f / q for every q whose exponent field is 1..252 (normal q and 1/q),
// checked exhaustively (tools/ubench_rcp.hip, profiles/r02zj_ubench_rcp.log);
// here |q| >= sqrt(2^-96).  3 VALU for the second root instead of the ~10 of
// an IEEE division.
__device__ __forceinline__ float rcp_k(float q) {
  const float r = __builtin_amdgcn_rcpf(q);
  return fmaf(fmaf(-q, r, 1.0f), r, r);
}
__device__ __forceinline__ float refine_root(const shade_rec &sr, float t_scan, bool near,
                                             float ox, float oy, float oz, float dx, float dy,
                                             float dz, float o2, float ox2, float oy2, float oz2,
                                             float &b_out) {
  const float r2 = sr.radius * sr.radius;
  const float ocx = ox - sr.cx, ocy = oy - sr.cy, ocz = oz - sr.cz;
  const float b = dot3(ocx, ocy, ocz, dx, dy, dz);
  b_out = b;
  float c;
  if (r2 < o2 + fabsf(sr.ks)) {
    c = fmaf(ocz, ocz, fmaf(ocy, ocy, fmaf(ocx, ocx, -r2)));
  } else {
    const float g = fmaf(sr.cz, oz2, fmaf(sr.cy, oy2, fmaf(sr.cx, ox2, o2)));
    c = g + sr.ks;
  }
  float disc;
  if (r2 < b * b) {
    const float fx = fmaf(-b, dx, ocx), fy = fmaf(-b, dy, ocy), fz = fmaf(-b, dz, ocz);
    disc = fmaf(-fz, fz, fmaf(-fy, fy, fmaf(-fx, fx, r2)));
  } else {
    disc = fmaf(b, b, -c);
  }
  const float sq = sqrt_k(disc);  // clamps disc below at 2^-96 > 0
  const float q = -(b + (b < 0.0f ? -sq : sq));
  float t = t_scan;
  if (q != 0.0f) {
    const float ta = q, tb = c * rcp_k(q);
    const float tr = near ? fminf(ta, tb) : fmaxf(ta, tb);
    if (__builtin_isfinite(tr)) t = tr;
  }
  return t;
}

// executed-work counters of one lane (RT_FLAG_COUNT_WORK builds only)
struct work_ctr {
  uint32_t tests = 0;     // ray-sphere tests
  uint32_t boxes = 0;     // ray-box tests
  uint32_t box_hits = 0;  // ... boxes this lane's own ray entered
  uint32_t roots = 0;     // root/interval sequences the wave ran
};

// One node of the stackless walk: a node is entered if ANY lane's ray meets
// its box (`hit`); an entered leaf scans its one or two pairs.  Returns the
// next node.
// LAYER: lim = min(lim_src, tmax) is refreshed after a leaf (the walk's
// combined far limit).
template <bool OPEN, bool STATS, bool LAYER>
__device__ __forceinline__ int walk_step(const bvh_node &nd, int node, bool hit,
                                         const RT_CONST pair_geom *__restrict__ geom,
                                         const RT_CONST int *__restrict__ orig,
                                         const ray_pre &rp, hit_state &hs, work_ctr &wc, float lim_src,
                                         float &lim) {
  if (STATS) {
    ++wc.boxes;
    wc.box_hits += hit ? 1u : 0u;
  }
  if (!__builtin_amdgcn_ballot_w64(hit)) return nd.skip;
  if (!nd.leaf) return node + 1;
  const int fp = (int)(nd.leaf & ~kTwoPairs) - 1;
  // a leaf of 1-2 spheres scans one pair, not a pair of padding
  if (nd.leaf & kTwoPairs) {
    scan_pairs<OPEN, 2, STATS, LAYER>(geom + fp, 2 * fp, orig, rp, hs, wc.roots);
    if (STATS) wc.tests += 4;
  } else {
    scan_pairs<OPEN, 1, STATS, LAYER>(geom + fp, 2 * fp, orig, rp, hs, wc.roots);
    if (STATS) wc.tests += 2;
  }
  if (LAYER) asm("v_min_f32 %0, %1, %2" : "=v"(lim) : "v"(lim_src), "v"(hs.tmax));
  return nd.skip;
}

// Per-lane 2-D DDA over the layer grid (layer mode): the lane visits the x-z
// cells its own segment crosses inside the layer's y-slab, [ta, tb] clipped to
// the grid box, in order, and tests the spheres listed in each cell with the
// leaf test's arithmetic (NOY fold: same bits as scan_pairs).  It stops once
// the next cell starts beyond min(tb, tmax).  Cell lists hold every sphere
// whose padded box (the BVH's reach) comes within the builder's pad of the
// cell (bvh_builder::build_grid), so the fp32 DDA's boundary errors cannot
// skip a sphere that could win.  Lanes walk independently: the wave runs
// until its last lane is done.
template <bool OPEN, bool STATS, bool GLDS>
__device__ __forceinline__ void grid_walk(float ox, float oz, float ix, float iz, float oix, float oiz,
                                          float ta, float tb, const ray_pre &rl, hit_state &hs,
                                          work_ctr &wc) {
  const kparams p = kernargs();
  // clip to the grid's inner box (the cells around it are an empty ring);
  // slab times as fma(x, 1/d, -o/d) like the BVH's (the ring and the cell
  // lists' pad absorb the rounding)
  const float ax = fmaf(p.grid_xi, ix, oix), bx = fmaf(p.grid_x1, ix, oix);
  const float az = fmaf(p.grid_zi, iz, oiz), bz = fmaf(p.grid_z1, iz, oiz);
  ta = fmaxf(ta, fmaxf(fminf(ax, bx), fminf(az, bz)));
  tb = fminf(tb, fminf(fmaxf(ax, bx), fmaxf(az, bz)));
  if (!(ta <= tb)) return;
  const float dx = rl.dx.x, dz = rl.dz.x;
  const float px = fmaf(ta, dx, ox), pz = fmaf(ta, dz, oz);
  const int nx = p.grid_nx, nz = p.grid_nz;
  int cx = (int)floorf((px - p.grid_x0) * p.grid_invg), cz = (int)floorf((pz - p.grid_z0) * p.grid_invg);
  asm("v_med3_i32 %0, %0, 1, %1" : "+v"(cx) : "s"(nx - 2));
  asm("v_med3_i32 %0, %0, 1, %1" : "+v"(cz) : "s"(nz - 2));
  // step directions from the sign of 1/d (= the sign bit of d, also for -0)
  const bool nxs = ix < 0.0f, nzs = iz < 0.0f;
  float tmx = fmaf(fmaf((float)(cx + (nxs ? 0 : 1)), p.grid_g, p.grid_x0), ix, oix);
  float tmz = fmaf(fmaf((float)(cz + (nzs ? 0 : 1)), p.grid_g, p.grid_z0), iz, oiz);
  const float tdx = p.grid_g * fabsf(ix), tdz = p.grid_g * fabsf(iz);
  // GLDS: items and cells in LDS (ds_read: shorter latency than the L1 path
  // and off the texture pipeline; 166 -> 157 ms)
  const RT_GLOBAL uint32_t *__restrict__ cells = as_global(p.grid_cells);
  const RT_GLOBAL f4 *__restrict__ items = as_global(p.grid_items);
  // GLDS: the walk's cell is the LDS byte address of its start entry, so a
  // DDA step adds +-2 or +-2 nx bytes
  const uint32_t lcells = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint16_t *)
                              reinterpret_cast<const uint16_t *>(s_grid_dyn + p.grid_n_items);
  // The walk stops on time alone: it leaves the inner box only at t ~ tb and
  // the next boundary is a whole cell further, so it never steps past the ring.
  int cell = GLDS ? (int)lcells + 2 * (cz * nx + cx) : cz * nx + cx;
  const int dcx = (nxs ? -1 : 1) * (GLDS ? 2 : 1), dcz = (nzs ? -nx : nx) * (GLDS ? 2 : 1);
  typedef const __attribute__((address_space(3))) uint16_t lds_u16;
  while (true) {
    const uint32_t ce = GLDS ? 0u : cells[(uint32_t)cell];
    const uint32_t first = ce >> 4;
    const uint32_t cnt = GLDS ? 0u : ce & 15u;
    // STATS: boxes = lane-level cell visits; box_hits / roots = wave-level DDA
    // / item iterations (counted once per wave, by its first active lane)
    if (STATS) {
      ++wc.boxes;
      if (!RT_COUNT_ITEMS && lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true))) ++wc.box_hits;
    }
    // items [first, first + cnt).  GLDS: cell i's items are [start_i,
    // start_{i+1}): two ds_read_u16 of adjacent entries give both LDS item
    // addresses, with no decoding (see the block's copy); the loop runs on
    // the item pointer alone, compared with an end the compiler cannot see
    // through (else it rewrites the exit into a separate counter)
    lds_f4 *ip = GLDS ? (lds_f4 *)(uintptr_t)((lds_u16 *)(uintptr_t)cell)[0] : nullptr;
    lds_f4 *ie = GLDS ? (lds_f4 *)(uintptr_t)((lds_u16 *)(uintptr_t)cell)[1] : nullptr;
    if (GLDS) asm volatile("" : "+v"(ie));
    uint32_t k = 0;
    if (GLDS ? ip != ie : cnt != 0) do {
      if (STATS && RT_COUNT_ITEMS == 1 && lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true))) ++wc.box_hits;
      const f4 it = GLDS ? *ip : items[first + k];
      const float h = fmaf(it.y, dz, fmaf(it.x, dx, rl.nk1.x));
      const float g = fmaf(it.y, rl.oz2.x, fmaf(it.x, rl.ox2.x, rl.o2.x));
      const float e = fmaf(h, h, -g);
      if (STATS && RT_COUNT_ITEMS == 2 && __builtin_amdgcn_ballot_w64(e >= it.z) &&
          lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
        ++wc.box_hits;
      // it.w holds tie2_of<false>(index); the open interval's is 0xfffffffe - it
      const uint32_t w = __float_as_uint(it.w);
      candidate<OPEN>(e >= it.z, h, e - it.z, OPEN ? 0xfffffffeu - w : w, hs);
      if (STATS) ++wc.tests;
      ++ip;
      ++k;
    } while (GLDS ? ip != ie : k < cnt);
    // one compare picks the step axis and the next boundary (tmx == tmz
    // steps z, as before); v_min_f32 written out: fminf would first
    // canonicalise its operands
    const bool sx = tmx < tmz;
    const float tnext = sx ? tmx : tmz;
    float lim;
    asm("v_min_f32 %0, %1, %2" : "=v"(lim) : "v"(tb), "v"(hs.tmax));
    if (tnext > lim) break;
    cell += sx ? dcx : dcz;
    if (sx) tmx += tdx;
    else tmz += tdz;
  }
}

// Closest hit of the ray (o, d) over all spheres: hittable_list::hit,
// src/cpu/hittable_list.h:28-43.  Wave-uniform: every active lane of the wave
// calls it together; the result does not depend on which lanes those are.
// The scene parameters are re-read from the kernarg segment on entry
// (kernargs()): they live in SGPRs for the walk only, not across the whole
// bounce loop (SGPR pressure).
template <bool OPEN, bool BVH, bool STATS, bool GRID, bool GLDS>
__device__ __forceinline__ hit_state closest_hit(float ox, float oy, float oz, float dx, float dy, float dz,
                                                 work_ctr &wc) {
  const kparams p = kernargs();
  const RT_CONST pair_geom *__restrict__ scan_geom = as_const(p.scan_geom);
  const RT_CONST pair_geom *__restrict__ geom = as_const(p.geom);
  const RT_CONST bvh_node *__restrict__ nodes = as_const(p.nodes);
  const RT_CONST int *__restrict__ orig = as_const(p.orig);
  const int n_pairs = p.n_pad / 2;
  const float nk1 = -dot3(ox, oy, oz, dx, dy, dz);
  const float o2 = dot3(ox, oy, oz, ox, oy, oz);
  const float ox2 = -2.0f * ox, oy2 = -2.0f * oy, oz2 = -2.0f * oz;
  hit_state hs = no_hit();
  const ray_pre rp{{dx, dx}, {dy, dy}, {dz, dz}, {nk1, nk1},
                   {o2, o2}, {ox2, ox2}, {oy2, oy2}, {oz2, oz2}};
  // the BVH boxes are padded for ray origins within |O| <= oref (see
  // bvh_builder); a wave-step with any lane beyond that scans everything
  const bool scan_all = !BVH || __builtin_amdgcn_ballot_w64(o2 > p.oref2) != 0;
  if (scan_all) {
    // brute force: 8 spheres (4 pairs) per iteration over the whole array
    for (int k = 0; k < n_pairs; k += 4)
      scan_pairs<OPEN, 4, STATS>(scan_geom + k, 2 * k, nullptr, rp, hs, wc.roots);
    if (STATS) wc.tests += 2 * n_pairs;
  } else {
    // wave-uniform stackless BVH walk: a node is entered if ANY lane's ray
    // meets its (conservatively padded) box before that lane's tmax
    // the reciprocals are clamped to +-1e18 (one v_med3): an exactly
    // axis-parallel ray (it happens ~20 times per 4K frame) would otherwise
    // give slab bounds (-inf, inf - inf = NaN), and IEEE min/max then return
    // -inf, culling a box the ray is inside.  With the clamp every slab value
    // is finite; the ray bends by < 1e-14 over any length.
    const float ix = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dx), -1e18f, 1e18f);
    const float iy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dy), -1e18f, 1e18f);
    const float iz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dz), -1e18f, 1e18f);
    const float oix = -ox * ix, oiy = -oy * iy, oiz = -oz * iz;
    // the wave walks the DFS order of its majority direction octant, so
    // coherent rays visit near children first and tmax culls the rest (BVH
    // walks only: the grid build never computes it)
    auto walk_order = [&]() {
      const uint32_t half = __builtin_popcountll(__builtin_amdgcn_ballot_w64(true)) / 2;
      const int oct = (__builtin_popcountll(__builtin_amdgcn_ballot_w64(dx < 0.0f)) > half ? 1 : 0) |
                      (__builtin_popcountll(__builtin_amdgcn_ballot_w64(dy < 0.0f)) > half ? 2 : 0) |
                      (__builtin_popcountll(__builtin_amdgcn_ballot_w64(dz < 0.0f)) > half ? 4 : 0);
      return nodes + (size_t)oct * p.n_nodes;
    };
    const RT_CONST bvh_node *__restrict__ order = GRID ? nullptr : walk_order();
    if (p.layer_mode) {
      // the spheres off the layer (in the final scene the ground and the three
      // big spheres) are scanned first: their hits shorten tmax for the walk
      for (int k = 0; k < p.n_extra_pairs; k += 2) {
        if (GRID)
          scan_pairs_scalar<OPEN, 2, STATS>(geom + p.extra_pair0 + k, 2 * (p.extra_pair0 + k), orig, rp, hs, wc.roots);
        else
          scan_pairs<OPEN, 2, STATS>(geom + p.extra_pair0 + k, 2 * (p.extra_pair0 + k), orig, rp, hs, wc.roots);
      }
      if (STATS) wc.tests += 2 * p.n_extra_pairs;
      // every node's y-range lies inside the layer's: its slab interval is
      // computed once per ray, and a node tests x and z only.  Nodes hold
      // (centre, half-width) per axis: with m = (c - o) / d, the slab is
      // m -+ h |1/d| whatever the sign of d, so x and z share the v_pk_fma_f32s
      // and no min/max orders the slab ends (3 v_pk_fma_f32 + 3 VALU per box
      // instead of 2 + 7)
      const f2 tyl = fma2(p.layer, f2{iy, iy}, f2{oiy, oiy});
      const float tyl_n = fmaxf(fminf(tyl.x, tyl.y), 0.0f);
      const float tyl_f = fmaxf(tyl.x, tyl.y);
      float tyl_fc = fminf(tyl_f, hs.tmax);  // refreshed by walk_step after every leaf
      if (GRID) {  // the layer grid (its own kernel build: no BVH walk code)
        ray_pre rg = rp;
        rg.nk1 = fma2(f2{p.layer_cy, p.layer_cy}, rp.dy, rp.nk1);
        rg.o2 = fma2(f2{p.layer_cy, p.layer_cy}, rp.oy2, rp.o2);
        if (tyl_n <= tyl_fc) grid_walk<OPEN, STATS, GLDS>(ox, oz, ix, iz, oix, oiz, tyl_n, tyl_fc, rg, hs, wc);
        return hs;
      }
      // a wave none of whose rays crosses the layer before tmax skips the walk
      int node = __builtin_amdgcn_ballot_w64(tyl_n <= tyl_fc) ? 0 : p.n_nodes;
      const f2 vi = {ix, iz}, vo = {oix, oiz}, va = {fabsf(ix), fabsf(iz)};
      // leaves: the layer's shared centre y folded into the per-ray terms once
      ray_pre rl = rp;
      rl.nk1 = fma2(f2{p.layer_cy, p.layer_cy}, rp.dy, rp.nk1);
      rl.o2 = fma2(f2{p.layer_cy, p.layer_cy}, rp.oy2, rp.o2);
      while (node < p.n_nodes) {
        const bvh_node nd = cload(order + node);
        // bz is unused here, but naming it keeps the node one s_load_dwordx8
        // (else x2 + x4: measured 1 % slower)
        asm volatile("" ::"s"(nd.bz.x), "s"(nd.bz.y));
        const f2 m = fma2(nd.bx, vi, vo);
        const f2 tn2 = fma2(-nd.by, va, m);
        const f2 tf2 = fma2(nd.by, va, m);
        // v_max3 / v_min3 written out: fmaxf / fminf would first canonicalise
        // the loop-carried operands (extra v_max per node); the compare that
        // follows needs no canonical input
        float tn, tf;
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(tn) : "v"(tn2.x), "v"(tn2.y), "v"(tyl_n));
        asm("v_min3_f32 %0, %1, %2, %3" : "=v"(tf) : "v"(tf2.x), "v"(tf2.y), "v"(tyl_fc));
        node = walk_step<OPEN, STATS, true>(nd, node, tn <= tf, geom, orig, rl, hs, wc, tyl_f, tyl_fc);
      }
    } else if (!GRID) {  // (the grid build runs on layer scenes only)
      const f2 vix = {ix, ix}, viy = {iy, iy}, viz = {iz, iz};
      const f2 vox = {oix, oix}, voy = {oiy, oiy}, voz = {oiz, oiz};
      int node = 0;
      while (node < p.n_nodes) {
        const bvh_node nd = cload(order + node);
        const f2 tx = fma2(nd.bx, vix, vox);
        const f2 ty = fma2(nd.by, viy, voy);
        const f2 tz = fma2(nd.bz, viz, voz);
        const float tn = fmaxf(fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y)), 0.0f);
        const float tf = fminf(fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y)), hs.tmax);
        float unused = 0.0f;
        node = walk_step<OPEN, STATS, false>(nd, node, tn <= tf, geom, orig, rp, hs, wc, 0.0f, unused);
      }
    }
  }
  return hs;
}


// 8 waves per SIMD (<= 64 VGPRs; the layer-grid build uses 61 VGPRs and 72
// SGPRs, and 6 or 7 waves with more registers ran 2 % slower).  The walk is a serial latency
// chain per wave (scalar node load -> slab test -> ballot -> branch), so more
// resident waves keep the VALU busier: 312 vs 322 ms at 7 waves, although the
// 8-wave budget spills a few values (none inside the walk; the pool's
// per-step ones are pinned to VGPRs, see take below).  That
// became possible once the scene pointers and parameters were re-read from
// the kernarg segment where they are used (kernargs(), as_const()) instead of
// being held in SGPRs for the whole kernel: 94 SGPRs + 21 spilled -> 69 at 7
// waves.
template <bool OPEN, bool METAL_UNIT, bool BVH, bool STATS, bool GRID, bool GLDS>
__global__ __launch_bounds__(kBlock, 8) void render_kernel(const kparams p) {
  // Per-lane values that the bounce loop rarely needs are not kept live (VGPR
  // pressure at 8 waves): the wave keeps its tile origin (col0, lrow0, SGPRs),
  // the lane its current pixel slot, sample and global pixel index; column and
  // row are recomputed where they are used.
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6;
  const unsigned bid = p.block_order ? as_const(p.block_order)[blockIdx.x] : blockIdx.x;
  const int unit = (int)(bid % (unsigned)p.units);
  const int tile = (int)(bid / (unsigned)p.units) * kWavesPerBlock + wave;
  const int col0 = (tile % p.tiles_x) * kTile, lrow0 = (tile / p.tiles_x) * kTile;
  // this wave's samples: an even share [unit spp / units, (unit + 1) spp / units)
  const uint32_t s_begin = (uint32_t)((uint64_t)unit * (uint32_t)p.spp / (uint32_t)p.units);
  const uint32_t s_end = (uint32_t)((uint64_t)(unit + 1) * (uint32_t)p.spp / (uint32_t)p.units);
  // The wave's work pool: item k of [0, kend) is sample
  // s_begin + k / 64 of the tile's pixel slot k % 64 (x = slot % 8, y = slot /
  // 8).  A lane whose path ends takes the next item, so no lane idles while
  // the tile has samples left; a pixel's sum is an exact integer, whichever
  // lanes traced its samples in whatever order.
  const uint32_t kend = (s_end > s_begin ? s_end - s_begin : 0u) << 6;
  __shared__ uint32_t s_sum[3][kBlock];                 // the tiles' fixed-point pixel sums
  __shared__ uint32_t s_rowpix[kWavesPerBlock][kTile];  // global pixel index of (x = 0, y)
  bool own_valid;
  {
    const int lane = lane_now();
    const int col = col0 + (lane & (kTile - 1));
    const int lrow = lrow0 + (lane >> 3);
    const int band = lrow / p.row_block;
    const int grow = (band * p.band_stride + p.band_offset) * p.row_block + (lrow - band * p.row_block);
    own_valid = col < p.width && lrow < p.local_rows && grow < p.height;
    if ((lane & (kTile - 1)) == 0) s_rowpix[wave][lane >> 3] = (uint32_t)grow * (uint32_t)p.width + (uint32_t)col0;
  }
  s_sum[0][threadIdx.x] = s_sum[1][threadIdx.x] = s_sum[2][threadIdx.x] = 0u;
  // slots whose pixel is in the frame (all 64 but in the last tile column / row)
  const uint64_t vmask = __builtin_amdgcn_ballot_w64(own_valid);
  if (GLDS) {  // the block's copy of the layer grid (kparams grid_n_items)
    const RT_GLOBAL f4 *gi = as_global(p.grid_items);
    for (int i = (int)threadIdx.x; i < p.grid_n_items; i += kBlock) s_grid_dyn[i] = gi[i];
    uint16_t *sc = reinterpret_cast<uint16_t *>(s_grid_dyn + p.grid_n_items);
    const RT_GLOBAL uint32_t *gc = as_global(p.grid_cells);
    // cell i's items are [start_i, start_{i+1}) (the builder numbers every
    // cell's first item by the running count, ring cells included): the LDS
    // holds each start's LDS byte address, plus the end of the last cell
    const uint32_t base = (uint32_t)(uintptr_t)(lds_f4 *)s_grid_dyn;
    for (int i = (int)threadIdx.x; i <= p.grid_n_cells; i += kBlock)
      sc[i] = (uint16_t)(base + ((i < p.grid_n_cells ? gc[i] >> 4 : (uint32_t)p.grid_n_items) << 4));
    __syncthreads();
  }
  float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 1.f, dz = 0.f;
  float thr = 1.f, thg = 1.f, thb = 1.f;
  int depth = 0;
  uint32_t slot = 0, sample = 0, pix = 0;
  uint32_t segs = 0, steps = 0;
  work_ctr wc;  // executed work, STATS builds only
  // take pool item k: slot, sample and pixel; false if the slot is outside the
  // frame (the lane then stays alive without tracing and takes another item)
  // wave-uniform values the pool reads once per step, held in VGPRs: as SGPRs
  // they were spilled to VGPR lanes at 8 waves (v_readlane per step)
  uint32_t s_begin_v = s_begin;
  uint32_t rowpix_v = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)&s_rowpix[wave][0];
  asm volatile("" : "+v"(s_begin_v), "+v"(rowpix_v));
  auto take = [&](uint32_t k) -> bool {
    slot = k & 63u;
    sample = s_begin_v + (k >> 6);
    pix = ((const __attribute__((address_space(3))) uint32_t *)(uintptr_t)rowpix_v)[slot >> 3] + (slot & (kTile - 1));
    return ((vmask >> slot) & 1u) != 0;
  };
  // (col, global row) of the lane's pixel: col from the tile origin, row by
  // exact division (pix - col) / W
  auto pixel_cr = [&](const kparams &k, int &col, int &grow) {
    col = col0 + (int)(slot & (kTile - 1));
    grow = (int)(((pix - (uint32_t)col) >> k.wshift) * k.winv);
  };
  uint32_t knext = 64;  // the pool's next item (wave-uniform); lane l starts with item l
  bool alive = kend != 0 && p.max_depth > 0;  // depth 0: black, no hit test
  bool tracing = false;
  if (alive) {
    tracing = take((uint32_t)lane_now());
    if (tracing) {
      int col, grow;
      pixel_cr(p, col, grow);
      camera_ray(p, pcg4d(pix, sample, 0u, p.seed32), col, grow, ox, oy, oz, dx, dy, dz);
    }
  }

  while (true) {
    if (!__ballot(alive)) break;
    hit_state hs = no_hit();
    if (tracing) hs = closest_hit<OPEN, BVH, STATS, GRID, GLDS>(ox, oy, oz, dx, dy, dz, wc);
    ++steps;
    const int best = best_of<OPEN>(hs);
    // lanes that end their path here (a miss) or hold a slot outside the frame
    // take their next items now: the step's one hash then draws the new camera ray
    const bool miss = alive && (!tracing || best < 0);
    uint32_t kn;
    {
      const uint64_t need = __builtin_amdgcn_ballot_w64(miss);
      kn = knext + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      knext += (uint32_t)__builtin_popcountll(need);
    }
    bool path_done = false;  // absorbed, or the bounce limit: the lane parks for a step
    if (alive) {
      const kparams q = kernargs();  // shading's parameters, re-read per step
      if (tracing) ++segs;
      if (tracing && best < 0) {
        // miss: sky gradient, src/cpu/main.cc:27-29; the sample's radiance
        // goes into its pixel's fixed-point sum
        const float a = 0.5f * (dy + 1.0f);
        const float s0 = 1.0f - a;
        const int i = wave * 64 + (int)slot;
        atomicAdd(&s_sum[0][i], (uint32_t)(thr * fmaf(a, 0.5f, s0) * q.qscale));
        atomicAdd(&s_sum[1][i], (uint32_t)(thg * fmaf(a, 0.7f, s0) * q.qscale));
        atomicAdd(&s_sum[2][i], (uint32_t)(thb * (s0 + a) * q.qscale));
      }
      if (miss) {
        if (kn < kend) {
          tracing = take(kn);
        } else {
          alive = tracing = false;
        }
      }
      // One hash per lane and step: a hit draws its bounce, pcg4d(pix, sample,
      // depth + 1); a lane that took a new item draws its camera ray, pcg4d(pix,
      // sample, 0) (only absorbed paths need a second hash below)
      const uint4 r = pcg4d(pix, sample, miss ? 0u : (uint32_t)(depth + 1), q.seed32);
      // one polar draw per lane and step: a hit's unit vector (oracle unit_vec:
      // z = 1 - 2 u1), a new camera ray's lens sample
      const float uz = fmaf(-2.0f, unif(r.x), 1.0f);
      float ux, uy;
      polar(miss ? unif(r.z) : fmaf(-uz, uz, 1.0f), unif(miss ? r.w : r.y), ux, uy);

      if (!miss) {
        const float o2 = dot3(ox, oy, oz, ox, oy, oz);
        const float ox2 = -2.0f * ox, oy2 = -2.0f * oy, oz2 = -2.0f * oz;
        const float tmax = hs.tmax;
        const bool near = near_of(hs) != 0;
        const shade_rec sr = cload_g(as_global(q.shade) + best);
        float b;
        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b);
        // A refined root before t_min on a sphere the ray moves away from
        // (b > 0): the ray starts on that sphere and leaves its ball, which it
        // cannot meet again; the expanded quadratic's root was an fp32 artefact
        // (DESIGN.md 2, step 3).  Not a segment: the ray moves on to the
        // scan's root point, same direction, and walks again.
        if (t < 0.001f && b > 0.0f) {
          ox = fmaf(tmax, dx, ox);
          oy = fmaf(tmax, dy, oy);
          oz = fmaf(tmax, dz, oz);
          --segs;
        } else {
        const float px = fmaf(t, dx, ox), py = fmaf(t, dy, oy), pz = fmaf(t, dz, oz);
        float nx = (px - sr.cx) * sr.inv_r, ny = (py - sr.cy) * sr.inv_r, nz = (pz - sr.cz) * sr.inv_r;
        // set_face_normal (hittable.h:16-19): dot(d, outward) < 0 is, in exact
        // arithmetic, "the entering root was taken" (outward flips for r < 0);
        // the root form cannot flip sign at grazing incidence in fp32
        const bool front = near != (sr.inv_r < 0.0f);
        if (!front) {
          nx = -nx;
          ny = -ny;
          nz = -nz;
        }
        // shared by the material branches (computed once: lanes of one wave
        // usually hit several materials, so the branches all execute)
        const float dn = dot3(dx, dy, dz, nx, ny, nz);
        float rx, ry, rz;
        reflect3(dx, dy, dz, nx, ny, nz, dn, rx, ry, rz);
        float sx, sy, sz;
        bool scattered = true;
        if (sr.kind == RT_LAMBERTIAN) {
          // material.h:19-30
          sx = nx + ux;
          sy = ny + uy;
          sz = nz + uz;
          const float e = 1e-8f;
          if (fabsf(sx) < e && fabsf(sy) < e && fabsf(sz) < e) {
            sx = nx;
            sy = ny;
            sz = nz;
          }
        } else if (sr.kind == RT_METAL) {
          // material.h:40-46
          float fz = sr.param;
          if (!METAL_UNIT) fz *= ball_radius(r);  // random_in_unit_sphere
          sx = fmaf(fz, ux, rx);
          sy = fmaf(fz, uy, ry);
          sz = fmaf(fz, uz, rz);
          scattered = dot3(sx, sy, sz, nx, ny, nz) > 0.0f;
        } else {
          // dielectric, material.h:57-87 (r0 is the same for ior and 1/ior)
          const float ratio = front ? sr.inv_param : sr.param;
          const float cos_t = fminf(-dn, 1.0f);
          // ratio sin > 1 (material.h:64), squared: no square root
          const bool cannot = (ratio * ratio) * fmaf(-cos_t, cos_t, 1.0f) > 1.0f;
          if (cannot || schlick(cos_t, sr.r0) > unif(r.x)) {
            sx = rx;
            sy = ry;
            sz = rz;
          } else {
            refract3(dx, dy, dz, nx, ny, nz, cos_t, ratio, sx, sy, sz);
          }
        }
        // attenuation = albedo (dielectrics store 1,1,1: the product is exact)
        thr *= sr.ar;
        thg *= sr.ag;
        thb *= sr.ab;
        ++depth;
        if (!scattered || depth >= q.max_depth) {
          path_done = true;  // absorbed, or bounce limit (main.cc:16-17): black
        } else {
          ox = px;
          oy = py;
          oz = pz;
          dx = sx;  // normalised below, with the new camera rays
          dy = sy;
          dz = sz;
        }
        }
      } else if (tracing) {
        // a new item: its camera ray, with the lens sample drawn above
        int col, grow;
        pixel_cr(q, col, grow);
        camera_dir(q, r, ux, uy, col, grow, ox, oy, oz, dx, dy, dz);
        depth = 0;
        thr = thg = thb = 1.0f;
      }
    }
    // an absorbed path, or one at the bounce limit, parks its lane for a
    // step: the lane takes its next item with the misses of the next step
    // (one camera-ray path per step, with the step's one hash)
    if (path_done) tracing = false;
    // one normalize3 per lane and step: the bounce direction or the new
    // camera ray's (a finished lane's is unused)
    if (alive) normalize3(dx, dy, dz);
  }

  const int lane = lane_now();
  {
    const kparams q = kernargs();
    const int col = col0 + (lane & (kTile - 1)), lrow = lrow0 + (lane >> 3);
    if (col < q.width && lrow < q.local_rows) {  // padding pixels (row >= height) write zeros
      const size_t o = 3 * ((size_t)lrow * q.width + col);
      const int i = wave * 64 + lane;
      if (q.units == 1) {
        RT_GLOBAL float *out = as_global(q.out) + o;
        out[0] = (float)s_sum[0][i] * q.qinv;
        out[1] = (float)s_sum[1][i] * q.qinv;
        out[2] = (float)s_sum[2][i] * q.qinv;
      } else {  // the tile's units add their integer sums (finish_sums converts)
        uint32_t *acc = reinterpret_cast<uint32_t *>(q.out) + o;
        atomicAdd(acc + 0, s_sum[0][i]);
        atomicAdd(acc + 1, s_sum[1][i]);
        atomicAdd(acc + 2, s_sum[2][i]);
      }
    }
  }
  // one atomic per wave for the counters
  uint32_t s = segs;
  uint64_t lt = wc.tests, lb = wc.boxes, lh = wc.box_hits, lr = wc.roots;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    if (STATS) {
      lt += __shfl_xor(lt, off);
      lb += __shfl_xor(lb, off);
      lh += __shfl_xor(lh, off);
      lr += __shfl_xor(lr, off);
    }
  }
  if (lane == 0) {
    if (STATS) {  // pilot renders (units = 1, launch order): segments per tile
      const kparams k = kernargs();
      if (k.tile_cost) {
        // and nothing else: 6 same-address atomics from each of ~10^5 short
        // waves serialise (the 4-spp pilot took 9.5 ms instead of ~1.2)
        k.tile_cost[(int)blockIdx.x * kWavesPerBlock + wave] = s;
        return;
      }
    }
    unsigned long long *counters = kernargs().counters + 8 * (blockIdx.x & (kCounterSlots - 1));
    atomicAdd(&counters[0], (unsigned long long)s);
    atomicAdd(&counters[1], (unsigned long long)steps);
    if (STATS) {
      atomicAdd(&counters[2], (unsigned long long)lt);
      atomicAdd(&counters[3], (unsigned long long)lb);
      atomicAdd(&counters[4], (unsigned long long)lh);
      atomicAdd(&counters[5], (unsigned long long)lr);
    }
  }
}

// Several waves per tile (rt_params.units > 1): they added their integer pixel
// sums into the frame (zeroed first), which holds uint32 sums until this pass
// converts them in place, sum * 2^-F.  Memory-bound and tiny.
__global__ __launch_bounds__(256) void finish_sums(uint32_t *__restrict__ frame, uint64_t n, float qinv) {
  // every access goes through the uint32 view: the float result is stored as its bits
  for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256u)
    frame[j] = __float_as_uint((float)frame[j] * qinv);
}

// Known-answer evaluation of the render kernel's own device arithmetic
// (rt_device_kat; tests/test_parity_gpu.py checks it against the reference's
// vectors in tests/golden/kat.jsonl).  Case layout: 10 doubles in, 9 out.
//   RT_KAT_SPHERE_HIT  in  o[3] d[3] c[3] r      (sphere::hit, src/cpu/sphere.h:24-51,
//                                                  t_min 0.001, t_max inf)
//                      out hit, t (in units of the given d), p[3], normal[3], front_face
//                      -- the scan's candidate test, refine_root, the shading normal
//                      and set_face_normal, exactly as render_kernel runs them on a
//                      direction normalised by normalize3
//   RT_KAT_REFLECT     in  v[3] n[3]             out reflect3(v, n)
//   RT_KAT_REFRACT     in  v[3] n[3] eta         out refract3(v, n, eta)
//   RT_KAT_REFLECTANCE in  cosine ref_idx        out schlick(cosine, r0(ref_idx))
__global__ __launch_bounds__(64) void kat_kernel(int kind, const double *__restrict__ in, int n,
                                                 double *__restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const double *a = in + 10 * (size_t)i;
  double *o = out + 9 * (size_t)i;
  for (int k = 0; k < 9; ++k) o[k] = 0.0;
  if (kind == RT_KAT_SPHERE_HIT) {
    const float ox = (float)a[0], oy = (float)a[1], oz = (float)a[2];
    float dx = (float)a[3], dy = (float)a[4], dz = (float)a[5];
    const double len = sqrt(a[3] * a[3] + a[4] * a[4] + a[5] * a[5]);
    normalize3(dx, dy, dz);
    shade_rec sr;
    sr.cx = (float)a[6];
    sr.cy = (float)a[7];
    sr.cz = (float)a[8];
    sr.radius = (float)a[9];
    sr.inv_r = 1.0f / sr.radius;
    const double cx = sr.cx, cy = sr.cy, cz = sr.cz, rr = sr.radius;
    sr.ks = (float)(cx * cx + cy * cy + cz * cz - rr * rr);  // as rt_scene_upload
    const float nk1 = -dot3(ox, oy, oz, dx, dy, dz);
    const float o2 = dot3(ox, oy, oz, ox, oy, oz);
    const float ox2 = -2.0f * ox, oy2 = -2.0f * oy, oz2 = -2.0f * oz;
    const float h = fmaf(sr.cz, dz, fmaf(sr.cx, dx, fmaf(sr.cy, dy, nk1)));
    const float g = fmaf(sr.cz, oz2, fmaf(sr.cx, ox2, fmaf(sr.cy, oy2, o2)));
    const float e = fmaf(h, h, -g);
    hit_state hs = no_hit();
    candidate<false>(e >= sr.ks, h, e - sr.ks, tie2_of<false>(0u), hs);
    if (best_of<false>(hs) < 0) return;
    float b_unused;
    const float t = refine_root(sr, hs.tmax, near_of(hs) != 0, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b_unused);
    const float px = fmaf(t, dx, ox), py = fmaf(t, dy, oy), pz = fmaf(t, dz, oz);
    float nx = (px - sr.cx) * sr.inv_r, ny = (py - sr.cy) * sr.inv_r, nz = (pz - sr.cz) * sr.inv_r;
    const bool front = (near_of(hs) != 0) != (sr.inv_r < 0.0f);
    if (!front) {
      nx = -nx;
      ny = -ny;
      nz = -nz;
    }
    o[0] = 1.0;
    o[1] = (double)t / len;
    o[2] = px;
    o[3] = py;
    o[4] = pz;
    o[5] = nx;
    o[6] = ny;
    o[7] = nz;
    o[8] = front ? 1.0 : 0.0;
  } else if (kind == RT_KAT_REFLECT || kind == RT_KAT_REFRACT) {
    const float vx = (float)a[0], vy = (float)a[1], vz = (float)a[2];
    const float nx = (float)a[3], ny = (float)a[4], nz = (float)a[5];
    float x, y, z;
    if (kind == RT_KAT_REFLECT) {
      reflect3(vx, vy, vz, nx, ny, nz, dot3(vx, vy, vz, nx, ny, nz), x, y, z);
    } else {
      const float cos_t = fminf(-dot3(vx, vy, vz, nx, ny, nz), 1.0f);
      refract3(vx, vy, vz, nx, ny, nz, cos_t, (float)a[6], x, y, z);
    }
    o[0] = x;
    o[1] = y;
    o[2] = z;
  } else if (kind == RT_KAT_REFLECTANCE) {
    const double r0 = (1.0 - a[1]) / (1.0 + a[1]);  // as rt_scene_upload's shade_rec.r0
    o[0] = schlick((float)a[0], (float)(r0 * r0));
  }
}

// write_color on the device (rt_tonemap_async): the level of a channel is
// (int)(256 * clamp(sqrt(sum * scale), 0, 0.999)) in fp64 with scale = 1.0 / spp
// (src/cpu/color.h:8-23), or in fp32 with scale = 1.0f / spp
// (src/gpu/color.h:16-38).  sqrt is monotone, so the level is the number of
// thresholds T[k] = min{q : sqrt_rn(q) >= k / 256}, k = 1..255, that q = sum *
// scale reaches (tonemap_thresholds, on the host with its correctly rounded
// sqrt).  The device estimates the level with its own sqrt and corrects it by
// one step against T: the result does not depend on how the device rounds
// sqrt.  NaN sums map to 0 (rt_tonemap_u8 does the same).  Four channels per
// lane: one 16-B load, one 4-B store (HBM-bound, 15 B per pixel).
template <bool FP32, typename T>
__device__ __forceinline__ uint32_t tone_level(float s, T scale, const T *__restrict__ thr) {
  const T q = (T)s * scale;
  const T y = (T)256 * (FP32 ? (T)sqrtf((float)q) : (T)sqrt((double)q));
  int l = y >= (T)255 ? 255 : (y > (T)0 ? (int)y : 0);
  if (l < 255 && q >= thr[l + 1]) ++l;
  else if (l > 0 && q < thr[l]) --l;
  return (uint32_t)l;
}

template <bool FP32, typename T>
__global__ __launch_bounds__(256) void tonemap_kernel(const float *__restrict__ sums, uint64_t n, T scale,
                                                      const T *__restrict__ thr_g, uint8_t *__restrict__ out) {
  __shared__ T thr[256];
  thr[threadIdx.x] = thr_g[threadIdx.x];
  __syncthreads();
  const uint64_t n4 = n / 4;
  const bool vec = ((uintptr_t)sums % 16 == 0) && ((uintptr_t)out % 4 == 0);
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  if (vec) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n4; i += stride) {
      const f4 v = reinterpret_cast<const f4 *>(sums)[i];
      reinterpret_cast<uint32_t *>(out)[i] =
          tone_level<FP32, T>(v.x, scale, thr) | tone_level<FP32, T>(v.y, scale, thr) << 8 |
          tone_level<FP32, T>(v.z, scale, thr) << 16 | tone_level<FP32, T>(v.w, scale, thr) << 24;
    }
  }
  for (uint64_t i = (vec ? 4 * n4 : 0) + (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += stride)
    out[i] = (uint8_t)tone_level<FP32, T>(sums[i], scale, thr);
}

}  // namespace rtk

// ------------------------------------------------------------ context ----
struct rt_context {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  rtk::pair_geom *d_geom = nullptr;      // brute-force order
  rtk::pair_geom *d_bvh_geom = nullptr;  // BVH leaf order
  rtk::bvh_node *d_nodes = nullptr;
  int *d_orig = nullptr;                 // BVH slot -> original index (-1 = padding)
  rtk::shade_rec *d_shade = nullptr;
  uint32_t n_spheres = 0, n_pad = 0, n_nodes = 0, n_bvh_slots = 0;
  float oref2 = 0.0f;
  bool layer_mode = false;
  float layer_lo = 0.0f, layer_hi = 0.0f, layer_cy = 0.0f;
  uint32_t extra_pair0 = 0, n_extra_pairs = 0;
  uint32_t *d_grid_cells = nullptr;  // layer grid (nullptr: none)
  float *d_grid_items = nullptr;
  size_t grid_n_items = 0;
  bool grid_lds = false;  // the grid fits the LDS budget (render_kernel GLDS builds)
  float grid_x0 = 0, grid_z0 = 0, grid_xi = 0, grid_zi = 0, grid_x1 = 0, grid_z1 = 0, grid_g = 0;
  int grid_nx = 0, grid_nz = 0;
  unsigned long long *d_counters = nullptr;
  float *d_frame = nullptr;
  size_t frame_floats = 0;
  // block schedule from a pilot render, cached per frame geometry
  uint32_t *d_order = nullptr;
  size_t order_n = 0;
  std::vector<uint64_t> order_key;
  uint64_t last_samples = 0;
  bool last_stats = false;
  // Renders of one context may be enqueued on different streams; they share
  // the scratch buffer above (block order), so each render first
  // waits for the previous one: ev_done is recorded after every render on
  // last_stream, and a render on another stream waits on it (no host sync).
  hipEvent_t ev_done = nullptr;
  hipStream_t last_stream = nullptr;
  bool have_done = false;
  double tonemap_thr64[257];  // rt_tonemap_async level thresholds (see tonemap_thresholds)
  float tonemap_thr32[257];
  double *d_thr64 = nullptr;
  float *d_thr32 = nullptr;
};

namespace {

int hip_fail(hipError_t e) {
  rt_internal_set_hip_error((int)e);
  return RT_ERR_HIP;
}

// T[k] = the smallest q >= 0 whose correctly rounded square root reaches
// k / 256 (k = 1..255; T[0] unused), in fp64 and in fp32.  (k / 256)^2 is
// exact in both; step down while the square root still rounds up to k / 256.
void tonemap_thresholds(double *t64, float *t32) {
  t64[0] = 0.0;
  t32[0] = 0.0f;
  for (int k = 1; k < 256; ++k) {
    const double x = k / 256.0;
    double q = x * x;
    while (q > 0.0 && std::sqrt(std::nextafter(q, 0.0)) >= x) q = std::nextafter(q, 0.0);
    t64[k] = q;
    const float xf = (float)k / 256.0f;
    float qf = xf * xf;
    while (qf > 0.0f && std::sqrt(std::nextafter(qf, 0.0f)) >= xf) qf = std::nextafter(qf, 0.0f);
    t32[k] = qf;
  }
  t64[256] = INFINITY;
  t32[256] = INFINITY;
}

#define RT_HIP(call)                         \
  do {                                       \
    hipError_t _e = (call);                  \
    if (_e != hipSuccess) return hip_fail(_e); \
  } while (0)

bool params_ok(const rt_params *p) {
  return p && p->width >= 1 && p->height >= 1 && p->spp >= 0 && p->spp < (1 << 24) &&
         p->max_depth >= 0 && p->max_depth < (1 << 24) &&
         p->row_block >= 1 && p->band_stride >= 1 && p->band_offset >= 0 &&
         p->band_offset < p->band_stride && p->local_rows >= 0 &&
         (uint64_t)p->width * (uint64_t)p->height < (1ull << 32);
}

// ---------------------------------------------------------- BVH build ----
// Binary BVH over the spheres' boxes, full-sweep SAH on centroids (O(n log^2 n),
// 10k spheres in a few ms), leaves of <= 4 spheres padded to 2 pairs, nodes in
// DFS pre-order with skip links for the stackless wave-uniform walk.
//
// Conservativeness.  The walk must never skip a sphere whose COMPUTED scan
// root would win, or the result would differ from the brute-force scan.  The
// scan's hit point P = O + t d satisfies |P - C|^2 = r^2 + (disc_computed -
// disc_exact), and the expanded quadratic's discriminant error is bounded by
// ~12 roundings of magnitude (|C| + |O|)^2, i.e. < 2^-19 (|C| + |O|)^2.  So
// each sphere's box is C +- sqrt(r^2 + 2^-19 (|C| + oref)^2), valid for ray
// origins |O| <= oref (the kernel scans everything for a wave-step that has
// any lane beyond oref), and node boxes get a further relative 2^-18 plus an
// outward fp32 rounding to cover the slab test's own rounding.
struct bvh_builder {
  struct box {
    double lo[3], hi[3];
  };
  std::vector<box> sb;             // per-sphere boxes
  std::vector<double> cen;         // centroids, 3 per sphere
  std::vector<uint32_t> ord;       // sphere order being partitioned
  std::vector<rtk::bvh_node> nodes;
  std::vector<int> slots;          // slot -> original index, -1 padding
  static constexpr int kLeaf = 2 * rtk::kLeafPairs;
  // tuning knobs, read once per build (A/B experiments; defaults measured best)
  int max_leaf = env_int("RTOW_BVH_LEAF", kLeaf, 1, kLeaf);
  double collapse_area = env_double("RTOW_BVH_COLLAPSE", 0.35);
  double side_weight = env_double("RTOW_BVH_SIDE", 1.0);  // SAH weight of the x- and z-facing sides
  static int env_int(const char *name, int dflt, int lo, int hi) {
    const char *v = std::getenv(name);
    return v ? std::max(lo, std::min(hi, std::atoi(v))) : dflt;
  }
  // experiment knobs: only a finite value in [lo, hi] is taken, anything else
  // (unset, garbage, 0, negative, NaN, inf) keeps the default
  static double env_double(const char *name, double dflt, double lo = 0.01, double hi = 100.0) {
    const char *v = std::getenv(name);
    if (!v) return dflt;
    char *end = nullptr;
    const double x = std::strtod(v, &end);
    return (end != v && std::isfinite(x) && x >= lo && x <= hi) ? x : dflt;
  }

  double area(const box &b) const {
    const double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return side_weight * (dx * dy + dy * dz) + dz * dx;
  }
  static void grow(box &a, const box &b) {
    for (int k = 0; k < 3; ++k) {
      a.lo[k] = std::min(a.lo[k], b.lo[k]);
      a.hi[k] = std::max(a.hi[k], b.hi[k]);
    }
  }
  static box empty() {
    box b;
    for (int k = 0; k < 3; ++k) {
      b.lo[k] = 1e300;
      b.hi[k] = -1e300;
    }
    return b;
  }
  // a node box's axis k as emitted: padded, rounded outward (monotonic in
  // the box, so a sub-box's emitted range lies inside its parent's)
  static void emit_axis(const box &b, int k, float &lo, float &hi) {
    const double m = std::max(std::fabs(b.lo[k]), std::fabs(b.hi[k]));
    const double pad = 0x1p-18 * (m + (b.hi[k] - b.lo[k])) + 1e-6;
    lo = std::nextafter((float)(b.lo[k] - pad), -INFINITY);
    hi = std::nextafter((float)(b.hi[k] + pad), INFINITY);
  }
  void set_box(rtk::bvh_node &nd, const box &b) {
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) emit_axis(b, k, lo[k], hi[k]);
    nd.bx[0] = lo[0];
    nd.bx[1] = hi[0];
    nd.by[0] = lo[1];
    nd.by[1] = hi[1];
    nd.bz[0] = lo[2];
    nd.bz[1] = hi[2];
  }
  // tree in memory; emitted afterwards in 8 DFS orders (one per direction
  // octant, near child first along the node's split axis)
  struct tnode {
    box b;
    int axis = 0;
    int left = -1, right = -1;
    uint32_t leaf = 0;  // 1 + first pair, or 0
  };
  std::vector<tnode> tree;
  int build(uint32_t b, uint32_t e) {
    const int id = (int)tree.size();
    tree.push_back(tnode{});
    box all = empty();
    for (uint32_t i = b; i < e; ++i) grow(all, sb[ord[i]]);
    tree[id].b = all;
    const uint32_t n = e - b;
    if (n <= (uint32_t)max_leaf) {
      const uint32_t first_slot = (uint32_t)slots.size();
      const uint32_t width = n <= 2 ? 2u : (uint32_t)kLeaf;  // one pair or two
      for (uint32_t i = b; i < e; ++i) slots.push_back((int)ord[i]);
      while (slots.size() < first_slot + width) slots.push_back(-1);
      tree[id].leaf = (first_slot / 2 + 1) | (width == 4 ? rtk::kTwoPairs : 0u);
      return id;
    }
    // SAH over the 3 axes, sweeping sorted centroids (ties: original index)
    double best_cost = 1e300;
    int best_axis = 0;
    uint32_t best_split = b + n / 2;
    std::vector<double> left(n);
    for (int ax = 0; ax < 3; ++ax) {
      std::sort(ord.begin() + b, ord.begin() + e, [&](uint32_t x, uint32_t y) {
        const double cx = cen[3 * x + ax], cy = cen[3 * y + ax];
        return cx < cy || (cx == cy && x < y);
      });
      box acc = empty();
      for (uint32_t i = 0; i < n; ++i) {
        grow(acc, sb[ord[b + i]]);
        left[i] = area(acc);
      }
      acc = empty();
      for (uint32_t i = n - 1; i >= 1; --i) {
        grow(acc, sb[ord[b + i]]);
        // split before i: left = [0, i), right = [i, n).  Spheres are tested
        // in pairs (one v_pk_fma_f32 chain per pair), so a subtree costs its
        // area times its pair count, ceil(count / 2): 3 spheres cost as much
        // as 4, and splits into even counts are preferred (397 vs 412 ms)
        const double cost = left[i - 1] * ((i + 1) / 2) + area(acc) * ((n - i + 1) / 2);
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = ax;
          best_split = b + i;
        }
      }
    }
    std::sort(ord.begin() + b, ord.begin() + e, [&](uint32_t x, uint32_t y) {
      const double cx = cen[3 * x + best_axis], cy = cen[3 * y + best_axis];
      return cx < cy || (cx == cy && x < y);
    });
    const int l = build(b, best_split);
    const int r = build(best_split, e);
    tree[id].axis = best_axis;
    tree[id].left = l;
    tree[id].right = r;
    return id;
  }
  // Collapsed internal nodes get no box of their own: their children take
  // their place in the DFS order (a wider tree; the stackless walk handles any
  // arity).  A wave enters a node when ANY of its 64 rays meets the box, so
  // node entry rates are high (60-94 % per level measured, tools/node_stats.py)
  // and the box tests of nodes a wave almost always enters are wasted:
  // collapsing X saves tests(X) and costs (tests(X) - enters(X)) per child.
  // Rule: collapse the root and every internal node whose surface area is more
  // than collapse_area (0.35) of its nearest emitted ancestor's (461 ->
  // 417 ms on the headline frame, neutral on the 10 000-sphere scene).  The
  // walk stays conservative: a parent's box contains its children's.

  bool collapsed(int t, int parent) const {
    if (tree[t].leaf) return false;
    if (t == 0) return true;  // the root (build() returns 0 for it): always entered
    // the root's children have no emitted ancestor: they stay
    return parent >= 0 && area(tree[t].b) > collapse_area * area(tree[parent].b);
  }
  // DFS pre-order for octant oct (bit k set = direction negative along axis k):
  // a ray moving towards -axis meets the upper (right) child first
  // (parent: nearest emitted ancestor, -1 at the root)
  void emit(int t, int oct, size_t base, int parent = -1) {
    const tnode &tn = tree[t];
    if (collapsed(t, parent)) {
      const bool neg = (oct >> tn.axis) & 1;
      emit(neg ? tn.right : tn.left, oct, base, parent);
      emit(neg ? tn.left : tn.right, oct, base, parent);
      return;
    }
    const size_t id = nodes.size();
    nodes.push_back(rtk::bvh_node{});
    if (tn.leaf) {
      rtk::bvh_node &nd = nodes[id];
      set_box(nd, tn.b);
      nd.skip = (int32_t)(id + 1 - base);
      nd.leaf = tn.leaf;
      return;
    }
    const bool neg = (oct >> tn.axis) & 1;
    emit(neg ? tn.right : tn.left, oct, base, t);
    emit(neg ? tn.left : tn.right, oct, base, t);
    rtk::bvh_node &nd = nodes[id];
    set_box(nd, tn.b);
    nd.skip = (int32_t)(nodes.size() - base);
    nd.leaf = 0;
  }
  // Layer-mode node: the emitted x and z slabs [lo, hi] as (centre, half-width),
  // bx = (cx, cz), by = (hx, hz).  The walk evaluates m = fma(c, 1/d, -o/d),
  // m -+ fma(h, |1/d|): three roundings of magnitude <= (|o| + |c - o| + h) |1/d|
  // against two for fma(lo, 1/d, -o/d), so h also covers |c - float(c)| and
  // 2^-22 (3 oref + 2|c| + h) on top of the (lo, hi) padding.
  void to_centre_form(rtk::bvh_node &nd) const {
    float c[2], h[2];
    const float lo[2] = {nd.bx[0], nd.bz[0]}, hi[2] = {nd.bx[1], nd.bz[1]};
    for (int k = 0; k < 2; ++k) {
      const double cd = 0.5 * ((double)lo[k] + (double)hi[k]);
      const double hd = 0.5 * ((double)hi[k] - (double)lo[k]);
      c[k] = (float)cd;
      const double cover = hd + std::fabs(cd - (double)c[k]) +
                           0x1p-22 * (3.0 * oref + 2.0 * std::fabs(cd) + hd);
      h[k] = std::nextafter((float)cover, INFINITY);
    }
    nd.bx[0] = c[0];
    nd.bx[1] = c[1];
    nd.by[0] = h[0];
    nd.by[1] = h[1];
    nd.bz[0] = nd.bz[1] = 0.0f;
  }
  size_t per_order = 0;
  // oref: the ray-origin bound the padding is valid for -- 64 or 16 beyond the
  // farthest sphere of radius <= 10, whichever is larger (the huge ground
  // sphere does not count: rays only start on its visible cap)
  static double origin_bound(const rt_scene_view *s) {
    double far = 0.0;
    for (uint32_t i = 0; i < s->n; ++i) {
      const double r = std::fabs((double)s->radius[i]);
      if (r > 10.0) continue;
      const double c = std::sqrt((double)s->cx[i] * s->cx[i] + (double)s->cy[i] * s->cy[i] +
                                 (double)s->cz[i] * s->cz[i]);
      far = std::max(far, c + r);
    }
    return std::max(64.0, far + 16.0);
  }
  double oref = 64.0;
  void run(const rt_scene_view *s) {
    const uint32_t n = s->n;
    oref = origin_bound(s);
    sb.resize(n);
    cen.resize(3 * (size_t)n);
    ord.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
      const double c[3] = {s->cx[i], s->cy[i], s->cz[i]};
      const double r = std::fabs((double)s->radius[i]);
      const double cn = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
      const double reach = std::sqrt(r * r + 0x1p-19 * (cn + oref) * (cn + oref));
      for (int k = 0; k < 3; ++k) {
        sb[i].lo[k] = c[k] - reach;
        sb[i].hi[k] = c[k] + reach;
        cen[3 * i + k] = c[k];
      }
      ord[i] = i;
    }
    if (!n) return;
    const uint32_t n_tree = split_layer(s);
    build(0, n_tree);
    for (int oct = 0; oct < 8; ++oct) emit(0, oct, nodes.size());
    per_order = nodes.size() / 8;
    if (layer_mode) {
      float lo, hi;
      emit_axis(tree[0].b, 1, lo, hi);  // contains every node's y-range
      layer_lo = lo;
      layer_hi = hi;
      for (rtk::bvh_node &nd : nodes) to_centre_form(nd);
      extra_pair0 = (uint32_t)slots.size() / 2;  // leaves end on a pair boundary
      for (uint32_t i = n_tree; i < n; ++i) slots.push_back((int)ord[i]);
      // padded to whole groups of two pairs: the kernel scans them two at a
      // time (one s_load_dwordx16, two independent chains)
      while ((slots.size() - 2 * extra_pair0) % 4) slots.push_back(-1);
      n_extra_pairs = (uint32_t)slots.size() / 2 - extra_pair0;
      build_grid(s, n_tree);
    }
  }
  // Layer grid: square x-z cells of side g over the layer spheres' padded
  // boxes; a cell lists every layer sphere whose padded box comes within pad
  // of it.  g is chosen for ~1 sphere per cell (RTOW_GRID_SCALE scales it);
  // cells list at most 15 spheres (else g shrinks).
  std::vector<uint32_t> grid_cells;
  std::vector<float> grid_items;  // 4 floats per item
  float grid_x0 = 0, grid_z0 = 0, grid_xi = 0, grid_zi = 0, grid_x1 = 0, grid_z1 = 0, grid_g = 0;
  int grid_nx = 0, grid_nz = 0;
  void build_grid(const rt_scene_view *s, uint32_t n_tree) {
    double x0 = 1e300, x1 = -1e300, z0 = 1e300, z1 = -1e300;
    for (uint32_t k = 0; k < n_tree; ++k) {
      const uint32_t i = ord[k];
      x0 = std::min(x0, sb[i].lo[0]);
      x1 = std::max(x1, sb[i].hi[0]);
      z0 = std::min(z0, sb[i].lo[2]);
      z1 = std::max(z1, sb[i].hi[2]);
    }
    const double pad = 0x1p-10 * std::max(1.0, std::max(x1 - x0, z1 - z0) / 32.0);
    x0 -= 2 * pad;
    z0 -= 2 * pad;
    x1 += 2 * pad;
    z1 += 2 * pad;
    const double scale = env_double("RTOW_GRID_SCALE", 1.0, 0.05, 20.0);
    double g = scale * std::sqrt((x1 - x0) * (z1 - z0) / (double)n_tree);
    for (int attempt = 0; attempt < 8; ++attempt, g *= 0.8) {
      const int nx = (int)std::ceil((x1 - x0) / g), nz = (int)std::ceil((z1 - z0) / g);
      if ((long long)nx * nz > (1 << 20)) return;
      std::vector<std::vector<uint32_t>> lists((size_t)nx * nz);
      bool ok = true;
      for (uint32_t k = 0; k < n_tree && ok; ++k) {
        const uint32_t i = ord[k];
        const int a0 = std::max(0, (int)std::floor((sb[i].lo[0] - pad - x0) / g));
        const int a1 = std::min(nx - 1, (int)std::floor((sb[i].hi[0] + pad - x0) / g));
        const int b0 = std::max(0, (int)std::floor((sb[i].lo[2] - pad - z0) / g));
        const int b1 = std::min(nz - 1, (int)std::floor((sb[i].hi[2] + pad - z0) / g));
        for (int b = b0; b <= b1; ++b)
          for (int a = a0; a <= a1; ++a) {
            std::vector<uint32_t> &l = lists[(size_t)b * nx + a];
            l.push_back(i);
            if (l.size() > 15) ok = false;
          }
      }
      if (!ok) continue;
      // stored with a ring of empty cells around the listed nx x nz (the
      // kernel's DDA may step one cell past the listed region before it stops)
      const int rx = nx + 2, rz = nz + 2;
      // in stored (ring) order, every cell's first item is the running item
      // count, ring cells included: cell rc's items are [first_rc, first_rc+1)
      grid_cells.assign((size_t)rx * rz, 0);
      grid_items.clear();
      for (size_t rc = 0; rc < grid_cells.size(); ++rc) {
        const int a = (int)(rc % rx) - 1, b = (int)(rc / rx) - 1;
        const bool listed = a >= 0 && a < nx && b >= 0 && b < nz;
        const size_t c = listed ? (size_t)b * nx + a : 0;
        grid_cells[rc] = (uint32_t)(grid_items.size() / 4) << 4 | (listed ? (uint32_t)lists[c].size() : 0u);
        if (!listed) continue;
        for (uint32_t i : lists[c]) {
          const double x = s->cx[i], y = s->cy[i], z = s->cz[i], r = s->radius[i];
          grid_items.push_back(s->cx[i]);
          grid_items.push_back(s->cz[i]);
          grid_items.push_back((float)(x * x + y * y + z * z - r * r));
          // the tie key of the closed interval: 2 (0x7fffffff - index)
          const uint32_t tie2 = (0x7fffffffu - i) << 1;
          float f;
          std::memcpy(&f, &tie2, 4);
          grid_items.push_back(f);
        }
      }
      if (grid_items.size() / 4 >= (1u << 27)) {
        grid_cells.clear();
        grid_items.clear();
        return;
      }
      grid_x0 = (float)(x0 - g);
      grid_z0 = (float)(z0 - g);
      grid_xi = (float)x0;
      grid_zi = (float)z0;
      grid_g = (float)g;
      grid_nx = rx;
      grid_nz = rz;
      grid_x1 = (float)(x0 + nx * g);
      grid_z1 = (float)(z0 + nz * g);
      return;
    }
  }
  // Layer mode.  The final scene is a thin layer of small spheres (all at
  // y = 0.2 with r = 0.2) plus the ground and three big spheres.  If most
  // spheres share one (centre y, radius) and at most kMaxExtra do not, the BVH
  // is built over the layer spheres only (every box then has the layer's
  // y-range, so the walk computes that slab interval once per ray, and the
  // shared centre y folds into the per-ray terms of the leaf scan) and the
  // rest are scanned as plain pairs.  Reorders ord:
  // layer spheres first; returns their count (n when not in layer mode).
  static constexpr uint32_t kMinLayer = 64, kMaxExtra = 16;
  bool layer_mode = false;
  float layer_lo = 0.0f, layer_hi = 0.0f, layer_cy = 0.0f;
  uint32_t extra_pair0 = 0, n_extra_pairs = 0;
  uint32_t split_layer(const rt_scene_view *s) {
    const uint32_t n = s->n;
    std::vector<std::pair<float, float>> key(n);
    for (uint32_t i = 0; i < n; ++i) key[i] = {s->cy[i], std::fabs(s->radius[i])};
    std::vector<uint32_t> by_key(n);
    for (uint32_t i = 0; i < n; ++i) by_key[i] = i;
    std::sort(by_key.begin(), by_key.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b] || (key[a] == key[b] && a < b); });
    uint32_t best = 0, best_n = 0;
    for (uint32_t i = 0; i < n;) {
      uint32_t j = i;
      while (j < n && key[by_key[j]] == key[by_key[i]]) ++j;
      if (j - i > best_n) {
        best_n = j - i;
        best = by_key[i];
      }
      i = j;
    }
    if (best_n < kMinLayer) return n;
    double y0 = 1e300, y1 = -1e300;
    for (uint32_t i = 0; i < n; ++i)
      if (key[i] == key[best]) {
        y0 = std::min(y0, sb[i].lo[1]);
        y1 = std::max(y1, sb[i].hi[1]);
      }
    std::vector<uint32_t> in, out;
    for (uint32_t i = 0; i < n; ++i) (key[i] == key[best] ? in : out).push_back(i);
    if (out.size() > kMaxExtra) return n;
    layer_mode = true;
    layer_cy = key[best].first;
    std::copy(in.begin(), in.end(), ord.begin());
    std::copy(out.begin(), out.end(), ord.begin() + in.size());
    return (uint32_t)in.size();
  }
};

// scan record of one slot (ks = |C|^2 - r^2 in fp64, rounded once; padding
// slots have ks = +inf and are never candidates)
void fill_slot(rtk::pair_geom &g, int l, const rt_scene_view *s, int i) {
  if (i >= 0) {
    const double x = s->cx[i], y = s->cy[i], z = s->cz[i], r = s->radius[i];
    g.cx[l] = s->cx[i];
    g.cy[l] = s->cy[i];
    g.cz[l] = s->cz[i];
    g.ks[l] = (float)(x * x + y * y + z * z - r * r);
  } else {
    g.cx[l] = g.cy[l] = g.cz[l] = 0.0f;
    g.ks[l] = __builtin_huge_valf();
  }
}

template <bool O, bool U, bool B, bool S, bool G = false, bool L = false>
void launch(unsigned blocks, hipStream_t st, const rtk::kparams &kp0, rt_context *c, float *out) {
  rtk::kparams kp = kp0;
  kp.scan_geom = c->d_geom;
  kp.geom = c->d_bvh_geom;
  kp.nodes = c->d_nodes;
  kp.orig = c->d_orig;
  kp.shade = c->d_shade;
  kp.out = out;
  if (!kp.counters) kp.counters = c->d_counters;  // (the pilot brings its own)
  const size_t lds = L ? rtk::grid_lds_bytes(kp.grid_n_items, kp.grid_n_cells) : 0u;
  rtk::render_kernel<O, U, B, S, G, L><<<blocks, rtk::kBlock, lds, st>>>(kp);
}

using launch_fn = void (*)(unsigned, hipStream_t, const rtk::kparams &, rt_context *, float *);
// index: open | unit<<1 | bvh<<2 | stats<<3 | grid<<4 | lds<<5 (grid: the layer
// grid walk, a build of its own; lds: its grid copied into LDS; without bvh
// the grid bits select the scan)
#define RT_L4(b, s) launch<false, false, b, s>, launch<true, false, b, s>, launch<false, true, b, s>, \
                    launch<true, true, b, s>
#define RT_G4(s, l) launch<false, false, true, s, true, l>, launch<true, false, true, s, true, l>, \
                    launch<false, true, true, s, true, l>, launch<true, true, true, s, true, l>
const launch_fn kLaunch[64] = {
    RT_L4(false, false), RT_L4(true, false), RT_L4(false, true), RT_L4(true, true),      // grid 0, lds 0
    RT_L4(false, false), RT_G4(false, false), RT_L4(false, true), RT_G4(true, false),    // grid 1, lds 0
    RT_L4(false, false), RT_L4(true, false), RT_L4(false, true), RT_L4(true, true),      // grid 0, lds 1
    RT_L4(false, false), RT_G4(false, true), RT_L4(false, true), RT_G4(true, true),      // grid 1, lds 1
};
#undef RT_L4
#undef RT_G4

void free_scene(rt_context *c) {
  (void)hipFree(c->d_geom);
  (void)hipFree(c->d_bvh_geom);
  (void)hipFree(c->d_nodes);
  (void)hipFree(c->d_orig);
  (void)hipFree(c->d_shade);
  (void)hipFree(c->d_grid_cells);
  (void)hipFree(c->d_grid_items);
  c->d_grid_cells = nullptr;
  c->d_grid_items = nullptr;
  c->grid_nx = c->grid_nz = 0;
  c->grid_n_items = 0;
  c->grid_lds = false;
  c->d_geom = c->d_bvh_geom = nullptr;
  c->d_nodes = nullptr;
  c->d_orig = nullptr;
  c->d_shade = nullptr;
  c->n_spheres = c->n_pad = c->n_nodes = c->n_bvh_slots = 0;
  c->layer_mode = false;
  c->extra_pair0 = c->n_extra_pairs = 0;
  c->order_key.clear();  // the pilot's tile costs belong to the old scene
}

template <class T>
hipError_t upload_vec(T **dst, const std::vector<T> &v, hipStream_t st) {
  hipError_t e = hipMalloc(dst, sizeof(T) * (v.empty() ? 1 : v.size()));
  if (e == hipSuccess && !v.empty())
    e = hipMemcpyAsync(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st);
  return e;
}

}  // namespace

// What rt_scene_upload (and rt_internal_accel_info) accept: arrays present,
// known materials, finite centres and radii, non-zero radii, and albedos in
// [0, 1] (energy-conserving materials: a sample's radiance is then at most 1,
// which the fixed-point pixel sums rely on; dielectrics
// ignore theirs).  The builder's sorts need finite keys.
static bool scene_ok(const rt_scene_view *s) {
  if (!s || (s->n && (!s->cx || !s->cy || !s->cz || !s->radius || !s->mat_kind || !s->mat_param ||
                      !s->albedo_rgb)))
    return false;
  for (uint32_t i = 0; i < s->n; ++i) {
    if (s->mat_kind[i] > RT_DIELECTRIC || !(s->radius[i] != 0.0f) || !std::isfinite(s->radius[i]) ||
        !std::isfinite(s->cx[i]) || !std::isfinite(s->cy[i]) || !std::isfinite(s->cz[i]))
      return false;
    for (int k = 0; k < 3 && s->mat_kind[i] != RT_DIELECTRIC; ++k)
      if (!(s->albedo_rgb[3 * i + k] >= 0.0f && s->albedo_rgb[3 * i + k] <= 1.0f)) return false;
  }
  return true;
}

extern "C" {

int rt_device_count(int *count) {
  if (!count) return RT_ERR_INVALID;
  hipError_t e = hipGetDeviceCount(count);
  if (e == hipErrorNoDevice) {
    *count = 0;
    return RT_OK;
  }
  if (e != hipSuccess) return hip_fail(e);
  return RT_OK;
}

int rt_context_create(int device_ordinal, rt_context **out) {
  if (!out) return RT_ERR_INVALID;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || device_ordinal < 0 || device_ordinal >= n) {
    if (e != hipSuccess) rt_internal_set_hip_error((int)e);
    return RT_ERR_NO_DEVICE;
  }
  rt_context *c = new (std::nothrow) rt_context();
  if (!c) return RT_ERR_NOMEM;
  c->device = device_ordinal;
  int st = RT_OK;
  do {
    if ((e = hipSetDevice(device_ordinal)) != hipSuccess) break;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) break;
    if ((e = hipEventCreate(&c->ev0)) != hipSuccess) break;
    if ((e = hipEventCreate(&c->ev1)) != hipSuccess) break;
    if ((e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming)) != hipSuccess) break;
    if ((e = hipMalloc(&c->d_counters, 8 * rtk::kCounterSlots * sizeof(unsigned long long))) != hipSuccess) break;
    tonemap_thresholds(c->tonemap_thr64, c->tonemap_thr32);
    if ((e = hipMalloc(&c->d_thr64, sizeof c->tonemap_thr64)) != hipSuccess) break;
    if ((e = hipMalloc(&c->d_thr32, sizeof c->tonemap_thr32)) != hipSuccess) break;
    if ((e = hipMemcpy(c->d_thr64, c->tonemap_thr64, sizeof c->tonemap_thr64, hipMemcpyHostToDevice)) != hipSuccess) break;
    if ((e = hipMemcpy(c->d_thr32, c->tonemap_thr32, sizeof c->tonemap_thr32, hipMemcpyHostToDevice)) != hipSuccess) break;
    {
      float tab[2 * RT_TURN_TABLE];
      rt_turn_table(tab);
      if ((e = hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_turn_tab), tab, sizeof tab)) != hipSuccess) break;
    }
  } while (0);
  if (e != hipSuccess) {
    st = hip_fail(e);
    rt_context_destroy(c);
    return st;
  }
  *out = c;
  return RT_OK;
}

void rt_context_destroy(rt_context *c) {
  if (!c) return;
  if (c->device >= 0) {
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();  // renders on caller streams may still use the buffers
  }
  free_scene(c);
  (void)hipFree(c->d_counters);
  (void)hipFree(c->d_frame);
  (void)hipFree(c->d_order);
  (void)hipFree(c->d_thr64);
  (void)hipFree(c->d_thr32);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int rt_scene_upload(rt_context *c, const rt_scene_view *s) {
  if (!c || !scene_ok(s)) return RT_ERR_INVALID;
  const uint32_t n = s->n;
  const uint32_t n_pad = (n + rtk::kSpherePad - 1) / rtk::kSpherePad * rtk::kSpherePad;
  std::vector<rtk::pair_geom> geom(n_pad / 2);
  for (uint32_t i = 0; i < n_pad; ++i) fill_slot(geom[i / 2], i & 1, s, i < n ? (int)i : -1);
  std::vector<rtk::shade_rec> shade(n);
  for (uint32_t i = 0; i < n; ++i) {
    rtk::shade_rec &r = shade[i];
    std::memset(&r, 0, sizeof r);
    r.cx = s->cx[i];
    r.cy = s->cy[i];
    r.cz = s->cz[i];
    r.inv_r = 1.0f / s->radius[i];
    const bool glass = s->mat_kind[i] == RT_DIELECTRIC;
    r.ar = glass ? 1.0f : s->albedo_rgb[3 * i + 0];
    r.ag = glass ? 1.0f : s->albedo_rgb[3 * i + 1];
    r.ab = glass ? 1.0f : s->albedo_rgb[3 * i + 2];
    r.param = s->mat_param[i];
    r.kind = s->mat_kind[i];
    r.radius = s->radius[i];
    const double x = s->cx[i], y = s->cy[i], z = s->cz[i], rr = s->radius[i];
    r.ks = (float)(x * x + y * y + z * z - rr * rr);
    const double ior = s->mat_param[i];
    r.inv_param = (float)(1.0 / ior);
    const double r0 = (1.0 - ior) / (1.0 + ior);
    r.r0 = (float)(r0 * r0);
  }
  bvh_builder bb;
  bb.run(s);
  std::vector<rtk::pair_geom> bgeom(bb.slots.size() / 2);
  for (size_t k = 0; k < bb.slots.size(); ++k) fill_slot(bgeom[k / 2], (int)(k & 1), s, bb.slots[k]);

  RT_HIP(hipSetDevice(c->device));
  // renders enqueued on caller streams may still read the old scene
  RT_HIP(hipDeviceSynchronize());
  free_scene(c);
  hipError_t e = upload_vec(&c->d_geom, geom, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_bvh_geom, bgeom, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_nodes, bb.nodes, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_orig, bb.slots, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_shade, shade, c->stream);
  if (e == hipSuccess && !bb.grid_cells.empty()) {
    e = upload_vec(&c->d_grid_cells, bb.grid_cells, c->stream);
    if (e == hipSuccess) e = upload_vec(&c->d_grid_items, bb.grid_items, c->stream);
    c->grid_n_items = bb.grid_items.size() / 4;
    // u16 cells need first < 4096; RTOW_GRID_LDS=0 keeps the grid in global memory
    c->grid_lds = c->grid_n_items < 4096 &&
                  rtk::grid_lds_bytes((int)c->grid_n_items, bb.grid_nx * bb.grid_nz) <= rtk::kGridLdsMax &&
                  bvh_builder::env_double("RTOW_GRID_LDS", 1.0, 0.0, 1.0) != 0.0;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    free_scene(c);
    return hip_fail(e);
  }
  c->n_spheres = n;
  c->n_pad = n_pad;
  c->n_nodes = (uint32_t)bb.per_order;  // nodes holds 8 orders of this many
  c->n_bvh_slots = (uint32_t)bb.slots.size();
  c->oref2 = (float)(0.99 * bb.oref * bb.oref);
  c->layer_mode = bb.layer_mode;
  c->layer_lo = bb.layer_lo;
  c->layer_cy = bb.layer_cy;
  c->layer_hi = bb.layer_hi;
  c->extra_pair0 = bb.extra_pair0;
  c->n_extra_pairs = bb.n_extra_pairs;
  c->grid_x0 = bb.grid_x0;
  c->grid_xi = bb.grid_xi;
  c->grid_zi = bb.grid_zi;
  c->grid_z0 = bb.grid_z0;
  c->grid_x1 = bb.grid_x1;
  c->grid_z1 = bb.grid_z1;
  c->grid_g = bb.grid_g;
  c->grid_nx = bb.grid_nx;
  c->grid_nz = bb.grid_nz;
  return RT_OK;
}

}  // extern "C"

namespace {

// Local rows that lie inside the frame: a rank's last band slots may be
// padding (global row >= height), which the kernel leaves at zero untraced.
uint64_t valid_rows(const rt_params *prm) {
  uint64_t n = 0;
  for (int r0 = 0; r0 < prm->local_rows; r0 += prm->row_block) {
    const long long g0 = ((long long)(r0 / prm->row_block) * prm->band_stride + prm->band_offset) *
                         (long long)prm->row_block;
    const long long in_band = std::min<long long>(prm->row_block, prm->local_rows - r0);
    n += (uint64_t)std::max<long long>(0, std::min<long long>(in_band, prm->height - g0));
  }
  return n;
}

// rt_render_async's body.  ev_start (may be null) is recorded on the stream
// just before the render kernel itself, after any one-time setup (the pilot,
// buffer growth), so that rt_render's kernel_ms times the render alone.
int render_enqueue(rt_context *c, const rt_camera *cam, const rt_params *prm, float *accum_rgb, hipStream_t st,
                   hipEvent_t ev_start) {
  RT_HIP(hipSetDevice(c->device));
  // renders of one context are serialised, whatever streams they come on:
  // they share the block-order scratch buffer
  if (c->have_done && c->last_stream != st) RT_HIP(hipStreamWaitEvent(st, c->ev_done, 0));
  const uint64_t samples = (uint64_t)prm->width * valid_rows(prm) * (uint64_t)prm->spp;
  if (prm->flags & RT_FLAG_KEEP_COUNTERS) {
    c->last_samples += samples;
  } else {
    RT_HIP(hipMemsetAsync(c->d_counters, 0, 8 * rtk::kCounterSlots * sizeof(unsigned long long), st));
    c->last_samples = samples;
  }
  c->last_stats = (prm->flags & RT_FLAG_COUNT_WORK) != 0;
  if (prm->width == 0 || prm->local_rows == 0) {
    if (ev_start) RT_HIP(hipEventRecord(ev_start, st));
    return RT_OK;
  }

  rtk::kparams kp;
  std::memset(&kp, 0, sizeof kp);
  kp.cam = *cam;
  kp.width = prm->width;
  kp.height = prm->height;
  kp.spp = prm->spp;
  kp.max_depth = prm->max_depth;
  kp.row_block = prm->row_block;
  kp.band_stride = prm->band_stride;
  kp.band_offset = prm->band_offset;
  kp.local_rows = prm->local_rows;
  kp.tiles_x = (prm->width + rtk::kTile - 1) / rtk::kTile;
  kp.n_pad = (int)c->n_pad;
  kp.n_nodes = (int)c->n_nodes;
  kp.oref2 = c->oref2;
  kp.layer = rtk::f2{c->layer_lo, c->layer_hi};
  kp.layer_mode = c->layer_mode ? 1 : 0;
  kp.layer_cy = c->layer_cy;
  kp.extra_pair0 = (int)c->extra_pair0;
  kp.n_extra_pairs = (int)c->n_extra_pairs;
  kp.grid_cells = c->d_grid_cells;
  kp.grid_items = (const rtk::f4 *)c->d_grid_items;
  kp.grid_n_items = (int)c->grid_n_items;
  kp.grid_n_cells = c->grid_nx * c->grid_nz;
  kp.grid_x0 = c->grid_x0;
  kp.grid_xi = c->grid_xi;
  kp.grid_zi = c->grid_zi;
  kp.grid_z0 = c->grid_z0;
  kp.grid_x1 = c->grid_x1;
  kp.grid_z1 = c->grid_z1;
  kp.grid_g = c->grid_g;
  kp.grid_invg = c->grid_g > 0.0f ? 1.0f / c->grid_g : 0.0f;
  kp.grid_nx = c->grid_nx;
  kp.grid_nz = c->grid_nz;
  kp.seed32 = (uint32_t)prm->seed ^ ((uint32_t)(prm->seed >> 32) * 0x9E3779B9u);
  kp.flags = prm->flags;
  kp.inv_wm1 = (float)(1.0 / (prm->width - 1));
  kp.inv_hm1 = (float)(1.0 / (prm->height - 1));
  {
    uint32_t w = (uint32_t)prm->width, sh = 0;
    while (!(w & 1u)) {
      w >>= 1;
      ++sh;
    }
    uint32_t inv = w;  // Newton: inv = inv (2 - w inv) doubles the correct low bits
    for (int k = 0; k < 5; ++k) inv *= 2u - w * inv;
    kp.wshift = sh;
    kp.winv = inv;
  }
  const int tiles_y = (prm->local_rows + rtk::kTile - 1) / rtk::kTile;
  const long long tiles = (long long)kp.tiles_x * tiles_y;
  const unsigned blocks = (unsigned)((tiles + rtk::kWavesPerBlock - 1) / rtk::kWavesPerBlock);
  const int v = ((prm->flags & RT_FLAG_OPEN_INTERVAL) ? 1 : 0) |
                ((prm->flags & RT_FLAG_METAL_UNIT_VECTOR) ? 2 : 0) |
                ((prm->flags & RT_FLAG_ACCEL_BVH) ? 4 : 0) |
                ((prm->flags & RT_FLAG_COUNT_WORK) ? 8 : 0) |
                ((c->d_grid_cells && !(prm->flags & RT_FLAG_LAYER_BVH)) ? 16 : 0) |
                ((c->d_grid_cells && c->grid_lds && !(prm->flags & RT_FLAG_LAYER_BVH)) ? 32 : 0);
  // How many waves share a tile's samples (even shares; the integer pixel
  // sums make any split give the same image).  One wave per tile traces all
  // of its tile's samples; when a rank holds few tiles (a 1/8 share of a 4K
  // frame is ~2 waves per wave slot), the slowest tiles (long glass / metal
  // paths) then set the frame time, so the samples are split over `units`
  // waves (tools/rank_times.py).
  long long units = prm->units;
  if (units <= 0) {
    const bool pilot = (prm->flags & RT_FLAG_PILOT_SCHEDULE) != 0;
    units = pilot ? std::llround((double)rtk::kPilotTilesPerUnit / (double)std::max(1LL, tiles))
                  : (tiles < rtk::kSplitTiles ? rtk::kUnits : 1);
    units = std::min<long long>(std::max(units, 1LL), rtk::kUnits);
  }
  if (prm->spp <= 0 || prm->max_depth <= 0) units = 1;  // nothing is traced
  units = std::max(1LL, std::min<long long>(units, prm->spp));  // >= 1 sample per unit
  kp.units = (int)units;
  {
    int f = 31;  // F = 31 - floor(log2(spp)): spp samples of at most 2^F each fit a uint32
    for (int s = prm->spp; s > 1; s >>= 1) --f;
    kp.qscale = std::ldexp(1.0f, f);
    kp.qinv = std::ldexp(1.0f, -f);
  }
  const uint64_t frame_floats = (uint64_t)prm->local_rows * (uint64_t)prm->width * 3u;
  if ((prm->flags & RT_FLAG_PILOT_SCHEDULE) && prm->spp > 0 && prm->max_depth > 0 && blocks > 1) {
    // Expensive tiles first (RT_FLAG_PILOT_SCHEDULE): a 4-spp pilot (same
    // geometry, one wave per tile, the instrumented build that reports each
    // tile's segments) runs once per frame geometry; blocks are then launched
    // in decreasing cost of their tiles (longest-processing-time first), the
    // units of a tile group adjacent.  Without it the hardware launches
    // blocks in index order and the last wave slots to fill may get the most
    // expensive tiles.  Scheduling only: the image does not depend on it.
    // Everything stays on st (the sort runs on the device, rt_sched.hip).
    std::vector<uint64_t> key = {(uint64_t)prm->width, (uint64_t)prm->height, (uint64_t)prm->local_rows,
                                 (uint64_t)prm->row_block, (uint64_t)prm->band_stride,
                                 (uint64_t)prm->band_offset, (uint64_t)units, (uint64_t)(prm->flags & 0x12ffu)};
    const uint32_t *cw = reinterpret_cast<const uint32_t *>(cam);
    for (size_t k = 0; k < sizeof(rt_camera) / 4; ++k) key.push_back(cw[k]);
    if (key != c->order_key || c->order_n != (size_t)blocks * units) {
      c->order_key.clear();  // valid again only once the new order is enqueued
      // tile costs, then 8 scratch counters (the context's are not touched)
      const size_t n_cost = (size_t)blocks * rtk::kWavesPerBlock;
      const size_t cost_bytes = (n_cost * sizeof(uint32_t) + 7) / 8 * 8;
      uint32_t *d_cost = nullptr;
      RT_HIP(hipMallocAsync((void **)&d_cost, cost_bytes + 8 * sizeof(unsigned long long), st));
      hipError_t e = hipMemsetAsync(d_cost, 0, cost_bytes + 8 * sizeof(unsigned long long), st);
      if (e == hipSuccess) {
        rtk::kparams pk = kp;
        pk.spp = std::min(prm->spp, 4);
        pk.units = 1;
        pk.tile_cost = d_cost;
        pk.counters = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(d_cost) + cost_bytes);
        kLaunch[(v & 55) | 8](blocks, st, pk, c, accum_rgb);
        e = hipGetLastError();
      }
      if (e == hipSuccess && c->d_order) e = hipFreeAsync(c->d_order, st);
      if (e == hipSuccess) {
        c->d_order = nullptr;
        c->order_n = 0;
        e = hipMallocAsync((void **)&c->d_order, (size_t)blocks * units * sizeof(uint32_t), st);
      }
      if (e == hipSuccess) e = rt_internal_block_order(d_cost, blocks, (uint32_t)units, c->d_order, st);
      (void)hipFreeAsync(d_cost, st);  // also on error: no leak
      if (e != hipSuccess) return hip_fail(e);
      c->order_n = (size_t)blocks * units;
      c->order_key = key;
    }
    kp.block_order = c->d_order;
  }
  // several units per tile add their integer sums into the zeroed frame
  // (after the pilot, which renders into it too), finish_sums converts them
  if (units > 1) RT_HIP(hipMemsetAsync(accum_rgb, 0, frame_floats * sizeof(float), st));
  if (ev_start) RT_HIP(hipEventRecord(ev_start, st));
  kLaunch[v]((unsigned)(blocks * units), st, kp, c, accum_rgb);
  RT_HIP(hipGetLastError());
  if (units > 1) {
    const unsigned grid = (unsigned)std::min<uint64_t>((frame_floats + 255) / 256, 256u * 64u);
    rtk::finish_sums<<<grid, 256, 0, st>>>(reinterpret_cast<uint32_t *>(accum_rgb), frame_floats, kp.qinv);
    RT_HIP(hipGetLastError());
  }
  RT_HIP(hipEventRecord(c->ev_done, st));
  c->last_stream = st;
  c->have_done = true;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_async(rt_context *c, const rt_camera *cam, const rt_params *prm, float *accum_rgb,
                    void *stream) {
  if (!c || !cam || !params_ok(prm) || (!accum_rgb && prm->local_rows && prm->width))
    return RT_ERR_INVALID;
  if (cam->model != RT_CAMERA_CPU && cam->model != RT_CAMERA_GPU) return RT_ERR_INVALID;
  if (cam->model == RT_CAMERA_CPU && (prm->width < 2 || prm->height < 2)) return RT_ERR_INVALID;
  if (!c->d_geom) return RT_ERR_NO_SCENE;
  return render_enqueue(c, cam, prm, accum_rgb, stream ? (hipStream_t)stream : c->stream, nullptr);
}

int rt_reset_stats(rt_context *c, void *stream) {
  if (!c) return RT_ERR_INVALID;
  RT_HIP(hipSetDevice(c->device));
  RT_HIP(hipMemsetAsync(c->d_counters, 0, 8 * rtk::kCounterSlots * sizeof(unsigned long long),
                        stream ? (hipStream_t)stream : c->stream));
  c->last_samples = 0;
  return RT_OK;
}

int rt_collect_stats(rt_context *c, rt_stats *stats) {
  if (!c || !stats) return RT_ERR_INVALID;
  unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0}, hs[8 * rtk::kCounterSlots];
  RT_HIP(hipSetDevice(c->device));
  RT_HIP(hipMemcpy(hs, c->d_counters, sizeof hs, hipMemcpyDeviceToHost));
  for (int i = 0; i < 8 * rtk::kCounterSlots; ++i) h[i & 7] += hs[i];
  stats->segments = h[0];
  stats->wave_steps = h[1];
  stats->samples = c->last_samples;
  stats->bf_tests = h[0] * (uint64_t)c->n_spheres;
  stats->sphere_tests = c->last_stats ? h[2] : 0;
  stats->box_tests = c->last_stats ? h[3] : 0;
  stats->box_hits = c->last_stats ? h[4] : 0;
  stats->root_tests = c->last_stats ? h[5] : 0;
  stats->kernel_ms = 0.0;
  return RT_OK;
}

int rt_render(rt_context *c, const rt_camera *cam, const rt_params *prm, float *host_rgb,
              rt_stats *stats) {
  if (!c || !params_ok(prm) || (!host_rgb && prm->local_rows && prm->width)) return RT_ERR_INVALID;
  const size_t nf = 3 * (size_t)prm->width * (size_t)prm->local_rows;
  RT_HIP(hipSetDevice(c->device));
  if (nf > c->frame_floats) {
    // (only rt_render uses d_frame, and it returns after its work is done)
    (void)hipFree(c->d_frame);
    c->d_frame = nullptr;
    c->frame_floats = 0;
    RT_HIP(hipMalloc(&c->d_frame, nf * sizeof(float)));
    c->frame_floats = nf;
  }
  if (!cam || (cam->model != RT_CAMERA_CPU && cam->model != RT_CAMERA_GPU)) return RT_ERR_INVALID;
  if (cam->model == RT_CAMERA_CPU && (prm->width < 2 || prm->height < 2)) return RT_ERR_INVALID;
  if (!c->d_geom) return RT_ERR_NO_SCENE;
  // ev0 is recorded right before the render kernel (after a first-frame pilot)
  int st = render_enqueue(c, cam, prm, c->d_frame, c->stream, c->ev0);
  if (st != RT_OK) return st;
  RT_HIP(hipEventRecord(c->ev1, c->stream));
  RT_HIP(hipEventSynchronize(c->ev1));
  float ms = 0.f;
  RT_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  if (nf) RT_HIP(hipMemcpy(host_rgb, c->d_frame, nf * sizeof(float), hipMemcpyDeviceToHost));
  if (stats) {
    st = rt_collect_stats(c, stats);
    if (st != RT_OK) return st;
    stats->kernel_ms = ms;
  }
  return RT_OK;
}

// Host-only view of what rt_scene_upload would build (no device needed):
// tests/test_host.py checks the builder's invariants on CPU, and
// tools/host_sanitize.sh runs it under ASan / UBSan.  out[16]:
//   0 nodes per DFS order   1 BVH slots          2 layer mode     3 extra_pair0
//   4 n_extra_pairs         5 grid_nx (w/ ring)  6 grid_nz        7 grid items
//   8 grid LDS bytes        9 grid fits the LDS 10 max items/cell 11 start invariant
//  12 empty ring cells ok  13 oref * 1000      14 layer slots    15 listed cells
int rt_internal_accel_info(const rt_scene_view *s, uint64_t *out) {
  if (!out || !scene_ok(s)) return RT_ERR_INVALID;
  bvh_builder bb;
  bb.run(s);
  std::memset(out, 0, 16 * sizeof(uint64_t));
  out[0] = bb.per_order;
  out[1] = bb.slots.size();
  out[2] = bb.layer_mode ? 1u : 0u;
  out[3] = bb.extra_pair0;
  out[4] = bb.n_extra_pairs;
  out[5] = (uint64_t)bb.grid_nx;
  out[6] = (uint64_t)bb.grid_nz;
  const uint64_t items = bb.grid_items.size() / 4, cells = bb.grid_cells.size();
  out[7] = items;
  out[8] = cells ? rtk::grid_lds_bytes((int)items, (int)cells) : 0u;
  out[9] = cells && items < 4096 && out[8] <= rtk::kGridLdsMax;
  // every stored cell's first item is the running count (ring cells included),
  // so cell i's items are [first_i, first_{i+1}) -- what the LDS walk reads
  uint64_t maxc = 0, listed = 0;
  bool start_ok = true, ring_ok = true;
  for (uint64_t i = 0; i < cells; ++i) {
    const uint32_t first = bb.grid_cells[i] >> 4, cnt = bb.grid_cells[i] & 15u;
    const uint64_t next = i + 1 < cells ? (bb.grid_cells[i + 1] >> 4) : items;
    start_ok = start_ok && first + cnt == next;
    maxc = std::max<uint64_t>(maxc, cnt);
    listed += cnt ? 1u : 0u;
    const int a = (int)(i % bb.grid_nx), b = (int)(i / bb.grid_nx);
    if (a == 0 || b == 0 || a == bb.grid_nx - 1 || b == bb.grid_nz - 1) ring_ok = ring_ok && cnt == 0;
  }
  out[10] = maxc;
  out[11] = cells ? (start_ok ? 1u : 0u) : 0u;
  out[12] = cells ? (ring_ok ? 1u : 0u) : 0u;
  out[13] = (uint64_t)(bb.oref * 1000.0);
  out[14] = bb.layer_mode ? (uint64_t)(2 * bb.extra_pair0) : 0u;
  out[15] = listed;
  return RT_OK;
}

int rt_device_kat(int device, int kind, const double *in, size_t n_cases, double *out) {
  if (kind < RT_KAT_SPHERE_HIT || kind > RT_KAT_REFLECTANCE || (n_cases && (!in || !out)) ||
      n_cases > (1u << 20))
    return RT_ERR_INVALID;
  if (!n_cases) return RT_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return RT_ERR_NO_DEVICE;
  RT_HIP(hipSetDevice(device));
  double *d = nullptr;
  RT_HIP(hipMalloc(&d, 19 * sizeof(double) * n_cases));
  hipError_t e = hipMemcpy(d, in, 10 * sizeof(double) * n_cases, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    rtk::kat_kernel<<<(unsigned)((n_cases + 63) / 64), 64>>>(kind, d, (int)n_cases, d + 10 * n_cases);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, d + 10 * n_cases, 9 * sizeof(double) * n_cases, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e);
  return RT_OK;
}

int rt_tonemap_async(rt_context *c, const float *d_sums, size_t n_pixels, int spp, int mode, uint8_t *d_out,
                     void *stream) {
  if (!c || spp < 1 || (mode != RT_TONEMAP_CPU && mode != RT_TONEMAP_GPU) || ((!d_sums || !d_out) && n_pixels))
    return RT_ERR_INVALID;
  if (!n_pixels) return RT_OK;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  RT_HIP(hipSetDevice(c->device));
  const uint64_t n = 3 * (uint64_t)n_pixels;
  const unsigned grid = (unsigned)std::min<uint64_t>((n / 4 + 255) / 256 + 1, 256u * 32u);
  if (mode == RT_TONEMAP_CPU)
    rtk::tonemap_kernel<false, double><<<grid, 256, 0, st>>>(d_sums, n, 1.0 / spp, c->d_thr64, d_out);
  else
    rtk::tonemap_kernel<true, float><<<grid, 256, 0, st>>>(d_sums, n, 1.0f / (float)spp, c->d_thr32, d_out);
  RT_HIP(hipGetLastError());
  return RT_OK;
}

}  // extern "C"
