// rt_kernel.hip -- the MI355X (gfx950) render kernel and its device helpers
// (the device half of the C ABI in include/rt.h; the host half is rt_api.cpp,
// the acceleration-structure builder rt_accel.cpp, the layout they share
// rt_layout.h).
//
// Replaces render<<<>>> (src/gpu/camera.h:169-195) and, inside it, get_ray
// (camera.h:153-167 / src/cpu/camera.h:28-34), ray_color (src/cpu/main.cc:12-30,
// iterative as in src/gpu/camera.h:112-138), hittable_list::hit / sphere::hit
// (src/cpu/hittable_list.h:28-43, src/cpu/sphere.h:24-51) and the three
// material::scatter functions (src/cpu/material.h:15-88).
//
// Design:
//  * one wave64 per 8x8 pixel tile, 4 waves per block; the wave owns a pool of
//    its tile's (pixel, sample) items and a lane whose path ends takes the
//    next one ("path regeneration"), so no lane idles while the tile has
//    samples left; the wave exits on __ballot(alive) == 0;
//  * pixel sums are exact fixed-point integers (LDS atomics), so any split of
//    the samples over lanes, waves, launches or GPUs gives the same bits;
//  * closest hit: a per-lane DDA over a layer grid (the default for layer
//    scenes, 3.3), a wave-uniform stackless BVH walk (3.1-3.2) or the
//    brute-force scan; sphere and node records are scalar (SMEM) loads into
//    SGPRs, the grid lives in LDS when it fits;
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
#include <array>
#include <cmath>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "rt_internal.h"
#include "rt_layout.h"
#include "rt_turn_table.h"

namespace rtk {

// STATS builds: the grid walk's box_hits counts wave-level DDA iterations, or
// with RT_COUNT_ITEMS=1 wave-level item iterations, =2 wave-level item
// iterations that run the root sequence (tools/grid_wave_counts.py)
#ifndef RT_COUNT_ITEMS
#define RT_COUNT_ITEMS 0
#endif

// RT_LANE_PROFILE builds (tools/lane_profile.py, a measurement variant built
// by tools/build_variant.sh; never the product): per source region of the
// bounce loop, how many times a wave ran it, the lanes active (exec) and the
// lanes that needed it (`useful`), counted in LDS by the wave's first active
// lane and added to g_lane_prof at the wave's end (DESIGN.md 8's lane table).
// The default build compiles every LP() to nothing.
enum {
  kLpStep = 0, kLpClosest, kLpExtrasLead, kLpExtrasRound, kLpGridWalk, kLpDda, kLpItem, kLpGridCand,
  kLpSky, kLpHit, kLpLamb, kLpMetal, kLpDiel, kLpCamera, kLpSkip, kLpTail, kLpRegions
};
#ifdef RT_LANE_PROFILE
__device__ unsigned long long g_lane_prof[kLpRegions * 3];
__shared__ uint32_t s_lane_prof[4][kLpRegions][3];
__device__ __forceinline__ void lane_prof(int r, bool useful) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(true);
  const uint64_t u = __builtin_amdgcn_ballot_w64(useful);
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  if (l == __builtin_ctzll(m)) {
    uint32_t *c = s_lane_prof[__builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6][r];
    c[0] += 1u;
    c[1] += (uint32_t)__builtin_popcountll(m);
    c[2] += (uint32_t)__builtin_popcountll(u);
  }
}
#define LP(r, useful) lane_prof((r), (useful))
#else
#define LP(r, useful) ((void)0)
#endif

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// the dynamic LDS of the LDS grid placements: kGridLds the grid items, then
// the u16 cell starts; kGridCells the u16 cell starts only
extern __shared__ f4 s_grid_dyn[];
typedef const __attribute__((address_space(3))) f4 lds_f4;

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

// The dither of a sample's fixed-point sum at spp >= 4096 (DESIGN.md 2, step
// 6): the sample adds trunc(x) + (frac(x) > u) for x = v 2^F, whose mean is x
// for u uniform in [0, 1), whatever v is.  u is a draw of its own, keyed by
// the pixel and the sample (a pcg4d with the bit-inverted seed, so it is
// independent of every draw of the path).
__device__ __forceinline__ float dither_u(uint32_t pix, uint32_t sample, uint32_t seed32) {
  return unif(pcg4d(pix, sample, 0u, ~seed32).x);
}

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
  // a 32-bit byte offset from the table's base (saddr addressing: no 64-bit
  // index arithmetic); 0 <= fl < 1024
  const f2 sc = *(const RT_GLOBAL f2 *)((const RT_GLOBAL char *)as_global(g_turn_tab) + ((uint32_t)fl << 3));
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
// Returns the ray's t_min: 0.001 in units of the unnormalised direction, as
// the reference tests its roots (src/cpu/main.cc:19 world.hit(r, 0.001, ..),
// sphere.h:37-41; src/gpu/camera.h:117 interval(0.001, inf)), i.e. 0.001 |x|
// on the normalised ray, with |x| = l2 r.
__device__ __forceinline__ float normalize3(float &x, float &y, float &z) {
  const float l2 = fmaf(z, z, fmaf(y, y, x * x));
  float r = __uint_as_float(0x5f375a86u - (__float_as_uint(l2) >> 1));
  const float h = 0.5f * l2;
#pragma unroll
  for (int k = 0; k < 3; ++k) r = r * fmaf(-h, r * r, 1.5f);
  x *= r;
  y *= r;
  z *= r;
  return 0.001f * (l2 * r);
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
    // a real (wave-uniform) branch: without the barrier the compiler computes
    // the lens origin for every camera and selects (9 VALU per new path)
    asm volatile("" ::: "memory");
    ox = fmaf(ddy, p.cam.lens_v[0], fmaf(ddx, p.cam.lens_u[0], ox));
    oy = fmaf(ddy, p.cam.lens_v[1], fmaf(ddx, p.cam.lens_u[1], oy));
    oz = fmaf(ddy, p.cam.lens_v[2], fmaf(ddx, p.cam.lens_u[2], oz));
  }
  dx = tx - ox;
  dy = ty - oy;
  dz = tz - oz;
}

// the whole camera ray for r = pcg4d(pix, sample, 0, seed32); returns its t_min
__device__ __forceinline__ float camera_ray(const kparams &p, const uint4 r, int col, int grow,
                                            float &ox, float &oy, float &oz,
                                            float &dx, float &dy, float &dz) {
  float ddx = 0.0f, ddy = 0.0f;
  if (p.cam.has_lens) polar(unif(r.z), unif(r.w), ddx, ddy);
  camera_dir(p, r, ddx, ddy, col, grow, ox, oy, oz, dx, dy, dz);
  return normalize3(dx, dy, dz);
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
// tie2 = tie2_of<OPEN>(index); tmin = the ray's t_min (normalize3).
// Branch-free: a lane whose line misses the sphere (c false) computes a
// garbage root (sqrt_k clamps its negative argument) and keeps its hit.  The
// hot call sites (the extras' sequences, the grid item) branch on the WAVE
// first (a ballot: one uniform branch instead of an exec-mask if / join per
// call; SALU per headline launch 3.52 -> 3.14e10).
template <bool OPEN>
__device__ __forceinline__ void candidate(bool c, float h, float disc, uint32_t tie2, float tmin, hit_state &hs) {
  const float sq = sqrt_k(disc);
  const float t0 = h - sq, t1 = h + sq;
  const bool use0 = OPEN ? (t0 > tmin) : (t0 >= tmin);
  const float root = use0 ? t0 : t1;
  // root >= t_min  <=>  t1 >= t_min (t1 >= t0; with use0, t0 >= t_min)
  const bool above = OPEN ? (t1 > tmin) : (t1 >= tmin);
  const uint32_t lo = tie2 + (use0 ? 1u : 0u);
  const uint64_t key = ((uint64_t)__float_as_uint(root) << 32) | lo;
  const uint64_t cur = ((uint64_t)__float_as_uint(hs.tmax) << 32) | hs.lo;
  if (c & above & (key < cur)) {
    hs.tmax = root;
    hs.lo = lo;
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
                                           float tmin, hit_state &hs, uint32_t &roots) {
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
      if (c[2 * j]) candidate<OPEN>(true, h[j].x, e[j].x - q[j].ks.x, tie2_of<OPEN>((uint32_t)i0), tmin, hs);
      if (c[2 * j + 1]) candidate<OPEN>(true, h[j].y, e[j].y - q[j].ks.y, tie2_of<OPEN>((uint32_t)i1), tmin, hs);
    }
  }
}

// The extras of the grid build (the spheres off the layer: in the final scene
// the ground and the three big spheres), four per group, with their candidates'
// root sequences compacted: a lane's candidates among spheres J0..3 run one
// per round, the lowest remaining slot first, so a round runs for every lane
// that still has one and the wave runs as many rounds as its busiest lane has
// candidates (usually one: a line seldom meets two of the big spheres),
// instead of one sequence per sphere that ANY lane meets (each of the three
// big spheres is a candidate for ~10 % of lines, so for some lane of almost
// every wave).  Slot 0 of the first group (the builder puts the largest extra
// there: the ground, a candidate for almost every line) runs its own sequence
// first (LEAD).  The candidate rule is order-independent, so the closest hit
// is the same bits as a scan of the four in any order.
template <bool OPEN, bool STATS, bool LEAD>
__device__ __forceinline__ void scan_extras(const RT_CONST pair_geom *__restrict__ g, int slot0,
                                            const RT_CONST int *__restrict__ orig, const ray_pre &r,
                                            float tmin, hit_state &hs, uint32_t &roots) {
  float h[4], d[4];
  uint32_t t[4];
  bool c[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const pair_geom q = cload(g + j);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float cx = s ? q.cx.y : q.cx.x, cy = s ? q.cy.y : q.cy.x, cz = s ? q.cz.y : q.cz.x;
      const float ks = s ? q.ks.y : q.ks.x;
      const float hy = fmaf(cy, r.dy.x, r.nk1.x);
      const float gy = fmaf(cy, r.oy2.x, r.o2.x);
      const float hh = fmaf(cz, r.dz.x, fmaf(cx, r.dx.x, hy));
      const float gg = fmaf(cz, r.oz2.x, fmaf(cx, r.ox2.x, gy));
      const float ee = fmaf(hh, hh, -gg);
      const int k = 2 * j + s;
      h[k] = hh;
      d[k] = ee - ks;
      c[k] = ee >= ks;
      t[k] = tie2_of<OPEN>((uint32_t)orig[slot0 + k]);
    }
  }
  constexpr int J0 = LEAD ? 1 : 0;
  if (LEAD) {
    if (__builtin_amdgcn_ballot_w64(c[0])) {  // a wave-uniform branch
      LP(kLpExtrasLead, c[0]);
      if (STATS) ++roots;
      candidate<OPEN>(c[0], h[0], d[0], t[0], tmin, hs);
    }
  }
#pragma unroll
  for (int round = J0; round < 4; ++round) {
    // this lane's lowest remaining candidate (the default slot 3 is only
    // read by lanes with none left, which do not run the sequence)
    float hh = h[3], dd = d[3];
    uint32_t tt = t[3];
#pragma unroll
    for (int j = 2; j >= J0; --j)
      if (c[j]) {
        hh = h[j];
        dd = d[j];
        tt = t[j];
      }
    bool taken = false;
#pragma unroll
    for (int j = J0; j < 4; ++j) {
      const bool f = c[j] && !taken;
      c[j] = c[j] && !f;
      taken = taken || f;
    }
    if (!__builtin_amdgcn_ballot_w64(taken)) break;
    LP(kLpExtrasRound, taken);
    if (STATS) ++roots;
    candidate<OPEN>(taken, hh, dd, tt, tmin, hs);
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
                                         const ray_pre &rp, float tmin, hit_state &hs, work_ctr &wc,
                                         float lim_src, float &lim) {
  if (STATS) {
    ++wc.boxes;
    wc.box_hits += hit ? 1u : 0u;
  }
  if (!__builtin_amdgcn_ballot_w64(hit)) return nd.skip;
  if (!nd.leaf) return node + 1;
  const int fp = (int)(nd.leaf & ~kTwoPairs) - 1;
  // a leaf of 1-2 spheres scans one pair, not a pair of padding
  if (nd.leaf & kTwoPairs) {
    scan_pairs<OPEN, 2, STATS, LAYER>(geom + fp, 2 * fp, orig, rp, tmin, hs, wc.roots);
    if (STATS) wc.tests += 4;
  } else {
    scan_pairs<OPEN, 1, STATS, LAYER>(geom + fp, 2 * fp, orig, rp, tmin, hs, wc.roots);
    if (STATS) wc.tests += 2;
  }
  if (LAYER) asm("v_min_f32 %0, %1, %2" : "=v"(lim) : "v"(lim_src), "v"(hs.tmax));
  return nd.skip;
}

// one grid item (cx, cz, ks, closed tie key): the leaf test's arithmetic in
// plain fp32 (NOY fold: the same bits as scan_pairs) and the candidate rule
template <bool OPEN, bool STATS>
__device__ __forceinline__ void grid_item(const f4 it, float dx, float dz, const ray_pre &rl, float tmin,
                                          hit_state &hs, work_ctr &wc) {
  if (STATS && RT_COUNT_ITEMS == 1 && lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true))) ++wc.box_hits;
  const float h = fmaf(it.y, dz, fmaf(it.x, dx, rl.nk1.x));
  const float g = fmaf(it.y, rl.oz2.x, fmaf(it.x, rl.ox2.x, rl.o2.x));
  const float e = fmaf(h, h, -g);
  if (STATS && RT_COUNT_ITEMS == 2 && __builtin_amdgcn_ballot_w64(e >= it.z) &&
      lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
    ++wc.box_hits;
  // it.w holds tie2_of<false>(index); the open interval's is 0xfffffffe - it
  const uint32_t w = __float_as_uint(it.w);
  const bool c = e >= it.z;
  LP(kLpItem, true);
  // a wave-uniform branch; the sequence runs under the item loop's own mask
  if (__builtin_amdgcn_ballot_w64(c)) {
    LP(kLpGridCand, c);
    candidate<OPEN>(c, h, e - it.z, OPEN ? 0xfffffffeu - w : w, tmin, hs);
  }
  if (STATS) ++wc.tests;
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
template <bool OPEN, bool STATS, int GP>
__device__ __forceinline__ void grid_walk(float ox, float oz, float ix, float iz, float oix, float oiz,
                                          float ta, float tb, const ray_pre &rl, float tmin, hit_state &hs,
                                          work_ctr &wc) {
  const kparams p = kernargs();
  // clip to the grid's inner box (the cells around it are an empty ring);
  // slab times as fma(x, 1/d, -o/d) like the BVH's (the ring and the cell
  // lists' pad absorb the rounding)
  const float ax = fmaf(p.grid_xi, ix, oix), bx = fmaf(p.grid_x1, ix, oix);
  const float az = fmaf(p.grid_zi, iz, oiz), bz = fmaf(p.grid_z1, iz, oiz);
  ta = fmaxf(ta, fmaxf(fminf(ax, bx), fminf(az, bz)));
  tb = fminf(tb, fminf(fmaxf(ax, bx), fmaxf(az, bz)));
  LP(kLpGridWalk, ta <= tb);
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
  // kGridLds: items and cells in LDS (ds_read: shorter latency than the L1
  // path and off the texture pipeline; 166 -> 157 ms).
  // kGridCells: the cells in LDS, the items from L1 / L2.
  const RT_GLOBAL uint32_t *__restrict__ cells = as_global(p.grid_cells);
  const RT_GLOBAL f4 *__restrict__ items = as_global(p.grid_items);
  // LDS placements: the walk's cell is the LDS byte address of its start
  // entry, so a DDA step adds +-2 or +-2 nx bytes
  constexpr bool LC = GP != kGridGlobal;
  const uint32_t lcells = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint16_t *)
                              reinterpret_cast<const uint16_t *>(s_grid_dyn + (GP == kGridLds ? p.grid_n_items : 0));
  // The walk stops on time alone: it leaves the inner box only at t ~ tb and
  // the next boundary is a whole cell further, so it never steps past the ring.
  int cell = LC ? (int)lcells + 2 * (cz * nx + cx) : cz * nx + cx;
  const int dcx = (nxs ? -1 : 1) * (LC ? 2 : 1), dcz = (nzs ? -nx : nx) * (LC ? 2 : 1);
  typedef const __attribute__((address_space(3))) uint16_t lds_u16;
  while (true) {
    LP(kLpDda, true);
    // STATS: boxes = lane-level cell visits; box_hits / roots = wave-level DDA
    // / item iterations (counted once per wave, by its first active lane)
    if (STATS) {
      ++wc.boxes;
      if (!RT_COUNT_ITEMS && lane_now() == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true))) ++wc.box_hits;
    }
    // kGridLds: cell i's items are [start_i, start_{i+1}): two ds_read_u16 of
    // adjacent entries give both LDS item addresses, with no decoding (see the
    // block's copy); the loop runs on the item pointer alone, compared with an
    // end the compiler cannot see through (else it rewrites the exit into a
    // separate counter).  kGridCells: the same two entries are item indices.
    // kGridGlobal: one u32 cell (first << 4 | count).
    if (GP == kGridLds) {
      lds_f4 *ip = (lds_f4 *)(uintptr_t)((lds_u16 *)(uintptr_t)cell)[0];
      lds_f4 *ie = (lds_f4 *)(uintptr_t)((lds_u16 *)(uintptr_t)cell)[1];
      // (both bounds behind one barrier: one wait for the two reads)
      asm volatile("" : "+v"(ip), "+v"(ie));
      if (ip != ie) do {
        grid_item<OPEN, STATS>(*ip, dx, dz, rl, tmin, hs, wc);
        ++ip;
      } while (ip != ie);
    } else {
      uint32_t k, ke;
      if (GP == kGridCells) {
        k = ((lds_u16 *)(uintptr_t)cell)[0];
        ke = ((lds_u16 *)(uintptr_t)cell)[1];
        asm volatile("" : "+v"(ke));
      } else {
        const uint32_t ce = cells[(uint32_t)cell];
        k = ce >> 4;
        ke = k + (ce & 15u);
      }
      // byte offsets from the items' base (saddr loads: no 64-bit address
      // per item; the loop steps the offset by 16)
      uint32_t ko = k << 4;
      const uint32_t koe = ke << 4;
      if (ko != koe) do {
        grid_item<OPEN, STATS>(*(const RT_GLOBAL f4 *)((const RT_GLOBAL char *)items + ko), dx, dz, rl, tmin, hs,
                               wc);
        ko += 16;
      } while (ko != koe);
    }
    // one compare picks the step axis and the next boundary (tmx == tmz
    // steps z, as before); v_min_f32 written out: fminf would first
    // canonicalise its operands
    const bool sx = tmx < tmz;
    const float tnext = sx ? tmx : tmz;
    float lim;
    asm("v_min_f32 %0, %1, %2" : "=v"(lim) : "v"(tb), "v"(hs.tmax));
    const bool stop = tnext > lim;
    // the step is taken before the exit test (a stopping lane's cell and
    // boundaries are dead after the loop): no exec-mask branch around it
    cell += sx ? dcx : dcz;
    tmx = sx ? tmx + tdx : tmx;
    tmz = sx ? tmz : tmz + tdz;
    asm volatile("" : "+v"(cell), "+v"(tmx), "+v"(tmz));
    if (stop) break;
  }
}

// Closest hit of the ray (o, d) over all spheres: hittable_list::hit,
// src/cpu/hittable_list.h:28-43.  Wave-uniform: every active lane of the wave
// calls it together; the result does not depend on which lanes those are.
// The scene parameters are re-read from the kernarg segment on entry
// (kernargs()): they live in SGPRs for the walk only, not across the whole
// bounce loop (SGPR pressure).
template <bool OPEN, bool BVH, bool STATS, bool GRID, int GP>
__device__ __forceinline__ hit_state closest_hit(float ox, float oy, float oz, float dx, float dy, float dz,
                                                 float tmin, work_ctr &wc) {
  const kparams p = kernargs();
  const RT_CONST pair_geom *__restrict__ scan_geom = as_const(p.scan_geom);
  const RT_CONST pair_geom *__restrict__ geom = as_const(p.geom);
  const RT_CONST bvh_node *__restrict__ nodes = as_const(p.nodes);
  const RT_CONST int *__restrict__ orig = as_const(p.orig);
  const int n_pairs = p.n_pad / 2;
  LP(kLpClosest, true);
  const float nk1 = -dot3(ox, oy, oz, dx, dy, dz);
  const float o2 = dot3(ox, oy, oz, ox, oy, oz);
  const float ox2 = -2.0f * ox, oy2 = -2.0f * oy, oz2 = -2.0f * oz;
  hit_state hs = no_hit();
  // the per-ray terms, splatted into pairs for the packed scans (the grid
  // build's extras and walk read the .x halves only)
  auto splat = [&]() {
    return ray_pre{{dx, dx}, {dy, dy}, {dz, dz}, {nk1, nk1}, {o2, o2}, {ox2, ox2}, {oy2, oy2}, {oz2, oz2}};
  };
  // the BVH boxes are padded for ray origins within |O| <= oref (see
  // bvh_builder); a wave-step with any lane beyond that scans everything
  const bool scan_all = !BVH || __builtin_amdgcn_ballot_w64(o2 > p.oref2) != 0;
  if (scan_all) {
    // brute force: 8 spheres (4 pairs) per iteration over the whole array
    const ray_pre rp = splat();
    for (int k = 0; k < n_pairs; k += 4)
      scan_pairs<OPEN, 4, STATS>(scan_geom + k, 2 * k, nullptr, rp, tmin, hs, wc.roots);
    if (STATS) wc.tests += 2 * n_pairs;
  } else {
    const ray_pre rp = splat();
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
    if (GRID || p.layer_mode) {  // (the grid build runs on layer scenes only)
      // the spheres off the layer (in the final scene the ground and the three
      // big spheres) are scanned first: their hits shorten tmax for the walk
      if (GRID) {
        // the first group leads with its largest sphere (the builder's order)
        // (kparams extra_geom / extra_orig: the host resolved the offsets)
        const RT_CONST pair_geom *__restrict__ xg = as_const(p.extra_geom);
        const RT_CONST int *__restrict__ xo = as_const(p.extra_orig);
        if (p.n_extra_pairs > 0) scan_extras<OPEN, STATS, true>(xg, 0, xo, rp, tmin, hs, wc.roots);
        for (int k = 2; k < p.n_extra_pairs; k += 2)
          scan_extras<OPEN, STATS, false>(xg + k, 2 * k, xo, rp, tmin, hs, wc.roots);
      } else {
        for (int k = 0; k < p.n_extra_pairs; k += 2)
          scan_pairs<OPEN, 2, STATS>(geom + p.extra_pair0 + k, 2 * (p.extra_pair0 + k), orig, rp, tmin, hs,
                                     wc.roots);
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
        ray_pre rg = rp;  // (.x halves only: the walk is per lane)
        rg.nk1.x = fmaf(p.layer_cy, dy, nk1);
        rg.o2.x = fmaf(p.layer_cy, oy2, o2);
        if (tyl_n <= tyl_fc) grid_walk<OPEN, STATS, GP>(ox, oz, ix, iz, oix, oiz, tyl_n, tyl_fc, rg, tmin, hs, wc);
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
        node = walk_step<OPEN, STATS, true>(nd, node, tn <= tf, geom, orig, rl, tmin, hs, wc, tyl_f, tyl_fc);
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
        node = walk_step<OPEN, STATS, false>(nd, node, tn <= tf, geom, orig, rp, tmin, hs, wc, 0.0f, unused);
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
// WIDE (scenes with an albedo above 1, rt_scene_upload): 64-bit pixel sums
//  and the radiance clamps below; the default build's
// code and registers are untouched.
template <bool OPEN, bool METAL_UNIT, bool BVH, bool STATS, bool GRID, int GP, bool WIDE>
__global__ __launch_bounds__(kBlock, 8) void render_kernel(const kparams p) {
  typedef typename std::conditional<WIDE, unsigned long long, uint32_t>::type sum_t;
  // Per-lane values that the bounce loop rarely needs are not kept live (VGPR
  // pressure at 8 waves): the wave keeps its tile origin (col0, lrow0, SGPRs),
  // the lane its current pixel slot, sample and global pixel index; column and
  // row are recomputed where they are used.
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >> 6;
  const unsigned entry = blockIdx.x * (unsigned)p.block_stride + (unsigned)p.block_base;
  const unsigned bid = p.block_order ? as_const(p.block_order)[entry] : entry;
  const int unit = (int)(bid % (unsigned)p.units);
  const int tile = (int)(bid / (unsigned)p.units) * kWavesPerBlock + wave;
  const int col0 = (tile % p.tiles_x) * kTile, lrow0 = (tile / p.tiles_x) * kTile;
  // this wave's samples: an even share of the launch's [s_lo, s_lo + s_cnt)
  const uint32_t s_begin = (uint32_t)p.s_lo + (uint32_t)((uint64_t)unit * (uint32_t)p.s_cnt / (uint32_t)p.units);
  const uint32_t s_end = (uint32_t)p.s_lo + (uint32_t)((uint64_t)(unit + 1) * (uint32_t)p.s_cnt / (uint32_t)p.units);
  // The wave's work pool: item k of [0, kend) is sample
  // s_begin + k / 64 of the tile's pixel slot k % 64 (x = slot % 8, y = slot /
  // 8).  A lane whose path ends takes the next item, so no lane idles while
  // the tile has samples left; a pixel's sum is an exact integer, whichever
  // lanes traced its samples in whatever order.
  const uint32_t kend = (s_end > s_begin ? s_end - s_begin : 0u) << 6;
  __shared__ sum_t s_sum[3][kBlock];                    // the tiles' fixed-point pixel sums
  // per tile row: the global pixel index of (x = 0, y) and how many of the
  // row's 8 slots are in the frame (0 for a row outside it): one ds_read_b64
  // per pool take gives both
  typedef uint32_t u2v __attribute__((ext_vector_type(2)));
  __shared__ u2v s_rowpix[kWavesPerBlock][kTile];
  {
    const int lane = lane_now();
    const int col = col0 + (lane & (kTile - 1));
    const int lrow = lrow0 + (lane >> 3);
    const int band = lrow / p.row_block;
    const int grow = (band * p.band_stride + p.band_offset) * p.row_block + (lrow - band * p.row_block);
    (void)col;
    if ((lane & (kTile - 1)) == 0) {
      const bool row_in = lrow < p.local_rows && grow < p.height;
      const uint32_t ncols = row_in ? (uint32_t)min(kTile, p.width - col0) : 0u;
      s_rowpix[wave][lane >> 3] = u2v{(uint32_t)grow * (uint32_t)p.width + (uint32_t)col0, ncols};
    }
  }
  s_sum[0][threadIdx.x] = s_sum[1][threadIdx.x] = s_sum[2][threadIdx.x] = 0u;
#ifdef RT_LANE_PROFILE
  if ((threadIdx.x & 63) < kLpRegions * 3) (&s_lane_prof[threadIdx.x >> 6][0][0])[threadIdx.x & 63] = 0u;
#endif
  if (GP == kGridLds) {  // the block's copy of the layer grid (kparams grid_n_items)
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
  } else if (GP == kGridCells) {  // the cell starts only, as item indices (< 2^16)
    uint16_t *sc = reinterpret_cast<uint16_t *>(s_grid_dyn);
    const RT_GLOBAL uint32_t *gc = as_global(p.grid_cells);
    for (int i = (int)threadIdx.x; i <= p.grid_n_cells; i += kBlock)
      sc[i] = (uint16_t)(i < p.grid_n_cells ? gc[i] >> 4 : (uint32_t)p.grid_n_items);
    __syncthreads();
  }
  float ox = 0.f, oy = 0.f, oz = 0.f, dx = 0.f, dy = 1.f, dz = 0.f;
  float tmin = 0.001f;  // the ray's t_min (normalize3: 0.001 |d| of its unnormalised direction)
  float thr = 1.f, thg = 1.f, thb = 1.f;
  int depth = 0;
  uint32_t slot = 0, sample = 0, pix = 0;
  int origin_sphere = -1;  // the sphere the ray starts on (-1: a camera ray)
  uint32_t segs = 0, steps = 0;
  work_ctr wc;  // executed work, STATS builds only
  // take pool item k: slot, sample and pixel; false if the slot is outside the
  // frame (the lane then stays alive without tracing and takes another item)
  // wave-uniform values the pool reads once per step, held in VGPRs: as SGPRs
  // they were spilled to VGPR lanes at 8 waves (v_readlane per step)
  uint32_t s_begin_v = s_begin;
  uint32_t rowpix_v = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) u2v *)&s_rowpix[wave][0];
  asm volatile("" : "+v"(s_begin_v), "+v"(rowpix_v));
  auto take = [&](uint32_t k) -> bool {
    slot = k & 63u;
    sample = s_begin_v + (k >> 6);
    const u2v e = ((const __attribute__((address_space(3))) u2v *)(uintptr_t)rowpix_v)[slot >> 3];
    pix = e.x + (slot & (kTile - 1));
    return (slot & (kTile - 1)) < e.y;
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
      tmin = camera_ray(p, pcg4d(pix, sample, 0u, p.seed32), col, grow, ox, oy, oz, dx, dy, dz);
    }
  }

  // a divergent loop: a lane leaves it when its wave's pool has no item left
  // for it (the step body then runs under the alive lanes' mask, with no
  // wave-level any-alive ballot per step)
  while (alive) {
    LP(kLpStep, tracing);
    hit_state hs = no_hit();
    if (tracing) hs = closest_hit<OPEN, BVH, STATS, GRID, GP>(ox, oy, oz, dx, dy, dz, tmin, wc);
    ++steps;
    const int best = best_of<OPEN>(hs);
    // lanes that end their path here (a miss) or hold a slot outside the frame
    // take their next items now: the step's one hash then draws the new camera ray
    const bool miss = !tracing || best < 0;
    uint32_t kn;
    {
      const uint64_t need = __builtin_amdgcn_ballot_w64(miss);
      kn = knext + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
      knext += (uint32_t)__builtin_popcountll(need);
    }
    bool path_done = false;  // absorbed, or the bounce limit: the lane parks for a step
    bool skipped = false;    // a spurious root: same ray from further along, same t_min
    {
      const kparams q = kernargs();  // shading's parameters, re-read per step
      if (tracing) ++segs;
      if (tracing && best < 0) {
        LP(kLpSky, true);
        // miss: sky gradient, src/cpu/main.cc:27-29; the sample's radiance
        // goes into its pixel's fixed-point sum
        const float a = 0.5f * (dy + 1.0f);
        const float s0 = 1.0f - a;
        const int i = wave * 64 + (int)slot;
        float xr = thr * fmaf(a, 0.5f, s0), xg = thg * fmaf(a, 0.7f, s0), xb = thb * (s0 + a);
        if (WIDE) {  // radiance above the format's bound is clamped (v <= vcap, rt_api.cpp sum_format)
          xr = fminf(xr, q.vcap);
          xg = fminf(xg, q.vcap);
          xb = fminf(xb, q.vcap);
        }
        xr *= q.qscale;
        xg *= q.qscale;
        xb *= q.qscale;
        sum_t nr = (sum_t)xr, ng = (sum_t)xg, nb = (sum_t)xb;
        if (q.dither) {  // spp >= 4096: stochastic rounding
          const float u = dither_u(pix, sample, q.seed32);
          nr += __builtin_amdgcn_fractf(xr) > u ? 1u : 0u;
          ng += __builtin_amdgcn_fractf(xg) > u ? 1u : 0u;
          nb += __builtin_amdgcn_fractf(xb) > u ? 1u : 0u;
        }
        atomicAdd(&s_sum[0][i], nr);
        atomicAdd(&s_sum[1][i], ng);
        atomicAdd(&s_sum[2][i], nb);
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
        LP(kLpHit, true);
        const float o2 = dot3(ox, oy, oz, ox, oy, oz);
        const float ox2 = -2.0f * ox, oy2 = -2.0f * oy, oz2 = -2.0f * oz;
        const float tmax = hs.tmax;
        const bool near = near_of(hs) != 0;
        // a 32-bit byte offset from the records' base (saddr addressing)
        static_assert(sizeof(shade_rec) == 64, "best << 6");
        const shade_rec sr = cload_g((const RT_GLOBAL shade_rec *)((const RT_GLOBAL char *)as_global(q.shade) +
                                                                   ((uint32_t)best << 6)));
        float b;
        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b);
        // A refined root before t_min on a sphere the ray moves away from
        // (b > 0): the ray starts on that sphere and leaves its ball, which it
        // cannot meet again; the expanded quadratic's root was an fp32 artefact
        // (DESIGN.md 2, step 3).  So is the exiting root of the very sphere
        // the ray starts on when it moves away from its centre: in exact
        // arithmetic that root is t = 0 (the origin is on the surface), but an
        // fp32 hit point can sit inside the ball by an ulp, which a bounce
        // with a tiny t_min (lambertian n + u with u ~ -n) then "exits" --
        // 6x as many paths entered sealed balls as in the reference's fp64
        // (DESIGN.md 2, step 4).  Not a segment: the ray walks again, same
        // direction -- in the first case from the scan's root point (>= t_min
        // further), in the second from the same origin with t_min raised just
        // past the scan's root, so that root cannot be taken again (moving the
        // origin instead can take ~t_exit / t_min re-walks, unbounded as
        // |n + u| -> 0).
        if (b > 0.0f && (t < tmin || (best == origin_sphere && !near))) {
          if (t < tmin) {
            ox = fmaf(tmax, dx, ox);
            oy = fmaf(tmax, dy, oy);
            oz = fmaf(tmax, dz, oz);
          } else {
            tmin = __uint_as_float(__float_as_uint(tmax) + 1u);  // nextafter(tmax, +inf), tmax > 0 finite
          }
          LP(kLpSkip, true);
          skipped = true;
          --segs;
        } else {
        const float px = fmaf(t, dx, ox), py = fmaf(t, dy, oy), pz = fmaf(t, dz, oz);
        // set_face_normal (hittable.h:16-19): dot(d, outward) < 0 is, in exact
        // arithmetic, "the entering root was taken" (outward flips for r < 0);
        // the root form cannot flip sign at grazing incidence in fp32.  The
        // flip is folded into the 1/r factor: (p - c) (-1/r) = -((p - c) / r)
        // exactly, one select instead of three negations
        const bool front = near != (sr.inv_r < 0.0f);
        const float fir = front ? sr.inv_r : -sr.inv_r;
        const float nx = (px - sr.cx) * fir, ny = (py - sr.cy) * fir, nz = (pz - sr.cz) * fir;
        // shared by the material branches (computed once: lanes of one wave
        // usually hit several materials, so the branches all execute)
        const float dn = dot3(dx, dy, dz, nx, ny, nz);
        float rx, ry, rz;
        reflect3(dx, dy, dz, nx, ny, nz, dn, rx, ry, rz);
        // three independent material blocks, each under its own lane mask (an
        // if / else-if chain compiles to a structurised exec-mask cascade of
        // ~35 scalar instructions; kinds are 0..2, rt_scene_upload checks)
        float sx = rx, sy = ry, sz = rz;
        bool scattered = true;
        const uint32_t kind = sr.kind;
        if (kind == RT_LAMBERTIAN) {
          LP(kLpLamb, true);
          // The opaque-inside rule: a sealed lambertian
          // sphere (no other ball overlaps its ball, rt_accel.cpp
          // sealed_spheres) hit at its exiting root -- the ray started inside
          // its ball, having got in past the surface within t_min of a contact
          // point (a glass sphere resting on the ground) -- ends the path black.
          // In the reference's arithmetic such a path hits the same sphere at
          // t = |r| after every scatter (its chords are n + u long) until the
          // depth cap; here it ends at once, without segments of up to 2000
          // units from origins beyond the grid's padding bound (C4's rank share
          // 408 -> 143 ms at 100 spp, profiles/r03d_c4_ab.log).  Keyed on the
          // root (near), not the face: a negative radius flips the face only.
          scattered = near || !sr.sealed;
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
        }
        if (kind == RT_METAL) {
          LP(kLpMetal, true);
          // material.h:40-46
          float fz = sr.param;
          if (!METAL_UNIT) fz *= ball_radius(r);  // random_in_unit_sphere
          sx = fmaf(fz, ux, rx);
          sy = fmaf(fz, uy, ry);
          sz = fmaf(fz, uz, rz);
          scattered = dot3(sx, sy, sz, nx, ny, nz) > 0.0f;
        }
        if (kind >= RT_DIELECTRIC) {
          LP(kLpDiel, true);
          // dielectric, material.h:57-87 (r0 is the same for ior and 1/ior)
          const float ratio = front ? sr.inv_param : sr.param;
          const float cos_t = fminf(-dn, 1.0f);
          // ratio sin > 1 (material.h:64), squared: no square root
          const bool cannot = (ratio * ratio) * fmaf(-cos_t, cos_t, 1.0f) > 1.0f;
          // (s = the reflection, set above, unless it refracts)
          if (!(cannot || schlick(cos_t, sr.r0) > unif(r.x))) refract3(dx, dy, dz, nx, ny, nz, cos_t, ratio, sx, sy, sz);
        }
        // attenuation = albedo (dielectrics store 1,1,1: the product is exact)
        thr *= sr.ar;
        thg *= sr.ag;
        thb *= sr.ab;
        if (WIDE) {  // albedos above 1: the throughput stays finite (inf x 0 would be NaN)
          thr = fminf(thr, 0x1p100f);
          thg = fminf(thg, 0x1p100f);
          thb = fminf(thb, 0x1p100f);
        }
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
          origin_sphere = best;
        }
        }
      } else if (tracing) {
        LP(kLpCamera, true);
        // a new item: its camera ray, with the lens sample drawn above
        int col, grow;
        pixel_cr(q, col, grow);
        camera_dir(q, r, ux, uy, col, grow, ox, oy, oz, dx, dy, dz);
        depth = 0;
        origin_sphere = -1;
        thr = thg = thb = 1.0f;
      }
    }
    // an absorbed path, or one at the bounce limit, parks its lane for a
    // step: the lane takes its next item with the misses of the next step
    // (one camera-ray path per step, with the step's one hash)
    if (path_done) tracing = false;
    LP(kLpTail, true);
    // one normalize3 per lane and step: the bounce direction or the new
    // camera ray's (a finished lane's is unused), and with it the ray's t_min
    // (a skipped ray keeps its own)
    const float tmin_new = normalize3(dx, dy, dz);
    tmin = skipped ? tmin : tmin_new;
  }

  const int lane = lane_now();
  {
    const kparams q = kernargs();
    const int col = col0 + (lane & (kTile - 1)), lrow = lrow0 + (lane >> 3);
    if (col < q.width && lrow < q.local_rows) {  // padding pixels (row >= height) write zeros
      const size_t o = 3 * ((size_t)lrow * q.width + col);
      const int i = wave * 64 + lane;
      if (!q.sum_atomic) {
        RT_GLOBAL float *out = as_global(q.out) + o;
        out[0] = (float)s_sum[0][i] * q.qinv;
        out[1] = (float)s_sum[1][i] * q.qinv;
        out[2] = (float)s_sum[2][i] * q.qinv;
      } else {  // the tile's units / launches add their integer sums (finish_sums converts)
        // (global, not generic, atomics: the product's device code holds no
        // flat memory instruction, DESIGN.md 8 "the v7 fault")
        RT_GLOBAL sum_t *acc = reinterpret_cast<RT_GLOBAL sum_t *>(as_global(q.out)) + o;  // WIDE: the 64-bit scratch frame
        __hip_atomic_fetch_add(acc + 0, s_sum[0][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(acc + 1, s_sum[1][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(acc + 2, s_sum[2][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
#ifdef RT_LANE_PROFILE
  if (lane < kLpRegions * 3)
    atomicAdd(&g_lane_prof[lane], (unsigned long long)(&s_lane_prof[wave][0][0])[lane]);
#endif
  // one atomic per wave for the counters
  uint32_t s = segs;
  // wave-steps: the most any lane of the wave looped
  uint32_t ws = steps;
  uint64_t lt = wc.tests, lb = wc.boxes, lh = wc.box_hits, lr = wc.roots;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s += __shfl_xor(s, off);
    ws = max(ws, (uint32_t)__shfl_xor(ws, off));
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
        as_global(k.tile_cost)[(int)blockIdx.x * kWavesPerBlock + wave] = s;
        return;
      }
    }
    RT_GLOBAL unsigned long long *counters = as_global(kernargs().counters) + 8 * (blockIdx.x & (kCounterSlots - 1));
    auto add = [](RT_GLOBAL unsigned long long *a, unsigned long long v) {
      __hip_atomic_fetch_add(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    add(&counters[0], s);
    add(&counters[1], ws);
    if (STATS) {
      add(&counters[2], lt);
      add(&counters[3], lb);
      add(&counters[4], lh);
      add(&counters[5], lr);
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

// The same for WIDE renders: the 64-bit sums live in the context's scratch
// frame (the caller's fp32 frame has 4 bytes per channel), converted into it.
__global__ __launch_bounds__(256) void finish_sums_wide(const uint64_t *__restrict__ sums, float *__restrict__ frame,
                                                        uint64_t n, float qinv) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256u)
    frame[j] = (float)sums[j] * qinv;
}

// Known-answer evaluation of the render kernel's own device arithmetic
// (rt_device_kat; tests/test_parity_gpu.py checks it against the reference's
// vectors in tests/golden/kat.jsonl).  Case layout: 10 doubles in, 9 out.
//   RT_KAT_SPHERE_HIT  in  o[3] d[3] c[3] r      (sphere::hit, src/cpu/sphere.h:24-51,
//                                                  t_min 0.001 in units of d, t_max inf)
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
    const float tmin = normalize3(dx, dy, dz);
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
    candidate<false>(e >= sr.ks, h, e - sr.ks, tie2_of<false>(0u), tmin, hs);
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

// ------------------------------------------------------------ launches ----
// render_kernel variant V (rt_layout.h kVar*): the grid bits count only with
// the BVH flag on a layer scene (without it they select the scan), and the
// placement only with the grid walk.
template <int V>
void launch_variant(unsigned blocks, size_t lds, hipStream_t st, const kparams &kp) {
  constexpr bool O = V & kVarOpen, U = V & kVarMetalUnit, B = V & kVarBvh, S = V & kVarStats;
  constexpr bool G = B && (V & kVarGrid), W = V & kVarWide;
  constexpr int P = G ? ((V >> kVarPlaceShift) & 3) % 3 : kGridGlobal;
  render_kernel<O, U, B, S, G, P, W><<<blocks, kBlock, G ? lds : 0, st>>>(kp);
}
using launch_fn = void (*)(unsigned, size_t, hipStream_t, const kparams &);
template <int... V>
constexpr auto launch_table(std::integer_sequence<int, V...>) {
  return std::array<launch_fn, sizeof...(V)>{&launch_variant<V>...};
}
constexpr auto kLaunch = launch_table(std::make_integer_sequence<int, 2 * kVarWide>{});

hipError_t launch_render(int variant, unsigned blocks, size_t lds_bytes, hipStream_t st, const kparams &kp) {
  if (variant < 0 || variant >= (int)kLaunch.size()) return hipErrorInvalidValue;
  kLaunch[variant](blocks, lds_bytes, st, kp);
  return hipGetLastError();
}

hipError_t launch_finish_sums(uint32_t *frame, uint64_t n, float qinv, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 256u * 64u);
  finish_sums<<<grid, 256, 0, st>>>(frame, n, qinv);
  return hipGetLastError();
}

hipError_t launch_finish_sums_wide(const uint64_t *sums, float *frame, uint64_t n, float qinv, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 256u * 64u);
  finish_sums_wide<<<grid, 256, 0, st>>>(sums, frame, n, qinv);
  return hipGetLastError();
}

hipError_t launch_tonemap(bool fp32, const float *sums, uint64_t n, int spp, const void *thresholds,
                          uint8_t *out, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<uint64_t>((n / 4 + 255) / 256 + 1, 256u * 32u);
  if (!fp32)
    tonemap_kernel<false, double><<<grid, 256, 0, st>>>(sums, n, 1.0 / spp, (const double *)thresholds, out);
  else
    tonemap_kernel<true, float><<<grid, 256, 0, st>>>(sums, n, 1.0f / (float)spp, (const float *)thresholds, out);
  return hipGetLastError();
}

hipError_t launch_kat(int kind, const double *in, int n, double *out) {
  kat_kernel<<<(unsigned)((n + 63) / 64), 64>>>(kind, in, n, out);
  return hipGetLastError();
}

hipError_t upload_turn_table() {
  float tab[2 * RT_TURN_TABLE];
  rt_turn_table(tab);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_turn_tab), tab, sizeof tab);
}

}  // namespace rtk

#ifdef RT_LANE_PROFILE
// the measurement variant's counters (tools/lane_profile.py): read (and, with
// reset != 0, zero) the kLpRegions x (waves, exec lanes, useful lanes) sums
extern "C" int rt_lane_profile_read(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtk::g_lane_prof), sizeof(rtk::g_lane_prof)) != hipSuccess) return -2;
  if (reset) {
    static const unsigned long long zero[rtk::kLpRegions * 3] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtk::g_lane_prof), zero, sizeof(zero)) != hipSuccess) return -2;
  }
  return rtk::kLpRegions;
}
#endif
