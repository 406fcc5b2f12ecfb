// rt_api.cpp -- the host half of the C ABI (include/rt.h): device contexts,
// scene upload, the render launches (pilot schedule, unit shares, bounded
// block- and sample-range launches), stats, the device tonemap and the diagnostics.
// Host C++ over the HIP runtime; the kernels and their launch wrappers live
// in rt_kernel.hip, the acceleration-structure builder in rt_accel.cpp.
//
// Replaces the host side of src/gpu/main.cu:86-156: new_world / new_camera
// (scene and camera reach the device by copy and by value), the one
// render<<<>>> launch (here: one or more bounded launches) and
// checkCudaErrors' exit(99) (status codes; the CLI maps them to exit 99).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <new>
#include <vector>

#include "rt_internal.h"
#include "rt_accel.h"
#include "rt_layout.h"

extern "C" void rt_internal_set_hip_error(int e);
extern "C" hipError_t rt_internal_block_order(const uint32_t *tile_cost, uint32_t blocks, uint32_t units,
                                              uint32_t *order, hipStream_t st);

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
  int grid_placement = rtk::kGridGlobal;  // rtk::kGrid*: where a launch keeps the grid
  float grid_x0 = 0, grid_z0 = 0, grid_xi = 0, grid_zi = 0, grid_x1 = 0, grid_z1 = 0, grid_g = 0;
  int grid_nx = 0, grid_nz = 0;
  double grid_scale = 1.0;
  // the layer grid's cell size fitted per frame geometry (rtk::grid_fitter,
  // DESIGN.md 3.3): the fitter, the geometry its grid was fitted for, and the
  // host copy the last refit uploads from (ev_fit: after that copy)
  rtk::grid_fitter *fitter = nullptr;
  std::vector<uint64_t> fit_key;
  rtk::grid_geom fit_grid;
  size_t cells_cap = 0, items_cap = 0;  // d_grid_cells / d_grid_items capacity (u32 / items)
  hipEvent_t ev_fit = nullptr;
  bool fit_pending = false;
  bool grid_fit = true;         // RT_OPT_GRID_FIT
  bool grid_scale_set = false;  // RT_OPT_GRID_SCALE given: no fitting
  unsigned long long *d_counters = nullptr;
  float *d_frame = nullptr;
  size_t frame_floats = 0;
  // block schedule from a pilot render, cached per frame geometry
  uint32_t *d_order = nullptr;
  size_t order_n = 0;
  std::vector<uint64_t> order_key;
  uint64_t last_samples = 0;
  uint32_t last_launches = 0;  // launches since the counters were last zeroed
  uint32_t enq_launches = 0;   // launches of the last render_enqueue
  bool last_stats = false;
  // Renders of one context may be enqueued on different streams; they share
  // the scratch buffer above (block order), so each render first
  // waits for the previous one: ev_done is recorded after every render on
  // last_stream, and a render on another stream waits on it (no host sync).
  hipEvent_t ev_done = nullptr;
  hipStream_t last_stream = nullptr;
  bool have_done = false;
  // one event after each bounded launch of the last render: rt_render waits
  // on them in turn (a fault surfaces after the launch it happened in),
  // rt_render_progress queries them
  std::vector<hipEvent_t> ev_launch;
  double tonemap_thr64[257];  // rt_tonemap_async level thresholds (see tonemap_thresholds)
  float tonemap_thr32[257];
  double *d_thr64 = nullptr;
  float *d_thr32 = nullptr;
  // the scene's largest lambertian / metal albedo: above 1, 64-bit pixel sums
  // (sum_format), with a 64-bit scratch frame for atomic renders
  double max_albedo = 0.0;
  uint64_t *d_wide = nullptr;
  size_t wide_n = 0;
  // rt_context_set_option
  rtk::accel_options opt;
  double launch_samples = rtk::kLaunchSamples;
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

void free_scene(rt_context *c) {
  (void)hipFree(c->d_geom);
  (void)hipFree(c->d_bvh_geom);
  (void)hipFree(c->d_nodes);
  (void)hipFree(c->d_orig);
  (void)hipFree(c->d_shade);
  (void)hipFree(c->d_grid_cells);
  (void)hipFree(c->d_grid_items);
  delete c->fitter;
  c->fitter = nullptr;
  c->fit_key.clear();
  c->cells_cap = c->items_cap = 0;
  c->d_grid_cells = nullptr;
  c->d_grid_items = nullptr;
  c->grid_nx = c->grid_nz = 0;
  c->grid_n_items = 0;
  c->grid_placement = rtk::kGridGlobal;
  c->d_geom = c->d_bvh_geom = nullptr;
  c->d_nodes = nullptr;
  c->d_orig = nullptr;
  c->d_shade = nullptr;
  c->n_spheres = c->n_pad = c->n_nodes = c->n_bvh_slots = 0;
  c->layer_mode = false;
  c->extra_pair0 = c->n_extra_pairs = 0;
  c->order_key.clear();  // the pilot's tile costs belong to the old scene
  c->max_albedo = 0.0;
}

template <class T>
hipError_t upload_vec(T **dst, const std::vector<T> &v, hipStream_t st) {
  hipError_t e = hipMalloc(dst, sizeof(T) * (v.empty() ? 1 : v.size()));
  if (e == hipSuccess && !v.empty())
    e = hipMemcpyAsync(*dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, st);
  return e;
}

// F = 31 - floor(log2(spp)): spp samples of at most 2^F each fit a uint32
int sum_bits(int spp) {
  int f = 31;
  for (int s = spp; s > 1; s >>= 1) --f;
  return f;
}

// The pixel sums' format (the oracle restates it).
// Albedos in [0, 1]: a sample's radiance is at most 1; uint32 sums, F = 31 -
// floor(log2 spp).  An albedo A above 1 (the reference accepts any,
// src/cpu/material.h:17,38): radiance up to A^(max_depth - 1), so 64-bit sums
// with vcap = min(A^(max_depth - 1), 2^24) (rounded down to fp32), a sample's
// radiance clamped at vcap, and F = 62 - floor(log2 spp) - ceil(log2 vcap)
// (spp samples of at most vcap 2^F, +1 each for the dither, fit 64 bits; F >=
// 14).  A^(max_depth - 1) bounds the radiance in exact arithmetic; the fp32
// throughput can exceed it by a few ulps, so below 2^24 the clamp may trim a
// sample at the ulp level (the oracle clamps alike: same bits).  At vcap =
// 2^24 > spp a clamped sample alone makes its pixel's mean >= 1, white in
// either write_color; only the fp32 sums of such pixels saturate.
struct sum_fmt {
  bool wide;
  int f;
  float vcap;
};
sum_fmt sum_format(int spp, int max_depth, double max_albedo) {
  if (!(max_albedo > 1.0)) return {false, sum_bits(spp), 1.0f};
  double v = max_depth > 1 ? std::pow(max_albedo, (double)(max_depth - 1)) : 1.0;
  v = std::min(std::max(v, 1.0), 16777216.0);
  float vc = (float)v;
  if ((double)vc > v) vc = std::nextafter(vc, 0.0f);
  int e = 0;
  const double m = std::frexp((double)vc, &e);  // vc = m 2^e, m in [0.5, 1)
  const int ceil_log2 = m == 0.5 ? e - 1 : e;
  return {true, sum_bits(spp) + 31 - ceil_log2, vc};
}

}  // namespace

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
    if ((e = rtk::upload_turn_table()) != hipSuccess) break;
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
  (void)hipFree(c->d_wide);
  (void)hipFree(c->d_thr64);
  (void)hipFree(c->d_thr32);
  for (hipEvent_t ev : c->ev_launch) (void)hipEventDestroy(ev);
  if (c->ev_done) (void)hipEventDestroy(c->ev_done);
  if (c->ev_fit) (void)hipEventDestroy(c->ev_fit);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int rt_context_set_option(rt_context *c, int option, double v) {
  if (!c || !std::isfinite(v)) return RT_ERR_INVALID;
  const bool dflt = v == 0.0;
  switch (option) {
    case RT_OPT_GRID_PLACEMENT: {
      static const int kMap[4] = {-1, rtk::kGridLds, rtk::kGridCells, rtk::kGridGlobal};
      if (v != std::floor(v) || v < 0 || v > 3) return RT_ERR_INVALID;
      c->opt.grid_placement = kMap[(int)v];
      return RT_OK;
    }
    case RT_OPT_GRID_SCALE:
      if (!dflt && !(v >= 0.05 && v <= 20.0)) return RT_ERR_INVALID;
      c->opt.grid_scale = dflt ? 1.0 : v;
      c->grid_scale_set = !dflt;
      return RT_OK;
    case RT_OPT_GRID_FIT:
      if (v != 0.0 && v != 1.0) return RT_ERR_INVALID;
      c->grid_fit = v != 0.0;
      return RT_OK;
    case RT_OPT_INTERNAL_GRID_PHASE_X:
    case RT_OPT_INTERNAL_GRID_PHASE_Z:
      if (!(v >= 0.0 && v < 1.0)) return RT_ERR_INVALID;
      (option == RT_OPT_INTERNAL_GRID_PHASE_X ? c->opt.grid_phase_x : c->opt.grid_phase_z) = v;
      return RT_OK;
    case RT_OPT_BVH_LEAF:
      if (v != std::floor(v) || v < 0 || v > 4) return RT_ERR_INVALID;
      c->opt.bvh_leaf = dflt ? 4 : (int)v;
      return RT_OK;
    case RT_OPT_BVH_COLLAPSE:
      if (!dflt && !(v > 0.0 && v <= 100.0)) return RT_ERR_INVALID;
      c->opt.collapse = dflt ? 0.35 : v;
      return RT_OK;
    case RT_OPT_BVH_SIDE:
      if (!dflt && !(v > 0.0 && v <= 100.0)) return RT_ERR_INVALID;
      c->opt.side = dflt ? 1.0 : v;
      return RT_OK;
    case RT_OPT_LAUNCH_SAMPLES:
      if (!dflt && !(v >= 1.0)) return RT_ERR_INVALID;
      c->launch_samples = dflt ? rtk::kLaunchSamples : std::floor(v);
      return RT_OK;
    default:
      return RT_ERR_INVALID;
  }
}

int rt_scene_upload(rt_context *c, const rt_scene_view *s) {
  if (!c || !rtk::scene_ok(s)) return RT_ERR_INVALID;
  rtk::accel_build a;
  rtk::accel_options o = c->opt;
  o.wide = rtk::max_albedo(s) > 1.0;
  rtk::grid_fitter *fitter = nullptr;
  rtk::build_accel(s, o, a, c->grid_fit && !c->grid_scale_set ? &fitter : nullptr);

  RT_HIP(hipSetDevice(c->device));
  // renders enqueued on caller streams may still read the old scene: they
  // are serialised and each ends by recording ev_done, so the last one's
  // event covers them all (this context's work only, not the whole device)
  {
    hipError_t e0 = c->have_done ? hipEventSynchronize(c->ev_done) : hipSuccess;
    if (e0 == hipSuccess) e0 = hipStreamSynchronize(c->stream);
    if (e0 != hipSuccess) {
      delete fitter;
      return hip_fail(e0);
    }
  }
  free_scene(c);
  c->fitter = fitter;
  hipError_t e = upload_vec(&c->d_geom, a.scan_geom, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_bvh_geom, a.bvh_geom, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_nodes, a.nodes, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_orig, a.slots, c->stream);
  if (e == hipSuccess) e = upload_vec(&c->d_shade, a.shade, c->stream);
  if (e == hipSuccess && !a.grid_cells.empty()) {
    e = upload_vec(&c->d_grid_cells, a.grid_cells, c->stream);
    if (e == hipSuccess) e = upload_vec(&c->d_grid_items, a.grid_items, c->stream);
    c->cells_cap = a.grid_cells.size();
    c->items_cap = a.grid_items.size() / 4;
    c->grid_n_items = a.grid_items.size() / 4;
    c->grid_placement = a.grid_placement;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    free_scene(c);
    return hip_fail(e);
  }
  c->n_spheres = a.n;
  c->max_albedo = rtk::max_albedo(s);
  c->n_pad = a.n_pad;
  c->n_nodes = (uint32_t)a.per_order;  // nodes holds 8 orders of this many
  c->n_bvh_slots = (uint32_t)a.slots.size();
  c->oref2 = (float)(0.99 * a.oref * a.oref);
  c->layer_mode = a.layer_mode;
  c->layer_lo = a.layer_lo;
  c->layer_cy = a.layer_cy;
  c->layer_hi = a.layer_hi;
  c->extra_pair0 = a.extra_pair0;
  c->n_extra_pairs = a.n_extra_pairs;
  c->grid_x0 = a.grid_x0;
  c->grid_xi = a.grid_xi;
  c->grid_zi = a.grid_zi;
  c->grid_z0 = a.grid_z0;
  c->grid_x1 = a.grid_x1;
  c->grid_z1 = a.grid_z1;
  c->grid_g = a.grid_g;
  c->grid_nx = a.grid_nx;
  c->grid_nz = a.grid_nz;
  c->grid_scale = a.grid_scale;
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

// the kernel arguments of the context's current layer grid
void grid_kparams(const rt_context *c, rtk::kparams &kp) {
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
}

// The kernel arguments of a render of (cam, prm) into accum_rgb with the
// context's scene and current grid (launch ranges, units and the sum format
// are set by the caller)
void fill_kparams(const rt_context *c, const rt_camera *cam, const rt_params *prm, float *accum_rgb,
                  rtk::kparams &kp) {
  std::memset(&kp, 0, sizeof kp);
  kp.block_stride = 1;  // entry = blockIdx.x (the pilot; the launches below set their ranges)
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
  grid_kparams(c, kp);
  kp.seed32 = (uint32_t)prm->seed ^ ((uint32_t)(prm->seed >> 32) * 0x9E3779B9u);
  kp.flags = prm->flags;
  kp.inv_wm1 = (float)(1.0 / (prm->width - 1));
  kp.inv_hm1 = (float)(1.0 / (prm->height - 1));
  kp.scan_geom = c->d_geom;
  kp.geom = c->d_bvh_geom;
  kp.nodes = c->d_nodes;
  kp.orig = c->d_orig;
  kp.extra_geom = c->d_bvh_geom ? c->d_bvh_geom + c->extra_pair0 : nullptr;
  kp.extra_orig = c->d_orig ? c->d_orig + 2 * (size_t)c->extra_pair0 : nullptr;
  kp.shade = c->d_shade;
  kp.out = accum_rgb;
  kp.counters = c->d_counters;
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
}

// render_kernel variant bits of a render (rt_layout.h kVar*)
int render_variant(const rt_context *c, const rt_params *prm, bool wide) {
  const bool grid = c->d_grid_cells && !(prm->flags & RT_FLAG_LAYER_BVH);
  const int place = grid ? c->grid_placement : rtk::kGridGlobal;
  return (wide ? rtk::kVarWide : 0) | ((prm->flags & RT_FLAG_OPEN_INTERVAL) ? rtk::kVarOpen : 0) |
         ((prm->flags & RT_FLAG_METAL_UNIT_VECTOR) ? rtk::kVarMetalUnit : 0) |
         ((prm->flags & RT_FLAG_ACCEL_BVH) ? rtk::kVarBvh : 0) |
         ((prm->flags & RT_FLAG_COUNT_WORK) ? rtk::kVarStats : 0) | (grid ? rtk::kVarGrid : 0) |
         (place << rtk::kVarPlaceShift);
}

// rt_render_async's body.  ev_start (may be null) is recorded on the stream
// just before the render kernel itself, after any one-time setup (the pilot,
// buffer growth), so that rt_render's kernel_ms times the render alone.
// How a render is cut into launches (render_enqueue; rt_internal_launch_plan
// shows it on the host).
struct launch_plan {
  long long units, ranges, chunks, entries;
};
launch_plan plan_launches(const rt_params *prm, double launch_samples) {
  const long long tiles_x = (prm->width + rtk::kTile - 1) / rtk::kTile;
  const long long tiles = tiles_x * ((prm->local_rows + rtk::kTile - 1) / rtk::kTile);
  const long long blocks = (tiles + rtk::kWavesPerBlock - 1) / rtk::kWavesPerBlock;
  const bool traced = prm->spp > 0 && prm->max_depth > 0;
  const double frame_px = (double)prm->width * (double)prm->local_rows;
  const double total = traced ? frame_px * prm->spp : 0.0;
  const double budget = std::max(launch_samples, total / (double)rtk::kMaxLaunches);
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
  if (!traced) units = 1;  // nothing is traced
  units = std::max(1LL, std::min<long long>(units, prm->spp));  // >= 1 sample per unit
  // Bounded launches: about `budget` samples per launch at most.
  // The plain split is by samples: `chunks` launches over every work entry
  // (a block of 4 tiles and a unit's share of their samples), each tracing
  // spp / chunks samples per pixel.  That keeps the launches wide (their
  // tails short) but shortens each wave's sample pool, whose own tail idles
  // lanes: ~2.2 / s of them at s samples per pixel per wave (lane efficiency
  // 0.995 at 500, 0.981 at 125, 0.861 at 16: C4's full frame on one GPU,
  // profiles/r03n_bench_c4.log).  Below kMinPoolSpp the work entries are
  // split too, into `ranges` strided subsets (range r runs entries r, r +
  // ranges, ... of block_order, so every launch keeps the expensive-first
  // order over a mix of the frame), and the samples into fewer, longer
  // chunks of about kPoolSpp per wave.  (Contiguous entry ranges lost 6 % on
  // C3's full frame to their launch tails,
  // profiles/r03o_contiguous_ranges_bench_c3.log.)  The
  // integer pixel sums make every split give the same image.
  long long entries = (long long)blocks * units;
  long long ranges = 1, chunks = 1;
  if (total > budget) {
    chunks = std::min<long long>(prm->spp, (long long)std::ceil(total / budget));
    const long long u1 = std::max(1LL, std::min<long long>(units, prm->spp / chunks));
    if ((double)prm->spp / (double)(u1 * chunks) >= rtk::kMinPoolSpp) {
      units = u1;
    } else {
      chunks = std::max(1LL, (long long)std::floor((double)prm->spp / ((double)units * rtk::kPoolSpp)));
      units = std::max(1LL, std::min<long long>(units, prm->spp / chunks));
      entries = (long long)blocks * units;
      ranges = std::min<long long>(entries, (long long)std::ceil(total / ((double)chunks * budget)));
      // entries too few for the budget: more sample ranges
      if (total / ((double)ranges * (double)chunks) > budget)
        chunks = std::min<long long>(prm->spp, (long long)std::ceil(total / ((double)ranges * budget)));
      units = std::max(1LL, std::min<long long>(units, prm->spp / chunks));
      entries = (long long)blocks * units;
      ranges = std::max(1LL, std::min({ranges, entries, rtk::kMaxLaunches / chunks}));
    }
  }
  return launch_plan{units, ranges, chunks, entries};
}

int render_enqueue_body(rt_context *c, const rt_camera *cam, const rt_params *prm, float *accum_rgb, hipStream_t st,
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
    c->last_launches = 0;
  }
  c->last_stats = (prm->flags & RT_FLAG_COUNT_WORK) != 0;
  c->enq_launches = 0;
  if (prm->width == 0 || prm->local_rows == 0) {
    if (ev_start) RT_HIP(hipEventRecord(ev_start, st));
    return RT_OK;
  }

  rtk::kparams kp;
  fill_kparams(c, cam, prm, accum_rgb, kp);
  const int tiles_y = (prm->local_rows + rtk::kTile - 1) / rtk::kTile;
  const long long tiles = (long long)kp.tiles_x * tiles_y;
  const unsigned blocks = (unsigned)((tiles + rtk::kWavesPerBlock - 1) / rtk::kWavesPerBlock);
  const bool grid = c->d_grid_cells && !(prm->flags & RT_FLAG_LAYER_BVH);
  if (grid && c->fitter && (prm->flags & RT_FLAG_ACCEL_BVH)) {
    // the layer grid's cell size for this frame geometry (rtk::grid_fitter:
    // a host-side model, once per geometry; the image is the same for every
    // size).  The new grid is copied into the context's buffers on st, after
    // every earlier render (renders of one context are serialised).
    std::vector<uint64_t> key = {(uint64_t)prm->width, (uint64_t)prm->height};
    const uint32_t *cw = reinterpret_cast<const uint32_t *>(cam);
    for (size_t k = 0; k < sizeof(rt_camera) / 4; ++k) key.push_back(cw[k]);
    if (key != c->fit_key) {
      const double scale = c->fitter->choose(*cam, prm->width, prm->height, nullptr);
      if (scale != c->grid_scale) {
        if (c->fit_pending) RT_HIP(hipEventSynchronize(c->ev_fit));  // fit_grid is still being read
        c->fit_pending = false;
        rtk::grid_geom &q = c->fit_grid;
        if (!c->fitter->build(scale, q)) return RT_ERR_INVALID;  // (every candidate fits: unreachable)
        // Transactional: larger buffers are allocated before the
        // old ones are freed, so a failed allocation leaves the old grid whole
        // (buffers, fields and fit_key describe it); once a copy into the
        // buffers has failed they hold neither grid, and grid_scale = NaN makes
        // the next grid render refit before it launches.
        if (q.cells.size() > c->cells_cap || q.items.size() / 4 > c->items_cap) {
          void *nc = nullptr, *ni = nullptr;
          hipError_t ea = hipMalloc(&nc, q.cells.size() * sizeof(uint32_t));
          if (ea == hipSuccess) ea = hipMalloc(&ni, q.items.size() * sizeof(float));
          if (ea == hipSuccess) ea = hipStreamSynchronize(st);  // earlier renders on st still read the old grid
          if (ea != hipSuccess) {
            (void)hipFree(nc);
            (void)hipFree(ni);
            return hip_fail(ea);
          }
          (void)hipFree(c->d_grid_cells);
          (void)hipFree(c->d_grid_items);
          c->d_grid_cells = static_cast<uint32_t *>(nc);
          c->d_grid_items = static_cast<float *>(ni);
          c->cells_cap = q.cells.size();
          c->items_cap = q.items.size() / 4;
        }
        c->grid_scale = std::numeric_limits<double>::quiet_NaN();
        c->fit_key.clear();
        RT_HIP(hipMemcpyAsync(c->d_grid_cells, q.cells.data(), q.cells.size() * sizeof(uint32_t),
                              hipMemcpyHostToDevice, st));
        RT_HIP(hipMemcpyAsync(c->d_grid_items, q.items.data(), q.items.size() * sizeof(float), hipMemcpyHostToDevice,
                              st));
        if (!c->ev_fit) RT_HIP(hipEventCreateWithFlags(&c->ev_fit, hipEventDisableTiming));
        RT_HIP(hipEventRecord(c->ev_fit, st));
        c->fit_pending = true;
        c->grid_n_items = q.items.size() / 4;
        c->grid_x0 = q.x0;
        c->grid_z0 = q.z0;
        c->grid_xi = q.xi;
        c->grid_zi = q.zi;
        c->grid_x1 = q.x1;
        c->grid_z1 = q.z1;
        c->grid_g = q.g;
        c->grid_nx = q.nx;
        c->grid_nz = q.nz;
        c->grid_scale = q.scale;
        grid_kparams(c, kp);
      }
      c->fit_key = key;
    }
  }
  const int place = grid ? c->grid_placement : rtk::kGridGlobal;
  const sum_fmt fmt = sum_format(prm->spp, prm->max_depth, c->max_albedo);
  const int v = render_variant(c, prm, fmt.wide);
  const size_t lds = rtk::grid_lds_bytes(place, kp.grid_n_items, kp.grid_n_cells);
  const bool traced = prm->spp > 0 && prm->max_depth > 0;
  const launch_plan lp = plan_launches(prm, c->launch_samples);
  const long long units = lp.units, ranges = lp.ranges, chunks = lp.chunks, entries = lp.entries;
  const long long launches = ranges * chunks;
  kp.units = (int)units;
  const int f = fmt.f;
  kp.qscale = std::ldexp(1.0f, f);
  kp.qinv = std::ldexp(1.0f, -f);
  kp.vcap = fmt.vcap;
  // F < 20 (spp >= 4096): truncation would bias a dark pixel by up to 2^-F per
  // sample (0.03 level at F = 20); stochastic rounding is unbiased for every
  // spp
  kp.dither = f < 20 ? 1 : 0;
  // disjoint block ranges write disjoint pixels: float stores suffice
  kp.sum_atomic = (units > 1 || chunks > 1) ? 1 : 0;
  const uint64_t frame_floats = (uint64_t)prm->local_rows * (uint64_t)prm->width * 3u;
  if ((prm->flags & RT_FLAG_PILOT_SCHEDULE) && traced && blocks > 1) {
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
        // the instrumented build with the grid in global memory, 4 samples,
        // one unit, float stores
        rtk::kparams pk = kp;
        pk.s_lo = 0;
        pk.s_cnt = std::min(prm->spp, 4);
        pk.units = 1;
        pk.sum_atomic = 0;
        pk.tile_cost = d_cost;
        pk.counters = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(d_cost) + cost_bytes);
        e = rtk::launch_render((v & ~(3 << rtk::kVarPlaceShift)) | rtk::kVarStats, blocks, 0, st, pk);
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
  // several units or launches per tile add their integer sums into the
  // zeroed frame (after the pilot, which renders into it too); finish_sums
  // converts them
  if (kp.sum_atomic && fmt.wide) {
    // 64-bit sums do not fit the caller's fp32 frame: a scratch frame of the
    // context's (renders of one context are serialised), converted at the end
    if (c->wide_n < frame_floats) {
      (void)hipFree(c->d_wide);
      c->d_wide = nullptr;
      c->wide_n = 0;
      RT_HIP(hipMalloc(&c->d_wide, frame_floats * sizeof(uint64_t)));
      c->wide_n = frame_floats;
    }
    RT_HIP(hipMemsetAsync(c->d_wide, 0, frame_floats * sizeof(uint64_t), st));
    kp.out = reinterpret_cast<float *>(c->d_wide);
  } else if (kp.sum_atomic) {
    RT_HIP(hipMemsetAsync(accum_rgb, 0, frame_floats * sizeof(float), st));
  }
  {
    while (c->ev_launch.size() < (size_t)launches) {
      hipEvent_t ev = nullptr;
      RT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      c->ev_launch.push_back(ev);
    }
  }
  if (ev_start) RT_HIP(hipEventRecord(ev_start, st));
  long long k = 0;
  kp.block_stride = (int)ranges;
  for (long long r = 0; r < ranges; ++r) {
    // entries r, r + ranges, r + 2 ranges, ... in block_order's order (most
    // expensive first with the pilot)
    kp.block_base = (int)r;
    const long long n_r = (entries - r + ranges - 1) / ranges;
    for (long long ch = 0; ch < chunks; ++ch, ++k) {
      const long long s0 = ch * prm->spp / chunks, s1 = (ch + 1) * prm->spp / chunks;
      kp.s_lo = (int)s0;
      kp.s_cnt = (int)(s1 - s0);
      // a launch that cannot start (bad configuration, lost device) stops the render here
      RT_HIP(rtk::launch_render(v, (unsigned)n_r, lds, st, kp));
      RT_HIP(hipEventRecord(c->ev_launch[(size_t)k], st));
    }
  }
  c->last_launches += (uint32_t)launches;
  c->enq_launches = (uint32_t)launches;
  if (kp.sum_atomic && fmt.wide)
    RT_HIP(rtk::launch_finish_sums_wide(c->d_wide, accum_rgb, frame_floats, kp.qinv, st));
  else if (kp.sum_atomic)
    RT_HIP(rtk::launch_finish_sums(reinterpret_cast<uint32_t *>(accum_rgb), frame_floats, kp.qinv, st));
  RT_HIP(hipEventRecord(c->ev_done, st));
  c->last_stream = st;
  c->have_done = true;
  return RT_OK;
}

// A render that fails after enqueuing some of its work on st (a refit copy,
// the pilot, the k-th launch) still ends with ev_done recorded on st, so that
// the next render on another stream, and rt_scene_upload before it frees the
// scene, wait for that work too (before, only hipFree's implicit
// device synchronisation covered it).
int render_enqueue(rt_context *c, const rt_camera *cam, const rt_params *prm, float *accum_rgb, hipStream_t st,
                   hipEvent_t ev_start) {
  const int r = render_enqueue_body(c, cam, prm, accum_rgb, st, ev_start);
  if (r != RT_OK && c->ev_done && hipEventRecord(c->ev_done, st) == hipSuccess) {
    c->last_stream = st;
    c->have_done = true;
  }
  return r;
}

// rt_render's frame buffer (only it uses d_frame, and it returns after its
// work is done)
hipError_t ensure_frame(rt_context *c, size_t nf) {
  if (nf <= c->frame_floats) return hipSuccess;
  (void)hipFree(c->d_frame);
  c->d_frame = nullptr;
  c->frame_floats = 0;
  const hipError_t e = hipMalloc(&c->d_frame, nf * sizeof(float));
  if (e == hipSuccess) c->frame_floats = nf;
  return e;
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

int rt_render_progress(rt_context *c, uint32_t *done, uint32_t *total) {
  if (!c || !done || !total) return RT_ERR_INVALID;
  const uint32_t n = std::min<uint32_t>(c->enq_launches, (uint32_t)c->ev_launch.size());
  *total = n;
  *done = 0;
  RT_HIP(hipSetDevice(c->device));
  // launches complete in order on their stream: count the leading finished ones
  for (uint32_t k = 0; k < n; ++k) {
    const hipError_t e = hipEventQuery(c->ev_launch[k]);
    if (e == hipErrorNotReady) break;
    if (e != hipSuccess) return hip_fail(e);  // a fault in or before launch k
    ++*done;
  }
  return RT_OK;
}

int rt_reset_stats(rt_context *c, void *stream) {
  if (!c) return RT_ERR_INVALID;
  RT_HIP(hipSetDevice(c->device));
  RT_HIP(hipMemsetAsync(c->d_counters, 0, 8 * rtk::kCounterSlots * sizeof(unsigned long long),
                        stream ? (hipStream_t)stream : c->stream));
  c->last_samples = 0;
  c->last_launches = 0;
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
  stats->launches = c->last_launches;
  return RT_OK;
}

int rt_render(rt_context *c, const rt_camera *cam, const rt_params *prm, float *host_rgb,
              rt_stats *stats) {
  if (!c || !params_ok(prm) || (!host_rgb && prm->local_rows && prm->width)) return RT_ERR_INVALID;
  const size_t nf = 3 * (size_t)prm->width * (size_t)prm->local_rows;
  RT_HIP(hipSetDevice(c->device));
  RT_HIP(ensure_frame(c, nf));
  if (!cam || (cam->model != RT_CAMERA_CPU && cam->model != RT_CAMERA_GPU)) return RT_ERR_INVALID;
  if (cam->model == RT_CAMERA_CPU && (prm->width < 2 || prm->height < 2)) return RT_ERR_INVALID;
  if (!c->d_geom) return RT_ERR_NO_SCENE;
  // ev0 is recorded right before the render kernel (after a first-frame pilot)
  int st = render_enqueue(c, cam, prm, c->d_frame, c->stream, c->ev0);
  const uint32_t n_launch = std::min<uint32_t>(c->enq_launches, (uint32_t)c->ev_launch.size());
  if (st != RT_OK) return st;
  RT_HIP(hipEventRecord(c->ev1, c->stream));
  // wait launch by launch: a fault surfaces after the launch it happened in
  for (uint32_t k = 0; k < n_launch; ++k) RT_HIP(hipEventSynchronize(c->ev_launch[k]));
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

// Host-only view of how rt_render would cut a render into launches (no
// device needed): tests/test_host.py checks the plans of the BASELINE configs.
int rt_internal_launch_plan(const rt_params *prm, double launch_samples, uint64_t *out, size_t n_out) {
  if (!out || !params_ok(prm) || !(launch_samples >= 0.0)) return RT_ERR_INVALID;
  const launch_plan lp = plan_launches(prm, launch_samples > 0.0 ? launch_samples : rtk::kLaunchSamples);
  const uint64_t v[RT_LAUNCH_PLAN_N] = {(uint64_t)lp.ranges, (uint64_t)lp.chunks, (uint64_t)lp.units,
                                        (uint64_t)lp.entries, (uint64_t)(lp.ranges * lp.chunks)};
  for (size_t i = 0; i < n_out && i < RT_LAUNCH_PLAN_N; ++i) out[i] = v[i];
  return RT_OK;
}

// Host-only view of what rt_scene_upload would build (no device needed):
// tests/test_host.py checks the builder's invariants on CPU, and
// tools/host_sanitize.sh runs it under ASan / UBSan.  See include/rt.h for
// the out[] layout.
int rt_internal_accel_info(const rt_scene_view *s, int grid_placement, double grid_scale, uint64_t *out,
                           size_t n_out) {
  if (!out || !rtk::scene_ok(s) || grid_placement < 0 || grid_placement > 3 ||
      !(grid_scale == 0.0 || (grid_scale >= 0.05 && grid_scale <= 20.0)))
    return RT_ERR_INVALID;
  static const int kMap[4] = {-1, rtk::kGridLds, rtk::kGridCells, rtk::kGridGlobal};
  rtk::accel_options o;
  o.wide = rtk::max_albedo(s) > 1.0;
  o.grid_placement = kMap[grid_placement];
  o.grid_scale = grid_scale == 0.0 ? 1.0 : grid_scale;
  rtk::accel_build a;
  rtk::build_accel(s, o, a);
  uint64_t v[RT_ACCEL_INFO_N];
  std::memset(v, 0, sizeof v);
  v[0] = a.per_order;
  v[1] = a.slots.size();
  v[2] = a.layer_mode ? 1u : 0u;
  v[3] = a.extra_pair0;
  v[4] = a.n_extra_pairs;
  v[5] = (uint64_t)a.grid_nx;
  v[6] = (uint64_t)a.grid_nz;
  const uint64_t items = a.grid_items.size() / 4, cells = a.grid_cells.size();
  v[7] = items;
  v[8] = cells ? rtk::grid_lds_bytes(a.grid_placement, (long long)items, (long long)cells) : 0u;
  v[9] = cells && a.grid_placement == rtk::kGridLds;
  // every stored cell's first item is the running count (ring cells included),
  // so cell i's items are [first_i, first_{i+1}) -- what the LDS walk reads
  uint64_t maxc = 0, listed = 0;
  bool start_ok = true, ring_ok = true;
  for (uint64_t i = 0; i < cells; ++i) {
    const uint32_t first = a.grid_cells[i] >> 4, cnt = a.grid_cells[i] & 15u;
    const uint64_t next = i + 1 < cells ? (a.grid_cells[i + 1] >> 4) : items;
    start_ok = start_ok && first + cnt == next;
    maxc = std::max<uint64_t>(maxc, cnt);
    listed += cnt ? 1u : 0u;
    const int x = (int)(i % a.grid_nx), z = (int)(i / a.grid_nx);
    if (x == 0 || z == 0 || x == a.grid_nx - 1 || z == a.grid_nz - 1) ring_ok = ring_ok && cnt == 0;
  }
  v[10] = maxc;
  v[11] = cells ? (start_ok ? 1u : 0u) : 0u;
  v[12] = cells ? (ring_ok ? 1u : 0u) : 0u;
  v[13] = (uint64_t)(a.oref * 1000.0);
  v[14] = a.layer_mode ? (uint64_t)(2 * a.extra_pair0) : 0u;
  v[15] = listed;
  static const uint64_t kPlaceOut[3] = {RT_GRID_GLOBAL, RT_GRID_LDS, RT_GRID_CELLS_LDS};
  v[16] = cells ? kPlaceOut[a.grid_placement] : 0u;
  v[17] = (uint64_t)std::llround(a.grid_scale * 1000.0);
  std::memcpy(out, v, std::min<size_t>(n_out, RT_ACCEL_INFO_N) * sizeof(uint64_t));
  return RT_OK;
}

int rt_internal_grid_fit(const rt_scene_view *s, const rt_camera *cam, int width, int height, double *scale,
                         double *costs, size_t n_costs, size_t *n) {
  return rt_internal_grid_fit_phase(s, cam, width, height, 0.0, 0.0, scale, costs, n_costs, n);
}

int rt_internal_grid_fit_phase(const rt_scene_view *s, const rt_camera *cam, int width, int height, double phase_x,
                               double phase_z, double *scale, double *costs, size_t n_costs, size_t *n) {
  if (!rtk::scene_ok(s) || !cam || !scale || width < 1 || height < 1 || (n_costs && !costs)) return RT_ERR_INVALID;
  if (!(phase_x >= 0.0 && phase_x < 1.0 && phase_z >= 0.0 && phase_z < 1.0)) return RT_ERR_INVALID;
  rtk::accel_options o;
  o.grid_phase_x = phase_x;
  o.grid_phase_z = phase_z;
  o.wide = rtk::max_albedo(s) > 1.0;
  rtk::accel_build a;
  rtk::grid_fitter *f = nullptr;
  rtk::build_accel(s, o, a, &f);
  *scale = 0.0;
  if (n) *n = 0;
  if (!f) return RT_OK;
  std::vector<std::pair<double, double>> cs;
  *scale = f->choose(*cam, width, height, &cs);
  delete f;
  if (n) *n = cs.size();
  for (size_t i = 0; i < cs.size() && i < n_costs; ++i) {
    costs[2 * i] = cs[i].first;
    costs[2 * i + 1] = cs[i].second;
  }
  return RT_OK;
}

int rt_internal_grid_scale(rt_context *c, double *scale) {
  if (!c || !scale) return RT_ERR_INVALID;
  *scale = c->d_grid_cells ? c->grid_scale : 0.0;
  return RT_OK;
}

int rt_internal_sealed(const rt_scene_view *s, uint8_t *out, size_t n_out) {
  if (!rtk::scene_ok(s) || (n_out && !out)) return RT_ERR_INVALID;
  std::vector<uint8_t> v;
  rtk::sealed_spheres(s, v);
  if (n_out && !v.empty()) std::memcpy(out, v.data(), std::min<size_t>(n_out, v.size()));
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
  if (e == hipSuccess) e = rtk::launch_kat(kind, d, (int)n_cases, d + 10 * n_cases);
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
  if (mode == RT_TONEMAP_CPU)
    RT_HIP(rtk::launch_tonemap(false, d_sums, n, spp, c->d_thr64, d_out, st));
  else
    RT_HIP(rtk::launch_tonemap(true, d_sums, n, spp, c->d_thr32, d_out, st));
  return RT_OK;
}

}  // extern "C"
