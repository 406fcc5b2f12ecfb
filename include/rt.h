/*
 * rt.h -- C ABI of the MI355X-native render path (librtow.so).
 *
 * The reference (kouei/ray-tracing-in-one-weekend) has no library or FFI; its
 * "interface" is (1) the process surface of cpu_ray_tracer / gpu_ray_tracer and
 * (2) the in-process kernel contract
 *     render(color *frame_buffer, camera *cam, hittable *world, seed)
 * (src/gpu/camera.h:169-195).  This header replaces (2) with plain pointers and
 * sizes; (1) is kept by the rt_* CLIs built on top of it.  Each entry point
 * names the reference code it stands in for.
 *
 * Conventions
 *  - Every function returns 0 (RT_OK) or a negative rt_status; no exit() inside.
 *  - Host arrays passed in are copied; the caller keeps ownership.
 *  - A context is bound to one HIP device and must be used from one host
 *    thread at a time.  Multi-GPU = one context per device (one process per
 *    GPU in bench.py, RCCL gather of the frame tiles).
 *  - Frame buffers are W * rows * 3 fp32, row-major, row 0 = TOP image row,
 *    holding UNNORMALISED per-pixel sums over spp samples (the reference's
 *    frame_buffer contract, src/gpu/camera.h:194).
 */
#ifndef RTOW_RT_H
#define RTOW_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 6 (round 6): the diagnostics (rt_device_kat, rt_internal_*) and the grid
 * phase options moved to rt_internal.h; this header is the drop-in boundary
 * alone.  5 (round 5): rt_tune_grid and rt_internal_grid_candidates removed,
 * RT_OPT_GRID_FIT, t_min in units of the unnormalised direction */
#define RT_ABI_VERSION 6

typedef enum {
  RT_OK = 0,
  RT_ERR_INVALID = -1,    /* bad argument (null pointer, bad size, bad enum) */
  RT_ERR_HIP = -2,        /* a HIP runtime call failed (see rt_last_hip_error) */
  RT_ERR_NOMEM = -3,      /* host or device allocation failed */
  RT_ERR_NO_DEVICE = -4,  /* no HIP device with that ordinal */
  RT_ERR_CAPACITY = -5,   /* caller buffer too small */
  RT_ERR_NO_SCENE = -6,   /* rt_render before rt_scene_upload */
  RT_ERR_IO = -7          /* write to fd failed */
} rt_status;

/* material kinds -- src/cpu/material.h:15-88 (lambertian, metal, dielectric) */
typedef enum { RT_LAMBERTIAN = 0, RT_METAL = 1, RT_DIELECTRIC = 2 } rt_material_kind;

/* camera models -- src/cpu/camera.h (default, parity) / src/gpu/camera.h */
typedef enum { RT_CAMERA_CPU = 0, RT_CAMERA_GPU = 1 } rt_camera_model;

/* render flags (semantic switches between the two reference variants,
 * SURVEY Appendix A).  0 = src/cpu semantics. */
enum {
  RT_FLAG_OPEN_INTERVAL = 1u << 0,     /* interval::surrounds, src/gpu/sphere.h:31-36 */
  RT_FLAG_METAL_UNIT_VECTOR = 1u << 1, /* fuzz*random_unit_vector, src/gpu/material.h:51-52 */
  RT_FLAG_GPU_SEMANTICS = RT_FLAG_OPEN_INTERVAL | RT_FLAG_METAL_UNIT_VECTOR,
  /* bookkeeping, not semantics: do not zero the context's segment counters
   * before this launch (rt_collect_stats then reports the sum over launches
   * since the last rt_reset_stats) */
  RT_FLAG_KEEP_COUNTERS = 1u << 8,
  /* acceleration, not semantics: walk a BVH built by rt_scene_upload instead
   * of scanning every sphere.  Same per-sphere arithmetic and an
   * order-independent tie rule, so the result is bit-identical to the scan. */
  RT_FLAG_ACCEL_BVH = 1u << 9,
  /* count executed ray-sphere and ray-box tests (rt_stats.sphere_tests /
   * box_tests); selects an instrumented kernel build, for measurement runs */
  RT_FLAG_COUNT_WORK = 1u << 10,
  /* scheduling, not semantics: launch the most expensive tiles first.  The
   * first render of a new frame geometry (size, band, camera, flags) runs a
   * 4-spp pilot that measures every tile's segments and sorts the blocks on
   * the device (enqueued, no host sync); later renders reuse the order
   * (DESIGN.md 6). */
  RT_FLAG_PILOT_SCHEDULE = 1u << 11,
  /* acceleration, not semantics (with RT_FLAG_ACCEL_BVH): when the scene is a
   * thin layer of like spheres plus a few others, rt_scene_upload builds an
   * x-z grid over the layer and the render walks it per lane;
   * this flag walks the layer BVH instead.  Same image either way. */
  RT_FLAG_LAYER_BVH = 1u << 12
};

/* Scene as structure-of-arrays; n spheres.  Replaces the device-heap
 * hittable_list of virtual sphere objects (src/gpu/hittable_list.h:49-65,
 * src/gpu/sphere.h) and the shared_ptr list of src/cpu/hittable_list.h. */
typedef struct {
  uint32_t n;
  const float *cx, *cy, *cz, *radius; /* n each; radius may be negative */
  const uint32_t *mat_kind;           /* n, rt_material_kind */
  const float *albedo_rgb;            /* 3n (ignored for dielectric) */
  const float *mat_param;             /* n: metal fuzz (already min(f,1)) | ior */
} rt_scene_view;

/* Caller-owned output buffers for the host scene builders. */
typedef struct {
  uint32_t capacity; /* entries available in every array below */
  uint32_t n;        /* written: number of spheres */
  float *cx, *cy, *cz, *radius;
  uint32_t *mat_kind;
  float *albedo_rgb; /* 3 * capacity */
  float *mat_param;
} rt_scene_buf;

/* Camera, already reduced to what get_ray needs (fp32, computed in fp64).
 *  CPU model (src/cpu/camera.h:28-34):
 *    s=(i+x)/(W-1), t=(j+y)/(H-1) with j counted from the bottom row,
 *    target = corner + s*horiz + t*vert        (corner = lower_left_corner)
 *  GPU model (src/gpu/camera.h:153-167):
 *    target = corner + (i+x-0.5)*horiz + (row+y-0.5)*vert
 *                                               (corner = pixel00_loc,
 *                                                horiz/vert = pixel_delta_u/v)
 *  origin = eye + dx*lens_u + dy*lens_v, (dx,dy) uniform in the unit disk,
 *  applied only when has_lens != 0. */
typedef struct {
  int32_t model; /* rt_camera_model */
  int32_t has_lens;
  float eye[3];
  float corner[3];
  float horiz[3];
  float vert[3];
  float lens_u[3]; /* lens_radius * u  (gpu: defocus_disk_u) */
  float lens_v[3]; /* lens_radius * v  (gpu: defocus_disk_v) */
} rt_camera;

/* Render parameters.  Rows are partitioned across ranks in interleaved bands
 * (SURVEY 8e): local row r of this rank is global row
 *     ((r / row_block) * band_stride + band_offset) * row_block + r % row_block
 * Rows >= height are padding and come out as zeros.  A single-GPU render is
 * row_block = height (or any), band_stride = 1, band_offset = 0,
 * local_rows = height. */
typedef struct {
  int32_t width, height;
  int32_t spp, max_depth; /* each < 2^24 (the RNG's counters) */
  uint64_t seed;
  int32_t row_block;
  int32_t band_stride;
  int32_t band_offset;
  int32_t local_rows;
  uint32_t flags;
  /* scheduling, not semantics: split every tile's samples into this many
   * even shares, one wave each; 0 = choose from the tile count (1 for a 4K
   * frame on one GPU, up to 8 when a rank's share of the frame is small) */
  uint32_t units;
} rt_params;

/* Pixel sums (part of the result, like the RNG): a sample's radiance v (at
 * most 1 when every albedo lies in [0, 1]) adds q(v * 2^F) to its pixel's
 * uint32 sum, F = 31 - floor(log2(spp)); the frame holds sum * 2^-F.  A scene
 * with an albedo A > 1 (energy-creating, as the reference allows) uses 64-bit
 * sums: v is clamped at vcap = min(A^(max_depth-1), 2^24) and F = 62 -
 * floor(log2(spp)) - ceil(log2(vcap)).  A^(max_depth-1) bounds a sample's
 * radiance in exact arithmetic; the fp32 throughput, a product of rounded
 * factors, can exceed it by a few ulps, so below 2^24 the clamp may trim such a
 * sample at the ulp level (the oracle applies the same clamp).  At 2^24 > spp a
 * clamped sample alone makes its pixel white in write_color, so there only the
 * fp32 sums of saturated pixels differ from an unclamped sum.  q truncates
 * for spp < 4096 (F >= 20: a bias below 2^-20 per sample, under 0.03 of a
 * tonemap level on the darkest visible pixel) and rounds stochastically for
 * 4096 <= spp < 2^24, trunc(x) + (frac(x) > u) with u a uniform draw keyed by
 * (pixel, sample): unbiased for every spp the ABI accepts.  Integer sums do
 * not depend on the order, so samples can be traced by any lanes, waves
 * (rt_params.units), launches or GPUs without changing a single bit of the
 * image.  The reference sums in fp64 (src/cpu/main.cc:114-119) or fp32
 * (src/gpu/camera.h:189-194) with no such format.
 * RT_CHUNK_SPP is kept for source compatibility (ABI 1 summed fp32 in chunks
 * of 64 samples; ABI 2 was never released); nothing depends on it any more. */
#define RT_CHUNK_SPP 64

typedef struct {
  uint64_t segments;     /* closest-hit queries (= hittable_list::hit calls) */
  uint64_t samples;      /* primary samples rendered (width * in-frame rows * spp) */
  uint64_t bf_tests;     /* brute-force equivalent ray-sphere tests: segments * spheres */
  uint64_t sphere_tests; /* executed lane-level ray-sphere tests (RT_FLAG_COUNT_WORK only) */
  uint64_t box_tests;    /* executed lane-level ray-box tests (RT_FLAG_COUNT_WORK only) */
  uint64_t box_hits;     /* ... of which the lane's own ray entered the box (the rest are
                            visits forced by other lanes of the wave) */
  uint64_t wave_steps;   /* sum over waves of bounce iterations (lane-efficiency denominator / 64) */
  double kernel_ms;      /* hipEvent time of the render kernel (0 if async) */
  uint64_t root_tests;   /* RT_FLAG_COUNT_WORK: per alive lane and bounce, the spheres whose
                            root / interval code the wave executed (some lane's line met it) */
  uint64_t launches;     /* render kernel launches (bounded block / sample ranges, RT_OPT_LAUNCH_SAMPLES) */
} rt_stats;

typedef struct rt_context rt_context;

/* ---- misc ---- */
int rt_abi_version(void);
const char *rt_strerror(int status);
int rt_last_hip_error(void); /* hipError_t of the last RT_ERR_HIP on this thread */
int rt_device_count(int *count);

/* ---- host scene / camera builders (run once per frame, fp64 host code) ---- */

/* Final random-spheres scene, random_scene() src/cpu/main.cc:32-76.
 * Draws from std::mt19937 (default seed 5489) through
 * uniform_real_distribution<double> in the order g++ 11 evaluates the
 * reference's argument lists (z-jitter before x-jitter, vec3 components
 * z,y,x -- SURVEY 8a-1), then casts to fp32.  half_extent = 11 gives the
 * reference's 22x22 grid (486 spheres); 50 gives the 10 000-sphere stress
 * scene of BASELINE config 5.  If rng_next is non-null it receives the next
 * random_double() after the scene (the reference renders from that point). */
int rt_scene_final(int half_extent, rt_scene_buf *out, double *rng_next);

/* Five-sphere book scene (archive-gpu/image22/main.cu:23-38; hollow glass
 * sphere of negative radius). */
int rt_scene_five(rt_scene_buf *out);

/* camera::camera, src/cpu/camera.h:8-26 */
int rt_camera_cpu(const double lookfrom[3], const double lookat[3],
                  const double vup[3], double vfov_deg, double aspect,
                  double aperture, double focus_dist, rt_camera *out);

/* new_camera, src/gpu/camera.h:53-110 (image size decides the viewport) */
int rt_camera_gpu(const double lookfrom[3], const double lookat[3],
                  const double vup[3], double vfov_deg, int width, int height,
                  double defocus_angle_deg, double focus_dist, rt_camera *out);

/* ---- device context ---- */
int rt_context_create(int device_ordinal, rt_context **out);
/* Waits for everything enqueued on the context's device, then frees. */
void rt_context_destroy(rt_context *ctx);

/* Options of a context: placement, shape and launch granularity, never
 * semantics (every value renders the same image).  value 0 restores the
 * default; RT_ERR_INVALID for an unknown option or a value out of range.
 * The structure options are read by the next rt_scene_upload, the launch
 * option by every render.  They replace environment variables, so a
 * render's behaviour depends only on its arguments. */
typedef enum {
  /* where a launch keeps the layer grid: RT_GRID_AUTO (0),
   * RT_GRID_LDS (1: cells and items in LDS when they fit), RT_GRID_CELLS_LDS
   * (2: cells in LDS, items from L1/L2; the cells are built coarser until they
   * fit), RT_GRID_GLOBAL (3) */
  RT_OPT_GRID_PLACEMENT = 1,
  RT_OPT_GRID_SCALE = 2,      /* layer-grid cell side multiplier, 0.05..20 (default 1) */
  RT_OPT_BVH_LEAF = 3,        /* spheres per BVH leaf, 1..4 (default 4) */
  RT_OPT_BVH_COLLAPSE = 4,    /* BVH node collapse area ratio (default 0.35) */
  RT_OPT_BVH_SIDE = 5,        /* SAH weight of the x- and z-facing sides (default 1) */
  /* about this many samples (pixels x samples per pixel) per render kernel
   * launch at most (default 2^35, ~1.2 s at C4's density; 2^32 until round
   * 5): a render is split into launches of bounded length (no
   * monolithic launch; a C4 frame on one GPU runs as 16).  The render's
   * work entries (4-tile blocks x units) are first split by samples: `chunks`
   * launches over every entry, each tracing spp / chunks samples per pixel.
   * When that would leave a wave fewer than 100 samples per pixel, the
   * entries are split as well, into `ranges` strided subsets (range r runs
   * entries r, r + ranges, r + 2 ranges, ... of the block order, however few
   * that is), and the samples into chunks of about 250 per wave; a launch
   * holds at least one sample per pixel.  At most 65536 launches per render:
   * a smaller budget is raised to total samples / 65536.
   * rt_internal_launch_plan shows the plan. */
  RT_OPT_LAUNCH_SAMPLES = 6,
  /* 1 (default): the layer grid's cell size is fitted to each frame geometry
   * (camera and frame size) on its first render, by a host-side model of the
   * walk's cost over the builder's candidate sizes (scale s0 (1 + 0.01 k),
   * k = 0..30, that fit the grid's LDS placement); 0: the builder's grid.
   * No fitting either when RT_OPT_GRID_SCALE is set (non-zero).  Set before
   * rt_scene_upload.  Scheduling only: every size renders the same image. */
  RT_OPT_GRID_FIT = 7
  /* 8, 9: internal tuning options (rt_internal.h) */
} rt_option;
enum { RT_GRID_AUTO = 0, RT_GRID_LDS = 1, RT_GRID_CELLS_LDS = 2, RT_GRID_GLOBAL = 3 };
int rt_context_set_option(rt_context *ctx, int option, double value);

/* Copies the scene to the device (scan records, BVH, shading records) and
 * builds the BVH.  Replaces new_world<<<1,1>>> (src/gpu/main.cu:18-75).
 * Synchronises the device first: renders still running on any stream keep
 * the previous scene.  Centres must be finite, radii finite and non-zero,
 * and the albedos of lambertian and metal spheres finite and >= 0
 * (RT_ERR_INVALID otherwise: a negative albedo gives the reference's
 * write_color a NaN).  Albedos above 1 are accepted, as the reference's
 * constructors accept them (src/cpu/material.h:17,38): renders of such a
 * scene use 64-bit pixel sums (see rt_params).  Metal fuzz above 1 is
 * clamped to 1, as the reference's metal constructors do
 * (src/cpu/material.h:38, src/gpu/material.h:45). */
int rt_scene_upload(rt_context *ctx, const rt_scene_view *scene);

/* Enqueue the render kernel on `stream` (a hipStream_t, NULL = the context's
 * own stream) writing params->width * params->local_rows * 3 floats to the
 * DEVICE pointer accum_rgb.  Replaces render<<<>>> (src/gpu/camera.h:169-195),
 * one monolithic launch in the reference (src/gpu/main.cu:130): here the
 * frame is split into launches of about RT_OPT_LAUNCH_SAMPLES samples at
 * most (block ranges, then sample ranges), each checked for a launch error
 * as it is enqueued.
 * Does not synchronise, also not on the first render of a frame geometry
 * with RT_FLAG_PILOT_SCHEDULE (the pilot and its sort are enqueued too).
 * Renders of one context on different streams run one after another (each
 * waits for the previous one's event): they share the context's scratch
 * buffers.  Segment counters are read by rt_collect_stats after the stream has
 * completed. */
int rt_render_async(rt_context *ctx, const rt_camera *cam, const rt_params *params,
                    float *accum_rgb, void *stream);

/* Synchronous convenience: render into a context-owned device buffer, time the
 * kernel with hipEvents, copy the sums to HOST memory host_rgb
 * (width*local_rows*3 floats) and fill stats (may be NULL).  kernel_ms spans
 * the render launches (and finish_sums when several units or launches share a
 * tile), not a first-frame pilot.  Waits launch by launch, so a device fault
 * is reported after the launch it happened in. */
int rt_render(rt_context *ctx, const rt_camera *cam, const rt_params *params,
              float *host_rgb, rt_stats *stats);

/* Progress of the last rt_render_async / rt_render of this context, without
 * blocking: how many of its bounded launches (RT_OPT_LAUNCH_SAMPLES) have
 * completed, of how many.  RT_ERR_HIP if the device reported a fault in one
 * of them -- the early failure report the reference's one launch cannot give
 * (src/gpu/main.cu:130-131 learns of a fault only at cudaDeviceSynchronize). */
int rt_render_progress(rt_context *ctx, uint32_t *launches_done, uint32_t *launches_total);

/* Stats of the last rt_render_async (or, with RT_FLAG_KEEP_COUNTERS, of all
 * launches since rt_reset_stats); call after the stream has completed. */
int rt_collect_stats(rt_context *ctx, rt_stats *stats);

/* Zero the segment counters (enqueued on `stream`, NULL = context stream). */
int rt_reset_stats(rt_context *ctx, void *stream);

/* ---- output (write_color src/cpu/color.h:8-23, output_image
 *      src/gpu/camera.h:197-210) ---- */

/* tonemap arithmetic: the two references' write_color */
typedef enum {
  RT_TONEMAP_CPU = 0, /* src/cpu/color.h:8-23: scale = 1.0/spp, sqrt, clamp in fp64 */
  RT_TONEMAP_GPU = 1  /* src/gpu/color.h:16-38: scale = 1.0f/spp, sqrtf, clamp in fp32 */
} rt_tonemap_mode;

/* int(256 * clamp(sqrt(sum/spp), 0, 0.999)) per channel, fp64 like src/cpu. */
int rt_tonemap_u8(const float *sums_rgb, size_t n_pixels, int spp, uint8_t *out_rgb);

/* The same on the host in either arithmetic (RT_TONEMAP_GPU: the fp32 levels of
 * src/gpu's output_image, which can differ by one from the fp64 ones on a level
 * boundary).  Threaded for large frames. */
int rt_tonemap_u8_mode(const float *sums_rgb, size_t n_pixels, int spp, int mode, uint8_t *out_rgb);

/* write_color on the DEVICE: d_sums (3 * n_pixels fp32 sums, e.g. a frame tile
 * from rt_render_async) -> d_out (3 * n_pixels bytes), enqueued on `stream`
 * (NULL = the context's stream).  Bit-identical to rt_tonemap_u8_mode with
 * the same mode.  Lets a multi-GPU render gather bytes (3 B per pixel) instead
 * of fp32 sums (12 B). */
int rt_tonemap_async(rt_context *ctx, const float *d_sums, size_t n_pixels, int spp, int mode,
                     uint8_t *d_out, void *stream);

/* "P3\nW H\n255\n" + one "r g b\n" line per pixel (binary P6 if binary!=0).
 * Rows are written top to bottom, as both references do.  Streams: P3 text is
 * formatted in bounded chunks by several threads and written in order (no
 * whole-file buffer), so a 16384 x 16384 frame needs megabytes, not 3 GB. */
int rt_write_ppm(int fd, const uint8_t *rgb, int width, int height, int binary);

#ifdef __cplusplus
}
#endif
#endif /* RTOW_RT_H */
