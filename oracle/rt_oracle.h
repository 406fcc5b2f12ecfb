/* oracle/rt_oracle.h -- TEST INFRASTRUCTURE ONLY (see rt_oracle.cc).
 * C ABI of the CPU restatement; loaded by tests/ via ctypes. */
#ifndef RTOW_ORACLE_H
#define RTOW_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "rt.h"
#ifdef __cplusplus
extern "C" {
#endif
/* fp64 restatement of src/cpu: height = (int)(width/aspect); writes
 * width*height*3 tonemapped bytes, TOP row first (src/cpu/main.cc:109-123).
 * scene 0 = final random scene (main.cc:32-76), 1 = five-sphere book scene.
 * rgb_out == NULL: size query (fills *height_out). */
/* Attribution only: segments the last rto_reference_render(_view) traced
 * after a path's first hit on the inside of a sealed lambertian sphere (the
 * opaque-inside rule's spheres), which the kernel's rule
 * does not trace. */
unsigned long long rto_reference_trapped(void);
/* Attribution only: paths the last rto_reference_render(_view) ended at the
 * depth cap (ray_color's depth <= 0, src/cpu/main.cc:16-17), and kernel-mode
 * paths ended there since the last reset (reset != 0 zeroes it). */
unsigned long long rto_reference_capped(void);
unsigned long long rto_kernel_capped(int reset);
/* Attribution only: kernel-mode counters summed over every render since the
 * last reset: out[0] spurious-root skips, out[1] paths' first hits on the
 * inside of a sealed sphere, out[2] those whose ray had just been moved on by
 * a skip.  reset != 0 zeroes them after reading. */
void rto_kernel_attrib(unsigned long long *out, int reset);
/* ... the first entries' (sphere entered, previous segment's sphere, depth,
 * t_min * 1e6), at most n of them (and 4096); returns how many. */
int rto_kernel_attrib_events(long long *out, int n, int reset);
int rto_reference_render(int width, double aspect, int spp, int max_depth, int scene,
                         uint8_t *rgb_out, int *height_out, unsigned long long *segments);
/* The same for any scene (the final scene's camera, src/cpu/main.cc:90-97;
 * no scene draws precede the samples): what the reference harness renders
 * for a `file:` scene (oracle/ref_harness.cc). */
int rto_reference_render_view(const rt_scene_view *scene, int width, double aspect, int spp, int max_depth,
                              uint8_t *rgb_out, int *height_out, unsigned long long *segments);
/* The kernel's sampling draws (unit vector, unit-ball point, unit-disk
 * point, lambertian direction about +z) on n keys: 3 floats each. */
int rto_sample_probe(int kind, uint32_t n, uint32_t seed, float *out);
/* fp32 restatement of the kernel algorithm; same arguments as rt_render. */
int rto_kernel_render(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p,
                      float *out, unsigned long long *segments, int threads);
/* The same, plus (exact != NULL) each pixel's fp64 sum of the unquantised
 * sample radiances (3 doubles per pixel, laid out like out) -- the reference's
 * own accumulation (src/cpu/main.cc:114-119) of the same samples.  opts bits
 * select superseded forms of the specification, for the tests and attribution
 * tools that show why they changed:
 *   RTO_OPT_NO_DITHER  the sum format without its stochastic rounding
 *                      (truncation at every spp: the round-2 format);
 *   RTO_OPT_TMIN_WORLD t_min = 0.001 in world units on the normalised ray (the
 *                      round-1..4 form) instead of 0.001 in units of the
 *                      unnormalised direction, as the reference tests it;
 *   RTO_OPT_NO_SEALED  without the opaque-inside rule:
 *                      paths inside a sealed lambertian ball bounce on;
 *   RTO_OPT_FP64_ROOTS each candidate's roots (and so the t_min decision)
 *                      from fp64 arithmetic on the fp32 ray and sphere
 *                      (attribution only: is the fp32 root the cause?);
 *   RTO_OPT_NO_SAME_EXIT without round 5's same-sphere exit rule (the exiting
 *                      root of the sphere a ray starts on, moving away from
 *                      its centre, taken as a hit: the round-4 form);
 *   RTO_OPT_FP64_HIT   the winning sphere's root, hit point and normal from
 *                      fp64 arithmetic on the fp32 ray and sphere, rounded
 *                      once (attribution only: is the fp32 hit point the
 *                      cause?). */
enum { RTO_OPT_NO_DITHER = 1, RTO_OPT_TMIN_WORLD = 2, RTO_OPT_NO_SEALED = 4, RTO_OPT_FP64_ROOTS = 8,
       RTO_OPT_NO_SAME_EXIT = 16, RTO_OPT_FP64_HIT = 32 };
int rto_kernel_render_exact(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p,
                            float *out, double *exact, int opts, unsigned long long *segments,
                            int threads);
/* fp64 final scene rows: kind, cx, cy, cz, r, albedo rgb, param (9 doubles). */
/* src/gpu's own per-sample arithmetic with switches (mode: GREF_* bits in
 * rt_oracle.cc), for attributing differences to the reference CUDA output;
 * GPU semantics (open interval, metal fuzz with random_unit_vector). */
int rto_gpuref_render(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p, int mode,
                      float *out, unsigned long long *segments, int threads);
/* debug: print one sample's segments and candidates to stdout */
int rto_trace(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p, int col,
              int grow, long sample);
int rto_reference_scene(int half_extent, double *rows, size_t capacity, size_t *n_out,
                        double *rng_next);
/* the kernel specification's sealed spheres (opaque-inside rule), one byte each */
int rto_sealed(const rt_scene_view *scene, uint8_t *out);
#ifdef __cplusplus
}
#endif
#endif
