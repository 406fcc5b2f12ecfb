/*
 * rt_internal.h -- librtow.so's diagnostic and tuning entry points.
 *
 * NOT part of the drop-in boundary (include/rt.h): nothing here
 * replaces reference code.  These functions exist for the test suite
 * (tests/), the measurement tools (tools/) and host sanitizer runs: the
 * device arithmetic's known-answer vectors, and host-only views of what the
 * BVH / layer-grid builder, the launch planner and the grid fitter decide.
 * A caller of the reference's render path needs rt.h only.
 */
#ifndef RTOW_RT_INTERNAL_H
#define RTOW_RT_INTERNAL_H

#include "rt.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tuning options for rt_context_set_option beyond rt_option (tools only):
 * the layer grid's origin shifted by this fraction of a cell in x / z,
 * [0, 1) (default 0: the grid starts at the layer's padded bounds).  Read by
 * the next rt_scene_upload; applies to the fitter's candidates too.
 * Scheduling only: every grid renders the same image.  Measured in round 5
 * and not adopted by the fitter. */
enum { RT_OPT_INTERNAL_GRID_PHASE_X = 8, RT_OPT_INTERNAL_GRID_PHASE_Z = 9 };

/* Known-answer evaluation of the render kernel's own device arithmetic on
 * `device` (synchronous).  10 doubles in, 9 out per case (layouts in
 * rt_kernel.hip, kat_kernel):
 *   RT_KAT_SPHERE_HIT   sphere::hit            src/cpu/sphere.h:24-51
 *   RT_KAT_REFLECT      reflect                src/cpu/vec3.h:122-124
 *   RT_KAT_REFRACT      refract                src/cpu/vec3.h:126-131
 *   RT_KAT_REFLECTANCE  dielectric::reflectance src/cpu/material.h:82-87 */
enum { RT_KAT_SPHERE_HIT = 0, RT_KAT_REFLECT = 1, RT_KAT_REFRACT = 2, RT_KAT_REFLECTANCE = 3 };
int rt_device_kat(int device, int kind, const double *in, size_t n_cases, double *out);

/* Host only (no device): what rt_scene_upload would build for `scene` with
 * the given RT_OPT_GRID_PLACEMENT / RT_OPT_GRID_SCALE values (0 = default) --
 * BVH size, layer split, layer-grid dimensions, LDS footprint and the grid's
 * invariants (cell i's items are [first_i, first_{i+1}); ring cells empty).
 * Writes min(n_out, RT_ACCEL_INFO_N) values:
 *   0 nodes per DFS order   1 BVH slots          2 layer mode     3 extra_pair0
 *   4 n_extra_pairs         5 grid_nx (w/ ring)  6 grid_nz        7 grid items
 *   8 grid LDS bytes        9 whole grid in LDS 10 max items/cell 11 start invariant
 *  12 empty ring cells ok  13 oref * 1000      14 layer slots    15 listed cells
 *  16 placement (RT_GRID_*, 0: no grid)         17 cell scale * 1000
 * For tests and sanitizer runs. */
#define RT_ACCEL_INFO_N 18
int rt_internal_accel_info(const rt_scene_view *scene, int grid_placement, double grid_scale, uint64_t *out,
                           size_t n_out);

/* Host only (no device): how rt_render would cut a render with these
 * parameters into launches under a launch-sample budget (0 = the default,
 * 2^35; see RT_OPT_LAUNCH_SAMPLES).  Writes min(n_out, RT_LAUNCH_PLAN_N)
 * values: 0 block ranges, 1 sample ranges per block range, 2 units (waves per
 * tile), 3 work entries (blocks x units), 4 launches (ranges x sample ranges).
 * For tests. */
#define RT_LAUNCH_PLAN_N 5
int rt_internal_launch_plan(const rt_params *params, double launch_samples, uint64_t *out, size_t n_out);

/* Host only (no device): the layer-grid cell scale RT_OPT_GRID_FIT would
 * pick for `scene` (default builder options, the automatic placement) seen by
 * `cam` in a width x height frame; *scale = 0 without a grid in an LDS
 * placement.  With costs != NULL, the modelled cost of each candidate that
 * fits: (scale, cost) pairs, min(n_costs, *n) of them (*n = their count).
 * For tests and tools. */
int rt_internal_grid_fit(const rt_scene_view *scene, const rt_camera *cam, int width, int height, double *scale,
                         double *costs, size_t n_costs, size_t *n);
/* The same with the grid's origin shifted by (phase_x, phase_z) cells, each
 * in [0, 1) (RT_OPT_INTERNAL_GRID_PHASE_X / _Z).  For tools. */
int rt_internal_grid_fit_phase(const rt_scene_view *scene, const rt_camera *cam, int width, int height,
                               double phase_x, double phase_z, double *scale, double *costs, size_t n_costs,
                               size_t *n);
/* The cell scale of the context's current layer grid (after RT_OPT_GRID_FIT
 * refits it for a render's frame geometry); 0 without a grid.  For tests and
 * the bench record. */
int rt_internal_grid_scale(rt_context *ctx, double *scale);

/* Host only (no device): for each sphere of `scene`, 1 if the kernel's
 * opaque-inside rule applies to it (a sealed lambertian sphere: no other
 * ball overlaps its ball), else 0.  Writes
 * min(n_out, scene->n) bytes.  For tests. */
int rt_internal_sealed(const rt_scene_view *scene, uint8_t *out, size_t n_out);

#ifdef __cplusplus
}
#endif
#endif /* RTOW_RT_INTERNAL_H */
