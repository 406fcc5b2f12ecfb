// rt_accel.h -- internal to librtow: the host-side builder of the render
// kernel's scene records and acceleration structures (rt_accel.cpp), used by
// rt_scene_upload and rt_internal_accel_info (rt_api.cpp).
#ifndef RTOW_RT_ACCEL_H
#define RTOW_RT_ACCEL_H

#include <cstdint>
#include <vector>

#include "rt_internal.h"
#include "rt_layout.h"

namespace rtk {

// builder options (rt_context_set_option; scheduling and placement only:
// every value renders the same image)
struct accel_options {
  int bvh_leaf = 4;          // RT_OPT_BVH_LEAF: spheres per BVH leaf, 1..4
  double collapse = 0.35;    // RT_OPT_BVH_COLLAPSE
  double side = 1.0;         // RT_OPT_BVH_SIDE
  double grid_scale = 1.0;   // RT_OPT_GRID_SCALE
  double grid_phase_x = 0.0, grid_phase_z = 0.0;  // RT_OPT_INTERNAL_GRID_PHASE_X / _Z
  int grid_placement = -1;   // RT_OPT_GRID_PLACEMENT: -1 auto, else kGridGlobal / kGridLds / kGridCells
  bool wide = false;         // 64-bit pixel sums (an albedo above 1): less LDS for the grid
};

// everything rt_scene_upload copies to the device, plus the builder's facts
struct accel_build {
  uint32_t n = 0, n_pad = 0;
  std::vector<pair_geom> scan_geom;  // brute-force order, n_pad / 2 pairs
  std::vector<shade_rec> shade;      // n
  std::vector<pair_geom> bvh_geom;   // BVH leaf order (+ extras in layer mode)
  std::vector<int> slots;            // BVH slot -> original index, -1 padding
  std::vector<bvh_node> nodes;       // 8 DFS orders
  size_t per_order = 0;
  double oref = 64.0;
  bool layer_mode = false;
  float layer_lo = 0.0f, layer_hi = 0.0f, layer_cy = 0.0f;
  uint32_t extra_pair0 = 0, n_extra_pairs = 0;
  // layer grid (empty: none)
  std::vector<uint32_t> grid_cells;
  std::vector<float> grid_items;  // 4 floats per item
  float grid_x0 = 0, grid_z0 = 0, grid_xi = 0, grid_zi = 0, grid_x1 = 0, grid_z1 = 0, grid_g = 0;
  int grid_nx = 0, grid_nz = 0;
  double grid_scale = 1.0;        // the cell scale the grid was built with
  int grid_placement = kGridGlobal;
};

// Layer-grid cell size per frame geometry (rt_api.cpp).  The
// walk's cost is not smooth in the cell size: what counts is where the cell
// borders fall relative to the spheres the frame's rays meet most (C4's rank
// share: 246-258 ms between scales 0.01 apart).  The fitter keeps a copy of a
// scene's layer spheres and, for a camera, models each candidate scale
// s0 (1 + 0.01 k), k = 0..kFitSteps, that fits the placement: the items per
// cell averaged over where 64 x 64 camera directions meet the layer plane
// (smoothed over 3 x 3 cells: bounces stay near), plus kFitCellCost for the
// cell step, per cell side, i.e. per unit of ray length.  It keeps the
// cheapest.  Fitted on round-4 sweeps: picks within 0.4 % of the best fixed
// scale on C4's share and the best on the headline frame (tools/grid_fit.py).
constexpr int kFitSteps = 30;
constexpr double kFitCellCost = 0.5;
struct grid_geom {
  std::vector<uint32_t> cells;
  std::vector<float> items;  // 4 floats per item
  float x0 = 0, z0 = 0, xi = 0, zi = 0, x1 = 0, z1 = 0, g = 0;
  int nx = 0, nz = 0;
  double scale = 1.0;
};
class grid_fitter {
 public:
  // nullptr unless the scene walks a layer grid in an LDS placement
  static grid_fitter *make(const rt_scene_view *s, const accel_options &o, int placement, double scale0);
  ~grid_fitter();
  // the modelled cheapest candidate scale for this camera and frame (scale0
  // when the camera does not see the layer); costs (may be null) receives
  // (scale, modelled cost) per candidate that fits
  double choose(const rt_camera &cam, int width, int height, std::vector<std::pair<double, double>> *costs) const;
  // the grid at that scale (false: it does not fit the placement)
  bool build(double scale, grid_geom &out) const;
  double scale0() const;
  // the same from build_accel's builder (moved in; internal)
  static grid_fitter *make_from(const rt_scene_view *s, const accel_options &o, int placement, double scale0,
                                void *builder);

 private:
  struct impl;
  impl *p_ = nullptr;
};

// arrays present, known materials, finite centres and radii, non-zero radii,
// finite albedos >= 0 (rt_scene_upload's contract, include/rt.h)
bool scene_ok(const rt_scene_view *s);
// the largest lambertian / metal albedo channel (0 if none): above 1 the
// render needs 64-bit pixel sums (rt_api.cpp sum_format)
double max_albedo(const rt_scene_view *s);
// per sphere: 1 if the opaque-inside rule applies to it (sealed lambertian ball)
void sealed_spheres(const rt_scene_view *s, std::vector<uint8_t> &out);
// fitter (may be null): a grid fitter for the scene's layer grid, when it sits
// in an LDS placement (else null); the caller owns it
void build_accel(const rt_scene_view *s, const accel_options &o, accel_build &out, grid_fitter **fitter = nullptr);

}  // namespace rtk

#endif  // RTOW_RT_ACCEL_H
