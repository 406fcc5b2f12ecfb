// rt_accel.cpp -- host-side builder of the render kernel's scene records and
// acceleration structures (rt_scene_upload, rt_internal_accel_info): the scan
// records, shading records, the BVH in 8 DFS orders, layer mode and the layer
// grid, and where the grid lives during a launch.  Host
// C++ only: no HIP calls, so the builder runs under ASan / UBSan on the CPU
// (tools/host_sanitize.sh) and rebuilding it does not recompile the kernel.
#include "rt_accel.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace rtk {
namespace {

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
  std::vector<bvh_node> nodes;
  std::vector<int> slots;          // slot -> original index, -1 padding
  static constexpr int kLeaf = 2 * kLeafPairs;
  // builder options (rt_context_set_option; defaults measured best)
  int max_leaf = kLeaf;
  double collapse_area = 0.35;
  double side_weight = 1.0;  // SAH weight of the x- and z-facing sides
  double grid_scale = 1.0;   // layer-grid cell side multiplier
  double grid_phase_x = 0.0, grid_phase_z = 0.0;  // grid origin shifted by these fractions of a cell, [0, 1)

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
  void set_box(bvh_node &nd, const box &b) {
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
      tree[id].leaf = (first_slot / 2 + 1) | (width == 4 ? kTwoPairs : 0u);
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
    nodes.push_back(bvh_node{});
    if (tn.leaf) {
      bvh_node &nd = nodes[id];
      set_box(nd, tn.b);
      nd.skip = (int32_t)(id + 1 - base);
      nd.leaf = tn.leaf;
      return;
    }
    const bool neg = (oct >> tn.axis) & 1;
    emit(neg ? tn.right : tn.left, oct, base, t);
    emit(neg ? tn.left : tn.right, oct, base, t);
    bvh_node &nd = nodes[id];
    set_box(nd, tn.b);
    nd.skip = (int32_t)(nodes.size() - base);
    nd.leaf = 0;
  }
  // Layer-mode node: the emitted x and z slabs [lo, hi] as (centre, half-width),
  // bx = (cx, cz), by = (hx, hz).  The walk evaluates m = fma(c, 1/d, -o/d),
  // m -+ fma(h, |1/d|): three roundings of magnitude <= (|o| + |c - o| + h) |1/d|
  // against two for fma(lo, 1/d, -o/d), so h also covers |c - float(c)| and
  // 2^-22 (3 oref + 2|c| + h) on top of the (lo, hi) padding.
  void to_centre_form(bvh_node &nd) const {
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
  uint32_t n_layer = 0;  // layer mode: spheres in the layer (ord[0, n_layer))
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
      for (bvh_node &nd : nodes) to_centre_form(nd);
      extra_pair0 = (uint32_t)slots.size() / 2;  // leaves end on a pair boundary
      for (uint32_t i = n_tree; i < n; ++i) slots.push_back((int)ord[i]);
      // padded to whole groups of two pairs: the kernel scans them two at a
      // time (one s_load_dwordx16, two independent chains)
      while ((slots.size() - 2 * extra_pair0) % 4) slots.push_back(-1);
      n_extra_pairs = (uint32_t)slots.size() / 2 - extra_pair0;
      n_layer = n_tree;
      build_grid(s, n_tree);
    }
  }
  // Layer grid: square x-z cells of side g over the layer spheres' padded
  // boxes; a cell lists every layer sphere whose padded box comes within pad
  // of it.  g is chosen for ~1 sphere per cell (grid_scale scales it);
  // cells list at most 15 spheres (else g shrinks).
  std::vector<uint32_t> grid_cells;
  std::vector<float> grid_items;  // 4 floats per item
  float grid_x0 = 0, grid_z0 = 0, grid_xi = 0, grid_zi = 0, grid_x1 = 0, grid_z1 = 0, grid_g = 0;
  int grid_nx = 0, grid_nz = 0;
  void build_grid(const rt_scene_view *s, uint32_t n_tree) {
    grid_cells.clear();
    grid_items.clear();
    grid_nx = grid_nz = 0;
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
    double g = grid_scale * std::sqrt((x1 - x0) * (z1 - z0) / (double)n_tree);
    const double bx0 = x0, bz0 = z0;
    for (int attempt = 0; attempt < 8; ++attempt, g *= 0.8) {
      // the phase moves the cell borders relative to the spheres (the image is
      // the same for every grid)
      x0 = bx0 - grid_phase_x * g;
      z0 = bz0 - grid_phase_z * g;
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
    // the largest extra first: the grid build's extras scan runs slot 0's root
    // sequence on its own and compacts the others' (rt_kernel.hip scan_extras);
    // the ground, a candidate for almost every line, belongs there.  The
    // closest hit does not depend on the order (ties go by original index).
    std::stable_sort(out.begin(), out.end(), [&](uint32_t a, uint32_t b) {
      return std::fabs((double)s->radius[a]) > std::fabs((double)s->radius[b]);
    });
    layer_mode = true;
    layer_cy = key[best].first;
    std::copy(in.begin(), in.end(), ord.begin());
    std::copy(out.begin(), out.end(), ord.begin() + in.size());
    return (uint32_t)in.size();
  }
};

// scan record of one slot (ks = |C|^2 - r^2 in fp64, rounded once; padding
// slots have ks = +inf and are never candidates)
void fill_slot(pair_geom &g, int l, const rt_scene_view *s, int i) {
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

}  // namespace

// Sealed spheres (the opaque-inside rule).  A lambertian
// sphere of radius |r| > 2 t_min whose ball no other sphere's ball overlaps
// (touching at one point is allowed: the final scene's glass sphere rests on
// the ground, |C_a - C_b| = r_a + r_b exactly).  In the reference's arithmetic a path inside such
// a sphere never leaves: its lambertian scatter off the inner wall is n + u
// (|u| = 1, src/cpu/material.h:19-30, src/gpu/material.h:20-40), so |d| = 2
// cos(angle to n) and the chord to the far wall is 2 |r| cos / |d| = |r| in
// the ray's own units -- always past t_min -- and no other surface lies
// inside the ball.  The path then hits the same sphere again and again until
// the depth cap and returns black; the kernel ends it black at its first
// inner hit.  Metal is not sealed (a reflection keeps the entering chord,
// which may be shorter than t_min), and a ball that another ball overlaps has
// exits through that sphere (a glass sphere half-embedded in it refracts the
// path out).  fp64 on the fp32 scene; sweep over x-intervals, O(n log n + overlapping x-pairs).
void sealed_spheres(const rt_scene_view *s, std::vector<uint8_t> &out) {
  const uint32_t n = s->n;
  out.assign(n, 0);
  std::vector<uint8_t> overlapped(n, 0);
  std::vector<uint32_t> ord(n);
  for (uint32_t i = 0; i < n; ++i) ord[i] = i;
  auto lo = [&](uint32_t i) { return (double)s->cx[i] - std::fabs((double)s->radius[i]); };
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return lo(a) < lo(b) || (lo(a) == lo(b) && a < b); });
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t i = ord[k];
    const double ri = std::fabs((double)s->radius[i]), hi = (double)s->cx[i] + ri;
    for (uint32_t m = k + 1; m < n && lo(ord[m]) < hi; ++m) {
      const uint32_t j = ord[m];
      const double dx = (double)s->cx[i] - s->cx[j], dy = (double)s->cy[i] - s->cy[j],
                   dz = (double)s->cz[i] - s->cz[j];
      const double rs = ri + std::fabs((double)s->radius[j]);
      if (dx * dx + dy * dy + dz * dz < rs * rs) overlapped[i] = overlapped[j] = 1;
    }
  }
  for (uint32_t i = 0; i < n; ++i)
    out[i] = s->mat_kind[i] == RT_LAMBERTIAN && !overlapped[i] && std::fabs((double)s->radius[i]) > 0.002 ? 1 : 0;
}

// What rt_scene_upload (and rt_internal_accel_info) accept: arrays present,
// known materials, finite centres and radii, non-zero radii, and finite
// albedos >= 0 (dielectrics ignore theirs).  Albedos above 1 (energy-creating,
// as the reference's constructors allow, src/cpu/material.h:17,38) switch the
// render to 64-bit pixel sums; negative ones give the
// reference's write_color a NaN.  The builder's sorts need finite keys.
bool scene_ok(const rt_scene_view *s) {
  if (!s || (s->n && (!s->cx || !s->cy || !s->cz || !s->radius || !s->mat_kind || !s->mat_param ||
                      !s->albedo_rgb)))
    return false;
  for (uint32_t i = 0; i < s->n; ++i) {
    if (s->mat_kind[i] > RT_DIELECTRIC || !(s->radius[i] != 0.0f) || !std::isfinite(s->radius[i]) ||
        !std::isfinite(s->cx[i]) || !std::isfinite(s->cy[i]) || !std::isfinite(s->cz[i]))
      return false;
    for (int k = 0; k < 3 && s->mat_kind[i] != RT_DIELECTRIC; ++k)
      if (!(s->albedo_rgb[3 * i + k] >= 0.0f && std::isfinite(s->albedo_rgb[3 * i + k]))) return false;
  }
  return true;
}

double max_albedo(const rt_scene_view *s) {
  double a = 0.0;
  for (uint32_t i = 0; i < s->n; ++i)
    for (int k = 0; k < 3 && s->mat_kind[i] != RT_DIELECTRIC; ++k) a = std::max(a, (double)s->albedo_rgb[3 * i + k]);
  return a;
}


void build_accel(const rt_scene_view *s, const accel_options &o, accel_build &a, grid_fitter **fitter) {
  if (fitter) *fitter = nullptr;
  const uint32_t n = s->n;
  a = accel_build{};
  a.n = n;
  a.n_pad = (n + kSpherePad - 1) / kSpherePad * kSpherePad;
  a.scan_geom.assign(a.n_pad / 2, pair_geom{});
  for (uint32_t i = 0; i < a.n_pad; ++i) fill_slot(a.scan_geom[i / 2], i & 1, s, i < n ? (int)i : -1);
  a.shade.assign(n, shade_rec{});
  std::vector<uint8_t> sealed;
  sealed_spheres(s, sealed);
  for (uint32_t i = 0; i < n; ++i) {
    shade_rec &r = a.shade[i];
    std::memset(&r, 0, sizeof r);
    r.cx = s->cx[i];
    r.cy = s->cy[i];
    r.cz = s->cz[i];
    r.inv_r = 1.0f / s->radius[i];
    const bool glass = s->mat_kind[i] == RT_DIELECTRIC;
    r.ar = glass ? 1.0f : s->albedo_rgb[3 * i + 0];
    r.ag = glass ? 1.0f : s->albedo_rgb[3 * i + 1];
    r.ab = glass ? 1.0f : s->albedo_rgb[3 * i + 2];
    // metal fuzz is clamped to 1 as the reference's constructors do
    // (src/cpu/material.h:38, src/gpu/material.h:45: fuzz(f < 1 ? f : 1))
    r.param = s->mat_kind[i] == RT_METAL ? std::min(s->mat_param[i], 1.0f) : s->mat_param[i];
    r.kind = s->mat_kind[i];
    r.radius = s->radius[i];
    const double x = s->cx[i], y = s->cy[i], z = s->cz[i], rr = s->radius[i];
    r.ks = (float)(x * x + y * y + z * z - rr * rr);
    const double ior = s->mat_param[i];
    r.inv_param = (float)(1.0 / ior);
    const double r0 = (1.0 - ior) / (1.0 + ior);
    r.r0 = (float)(r0 * r0);
    r.sealed = sealed[i];
  }
  bvh_builder bb;
  bb.max_leaf = std::max(1, std::min(bvh_builder::kLeaf, o.bvh_leaf));
  bb.collapse_area = o.collapse;
  bb.side_weight = o.side;
  bb.grid_scale = o.grid_scale;
  bb.grid_phase_x = o.grid_phase_x;
  bb.grid_phase_z = o.grid_phase_z;
  bb.run(s);
  // Grid placement.  The whole grid in LDS when it fits the
  // per-block budget (u16 LDS addresses: < 4096 items); else, for auto or
  // kGridCells, only the u16 cell starts in LDS -- the cells rebuilt coarser
  // until they fit (at most 1.6x the requested side), item indices < 2^16;
  // else global memory.
  int place = kGridGlobal;
  const size_t lds_max = o.wide ? kGridLdsMaxWide : kGridLdsMax;
  const auto n_items = [&] { return (long long)(bb.grid_items.size() / 4); };
  const auto n_cells = [&] { return (long long)bb.grid_cells.size(); };
  if (!bb.grid_cells.empty()) {
    const bool lds_fits = n_items() < 4096 && grid_lds_bytes(kGridLds, n_items(), n_cells()) <= lds_max;
    if ((o.grid_placement < 0 || o.grid_placement == kGridLds) && lds_fits) {
      place = kGridLds;
    } else if (o.grid_placement < 0 || o.grid_placement == kGridCells) {
      const double scale0 = bb.grid_scale;
      for (int k = 0; k < 8 && !bb.grid_cells.empty(); ++k) {
        const size_t need = grid_lds_bytes(kGridCells, n_items(), n_cells());
        if (need <= lds_max && n_items() < 65536) {
          place = kGridCells;
          break;
        }
        const double grow = std::max(1.02, 1.01 * std::sqrt((double)need / (double)lds_max));
        if (bb.grid_scale * grow > 1.6 * scale0) break;
        bb.grid_scale *= grow;
        bb.build_grid(s, bb.n_layer);
      }
      if (place != kGridCells && bb.grid_scale != scale0) {  // back to the requested cells
        bb.grid_scale = scale0;
        bb.build_grid(s, bb.n_layer);
      }
    }
  }
  a.bvh_geom.assign(bb.slots.size() / 2, pair_geom{});
  for (size_t k = 0; k < bb.slots.size(); ++k) fill_slot(a.bvh_geom[k / 2], (int)(k & 1), s, bb.slots[k]);
  a.slots = bb.slots;
  a.nodes = bb.nodes;
  a.per_order = bb.per_order;
  a.oref = bb.oref;
  a.layer_mode = bb.layer_mode;
  a.layer_lo = bb.layer_lo;
  a.layer_hi = bb.layer_hi;
  a.layer_cy = bb.layer_cy;
  a.extra_pair0 = bb.extra_pair0;
  a.n_extra_pairs = bb.n_extra_pairs;
  a.grid_cells = bb.grid_cells;
  a.grid_items = bb.grid_items;
  a.grid_x0 = bb.grid_x0;
  a.grid_z0 = bb.grid_z0;
  a.grid_xi = bb.grid_xi;
  a.grid_zi = bb.grid_zi;
  a.grid_x1 = bb.grid_x1;
  a.grid_z1 = bb.grid_z1;
  a.grid_g = bb.grid_g;
  a.grid_nx = bb.grid_nx;
  a.grid_nz = bb.grid_nz;
  a.grid_scale = bb.grid_scale;
  a.grid_placement = bb.grid_cells.empty() ? kGridGlobal : place;
  // the builder's layer split and boxes go on into the grid fitter
  if (fitter && !bb.grid_cells.empty())
    *fitter = grid_fitter::make_from(s, o, a.grid_placement, bb.grid_scale, &bb);
}

// ---------------------------------------------------------- grid fitter --
struct grid_fitter::impl {
  // the scene's arrays (the view the builder reads points into them)
  std::vector<float> cx, cy, cz, radius, albedo, param;
  std::vector<uint32_t> kind;
  rt_scene_view view{};
  mutable bvh_builder bb;  // after run(): boxes, layer order; build_grid rebuilds the grid
  int placement = kGridGlobal;
  size_t lds_max = 0;
  double s0 = 1.0;
  // the grid at scale s into bb's grid fields; false if it does not fit the placement
  bool grid_at(double scale) const {
    bb.grid_scale = scale;
    bb.build_grid(&view, bb.n_layer);
    if (bb.grid_cells.empty()) return false;
    const long long items = (long long)(bb.grid_items.size() / 4), cells = (long long)bb.grid_cells.size();
    if (placement == kGridLds)
      return items < 4096 && grid_lds_bytes(kGridLds, items, cells) <= lds_max;
    return items < 65536 && grid_lds_bytes(kGridCells, items, cells) <= lds_max;
  }
};

grid_fitter *grid_fitter::make(const rt_scene_view *s, const accel_options &o, int placement, double scale0) {
  return make_from(s, o, placement, scale0, nullptr);
}

// builder: a bvh_builder that has run on s (build_accel's, moved here), or null
grid_fitter *grid_fitter::make_from(const rt_scene_view *s, const accel_options &o, int placement, double scale0,
                                    void *builder) {
  if (placement != kGridLds && placement != kGridCells) return nullptr;
  grid_fitter *f = new grid_fitter();
  impl *q = f->p_ = new impl();
  const uint32_t n = s->n;
  q->cx.assign(s->cx, s->cx + n);
  q->cy.assign(s->cy, s->cy + n);
  q->cz.assign(s->cz, s->cz + n);
  q->radius.assign(s->radius, s->radius + n);
  q->kind.assign(s->mat_kind, s->mat_kind + n);
  q->albedo.assign(s->albedo_rgb, s->albedo_rgb + 3 * (size_t)n);
  q->param.assign(s->mat_param, s->mat_param + n);
  q->view = *s;
  q->view.cx = q->cx.data();
  q->view.cy = q->cy.data();
  q->view.cz = q->cz.data();
  q->view.radius = q->radius.data();
  q->view.mat_kind = q->kind.data();
  q->view.albedo_rgb = q->albedo.data();
  q->view.mat_param = q->param.data();
  if (builder) {
    q->bb = std::move(*static_cast<bvh_builder *>(builder));
  } else {
    q->bb.max_leaf = std::max(1, std::min(bvh_builder::kLeaf, o.bvh_leaf));
    q->bb.collapse_area = o.collapse;
    q->bb.side_weight = o.side;
    q->bb.grid_scale = scale0;
    q->bb.grid_phase_x = o.grid_phase_x;
    q->bb.grid_phase_z = o.grid_phase_z;
    q->bb.run(&q->view);
  }
  q->placement = placement;
  q->lds_max = o.wide ? kGridLdsMaxWide : kGridLdsMax;
  q->s0 = scale0;
  if (!q->bb.layer_mode || !q->grid_at(scale0)) {
    delete f;
    return nullptr;
  }
  return f;
}

grid_fitter::~grid_fitter() { delete p_; }
double grid_fitter::scale0() const { return p_->s0; }

double grid_fitter::choose(const rt_camera &cam, int width, int height,
                           std::vector<std::pair<double, double>> *costs) const {
  const impl &q = *p_;
  if (costs) costs->clear();
  double best = q.s0, best_cost = INFINITY;
  for (int k = 0; k <= kFitSteps; ++k) {
    const double scale = q.s0 * (1.0 + 0.01 * k);
    if (!q.grid_at(scale)) continue;
    const bvh_builder &b = q.bb;
    const int nx = b.grid_nx, nz = b.grid_nz;
    const double g = b.grid_g;
    // where 64 x 64 camera directions over the frame meet the layer plane
    std::vector<double> w((size_t)nx * nz, 0.0);
    constexpr int kS = 64;
    for (int j = 0; j < kS; ++j)
      for (int i = 0; i < kS; ++i) {
        double fs = (i + 0.5) / kS, ft = (j + 0.5) / kS;
        if (cam.model == RT_CAMERA_GPU) {
          fs = fs * width - 0.5;
          ft = ft * height - 0.5;
        }
        double d[3];
        for (int a = 0; a < 3; ++a) d[a] = cam.corner[a] + fs * cam.horiz[a] + ft * cam.vert[a] - cam.eye[a];
        if (!(d[1] != 0.0)) continue;
        const double t = (b.layer_cy - cam.eye[1]) / d[1];
        if (!(t > 0.0)) continue;
        const double x = (cam.eye[0] + t * d[0] - b.grid_x0) / g, z = (cam.eye[2] + t * d[2] - b.grid_z0) / g;
        if (!(x >= 0.0 && x < nx && z >= 0.0 && z < nz)) continue;
        w[(size_t)z * nx + (size_t)x] += 1.0;
      }
    // 3 x 3 box-smoothed weight of each cell times its item count
    double sw = 0.0, swi = 0.0;
    for (int z = 0; z < nz; ++z)
      for (int x = 0; x < nx; ++x) {
        double v = 0.0;
        for (int dz = -1; dz <= 1; ++dz)
          for (int dx = -1; dx <= 1; ++dx) {
            const int zz = z + dz, xx = x + dx;
            if (zz >= 0 && zz < nz && xx >= 0 && xx < nx) v += w[(size_t)zz * nx + xx];
          }
        sw += v;
        swi += v * (double)(b.grid_cells[(size_t)z * nx + x] & 15u);
      }
    if (!(sw > 0.0)) return q.s0;  // the camera does not see the layer: the builder's grid
    const double cost = (swi / sw + kFitCellCost) / g;
    if (costs) costs->push_back({scale, cost});
    if (cost < best_cost) {
      best_cost = cost;
      best = scale;
    }
  }
  return best;
}

bool grid_fitter::build(double scale, grid_geom &out) const {
  const impl &q = *p_;
  if (!q.grid_at(scale)) return false;
  const bvh_builder &b = q.bb;
  out.cells = b.grid_cells;
  out.items = b.grid_items;
  out.x0 = b.grid_x0;
  out.z0 = b.grid_z0;
  out.xi = b.grid_xi;
  out.zi = b.grid_zi;
  out.x1 = b.grid_x1;
  out.z1 = b.grid_z1;
  out.g = b.grid_g;
  out.nx = b.grid_nx;
  out.nz = b.grid_nz;
  out.scale = b.grid_scale;
  return true;
}

}  // namespace rtk
