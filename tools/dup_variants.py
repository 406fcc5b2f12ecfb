#!/usr/bin/env python3
"""Experiment: marginal cost of one kernel component, measured by doing it TWICE.

Builds build/variants/dup_<part>.so: the render kernel with one component
computed a second time on asm-laundered inputs (the compiler cannot merge the
copies) and its result consumed by an empty asm, so the image stays bit-identical
(checked by tools/ab_flags.py's sha256) while the kernel time grows by what that
component costs in place -- issue slots AND the latency it exposes.

    python tools/dup_variants.py [part ...]     (default: all)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "csrc", "rt_kernel.hip")

EDITS = {
    # the ray-box slab test of every BVH node visit
    "box": [("        node = walk_step<OPEN, STATS, true>(nd, node, tn <= tf, geom, orig, rl, hs, wc, tyl_f, tyl_fc);",
             """        f2 vi2 = vi, va2 = va;
        asm volatile("" : "+v"(vi2), "+v"(va2));
        const f2 m2 = fma2(nd.bx, vi2, vo);
        const f2 tn22 = fma2(-nd.by, va2, m2), tf22 = fma2(nd.by, va2, m2);
        const float n2 = fmaxf(fmaxf(tn22.x, tn22.y), tyl_n);
        const float f2_ = fminf(fminf(tf22.x, tf22.y), tyl_fc);
        asm volatile("" :: "v"(n2), "v"(f2_));
        node = walk_step<OPEN, STATS, true>(nd, node, tn <= tf, geom, orig, rl, hs, wc, tyl_f, tyl_fc);""")],
    # the scan of the spheres off the layer (layer mode)
    "extras": [("      if (STATS) wc.tests += 2 * p.n_extra_pairs;",
                """      if (STATS) wc.tests += 2 * p.n_extra_pairs;
      {
        hit_state h2 = no_hit();
        ray_pre r2 = rp;
        asm volatile("" : "+v"(r2.dx), "+v"(r2.nk1));
        for (int k = 0; k < p.n_extra_pairs; k += 2)
          scan_pairs<OPEN, 2, STATS>(geom + p.extra_pair0 + k, 2 * (p.extra_pair0 + k), orig, r2, h2, wc.roots);
        asm volatile("" :: "v"(h2.tmax), "v"(h2.lo));
      }""")],
    # the bounce's / camera ray's pcg4d (one per lane and step)
    "pcg": [("      const uint4 r = pcg4d(pix, sample, miss ? 0u : (uint32_t)(depth + 1), q.seed32);",
             """      const uint4 r = pcg4d(pix, sample, miss ? 0u : (uint32_t)(depth + 1), q.seed32);
      {
        uint32_t pq = pix;
        asm volatile("" : "+v"(pq));
        const uint4 r2 = pcg4d(pq, sample, miss ? 0u : (uint32_t)(depth + 1), q.seed32);
        asm volatile("" :: "v"(r2.x), "v"(r2.y), "v"(r2.z), "v"(r2.w));
      }""")],
    # the per-step polar draw (sqrt + sin/cos)
    "sincos": [("  sincos_turn(u, s, c);\n  x = rho * c;",
                """  sincos_turn(u, s, c);
  float uu = u, s2, c2;
  asm volatile("" : "+v"(uu));
  sincos_turn(uu, s2, c2);
  asm volatile("" :: "v"(s2), "v"(c2));
  x = rho * c;""")],
    # the winner's root refinement
    "refine": [("        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b);",
                """        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b);
        float tq = tmax, b2;
        asm volatile("" : "+v"(tq));
        const float t2 = refine_root(sr, tq, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2, b2);
        asm volatile("" :: "v"(t2), "v"(b2));""")],
    # the whole layer-grid walk (DDA + cell items + candidates), a second time
    "gridwalk": [("        if (tyl_n <= tyl_fc) grid_walk<OPEN, STATS, GLDS>(ox, oz, ix, iz, oix, oiz, tyl_n, tyl_fc, rg, hs, wc);",
                  """        if (tyl_n <= tyl_fc) {
          hit_state h2 = hs;
          float ta2 = tyl_n;
          asm volatile("" : "+v"(ta2), "+v"(h2.tmax));
          grid_walk<OPEN, STATS, GLDS>(ox, oz, ix, iz, oix, oiz, ta2, tyl_fc, rg, h2, wc);
          asm volatile("" :: "v"(h2.tmax), "v"(h2.lo));
        }
        if (tyl_n <= tyl_fc) grid_walk<OPEN, STATS, GLDS>(ox, oz, ix, iz, oix, oiz, tyl_n, tyl_fc, rg, hs, wc);""")],
    # the grid walk's item loads (16 B per lane from LDS)
    "itemload": [("      const f4 it = GLDS ? *ip : items[first + k];",
                  """      const f4 it = GLDS ? *ip : items[first + k];
      {
        lds_f4 *ip2 = ip;
        asm volatile("" : "+v"(ip2));
        const f4 it2 = *ip2;
        asm volatile("" :: "v"(it2.x), "v"(it2.y), "v"(it2.z), "v"(it2.w));
      }""")],
    # the grid walk's item test (load + 5 fma + compare), without the candidate
    "itemtest": [("      const f4 it = GLDS ? *ip : items[first + k];",
                  """      const f4 it = GLDS ? *ip : items[first + k];
      {
        lds_f4 *ip2 = ip;
        asm volatile("" : "+v"(ip2));
        const f4 i2 = *ip2;
        const float h2 = fmaf(i2.y, dz, fmaf(i2.x, dx, rl.nk1.x));
        const float g2 = fmaf(i2.y, rl.oz2.x, fmaf(i2.x, rl.ox2.x, rl.o2.x));
        const float e2 = fmaf(h2, h2, -g2);
        const uint64_t m2 = __builtin_amdgcn_ballot_w64(e2 >= i2.z);
        asm volatile("" :: "s"(m2));
      }""")],
    # the grid walk's cell loads (two ds_read_u16 per cell)
    "cellload": [("    if (GLDS) asm volatile(\"\" : \"+v\"(ie));",
                  """    if (GLDS) asm volatile("" : "+v"(ie));
    if (GLDS) {
      int c2 = cell;
      asm volatile("" : "+v"(c2));
      const uint32_t a2 = ((lds_u16 *)(uintptr_t)c2)[0], b2 = ((lds_u16 *)(uintptr_t)c2)[1];
      asm volatile("" :: "v"(a2), "v"(b2));
    }""")],
    # every candidate's root / interval sequence (sqrt, roots, tie rule)
    "candidate": [("__device__ __forceinline__ void candidate(bool c, float h, float disc, uint32_t tie2, hit_state &hs) {\n  if (c) {",
                   """__device__ __forceinline__ void candidate(bool c, float h, float disc, uint32_t tie2, hit_state &hs) {\n  if (c) {
    {
      float h2 = h, d2 = disc;
      asm volatile("" : "+v"(h2), "+v"(d2));
      const float sq2 = sqrt_k(d2);
      const float a0 = h2 - sq2, a1 = h2 + sq2;
      const bool u0 = OPEN ? (a0 > 0.001f) : (a0 >= 0.001f);
      const float rt = u0 ? a0 : a1;
      const bool ab = OPEN ? (a1 > 0.001f) : (a1 >= 0.001f);
      const uint32_t lo2 = tie2 + (u0 ? 1u : 0u);
      const uint64_t k2 = ((uint64_t)__float_as_uint(rt) << 32) | lo2;
      const uint64_t c2 = ((uint64_t)__float_as_uint(hs.tmax) << 32) | hs.lo;
      float o = (ab & (k2 < c2)) ? rt : 0.0f;
      asm volatile("" :: "v"(o));
    }""")],
    # the camera direction of a new item (path regeneration)
    "camera": [("        camera_dir(q, r, ux, uy, col, grow, ox, oy, oz, dx, dy, dz);",
                """        camera_dir(q, r, ux, uy, col, grow, ox, oy, oz, dx, dy, dz);
        {
          uint4 r2 = r;
          asm volatile("" : "+v"(r2.x), "+v"(r2.y), "+v"(r2.z), "+v"(r2.w));
          float a0, a1, a2, a3, a4, a5;
          camera_dir(q, r2, ux, uy, col, grow, a0, a1, a2, a3, a4, a5);
          asm volatile("" :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5));
        }""")],
    # the per-step normalisation of the new direction
    "normalize": [("    if (alive) normalize3(dx, dy, dz);",
                   """    if (alive) {
      float x2 = dx, y2 = dy, z2 = dz;
      asm volatile("" : "+v"(x2), "+v"(y2), "+v"(z2));
      normalize3(x2, y2, z2);
      asm volatile("" :: "v"(x2), "v"(y2), "v"(z2));
    }
    if (alive) normalize3(dx, dy, dz);""")],
    # the material scatter (all three branches as the wave runs them)
}


def main():
    parts = sys.argv[1:] or list(EDITS)
    src = open(SRC).read()
    out = os.path.join(ROOT, "build", "variants")
    os.makedirs(out, exist_ok=True)
    for part in parts:
        s = src
        for old, new in EDITS[part]:
            assert s.count(old) == 1, (part, old[:60])
            s = s.replace(old, new)
        d = os.path.join(out, "src_dup_" + part)
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, "rt_kernel.hip")
        open(p, "w").write(s)
        subprocess.run([os.path.join(ROOT, "tools", "build_variant.sh"), "dup_" + part, p], check=True)
        print("built", f"dup_{part}.so")


if __name__ == "__main__":
    main()
