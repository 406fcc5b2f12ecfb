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
SRC = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "csrc", "rt_render.hip")

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
        hit_state h2{__builtin_huge_valf(), -1, 1};
        ray_pre r2 = rp;
        asm volatile("" : "+v"(r2.dx), "+v"(r2.nk1));
        for (int k = 0; k < p.n_extra_pairs; k += 2)
          scan_pairs<OPEN, 2, STATS>(geom + p.extra_pair0 + k, 2 * (p.extra_pair0 + k), orig, r2, h2, wc.roots);
        asm volatile("" :: "v"(h2.tmax), "v"(h2.best));
      }""")],
    # the correctly rounded sqrt of each candidate sphere
    "rootsqrt": [("    const float sq = sqrt_k(disc);\n    const float t0 = h - sq, t1 = h + sq;",
                  """    const float sq = sqrt_k(disc);
    float dd = disc;
    asm volatile("" : "+v"(dd));
    const float sq2 = sqrt_k(dd);
    asm volatile("" :: "v"(sq2));
    const float t0 = h - sq, t1 = h + sq;""")],
    # the bounce's pcg4d
    "pcg": [("      const uint4 r = pcg4d(pix, miss ? sample : sample - 1u, miss ? 0u : (uint32_t)(depth + 1), q.seed32);",
             """      const uint4 r = pcg4d(pix, miss ? sample : sample - 1u, miss ? 0u : (uint32_t)(depth + 1), q.seed32);
      uint32_t pq = pix;
      asm volatile("" : "+v"(pq));
      const uint4 r2 = pcg4d(pq, miss ? sample : sample - 1u, miss ? 0u : (uint32_t)(depth + 1), q.seed32);
        asm volatile("" :: "v"(r2.x), "v"(r2.y), "v"(r2.z));""")],
    # sin/cos of the bounce's unit vector
    "sincos": [("  sincos_turn(u2, s, c);\n  x = r * c;",
                """  sincos_turn(u2, s, c);
  float uu = u2, s2, c2;
  asm volatile("" : "+v"(uu));
  sincos_turn(uu, s2, c2);
  asm volatile("" :: "v"(s2), "v"(c2));
  x = r * c;""")],
    # the winner's root refinement
    "refine": [("        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2);",
                """        const float t = refine_root(sr, tmax, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2);
        float tq = tmax;
        asm volatile("" : "+v"(tq));
        const float t2 = refine_root(sr, tq, near, ox, oy, oz, dx, dy, dz, o2, ox2, oy2, oz2);
        asm volatile("" :: "v"(t2));""")],
    # the camera ray of the next sample (path regeneration)
    "camera": [("          camera_ray(k, rc, col, grow, ox, oy, oz, dx, dy, dz);",
                """          camera_ray(k, rc, col, grow, ox, oy, oz, dx, dy, dz);
          {
            uint4 r2 = rc;
            asm volatile("" : "+v"(r2.x), "+v"(r2.y), "+v"(r2.z), "+v"(r2.w));
            float a0, a1, a2, a3, a4, a5;
            camera_ray(k, r2, col, grow, a0, a1, a2, a3, a4, a5);
            asm volatile("" :: "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5));
          }""")],
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
        p = os.path.join(d, "rt_render.hip")
        open(p, "w").write(s)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "csrc"), "-shared",
                        "-o", os.path.join(out, f"dup_{part}.so"), p,
                        os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "csrc", "rt_host.cpp")],
                       check=True)
        print("built", f"dup_{part}.so")


if __name__ == "__main__":
    main()
