#!/usr/bin/env python3
"""Check RT_OPT_GRID_FIT's pick against a sweep of fixed cell scales (GPU box).

For one frame geometry (a bench preset, optionally one rank's share), renders
  * the default path (the fitter picks the cell scale for this camera), and
  * every candidate scale s0 (1 + 0.01 k), k = 0..30, fixed (RT_OPT_GRID_SCALE),
each `--reps` times (median kernel time), and prints one JSON line per scale
and a summary: the fitted scale, its time, the best fixed scale and time, and
the pick's excess over the best (within 0.5 %).

    python tools/grid_fit_check.py --preset c2
    python tools/grid_fit_check.py --preset c4 --world 8 --rank 0 --spp 200
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def main():
    import bench
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="c2")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=31, help="candidates k = 0 .. steps-1")
    a = ap.parse_args()
    w, h, spp, half = bench.PRESETS[a.preset]
    spp = a.spp or spp
    scene = rtow.final_scene(half_extent=half)
    cam = rtow.camera_cpu(aspect=w / h)
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_PILOT_SCHEDULE
    p = rtow.make_params(w, h, spp, seed=0, flags=flags, rank=a.rank, world=a.world)
    fit, _ = rtow.grid_fit(scene, cam, w, h)
    s0 = rtow.accel_info(scene)["grid_scale_milli"] / 1000.0

    def timed(ctx):
        ms = []
        for _ in range(a.reps + 1):  # the first render pays the pilot
            _, st = ctx.render(cam, p)
            ms.append(st.kernel_ms)
        return statistics.median(ms[1:]), st.segments

    out = []
    ctx = rtow.Context(0)
    ctx.upload(scene)
    t, segs = timed(ctx)
    picked = ctx.grid_scale()
    print(json.dumps({"preset": a.preset, "rank": a.rank, "world": a.world, "spp": spp, "mode": "fit",
                      "scale": round(picked, 4), "host_pick": round(fit, 4), "kernel_ms": round(t, 2),
                      "segments": segs}), flush=True)
    ctx.close()
    for k in range(a.steps):
        sc = s0 * (1.0 + 0.01 * k)
        ctx = rtow.Context(0)
        ctx.upload(scene, grid_scale=sc)
        tk, sk = timed(ctx)
        assert sk == segs
        ctx.close()
        out.append((sc, tk))
        print(json.dumps({"preset": a.preset, "rank": a.rank, "mode": "fixed", "scale": round(sc, 4),
                          "kernel_ms": round(tk, 2)}), flush=True)
    best = min(out, key=lambda x: x[1])
    print(json.dumps({"preset": a.preset, "rank": a.rank, "world": a.world, "summary": True,
                      "fit_scale": round(picked, 4), "fit_ms": round(t, 2),
                      "best_fixed_scale": round(best[0], 4), "best_fixed_ms": round(best[1], 2),
                      "builder_ms": round(out[0][1], 2),
                      "fit_excess_over_best": round(t / best[1] - 1, 4)}), flush=True)


if __name__ == "__main__":
    main()
