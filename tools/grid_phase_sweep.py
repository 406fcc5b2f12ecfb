#!/usr/bin/env python3
"""The layer grid's origin phase (RT_OPT_INTERNAL_GRID_PHASE_X / _Z) against the walk's
time (GPU box).  For one frame geometry (a bench preset, optionally one rank's
share) and one cell scale (default: the fitter's pick), renders the grid with
its origin shifted by (i / P, j / P) cells, i, j = 0..P-1, each `--reps` times
(median kernel time), next to the host model's cost of that grid
(rt_internal_grid_fit_phase), and prints one JSON line per phase plus a
summary (spread, the model's correlation with the times).  Every grid renders
the same image: the segment counts are asserted equal.

    python tools/grid_phase_sweep.py --preset c2 --phases 4
    python tools/grid_phase_sweep.py --preset c4 --world 8 --rank 0 --spp 200
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def main():
    import numpy as np
    import bench
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="c2")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--phases", type=int, default=4, help="P: phases i / P per axis")
    ap.add_argument("--scale", type=float, default=0.0, help="cell scale (0: the fitter's pick)")
    ap.add_argument("--extra", default="", help="more 'scale:px:pz' grids to time, comma-separated")
    a = ap.parse_args()
    w, h, spp, half = bench.PRESETS[a.preset]
    spp = a.spp or spp
    scene = rtow.final_scene(half_extent=half)
    cam = rtow.camera_cpu(aspect=w / h)
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_PILOT_SCHEDULE
    p = rtow.make_params(w, h, spp, seed=0, flags=flags, rank=a.rank, world=a.world)
    pick, _ = rtow.grid_fit(scene, cam, w, h)
    scale = a.scale or pick

    def model(sc, ph):
        _, costs = rtow.grid_fit(scene, cam, w, h, ph)
        m = [c for s, c in costs if abs(s - sc) < 1e-9]
        return m[0] if m else None

    def timed(sc, ph):
        ctx = rtow.Context(0)
        ctx.upload(scene, grid_scale=sc, grid_phase=ph)
        ms = []
        for _ in range(a.reps + 1):  # the first render pays the pilot
            _, st = ctx.render(cam, p)
            ms.append(st.kernel_ms)
        ctx.close()
        return statistics.median(ms[1:]), st.segments

    grids = [(scale, (i / a.phases, j / a.phases)) for i in range(a.phases) for j in range(a.phases)]
    for e in filter(None, a.extra.split(",")):
        sc, px, pz = (float(x) for x in e.split(":"))
        grids.append((sc, (px, pz)))
    rows, segs = [], None
    for sc, ph in grids:
        t, s = timed(sc, ph)
        assert segs is None or s == segs, "a grid changed the image"
        segs = s
        m = model(sc, ph)
        rows.append((sc, ph, t, m))
        print(json.dumps({"preset": a.preset, "rank": a.rank, "world": a.world, "spp": spp, "scale": round(sc, 4),
                          "phase": [round(ph[0], 4), round(ph[1], 4)], "kernel_ms": round(t, 2),
                          "model_cost": None if m is None else round(m, 4)}), flush=True)
    ts = np.array([r[2] for r in rows])
    both = [(r[3], r[2]) for r in rows if r[3] is not None]
    corr = float(np.corrcoef(*zip(*both))[0, 1]) if len(both) > 2 else None
    best = min(rows, key=lambda r: r[2])
    print(json.dumps({"preset": a.preset, "rank": a.rank, "world": a.world, "summary": True, "scale": round(scale, 4),
                      "phase0_ms": round(rows[0][2], 2), "best_ms": round(best[2], 2),
                      "best": [round(best[0], 4), round(best[1][0], 4), round(best[1][1], 4)],
                      "min_ms": round(float(ts.min()), 2), "max_ms": round(float(ts.max()), 2),
                      "model_time_corr": None if corr is None else round(corr, 3), "segments": segs}), flush=True)


if __name__ == "__main__":
    main()
