#!/usr/bin/env python3
"""Wall time of rt_scene_upload (host build of the scan records, BVH, layer
grid and the grid fitter's copy, plus the device copies) and of the first
render's grid fit, for the headline scene (486 spheres) and C4's (10 001),
best of --reps (GPU box).  VERDICT r4 item 3.

    python tools/upload_time.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def main():
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    ctx = rtow.Context(0)
    for half, (w, h) in ((11, (3840, 2160)), (50, (16384, 16384))):
        scene = rtow.final_scene(half_extent=half)
        up, fit = [], []
        for _ in range(a.reps):
            t = time.perf_counter()
            ctx.upload(scene)
            up.append(time.perf_counter() - t)
            t = time.perf_counter()
            rtow.grid_fit(scene, rtow.camera_cpu(aspect=w / h), w, h)
            fit.append(time.perf_counter() - t)
        print(json.dumps({"spheres": scene.n, "upload_ms_best": round(min(up) * 1e3, 2),
                          "upload_ms_median": round(sorted(up)[len(up) // 2] * 1e3, 2),
                          "host_grid_fit_ms_best_incl_builder": round(min(fit) * 1e3, 2),
                          "grid_placement": rtow.accel_info(scene)["grid_placement"]}), flush=True)


if __name__ == "__main__":
    main()
