#!/usr/bin/env python3
"""Render the share of ONE rank of a G-GPU frame on one GPU and report its
kernel time and Mray/s: exactly the work each GPU of a G-GPU run does (the
interleaved bands balance the ranks to ~1 %, tools/rank_times.py).  Used for
the 8-GPU BASELINE configs (c3: 7680x4320x1000, c4: 16384^2 x 2000 spp with
10 000 spheres) that one box cannot run whole.

    python tools/rank_share.py --preset c4 --world 8 --rank 0 [--spp N] [--reps R]
                               [--count-work] [--grid-mode auto|lds|cells|global]

--count-work renders once more with the instrumented build (RT_FLAG_COUNT_WORK)
and adds the executed work per segment: sphere tests, DDA cell steps, root
sequences and the lane efficiency.  --grid-mode forces one layer-grid
placement (scheduling/placement only: the image is the same).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def main():
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(bench.PRESETS), default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, nargs="+", default=[0])
    ap.add_argument("--spp", type=int, default=0, help="override the preset's spp (0: keep)")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--count-work", action="store_true")
    ap.add_argument("--grid-mode", default="auto")
    ap.add_argument("--flags", default="", help="extra '+'-joined RT_FLAG_ names")
    ap.add_argument("--units", type=int, default=0, help="rt_params.units (0: automatic)")
    ap.add_argument("--grid-scale", type=float, default=0.0)
    ap.add_argument("--row-block", type=int, default=8, help="rows per interleaved band")
    ap.add_argument("--launch-samples", type=float, default=0.0,
                    help="RT_OPT_LAUNCH_SAMPLES, the launch budget in samples (0: the default 2^35)")
    a = ap.parse_args()
    import rtow
    w, h, spp, half = bench.PRESETS[a.preset]
    spp = a.spp or spp
    ctx = rtow.Context(0)
    if a.launch_samples:
        ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, a.launch_samples)
    t = time.perf_counter()
    scene = rtow.final_scene(half_extent=half)
    ctx.upload(scene, grid_mode=a.grid_mode, grid_scale=a.grid_scale)
    t_up = time.perf_counter() - t
    cam = rtow.camera_cpu(aspect=w / h)
    flags = rtow.RT_FLAG_ACCEL_BVH
    for name in filter(None, a.flags.split("+")):
        flags |= getattr(rtow, "RT_FLAG_" + name)
    for r in a.rank:
        p = rtow.make_params(w, h, spp, seed=0, flags=flags, rank=r, world=a.world, units=a.units,
                             row_block=a.row_block)
        for _ in range(a.reps):
            t = time.perf_counter()
            img, st = ctx.render(cam, p)
            wall = time.perf_counter() - t
            rec = {"preset": a.preset, "frame": f"{w}x{h}x{spp}", "spheres": scene.n, "world": a.world,
                   "rank": r, "local_rows": p.local_rows, "row_block": a.row_block, "grid_mode": a.grid_mode, "flags": a.flags,
                   "units": a.units,
                   "kernel_ms": round(st.kernel_ms, 1), "launches": getattr(st, "launches", 1),
                   "wall_ms_incl_copy": round(wall * 1e3, 1), "segments": st.segments,
                   "mray_s": round(st.segments / st.kernel_ms / 1e3, 1), "upload_s": round(t_up, 2)}
            print(json.dumps(rec), flush=True)
        if a.count_work:
            pw = rtow.make_params(w, h, spp, seed=0, flags=flags | rtow.RT_FLAG_COUNT_WORK, rank=r,
                                  world=a.world)
            _, sw = ctx.render(cam, pw)
            seg = max(1, sw.segments)
            print(json.dumps({"preset": a.preset, "rank": r, "work": True, "segments": sw.segments,
                              "lane_efficiency": round(seg / (64.0 * max(1, sw.wave_steps)), 4),
                              "sphere_tests_per_seg": round(sw.sphere_tests / seg, 3),
                              "cell_steps_per_seg": round(sw.box_tests / seg, 3),
                              "wave_dda_iters_per_seg": round(sw.box_hits / seg, 4),
                              "root_seqs_per_seg": round(sw.root_tests / seg, 3),
                              "wave_steps": sw.wave_steps,
                              "kernel_ms_count_build": round(sw.kernel_ms, 1)}), flush=True)


if __name__ == "__main__":
    main()
