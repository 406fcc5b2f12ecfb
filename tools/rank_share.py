#!/usr/bin/env python3
"""Render the share of ONE rank of a G-GPU frame on one GPU and report its
kernel time and Mray/s: exactly the work each GPU of a G-GPU run does (the
interleaved bands balance the ranks to ~1 %, tools/rank_times.py).  Used for
the 8-GPU BASELINE configs (c3: 7680x4320x1000, c4: 16384^2 x 2000 spp with
10 000 spheres) that one box cannot run whole.

    python tools/rank_share.py --preset c4 --world 8 --rank 0 [--spp N]
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
    a = ap.parse_args()
    import rtow
    w, h, spp, half = bench.PRESETS[a.preset]
    spp = a.spp or spp
    ctx = rtow.Context(0)
    t = time.perf_counter()
    scene = rtow.final_scene(half_extent=half)
    ctx.upload(scene)
    t_up = time.perf_counter() - t
    cam = rtow.camera_cpu(aspect=w / h)
    for r in a.rank:
        p = rtow.make_params(w, h, spp, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH, rank=r, world=a.world)
        t = time.perf_counter()
        img, st = ctx.render(cam, p)
        wall = time.perf_counter() - t
        print(json.dumps({"preset": a.preset, "frame": f"{w}x{h}x{spp}", "spheres": scene.n, "world": a.world,
                          "rank": r, "local_rows": p.local_rows, "kernel_ms": round(st.kernel_ms, 1),
                          "wall_ms_incl_copy": round(wall * 1e3, 1), "segments": st.segments,
                          "mray_s": round(st.segments / st.kernel_ms / 1e3, 1),
                          "upload_s": round(t_up, 2)}), flush=True)


if __name__ == "__main__":
    main()
