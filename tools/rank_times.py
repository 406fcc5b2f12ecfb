#!/usr/bin/env python3
"""Kernel time of every rank's share of the headline frame, rendered one after
another on ONE GPU: predicts the strong-scaling speed-up at N GPUs (slowest
rank vs the whole frame), before any gather cost.

    python tools/rank_times.py [--world 2 4 8] [--w 3840 --h 2160 --spp 500]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--units", type=int, nargs="+", default=[0], help="rt_params.units values (0 = auto)")
    ap.add_argument("--pilot", action="store_true",
                    help="RT_FLAG_PILOT_SCHEDULE; every share is rendered twice and the second "
                         "(with the cached tile order) is timed")
    a = ap.parse_args()
    import rtow
    ctx = rtow.Context(0)
    ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=a.w / a.h)
    flags = rtow.RT_FLAG_ACCEL_BVH | (rtow.RT_FLAG_PILOT_SCHEDULE if a.pilot else 0)
    reps = 2 if a.pilot else 1
    p = rtow.make_params(a.w, a.h, a.spp, seed=0, flags=flags)
    for _ in range(reps):
        _, st = ctx.render(cam, p)
    full = st.kernel_ms
    print(json.dumps({"world": 1, "kernel_ms": round(full, 2)}), flush=True)
    for g in a.world:
        for u in a.units:
            ms = []
            for r in range(g):
                p = rtow.make_params(a.w, a.h, a.spp, seed=0, flags=flags, rank=r, world=g,
                                     row_block=a.row_block, units=u)
                for _ in range(reps):
                    _, st = ctx.render(cam, p)
                ms.append(st.kernel_ms)
            print(json.dumps({"world": g, "units": u, "rank_ms": [round(x, 2) for x in ms],
                              "max_ms": round(max(ms), 2), "ideal_ms": round(full / g, 2),
                              "speedup_bound": round(full / max(ms), 3)}), flush=True)


if __name__ == "__main__":
    main()
