#!/usr/bin/env python3
"""Kernel time of the whole headline frame on one GPU for given rt_params.units
values (scheduling only: the image is identical for every value).

    python tools/units_frame.py [--units 1 2 4] [--w 3840 --h 2160 --spp 500]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--units", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--pilot", action="store_true",
                    help="RT_FLAG_PILOT_SCHEDULE: each value renders twice, the second (cached order) is timed")
    a = ap.parse_args()
    import rtow
    ctx = rtow.Context(0)
    ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=a.w / a.h)
    ref = None
    for u in a.units:
        flags = rtow.RT_FLAG_ACCEL_BVH | (rtow.RT_FLAG_PILOT_SCHEDULE if a.pilot else 0)
        p = rtow.make_params(a.w, a.h, a.spp, seed=0, flags=flags)
        p.units = u
        for _ in range(2 if a.pilot else 1):
            img, st = ctx.render(cam, p)
        if ref is None:
            ref = img
        print(json.dumps({"frame": f"{a.w}x{a.h}x{a.spp}", "pilot": a.pilot, "units": u, "kernel_ms": round(st.kernel_ms, 3),
                          "identical": bool(np.array_equal(ref, img))}), flush=True)


if __name__ == "__main__":
    main()
