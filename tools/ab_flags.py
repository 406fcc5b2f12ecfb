#!/usr/bin/env python3
"""A/B kernel time of render flags on one frame (default: headline 3840x2160x500).

    python tools/ab_flags.py [--w --h --spp] [--reps 2] [--option NAME=VALUE ...] FLAGS_A FLAGS_B ...

Each FLAGS_* is a '+'-joined list of rtow flag names without the RT_FLAG_
prefix (e.g. ACCEL_BVH+PILOT_SCHEDULE) or 0.  --option sets a context option
(rt_context_set_option, the name without RT_OPT_: GRID_SCALE=1.1,
GRID_PLACEMENT=3, BVH_LEAF=2, ...) before the scene upload.  Prints kernel ms
per variant and checks that all variants produce identical sums.
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
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--half-extent", type=int, default=11)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import rtow
    ctx = rtow.Context(0)
    opts = {}
    for o in a.option:
        name, value = o.split("=", 1)
        ctx.set_option(getattr(rtow, "RT_OPT_" + name), float(value))
        opts[name] = float(value)
    ctx.upload(rtow.final_scene(half_extent=a.half_extent))
    cam = rtow.camera_cpu(aspect=a.w / a.h)
    ref = None
    for v in a.variants:
        flags = 0
        for name in v.split("+"):
            if name != "0":
                flags |= getattr(rtow, "RT_FLAG_" + name)
        ms = []
        for _ in range(a.reps):
            img, st = ctx.render(cam, rtow.make_params(a.w, a.h, a.spp, seed=0, flags=flags))
            ms.append(st.kernel_ms)
        same = None
        if ref is None:
            ref = img
        else:
            same = bool(np.array_equal(ref, img))
        import hashlib
        print(json.dumps({"lib": os.path.basename(rtow.LIB_PATH), "variant": v, "options": opts,
                          "kernel_ms": [round(x, 3) for x in ms], "segments": st.segments,
                          "identical_to_first": same,
                          "sha256": hashlib.sha256(img.tobytes()).hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
