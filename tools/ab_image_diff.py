#!/usr/bin/env python3
"""Image difference between two librtow builds on one frame (GPU box).

    RTOW_LIB=<lib A> python tools/ab_image_diff.py save A.npy [--w --h --spp --seed]
    RTOW_LIB=<lib B> python tools/ab_image_diff.py diff A.npy [--w --h --spp --seed]

`save` renders the frame (headline 3840x2160x500 by default, the bench's
flags) and stores its fp32 sums; `diff` renders it with another build and
prints one JSON line: segments of both, how many fp32 sums and how many
tonemapped pixels (src/cpu write_color) differ, and the largest level
difference per channel.  Used for the opaque-inside rule's A/B (DESIGN.md 2
step 4).
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
    ap.add_argument("mode", choices=["save", "diff"])
    ap.add_argument("path")
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--half-extent", type=int, default=11)
    a = ap.parse_args()
    import rtow
    ctx = rtow.Context(0)
    ctx.upload(rtow.final_scene(half_extent=a.half_extent))
    cam = rtow.camera_cpu(aspect=a.w / a.h)
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_PILOT_SCHEDULE
    img, st = ctx.render(cam, rtow.make_params(a.w, a.h, a.spp, seed=a.seed, flags=flags))
    lib = os.path.basename(rtow.LIB_PATH)
    if a.mode == "save":
        np.save(a.path, img)
        with open(a.path + ".json", "w") as f:
            json.dump({"lib": lib, "segments": st.segments, "kernel_ms": st.kernel_ms}, f)
        print(json.dumps({"saved": a.path, "lib": lib, "segments": st.segments}))
        return
    ref = np.load(a.path)
    meta = json.load(open(a.path + ".json"))
    ta, tb = rtow.tonemap(ref, a.spp).reshape(-1, 3), rtow.tonemap(img, a.spp).reshape(-1, 3)
    dl = np.abs(ta.astype(np.int32) - tb.astype(np.int32))
    px = np.any(dl > 0, axis=1)
    print(json.dumps({"frame": "%dx%dx%d seed %d" % (a.w, a.h, a.spp, a.seed),
                      "lib_a": meta["lib"], "lib_b": lib, "segments_a": meta["segments"], "segments_b": st.segments,
                      "segments_delta": st.segments - meta["segments"],
                      "sums_differing": int((ref != img).sum()),
                      "pixels_differing_sums": int(np.any(ref != img, axis=2).sum()),
                      "pixels_differing_levels": int(px.sum()), "pixels": int(px.size),
                      "max_level_diff_rgb": dl.max(axis=0).tolist(),
                      "max_sum_diff": float(np.abs(ref.astype(np.float64) - img).max()),
                      "mean_level_diff_rgb": (tb.astype(np.float64).mean(0) - ta.astype(np.float64).mean(0)).round(6).tolist()}))


if __name__ == "__main__":
    main()
