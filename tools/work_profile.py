#!/usr/bin/env python3
"""Per-segment work counters of the render kernel (RT_FLAG_COUNT_WORK build).

    python tools/work_profile.py [--w 3840 --h 2160 --spp 500] [--accel bvh|scan]

Prints, per traced segment (lane-weighted, i.e. per wave-step as the wave
executes it): box visits, leaf visits, sphere tests and root/interval
sequences -- the inputs of the VALU budget in DESIGN.md section 7.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=3840)
    ap.add_argument("--h", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--accel", default="bvh", choices=["bvh", "scan"])
    ap.add_argument("--half-extent", type=int, default=11)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--flags", default="", help="extra '+'-joined RT_FLAG_ names, e.g. SORT_RAYS")
    a = ap.parse_args()
    import rtow
    ctx = rtow.Context(0)
    scene = rtow.final_scene(half_extent=a.half_extent)
    ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=a.w / a.h)
    flags = rtow.RT_FLAG_COUNT_WORK | (rtow.RT_FLAG_ACCEL_BVH if a.accel == "bvh" else 0)
    for name in filter(None, a.flags.split("+")):
        flags |= getattr(rtow, "RT_FLAG_" + name)
    _, st = ctx.render(cam, rtow.make_params(a.w, a.h, a.spp, max_depth=a.depth, seed=0, flags=flags))
    seg = st.segments
    out = {
        "workload": f"{a.w}x{a.h}x{a.spp} depth={a.depth} spheres={scene.n} accel={a.accel} {a.flags}",
        "segments": seg,
        "lane_efficiency": round(seg / (64.0 * st.wave_steps), 4),
        "box_visits_per_seg": round(st.box_tests / seg, 3),
        "own_box_hits_per_seg": round(st.box_hits / seg, 3),
        "leaf_visits_per_seg": round(st.sphere_tests / seg / 4, 3) if a.accel == "bvh" else None,
        "sphere_tests_per_seg": round(st.sphere_tests / seg, 3),
        "root_seqs_per_seg": round(st.root_tests / seg, 3),
        "kernel_ms_count_build": round(st.kernel_ms, 3),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
