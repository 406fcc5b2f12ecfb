#!/usr/bin/env python3
"""Active lanes per source region of the headline kernel (VERDICT r5 item 4:
"which blocks carry the 38 % of idle lanes").  GPU box.

Runs the RT_LANE_PROFILE measurement variant (build/lanes.so:
tools/build_variant.sh lanes ray-tracing-in-one-weekend_amd/csrc/rt_kernel.hip
-DRT_LANE_PROFILE) on the bench's frame (3840x2160 final scene, the layer
grid in LDS, pilot order) and prints, per region (rt_kernel.hip kLp*): wave
executions per wave-step, mean lanes in exec when the wave runs it, and mean
lanes that needed it (`useful`: e.g. a grid candidate's lanes whose line
meets the sphere; for most regions the lanes in exec).  The variant's image
equals the product's (checked: same segments).

    RTOW_LIB=build/lanes.so python tools/lane_profile.py [--spp 500]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))
REGIONS = ["step", "closest_hit", "extras_lead", "extras_round", "grid_walk", "dda_iter", "item_iter",
           "grid_cand", "sky", "hit", "lambertian", "metal", "dielectric", "camera", "skip", "tail"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--preset", choices=["c2", "c4"], default="c2",
                    help="c4: rank 0's 1/8 share of C4 (16384^2, 10 001 spheres, cells in LDS) at --spp")
    a = ap.parse_args()
    os.environ.setdefault("RTOW_LIB", os.path.join(ROOT, "build", "variants", "lanes.so"))
    import rtow
    L = rtow.lib()
    L.rt_lane_profile_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * (3 * len(REGIONS)))()
    W, H = (a.width, a.height) if a.preset == "c2" else (16384, 16384)
    world = 1 if a.preset == "c2" else 8
    cam = rtow.camera_cpu(aspect=W / H)
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_PILOT_SCHEDULE
    with rtow.Context(0) as ctx:
        ctx.upload(rtow.final_scene(half_extent=11 if a.preset == "c2" else 50))
        ctx.render(cam, rtow.make_params(W, H, a.spp, seed=1, flags=flags, world=world))  # pilot + grid fit
        assert L.rt_lane_profile_read(buf, 1) == len(REGIONS)
        _, st = ctx.render(cam, rtow.make_params(W, H, a.spp, seed=2, flags=flags, world=world))
        assert L.rt_lane_profile_read(buf, 1) == len(REGIONS)
    ws = st.wave_steps
    out = {"workload": (f"{W}x{H}x{a.spp} final scene, layer grid in LDS, pilot order" if a.preset == "c2" else
                        f"C4 rank 0 of 8: {W}x{H}x{a.spp}, 10 001 spheres, cells in LDS, pilot order"),
           "lib": os.path.relpath(rtow.LIB_PATH, ROOT), "segments": st.segments, "wave_steps": ws,
           "lane_efficiency": st.segments / (64.0 * ws), "regions": {}}
    print("%-13s %10s %9s %9s" % ("region", "per step", "exec", "useful"))
    for i, name in enumerate(REGIONS):
        w, ex, us = buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]
        r = {"runs_per_wave_step": w / ws, "exec_lanes": ex / w if w else 0.0, "useful_lanes": us / w if w else 0.0}
        out["regions"][name] = r
        print("%-13s %10.3f %9.1f %9.1f" % (name, r["runs_per_wave_step"], r["exec_lanes"], r["useful_lanes"]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
