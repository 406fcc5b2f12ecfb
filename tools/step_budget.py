#!/usr/bin/env python3
"""Wave-level execution counts of the headline frame's per-step regions
(GPU box).  One RT_FLAG_COUNT_WORK render per counting
build, each in its own process (a process loads one librtow):

  base   (RT_COUNT_ITEMS=0): box_hits = wave-level DDA iterations,
         roots = extras root sequences (LEAD + compacted rounds), counted by
         every lane the wave runs them for: / 64 ~ wave-level when the pool
         keeps all lanes busy (lane efficiency ~0.99)
  count1 (RT_COUNT_ITEMS=1): box_hits = wave-level grid item iterations
  count2 (RT_COUNT_ITEMS=2): box_hits = wave-level item iterations with a
         candidate (the grid's root sequences)

    python tools/step_budget.py [--spp 100]        # prints one JSON line

The per-wave-step instruction budget in DESIGN.md §8 is these counts times
the static region counts of tools/isa_regions.py.  count1 / count2 are built
by tools/build_variant.sh with -DRT_COUNT_ITEMS=1 / 2 (.gpurunignore keeps
build/variants off the GPU box: drop that line for the call that runs this).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBS = {"base": "ray-tracing-in-one-weekend_amd/librtow.so",
        "count1": "build/variants/count1.so", "count2": "build/variants/count2.so"}


def one(spp):
    sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))
    import rtow
    ctx = rtow.Context(0)
    ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=3840 / 2160)
    p = rtow.make_params(3840, 2160, spp, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_COUNT_WORK)
    _, st = ctx.render(cam, p)
    print(json.dumps({"segments": st.segments, "wave_steps": st.wave_steps, "box_hits": st.box_hits,
                      "roots": st.root_tests, "lane_cells": st.box_tests, "tests": st.sphere_tests}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        return one(a.spp)
    r = {}
    for name, lib in LIBS.items():
        env = dict(os.environ, RTOW_LIB=os.path.join(ROOT, lib))
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", "--spp", str(a.spp)],
                             env=env, check=True, capture_output=True, text=True, timeout=300).stdout
        r[name] = json.loads(out.strip().splitlines()[-1])
    b = r["base"]
    ws = b["wave_steps"]
    assert all(v["segments"] == b["segments"] for v in r.values())
    print(json.dumps({"workload": f"3840x2160x{a.spp} final scene, grid build", "segments": b["segments"],
                      "wave_steps": ws, "segments_per_wave_step": round(b["segments"] / ws, 2),
                      "per_wave_step": {"dda_iters": round(b["box_hits"] / ws, 3),
                                        "extras_root_seqs_lane_summed": round(b["roots"] / ws, 3),
                                        "extras_root_seqs_wave_approx": round(b["roots"] / ws / 64, 3),
                                        "item_iters": round(r["count1"]["box_hits"] / ws, 3),
                                        "grid_candidate_seqs": round(r["count2"]["box_hits"] / ws, 3),
                                        "lane_cells": round(b["lane_cells"] / ws, 2)}}), flush=True)


if __name__ == "__main__":
    main()
