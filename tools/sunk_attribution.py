#!/usr/bin/env python3
"""Attribution of the random-scene residual: the kernel
algorithm (oracle kernel mode, the fp32 specification the HIP kernel matches
bit for bit) against the reference's own noise on tests/random_scenes.py's 24
scenes at 96x54x64 -- the 24 reference streams of tests/golden/
ref_random_scenes_means.json (oracle/_ref/ref_harness, src/cpu) -- with each
of the oracle's switches (oracle/rt_oracle.h RTO_OPT_*), so that the scenes
whose bias or segment count sits outside the reference's noise show which
part of the specification moves them.

Per scene and option set: image-mean bias per channel (level) and its z
(kernel seeds' and reference streams' standard errors combined), segments
relative to the reference mean and their z.  CPU only.  Round 6's results
(profiles/r06_sunk_attribution.log) and the depth-cap counts that explain
them (tools/cavity_attribution.py): DESIGN.md 4, "ground-cut spheres".

Usage: python tools/sunk_attribution.py [--scenes 3,17] [--seeds 8] [--opts spec,fp64_hit,...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]

import rtow  # noqa: E402
import random_scenes  # noqa: E402
import oracle_lib as ol  # noqa: E402

OPTS = {
    "spec": 0,
    "no_sealed": ol.RTO_OPT_NO_SEALED,
    "no_same_exit": ol.RTO_OPT_NO_SAME_EXIT,
    "fp64_roots": ol.RTO_OPT_FP64_ROOTS,
    "tmin_world": ol.RTO_OPT_TMIN_WORLD,
}
for name in ("RTO_OPT_FP64_HIT", "RTO_OPT_FP64_PATH"):
    if hasattr(ol, name):
        OPTS[name[8:].lower()] = getattr(ol, name)


def sunk_spheres(scene):
    return random_scenes.ground_cut_spheres(scene)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="all")
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--opts", default="spec")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "ref_random_scenes_means.json")) as f:
        gold = json.load(f)
    scenes = range(24) if a.scenes == "all" else [int(x) for x in a.scenes.split(",")]
    w, h, spp = 96, 54, 64
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    rows = []
    for case in scenes:
        g = gold[str(case)]
        ref = np.array(g["means"], np.float64)
        rseg = np.array(g["segments"], np.float64)
        scene = random_scenes.free_scene(rtow, case)
        sunk = sunk_spheres(scene)
        for oname in a.opts.split(","):
            opt = OPTS[oname]
            img, segs = [], []
            for seed in range(1, a.seeds + 1):
                p = rtow.make_params(w, h, spp, seed=seed)
                sums, _, seg = ol._kernel_render_opts(scene, cam, p, opt, False, 0)
                img.append(rtow.tonemap(sums, spp).reshape(-1, 3).astype(np.float64).mean(0))
                segs.append(seg)
            img, segs = np.array(img), np.array(segs, np.float64)
            bias = img.mean(0) - ref.mean(0)
            sig = np.sqrt(img.var(0, ddof=1) / len(img) + ref.var(0, ddof=1) / len(ref))
            ssig = np.sqrt(segs.var(ddof=1) / len(segs) + rseg.var(ddof=1) / len(rseg))
            row = {"scene": case, "opt": oname, "n": scene.n, "sunk": len(sunk),
                   "bias": [round(float(x), 4) for x in bias], "z": [round(float(x), 2) for x in bias / sig],
                   "seg_rel": float(segs.mean() / rseg.mean() - 1), "seg_z": float((segs.mean() - rseg.mean()) / ssig),
                   "segs": segs.tolist()}
            rows.append(row)
            print("scene %2d %-13s n %2d sunk %d  bias %s  z %s  segs %+.2e (%+.1f sigma)" % (
                case, oname, scene.n, len(sunk), " ".join("%+.4f" % x for x in bias),
                " ".join("%+5.1f" % x for x in bias / sig), row["seg_rel"], row["seg_z"]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
