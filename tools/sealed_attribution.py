#!/usr/bin/env python3
"""The opaque-inside rule's segments (VERDICT r4 Weak 1):
how many segments the REFERENCE's arithmetic (the fp64 restatement, byte-
identical to src/cpu) traces after a path's first hit on the inside of a
sealed lambertian sphere -- segments the kernel's rule does not trace -- and
how many the kernel algorithm (the oracle's kernel mode) drops with the rule
against the same algorithm without it (paired seeds).

    python tools/sealed_attribution.py [--spp 10 100] [--seeds 16]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]

import rtow  # noqa: E402
from oracle_lib import kernel_render, lib, reference_render  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, nargs="+", default=[10, 100])
    ap.add_argument("--seeds", type=int, default=16)
    a = ap.parse_args()
    L = lib()
    L.rto_reference_trapped.restype = ctypes.c_ulonglong
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=400 / 225)
    for spp in a.spp:
        _, ref_segs = reference_render(400, 16.0 / 9.0, spp)
        trapped = int(L.rto_reference_trapped())
        rule, norule = [], []
        for s in range(a.seeds):
            rule.append(kernel_render(scene, cam, rtow.make_params(400, 225, spp, seed=s))[1])
            norule.append(kernel_render(scene, cam, rtow.make_params(400, 225, spp, seed=s), no_sealed=True)[1])
        rule, norule = np.array(rule, float), np.array(norule, float)
        d = norule - rule
        print(json.dumps({"frame": "final scene 400x225x%d" % spp, "reference_segments": ref_segs,
                          "reference_trapped_segments": trapped,
                          "reference_trapped_share": trapped / ref_segs,
                          "kernel_segments_rule_mean": rule.mean(), "kernel_segments_norule_mean": norule.mean(),
                          "kernel_dropped_share": d.mean() / rule.mean(),
                          "kernel_dropped_share_sem": d.std(ddof=1) / np.sqrt(len(d)) / rule.mean(),
                          "kernel_rule_vs_reference": rule.mean() / ref_segs - 1,
                          "kernel_norule_vs_reference": norule.mean() / ref_segs - 1}),
              flush=True)


if __name__ == "__main__":
    main()
