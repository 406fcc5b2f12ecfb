#!/usr/bin/env python3
"""Random known-answer vectors for sphere::hit: the REFERENCE's own
sphere::hit (src/cpu/sphere.h:24-51, through oracle/_ref/ref_harness `hits`)
on 600 seeded random rays and spheres -- small, large, negative-radius and
ground spheres; rays from outside aimed near the sphere, from the surface
(secondary rays leaving or entering), and from inside; unnormalised
directions -- written to tests/golden/kat_hits.jsonl.  Every input is an
fp32 value printed exactly, so the device (which takes fp32 inputs) and the
reference see the same numbers.  Build container only.

Usage: python tests/golden/make_hit_kat.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def cases(n=600, seed=2026):
    rng = np.random.default_rng(seed)
    f32 = np.float32
    out = []
    for k in range(n):
        kind = k % 4
        if kind == 3:  # the ground
            c, r = np.array([0.0, -1000.0, 0.0]), 1000.0
        else:
            c = rng.uniform(-10, 10, 3)
            r = [rng.uniform(0.05, 0.5), rng.uniform(0.5, 3.0), -rng.uniform(0.05, 2.0)][kind]
        a = abs(r)
        where = rng.uniform()
        if where < 0.5:  # from outside, aimed within ~1.5 radii of the centre
            o = c + rng.normal(size=3) / 1.0 * rng.uniform(2 * a, 20 + 2 * a) if kind != 3 else \
                np.array([rng.uniform(-30, 30), rng.uniform(0.001, 5), rng.uniform(-30, 30)])
            target = c + rng.normal(size=3) * 0.8 * a if kind != 3 else \
                np.array([rng.uniform(-60, 60), 0.0, rng.uniform(-60, 60)])
            d = target - o
        elif where < 0.8:  # from the surface: a secondary ray leaving or entering
            nrm = rng.normal(size=3)
            nrm /= np.linalg.norm(nrm)
            if kind == 3:
                nrm = np.array([rng.uniform(-0.05, 0.05), 1.0, rng.uniform(-0.05, 0.05)])
                nrm /= np.linalg.norm(nrm)
            o = c + a * nrm
            d = rng.normal(size=3) + (1.0 if rng.uniform() < 0.5 else -1.0) * nrm
        else:  # from inside
            o = c + rng.normal(size=3) * 0.3 * a if kind != 3 else np.array([0.0, -5.0, 0.0])
            d = rng.normal(size=3)
        d = d * rng.uniform(0.1, 5.0)
        vals = np.concatenate([o, d, c, [r]]).astype(f32)
        if np.linalg.norm(vals[3:6]) > 0:
            out.append(vals)
    return np.array(out)


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_hit_kat.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    cs = cases()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for v in cs:
            f.write(" ".join("%.17g" % float(x) for x in v) + "\n")
        path = f.name
    r = subprocess.run([HARNESS, "hits", path], check=True, capture_output=True)
    with open(os.path.join(HERE, "kat_hits.jsonl"), "wb") as g:
        g.write(r.stdout)
    print(len(cs), "cases,", r.stdout.count(b'"hit": true'), "hits")


if __name__ == "__main__":
    main()
