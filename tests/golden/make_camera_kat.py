#!/usr/bin/env python3
"""Random known-answer vectors for the src/cpu camera (camera.h:8-26): the
REFERENCE's own camera constructor (oracle/_ref/ref_harness `cameras`) on 200
seeded random parameter sets -- eye and target anywhere, vup tilted, vfov
5-150 degrees, aspect 0.3-4, aperture 0-2, focus 0.5-50 -- written to
tests/golden/kat_cameras.jsonl.  Build container only.

Usage: python tests/golden/make_camera_kat.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def params(n=200, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        frm, at = rng.uniform(-50, 50, 3), rng.uniform(-10, 10, 3)
        vup = np.array([0.0, 1.0, 0.0]) + rng.normal(size=3) * rng.choice([0.0, 0.3])
        w = frm - at
        if np.linalg.norm(w) < 0.5 or np.linalg.norm(np.cross(vup, w)) < 0.2 * np.linalg.norm(vup) * np.linalg.norm(w):
            continue  # eye on the target, or vup along the view
        out.append(np.concatenate([frm, at, vup, [rng.uniform(5, 150), rng.uniform(0.3, 4.0),
                                                  rng.choice([0.0, rng.uniform(0, 2)]), rng.uniform(0.5, 50)]]))
    return np.array(out)


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_camera_kat.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for v in params():
            f.write(" ".join("%.17g" % float(x) for x in v) + "\n")
        path = f.name
    r = subprocess.run([HARNESS, "cameras", path], check=True, capture_output=True)
    with open(os.path.join(HERE, "kat_cameras.jsonl"), "wb") as g:
        g.write(r.stdout)
    print(r.stdout.count(b"\n"), "cameras")


if __name__ == "__main__":
    main()
