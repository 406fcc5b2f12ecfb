#!/usr/bin/env python3
"""Random known-answer vectors for reflect / refract (src/cpu/vec3.h:124-131)
and dielectric::reflectance (src/cpu/material.h:82-87): the REFERENCE's own
functions (oracle/_ref/ref_harness `vectors`) on 300 seeded cases -- unit
incident directions against unit normals at every angle on the refracting
side (cos theta in (0, 1]), refraction ratios 1/2.4 .. 2.4 where refraction
exists, cosines and indices for Schlick -- as fp32 values printed exactly ->
tests/golden/kat_vectors.jsonl.  Build container only.

Usage: python tests/golden/make_vector_kat.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def cases(n=300, seed=11):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        nrm = rng.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        v = rng.normal(size=3)
        v /= np.linalg.norm(v)
        if v @ nrm > 0:
            v = v - 2 * (v @ nrm) * nrm  # incident: against the normal
        cos_t = -(v @ nrm)
        eta = float(rng.choice([1 / 1.5, 1.5, 1 / 2.4, 2.4, 1 / 1.33, 1.33, 1.0]))
        if eta * np.sqrt(max(0.0, 1 - cos_t * cos_t)) > 0.999:  # total internal reflection: no refraction
            continue
        vals = np.concatenate([v, nrm, [eta, rng.uniform(0, 1), rng.choice([1 / 1.5, 1.5, 2.4, 0.7])]])
        out.append(vals.astype(np.float32))
    return out


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_vector_kat.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for v in cases():
            f.write(" ".join("%.17g" % float(x) for x in v) + "\n")
        path = f.name
    r = subprocess.run([HARNESS, "vectors", path], check=True, capture_output=True)
    with open(os.path.join(HERE, "kat_vectors.jsonl"), "wb") as g:
        g.write(r.stdout)
    print(r.stdout.count(b"\n"), "vectors")


if __name__ == "__main__":
    main()
