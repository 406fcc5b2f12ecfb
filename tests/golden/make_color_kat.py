#!/usr/bin/env python3
"""Known-answer vectors for write_color (src/cpu/color.h:8-23) at its level
boundaries: the REFERENCE's own write_color (oracle/_ref/ref_harness
`colors`) on fp32 pixel sums within a few ulps of every level's threshold
(sum = (k / 256)^2 * spp for random k and spp), plus 0, NaN-free extremes and
sums above spp -> tests/golden/kat_colors.txt (one `r g b spp | levels`
line each).  Build container only.

Usage: python tests/golden/make_color_kat.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def sums(n=700, seed=5):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        spp = int(rng.choice([1, 3, 7, 10, 64, 100, 500, 1000, 4096, 2 ** 20]))
        vals = []
        for _c in range(3):
            k = int(rng.integers(0, 257))
            base = np.float32((k / 256.0) ** 2 * spp)
            ulps = int(rng.integers(-3, 4))
            v = base
            for _u in range(abs(ulps)):
                v = np.nextafter(v, np.float32(np.inf if ulps > 0 else -np.inf), dtype=np.float32)
            vals.append(max(np.float32(0), v))
        out.append((vals, spp))
    out += [([np.float32(0)] * 3, 10), ([np.float32(1e9), np.float32(1e-9), np.float32(3.3)], 7),
            ([np.float32(5000), np.float32(4096), np.float32(4095.9)], 4096)]
    return out


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_color_kat.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    ss = sums()
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for vals, spp in ss:
            f.write(" ".join("%.17g" % float(v) for v in vals) + " %d\n" % spp)
        path = f.name
    r = subprocess.run([HARNESS, "colors", path], check=True, capture_output=True, text=True)
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(ss)
    with open(os.path.join(HERE, "kat_colors.txt"), "w") as g:
        for (vals, spp), line in zip(ss, lines):
            g.write(" ".join("%.17g" % float(v) for v in vals) + " %d | %s\n" % (spp, line))
    print(len(ss), "colors")


if __name__ == "__main__":
    main()
