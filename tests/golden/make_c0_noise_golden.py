#!/usr/bin/env python3
"""Noise floor of the C0 comparison (VERDICT r4 Weak 1: C0's blue bias of
-0.10/255 against one reference render, unattributed): the REFERENCE itself
(oracle/_ref/ref_harness, built from /root/reference's src/cpu) rendering C0
(the final scene, 400x225, 10 spp, depth 50) from 8 independent streams (SKIP
= k * 10^7 draws after the scene; k = 0 is the committed ref_c0 PPM) -> each
stream's image mean per channel and segment count, plus its 16x16 block means,
in tests/golden/ref_c0_streams.json.  tests/test_oracle.py bounds the kernel
algorithm's bias at C0 by the spread of these streams.  Build container only.

Usage: python tests/golden/make_c0_noise_golden.py
"""
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
STREAMS = 8


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_c0_noise_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import numpy as np
    from oracle_lib import read_ppm_bytes

    def one(k):
        r = subprocess.run([HARNESS, "render", "400", "16", "9", "10", "50", "final", str(k * 10_000_000)],
                           check=True, capture_output=True)
        img = read_ppm_bytes(r.stdout).reshape(225, 400, 3).astype(np.float64)
        seg = json.loads(r.stderr.decode().strip().splitlines()[-1])["segments"]
        blocks = img[:224, :400].reshape(14, 16, 25, 16, 3).mean(axis=(1, 3))
        return k, img.reshape(-1, 3).mean(0).tolist(), seg, blocks

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = sorted(ex.map(one, range(STREAMS)))
    out = {"width": 400, "height": 225, "spp": 10, "depth": 50, "scene": "final",
           "skip": [k * 10_000_000 for k, _, _, _ in res],
           "means": [[round(x, 6) for x in m] for _, m, _, _ in res],
           "segments": [s for _, _, s, _ in res],
           "block_means_16": [np.round(b, 4).tolist() for _, _, _, b in res]}
    with open(os.path.join(HERE, "ref_c0_streams.json"), "w") as f:
        json.dump(out, f)
    print("wrote", STREAMS, "streams")


if __name__ == "__main__":
    main()
