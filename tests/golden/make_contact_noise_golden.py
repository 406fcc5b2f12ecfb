#!/usr/bin/env python3
"""Noise floor of the contact fixture (tests/fixture_scenes.py `contact`, the
t_min and same-sphere exit attributions): the
REFERENCE (oracle/_ref/ref_harness, src/cpu) renders it at the fixture size
from 8 independent streams (SKIP = k * 10^7 draws; k = 0 is the committed
ref_contact PPM) -> each stream's image mean per channel and segment count in
tests/golden/ref_contact_streams.json.  Build container only.

Usage: python tests/golden/make_contact_noise_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
STREAMS = 8


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_contact_noise_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]
    import numpy as np
    import rtow
    import fixture_scenes
    from oracle_lib import read_ppm_bytes
    from random_scenes import dump_scene_exact
    w, h, spp = fixture_scenes.FIXTURE_SIZE
    path = os.path.join(tempfile.mkdtemp(), "contact.txt")
    dump_scene_exact(fixture_scenes.contact_scene(rtow), path)

    def one(k):
        r = subprocess.run([HARNESS, "render", str(w), "16", "9", str(spp), "50", "file:" + path,
                            str(k * 10_000_000)], check=True, capture_output=True)
        img = read_ppm_bytes(r.stdout).reshape(-1, 3).astype(np.float64)
        seg = json.loads(r.stderr.decode().strip().splitlines()[-1])["segments"]
        return k, img.mean(0).tolist(), seg

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = sorted(ex.map(one, range(STREAMS)))
    out = {"width": w, "height": h, "spp": spp, "depth": 50, "scene": "contact",
           "skip": [k * 10_000_000 for k, _, _ in res],
           "means": [[round(x, 6) for x in m] for _, m, _ in res],
           "segments": [s for _, _, s in res]}
    with open(os.path.join(HERE, "ref_contact_streams.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", STREAMS, "streams")


if __name__ == "__main__":
    main()
