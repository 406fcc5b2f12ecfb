#!/usr/bin/env python3
"""Noise floor of the random-scene comparison (VERDICT r4 Missing 2 / Weak 1):
the REFERENCE itself (oracle/_ref/ref_harness, built from /root/reference's
src/cpu) rendering each of tests/random_scenes.py's 24 scenes at the test's
96x54x64, depth 50, with the final scene's camera, from 6 independent
streams (SKIP = k * 10^7 draws after the scene; one stream draws ~5*10^6; 6 streams until round 5, 24 since round 6) -> the image-mean of every
stream per channel, in tests/golden/ref_random_scenes_means.json.  The
stream-to-stream spread of those means is the reference's own noise on each
scene, against which tests/test_oracle.py bounds the kernel algorithm's bias.
Build container only.

Usage: python tests/golden/make_random_noise_golden.py
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
W, SPP, DEPTH, STREAMS = 96, 64, 50, 24


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_random_noise_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]
    import numpy as np
    import rtow
    import random_scenes
    from oracle_lib import read_ppm_bytes
    tmp = tempfile.mkdtemp()
    jobs = []
    for k in range(len(random_scenes.CASES)):
        path = os.path.join(tmp, "s%d.txt" % k)
        random_scenes.dump_scene_exact(random_scenes.free_scene(rtow, k), path)
        for j in range(STREAMS):
            jobs.append((k, j, path))

    def one(job):
        k, j, path = job
        r = subprocess.run([HARNESS, "render", str(W), "16", "9", str(SPP), str(DEPTH), "file:" + path,
                            str(j * 10_000_000)], check=True, capture_output=True)
        img = read_ppm_bytes(r.stdout).reshape(-1, 3).astype(np.float64)
        seg = json.loads(r.stderr.decode().strip().splitlines()[-1])["segments"]
        return k, j, img.mean(0).tolist(), seg

    out = {}
    with ThreadPoolExecutor(max_workers=int(os.environ.get("JOBS", min(8, os.cpu_count() or 1)))) as ex:
        for k, j, mean, seg in ex.map(one, jobs):
            e = out.setdefault(str(k), {"width": W, "spp": SPP, "depth": DEPTH, "means": [None] * STREAMS,
                                        "segments": [None] * STREAMS})
            e["means"][j] = [round(x, 6) for x in mean]
            e["segments"][j] = seg
    with open(os.path.join(HERE, "ref_random_scenes_means.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", len(out), "scenes")


if __name__ == "__main__":
    main()
