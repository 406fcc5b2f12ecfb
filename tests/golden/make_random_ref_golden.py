#!/usr/bin/env python3
"""Fixtures for tests/test_oracle.py::test_reference_mode_byte_identical_random_scenes:
the REFERENCE itself (oracle/_ref/ref_harness, built from /root/reference's
src/cpu) rendering tests/random_scenes.py's seeded scenes with the final
scene's camera -> SHA-256 of each P3 image and its segment count, in
tests/golden/ref_random_scenes.json.  Build container only.

Usage: python tests/golden/make_random_ref_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_random_ref_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]
    import rtow
    import random_scenes
    out = {}
    tmp = tempfile.mkdtemp()
    for k, (w, spp, depth) in enumerate(random_scenes.CASES):
        scene = random_scenes.free_scene(rtow, k)
        path = os.path.join(tmp, "s%d.txt" % k)
        random_scenes.dump_scene_exact(scene, path)
        r = subprocess.run([HARNESS, "render", str(w), "16", "9", str(spp), str(depth), "file:" + path, "0"],
                           check=True, capture_output=True)
        st = json.loads(r.stderr.decode().strip().splitlines()[-1])
        out[str(k)] = {"width": w, "spp": spp, "depth": depth, "spheres": scene.n,
                       "segments": st["segments"], "sha256": hashlib.sha256(r.stdout).hexdigest()}
        print(k, out[str(k)], flush=True)
    with open(os.path.join(HERE, "ref_random_scenes.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
