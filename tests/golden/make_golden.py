#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only in the build container (needs /root/reference): builds
oracle/_ref/ref_harness from the reference's own src/cpu sources
(oracle/Makefile, target `ref`) and records its outputs as data:

  scene_final_gcc.txt        random_scene() dump, %.17g  (src/cpu/main.cc:32-76)
  ref_c0_400x225x10.ppm.gz   C0 image, byte-identical to the patched reference
  ref_c0_shift_400x225x10.ppm.gz  same config, stream shifted by 10^7 draws
                             (the oracle's own stream-to-stream noise floor)
  ref_five_400x225x100.ppm.gz  five-sphere book scene (negative radius), 100 spp
  ref_stats.json             segments / sphere tests / seconds per render + SHA-256
  kat.jsonl                  known-answer vectors: camera basis, sphere::hit,
                             reflect, refract, reflectance, write_color

Usage: python tests/golden/make_golden.py
"""
import gzip
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def run(args, **kw):
    return subprocess.run([HARNESS] + args, check=True, capture_output=True, **kw)


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_golden.py needs /root/reference (build container only)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    with open(os.path.join(HERE, "scene_final_gcc.txt"), "wb") as f:
        f.write(run(["scene"]).stdout)
    with open(os.path.join(HERE, "kat.jsonl"), "wb") as f:
        f.write(run(["kat"]).stdout)
    stats = {}
    renders = {
        "ref_c0_400x225x10": ["render", "400", "16", "9", "10", "50", "final", "0"],
        "ref_c0_shift_400x225x10": ["render", "400", "16", "9", "10", "50", "final", "10000000"],
        "ref_five_400x225x100": ["render", "400", "16", "9", "100", "50", "five", "0"],
    }
    for name, args in renders.items():
        r = run(args)
        ppm = r.stdout
        st = json.loads(r.stderr.decode().strip().splitlines()[-1])
        st["sha256"] = hashlib.sha256(ppm).hexdigest()
        st["bytes"] = len(ppm)
        st["args"] = args
        stats[name] = st
        with gzip.GzipFile(os.path.join(HERE, name + ".ppm.gz"), "wb", mtime=0) as g:
            g.write(ppm)
        print(name, st)
    with open(os.path.join(HERE, "ref_stats.json"), "w") as f:
        json.dump(stats, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
