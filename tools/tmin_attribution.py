#!/usr/bin/env python3
"""t_min unit attribution.

The reference tests its roots against t_min = 0.001 in units of the ray's
UNnormalised direction (src/cpu/main.cc:19, sphere.h:37-41; src/gpu
camera.h:117): camera rays |d| ~ 10, lambertian n + u with |d| in (0, 2],
metal reflect + fuzz p, glass ~1.  The round-1..4 specification tested 0.001
world units on the normalised ray.  This renders the oracle's kernel mode in
both forms (the same seeds: a paired comparison) against the reference's own
fixtures and prints, per scene set, the image-mean bias against the reference,
the 16x16 block error against the reference's stream-to-stream floor, the
segment counts, and the paired difference (ray units - world units) with its
standard error over seeds.

  python tools/tmin_attribution.py [--seeds 4] [--skip-c0] [--skip-random] [--skip-contact]

Needs only the committed fixtures (tests/golden) and oracle/librt_oracle.so.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]

import rtow  # noqa: E402
from oracle_lib import golden_ppm, golden_stats, kernel_render, read_ppm_bytes, reference_render_view  # noqa: E402


def block_means(img, b=16):
    h, w = img.shape[0] // b * b, img.shape[1] // b * b
    x = img[:h, :w].astype(np.float64)
    return x.reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def render_both(scene, cam, w, h, spp, seeds):
    out = {}
    for form in ("ray", "world"):
        imgs, segs = [], []
        for s in seeds:
            sums, seg = kernel_render(scene, cam, rtow.make_params(w, h, spp, seed=s), tmin_world=form == "world")
            imgs.append(rtow.tonemap(sums, spp).reshape(h, w, 3))
            segs.append(seg)
        out[form] = (imgs, segs)
    return out


def summarise(name, both, ref, ref2, ref_segs):
    rmean = ref.reshape(-1, 3).astype(np.float64).mean(0)
    rep = {"set": name}
    for form in ("ray", "world"):
        imgs, segs = both[form]
        b = np.array([i.reshape(-1, 3).astype(np.float64).mean(0) - rmean for i in imgs])
        rep[form] = {
            "bias": b.mean(0).round(4).tolist(),
            "bias_sem": (b.std(0, ddof=1) / np.sqrt(len(imgs))).round(4).tolist() if len(imgs) > 1 else None,
            "segments_dev": float(np.mean(segs) / ref_segs - 1),
        }
        if ref2 is not None:
            rep[form]["block_err"] = round(float(np.mean([np.abs(block_means(i) - block_means(ref)).mean()
                                                          for i in imgs])), 4)
    if ref2 is not None:
        rep["block_floor"] = round(float(np.abs(block_means(ref2) - block_means(ref)).mean()), 4)
        r, r2 = ref.reshape(-1, 3).astype(np.float64), ref2.reshape(-1, 3).astype(np.float64)
        rep["ref_bias_sigma"] = ((r - r2).std(0) / np.sqrt(r.shape[0])).round(4).tolist()
    # paired: the same seeds and draws in both forms
    d = np.array([a.reshape(-1, 3).astype(np.float64).mean(0) - b.reshape(-1, 3).astype(np.float64).mean(0)
                  for a, b in zip(both["ray"][0], both["world"][0])])
    ds = np.array(both["ray"][1], np.float64) - np.array(both["world"][1], np.float64)
    px = np.mean([np.count_nonzero(np.any(a != b, axis=2)) for a, b in zip(both["ray"][0], both["world"][0])])
    rep["paired"] = {"bias_delta": d.mean(0).round(5).tolist(),
                     "bias_delta_sem": (d.std(0, ddof=1) / np.sqrt(len(d))).round(5).tolist() if len(d) > 1 else None,
                     "segments_delta": float(ds.mean()), "segments_delta_rel": float(ds.mean() / ref_segs),
                     "pixels_differing": float(px)}
    print(json.dumps(rep), flush=True)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=4)
    ap.add_argument("--skip-c0", action="store_true")
    ap.add_argument("--skip-random", action="store_true")
    ap.add_argument("--skip-contact", action="store_true")
    a = ap.parse_args()
    seeds = list(range(a.seeds))
    st = golden_stats()
    if not a.skip_c0:
        w, h, spp = 400, 225, 100
        ref = read_ppm_bytes(golden_ppm("ref_final_400x225x100"))
        ref2 = read_ppm_bytes(golden_ppm("ref_final_shift_400x225x100"))
        both = render_both(rtow.final_scene(), rtow.camera_cpu(aspect=16.0 / 9.0), w, h, spp, seeds)
        summarise("final scene 400x225x100 (C0 @ 100 spp)", both, ref, ref2, st["ref_final_400x225x100"]["segments"])
    if not a.skip_contact:
        import fixture_scenes
        w, h, spp = fixture_scenes.FIXTURE_SIZE
        name = "ref_contact_%dx%dx%d" % (w, h, spp)
        if name in st:
            ref = read_ppm_bytes(golden_ppm(name)).reshape(h, w, 3)
            ref2 = read_ppm_bytes(golden_ppm("ref_contact_shift_%dx%dx%d" % (w, h, spp))).reshape(h, w, 3)
            both = render_both(fixture_scenes.contact_scene(rtow), rtow.camera_cpu(aspect=16.0 / 9.0), w, h, spp,
                               seeds)
            summarise("contact fixture %dx%dx%d" % (w, h, spp), both, ref, ref2, st[name]["segments"])
        else:
            print("(no contact fixture yet: tests/golden/make_golden.py --only contact)")
    if not a.skip_random:
        import random_scenes
        w, spp = 96, 64
        cam = rtow.camera_cpu(aspect=16.0 / 9.0)
        worst = {"ray": 0.0, "world": 0.0}
        agg = []
        for case in range(24):
            scene = random_scenes.free_scene(rtow, case)
            ref, rseg = reference_render_view(scene, w, 16.0 / 9.0, spp, 50)
            both = render_both(scene, cam, w, ref.shape[0], spp, [1 + s for s in seeds])
            rep = summarise("random scene %d 96x54x64" % case, both, ref, None, rseg)
            for f in worst:
                worst[f] = max(worst[f], float(np.abs(rep[f]["bias"]).max()))
            agg.append(rep)
        print(json.dumps({"random_worst_abs_bias": worst,
                          "random_max_abs_paired_delta": max(float(np.abs(r["paired"]["bias_delta"]).max())
                                                             for r in agg)}))


if __name__ == "__main__":
    main()
