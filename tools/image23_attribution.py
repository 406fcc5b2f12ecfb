#!/usr/bin/env python3
"""Attribute the brightness difference between the kernel specification in
src/gpu semantics and the reference's own CUDA run of its final scene,
gallery/gpu/image23.png, on the CPU (no GPU time).

The gallery run's scene is restated from its recovered time seed
(tests/gallery_lib.py).  Every variant renders the same rows -- every
`stride`-th band of 8 rows of the 1920x1080 frame at 500 spp, with src/gpu's
camera and fp32 write_color -- and is compared with the gallery's 8x8 block
sums of those rows (tests/golden/gallery_gpu_image23_blocksum8.npz):

  spec        the kernel specification (oracle kernel mode, RT_FLAG_GPU_SEMANTICS),
              seeds 1 and 2 (the seed-to-seed floor)
  gref0       oracle/rt_oracle.cc's src/gpu restatement with no switch (= spec up
              to the dielectric's sqrt / pow forms)
  +hit        src/gpu's sphere::hit quadratic, unrefined roots, set_face_normal by
              dot(d, outward) (no spurious-root or opaque-inside rule)
  +unnorm     ... and unnormalised directions
  +reject     ... and rejection-sampled unit vectors / lens disk
  +fp32sum    ... and fp32 pixel sums (= src/gpu's arithmetic throughout)

    python tools/image23_attribution.py [--stride 4] [--spp 500] > profiles/r03_image23_attribution.log
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]

GREF_NAIVE_HIT, GREF_UNNORM, GREF_REJECT, GREF_FP32_SUM = 1, 2, 4, 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stride", type=int, default=4, help="render every stride-th band of 8 rows")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    a = ap.parse_args()
    import rtow
    import oracle_lib
    from gallery_lib import src_gpu_final_scene
    from test_oracle import gallery_blocks
    L = oracle_lib.lib()
    L.rto_gpuref_render.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p,
                                                             ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    scene = src_gpu_final_scene(rtow)
    cam = rtow.camera_gpu(1920, 1080)  # src/gpu/camera.h:58-71
    W, H = 1920, 1080
    p = rtow.make_params(W, H, a.spp, seed=1, flags=rtow.RT_FLAG_GPU_SEMANTICS | rtow.RT_FLAG_ACCEL_BVH,
                         rank=0, world=a.stride, row_block=8)
    rows = rtow.local_to_global_rows(p)
    keep = rows < H
    g = gallery_blocks("image23")  # (135, 240, 3) 8x8 block means of the levels
    gb = g[(rows[keep][::8] // 8)]  # the bands this rank renders

    def blocks(img):
        img = img[keep].astype(np.float64)
        return img.reshape(-1, 8, W // 8, 8, 3).mean(axis=(1, 3))

    def render(mode, seed):
        p.seed = seed
        v = scene.view()
        out = np.zeros((p.local_rows, W, 3), np.float32)
        seg = ctypes.c_ulonglong()
        t = time.time()
        if mode is None:
            out, segs = oracle_lib.kernel_render(scene, cam, p)
        else:
            assert L.rto_gpuref_render(ctypes.addressof(v), ctypes.addressof(cam), ctypes.addressof(p), mode,
                                       out.ctypes.data, ctypes.byref(seg), 0) == 0
            segs = seg.value
        u8 = rtow.tonemap(out, a.spp, rtow.RT_TONEMAP_GPU)
        return blocks(u8), segs, time.time() - t

    variants = [("spec", None, 1), ("spec_seed2", None, 2), ("gref0", 0, 1), ("+hit", GREF_NAIVE_HIT, 1),
                ("+unnorm", GREF_NAIVE_HIT | GREF_UNNORM, 1),
                ("+reject", GREF_NAIVE_HIT | GREF_UNNORM | GREF_REJECT, 1),
                ("+fp32sum", GREF_NAIVE_HIT | GREF_UNNORM | GREF_REJECT | GREF_FP32_SUM, 1)]
    only = set(filter(None, a.only.split(",")))
    res = {}
    for name, mode, seed in variants:
        if only and name not in only:
            continue
        b, segs, dt = render(mode, seed)
        res[name] = b
        bias = b.reshape(-1, 3).mean(0) - gb.reshape(-1, 3).mean(0)
        err = float(np.abs(b - gb).mean())
        rec = {"variant": name, "mode": mode, "seed": seed, "bias_level": bias.round(4).tolist(),
               "block_err_level": round(err, 4), "segments": segs, "seconds": round(dt, 1),
               "bands": int(keep.sum() // 8), "spp": a.spp}
        if "spec" in res and name != "spec":
            rec["bias_vs_spec_level"] = (b - res["spec"]).reshape(-1, 3).mean(0).round(4).tolist()
        print(json.dumps(rec), flush=True)
    if "spec" in res and "spec_seed2" in res:
        print(json.dumps({"floor_block_err_level": round(float(np.abs(res["spec"] - res["spec_seed2"]).mean()), 4)}),
              flush=True)


if __name__ == "__main__":
    main()
