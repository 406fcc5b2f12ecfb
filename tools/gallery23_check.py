#!/usr/bin/env python3
"""The product (GPU semantics) on src/gpu's final scene from the gallery run's
seed, 1920x1080 at 500 spp, against gallery/gpu/image23.png's block sums:
block error vs our own seed-to-seed floor and the image-mean bias (GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import rtow  # noqa: E402
from gallery_lib import src_gpu_final_scene  # noqa: E402
from test_oracle import blocks8, gallery_blocks  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ctx = rtow.Context(0)
ctx.upload(src_gpu_final_scene(rtow))
cam = rtow.camera_gpu(1920, 1080)
blk = []
for seed in (1, 2):
    sums, st = ctx.render(cam, rtow.make_params(1920, 1080, spp, seed=seed,
                                                flags=rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_GPU_SEMANTICS))
    img = rtow.tonemap(sums, spp, rtow.RT_TONEMAP_GPU)
    blk.append(blocks8(img))
    if seed == 1 and len(sys.argv) > 2:  # keep the image (e.g. gpurun_out/g23.npy) to look at
        np.save(sys.argv[2], img)
a, b = blk
g = gallery_blocks("image23")
n = a.shape[0] * a.shape[1]
out = {"spp": spp, "bias": (a.reshape(-1, 3).mean(0) - g.reshape(-1, 3).mean(0)).round(4).tolist(),
       "sigma": ((a - b).reshape(-1, 3).std(0) / np.sqrt(n)).round(4).tolist(),
       "block_err": round(float(np.abs(a - g).mean()), 4), "block_floor": round(float(np.abs(a - b).mean()), 4),
       "block_err_p99": round(float(np.percentile(np.abs(a - g), 99)), 3),
       "block_floor_p99": round(float(np.percentile(np.abs(a - b), 99)), 3)}
print(json.dumps(out))
d = np.abs(a - g).max(axis=2)
i, j = np.unravel_index(np.argsort(d, axis=None)[-5:], d.shape)
print("largest block differences (row, col, levels):", [(int(x), int(y), round(float(d[x, y]), 2)) for x, y in zip(i, j)])
ctx.close()
