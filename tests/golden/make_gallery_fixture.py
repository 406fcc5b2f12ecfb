#!/usr/bin/env python3
"""Record the reference's own GPU output images as small fixtures.

gallery/gpu/image20.png, image21.png and image22.png in the reference are the
PNGs of archive-gpu/image20..22's P3 output: the five-sphere scene (hollow
glass shell of negative radius) at 1920x1080, 10 spp, depth 50, through
src/gpu's camera model from (-2, 2, 1) towards (0, 0, -1), fp32 write_color
(color.h), curand per pixel:
  image20  vfov 90, no defocus   (archive-gpu/image20/camera.h:49-58)
  image21  vfov 20, no defocus   (archive-gpu/image21/camera.h:49-58)
  image22  vfov 20, defocus 10 deg at focus 3.4 (archive-gpu/image22/camera.h:58-71)
Their scene is fixed (main.cu:24-38).  gallery/gpu/image23.png is src/gpu's
own final-scene run (1920x1080, 500 spp, main.cu:88 time seed); its seed was
recovered (tests/gallery_lib.py), so it can be re-rendered here too.

Stored as data, not as the PNG: the exact 8x8 block sums of the 8-bit levels
per channel (uint16, 135 x 240 x 3; 1080 and 1920 are multiples of 8), which
tests/test_reference_gpu.py compares with the product's GPU-model render.

Usage (build container only; needs /root/reference and PIL):
    python tests/golden/make_gallery_fixture.py
"""
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
CONFIGS = {
    "image20": "five-sphere scene 1920x1080 10spp depth 50, src/gpu camera from (-2, 2, 1) to (0, 0, -1), "
               "vfov 90, no defocus",
    "image21": "five-sphere scene 1920x1080 10spp depth 50, src/gpu camera from (-2, 2, 1) to (0, 0, -1), "
               "vfov 20, no defocus",
    "image22": "five-sphere scene 1920x1080 10spp depth 50, src/gpu camera from (-2, 2, 1) to (0, 0, -1), "
               "vfov 20, defocus 10 deg at focus 3.4",
    # src/gpu's own run: the final scene from time seed 1694284176 (tests/gallery_lib.py)
    "image23": "src/gpu final scene (seed 1694284176) 1920x1080 500spp depth 50, src/gpu camera from "
               "(13, 2, 3) to (0, 0, 0), vfov 20, defocus 0.6 at focus 10",
}


def main():
    for name, cam in CONFIGS.items():
        src = f"/root/reference/gallery/gpu/{name}.png"
        out = os.path.join(HERE, f"gallery_gpu_{name}_blocksum8.npz")
        img = np.asarray(Image.open(src).convert("RGB"), dtype=np.uint16)
        assert img.shape == (1080, 1920, 3), img.shape
        sums = img.reshape(135, 8, 240, 8, 3).sum(axis=(1, 3)).astype(np.uint16)
        np.savez_compressed(out, blocksum8=sums, source=np.array(f"gallery/gpu/{name}.png"),
                            config=np.array(f"{cam}, fp32 write_color"))
        print(out, sums.shape, "mean level", (sums.astype(np.float64) / 64).mean(axis=(0, 1)).round(3))


if __name__ == "__main__":
    main()
