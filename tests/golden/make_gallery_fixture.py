#!/usr/bin/env python3
"""Record the reference's own GPU output image as a small fixture.

gallery/gpu/image22.png in the reference is the PNG of archive-gpu/image22's
P3 output: the five-sphere scene (hollow glass shell of negative radius) at
1920x1080, 10 spp, depth 50, through src/gpu's camera model with defocus 10 deg
at focus 3.4 (archive-gpu/image22/camera.h:58-71), fp32 write_color
(color.h), curand per pixel.  It is the only output of the reference's CUDA
path that can be re-rendered here: its scene is fixed (main.cu:24-38), while
the final scene's gallery image is time-seeded.

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
SRC = "/root/reference/gallery/gpu/image22.png"
OUT = os.path.join(HERE, "gallery_gpu_image22_blocksum8.npz")


def main():
    img = np.asarray(Image.open(SRC).convert("RGB"), dtype=np.uint16)
    assert img.shape == (1080, 1920, 3), img.shape
    sums = img.reshape(135, 8, 240, 8, 3).sum(axis=(1, 3)).astype(np.uint16)
    np.savez_compressed(OUT, blocksum8=sums, source=np.array("gallery/gpu/image22.png"),
                        config=np.array("five-sphere scene 1920x1080 10spp depth 50, src/gpu camera "
                                        "defocus 10 deg focus 3.4, fp32 write_color"))
    print(OUT, sums.shape, "mean level", (sums.astype(np.float64) / 64).mean(axis=(0, 1)).round(3))


if __name__ == "__main__":
    main()
