#!/usr/bin/env python3
"""Layer-grid cell visit histogram of one rank share (GPU box; tool only).

Needs the histogram build of the kernel (tools/build_variant.sh hist
build/variants/src_hist/rt_kernel.hip, which counts per cell the lane visits
and item tests into a device array, read back by rt_debug_cell_hist):

    RTOW_LIB=build/variants/hist.so python tools/cell_hist.py --preset c4 --world 8 --rank 0 --spp 16

Prints, for LDS item budgets of 256..8192 items, the share of all item tests
that fall into the hottest cells whose items fit the budget (cells taken by
item tests per item), and the grid's totals.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def main():
    import bench
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="c4")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--grid-mode", default="auto")
    ap.add_argument("--grid-scale", type=float, default=0.0)
    ap.add_argument("--save", default="", help="write the raw per-cell counts (npz) here")
    a = ap.parse_args()
    w, h, spp, half = bench.PRESETS[a.preset]
    L = rtow.lib()
    L.rt_debug_cell_hist.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    ctx = rtow.Context(0)
    scene = rtow.final_scene(half_extent=half)
    ctx.upload(scene, grid_mode=a.grid_mode, grid_scale=a.grid_scale)
    info = rtow.accel_info(scene, a.grid_mode, a.grid_scale)
    cam = rtow.camera_cpu(aspect=w / h)
    p = rtow.make_params(w, h, a.spp, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH, rank=a.rank, world=a.world)
    hist = np.zeros(1 << 17, np.uint32)
    assert L.rt_debug_cell_hist(None, 0, 1) == 0
    _, st = ctx.render(cam, p)
    assert L.rt_debug_cell_hist(hist.ctypes.data, hist.size, 0) == 0
    tests = hist[0::2].astype(np.float64)
    visits = hist[1::2].astype(np.float64)
    m = visits > 0
    items = np.zeros_like(tests)
    items[m] = np.round(tests[m] / visits[m])
    order = np.argsort(-(visits))  # item tests per item of a cell = its visits
    ctest = np.cumsum(tests[order])
    citem = np.cumsum(items[order])
    tot = ctest[-1]
    out = {"preset": a.preset, "rank": a.rank, "spp": a.spp, "segments": st.segments,
           "grid_items": info["grid_items"], "grid_cells": info["grid_nx"] * info["grid_nz"],
           "cells_visited": int(m.sum()), "items_in_visited_cells": int(items.sum()),
           "item_tests_per_segment": round(tot / st.segments, 4), "coverage": {}}
    for budget in (256, 470, 512, 1024, 1500, 2048, 3000, 4096, 8192):
        k = int(np.searchsorted(citem, budget, side="right"))
        out["coverage"][budget] = round(float(ctest[k - 1] / tot) if k else 0.0, 4)
    print(json.dumps(out), flush=True)
    if a.save:
        np.savez_compressed(a.save, tests=hist[0::2][:info["grid_nx"] * info["grid_nz"]],
                            visits=hist[1::2][:info["grid_nx"] * info["grid_nz"]],
                            nx=info["grid_nx"], nz=info["grid_nz"], segments=st.segments)


if __name__ == "__main__":
    main()
