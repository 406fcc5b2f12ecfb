#!/usr/bin/env python3
"""Wave-level cost of the layer-grid walk under two loop structures (host
model, build container).  The kernel's walk is per
lane, but a wave iterates over the union of its lanes: per DDA iteration the
item loop runs as many iterations as the busiest active lane has items in
its current cell (rt_kernel.hip grid_walk).  This asks whether fusing two
consecutive cells' item ranges into one item loop ("batch 2": the wave runs
max(n1 + n2) item iterations per two DDA steps instead of max(n1) + max(n2))
would cut the wave's iterations enough to pay for its extra loop control.

Waves are modelled the way the kernel fills them: the 64 lanes of a wave
hold paths of one 8x8 tile of the headline frame at mixed depths (the
sample pool): camera rays of the tile's pixels and the bounce segments of
those paths (lambertian-like bounces, tools/grid_aniso_sim.py's tracer), in
the depth mix the kernel's counters give (segments per sample 2.7).  Per
wave: the cell sequence of every lane's segment through the fitted grid
(scale 1.11) with each cell's item count, then the iterations under both
structures.

    python tools/wave_walk_sim.py [--waves 300]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"), os.path.join(ROOT, "tools")]

import grid_aniso_sim as gs  # noqa: E402


def grid(lay, g):
    cx, cz, reach, ylo, yhi = lay
    x0, x1 = (cx - reach).min(), (cx + reach).max()
    z0, z1 = (cz - reach).min(), (cz + reach).max()
    nx, nz = int(math.ceil((x1 - x0) / g)), int(math.ceil((z1 - z0) / g))
    cnt = np.zeros((nz, nx), np.int64)
    for a, b, r in zip(cx, cz, reach):
        i0, i1 = max(0, int((a - r - x0) // g)), min(nx - 1, int((a + r - x0) // g))
        j0, j1 = max(0, int((b - r - z0) // g)), min(nz - 1, int((b + r - z0) // g))
        cnt[j0:j1 + 1, i0:i1 + 1] += 1
    return x0, z0, nx, nz, g, cnt, ylo, yhi


def cells_of(o, d, tmax, G):
    """item counts of the cells the segment's layer part crosses, in order"""
    x0, z0, nx, nz, g, cnt, ylo, yhi = G
    if d[1] == 0:
        return []
    ty0, ty1 = (ylo - o[1]) / d[1], (yhi - o[1]) / d[1]
    ta, tb = max(min(ty0, ty1), 0.0), min(max(ty0, ty1), tmax)
    for lo, hi, oo, dd in ((x0, x0 + nx * g, o[0], d[0]), (z0, z0 + nz * g, o[2], d[2])):
        if dd != 0:
            u0, u1 = (lo - oo) / dd, (hi - oo) / dd
            ta, tb = max(ta, min(u0, u1)), min(tb, max(u0, u1))
    if not ta <= tb:
        return []
    ox, oz, dx, dz = o[0], o[2], d[0], d[2]
    i = min(nx - 1, max(0, int((ox + ta * dx - x0) // g)))
    j = min(nz - 1, max(0, int((oz + ta * dz - z0) // g)))
    sx, sz = (1 if dx > 0 else -1), (1 if dz > 0 else -1)
    tdx = g / abs(dx) if dx != 0 else math.inf
    tdz = g / abs(dz) if dz != 0 else math.inf
    tmx = ((x0 + (i + (sx > 0)) * g) - ox) / dx if dx != 0 else math.inf
    tmz = ((z0 + (j + (sz > 0)) * g) - oz) / dz if dz != 0 else math.inf
    out = []
    while 0 <= i < nx and 0 <= j < nz:
        out.append(int(cnt[j, i]))
        if tmx < tmz:
            if tmx > tb:
                break
            i += sx
            tmx += tdx
        else:
            if tmz > tb:
                break
            j += sz
            tmz += tdz
    return out


def wave_cost(lanes, batch):
    """(DDA iterations, item iterations) of one wave: lanes = per-lane lists of
    cell item counts; batch cells' items share one item loop"""
    rounds = max((len(c) + batch - 1) // batch for c in lanes) if lanes else 0
    dda = items = 0
    for r in range(rounds):
        act = [c[r * batch:(r + 1) * batch] for c in lanes if len(c) > r * batch]
        dda += 1
        items += max(sum(x) for x in act)
    return dda, items


def main():
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", type=int, default=300)
    a = ap.parse_args()
    rng = np.random.default_rng(11)
    scene = rtow.final_scene()
    W, H = 3840, 2160
    cam = rtow.camera_cpu(aspect=W / H)
    lay_m = (np.abs(scene.cy - 0.2) < 1e-6) & (np.abs(scene.radius - 0.2) < 1e-6)
    cx, cz = scene.cx[lay_m].astype(np.float64), scene.cz[lay_m].astype(np.float64)
    cn = np.sqrt(cx ** 2 + 0.04 + cz ** 2)
    reach = np.sqrt(0.04 + 2.0 ** -19 * (cn + 64.0) ** 2)
    lay = (cx, cz, reach, 0.2 - reach.max(), 0.2 + reach.max())
    g0 = math.sqrt((cx.max() - cx.min() + 0.5) * (cz.max() - cz.min() + 0.5) / lay_m.sum())
    G = grid(lay, 1.11 * g0)
    C = np.stack([scene.cx, scene.cy, scene.cz], 1).astype(np.float64)
    R = np.abs(scene.radius.astype(np.float64))
    corner, horiz, vert, eye = (np.array(list(getattr(cam, f)), np.float64) for f in ("corner", "horiz", "vert", "eye"))
    tot = {1: [0, 0], 2: [0, 0]}
    lane_cells = lane_items = nl = 0
    for w in range(a.waves):
        # a tile of 8x8 pixels; its paths: camera ray + 2 bounces, 64 paths
        tx, ty = rng.integers(0, W // 8), rng.integers(0, H // 8)
        s = (tx * 8 + rng.random(64) * 8) / (W - 1)
        t = (ty * 8 + rng.random(64) * 8) / (H - 1)
        d = corner[None] + s[:, None] * horiz[None] + t[:, None] * vert[None] - eye[None]
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        o = np.repeat(eye[None], 64, 0)
        segs = []
        for depth in range(3):
            th, ih = gs.closest(o, d, C, R)
            segs.append((o.copy(), d.copy(), th.copy()))
            hit = np.isfinite(th)
            if not hit.any():
                break
            p = o + np.where(hit, th, 0)[:, None] * d
            nrm = np.where(hit[:, None], (p - C[np.maximum(ih, 0)]) / R[np.maximum(ih, 0), None], 0)
            u = rng.normal(size=p.shape)
            u /= np.linalg.norm(u, axis=1, keepdims=True)
            d2 = nrm + u
            d2 /= np.maximum(np.linalg.norm(d2, axis=1, keepdims=True), 1e-12)
            o, d = p, np.where(hit[:, None], d2, d)
            # a lane whose path ended keeps a camera ray next (path regeneration)
        # a wave-step's 64 lanes: segments drawn across depths (live paths only)
        pool = [(so[k], sd[k], st[k]) for (so, sd, st) in segs for k in range(64)
                if (st[k] > 0) and (so is segs[0][0] or np.isfinite(segs[0][2][k]))]
        idx = rng.choice(len(pool), 64, replace=len(pool) < 64)
        lanes = [cells_of(*pool[k], G) for k in idx]
        for c in lanes:
            lane_cells += len(c)
            lane_items += sum(c)
            nl += 1
        for b in (1, 2):
            dd, it = wave_cost(lanes, b)
            tot[b][0] += dd
            tot[b][1] += it
    res = {"waves": a.waves, "lane_cells_per_segment": lane_cells / nl, "lane_items_per_segment": lane_items / nl}
    for b in (1, 2):
        res[f"batch{b}"] = {"dda_iters_per_wave": tot[b][0] / a.waves, "item_iters_per_wave": tot[b][1] / a.waves}
    # VALU per wave-step: DDA iteration 10 (batch 2: two steps, 20), item iteration 10 (batch 2: +2 range switch)
    v1 = 10 * tot[1][0] + 10 * tot[1][1]
    v2 = 20 * tot[2][0] + 12 * tot[2][1]
    res["valu_ratio_batch2_over_batch1"] = v2 / v1
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
