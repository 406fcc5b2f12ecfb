#!/usr/bin/env python3
"""Host-side estimate of the layer walk's work for rectangular grid cells
(build container, no GPU): could cells longer along the camera's main
direction than across it cut the walk?  Traces a sample of the headline
camera's rays and one lambertian-like bounce each through the final scene
(numpy brute force), then walks each segment through layer grids of cell
sides (gx, gz) the way the kernel's DDA does (the layer slab clipped to the
segment's hit) and counts cells and item tests per segment.  The same count
for square cells, compared with the GPU's fixed-scale sweep
(profiles/r05h_fit_c2.log), says how far to trust it.

    python tools/grid_aniso_sim.py [--rays 20000]
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")]


def closest(o, d, C, R):
    """closest hit t (inf: none) and sphere index of unit rays o + t d"""
    n = o.shape[0]
    best_t = np.full(n, np.inf)
    best_i = np.full(n, -1)
    for k in range(0, C.shape[0], 64):
        c, r = C[k:k + 64], R[k:k + 64]
        oc = o[:, None, :] - c[None]
        b = (oc * d[:, None, :]).sum(-1)
        cc = (oc * oc).sum(-1) - r[None] ** 2
        disc = b * b - cc
        sq = np.sqrt(np.maximum(disc, 0))
        t0, t1 = -b - sq, -b + sq
        t = np.where(t0 > 1e-3, t0, np.where(t1 > 1e-3, t1, np.inf))
        t = np.where(disc >= 0, t, np.inf)
        j = t.argmin(1)
        tj = t[np.arange(n), j]
        upd = tj < best_t
        best_t = np.where(upd, tj, best_t)
        best_i = np.where(upd, k + j, best_i)
    return best_t, best_i


def segments(scene, cam, nrays, rng):
    C = np.stack([scene.cx, scene.cy, scene.cz], 1).astype(np.float64)
    R = np.abs(scene.radius.astype(np.float64))
    corner, horiz, vert, eye = (np.array(list(getattr(cam, f)), np.float64) for f in ("corner", "horiz", "vert", "eye"))
    s, t = rng.random(nrays), rng.random(nrays)
    d = corner[None] + s[:, None] * horiz[None] + t[:, None] * vert[None] - eye[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(eye[None], nrays, 0)
    th, ih = closest(o, d, C, R)
    segs = [(o, d, th)]
    hit = np.isfinite(th)
    p = o[hit] + th[hit, None] * d[hit]
    nrm = (p - C[ih[hit]]) / R[ih[hit], None]
    u = rng.normal(size=p.shape)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    d2 = nrm + u
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    t2, _ = closest(p, d2, C, R)
    segs.append((p, d2, t2))
    return segs


def walk_cost(segs, lay, gx, gz, phase=(0.0, 0.0)):
    """mean (cells, item tests) per segment for a grid of cell sides gx x gz"""
    cx, cz, reach, ylo, yhi = lay
    x0, x1 = (cx - reach).min(), (cx + reach).max()
    z0, z1 = (cz - reach).min(), (cz + reach).max()
    x0 -= phase[0] * gx
    z0 -= phase[1] * gz
    nx, nz = int(math.ceil((x1 - x0) / gx)), int(math.ceil((z1 - z0) / gz))
    cnt = np.zeros((nz, nx), np.int64)
    for a, b, r in zip(cx, cz, reach):
        i0, i1 = max(0, int((a - r - x0) // gx)), min(nx - 1, int((a + r - x0) // gx))
        j0, j1 = max(0, int((b - r - z0) // gz)), min(nz - 1, int((b + r - z0) // gz))
        cnt[j0:j1 + 1, i0:i1 + 1] += 1
    cells = items = n = 0
    for o, d, tmax in segs:
        n += o.shape[0]
        with np.errstate(divide="ignore", invalid="ignore"):
            ty0, ty1 = (ylo - o[:, 1]) / d[:, 1], (yhi - o[:, 1]) / d[:, 1]
        ta = np.maximum(np.minimum(ty0, ty1), 0.0)
        tb = np.minimum(np.maximum(ty0, ty1), tmax)
        for k in np.nonzero(ta <= tb)[0]:
            ox, oz, dx, dz = o[k, 0], o[k, 2], d[k, 0], d[k, 2]
            t0 = ta[k]
            # clip to the grid box
            for lo, hi, oo, dd in ((x0, x0 + nx * gx, ox, dx), (z0, z0 + nz * gz, oz, dz)):
                if dd == 0:
                    continue
                u0, u1 = (lo - oo) / dd, (hi - oo) / dd
                t0 = max(t0, min(u0, u1))
            tend = tb[k]
            for lo, hi, oo, dd in ((x0, x0 + nx * gx, ox, dx), (z0, z0 + nz * gz, oz, dz)):
                if dd != 0:
                    u0, u1 = (lo - oo) / dd, (hi - oo) / dd
                    tend = min(tend, max(u0, u1))
            if not t0 <= tend:
                continue
            i = min(nx - 1, max(0, int((ox + t0 * dx - x0) // gx)))
            j = min(nz - 1, max(0, int((oz + t0 * dz - z0) // gz)))
            sx, sz = (1 if dx > 0 else -1), (1 if dz > 0 else -1)
            tdx = gx / abs(dx) if dx != 0 else math.inf
            tdz = gz / abs(dz) if dz != 0 else math.inf
            tmx = ((x0 + (i + (sx > 0)) * gx) - ox) / dx if dx != 0 else math.inf
            tmz = ((z0 + (j + (sz > 0)) * gz) - oz) / dz if dz != 0 else math.inf
            while True:
                cells += 1
                items += cnt[j, i]
                if tmx < tmz:
                    if tmx > tend:
                        break
                    i += sx
                    tmx += tdx
                else:
                    if tmz > tend:
                        break
                    j += sz
                    tmz += tdz
                if not (0 <= i < nx and 0 <= j < nz):
                    break
    return cells / n, items / n


def main():
    import rtow
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=20000)
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=3840 / 2160)
    segs = segments(scene, cam, a.rays, rng)
    lay_m = (np.abs(scene.cy - 0.2) < 1e-6) & (np.abs(scene.radius - 0.2) < 1e-6)
    cx, cz = scene.cx[lay_m].astype(np.float64), scene.cz[lay_m].astype(np.float64)
    cn = np.sqrt(cx ** 2 + 0.04 + cz ** 2)
    reach = np.sqrt(0.04 + 2.0 ** -19 * (cn + 64.0) ** 2)
    lay = (cx, cz, reach, 0.2 - reach.max(), 0.2 + reach.max())
    g0 = math.sqrt((cx.max() - cx.min() + 0.5) * (cz.max() - cz.min() + 0.5) / lay_m.sum())
    out = []
    for scale in (1.0, 1.05, 1.11, 1.16, 1.22, 1.3):
        c, it = walk_cost(segs, lay, scale * g0, scale * g0)
        out.append({"scale": scale, "aspect": 1.0, "cells": round(c, 4), "items": round(it, 4)})
        print(json.dumps(out[-1]), flush=True)
    for scale in (1.0, 1.11, 1.22):
        for asp in (0.5, 0.7, 1.4, 2.0, 3.0):
            gx, gz = scale * g0 * math.sqrt(asp), scale * g0 / math.sqrt(asp)
            c, it = walk_cost(segs, lay, gx, gz)
            out.append({"scale": scale, "aspect": asp, "cells": round(c, 4), "items": round(it, 4)})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
