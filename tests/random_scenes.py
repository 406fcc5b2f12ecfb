"""Seeded random sphere scenes for the parity tests (test infrastructure).

free_scene(seed): 1-39 spheres around the final scene's view (centres in
[-6, 6] x [-1, 4] x [-6, 6], radii 0.05-2), materials drawn at random --
lambertian albedos in [0, 1], metal fuzz in [0, 1.5] (the reference clamps
it to 1, material.h:38), indices of refraction 1.5 / 0.7 / 2.4 / 1/1.5 --
with some glass spheres given a negative-radius inner shell and, in half the
scenes, the r = 1000 ground.  Overlapping spheres are allowed.
"""
import numpy as np


def free_scene(rtow, seed):
    rng = np.random.default_rng(7000 + seed)
    f32 = np.float32
    n = int(rng.integers(1, 40))
    cx = rng.uniform(-6, 6, n)
    cy = rng.uniform(-1, 4, n)
    cz = rng.uniform(-6, 6, n)
    r = rng.uniform(0.05, 2.0, n)
    kind = rng.integers(0, 3, n)
    for i in range(min(n, 3)):  # nested glass shells
        if kind[i] == 2 and rng.uniform() < 0.5:
            cx, cy, cz = np.append(cx, cx[i]), np.append(cy, cy[i]), np.append(cz, cz[i])
            r, kind = np.append(r, -0.9 * r[i]), np.append(kind, 2)
    if rng.uniform() < 0.5:  # a ground
        cx, cy, cz = np.append(cx, 0.0), np.append(cy, -1000.0), np.append(cz, 0.0)
        r, kind = np.append(r, 1000.0), np.append(kind, 0)
    m = len(cx)
    albedo = rng.uniform(0, 1, (m, 3))
    param = np.where(kind == 1, rng.uniform(0, 1.5, m),
                     np.where(kind == 2, rng.choice([1.5, 0.7, 2.4, 1 / 1.5], m), 0.0))
    return rtow.Scene(cx.astype(f32), cy.astype(f32), cz.astype(f32), r.astype(f32),
                      kind.astype(np.uint32), albedo.astype(f32), param.astype(f32))


def ground_cut_spheres(scene):
    """Indices of the spheres whose surface crosses the r = 1000 ground's
    (fp64: 1000 - |r| < |C - G| < 1000 + |r|), [] without the ground.  Such a
    sphere and the ground enclose a cavity (inside the ball, above the
    ground) that the reference's paths enter through the crease more often
    than the fp32 kernel algorithm's ("ground-cut spheres")."""
    g = [i for i in range(scene.n) if float(scene.radius[i]) == 1000.0 and float(scene.cy[i]) == -1000.0]
    if not g:
        return []
    out = []
    for i in range(scene.n):
        if i == g[0]:
            continue
        d = np.sqrt(float(scene.cx[i]) ** 2 + (float(scene.cy[i]) + 1000.0) ** 2 + float(scene.cz[i]) ** 2)
        r = abs(float(scene.radius[i]))
        if 1000.0 - r < d < 1000.0 + r:
            out.append(i)
    return out


def dump_scene_exact(scene, path):
    """The scene in ref_harness's `file:` format, each float32 value printed
    as its exact double (%.17g), so the reference reads the same doubles the
    oracle converts the float32 arrays to."""
    kinds = "LMD"
    with open(path, "w") as f:
        for i in range(scene.n):
            a = scene.albedo[i]
            f.write("%s %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n" % (
                kinds[int(scene.kind[i])], float(scene.cx[i]), float(scene.cy[i]), float(scene.cz[i]),
                float(scene.radius[i]), float(a[0]), float(a[1]), float(a[2]), float(scene.param[i])))


# (width, spp, depth) per case: 16:9 frames, so height = int(width * 9 / 16)
CASES = [(48 + 8 * (k % 5), 2 + k % 7, (50, 5, 2, 12)[k % 4]) for k in range(24)]


def degenerate_scenes(rtow):
    """Inputs that stress the BVH / layer-grid builder: coincident spheres,
    spheres on a line, a crowded layer (no grid cell size keeps <= 15 per
    cell), huge and tiny radii, far-away spheres, and the layer-mode size
    thresholds.  name -> Scene."""
    f32 = np.float32
    rng = np.random.default_rng(99)

    def mk(cx, cy, cz, r, kind=None, param=None):
        n = len(cx)
        kind = np.zeros(n, np.uint32) if kind is None else np.asarray(kind, np.uint32)
        param = np.where(kind == 2, 1.5, 0.3) if param is None else param
        return rtow.Scene(np.asarray(cx, f32), np.asarray(cy, f32), np.asarray(cz, f32), np.asarray(r, f32),
                          kind, np.full((n, 3), 0.6, f32), np.asarray(param, f32))

    out = {
        "coincident_100": mk([0.5] * 100, [0.2] * 100, [0.5] * 100, [0.2] * 100),
        "line_200": mk(np.linspace(-8, 8, 200), [0.2] * 200, [0.0] * 200, [0.05] * 200),
        "crowded_layer_300": mk(rng.uniform(-0.5, 0.5, 300), [0.2] * 300, rng.uniform(-0.5, 0.5, 300), [0.2] * 300),
        "huge_and_tiny": mk([0, 3, -3, 1, 0], [-10000.5, 0.5, 0.5, 0.1, 1], [0, 1, -1, 2, -2],
                            [10000.0, 1e-3, 2e-3, 0.3, 0.5], kind=[0, 1, 2, 0, 2]),
        "far_away": mk([1e5, -1e5, 0, 3], [0, 0, 1e5, 0.5], [0, 0, 0, 0], [100, 50, 1e4, 0.5]),
    }
    base = rtow.final_scene()
    for n in (1, 2, 3, 63, 64, 65):
        idx = np.r_[0, 1 + np.arange(n - 1)] if n > 1 else np.array([0])
        idx = idx[idx < base.n]
        out["final_prefix_%d" % n] = rtow.Scene(base.cx[idx], base.cy[idx], base.cz[idx], base.radius[idx],
                                                base.kind[idx], base.albedo[idx], base.param[idx])
    return out
