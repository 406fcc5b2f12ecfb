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
