"""Hand-built scenes for the opaque-inside rule's reference fixtures (test
infrastructure; tests/golden/make_golden.py renders them with the reference's
own src/cpu classes through ref_harness's file: mode, and the tests render them
with the oracle and the product).  The camera is ref_harness's file-scene
camera, i.e. rtow.camera_cpu()'s defaults: (13, 2, 3) -> (0, 0, 0), vfov 20,
aperture 0.1, focus 10.

embedded_glass: a glass sphere (r = 0.6) half-embedded in a lambertian sphere
    (r = 1) on the r = 1000 ground: the lambertian ball is overlapped, so
    paths that get inside it leave through the glass (Weak 1).
negative_opaque: a lambertian and a metal sphere of negative radius on the
    ground: set_face_normal flips their normals back to the geometric outward
    one (src/cpu/hittable.h:16-19), so they render lit.
hot: energy-creating albedos (lambertian 1.25 / 0.9 / 1.1 and metal 1.3 on the
    ground of albedo 1.05): the reference's constructors take any colour
    (src/cpu/material.h:17,38); the product switches to 64-bit pixel sums
    (VERDICT r3 item 5).
"""
import numpy as np

FIXTURE_SIZE = (320, 180, 256)  # width, height, spp of the reference fixtures


def _scene(rtow, rows):
    f32 = np.float32
    a = np.array([r[:5] for r in rows], np.float64)
    return rtow.Scene(a[:, 0].astype(f32), a[:, 1].astype(f32), a[:, 2].astype(f32), a[:, 3].astype(f32),
                      np.array([r[4] for r in rows], np.uint32),
                      np.array([r[5] for r in rows], f32), np.array([r[6] for r in rows], f32))


def embedded_glass_scene(rtow):
    # the glass centre lies on the lambertian sphere's surface, on its side facing the camera
    u = np.array([13.0, 1.0, 3.0])
    u /= np.linalg.norm(u)
    g = np.array([0.0, 1.0, 0.0]) + u
    return _scene(rtow, [
        (0.0, -1000.0, 0.0, 1000.0, 0, (0.5, 0.5, 0.5), 0.0),
        (0.0, 1.0, 0.0, 1.0, 0, (0.7, 0.6, 0.5), 0.0),
        (g[0], g[1], g[2], 0.6, 2, (1.0, 1.0, 1.0), 1.5),
    ])


def negative_opaque_scene(rtow):
    return _scene(rtow, [
        (0.0, -1000.0, 0.0, 1000.0, 0, (0.5, 0.5, 0.5), 0.0),
        (0.3, 0.7, -1.2, -0.7, 0, (0.8, 0.3, 0.2), 0.0),
        (0.6, 0.7, 1.2, -0.7, 1, (0.7, 0.7, 0.8), 0.2),
    ])


def hot_scene(rtow):
    return _scene(rtow, [
        (0.0, -1000.0, 0.0, 1000.0, 0, (1.05, 1.05, 1.05), 0.0),
        (0.0, 1.0, 0.0, 1.0, 0, (1.25, 0.9, 1.1), 0.0),
        (0.8, 0.5, 1.9, 0.5, 1, (1.3, 1.3, 1.3), 0.3),
        (1.2, 0.4, -1.6, 0.4, 2, (1.0, 1.0, 1.0), 1.5),
    ])


def _resting(x, z, r):
    """Centre of a sphere of radius r resting on the r = 1000 ground at (x, z):
    |C - (0, -1000, 0)| = 1000 + r (in fp64; the fp32 centre is within an ulp)."""
    return (x, -1000.0 + float(np.sqrt((1000.0 + r) ** 2 - x * x - z * z)), z)


def contact_scene(rtow):
    """Contacts, where the reference's t_min unit matters:
    small lambertian and metal spheres resting on the lambertian ground (r =
    0.05-0.3), two lambertian balls touching each other, and a lambertian ball
    touching a glass one, all in the view of the file-scene camera ((13, 2, 3)
    -> 0, 8.5 degrees above the ground).  A ray scattered off the ground next
    to a contact meets the other surface within a few t_min: the reference
    tests that root against 0.001 |d| (|d| = 2 cos theta for a lambertian
    bounce), the round-4 specification against 0.001 world units."""
    rows = [(0.0, -1000.0, 0.0, 1000.0, 0, (0.5, 0.5, 0.5), 0.0)]
    small = [(1.6, 0.9, 0.05, 0, (0.8, 0.3, 0.3), 0.0), (1.9, 0.5, 0.1, 0, (0.3, 0.8, 0.3), 0.0),
             (2.4, -0.2, 0.2, 0, (0.3, 0.3, 0.8), 0.0), (1.2, -1.1, 0.3, 0, (0.8, 0.8, 0.3), 0.0),
             (2.8, 1.3, 0.15, 1, (0.8, 0.8, 0.8), 0.0), (0.6, 1.6, 0.25, 1, (0.7, 0.6, 0.5), 0.4),
             (3.2, -1.0, 0.1, 1, (0.9, 0.9, 0.9), 0.1)]
    for x, z, r, kind, alb, param in small:
        rows.append(_resting(x, z, r) + (r, kind, alb, param))
    # two lambertian balls touching each other, both on the ground
    rows.append(_resting(-0.4, 1.4, 0.35) + (0.35, 0, (0.6, 0.5, 0.3), 0.0))
    rows.append(_resting(-0.4, 2.1, 0.35) + (0.35, 0, (0.3, 0.5, 0.6), 0.0))
    # a lambertian ball touching a glass ball
    rows.append(_resting(-0.6, -1.0, 0.5) + (0.5, 0, (0.7, 0.7, 0.7), 0.0))
    rows.append(_resting(-0.6, -2.0, 0.5) + (0.5, 2, (1.0, 1.0, 1.0), 1.5))
    return _scene(rtow, rows)


FIXTURES = {"embed": embedded_glass_scene, "negop": negative_opaque_scene, "hot": hot_scene,
            "contact": contact_scene}


# Segment counts: over 12 oracle seeds the relative deviation from the
# reference's count has a standard deviation of 1.7e-4 per render (embed) and
# 0.9e-4 (negop), and the reference's own count carries the same noise: the
# bound is 3 sigma of the difference of two independent renders.
SEG_BOUND = 3 * 2 ** 0.5 * 1.7e-4


def p2_check(rtow, key, sums, segs):
    """P2 of renders of fixture `key` (one per seed) against the
    reference's fixture and its stream-shifted twin: image-mean bias of the
    seeds' mean image within max(4 sigma_mean, 0.05) levels per channel, the
    seeds' mean 16x16 block error within 1.2x the reference's own floor, and
    every seed's segment count within SEG_BOUND of the reference's."""
    import json
    from oracle_lib import golden_ppm, golden_stats, read_ppm_bytes
    from test_oracle import block_means
    w, h, spp = FIXTURE_SIZE
    name, twin = "ref_%s_%dx%dx%d" % (key, w, h, spp), "ref_%s_shift_%dx%dx%d" % (key, w, h, spp)
    ref = read_ppm_bytes(golden_ppm(name)).reshape(h, w, 3)
    ref2 = read_ppm_bytes(golden_ppm(twin)).reshape(h, w, 3)
    imgs = [rtow.tonemap(s, spp).reshape(h, w, 3) for s in sums]
    r, r2 = ref.reshape(-1, 3).astype(np.float64), ref2.reshape(-1, 3).astype(np.float64)
    bias = np.mean([i.reshape(-1, 3).astype(np.float64).mean(0) for i in imgs], axis=0) - r.mean(0)
    bound = np.maximum(4 * (r - r2).std(0) / np.sqrt(r.shape[0]), 0.05)
    blk = float(np.mean([np.abs(block_means(i) - block_means(ref)).mean() for i in imgs]))
    floor = float(np.abs(block_means(ref2) - block_means(ref)).mean())
    ref_segs = golden_stats()[name]["segments"]
    dev = [s / ref_segs - 1 for s in segs]
    report = {"bias": bias.round(4).tolist(), "bias_bound": bound.round(4).tolist(), "block_err": round(blk, 4),
              "block_floor": round(floor, 4), "segments_dev": [round(d, 6) for d in dev]}
    print(name, json.dumps(report))
    assert np.all(np.abs(bias) <= bound), report
    assert blk <= 1.2 * floor, report
    assert all(abs(d) <= SEG_BOUND for d in dev), report
    return report
