"""GPU vs the REFERENCE itself (P2) and the device arithmetic vs the
reference's known-answer vectors.

Statistical tests compare the product's image (HIP kernel through the C ABI,
tonemapped by the device write_color) with fixtures rendered by the
reference's own src/cpu (oracle/_ref/ref_harness, tests/golden/make_golden.py).
Per-pixel equality is impossible by construction (src/cpu draws one
sequential mt19937 stream for all pixels), so the bounds are
derived from the reference's own stream-to-stream noise, measured on a second
fixture of the same config with the stream shifted by 10^7 draws:

  * image-mean bias per channel <= max(4 sigma_mean, 0.05) levels, where
    sigma_mean = std(ref - ref_shift) / sqrt(N_pixels) is the standard error
    of the difference of two independent renders' means (north-star bound:
    1/255 = 1 level; at 100 spp this is ~0.05 levels);
  * 16x16 block-mean error <= 1.2 x the reference's own block floor;
  * segments (closest-hit queries) within 0.2 % of the reference's count.
"""
import json
import os

import numpy as np
import pytest

from oracle_lib import golden_kat, golden_ppm, golden_stats, kernel_render, read_ppm_bytes
from test_oracle import IMAGE22, block_means, blocks8, gallery_compare, image22_camera

pytestmark = pytest.mark.gpu

GRID = 1 << 9


def device_tonemap(rtow, ctx, sums, spp, mode=0):
    """rt_tonemap_async on a copy of `sums` in device memory, on a torch stream."""
    import torch
    dev = torch.device("cuda", ctx.device)
    t = torch.from_numpy(np.ascontiguousarray(sums, np.float32)).to(dev)
    out = torch.zeros(t.shape, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    ctx.tonemap_async(t.data_ptr(), t.numel() // 3, spp, out.data_ptr(), mode, stream.cuda_stream)
    stream.synchronize()
    return out.cpu().numpy()


def p2_compare(img, name):
    ref = read_ppm_bytes(golden_ppm(name))
    # the shifted-stream twin: ref_final_400x225x100 -> ref_final_shift_400x225x100
    parts = name.split("_")
    ref2 = read_ppm_bytes(golden_ppm("_".join(parts[:-1] + ["shift", parts[-1]])))
    a = img.reshape(-1, 3).astype(np.float64)
    r = ref.reshape(-1, 3).astype(np.float64)
    r2 = ref2.reshape(-1, 3).astype(np.float64)
    bias = a.mean(0) - r.mean(0)
    sigma_mean = (r - r2).std(0) / np.sqrt(r.shape[0])
    bias_bound = np.maximum(4 * sigma_mean, 0.05)
    blk = np.abs(block_means(img) - block_means(ref)).mean()
    floor = np.abs(block_means(ref2) - block_means(ref)).mean()
    report = {"bias": bias.round(4).tolist(), "bias_bound": bias_bound.round(4).tolist(),
              "block_err": round(float(blk), 4), "block_floor": round(float(floor), 4)}
    print(name, json.dumps(report))
    assert np.all(np.abs(bias) <= bias_bound), report
    assert blk <= 1.2 * floor, report
    return report


def test_final_scene_100spp_vs_reference(rtow, gpu_ctx):
    """The final scene at 400x225 and 100 spp (10x C0's samples: a systematic
    bias of a few tenths of a level in any material's distribution would show)."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    sums, st = gpu_ctx.render(cam, rtow.make_params(400, 225, 100, seed=12345, flags=GRID))
    img = device_tonemap(rtow, gpu_ctx, sums, 100)
    assert np.array_equal(img, rtow.tonemap(sums, 100))
    p2_compare(img, "ref_final_400x225x100")
    ref_segs = golden_stats()["ref_final_400x225x100"]["segments"]
    assert abs(st.segments / ref_segs - 1) < 0.002, (st.segments, ref_segs)


def test_ten_thousand_sphere_scene_vs_reference(rtow, gpu_ctx):
    """BASELINE C4's 10 000-sphere scene (rt_scene_final(50)) rendered by the
    reference's own classes from a dump of the same spheres, 160x90 @ 16 spp."""
    gpu_ctx.upload(rtow.final_scene(half_extent=50))
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    sums, st = gpu_ctx.render(cam, rtow.make_params(160, 90, 16, seed=777, flags=GRID))
    img = device_tonemap(rtow, gpu_ctx, sums, 16)
    p2_compare(img, "ref_tenk_160x90x16")
    # the reference's own two streams differ by 0.30 % (625 108 vs 623 244);
    # before the spurious-root rule fp32 self-hits on
    # spheres far from the origin trapped paths: +1.1 %
    stats = golden_stats()
    ref_segs = stats["ref_tenk_160x90x16"]["segments"]
    floor = abs(stats["ref_tenk_shift_160x90x16"]["segments"] / ref_segs - 1)
    assert abs(st.segments / ref_segs - 1) < 2 * floor, (st.segments, ref_segs)


def test_five_scene_depth_of_field_vs_reference(rtow, gpu_ctx):
    """archive-gpu/image22's depth of field on the five-sphere scene (hollow
    glass shell of negative radius): defocus 10 deg at focus 3.4, i.e. lens
    radius 3.4 tan 5 deg (aperture 0.5949) with the src/cpu camera."""
    import math
    gpu_ctx.upload(rtow.five_scene())
    cam = rtow.camera_cpu(lookfrom=(-2, 2, 1), lookat=(0, 0, -1), aspect=16.0 / 9.0,
                          aperture=2 * 3.4 * math.tan(math.radians(5.0)), focus_dist=3.4)
    assert cam.has_lens
    sums, st = gpu_ctx.render(cam, rtow.make_params(400, 225, 64, seed=99, flags=GRID))
    img = device_tonemap(rtow, gpu_ctx, sums, 64)
    p2_compare(img, "ref_five_dof_400x225x64")
    ref_segs = golden_stats()["ref_five_dof_400x225x64"]["segments"]
    assert abs(st.segments / ref_segs - 1) < 0.003, (st.segments, ref_segs)


@pytest.mark.parametrize("flags", [0, 3])
def test_five_scene_gpu_camera_defocus_bit_exact(rtow, gpu_ctx, oracle, flags):
    """image22's own camera model (src/gpu new_camera with defocus_angle 10,
    focus_dist 3.4) on the negative-radius scene: bit-exact vs the oracle."""
    scene = rtow.five_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_gpu(192, 108, lookfrom=(-2, 2, 1), lookat=(0, 0, -1), defocus_angle=10.0,
                          focus_dist=3.4)
    assert cam.has_lens
    p = rtow.make_params(192, 108, 24, seed=22, flags=flags | GRID)
    want, segs = kernel_render(scene, cam, p)
    got, st = gpu_ctx.render(cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs


@pytest.mark.parametrize("name", ["image20", "image21", "image22"])
def test_gpu_semantics_vs_reference_gpu_gallery(rtow, gpu_ctx, name):
    """The product with src/gpu's semantics (RT_FLAG_GPU_SEMANTICS, src/gpu
    camera, device fp32 write_color) against the reference CUDA path's own
    outputs, gallery/gpu/image20..22.png: the five-sphere scene at 1920x1080
    and 10 spp through three cameras (image22 with depth of field); two seeds
    for the noise floor (bounds in test_oracle.gallery_compare)."""
    gpu_ctx.upload(rtow.five_scene())
    cam = image22_camera(rtow, name)
    blk = []
    for seed in (1, 2):
        p = rtow.make_params(IMAGE22["width"], IMAGE22["height"], IMAGE22["spp"], seed=seed,
                             flags=GRID | rtow.RT_FLAG_GPU_SEMANTICS)
        sums, _ = gpu_ctx.render(cam, p)
        img = device_tonemap(rtow, gpu_ctx, sums, IMAGE22["spp"], rtow.RT_TONEMAP_GPU)
        blk.append(blocks8(img))
    print(name, gallery_compare(*blk, name=name))


def test_final_scene_gpu_semantics_vs_reference_gpu_gallery_image23(rtow, gpu_ctx):
    """The reference's own CUDA run of its final scene, gallery/gpu/image23.png
    (src/gpu: 1920x1080, 500 spp, depth 50, defocus 0.6 at focus 10), re-rendered
    by the product with src/gpu's semantics from the same scene: the run's time
    seed is recovered (tests/gallery_lib.py) and its XORWOW draws restated.
    Two seeds of ours give the noise floor.  Ours is 0.17-0.19 level brighter
    and the block error is 1.64x the floor (0.23 vs 0.14 level).  That
    difference is explained (profiles/r03_image23_attribution.log,
    tests/test_oracle.py::test_image23_brightness_is_src_gpu_fp32_hit_arithmetic):
    the oracle's restatement of src/gpu's own fp32 hit arithmetic (its
    quadratic on unnormalised directions, unrefined roots) renders the same
    rows within 0.008 level of the gallery and 1.03x its floor, and the
    specification is +0.169 / +0.176 / +0.200 level above that restatement,
    i.e. +0.164 / +0.169 / +0.192 above the gallery.  Bounds: the bias within
    0.03 level of that explained value per channel (seed noise ~0.003), block
    error <= 1.75x our seed-to-seed floor."""
    from gallery_lib import src_gpu_final_scene
    from test_oracle import gallery_blocks
    gpu_ctx.upload(src_gpu_final_scene(rtow))
    cam = rtow.camera_gpu(1920, 1080)  # src/gpu/camera.h:58-71 defaults
    blk = []
    for seed in (1, 2):
        p = rtow.make_params(1920, 1080, 500, seed=seed, flags=GRID | rtow.RT_FLAG_GPU_SEMANTICS)
        sums, _ = gpu_ctx.render(cam, p)
        blk.append(blocks8(device_tonemap(rtow, gpu_ctx, sums, 500, rtow.RT_TONEMAP_GPU)))
    a, b = blk
    g = gallery_blocks("image23")
    bias = a.reshape(-1, 3).mean(0) - g.reshape(-1, 3).mean(0)
    err, floor = float(np.abs(a - g).mean()), float(np.abs(a - b).mean())
    report = {"bias": bias.round(4).tolist(), "block_err": round(err, 4), "block_floor": round(floor, 4)}
    print("image23", report)
    explained = np.array([0.164, 0.169, 0.192])
    assert np.all(np.abs(bias - explained) <= 0.03), report
    assert err <= 1.75 * floor, report


# ------------------------------------------------------------ write_color --

@pytest.mark.parametrize("mode", [0, 1])
def test_device_tonemap_bit_exact_vs_host(rtow, gpu_ctx, mode):
    """rt_tonemap_async == rt_tonemap_u8_mode on random sums, on both sides of
    every level boundary, on 0 / NaN / inf, and on an unaligned tail."""
    from test_host import _level_edges
    rng = np.random.default_rng(mode)
    for spp in (1, 10, 100, 500, 2000):
        edges = _level_edges(spp, mode == 1)
        rnd = (rng.random((200003, 3)) * 1.05 * spp).astype(np.float32)
        sums = np.concatenate([edges, rnd])
        got = device_tonemap(rtow, gpu_ctx, sums, spp, mode)
        want = rtow.tonemap(sums, spp, mode)
        assert np.array_equal(got, want), (spp, int((got != want).sum()))


def test_device_tonemap_matches_write_color_kat(rtow, gpu_ctx):
    """The reference's own write_color output lines (kat.jsonl)."""
    for k in golden_kat():
        if k["kind"] != "write_color":
            continue
        sums = np.array([k["sum"]], np.float32)
        got = device_tonemap(rtow, gpu_ctx, sums, k["spp"], 0)
        assert " ".join(str(int(v)) for v in got[0]) == k["out"], k


def test_device_tonemap_at_level_boundaries(rtow, gpu_ctx):
    """The device write_color (rt_tonemap_async, src/cpu mode) on 703 fp32
    sums within a few ulps of the level thresholds: the reference's own
    write_color levels (tests/golden/make_color_kat.py), all in one launch
    per spp."""
    from oracle_lib import color_kat
    by_spp = {}
    for sums, spp, want in color_kat():
        by_spp.setdefault(spp, []).append((sums, want))
    for spp, rows in by_spp.items():
        sums = np.stack([r[0] for r in rows]).reshape(-1, 1, 3)
        got = device_tonemap(rtow, gpu_ctx, sums, spp, 0).reshape(-1, 3)
        assert np.array_equal(got, np.array([r[1] for r in rows])), spp


# ------------------------------------------------------- KAT: device math --

def _kat(kind):
    return [k for k in golden_kat() if k["kind"] == kind]


def test_device_sphere_hit_kat(rtow, gpu_ctx):
    """sphere::hit (src/cpu/sphere.h:24-51) through the kernel's own scan test,
    root choice, refine_root and set_face_normal, in fp32 on the device: the
    hit flag and face are exact; t, p and the normal within 2e-6 relative
    (fp32 rounding of the inputs and of a normalised direction)."""
    ks = _kat("sphere_hit")
    assert len(ks) == 8
    cases = [k["o"] + k["d"] + k["c"] + [k["r"]] for k in ks]
    out = rtow.device_kat(rtow.RT_KAT_SPHERE_HIT, cases)
    for k, o in zip(ks, out):
        assert bool(o[0]) == k["hit"], k
        if not k["hit"]:
            continue
        scale = 1.0 + np.abs(np.array(k["p"])).max()
        assert abs(o[1] - k["t"]) <= 2e-6 * max(1.0, abs(k["t"])) * scale, (k, o)
        assert np.allclose(o[2:5], k["p"], rtol=0, atol=2e-6 * scale), (k, o)
        assert np.allclose(o[5:8], k["normal"], rtol=0, atol=4e-6), (k, o)
        assert bool(o[8]) == k["front_face"], k


def test_device_reflect_refract_kat(rtow, gpu_ctx):
    """reflect / refract (src/cpu/vec3.h:122-131) as the kernel's reflect3 /
    refract3 compute them in fp32: within 1e-6 absolute of the fp64 vectors."""
    r = _kat("reflect")
    out = rtow.device_kat(rtow.RT_KAT_REFLECT, [k["v"] + k["n"] for k in r])
    for k, o in zip(r, out):
        assert np.allclose(o[:3], k["out"], rtol=0, atol=1e-6), (k, o)
    f = _kat("refract")
    assert len(f) == 6
    out = rtow.device_kat(rtow.RT_KAT_REFRACT, [k["v"] + k["n"] + [k["eta"]] for k in f])
    for k, o in zip(f, out):
        assert np.allclose(o[:3], k["out"], rtol=0, atol=1e-6), (k, o)


def test_device_reflectance_kat(rtow, gpu_ctx):
    """Schlick (src/cpu/material.h:82-87): within 1e-6 of the fp64 value for
    ref_idx 1.5 and 1/1.5 at cosines 0 .. 1."""
    r = _kat("reflectance")
    assert len(r) == 10
    out = rtow.device_kat(rtow.RT_KAT_REFLECTANCE, [[k["cosine"], k["ref_idx"]] for k in r])
    for k, o in zip(r, out):
        assert abs(o[0] - k["out"]) <= 1e-6, (k, o)


def _hit_cases():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "kat_hits.jsonl")) as f:
        return [json.loads(line) for line in f]


def _ambiguous(k):
    """True where an fp32 evaluation may legitimately differ from the
    reference's fp64 sphere::hit: a near-zero discriminant (grazing: hit flag
    and face undecided), or a root within fp32 reach of t_min (0.001 in units
    of the unnormalised direction, in the reference and, since round 5, in the
    kernel: normalize3 returns 0.001 |d|)."""
    o, d, c = (np.array(k[x], np.float64) for x in ("o", "d", "c"))
    r = float(k["r"])
    oc = o - c
    a, hb, cc = d @ d, oc @ d, oc @ oc - r * r
    disc = hb * hb - a * cc
    scale = hb * hb + abs(a * cc)
    if abs(disc) <= 1e-5 * scale:
        return True
    if disc < 0:
        return False
    L = np.sqrt(a)
    for t in ((-hb - np.sqrt(disc)) / a, (-hb + np.sqrt(disc)) / a):
        if abs(t - 0.001) * L <= 1e-4:  # distance along the ray from the t_min point
            return True
    return False


def test_device_sphere_hit_random_kat(rtow, gpu_ctx):
    """sphere::hit on 600 random rays and spheres (tests/golden/make_hit_kat.py:
    the reference's own sphere::hit through oracle/_ref/ref_harness): small,
    large, negative-radius and ground spheres; rays from outside, from the
    surface and from inside; unnormalised directions.  Outside the cases an
    fp32 evaluation cannot decide (_ambiguous), the kernel's device
    arithmetic agrees on hit and face exactly, and on the hit distance, the
    point and the normal to within fp32 precision of the inputs' scale."""
    ks = _hit_cases()
    assert len(ks) == 600
    out = rtow.device_kat(rtow.RT_KAT_SPHERE_HIT, [k["o"] + k["d"] + k["c"] + [k["r"]] for k in ks])
    checked = hits = 0
    worst = [0.0, 0.0, 0.0]
    for k, o in zip(ks, out):
        if _ambiguous(k):
            continue
        checked += 1
        assert bool(o[0]) == k["hit"], k
        if not k["hit"]:
            continue
        hits += 1
        assert bool(o[8]) == k["front_face"], k
        L = float(np.linalg.norm(k["d"]))
        scale = 1.0 + max(float(np.abs(k["o"]).max()), float(np.abs(k["c"]).max()) + abs(k["r"]))
        et = abs(o[1] - k["t"]) * L / scale              # distance error / scale
        ep = float(np.abs(np.array(o[2:5]) - k["p"]).max()) / scale
        en = float(np.abs(np.array(o[5:8]) - k["normal"]).max()) * abs(k["r"]) / scale
        worst = [max(worst[0], et), max(worst[1], ep), max(worst[2], en)]
    print("checked", checked, "hits", hits, "worst (t, p, normal*r) / scale", worst)
    # 585 of 600 decidable (584 with the round-4 world-unit t_min window)
    assert checked >= 585 and hits >= 250
    # measured: 4.7e-7, 3.1e-7, 3.2e-7 (profiles/r03ad_hit_kat.log)
    assert worst[0] <= 1e-6 and worst[1] <= 1e-6 and worst[2] <= 1e-6, worst


def test_device_reflect_refract_reflectance_random_kat(rtow, gpu_ctx):
    """reflect / refract / reflectance on 300 random cases each
    (tests/golden/make_vector_kat.py: the reference's own functions through
    the harness; incidence at every angle, refraction ratios 1/2.4 .. 2.4 short
    of total internal reflection) as the kernel's reflect3 / refract3 /
    schlick compute them in fp32 on the device."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "kat_vectors.jsonl")) as f:
        ks = [json.loads(line) for line in f]
    rf = [k for k in ks if k["kind"] == "reflect"]
    rr = [k for k in ks if k["kind"] == "refract"]
    sc = [k for k in ks if k["kind"] == "reflectance"]
    assert len(rf) == len(rr) == len(sc) == 300
    out = rtow.device_kat(rtow.RT_KAT_REFLECT, [k["v"] + k["n"] for k in rf])
    e_rf = max(float(np.abs(np.array(o[:3]) - k["out"]).max()) for k, o in zip(rf, out))
    out = rtow.device_kat(rtow.RT_KAT_REFRACT, [k["v"] + k["n"] + [k["eta"]] for k in rr])
    e_rr = max(float(np.abs(np.array(o[:3]) - k["out"]).max()) for k, o in zip(rr, out))
    out = rtow.device_kat(rtow.RT_KAT_REFLECTANCE, [[k["cosine"], k["ref_idx"]] for k in sc])
    e_sc = max(abs(o[0] - k["out"]) for k, o in zip(sc, out))
    print("worst reflect", e_rf, "refract", e_rr, "reflectance", e_sc)
    # measured: 1.5e-7, 4.5e-7, 1.7e-7 (profiles/r03ag_vector_kat.log)
    assert e_rf <= 1e-6 and e_rr <= 2e-6 and e_sc <= 1e-6, (e_rf, e_rr, e_sc)


@pytest.mark.parametrize("key", ["embed", "negop", "hot", "contact"])
def test_rule_and_albedo_fixtures_vs_reference(rtow, gpu_ctx, key):
    """The opaque-inside rule's reference fixtures (tests/fixture_scenes.py,
    src/cpu through ref_harness file:, 320x180 @ 256 spp): a glass sphere
    half-embedded in a lambertian sphere (not sealed: paths inside it go on
    and may leave through the glass) and lambertian / metal spheres of
    negative radius (lit, not black); "hot": albedos above 1 (64-bit pixel
    sums).  The product through the C ABI, two
    seeds, each bit-exact vs the oracle; P2 bounds in fixture_scenes.p2_check."""
    import fixture_scenes
    scene = fixture_scenes.FIXTURES[key](rtow)
    w, h, spp = fixture_scenes.FIXTURE_SIZE
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    gpu_ctx.upload(scene)
    sums, segs = [], []
    for seed in (1, 2):
        p = rtow.make_params(w, h, spp, seed=seed, flags=GRID)
        got, st = gpu_ctx.render(cam, p)
        want, n = kernel_render(scene, cam, p)
        assert np.array_equal(got, want) and st.segments == n, (seed, int((got != want).sum()))
        img = device_tonemap(rtow, gpu_ctx, got, spp)
        assert np.array_equal(img, rtow.tonemap(got, spp))
        sums.append(got)
        segs.append(st.segments)
    fixture_scenes.p2_check(rtow, key, sums, segs)


@pytest.mark.parametrize("scene_name", ["final", "contact", "five", "embed", "negop", "hot", "tenk"])
def test_converged_per_pixel_vs_reference(rtow, gpu_ctx, scene_name):
    """north_star's "per-channel PPM delta <= 1/255 vs src/cpu", pixel by pixel
    (VERDICT r5 item 1): the product at 128x72, 16 384 spp, depth 50 (the
    layer grid walk where the scene has a layer, and the device write_color;
    2 seeds) against the reference's own converged renders (3 independent
    src/cpu streams, tests/golden/make_converged_golden.py) of the final
    scene, the contact fixture, the five-sphere book scene (a hollow glass
    sphere), the embed / negop / hot fixtures and BASELINE C4's 10 001-sphere
    scene (at 2048 spp: the grid's cells-in-LDS placement).  The fraction of channels
    more than one level from a reference stream is at most max(1e-3, 1.5x)
    the reference's own stream-to-stream fraction; no channel lies more than
    one level from all of the other streams on one side more often than a
    reference stream does against its peers (tests/converged.py: no spatial
    cluster); image-mean bias within 0.05 level.  Measured: DESIGN.md 4."""
    import converged
    R = converged.refs(scene_name)
    W, H, spp = converged.size(scene_name)
    assert R.shape == (3, H, W, 3)
    scene, cam = converged.scene_and_camera(rtow, scene_name)
    gpu_ctx.upload(scene)
    for seed in (1, 2):
        sums, st = gpu_ctx.render(cam, rtow.make_params(W, H, spp, seed=seed, flags=GRID))
        img = rtow.tonemap(sums, spp)
        s = converged.compare(img, R)
        print(scene_name, seed, {k: v for k, v in s.items() if k != "channels"})
        converged.check(s)
