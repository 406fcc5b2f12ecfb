"""The oracle (CPU restatement) pinned against the reference's own outputs.

Chain of evidence (DESIGN.md "Parity"):
  reference src/cpu  ==bytes==  oracle reference mode (fp64)        [this file]
  reference src/cpu  ~~stats~~  oracle kernel mode (fp32 algorithm)  [this file]
  reference CUDA     ~~stats~~  oracle kernel mode, GPU semantics    [this file: gallery image22]
  oracle kernel mode ==bits==   HIP kernel                           [test_parity_gpu.py]
"""
import hashlib
import os

import numpy as np
import pytest

from oracle_lib import (golden_ppm, golden_scene_rows, golden_stats, kernel_render, kernel_render_exact,
                        ppm_p3_bytes, read_ppm_bytes, reference_render, reference_render_view, reference_scene)

C0 = dict(width=400, aspect=16.0 / 9.0, spp=10)


def test_reference_scene_bit_exact_vs_reference_dump():
    rows, nxt = reference_scene(11)
    gold, gnxt = golden_scene_rows()
    assert rows.shape == gold.shape == (486, 9)
    # dielectric albedo is not a field of the reference class: dumped as 1,1,1
    assert np.array_equal(rows, gold)
    assert nxt == gnxt == 0.45473847890865138


def test_reference_mode_byte_identical_c0():
    """fp64 restatement == reference binary (src/cpu, g++ 11.4) byte for byte."""
    img, segs = reference_render(C0["width"], C0["aspect"], C0["spp"])
    st = golden_stats()["ref_c0_400x225x10"]
    data = ppm_p3_bytes(img)
    assert hashlib.sha256(data).hexdigest() == st["sha256"] == \
        "736ab8c692b16b9967223d6cc89a9a17f9f3741e2ce13ba8ade0ec3876574d22"
    assert data == golden_ppm("ref_c0_400x225x10")
    assert segs == st["segments"] == 2428989


@pytest.mark.slow
def test_reference_mode_byte_identical_five_scene():
    """Negative-radius hollow glass + metal + lambertian scene, 100 spp."""
    img, segs = reference_render(400, 16.0 / 9.0, 100, scene=1)
    st = golden_stats()["ref_five_400x225x100"]
    assert hashlib.sha256(ppm_p3_bytes(img)).hexdigest() == st["sha256"]
    assert segs == st["segments"]


@pytest.mark.parametrize("case", range(24))
def test_reference_mode_byte_identical_random_scenes(rtow, case):
    """fp64 restatement == the reference binary byte for byte (and segment for
    segment) on 24 seeded random scenes (tests/random_scenes.py: overlapping
    spheres, negative-radius glass shells, metal fuzz above 1, indices of
    refraction below 1, with and without the ground), 48-80 pixels wide, 2-8
    spp, depths 2-50.  Fixtures: tests/golden/make_random_ref_golden.py, which
    runs oracle/_ref/ref_harness (the reference's own src/cpu) on each scene."""
    import json
    import random_scenes
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_random_scenes.json")) as f:
        gold = json.load(f)[str(case)]
    w, spp, depth = random_scenes.CASES[case]
    assert (gold["width"], gold["spp"], gold["depth"]) == (w, spp, depth)
    scene = random_scenes.free_scene(rtow, case)
    assert scene.n == gold["spheres"]
    img, segs = reference_render_view(scene, w, 16.0 / 9.0, spp, depth)
    assert hashlib.sha256(ppm_p3_bytes(img)).hexdigest() == gold["sha256"]
    assert segs == gold["segments"]


def test_kernel_algorithm_matches_reference_random_scenes(rtow):
    """The fp32 kernel algorithm against the reference on the 24 random scenes
    at 96x54x64 (tests/random_scenes.py: overlapping and nested spheres,
    negative-radius glass shells, metal fuzz above 1, indices of refraction
    below 1, spheres cut by the ground), against the reference's own noise:
    its image means and segment counts from 24 independent streams (6 until
    round 5; tests/golden/make_random_noise_golden.py runs oracle/_ref/
    ref_harness, the reference's src/cpu) and 8 seeds of the kernel
    algorithm.  Every channel's bias is within 0.1 level (a tenth of
    north_star's 1/255) and 4 sigma of the two noises (round 6: worst 2.9
    sigma), and every scene's segment count within 4 sigma -- except that in
    the 8 scenes with a sphere cut by the ground the count may fall short by
    up to 3e-3: there the reference traps more paths in the cavity between
    the sphere and the ground, to the depth cap (measured and pinned by
    test_ground_cut_sphere_segment_deficit_is_depth_capped_paths; DESIGN.md
    4).  Round 4's single-render comparison put scene 12 at 0.21 level: the
    reference's own render-to-render noise there is 0.097 level.  This test
    also found round 3's unclamped metal fuzz above 1 (material.h:38):
    biases of up to -1.4 levels before the fix."""
    import json
    import random_scenes
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_random_scenes_means.json")) as f:
        gold = json.load(f)
    w, spp = 96, 64
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    worst = worst_z = worst_seg_z = 0.0
    for case in range(24):
        g = gold[str(case)]
        assert (g["width"], g["spp"], g["depth"]) == (w, spp, 50)
        ref = np.array(g["means"], np.float64)
        rseg = np.array(g["segments"], np.float64)
        assert len(ref) == len(rseg) == 24
        scene = random_scenes.free_scene(rtow, case)
        img, segs = [], []
        for seed in range(1, 9):
            sums, seg = kernel_render(scene, cam, rtow.make_params(w, int(w * 9 / 16), spp, seed=seed))
            img.append(rtow.tonemap(sums, spp).reshape(-1, 3).astype(np.float64).mean(0))
            segs.append(seg)
        img, segs = np.array(img), np.array(segs, np.float64)
        bias = img.mean(0) - ref.mean(0)
        sigma = np.sqrt(img.var(0, ddof=1) / len(img) + ref.var(0, ddof=1) / len(ref))
        worst = max(worst, float(np.abs(bias).max()))
        worst_z = max(worst_z, float(np.abs(bias / sigma).max()))
        assert np.abs(bias).max() <= 0.1, (case, bias)
        assert np.abs(bias / sigma).max() <= 4.0, (case, bias, sigma)
        rel = segs.mean() / rseg.mean() - 1.0
        z = (segs.mean() - rseg.mean()) / np.sqrt(segs.var(ddof=1) / len(segs) + rseg.var(ddof=1) / len(rseg))
        if random_scenes.ground_cut_spheres(scene):
            assert z <= 4.0 and rel >= -3e-3, (case, rel, z)
        else:
            worst_seg_z = max(worst_seg_z, abs(float(z)))
            assert abs(z) <= 4.0, (case, rel, z)
    print("worst bias %.4f level, worst %.2f sigma; segments (no ground-cut sphere) worst %.2f sigma"
          % (worst, worst_z, worst_seg_z))
    assert worst > 0.0


def test_ground_cut_sphere_segment_deficit_is_depth_capped_paths(rtow):
    """Why the kernel algorithm traces up to ~1.5e-3 fewer segments than the
    reference in scenes with spheres cut by the r = 1000 ground (VERDICT r5
    item 2; DESIGN.md 4, "ground-cut spheres"): such a sphere and the ground
    enclose a cavity (inside the ball, above the ground); a path that gets in
    through the crease bounces there until the depth cap, 50 segments, and
    returns black (src/cpu/main.cc:16-17).  The reference's fp64 arithmetic
    lets more paths in than the fp32 specification.  Pinned on random scene
    11 (8 ground-cut spheres) at 96x54x256 against the fp64 restatement of
    src/cpu (byte-identical to the reference; depth-capped paths counted by
    rto_reference_capped), with scene 15 (no ground-cut sphere) as control:
      * scene 15: the kernel algorithm's depth-capped paths equal the
        reference's within 3 Poisson sigma;
      * scene 11: the kernel algorithm ends significantly fewer paths at the
        cap (> 4 sigma; round 6: 975 vs 1 422 at 512 spp), 50 segments each,
        and that accounts for the segment deficit (deficit < 50 x the
        missing capped paths);
      * RTO_OPT_FP64_HIT (the winner's root, hit point and normal in fp64)
        moves the count halfway to the reference's: the fp32 hit point is
        the mechanism.  The image is the same either way (capped paths are
        black in both; test_kernel_algorithm_matches_reference_random_scenes)."""
    import ctypes
    import random_scenes
    from oracle_lib import RTO_OPT_FP64_HIT, _kernel_render_opts, lib, reference_render_view
    L = lib()
    L.rto_reference_capped.restype = ctypes.c_ulonglong
    L.rto_kernel_capped.restype = ctypes.c_ulonglong
    L.rto_kernel_capped.argtypes = [ctypes.c_int]
    w, h, spp = 96, 54, 256
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    got = {}
    for case in (11, 15):
        scene = random_scenes.free_scene(rtow, case)
        _, rseg = reference_render_view(scene, w, 16.0 / 9.0, spp)
        rcap = L.rto_reference_capped()
        row = {"ref": (rseg, rcap)}
        for name, opt in (("spec", 0), ("fp64_hit", RTO_OPT_FP64_HIT)):
            L.rto_kernel_capped(1)
            seg = sum(_kernel_render_opts(scene, cam, rtow.make_params(w, h, spp, seed=s), opt, False, 0)[2]
                      for s in (1, 2)) / 2.0
            row[name] = (seg, L.rto_kernel_capped(1) / 2.0)
        got[case] = row
        print(case, row)
    (rs, rc), (ks, kc), (_, hc) = got[15]["ref"], got[15]["spec"], got[15]["fp64_hit"]
    assert abs(kc - rc) <= 3.0 * np.sqrt(rc + kc / 2.0), got[15]
    (rs, rc), (ks, kc), (_, hc) = got[11]["ref"], got[11]["spec"], got[11]["fp64_hit"]
    assert rc - kc > 4.0 * np.sqrt(rc + kc / 2.0), got[11]
    assert 0.0 < rs - ks < 50.0 * (rc - kc), got[11]
    assert kc < hc < rc, got[11]


def test_kernel_algorithm_c0_bias_within_reference_stream_noise(rtow):
    """C0 (the final scene, 400x225, 10 spp, depth 50): the fp32 kernel
    algorithm against the reference's own noise, its image means and segment
    counts from 8 independent streams (tests/golden/make_c0_noise_golden.py
    runs oracle/_ref/ref_harness, src/cpu; stream 0 is the committed ref_c0
    PPM), with 16 seeds of the kernel algorithm.  VERDICT r4 Weak 1 read a
    blue bias of -0.10/255 off ONE reference render and one seed; against the
    streams (round 5) the bias is (+0.009, +0.006, +0.001) level
    at 16 seeds (sigma ~0.012), and segments +2.5e-4 (the reference's own
    render-to-render spread is 4.5e-4).  Bounds: every channel within 0.1
    level and 4 sigma, segments within 4 sigma."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_c0_streams.json")) as f:
        gold = json.load(f)
    w, h, spp = gold["width"], gold["height"], gold["spp"]
    ref0 = read_ppm_bytes(golden_ppm("ref_c0_400x225x10")).reshape(-1, 3).astype(np.float64).mean(0)
    assert np.allclose(ref0, gold["means"][0], atol=1e-5)  # stream 0 is the committed C0 render
    ref = np.array(gold["means"], np.float64)
    cam = rtow.camera_cpu(aspect=w / h)
    scene = rtow.final_scene()
    img, segs = [], []
    for seed in range(16):
        sums, seg = kernel_render(scene, cam, rtow.make_params(w, h, spp, seed=seed))
        img.append(rtow.tonemap(sums, spp).reshape(-1, 3).astype(np.float64).mean(0))
        segs.append(seg)
    img = np.array(img)
    bias = img.mean(0) - ref.mean(0)
    sigma = np.sqrt(img.var(0, ddof=1) / len(img) + ref.var(0, ddof=1) / len(ref))
    rs = np.array(gold["segments"], np.float64)
    seg_sigma = np.sqrt(np.var(segs, ddof=1) / len(segs) + rs.var(ddof=1) / len(rs))
    print("C0 bias", bias.round(4), "sigma", sigma.round(4), "segments", np.mean(segs) / rs.mean() - 1)
    assert np.abs(bias).max() <= 0.1, bias
    assert np.abs(bias / sigma).max() <= 4.0, (bias, sigma)
    assert abs(np.mean(segs) - rs.mean()) <= 4.0 * seg_sigma, (np.mean(segs), rs.mean(), seg_sigma)


def test_opaque_inside_rule_segments_attribution(rtow):
    """What the opaque-inside rule removes:
    the reference's own arithmetic (the fp64 restatement, byte-identical to
    src/cpu) traces 5.5e-5 of C0's segments after a path's first hit on the
    inside of a sealed lambertian sphere, and the rule drops about as many
    from the kernel algorithm (6.6e-5 at 16 seeds).  Before round 5's
    same-sphere exit rule it dropped 3.9e-4: fp32 hit points an ulp inside
    the ball a bounce starts from "entered" it.  Bounds (8 seeds): the
    reference's share below 1.5e-4, the kernel's drop between 1.5e-5 and
    1.5e-4, and without the same-sphere exit rule above 2.5e-4."""
    import ctypes
    from oracle_lib import RTO_OPT_NO_SAME_EXIT, RTO_OPT_NO_SEALED, _kernel_render_opts, lib
    L = lib()
    L.rto_reference_trapped.restype = ctypes.c_ulonglong
    _, ref_segs = reference_render(400, 16.0 / 9.0, 10)
    ref_share = L.rto_reference_trapped() / ref_segs
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=400 / 225)
    drop, drop_old = [], []
    for seed in range(8):
        p = rtow.make_params(400, 225, 10, seed=seed)
        run = lambda o: _kernel_render_opts(scene, cam, p, o, False, 0)[2]
        drop.append(run(RTO_OPT_NO_SEALED) - run(0))
        drop_old.append(run(RTO_OPT_NO_SEALED | RTO_OPT_NO_SAME_EXIT) - run(RTO_OPT_NO_SAME_EXIT))
    k_share, k_old = np.mean(drop) / ref_segs, np.mean(drop_old) / ref_segs
    print("reference trapped share %.2e, kernel rule drop %.2e (%.2e without the same-sphere exit rule)"
          % (ref_share, k_share, k_old))
    assert 0 < ref_share < 1.5e-4
    assert 1.5e-5 < k_share < 1.5e-4
    assert k_old > 2.5e-4


def test_metal_fuzz_above_one_is_clamped(rtow):
    """rt_scene_upload (and the oracle's kernel mode) clamp metal fuzz to 1 as
    the reference's metal constructors do (src/cpu/material.h:38,
    src/gpu/material.h:45): fuzz 3 renders exactly like fuzz 1."""
    import dataclasses
    base = rtow.final_scene()
    metal = np.flatnonzero(base.kind == rtow.RT_METAL)
    cam = rtow.camera_cpu(aspect=2.0)
    p = rtow.make_params(48, 24, 4, seed=3)
    imgs = []
    for f in (1.0, 3.0):
        param = base.param.copy()
        param[metal] = np.float32(f)
        sums, seg = kernel_render(dataclasses.replace(base, param=param), cam, p)
        imgs.append((sums, seg))
    assert np.array_equal(imgs[0][0], imgs[1][0]) and imgs[0][1] == imgs[1][1]


def _ks(x, cdf):
    """Kolmogorov-Smirnov distance of the sample x from the law `cdf`."""
    x = np.sort(np.asarray(x, np.float64))
    n = len(x)
    f = cdf(x)
    return max(float(np.max(np.arange(1, n + 1) / n - f)), float(np.max(f - np.arange(n) / n)))


def test_sampling_laws_match_the_reference_samplers():
    """The kernel replaces the reference's rejection samplers (vec3.h:96-118:
    random_in_unit_sphere, random_unit_vector, random_in_unit_disk) with
    closed-form draws from the counter RNG.  Same laws,
    checked on 400 000 draws each with Kolmogorov-Smirnov distances against
    the exact distributions (bound 0.004: p < 1e-5 at this n):
      unit vector: z uniform on [-1, 1], azimuth uniform, |v| = 1;
      ball point: radius CDF r^3 (uniform in the ball), direction uniform;
      disk point: r^2 uniform on [0, 1], angle uniform;
      lambertian direction (normal + unit vector, normalised): cos theta
      with CDF cos^2 (the cosine-weighted law of the reference's n +
      random_unit_vector)."""
    from oracle_lib import sample_probe
    n = 400_000
    u = sample_probe(0, n).astype(np.float64)
    assert np.abs(np.linalg.norm(u, axis=1) - 1).max() < 1e-6
    assert _ks(u[:, 2], lambda z: (z + 1) / 2) < 0.004
    assert _ks(np.arctan2(u[:, 1], u[:, 0]), lambda a: (a + np.pi) / (2 * np.pi)) < 0.004
    b = sample_probe(1, n).astype(np.float64)
    rho = np.linalg.norm(b, axis=1)
    assert rho.max() <= 1.0 and _ks(rho, lambda r: r ** 3) < 0.004
    assert _ks(b[:, 2] / np.maximum(rho, 1e-30), lambda z: (z + 1) / 2) < 0.004
    d = sample_probe(2, n).astype(np.float64)
    assert np.all(d[:, 2] == 0)
    r2 = d[:, 0] ** 2 + d[:, 1] ** 2
    assert r2.max() <= 1.0 and _ks(r2, lambda t: t) < 0.004
    assert _ks(np.arctan2(d[:, 1], d[:, 0]), lambda a: (a + np.pi) / (2 * np.pi)) < 0.004
    lam = sample_probe(3, n).astype(np.float64)
    assert np.abs(np.linalg.norm(lam, axis=1) - 1).max() < 1e-6
    assert lam[:, 2].min() >= -1e-6 and _ks(np.clip(lam[:, 2], 0, 1), lambda c: c ** 2) < 0.004


def block_means(img, b=16):
    h, w = img.shape[0] // b * b, img.shape[1] // b * b
    x = img[:h, :w].astype(np.float64)
    return x.reshape(h // b, b, w // b, b, 3).mean(axis=(1, 3))


def stat_compare(candidate_u8, ref_u8, ref2_u8):
    """image-mean bias and 16x16 block-mean error vs the reference's
    own stream-to-stream noise floor (ref vs ref2)."""
    bias = candidate_u8.reshape(-1, 3).astype(np.float64).mean(0) - \
        ref_u8.reshape(-1, 3).astype(np.float64).mean(0)
    blk = np.abs(block_means(candidate_u8) - block_means(ref_u8)).mean()
    floor = np.abs(block_means(ref2_u8) - block_means(ref_u8)).mean()
    return bias, blk, floor


def test_kernel_algorithm_statistically_matches_reference_c0(rtow):
    """The fp32 kernel algorithm (new RNG, closed-form sampling) renders the same
    image as src/cpu within the north-star tolerance (bias <= 1/255 / channel)."""
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    p = rtow.make_params(400, 225, 10, seed=0)
    sums, segs = kernel_render(scene, cam, p)
    img = rtow.tonemap(sums, 10)
    ref = read_ppm_bytes(golden_ppm("ref_c0_400x225x10"))
    ref2 = read_ppm_bytes(golden_ppm("ref_c0_shift_400x225x10"))
    bias, blk, floor = stat_compare(img, ref, ref2)
    assert np.all(np.abs(bias) <= 1.0), bias
    assert blk <= 1.5 * floor, (blk, floor)
    # same amount of work as the reference (segments/sample within 2 %)
    # (fp64 restatement of the same algorithm: -0.01 %; the winner-root refinement
    # removes the fp32 self-intersection excess, DESIGN.md "Kernel algorithm")
    assert abs(segs / golden_stats()["ref_c0_400x225x10"]["segments"] - 1) < 0.003


def test_kernel_algorithm_statistically_matches_reference_five_scene(rtow):
    scene = rtow.five_scene()
    cam = rtow.camera_cpu(lookfrom=(-2, 2, 1), lookat=(0, 0, -1), aspect=16.0 / 9.0,
                          aperture=0.0, focus_dist=3.4)
    p = rtow.make_params(400, 225, 100, seed=0)
    sums, _ = kernel_render(scene, cam, p)
    img = rtow.tonemap(sums, 100)
    ref = read_ppm_bytes(golden_ppm("ref_five_400x225x100"))
    bias = img.reshape(-1, 3).mean(0) - ref.reshape(-1, 3).astype(np.float64).mean(0)
    assert np.all(np.abs(bias) <= 1.0), bias
    blk = np.abs(block_means(img) - block_means(ref)).mean()
    assert blk < 1.5, blk


@pytest.mark.slow
def test_kernel_algorithm_matches_reference_ten_thousand_spheres(rtow):
    """BASELINE C4's 10 000-sphere scene (coordinates up to 50): the fp32 kernel
    algorithm does the reference's amount of work.  Without the spurious-root
    rule the expanded quadratic's fp32 roots on spheres
    far from the origin trapped paths inside them: +1.1 % segments, 119 paths
    at the depth cap instead of 15 (profiles/r02_spurious_root.log)."""
    scene = rtow.final_scene(half_extent=50)
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    sums, segs = kernel_render(scene, cam, rtow.make_params(160, 90, 16, seed=777))
    st = golden_stats()
    ref_segs = st["ref_tenk_160x90x16"]["segments"]
    floor = abs(st["ref_tenk_shift_160x90x16"]["segments"] / ref_segs - 1)  # 0.30 %
    assert abs(segs / ref_segs - 1) < 2 * floor, (segs, ref_segs)
    img = rtow.tonemap(sums, 16)
    ref = read_ppm_bytes(golden_ppm("ref_tenk_160x90x16"))
    ref2 = read_ppm_bytes(golden_ppm("ref_tenk_shift_160x90x16"))
    bias, blk, floor_blk = stat_compare(img, ref, ref2)
    assert np.all(np.abs(bias) <= 1.0), bias
    assert blk <= 1.2 * floor_blk, (blk, floor_blk)


def test_kernel_mode_partition_invariant(rtow):
    """RNG keyed by the global pixel: interleaved row bands over any rank count
    reassemble to the identical image."""
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=64 / 37)
    full, segs = kernel_render(scene, cam, rtow.make_params(64, 37, 3, seed=7))
    for world in (2, 3):
        got = np.zeros_like(full)
        total = 0
        for rank in range(world):
            p = rtow.make_params(64, 37, 3, seed=7, rank=rank, world=world, row_block=4)
            tile, s = kernel_render(scene, cam, p)
            rows = rtow.local_to_global_rows(p)
            keep = rows < 37
            got[rows[keep]] = tile[keep]
            assert np.all(tile[~keep] == 0)
            total += s
        assert np.array_equal(got, full)
        assert total == segs


def test_kernel_mode_seed_changes_image(rtow):
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=2.0)
    a, _ = kernel_render(scene, cam, rtow.make_params(32, 16, 2, seed=1))
    b, _ = kernel_render(scene, cam, rtow.make_params(32, 16, 2, seed=2))
    c, _ = kernel_render(scene, cam, rtow.make_params(32, 16, 2, seed=1))
    assert not np.array_equal(a, b)
    assert np.array_equal(a, c)


def test_kernel_mode_depth_zero_and_spp_zero(rtow):
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=2.0)
    z, s = kernel_render(scene, cam, rtow.make_params(16, 8, 4, max_depth=0))
    assert not z.any() and s == 0
    z, s = kernel_render(scene, cam, rtow.make_params(16, 8, 0))
    assert not z.any() and s == 0


# ------------------------------------------- the reference's own GPU output --

IMAGE22 = dict(width=1920, height=1080, spp=10)
# archive-gpu/imageN/camera.h: vfov, defocus angle (image20/21 have no lens:
# focal length |lookfrom - lookat| = sqrt(12), which scales the viewport only)
GALLERY = {"image20": (90.0, 0.0, 12 ** 0.5), "image21": (20.0, 0.0, 12 ** 0.5), "image22": (20.0, 10.0, 3.4)}


def image22_camera(rtow, name="image22"):
    """archive-gpu/image20..22/camera.h: src/gpu's camera model, lookfrom
    (-2, 2, 1), lookat (0, 0, -1); image22: vfov 20, defocus 10 deg at focus
    3.4 (camera.h:58-71)."""
    vfov, defocus, focus = GALLERY[name]
    return rtow.camera_gpu(IMAGE22["width"], IMAGE22["height"], lookfrom=(-2, 2, 1), lookat=(0, 0, -1),
                           vfov=vfov, defocus_angle=defocus, focus_dist=focus)


def gallery_blocks(name):
    """8x8 block means of gallery/gpu/<name>.png (tests/golden/make_gallery_fixture.py)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"gallery_gpu_{name}_blocksum8.npz")
    return np.load(path)["blocksum8"].astype(np.float64) / 64.0


def blocks8(img_u8):
    h, w = IMAGE22["height"], IMAGE22["width"]
    return img_u8.reshape(h // 8, 8, w // 8, 8, 3).astype(np.float64).mean(axis=(1, 3))


def gallery_compare(a, b, name="image22"):
    """Two renders of ours (block means a, b: different seeds) against the
    reference CUDA path's image (one curand stream per pixel, its own seed).
    Bounds: 8x8 block-mean error <= 1.1 x our own seed-to-seed floor, and
    image-mean bias per channel <= max(4 sigma, 0.1 level).  The reference's
    image22 is ~0.05 level darker in red and green than ours (5 sigma at 2 M
    pixels), from its fp32 hit arithmetic (attributed on image23);
    0.1 level is a tenth of north_star's 1/255."""
    g = gallery_blocks(name)
    n = a.shape[0] * a.shape[1]
    sigma = (a - b).reshape(-1, 3).std(0) / np.sqrt(n)
    bias = a.reshape(-1, 3).mean(0) - g.reshape(-1, 3).mean(0)
    err = float(np.abs(a - g).mean())
    floor = float(np.abs(a - b).mean())
    report = {"bias": bias.round(4).tolist(), "bias_bound": np.maximum(4 * sigma, 0.1).round(4).tolist(),
              "block_err": round(err, 4), "block_floor": round(floor, 4)}
    assert np.all(np.abs(bias) <= np.maximum(4 * sigma, 0.1)), report
    assert err <= 1.1 * floor, report
    return report


@pytest.mark.parametrize("name", sorted(GALLERY))
def test_kernel_gpu_semantics_matches_reference_gpu_gallery(rtow, name):
    """The oracle's kernel mode with src/gpu's semantics (open interval, fuzz x
    unit vector, src/gpu camera, fp32 write_color) against the outputs of the
    reference's CUDA path that are reproducible: gallery/gpu/image20..22.png,
    the five-sphere scene at 1920x1080 and 10 spp, three cameras (parity for
    the gpu_ray_tracer personality)."""
    scene = rtow.five_scene()
    cam = image22_camera(rtow, name)
    blk = []
    for seed in (1, 2):
        p = rtow.make_params(IMAGE22["width"], IMAGE22["height"], IMAGE22["spp"], seed=seed,
                             flags=rtow.RT_FLAG_GPU_SEMANTICS)
        sums, _ = kernel_render(scene, cam, p, threads=8)
        blk.append(blocks8(rtow.tonemap(sums, IMAGE22["spp"], rtow.RT_TONEMAP_GPU)))
    print(name, gallery_compare(*blk, name=name))


def test_src_gpu_scene_of_the_gallery_run(rtow):
    """tests/gallery_lib.py's restatement of src/gpu's new_world (curand XORWOW,
    the gallery run's recovered seed): 486 spheres, 373 lambertian / 84 metal /
    29 dielectric, pinned by a fingerprint of the fp32 arrays (the GPU test
    against gallery/gpu/image23.png renders exactly this scene)."""
    from gallery_lib import IMAGE23_SEED, Xorwow, src_gpu_final_scene
    s = src_gpu_final_scene(rtow)
    h = hashlib.sha256()
    for a in (s.cx, s.cy, s.cz, s.radius, s.kind, s.albedo, s.param):
        h.update(np.ascontiguousarray(a).tobytes())
    assert IMAGE23_SEED == 1694284176
    assert s.n == 486 and np.bincount(s.kind).tolist() == [373, 84, 29]
    assert h.hexdigest()[:16] == "f8b097d4cf72df1a"
    assert rtow.accel_info(s)["layer_mode"] == 1
    # curand_uniform lies in (0, 1], so random_float = 1 - it in [0, 1)
    r = Xorwow(0)
    u = [r.random_float() for _ in range(10000)]
    assert min(u) >= 0.0 and max(u) < 1.0


def _levels(sums, spp):
    """write_color's level before the int() (src/cpu/color.h:8-23), as a real number."""
    return 256.0 * np.sqrt(np.clip(sums / spp, 0.0, None))


@pytest.mark.parametrize("spp", [1 << 12, 1 << 20])
def test_sum_format_unbiased_at_high_spp(rtow, spp):
    """The fixed-point pixel sums against an fp64 sum of
    the same samples (the reference's accumulation, src/cpu/main.cc:114-119)
    at 4096 and 2^20 spp, where F = 19 and 11: with the stochastic rounding
    every pixel's level is within 0.05 of the fp64 one (unbiased; the rounding
    noise is ~1e-6 level), while plain truncation (the round-2 format) loses
    up to 2^-F per sample and its darkest pixels drift by more than the bound
    at 2^20 spp.  The five-sphere book scene (archive-gpu/image22) with its
    albedos darkened 10x, 8x2 pixels over its darkest rows, keeps the sample
    count CPU-sized."""
    scene = rtow.five_scene()
    scene.albedo = (scene.albedo * 0.1).astype(np.float32)
    cam = rtow.camera_gpu(8, 4, lookfrom=(-2, 2, 1), lookat=(0, 0, -1), vfov=90.0, defocus_angle=0.0,
                          focus_dist=3.4)
    p = rtow.make_params(8, 4, spp, seed=7, flags=rtow.RT_FLAG_GPU_SEMANTICS)
    p.local_rows = 2  # the two bottom rows are the darkest (under the spheres)
    p.row_block = 2
    p.band_stride = 2
    p.band_offset = 1
    got, exact, _ = kernel_render_exact(scene, cam, p)
    lv_got, lv_ex = _levels(got.astype(np.float64), spp), _levels(exact, spp)
    assert np.all(np.abs(lv_got - lv_ex) <= 0.05), np.abs(lv_got - lv_ex).max()
    assert abs(float((lv_got - lv_ex).mean())) <= 0.01
    trunc, exact2, _ = kernel_render_exact(scene, cam, p, no_dither=True)
    assert np.array_equal(exact, exact2)  # the same samples
    drift = lv_ex - _levels(trunc.astype(np.float64), spp)
    assert np.all(drift >= 0)  # truncation only ever loses
    if spp == 1 << 20:
        assert drift.max() > 0.05


def test_image23_brightness_is_src_gpu_fp32_hit_arithmetic(rtow):
    """the kernel specification in GPU semantics renders the
    reference's own CUDA run of its final scene (gallery/gpu/image23.png)
    0.17-0.20 level brighter.  The oracle's restatement of src/gpu's own
    per-sample arithmetic (rto_gpuref_render, GREF_NAIVE_HIT | GREF_UNNORM:
    sphere::hit's quadratic on unnormalised directions, unrefined roots,
    set_face_normal by dot(d, outward)) removes it: on five 8-row bands of the
    gallery frame at its 500 spp, its image-mean bias is within 0.05 level
    and its 8x8 block error within 1.15x its own seed-to-seed floor, while the
    specification stays 0.12-0.25 level brighter than the restatement
    (profiles/r03_image23_attribution.log: 34 bands, spec +0.165 / +0.173 /
    +0.193, restatement -0.005 / -0.007 / -0.008, block error 0.144 vs floor
    0.139; +8.4 % segments -- the extra self-intersections that darken
    src/gpu's image)."""
    import ctypes
    from gallery_lib import src_gpu_final_scene
    from oracle_lib import lib
    L = lib()
    L.rto_gpuref_render.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p,
                                                             ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    scene = src_gpu_final_scene(rtow)
    cam = rtow.camera_gpu(1920, 1080)
    W, H, spp, stride = 1920, 1080, 500, 27
    g = gallery_blocks("image23")

    def render(seed, mode):
        p = rtow.make_params(W, H, spp, seed=seed, flags=rtow.RT_FLAG_GPU_SEMANTICS, rank=0, world=stride)
        if mode is None:
            out, _ = kernel_render(scene, cam, p)
        else:
            v = scene.view()
            out = np.zeros((p.local_rows, W, 3), np.float32)
            seg = ctypes.c_ulonglong()
            assert L.rto_gpuref_render(ctypes.addressof(v), ctypes.addressof(cam), ctypes.addressof(p), mode,
                                       out.ctypes.data, ctypes.byref(seg), 0) == 0
        rows = rtow.local_to_global_rows(p)
        keep = rows < H
        img = rtow.tonemap(out[keep], spp, rtow.RT_TONEMAP_GPU).astype(np.float64)
        return img.reshape(-1, 8, W // 8, 8, 3).mean(axis=(1, 3)), g[rows[keep][::8] // 8]

    gref = 1 | 2  # GREF_NAIVE_HIT | GREF_UNNORM
    a, gb = render(1, gref)
    b, _ = render(2, gref)
    spec, _ = render(1, None)
    bias = a.reshape(-1, 3).mean(0) - gb.reshape(-1, 3).mean(0)
    err, floor = float(np.abs(a - gb).mean()), float(np.abs(a - b).mean())
    explained = spec.reshape(-1, 3).mean(0) - a.reshape(-1, 3).mean(0)
    report = {"bias": bias.round(4).tolist(), "err": round(err, 4), "floor": round(floor, 4),
              "spec_minus_restatement": explained.round(4).tolist()}
    print("image23 restatement", report)
    assert np.all(np.abs(bias) <= 0.05), report
    assert err <= 1.15 * floor, report
    assert np.all((explained >= 0.12) & (explained <= 0.25)), report


@pytest.mark.parametrize("key", ["embed", "negop", "hot", "contact"])
def test_rule_and_albedo_fixtures_vs_reference(rtow, key):
    """The opaque-inside rule against the reference's own
    src/cpu on the rule's fixtures (tests/fixture_scenes.py, 320x180 @ 256
    spp, two seeds): a glass sphere half-embedded in a lambertian sphere --
    the lambertian ball is overlapped, so the rule does not apply and paths
    inside it go on as in the reference -- and lambertian / metal spheres of
    negative radius, which the round-3 rule (keyed on the face, not the root)
    rendered black: bias -12.7 levels, 10.6 % fewer segments.  "hot": albedos
    above 1 (64-bit pixel sums, radiance clamp)."""
    import fixture_scenes
    scene = fixture_scenes.FIXTURES[key](rtow)
    w, h, spp = fixture_scenes.FIXTURE_SIZE
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    runs = [kernel_render(scene, cam, rtow.make_params(w, h, spp, seed=seed)) for seed in (1, 2)]
    fixture_scenes.p2_check(rtow, key, [s for s, _ in runs], [n for _, n in runs])


def test_tmin_in_ray_parameter_units_contact_fixture(rtow):
    """t_min is 0.001 in units of the ray's unnormalised direction, as the
    reference tests its roots (src/cpu/main.cc:19, sphere.h:37-41; src/gpu
    camera.h:117), and the exiting root of the sphere a ray starts on, moving
    away from its centre, is an fp32 artefact (round 5's specification,
    DESIGN.md 2 steps 3-4).  On the contact fixture (spheres resting on the
    ground and touching each other, tests/fixture_scenes.py), against the
    reference's segment counts from 8 independent streams (tests/golden/
    make_contact_noise_golden.py; per-render spread 9e-5), with the
    opaque-inside rule off (it only shortens paths the reference traces to
    the depth cap, black either way): over the 4 seeds this test runs, the
    specification matches the reference (-3.7e-5, -0.8 sigma; DESIGN.md 4's
    8-seed run: -2.2e-5, -0.5 sigma); the round-4 t_min unit (0.001 world
    units on the normalised ray) loses 1.83e-4 of the segments (paired);
    without the same-sphere exit rule the kernel traces 4.5e-4 too many (fake
    entries into balls it starts on; 4.7e-4 over 8 seeds)."""
    import json
    import fixture_scenes
    from oracle_lib import RTO_OPT_NO_SAME_EXIT, RTO_OPT_NO_SEALED, RTO_OPT_TMIN_WORLD, _kernel_render_opts
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_contact_streams.json")) as f:
        gold = json.load(f)
    rs = np.array(gold["segments"], np.float64)
    scene = fixture_scenes.contact_scene(rtow)
    w, h, spp = fixture_scenes.FIXTURE_SIZE
    assert (gold["width"], gold["spp"]) == (w, spp)
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    segs = {"spec": [], "world": [], "no_same_exit": []}
    opts = {"spec": RTO_OPT_NO_SEALED, "world": RTO_OPT_NO_SEALED | RTO_OPT_TMIN_WORLD,
            "no_same_exit": RTO_OPT_NO_SEALED | RTO_OPT_NO_SAME_EXIT}
    for seed in (1, 2, 3, 4):
        p = rtow.make_params(w, h, spp, seed=seed)
        for k in segs:
            segs[k].append(_kernel_render_opts(scene, cam, p, opts[k], False, 0)[2])
    sp = np.array(segs["spec"], np.float64)
    sigma = np.sqrt(sp.var(ddof=1) / len(sp) + rs.var(ddof=1) / len(rs))
    z = (sp.mean() - rs.mean()) / sigma
    paired_world = (sp - np.array(segs["world"])).mean() / rs.mean()
    excess_old = np.mean(segs["no_same_exit"]) / rs.mean() - 1
    print("spec vs reference %+.2e (%.1f sigma); ray - world units %+.2e; without the same-sphere exit rule %+.2e"
          % (sp.mean() / rs.mean() - 1, z, paired_world, excess_old))
    assert abs(z) <= 3.0, z
    assert paired_world >= 1.0e-4, paired_world
    assert excess_old >= 3.0e-4, excess_old




@pytest.mark.parametrize("scene_name", ["contact", "five", "final", "tenk"])
def test_converged_per_pixel_vs_reference(rtow, scene_name):
    """north_star's per-channel <= 1/255 bound, pixel by pixel, for the fp32
    kernel algorithm (the specification the HIP kernel matches bit for bit;
    VERDICT r5 item 1): at 128x72, 16 384 spp against the reference's 3
    converged src/cpu streams (tests/golden/make_converged_golden.py; bounds
    in tests/converged.py).  The contact fixture and the five-sphere scene
    render whole (~10 s each on 8 cores); the final scene and BASELINE C4's
    10 001-sphere scene (at 2048 spp: the reference scans every sphere) render
    an 8-row band through the frame's middle (rows 32-39: spheres, their
    contact shadows and the horizon), the band a 9-way interleaved split of
    the frame gives rank 4.  The GPU renders all seven converged scenes whole
    (test_reference_gpu.py)."""
    import converged
    R = converged.refs(scene_name)
    W, H, spp = converged.size(scene_name)
    scene, cam = converged.scene_and_camera(rtow, scene_name)
    if scene_name not in ("final", "tenk"):
        p, rows = rtow.make_params(W, H, spp, seed=1), None
    else:
        p = rtow.make_params(W, H, spp, seed=1, rank=4, world=9, row_block=8)
        assert p.local_rows == 8
        rows = np.arange(32, 40)
    sums, _ = kernel_render(scene, cam, p)
    s = converged.compare(rtow.tonemap(sums, spp), R, rows=rows)
    print(scene_name, {k: v for k, v in s.items() if k != "channels"})
    converged.check(s)
