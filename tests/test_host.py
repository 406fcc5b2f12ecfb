"""Host-side product code (no GPU): scene builder, cameras, tonemap, PPM writer,
C-ABI surface, row partition.  Pinned against the reference's own fixtures."""
import os
import re
import subprocess

import numpy as np
import pytest

from oracle_lib import golden_kat, golden_ppm, golden_scene_rows, ppm_p3_bytes, read_ppm_bytes, \
    reference_scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_final_scene_bit_exact_vs_reference(rtow):
    """rt_scene_final == reference random_scene() (g++ 11 draw order), cast to fp32."""
    s = rtow.final_scene()
    gold, nxt = golden_scene_rows()
    assert s.n == 486
    assert np.array_equal(s.kind, gold[:, 0].astype(np.uint32))
    for k, col in (("cx", 1), ("cy", 2), ("cz", 3), ("radius", 4)):
        assert np.array_equal(getattr(s, k), gold[:, col].astype(np.float32)), k
    non_glass = s.kind != 2
    assert np.array_equal(s.albedo[non_glass], gold[non_glass, 5:8].astype(np.float32))
    assert np.array_equal(s.param, gold[:, 8].astype(np.float32))
    assert s.rng_next == nxt
    counts = np.bincount(s.kind, minlength=3)
    assert counts.tolist() == [382, 77, 27]  # SURVEY 0.2 (g++ scene)


def test_stress_scene_matches_oracle_restatement(rtow):
    """10k-sphere generator (half extent 50, BASELINE config 5) == oracle's fp64 scene."""
    s = rtow.final_scene(half_extent=50)
    rows, nxt = reference_scene(50)
    assert s.n == rows.shape[0] and 9900 < s.n <= 10004
    assert np.array_equal(s.cx, rows[:, 1].astype(np.float32))
    assert np.array_equal(s.cz, rows[:, 3].astype(np.float32))
    assert np.array_equal(s.kind, rows[:, 0].astype(np.uint32))
    assert s.rng_next == nxt


def test_five_scene(rtow):
    s = rtow.five_scene()
    assert s.n == 5 and s.radius[3] == np.float32(-0.4) and s.kind.tolist() == [0, 0, 2, 2, 1]


def test_camera_cpu_vs_reference_kat(rtow):
    kat = [k for k in golden_kat() if k["kind"] == "camera"][0]
    cam = rtow.camera_cpu(aspect=kat["aspect"])
    f32 = lambda v: np.array(v, np.float64).astype(np.float32)
    assert np.array_equal(np.array(cam.eye[:], np.float32), f32(kat["origin"]))
    assert np.array_equal(np.array(cam.corner[:], np.float32), f32(kat["lower_left_corner"]))
    assert np.array_equal(np.array(cam.horiz[:], np.float32), f32(kat["horizontal"]))
    assert np.array_equal(np.array(cam.vert[:], np.float32), f32(kat["vertical"]))
    lu = np.array(kat["u"]) * kat["lens_radius"]
    assert np.array_equal(np.array(cam.lens_u[:], np.float32), lu.astype(np.float32))
    assert cam.has_lens == 1 and cam.model == 0


def test_camera_cpu_vs_reference_random_kat(rtow):
    """rt_camera_cpu on 200 random parameter sets (eye and target anywhere,
    tilted vup, vfov 5-150, aspect 0.3-4, aperture 0-2, focus 0.5-50) against
    the reference's own camera constructor (tests/golden/make_camera_kat.py):
    every field is the fp32 rounding of the reference's fp64 value."""
    import json
    with open(os.path.join(ROOT, "tests", "golden", "kat_cameras.jsonl")) as f:
        kats = [json.loads(line) for line in f]
    assert len(kats) == 200
    f32 = lambda v: np.array(v, np.float64).astype(np.float32)
    for k in kats:
        a = k["args"]
        cam = rtow.camera_cpu(lookfrom=a[0:3], lookat=a[3:6], vup=a[6:9], vfov=a[9], aspect=a[10], aperture=a[11],
                              focus_dist=a[12])
        assert np.array_equal(np.array(cam.eye[:], np.float32), f32(k["origin"])), k
        assert np.array_equal(np.array(cam.corner[:], np.float32), f32(k["lower_left_corner"])), k
        assert np.array_equal(np.array(cam.horiz[:], np.float32), f32(k["horizontal"])), k
        assert np.array_equal(np.array(cam.vert[:], np.float32), f32(k["vertical"])), k
        lu = np.array(k["u"]) * k["lens_radius"]
        lv = np.array(k["v"]) * k["lens_radius"]
        assert cam.has_lens == (1 if k["lens_radius"] > 0 else 0), k
        if cam.has_lens:
            assert np.array_equal(np.array(cam.lens_u[:], np.float32), lu.astype(np.float32)), k
            assert np.array_equal(np.array(cam.lens_v[:], np.float32), lv.astype(np.float32)), k


def test_tonemap_at_level_boundaries_vs_reference_write_color(rtow):
    """rt_tonemap_u8 (src/cpu mode) on 703 fp32 pixel sums within a few ulps
    of write_color's level thresholds, spp 1 .. 2^20: the reference's own
    write_color output (tests/golden/make_color_kat.py) level for level."""
    from oracle_lib import color_kat
    for sums, spp, want in color_kat():
        got = rtow.tonemap(sums.reshape(1, 1, 3), spp)
        assert [int(x) for x in got.reshape(3)] == want, (sums, spp, want)


def test_camera_gpu_model(rtow):
    """new_camera (src/gpu/camera.h:75-109): pixel deltas span the viewport."""
    cam = rtow.camera_gpu(1920, 1080)
    du = np.array(cam.horiz[:], np.float64)
    dv = np.array(cam.vert[:], np.float64)
    vh = 2 * np.tan(np.radians(10)) * 10
    assert abs(np.linalg.norm(dv) * 1080 - vh) < 1e-4
    assert abs(np.linalg.norm(du) * 1920 - vh * 1920 / 1080) < 1e-4
    assert dv[1] < 0  # rows go down
    assert abs(np.linalg.norm(cam.lens_u[:]) - 10 * np.tan(np.radians(0.3))) < 1e-6
    assert cam.model == 1 and cam.has_lens == 1
    assert rtow.camera_gpu(64, 32, defocus_angle=0.0).has_lens == 0


def test_tonemap_vs_write_color_kat(rtow):
    for k in golden_kat():
        if k["kind"] != "write_color":
            continue
        s = np.array(k["sum"], np.float64)
        if not np.all(s.astype(np.float32).astype(np.float64) == s):
            continue  # the product takes fp32 sums; KATs with non-float inputs skipped
        out = rtow.tonemap(s.astype(np.float32)[None, :], k["spp"])
        assert " ".join(str(int(x)) for x in out[0]) == k["out"], k


def test_tonemap_matches_reference_formula(rtow):
    rng = np.random.default_rng(0)
    sums = (rng.random((1000, 3)) * 12).astype(np.float32)
    got = rtow.tonemap(sums, 10)
    want = (256 * np.clip(np.sqrt(sums.astype(np.float64) / 10), 0, 0.999)).astype(np.int64)
    assert np.array_equal(got, want.astype(np.uint8))


def test_tonemap_gpu_mode_matches_fp32_formula(rtow):
    """RT_TONEMAP_GPU: src/gpu/color.h:16-38 in fp32 (scale = 1.0f/spp, sqrtf,
    clamp to [0, 0.999f], int(256.0f * x))."""
    rng = np.random.default_rng(1)
    for spp in (1, 7, 10, 500, 2000):
        sums = (rng.random((4000, 3)) * 1.2 * spp).astype(np.float32)
        got = rtow.tonemap(sums, spp, rtow.RT_TONEMAP_GPU)
        x = np.sqrt(sums * np.float32(np.float32(1.0) / np.float32(spp)))
        x = np.clip(x, np.float32(0.0), np.float32(0.999))
        want = (np.float32(256.0) * x).astype(np.int64)
        assert np.array_equal(got, want.astype(np.uint8))


def _level_edges(spp, fp32):
    """Sums on both sides of every level boundary (k/256)^2 * spp, plus 0, NaN, inf."""
    v = []
    dt = np.float32 if fp32 else np.float64
    for k in range(1, 256):
        s = dt(k * k / 65536.0) * dt(spp)
        f = np.float32(s)
        v += [np.nextafter(f, np.float32(0)), f, np.nextafter(f, np.float32(np.inf))]
    v += [0.0, np.nan, np.inf, 1e30]
    v = np.array(v, np.float32)
    return v[: len(v) // 3 * 3].reshape(-1, 3)


@pytest.mark.parametrize("mode", [0, 1])
def test_tonemap_level_boundaries(rtow, mode):
    """At every level boundary both modes follow their own arithmetic exactly;
    the fp32 and fp64 levels differ somewhere (why src/gpu's mode exists)."""
    for spp in (10, 100, 500):
        sums = _level_edges(spp, mode == 1)
        got = rtow.tonemap(sums, spp, mode)
        if mode == 0:
            x = np.sqrt(sums.astype(np.float64) * (1.0 / spp))
            x = np.where(np.isnan(x), 0.0, np.clip(x, 0.0, 0.999))
            want = (256 * x).astype(np.int64)
        else:
            with np.errstate(invalid="ignore"):
                x = np.sqrt(sums * np.float32(np.float32(1.0) / np.float32(spp)))
            x = np.where(np.isnan(x), np.float32(0), np.clip(x, np.float32(0.0), np.float32(0.999)))
            want = (np.float32(256.0) * x).astype(np.int64)
        assert np.array_equal(got, want.astype(np.uint8)), (spp, np.argwhere(got != want)[:5])
    sums = _level_edges(10, True)
    assert not np.array_equal(rtow.tonemap(sums, 10, 0), rtow.tonemap(sums, 10, 1))


def test_ppm_writer_streams_large_frames(rtow, tmp_path):
    """The threaded P3 writer (chunks of 65 536 pixels formatted by several
    threads, written in order) gives exactly write_color's text."""
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (1600, 1800, 3), dtype=np.uint8)
    img[0, :5] = [[0, 0, 0], [255, 255, 255], [9, 10, 99], [100, 1, 0], [7, 77, 177]]
    p3 = tmp_path / "big.ppm"
    rtow.write_ppm(str(p3), img)
    data = p3.read_bytes()
    tab = [str(v).encode() for v in range(256)]
    flat = img.reshape(-1, 3)
    want = b"P3\n1800 1600\n255\n" + b"".join(
        tab[r] + b" " + tab[g] + b" " + tab[b] + b"\n" for r, g, b in flat.tolist())
    assert data == want


def test_ppm_writer_p3_and_p6(rtow, tmp_path):
    ref = read_ppm_bytes(golden_ppm("ref_c0_400x225x10"))
    p3 = tmp_path / "a.ppm"
    rtow.write_ppm(str(p3), ref)
    assert p3.read_bytes() == golden_ppm("ref_c0_400x225x10") == ppm_p3_bytes(ref)
    p6 = tmp_path / "a.p6"
    rtow.write_ppm(str(p6), ref, binary=True)
    assert np.array_equal(read_ppm_bytes(p6.read_bytes()), ref)


def test_abi_exports_every_declared_symbol(rtow):
    """Every function include/rt.h (the drop-in boundary) and include/
    rt_internal.h (tests' and tools' diagnostics) declare is
    exported; the public header declares no diagnostic."""
    decl = r"^\s*(?:[\w\*\s]+?)\b(rt_\w+)\s*\("
    pub = sorted(set(re.findall(decl, open(os.path.join(ROOT, "include", "rt.h")).read(), re.M)))
    internal = sorted(set(re.findall(decl, open(os.path.join(ROOT, "include", "rt_internal.h")).read(), re.M)))
    assert len(pub) == 21 and len(internal) == 7, (pub, internal)
    assert not [n for n in pub if n.startswith("rt_internal_") or n == "rt_device_kat"], pub
    assert "RT_OPT_GRID_PHASE" not in open(os.path.join(ROOT, "include", "rt.h")).read()
    names = pub + internal
    L = rtow.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", rtow.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}$", out, re.M), n


@pytest.mark.parametrize("w,h,spp,world,budget,plan", [
    # headline frame (4.15e9 samples) and C1: one launch
    (3840, 2160, 500, 1, 0, (1, 1, 1, 32400)),
    (1920, 1080, 100, 1, 0, (1, 1, 4, 32400)),
    # C3 and C4 rank shares (1/8) at the default budget (2^35): C3 one
    # launch, C4 2 sample ranges of 1 000 spp
    (7680, 4320, 1000, 8, 0, (1, 1, 2, 32640)),
    (16384, 16384, 2000, 8, 0, (1, 2, 1, 131072)),
    # ... and at round 4's 2^32: C4's share 16 sample ranges of 125 spp
    (16384, 16384, 2000, 8, 1 << 32, (1, 16, 1, 131072)),
    # whole C3 frame on one GPU: one launch (8 sample ranges of 125 spp at 2^32)
    (7680, 4320, 1000, 1, 0, (1, 1, 1, 129600)),
    (7680, 4320, 1000, 1, 1 << 32, (1, 8, 1, 129600)),
    # whole C4 frame on one GPU: 16 sample ranges of 125 spp; at 2^32 sample
    # ranges alone would leave 16 spp per wave: 16 strided entry ranges x 8
    # sample ranges of 250 spp instead
    (16384, 16384, 2000, 1, 0, (1, 16, 1, 1048576)),
    (16384, 16384, 2000, 1, 1 << 32, (16, 8, 1, 1048576)),
    # the CLI's progress test: 1080p at 2100 spp with a 2^32 budget, 2 sample
    # ranges of 1050 spp
    (1920, 1080, 2100, 1, 1 << 32, (1, 2, 4, 32400)),
    # a small frame at 50 spp over the budget: 5 entry ranges, all 50 samples each
    (320, 180, 50, 1, 320 * 180 * 10, (5, 1, 1, 230)),
    # C4's share at 16 spp and a 2^24 budget: 32 entry ranges
    (16384, 16384, 16, 8, 1 << 24, (32, 1, 1, 131072)),
    # a budget below total / 65536 is raised: at most 65536 launches
    (16384, 16384, 2000, 1, 1, (8192, 8, 1, 1048576)),
])
def test_launch_plan(rtow, w, h, spp, world, budget, plan):
    """rt_internal_launch_plan: how rt_render cuts a render into bounded
    launches (include/rt.h RT_OPT_LAUNCH_SAMPLES): sample ranges over every
    work entry while each wave keeps >= 100 samples per pixel; else strided
    entry ranges x sample ranges of ~250 spp (a short sample pool idles lanes
    at its tail: C4's full frame in 16-spp sample ranges ran at lane
    efficiency 0.861, profiles/r03n_bench_c4.log)."""
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_PILOT_SCHEDULE
    units = 1 if budget == 320 * 180 * 10 else 0
    got = rtow.launch_plan(rtow.make_params(w, h, spp, flags=flags, world=world, units=units), budget)
    assert (got["ranges"], got["chunks"], got["units"], got["entries"]) == plan, got
    assert got["launches"] == got["ranges"] * got["chunks"] <= 65536
    samples = w * h * spp / world
    if got["launches"] > 1:  # each launch within the budget (up to padding pixels)
        assert samples / got["launches"] <= max(budget or 2 ** 35, samples / 65536) * 1.01


def test_invalid_arguments_return_status(rtow):
    L = rtow.lib()
    assert L.rt_scene_final(11, None, None) == -1
    assert L.rt_tonemap_u8(None, 4, 10, None) == -1
    assert L.rt_strerror(-4) == b"no such HIP device"
    assert L.rt_abi_version() == rtow.ABI_VERSION == 6
    with pytest.raises(rtow.RTError):
        rtow.camera_cpu(aspect=0.0)


def test_no_device_reports_error(rtow):
    if rtow.device_count() > 0:
        pytest.skip("device present")
    with pytest.raises(rtow.RTError) as e:
        rtow.Context(0)
    assert e.value.status == -4


@pytest.mark.parametrize("H,world,rb", [(2160, 8, 8), (2160, 2, 8), (1080, 4, 8), (75, 3, 4), (7, 8, 8)])
def test_row_partition_covers_every_row_once(rtow, H, world, rb):
    seen = np.zeros(H, np.int64)
    sizes = set()
    for r in range(world):
        p = rtow.make_params(64, H, 1, rank=r, world=world, row_block=rb)
        rows = rtow.local_to_global_rows(p)
        sizes.add(p.local_rows)
        np.add.at(seen, rows[rows < H], 1)
    assert np.all(seen == 1)
    assert len(sizes) == 1  # equal tiles for the gather


def test_cli_no_device_exit_99():
    exe = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "bin", "gpu_ray_tracer")
    import rtow
    if rtow.device_count() > 0:
        pytest.skip("device present")
    r = subprocess.run([exe, "--spp", "1", "--quiet"], capture_output=True)
    assert r.returncode == 99  # src/gpu/cuda_utility.h:16


@pytest.mark.parametrize("extra,msg", [
    (["--gpus", "2", "--devices", "0,0", "--gather", "rccl"], b"distinct devices"),
    (["--gpus", "3", "--devices", "0,0"], b"usage:"),
])
def test_cli_devices_argument_checks(extra, msg):
    """--devices is checked before any device is touched: one entry per band,
    and no RCCL gather over a repeated device (one rank per device)."""
    exe = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd", "bin", "cpu_ray_tracer")
    r = subprocess.run([exe, "--width", "16", "--quiet"] + extra, capture_output=True, timeout=60)
    assert r.returncode == 2 and msg in r.stderr


def test_accel_builder_invariants_on_host(rtow):
    """rt_internal_accel_info runs rt_scene_upload's BVH / layer-grid builder on
    the host: the final scene is a layer scene whose grid fits the LDS budget of
    8 blocks per CU; the 10 000-sphere scene's grid stays in global memory; the
    five-sphere scene has no layer; every grid numbers its cells' first items by
    the running count (cell i's items are [first_i, first_{i+1}), which the LDS
    walk reads as two adjacent u16) and keeps its ring of cells empty."""
    fin = rtow.accel_info(rtow.final_scene())
    assert fin["layer_mode"] == 1 and fin["n_extra_pairs"] == 2
    assert fin["grid_fits_lds"] == 1 and fin["grid_lds_bytes"] <= 160 * 1024 // 8 - 3328
    assert fin["grid_starts_ok"] == 1 and fin["grid_ring_empty"] == 1
    assert 1 <= fin["max_items_per_cell"] <= 15 and fin["grid_items"] >= 482
    big = rtow.accel_info(rtow.final_scene(50))
    assert big["layer_mode"] == 1 and big["grid_fits_lds"] == 0
    assert big["grid_starts_ok"] == 1 and big["grid_ring_empty"] == 1
    five = rtow.accel_info(rtow.five_scene())
    assert five["layer_mode"] == 0 and five["grid_items"] == 0


def test_grid_fit_picks_a_candidate_per_camera(rtow):
    """RT_OPT_GRID_FIT (rtk::grid_fitter): the host model of
    the layer walk's cost picks one of the builder's candidate cell scales
    s0 (1 + 0.01 k) for a camera; deterministic; the builder's scale when the
    camera does not see the layer; no fitting without an LDS grid.  The picks
    for the headline frame and C4's frame are the ones the GPU sweeps were
    checked against (tools/grid_fit_check.py, profiles/r05g_*)."""
    fin, c4 = rtow.final_scene(), rtow.final_scene(half_extent=50)
    cam = rtow.camera_cpu(aspect=16 / 9)
    sc, costs = rtow.grid_fit(fin, cam, 3840, 2160)
    s0 = rtow.accel_info(fin)["grid_scale_milli"] / 1000.0
    assert len(costs) >= 20 and abs(costs[0][0] - s0) < 1e-9
    assert sc == min(costs, key=lambda x: x[1])[0]
    assert rtow.grid_fit(fin, cam, 3840, 2160) == (sc, costs)
    assert abs(sc - 1.11) < 1e-9  # the fine sweep's best region (1.11 / 1.00 / 1.22)
    sc4, costs4 = rtow.grid_fit(c4, rtow.camera_cpu(aspect=1.0), 16384, 16384)
    s04 = rtow.accel_info(c4)["grid_scale_milli"] / 1000.0
    assert abs(sc4 / s04 - 1.05) < 1e-3  # (s0 from accel_info is rounded to 1e-3)
    up = rtow.camera_cpu(lookfrom=(0, 1, 0), lookat=(0, 5, 0.01), aspect=1.0)  # sky only
    assert rtow.grid_fit(fin, up, 64, 64)[0] == s0
    assert rtow.grid_fit(rtow.five_scene(), cam, 64, 36)[0] == 0.0


def test_grid_phase_keeps_the_grid_invariants(rtow):
    """RT_OPT_INTERNAL_GRID_PHASE_X / _Z (the grid's origin shifted by a fraction of a
    cell): the fitter's candidates at every phase are grids the
    placement holds, the model's costs differ with the phase (the cell borders
    move relative to the spheres) and phases outside [0, 1) are refused."""
    fin = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=16 / 9)
    base = rtow.grid_fit(fin, cam, 3840, 2160)
    seen = set()
    for ph in ((0.0, 0.0), (0.25, 0.25), (0.5, 0.0), (0.875, 0.125)):
        sc, costs = rtow.grid_fit(fin, cam, 3840, 2160, ph)
        assert len(costs) >= 20 and sc == min(costs, key=lambda x: x[1])[0]
        seen.add(tuple(round(c, 9) for _, c in costs))
    assert rtow.grid_fit(fin, cam, 3840, 2160, (0.0, 0.0)) == base
    assert len(seen) == 4
    for bad in ((1.0, 0.0), (0.0, -0.1)):
        with pytest.raises(rtow.RTError):
            rtow.grid_fit(fin, cam, 3840, 2160, bad)


def test_accel_builder_on_degenerate_scenes(rtow):
    """The builder on inputs that stress it (tests/random_scenes.py
    degenerate_scenes: coincident spheres, a line, a crowded layer, huge and
    tiny radii, far-away spheres, the layer-mode size thresholds): every grid
    it builds keeps its invariants, in every placement; the GPU renders of
    the same scenes are checked against the oracle in test_random_scenes_gpu.py."""
    import random_scenes
    for name, scene in random_scenes.degenerate_scenes(rtow).items():
        for mode in ("auto", "lds", "cells", "global"):
            info = rtow.accel_info(scene, grid_mode=mode)
            if info["grid_items"]:
                assert info["grid_starts_ok"] == 1 and info["grid_ring_empty"] == 1, (name, mode, info)
                assert 1 <= info["max_items_per_cell"] <= 15, (name, mode, info)
            assert info["bvh_slots"] >= scene.n, (name, info)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_code_under_asan_ubsan():
    """tools/host_sanitize.sh: the scene builders, cameras, BVH / grid builder,
    tonemaps and PPM writers under AddressSanitizer (with leak checks) and
    UndefinedBehaviorSanitizer, host code only, no device."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([os.path.join(root, "tools", "host_sanitize.sh")], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host_sanitize: ok" in r.stdout


def test_scene_validation_on_host(rtow):
    """rt_scene_upload's validation (shared with rt_internal_accel_info, so it
    runs without a device): non-finite centres, zero radii, unknown materials
    and negative or non-finite lambertian / metal albedos are RT_ERR_INVALID;
    albedos above 1 are accepted (64-bit pixel sums); a
    dielectric's albedo is ignored."""
    import dataclasses
    base = rtow.final_scene()
    assert rtow.accel_info(base)["layer_mode"] == 1
    lam = int(np.nonzero(base.kind == rtow.RT_LAMBERTIAN)[0][0])
    met = int(np.nonzero(base.kind == rtow.RT_METAL)[0][0])
    die = int(np.nonzero(base.kind == rtow.RT_DIELECTRIC)[0][0])

    def with_(name, i, value, col=None):
        a = getattr(base, name).copy()
        if col is None:
            a[i] = value
        else:
            a[i, col] = value
        return dataclasses.replace(base, **{name: a})

    bad = [with_("cx", 5, float("nan")), with_("cz", 5, float("inf")), with_("radius", 5, 0.0),
           with_("kind", 5, 7), with_("albedo", met, -0.1, 2), with_("albedo", lam, float("nan"), 1),
           with_("albedo", lam, float("inf"), 2)]
    for sc in bad:
        with pytest.raises(rtow.RTError) as ei:
            rtow.accel_info(sc)
        assert ei.value.status == rtow.RT_ERR_INVALID
    assert rtow.accel_info(with_("albedo", die, 9.0, 0))["layer_mode"] == 1
    # energy-creating albedos (the reference's constructors take any colour):
    # accepted; with 3 KB more static LDS for the 64-bit sums the final
    # scene's grid keeps only its cells in LDS
    hot = with_("albedo", lam, 1.5, 0)
    assert rtow.accel_info(hot)["layer_mode"] == 1
    assert rtow.accel_info(hot)["grid_placement"] == rtow.RT_GRID_CELLS_LDS
    assert rtow.accel_info(base)["grid_placement"] == rtow.RT_GRID_LDS


def test_turn_table_deterministic_and_accurate(tmp_path):
    """include/rt_turn_table.h (the kernel's and the oracle's sin/cos table):
    the same bits from gcc and from a restatement in Python doubles (the
    series uses only IEEE double arithmetic), and within 1 fp32 ulp of cos /
    sin of 2 pi i / 1024."""
    src = tmp_path / "t.c"
    src.write_text('#include <stdio.h>\n#include "rt_turn_table.h"\n'
                   'int main(void) { static float t[2 * RT_TURN_TABLE]; rt_turn_table(t);\n'
                   '  fwrite(t, sizeof t, 1, stdout); return 0; }\n')
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"), "-o", str(exe),
                    str(src)], check=True)
    got = np.frombuffer(subprocess.run([str(exe)], capture_output=True, check=True).stdout,
                        dtype=np.float32).reshape(-1, 2)
    n = 1024
    assert got.shape == (n, 2)
    want = np.empty((n, 2), np.float32)
    for i in range(n):
        x = 6.283185307179586476925 * float(i % (n // 4)) / float(n)
        c = s = 0.0
        term = 1.0
        for k in range(32):
            if k % 4 == 0:
                c += term
            elif k % 4 == 1:
                s += term
            elif k % 4 == 2:
                c -= term
            else:
                s -= term
            term = term * x / float(k + 1)
        fc, fs = np.float32(c), np.float32(s)
        want[i] = [(fc, fs), (-fs, fc), (-fc, -fs), (fs, -fc)][i // (n // 4)]
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    a = 2.0 * np.pi * np.arange(n) / n
    exact = np.stack([np.cos(a), np.sin(a)], axis=1)
    ulp = np.spacing(np.abs(exact).astype(np.float32)).astype(np.float64)
    assert np.all(np.abs(got.astype(np.float64) - exact) <= np.maximum(ulp, 1e-15))  # exact zeros where cos / sin vanish


def test_sealed_spheres_product_equals_oracle(rtow, oracle):
    """The opaque-inside rule applies to sealed spheres only (DESIGN.md 2 step
    4): lambertian, |r| > 2 t_min, no other ball overlapping its ball.  The
    product's sweep (rt_internal_sealed) equals the oracle's brute-force
    restatement on the final scene, C4's 10 000 spheres, the five-sphere
    scene, the rule's reference fixtures and 24 random scenes with
    overlapping and nested spheres."""
    import fixture_scenes
    import random_scenes
    scenes = {"final": rtow.final_scene(), "c4": rtow.final_scene(half_extent=50), "five": rtow.five_scene()}
    scenes.update({k: f(rtow) for k, f in fixture_scenes.FIXTURES.items()})
    scenes.update({"free%d" % k: random_scenes.free_scene(rtow, k) for k in range(24)})
    for name, s in scenes.items():
        a, b = rtow.sealed(s), oracle.sealed(s)
        assert np.array_equal(a, b), name
        assert not a[s.kind != 0].any(), name  # metal and glass are never sealed
    final, c4 = scenes["final"], scenes["c4"]
    # the ground is sealed (the big glass sphere touches it at one point,
    # |C_a - C_b| = 1001 = r_a + r_b exactly); the big lambertian sphere at
    # (-4, 1, 0) is overlapped by small spheres
    for s in (final, c4):
        assert s.radius[0] == 1000 and rtow.sealed(s)[0]
        big = np.flatnonzero((s.radius == 1) & (s.kind == 0))
        assert len(big) == 1 and not rtow.sealed(s)[big[0]]
    assert rtow.sealed(final).sum() == 347 and (final.kind == 0).sum() == 382
    emb = scenes["embed"]
    assert rtow.sealed(emb).tolist() == [True, False, False]  # the glass overlaps the r = 1 ball
    assert rtow.sealed(scenes["negop"]).tolist() == [True, True, False]  # |r| counts
    # five: the ground (r = 100) touches nothing; the centre sphere is sealed
    assert rtow.sealed(scenes["five"]).tolist() == [True, True, False, False, False]


def test_sealed_touching_and_tiny_spheres(rtow, oracle):
    """Touching at one point keeps both balls sealed; any overlap unseals
    both; a lambertian ball of |r| <= 2 t_min is never sealed."""
    f32 = np.float32

    def mk(rows):
        a = np.array(rows, np.float64)
        return rtow.Scene(a[:, 0].astype(f32), a[:, 1].astype(f32), a[:, 2].astype(f32), a[:, 3].astype(f32),
                          np.zeros(len(rows), np.uint32), np.full((len(rows), 3), 0.5, f32),
                          np.zeros(len(rows), f32))
    touching = mk([(0, 0, 0, 1), (3, 0, 0, 2), (0, 0.5, 0, 0.0015), (9, 9, 9, 0.003)])
    assert rtow.sealed(touching).tolist() == [False, True, False, True]  # (0, .5, 0) lies inside ball 0
    apart = mk([(0, 0, 0, 1), (3, 0, 0, 2), (9, 9, 9, 0.0019)])
    assert rtow.sealed(apart).tolist() == [True, True, False]
    overlap = mk([(0, 0, 0, 1), (2.999, 0, 0, 2)])
    assert rtow.sealed(overlap).tolist() == [False, False]
    for s in (touching, apart, overlap):
        assert np.array_equal(rtow.sealed(s), oracle.sealed(s))


def test_device_code_has_no_flat_memory_instructions(rtow, tmp_path):
    """No generic-pointer (flat) load, store or atomic anywhere in librtow.so's
    gfx950 code ("the v7 fault"): the walk reads LDS through
    address_space(3) pointers (ds_*) and the grid, records and frame through
    address_space(1) ones (global_*), so no address is ever formed from an
    LDS offset plus the shared aperture.  Round 5's unshipped v7 variant read
    its hot items through flat loads and faulted with
    HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION (profiles/r05p_v7tests_fault.log),
    the code of a flat address outside every aperture and outside the
    canonical range: an LDS-aperture pointer with a negative offset.  Since
    round 6 the epilogue's atomics are global too, so a flat instruction
    appearing here is a regression to look at."""
    import shutil
    llvm = "/opt/rocm/lib/llvm/bin"
    if not (os.path.exists(os.path.join(llvm, "llvm-objdump")) and shutil.which("objcopy")):
        pytest.skip("llvm-objdump / objcopy not available")
    fat = tmp_path / "fatbin.bin"
    co = tmp_path / "gfx950.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", rtow.LIB_PATH, str(fat)], check=True)
    subprocess.run([os.path.join(llvm, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + str(fat),
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + str(co)], check=True)
    dis = subprocess.run([os.path.join(llvm, "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)],
                         check=True, capture_output=True, text=True).stdout
    ops = re.findall(r"^\s+((?:flat|global|ds)_\w+)", dis, re.M)
    assert sum(o.startswith("global_") for o in ops) > 100 and sum(o.startswith("ds_") for o in ops) > 100
    flat = sorted(set(o for o in ops if o.startswith("flat_")))
    assert not flat, flat
