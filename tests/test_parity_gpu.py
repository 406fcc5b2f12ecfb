"""GPU parity: the HIP kernel (through the C ABI) against the oracle.

* bit-exact vs the kernel-mode CPU restatement on the same seeded inputs
  (fp32 sums compared with np.array_equal; segment counts equal);
* statistical vs the reference's own C0 image (north-star bound: image-mean
  bias <= 1/255 per channel; 16x16 block means within 1.5x the reference's
  stream-to-stream noise floor);
* size-independent properties at BASELINE sizes (determinism, partition
  invariance, sample / segment accounting, finiteness).
"""
import numpy as np
import pytest

from oracle_lib import golden_ppm, golden_stats, kernel_render, read_ppm_bytes
from test_oracle import stat_compare

pytestmark = pytest.mark.gpu

# RT_FLAG_ACCEL_BVH: layer scenes walk the layer grid; + RT_FLAG_LAYER_BVH: the layer BVH
ACCELS = {"scan": 0, "bvh": 1 << 9, "layer_bvh": (1 << 9) | (1 << 12)}


@pytest.fixture(params=list(ACCELS), ids=list(ACCELS))
def accel(request):
    """Both traversal modes must reproduce the brute-force oracle bit for bit."""
    return ACCELS[request.param]


# lane efficiency of the shipped kernel (segments / (64 x wave-steps)),
# measured on the GPU (profiles/r04_gpu_tests.log); the tests allow 0.02 /
# 0.005 below it
LANE_EFF_4SPP = 0.335
LANE_EFF_500SPP = 0.9945


def gpu_vs_oracle(rtow, ctx, scene, cam, params, accel=0):
    ctx.upload(scene)
    want, segs = kernel_render(scene, cam, params)
    params.flags |= accel
    got, st = ctx.render(cam, params)
    return got, st, want, segs


def assert_bit_exact(got, st, want, segs):
    assert np.isfinite(got).all()
    n_diff = int((got != want).sum())
    assert n_diff == 0, f"{n_diff} of {got.size} floats differ; max |d| = {np.abs(got - want).max()}"
    assert st.segments == segs


def test_c0_bit_exact_vs_oracle(rtow, gpu_ctx, accel):
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    p = rtow.make_params(400, 225, 10, seed=0)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


def test_c0_statistical_vs_reference(rtow, gpu_ctx):
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=16.0 / 9.0)
    sums, st = gpu_ctx.render(cam, rtow.make_params(400, 225, 10, seed=0))
    img = rtow.tonemap(sums, 10)
    ref = read_ppm_bytes(golden_ppm("ref_c0_400x225x10"))
    ref2 = read_ppm_bytes(golden_ppm("ref_c0_shift_400x225x10"))
    bias, blk, floor = stat_compare(img, ref, ref2)
    assert np.all(np.abs(bias) <= 1.0), bias
    assert blk <= 1.5 * floor, (blk, floor)
    ref_segs = golden_stats()["ref_c0_400x225x10"]["segments"]
    assert abs(st.segments / ref_segs - 1) < 0.003


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_gpu_camera_and_semantics_bit_exact(rtow, gpu_ctx, flags, accel):
    """--camera=gpu model (src/gpu/camera.h) and the src/gpu semantic switches."""
    scene = rtow.final_scene()
    cam = rtow.camera_gpu(160, 90)
    p = rtow.make_params(160, 90, 6, seed=1234567890123, flags=flags)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


@pytest.mark.parametrize("flags", [0, 3])
def test_five_scene_negative_radius_bit_exact(rtow, gpu_ctx, accel, flags):
    """Duplicate centres (r = 0.5 and -0.4 at one point): exercises the tie rule."""
    scene = rtow.five_scene()
    cam = rtow.camera_cpu(lookfrom=(-2, 2, 1), lookat=(0, 0, -1), aspect=200 / 112,
                          aperture=0.0, focus_dist=3.4)
    p = rtow.make_params(200, 112, 16, seed=3, flags=flags)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


def test_ten_thousand_spheres_bit_exact(rtow, gpu_ctx, accel):
    scene = rtow.final_scene(half_extent=50)
    assert 9900 < scene.n <= 10004
    cam = rtow.camera_cpu(aspect=2.0)
    p = rtow.make_params(48, 24, 2, seed=11)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


@pytest.mark.parametrize("w,h,spp,depth", [(13, 7, 3, 50), (8, 8, 1, 1), (65, 9, 2, 2), (1, 2, 4, 50)])
def test_ragged_and_shallow_bit_exact(rtow, gpu_ctx, w, h, spp, depth, accel):
    scene = rtow.final_scene()
    cam = rtow.camera_gpu(w, h) if w < 2 else rtow.camera_cpu(aspect=w / h)
    p = rtow.make_params(w, h, spp, max_depth=depth, seed=5)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


def test_bvh_equals_scan_at_full_hd(rtow, gpu_ctx):
    """At BASELINE size (1920x1080, 4 spp) the BVH walk reproduces the scan's
    fp32 sums exactly, and does fewer ray-sphere tests."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=1920 / 1080)
    p = rtow.make_params(1920, 1080, 4, seed=77, flags=1 << 10)
    a, sa = gpu_ctx.render(cam, p)
    p.flags |= 1 << 9
    b, sb = gpu_ctx.render(cam, p)
    assert np.array_equal(a, b)
    assert sa.segments == sb.segments
    assert sa.sphere_tests >= sa.bf_tests  # scan tests every (padded) slot
    assert sb.sphere_tests < sa.sphere_tests
    assert sb.box_tests > 0 and sa.box_tests == 0


def test_bvh_equals_scan_headline_frame(rtow, gpu_ctx):
    """The whole headline frame (3840x2160 @ 500 spp, ~1.1e10 segments): BVH and
    scan agree on every fp32 sum -- the padding bound holds at scale, where
    grazing roots that a padded-for-rounding box would drop do occur."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=3840 / 2160)
    p = rtow.make_params(3840, 2160, 500, seed=3)
    a, sa = gpu_ctx.render(cam, p)
    for acc in (ACCELS["bvh"], ACCELS["layer_bvh"]):  # the layer grid and the layer BVH
        p.flags = acc
        b, sb = gpu_ctx.render(cam, p)
        assert sa.segments == sb.segments
        n_diff = int((a != b).sum())
        assert n_diff == 0, (acc, n_diff)


def test_bvh_equals_scan_ten_thousand_spheres(rtow, gpu_ctx):
    """BASELINE config 5's 10 000-sphere scene at 1920x1080 x 4 spp: the BVH walk
    and the brute-force scan (10 004 tests per segment) agree on every sum."""
    gpu_ctx.upload(rtow.final_scene(half_extent=50))
    cam = rtow.camera_cpu(aspect=1920 / 1080)
    p = rtow.make_params(1920, 1080, 4, seed=21, flags=1 << 10)
    a, sa = gpu_ctx.render(cam, p)
    for acc in (ACCELS["bvh"], ACCELS["layer_bvh"]):
        p.flags = (1 << 10) | acc
        b, sb = gpu_ctx.render(cam, p)
        assert sa.segments == sb.segments
        assert np.array_equal(a, b)
        assert sb.sphere_tests * 50 < sa.sphere_tests  # >50x fewer sphere tests than the scan


def test_empty_scene_all_sky(rtow, gpu_ctx, accel):
    s = rtow.final_scene()
    empty = rtow.Scene(s.cx[:0], s.cy[:0], s.cz[:0], s.radius[:0], s.kind[:0], s.albedo[:0], s.param[:0])
    cam = rtow.camera_cpu(aspect=2.0)
    p = rtow.make_params(16, 8, 2, seed=1)
    got, st, want, segs = gpu_vs_oracle(rtow, gpu_ctx, empty, cam, p, accel)
    assert_bit_exact(got, st, want, segs)
    assert st.segments == 16 * 8 * 2


def test_spp_zero_and_depth_zero(rtow, gpu_ctx):
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=2.0)
    for p in (rtow.make_params(32, 16, 0), rtow.make_params(32, 16, 4, max_depth=0)):
        out, st = gpu_ctx.render(cam, p)
        assert not out.any() and st.segments == 0


def test_partition_bit_exact_across_ranks(rtow, gpu_ctx):
    """Interleaved row bands for G ranks reassemble to the G=1 image exactly."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=200 / 75)
    full, st1 = gpu_ctx.render(cam, rtow.make_params(200, 75, 4, seed=9))
    for world in (2, 8):
        got = np.zeros_like(full)
        segs = 0
        for rank in range(world):
            p = rtow.make_params(200, 75, 4, seed=9, rank=rank, world=world, row_block=8)
            tile, st = gpu_ctx.render(cam, p)
            rows = rtow.local_to_global_rows(p)
            keep = rows < 75
            got[rows[keep]] = tile[keep]
            assert not tile[~keep].any()
            segs += st.segments
        assert np.array_equal(got, full)
        assert segs == st1.segments


def test_full_hd_properties(rtow, gpu_ctx):
    """C1 geometry (1920x1080) at low spp: deterministic, finite, sane accounting."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=1920 / 1080)
    p = rtow.make_params(1920, 1080, 4, seed=42)
    a, st = gpu_ctx.render(cam, p)
    b, st2 = gpu_ctx.render(cam, p)
    assert np.array_equal(a, b) and st.segments == st2.segments
    assert np.isfinite(a).all() and (a >= 0).all()
    assert st.samples == 1920 * 1080 * 4
    assert 2.4 < st.segments / st.samples < 3.0
    # each sample contributes at most 1 per channel (attenuation <= 1, sky <= 1)
    assert a.max() <= 4.0 + 1e-5
    # lane efficiency of the path-regeneration loop (segments / (64 x
    # wave-steps)): at 4 spp a wave's pool holds 4 samples per pixel, and its
    # tail idles lanes
    eff = st.segments / (64.0 * st.wave_steps)
    print("lane efficiency 1920x1080x4: %.4f" % eff)
    assert LANE_EFF_4SPP - 0.02 < eff <= 1.0


def test_lane_efficiency_headline_pool(rtow, gpu_ctx):
    """The pool's lane efficiency at the headline's 500 samples per pixel per
    wave (a 1920x1080 frame at 500 spp, units 1: every wave holds its tile's
    whole pool) stays at the shipped kernel's measured value: a scheduling
    regression (the persistent-waves variant of round 3 ran at 0.30 at 4 spp)
    fails here."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=16 / 9)
    p = rtow.make_params(640, 360, 500, seed=5, units=1)
    _, st = gpu_ctx.render(cam, p)
    eff = st.segments / (64.0 * st.wave_steps)
    print("lane efficiency 640x360x500: %.4f" % eff)
    assert LANE_EFF_500SPP - 0.005 < eff <= 1.0


def test_headline_geometry_one_spp(rtow, gpu_ctx):
    """3840x2160 (the headline frame) at 1 spp: every pixel written, mean matches
    the 1920x1080 image statistics (scale invariance of the image mean)."""
    gpu_ctx.upload(rtow.final_scene())
    big, st = gpu_ctx.render(rtow.camera_cpu(aspect=3840 / 2160), rtow.make_params(3840, 2160, 1, seed=1))
    small, _ = gpu_ctx.render(rtow.camera_cpu(aspect=1920 / 1080), rtow.make_params(1920, 1080, 4, seed=2))
    assert np.isfinite(big).all()
    assert st.samples == 3840 * 2160
    m_big = big.reshape(-1, 3).mean(0)
    m_small = small.reshape(-1, 3).mean(0) / 4
    assert np.all(np.abs(m_big - m_small) < 0.01), (m_big, m_small)


@pytest.mark.parametrize("units", [1, 2, 3])
def test_chunked_sum_bit_exact_vs_oracle(rtow, gpu_ctx, units, accel):
    """spp > RT_CHUNK_SPP: three sample chunks (64, 64, 22), traced by 1, 2 or
    3 waves per tile from each wave's sample pool; the fixed-point pixel sums
    match the oracle bit for bit."""
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(aspect=2.0)
    p = rtow.make_params(24, 12, 150, seed=17, units=units)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, accel))


def test_units_do_not_change_the_image(rtow, gpu_ctx):
    """rt_params.units only schedules: 1..8 waves per tile and the automatic
    choice, alone and combined with an 8-rank partition, give the same sums."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=320 / 120)
    bvh = rtow.RT_FLAG_ACCEL_BVH
    ref, st = gpu_ctx.render(cam, rtow.make_params(320, 120, 500, seed=4, flags=bvh, units=1))
    for u in (0, 2, 3, 5, 8):
        got, st2 = gpu_ctx.render(cam, rtow.make_params(320, 120, 500, seed=4, flags=bvh, units=u))
        assert np.array_equal(got, ref), u
        assert st2.segments == st.segments
    got = np.zeros_like(ref)
    for rank in range(8):
        p = rtow.make_params(320, 120, 500, seed=4, flags=bvh, rank=rank, world=8, units=8)
        tile, _ = gpu_ctx.render(cam, p)
        rows = rtow.local_to_global_rows(p)
        keep = rows < 120
        got[rows[keep]] = tile[keep]
        assert not tile[~keep].any()
    assert np.array_equal(got, ref)


def test_pilot_schedule_does_not_change_the_image(rtow, gpu_ctx):
    """RT_FLAG_PILOT_SCHEDULE only reorders block launches (a 4-spp pilot per
    frame geometry, then expensive tiles first): the same sums and segment
    counts as launch order, for one wave per tile and for split chunks, on the
    first render of a geometry (pilot + sort) and on a cached one; the pilot
    leaves the context's counters alone (RT_FLAG_KEEP_COUNTERS)."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=320 / 120)
    bvh = rtow.RT_FLAG_ACCEL_BVH
    pilot = bvh | rtow.RT_FLAG_PILOT_SCHEDULE
    for units in (1, 3, 0):
        ref, st = gpu_ctx.render(cam, rtow.make_params(320, 120, 200, seed=9, flags=bvh, units=units))
        for _ in range(2):
            got, st2 = gpu_ctx.render(cam, rtow.make_params(320, 120, 200, seed=9, flags=pilot, units=units))
            assert np.array_equal(got, ref), units
            assert st2.segments == st.segments
    # a new geometry (another camera) gets its own pilot; counters accumulate
    # only the real renders
    cam2 = rtow.camera_cpu(aspect=320 / 120, lookfrom=(12.0, 2.5, 3.5))
    a, sa = gpu_ctx.render(cam2, rtow.make_params(320, 120, 64, seed=2, flags=bvh))
    gpu_ctx.reset_stats()
    p = rtow.make_params(320, 120, 64, seed=2, flags=pilot | rtow.RT_FLAG_KEEP_COUNTERS)
    b, _ = gpu_ctx.render(cam2, p)
    c, _ = gpu_ctx.render(cam2, p)
    assert np.array_equal(a, b) and np.array_equal(a, c)
    assert gpu_ctx.collect_stats().segments == 2 * sa.segments


def test_cli_bvh_and_scan_print_the_same_ppm(tmp_path):
    """bin/cpu_ray_tracer (the drop-in executable): P3 on stdout, identical bytes
    for --accel bvh (default) and --accel scan, and P6 with the same pixels."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "ray-tracing-in-one-weekend_amd", "bin", "cpu_ray_tracer")
    args = [exe, "--width", "96", "--height", "54", "--spp", "8", "--seed", "3", "--quiet"]
    a = subprocess.run(args, capture_output=True, timeout=120, check=True).stdout
    b = subprocess.run(args + ["--accel", "scan"], capture_output=True, timeout=120, check=True).stdout
    assert a.startswith(b"P3\n96 54\n255\n")
    assert a == b
    p6 = tmp_path / "x.ppm"
    subprocess.run(args + ["--p6", "--out", str(p6)], capture_output=True, timeout=120, check=True)
    raw = p6.read_bytes()
    head = b"P6\n96 54\n255\n"
    assert raw.startswith(head)
    vals = np.array(a.split()[4:], dtype=np.uint8)
    assert np.array_equal(np.frombuffer(raw[len(head):], np.uint8), vals)


def test_cli_rccl_gather_path_prints_the_same_ppm():
    """The CLI's multi-GPU path (render on per-device streams, one RCCL
    ncclGather of the tiles to device 0, one copy to the host), forced on the
    one GPU this box has: the same bytes as the host-copy path."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "ray-tracing-in-one-weekend_amd", "bin", "gpu_ray_tracer")
    args = [exe, "--width", "96", "--height", "54", "--spp", "8", "--seed", "5", "--quiet"]
    a = subprocess.run(args + ["--gather", "host"], capture_output=True, timeout=120, check=True).stdout
    b = subprocess.run(args + ["--gather", "rccl"], capture_output=True, timeout=120, check=True).stdout
    assert a.startswith(b"P3\n96 54\n255\n")
    assert a == b


def test_cli_reports_each_device_and_refuses_missing_gpus(rtow):
    """gpu_ray_tracer prints one stderr line per device (render ms and its
    launch count, write_color ms, gather ms) after the reference's timing
    lines, and refuses --gpus N beyond the visible devices (exit 2) instead of
    rendering on fewer and reporting the time as N GPUs' (VERDICT r2, item 7)."""
    import os
    import re
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "..", "ray-tracing-in-one-weekend_amd", "bin", "gpu_ray_tracer")
    args = [exe, "--width", "96", "--height", "54", "--spp", "8", "--seed", "5", "--out", os.devnull]
    r = subprocess.run(args + ["--gather", "rccl"], capture_output=True, timeout=120, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Time Cost (ms) = " in r.stderr
    assert re.search(r"GPU 0 \(device 0\): render [0-9.]+ ms in 1 launch\(es\), write_color [0-9.]+ ms, "
                     r"gather \(RCCL\) [0-9.]+ ms", r.stderr), r.stderr
    n = rtow.device_count()
    bad = subprocess.run(args + ["--gpus", str(n + 1)], capture_output=True, timeout=120, text=True)
    assert bad.returncode == 2 and f"only {n} HIP device" in bad.stderr
    # a render cut into several bounded launches reports its progress (a 2^32
    # budget, --launch-samples: the default 2^35 keeps this frame one launch)
    big = [exe, "--width", "1920", "--height", "1080", "--spp", "2100", "--seed", "5", "--out", os.devnull,
           "--launch-samples", "4294967296"]
    r = subprocess.run(big, capture_output=True, timeout=120, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Launches remaining: 0" in r.stderr and re.search(r"render [0-9.]+ ms in 2 launch", r.stderr), r.stderr


def test_render_progress_counts_bounded_launches(rtow, gpu_ctx):
    """rt_render_progress after an asynchronous render of 5 bounded launches:
    (5, 5) once the stream has drained, and the image equals one launch's."""
    import torch
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=320 / 180)
    p = rtow.make_params(320, 180, 50, seed=4, flags=1 << 9, units=1)
    want, _ = gpu_ctx.render(cam, p)
    assert gpu_ctx.progress() == (1, 1)
    gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 320 * 180 * 10)
    dev = torch.device("cuda", 0)
    t = torch.zeros((180, 320, 3), dtype=torch.float32, device=dev)
    st = torch.cuda.Stream(dev)
    gpu_ctx.render_async(cam, p, t.data_ptr(), st.cuda_stream)
    done, total = gpu_ctx.progress()
    assert total == 5 and 0 <= done <= 5
    torch.cuda.synchronize(dev)
    assert gpu_ctx.progress() == (5, 5)
    assert np.array_equal(t.cpu().numpy(), want)
    gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 0)


@pytest.mark.parametrize("kind,radius,ends", [(0, 0.5, True), (0, -0.5, True), (1, 0.5, False), (2, 0.5, False),
                                               (0, 3.0, False)])
def test_opaque_sphere_hit_from_inside_ends_the_path(rtow, gpu_ctx, kind, radius, ends, accel):
    """a camera inside a SEALED lambertian sphere (r =
    +-0.5 around the eye at (13, 2, 3), no other ball overlapping it) sees every
    primary ray hit that sphere at its exiting root, and the path ends there
    black: one segment per sample, an all-zero image -- what the reference's
    path, hitting the same sphere at t = |r| after every scatter until the
    depth cap, returns.  The rule is keyed on the root, so a negative radius
    ends the same way.  Inside a metal or glass sphere, or a lambertian one of
    r = 3 that the ground overlaps (not sealed), the paths go on.  GPU ==
    oracle bit for bit in every walk."""
    import dataclasses
    base = rtow.final_scene()
    f32 = np.float32
    big = dataclasses.replace(
        base, cx=np.append(base.cx, f32(13)), cy=np.append(base.cy, f32(2)), cz=np.append(base.cz, f32(3)),
        radius=np.append(base.radius, f32(radius)), kind=np.append(base.kind, np.uint32(kind)),
        albedo=np.vstack([base.albedo, np.array([[0.5, 0.6, 0.7]], f32)]),
        param=np.append(base.param, f32(1.5 if kind == 2 else 0.3)))
    assert rtow.sealed(big)[-1] == (kind == 0 and abs(radius) < 1)
    cam = rtow.camera_cpu(aspect=2.0)  # eye (13, 2, 3): the new sphere's centre
    p = rtow.make_params(32, 16, 4, seed=9)
    got, st, want, segs = gpu_vs_oracle(rtow, gpu_ctx, big, cam, p, accel)
    assert_bit_exact(got, st, want, segs)
    if ends:
        assert segs == 32 * 16 * 4 and not got.any()
    else:
        assert segs > 32 * 16 * 4


def test_scene_upload_rejects_non_finite_centres(rtow, gpu_ctx):
    s = rtow.final_scene()
    cx = s.cx.copy()
    cx[5] = np.nan
    bad = rtow.Scene(cx, s.cy, s.cz, s.radius, s.kind, s.albedo, s.param)
    with pytest.raises(Exception, match="rt_scene_upload"):
        gpu_ctx.upload(bad)
    gpu_ctx.upload(s)  # the context stays usable
    out, st = gpu_ctx.render(rtow.camera_cpu(aspect=2.0), rtow.make_params(16, 8, 1))
    assert st.segments > 0


def _with_extra_spheres(rtow, scene, spheres):
    """scene + spheres [(x, y, z, r, kind, (r, g, b), param), ...] appended."""
    import dataclasses
    ex = list(zip(*spheres))
    f32 = np.float32
    return dataclasses.replace(
        scene,
        cx=np.concatenate([scene.cx, np.array(ex[0], f32)]),
        cy=np.concatenate([scene.cy, np.array(ex[1], f32)]),
        cz=np.concatenate([scene.cz, np.array(ex[2], f32)]),
        radius=np.concatenate([scene.radius, np.array(ex[3], f32)]),
        kind=np.concatenate([scene.kind, np.array(ex[4], np.uint32)]),
        albedo=np.concatenate([scene.albedo, np.array(ex[5], f32).reshape(-1, 3)]),
        param=np.concatenate([scene.param, np.array(ex[6], f32)]))


@pytest.mark.parametrize("n_big", [12, 13])  # 4 + 12 = 16 spheres off the layer (layer mode), 17 (not)
def test_bvh_layer_mode_boundary_bit_exact(rtow, gpu_ctx, n_big):
    """Layer mode (the BVH over the thin layer of small spheres, the rest scanned
    as pairs) and the plain BVH, on either side of its kMaxExtra = 16 limit, with
    layer members of another radius inside the layer's y-range and a sphere that
    pokes out of it: bit-exact vs the brute-force oracle, and BVH == scan."""
    rng = np.random.default_rng(n_big)
    extra = [(float(rng.uniform(-9, 9)), 1.0 + float(rng.uniform(0, 1)), float(rng.uniform(-9, 9)),
              0.6 + 0.3 * float(rng.uniform()), i % 3, (0.7, 0.5, 0.3), 1.5 if i % 3 == 2 else 0.2)
             for i in range(n_big - 1)]
    extra += [(2.0, 0.25, 2.0, 0.2, 0, (0.9, 0.2, 0.2), 0.0)]     # pokes above the layer
    extra += [(1.0, 0.2, -2.0, 0.15, 1, (0.8, 0.8, 0.8), 0.1),    # inside the layer's y-range
              (-1.5, 0.2, 2.5, 0.1, 2, (1.0, 1.0, 1.0), 1.5)]
    scene = _with_extra_spheres(rtow, rtow.final_scene(), extra)
    cam = rtow.camera_cpu(aspect=96 / 54)
    p = rtow.make_params(96, 54, 6, seed=9)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, ACCELS["bvh"]))
    cam = rtow.camera_cpu(aspect=640 / 360)
    p = rtow.make_params(640, 360, 8, seed=10)
    a, sa = gpu_ctx.render(cam, p)
    p.flags |= ACCELS["bvh"]
    b, sb = gpu_ctx.render(cam, p)
    assert sa.segments == sb.segments
    assert np.array_equal(a, b)


@pytest.mark.parametrize("view", ["grazing", "axis", "below", "inside"])
def test_layer_grid_walk_edge_cases(rtow, gpu_ctx, view):
    """The layer grid's per-lane DDA on the rays that stress it: a camera in the
    layer looking along it (rays cross the whole grid, many nearly horizontal),
    an axis-aligned view (direction components exactly 0 for the centre
    column / row), a camera under the layer looking up through it, and one
    inside the grid looking down.  Bit-exact vs the oracle at a small size;
    grid == layer BVH == scan at a larger one."""
    looks = {"grazing": ((12.0, 0.2, 1.3), (-11.0, 0.18, -1.0)),
             "axis": ((0.0, 0.3, 14.0), (0.0, 0.3, 0.0)),
             "below": ((0.5, -0.5, 0.5), (3.0, 2.0, 2.0)),
             "inside": ((-2.0, 1.2, -3.0), (1.0, 0.0, 2.5))}[view]
    scene = rtow.final_scene()
    cam = rtow.camera_cpu(lookfrom=looks[0], lookat=looks[1], aspect=64 / 36)
    p = rtow.make_params(64, 36, 5, seed=31)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, ACCELS["bvh"]))
    cam = rtow.camera_cpu(lookfrom=looks[0], lookat=looks[1], aspect=480 / 270)
    p = rtow.make_params(480, 270, 16, seed=32)
    a, sa = gpu_ctx.render(cam, p)
    for acc in (ACCELS["bvh"], ACCELS["layer_bvh"]):
        p.flags = acc
        b, sb = gpu_ctx.render(cam, p)
        assert sa.segments == sb.segments
        assert np.array_equal(a, b), (view, acc)


@pytest.mark.parametrize("n_small", [80, 300])  # >= 64: layer mode; the grid builds / does not (> 15 per cell)
def test_dense_layer_grid_build_paths(rtow, gpu_ctx, n_small):
    """A dense layer (small spheres crowded into 1.5 x 1.5, overlapping): with 80
    the grid builds (its cells may shrink to keep <= 15 spheres per cell); with
    300 no cell size does, no grid is built and the layer BVH walks.  Either
    way bit-exact vs the oracle, and equal to the scan."""
    import dataclasses
    rng = np.random.default_rng(n_small)
    f32 = np.float32
    n = n_small + 1
    kind = np.array([0] + [int(k) for k in rng.integers(0, 3, n_small)], np.uint32)
    base = rtow.final_scene()
    scene = dataclasses.replace(
        base,
        cx=np.array([0.0] + list(rng.uniform(-0.75, 0.75, n_small)), f32),
        cy=np.array([-1000.0] + [0.2] * n_small, f32),
        cz=np.array([0.0] + list(rng.uniform(-0.75, 0.75, n_small)), f32),
        radius=np.array([1000.0] + [0.2] * n_small, f32),
        kind=kind,
        albedo=rng.uniform(0.2, 0.9, (n, 3)).astype(f32),
        param=np.where(kind == 2, 1.5, 0.3).astype(f32))
    cam = rtow.camera_cpu(lookfrom=(3.0, 1.5, 2.0), lookat=(0.0, 0.1, 0.0), aspect=64 / 36)
    p = rtow.make_params(64, 36, 5, seed=41)
    assert_bit_exact(*gpu_vs_oracle(rtow, gpu_ctx, scene, cam, p, ACCELS["bvh"]))
    cam = rtow.camera_cpu(lookfrom=(3.0, 1.5, 2.0), lookat=(0.0, 0.1, 0.0), aspect=320 / 180)
    p = rtow.make_params(320, 180, 16, seed=42)
    a, sa = gpu_ctx.render(cam, p)
    for acc in (ACCELS["bvh"], ACCELS["layer_bvh"]):
        p.flags = acc
        b, sb = gpu_ctx.render(cam, p)
        assert sa.segments == sb.segments
        assert np.array_equal(a, b), (n_small, acc)


@pytest.mark.parametrize("case", ["one_launch", "units3", "launches", "spp4100", "dither", "global", "depth1"])
def test_wide_sums_bit_exact_vs_oracle(rtow, gpu_ctx, case, accel):
    """Albedos above 1: the final scene with one lambertian
    sphere at albedo (1.2, 1.5, 0.9) and a metal one at 1.3 renders with
    64-bit pixel sums and the radiance clamp -- bit-exact
    vs the oracle in every walk, through float stores (one launch), 64-bit
    atomics into the context's scratch frame (units 3, or several bounded
    launches), 4100 spp (F = 31 with these albedos: no dither), the dither of
    the 64-bit format itself (a 2x2 frame at 2^19 spp with the metal sphere
    at albedo 1.5: vcap = 2^24, F = 62 - 19 - 24 = 19 < 20), the
    grid in global memory (the default placement is cells in LDS: 3 KB more
    static LDS), and depth 1 (vcap 1)."""
    import dataclasses
    base = rtow.final_scene()
    alb = base.albedo.copy()
    lam = int(np.nonzero(base.kind == rtow.RT_LAMBERTIAN)[0][5])
    met = int(np.nonzero(base.kind == rtow.RT_METAL)[0][3])
    alb[lam] = (1.2, 1.5, 0.9)
    alb[met] = (1.3, 1.3, 1.3)
    alb[0] = (1.02, 1.02, 1.02)  # the ground
    if case == "dither":
        alb[met] = (1.5, 1.5, 1.5)
    hot = dataclasses.replace(base, albedo=alb)
    cam = rtow.camera_cpu(aspect=2.0)
    spp = {"spp4100": 4100, "units3": 12, "dither": 1 << 19}.get(case, 24)
    w, h = (2, 2) if case == "dither" else (48, 24)
    p = rtow.make_params(w, h, spp, seed=31, max_depth=1 if case == "depth1" else 50,
                         units=3 if case == "units3" else 0)
    if case == "dither":  # the 64-bit format's F (rt_api.cpp sum_format) is below 20
        vcap = min(1.5 ** 49, 2.0 ** 24)
        assert 62 - int(np.floor(np.log2(spp))) - int(np.ceil(np.log2(vcap))) == 19
    if case == "launches":
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 48 * 24 * 5)
    try:
        if case == "global":
            gpu_ctx.upload(hot, grid_mode="global")
            want, segs = kernel_render(hot, cam, p)
            p.flags |= accel
            got, st = gpu_ctx.render(cam, p)
        else:
            assert rtow.accel_info(hot)["grid_placement"] == rtow.RT_GRID_CELLS_LDS  # 3 KB more static LDS
            got, st, want, segs = gpu_vs_oracle(rtow, gpu_ctx, hot, cam, p, accel)
    finally:
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 0)
        gpu_ctx.set_option(rtow.RT_OPT_GRID_PLACEMENT, rtow.RT_GRID_AUTO)
    assert_bit_exact(got, st, want, segs)
    if case == "launches":
        assert st.launches > 1
    assert got.max() > 0
