"""GPU tests at the BASELINE.json configs (C1, C3, C4) and on the context's
buffer lifecycle.

  C1  1x MI355X, 1920x1080 @ 100 spp (the automatic chunk split: units = 2)
  C3  8x MI355X, 7680x4320 @ 1000 spp: one rank's 1/8 band (world = 8), run
      here on one GPU at reduced spp -- rank 0 and rank 7
  C4  8x MI355X, 16384x16384, 10 000 spheres @ 2000 spp: rank 0's 1/8 band

Each asserts the accelerated walk (layer grid, the bench default) equals the
brute-force scan -- or the layer BVH where the scan is too slow -- bit for bit
with equal segment counts, plus an 8-row slice checked against the oracle's
kernel-mode restatement (the loop of /root/reference/src/cpu/main.cc:111-123).
"""
import numpy as np
import pytest

from oracle_lib import kernel_render

pytestmark = pytest.mark.gpu

GRID = 1 << 9                 # RT_FLAG_ACCEL_BVH: the layer grid on layer scenes
LAYER_BVH = (1 << 9) | (1 << 12)


def band_params(rtow, W, H, spp, world, rank, rows=None, **kw):
    """Rank `rank`'s interleaved 8-row bands of a `world`-way split; rows=8
    keeps only its first band (global rows rank*8 .. rank*8+7)."""
    p = rtow.make_params(W, H, spp, rank=rank, world=world, row_block=8, **kw)
    if rows is not None:
        p.local_rows = rows
    return p


def same(a, sa, b, sb):
    n_diff = int((a != b).sum())
    assert n_diff == 0, f"{n_diff} floats differ"
    assert sa.segments == sb.segments


def test_c1_full_frame_100spp_grid_equals_scan(rtow, gpu_ctx):
    """C1 at its own spp: 1920x1080 has 32 400 tiles, so the automatic units
    splits every pixel's two chunks (64 + 36) over 2 waves; the grid walk and
    the scan give the same sums, and so do units = 1 and the pilot schedule."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=1920 / 1080)
    p = rtow.make_params(1920, 1080, 100, seed=100)
    a, sa = gpu_ctx.render(cam, p)
    assert sa.samples == 1920 * 1080 * 100
    for flags, units in ((GRID, 0), (GRID, 1), (GRID | rtow.RT_FLAG_PILOT_SCHEDULE, 0)):
        q = rtow.make_params(1920, 1080, 100, seed=100, flags=flags, units=units)
        b, sb = gpu_ctx.render(cam, q)
        same(a, sa, b, sb)
    assert np.isfinite(a).all() and a.max() <= 100 + 1e-3


@pytest.mark.parametrize("rank", [0, 5])
def test_c1_band_bit_exact_vs_oracle(rtow, gpu_ctx, oracle, rank):
    """One 8-row band of C1 (rows rank*8.. of an 8-way split) at 100 spp,
    chunks split over 2 waves: bit-exact vs the oracle on those rows."""
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=1920 / 1080)
    p = band_params(rtow, 1920, 1080, 100, 8, rank, rows=8, seed=101, flags=GRID, units=2)
    got, st = gpu_ctx.render(cam, p)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs


@pytest.mark.parametrize("rank", [0, 7])
def test_c3_rank_share_grid_equals_scan(rtow, gpu_ctx, rank):
    """C3 (7680x4320, 8 GPUs): rank 0's and rank 7's whole 1/8 share (544
    rows in 8-row bands, 536 of them inside the frame for ranks 4-7) at 130
    spp (three chunks): the scan in one wave per tile == the grid with the
    pilot schedule (automatic units) == the grid with every tile's chunks
    split over 3 waves."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=7680 / 4320)
    p = band_params(rtow, 7680, 4320, 130, 8, rank, seed=300, units=1)
    # 540 bands of 8 rows over 8 ranks: every rank holds 68 band slots (544
    # rows, padded so tiles are equal); rank 7's last slot lies past row 4319
    assert p.local_rows == 544
    valid = int((rtow.local_to_global_rows(p) < 4320).sum())
    assert valid == (544 if rank < 4 else 536)
    a, sa = gpu_ctx.render(cam, p)
    assert sa.samples == 7680 * valid * 130
    for flags, units in ((GRID | rtow.RT_FLAG_PILOT_SCHEDULE, 0), (GRID, 3)):
        q = band_params(rtow, 7680, 4320, 130, 8, rank, seed=300, flags=flags, units=units)
        b, sb = gpu_ctx.render(cam, q)
        same(a, sa, b, sb)


@pytest.mark.parametrize("rank", [0, 7])
def test_c3_band_bit_exact_vs_oracle(rtow, gpu_ctx, oracle, rank):
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=7680 / 4320)
    p = band_params(rtow, 7680, 4320, 6, 8, rank, rows=8, seed=301, flags=GRID)
    got, st = gpu_ctx.render(cam, p)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs


def test_c4_rank_share_grid_equals_layer_bvh_and_scan(rtow, gpu_ctx):
    """C4 (16384x16384, 10 000 spheres, 8 GPUs): rank 0's whole 1/8 share
    (2048 rows of 16384) at 2 spp: layer grid == layer BVH == brute-force scan
    (10 004 tests per segment), on a scene whose grid has ~10 000 cells."""
    scene = rtow.final_scene(half_extent=50)
    assert 9900 < scene.n <= 10004
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=1.0)
    p = band_params(rtow, 16384, 16384, 2, 8, 0, seed=400, flags=GRID)
    assert p.local_rows == 2048
    a, sa = gpu_ctx.render(cam, p)
    for flags in (LAYER_BVH, 0):
        q = band_params(rtow, 16384, 16384, 2, 8, 0, seed=400, flags=flags)
        b, sb = gpu_ctx.render(cam, q)
        same(a, sa, b, sb)


def test_c4_band_bit_exact_vs_oracle(rtow, gpu_ctx, oracle):
    """One 8-row band of C4 (rank 3 of 8) at 1 spp, bit-exact vs the oracle's
    brute-force restatement over all 10 004 spheres."""
    scene = rtow.final_scene(half_extent=50)
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=1.0)
    p = band_params(rtow, 16384, 16384, 1, 8, 3, rows=8, seed=401, flags=GRID)
    got, st = gpu_ctx.render(cam, p)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs


def test_chunk_buffer_survives_frame_growth(rtow):
    """on one fresh context, a split-chunk render (units 2),
    then a larger frame through rt_render (which grows the context's frame
    buffer), then the first render again: the third image is bit-identical to
    the first (the chunk buffer was neither freed nor reused by the frame),
    and the context is destroyed cleanly."""
    cam_s = rtow.camera_cpu(aspect=160 / 90)
    cam_b = rtow.camera_cpu(aspect=3840 / 2160)
    with rtow.Context(0) as ctx:
        ctx.upload(rtow.final_scene())
        p = rtow.make_params(160, 90, 100, seed=7, flags=GRID, units=2)
        first, s1 = ctx.render(cam_s, p)
        big, _ = ctx.render(cam_b, rtow.make_params(3840, 2160, 1, seed=8, flags=GRID))
        third, s3 = ctx.render(cam_s, p)
        assert np.array_equal(first, third) and s1.segments == s3.segments
        # and a bigger split render after that (the chunk buffer grows)
        q = rtow.make_params(640, 360, 130, seed=9, flags=GRID, units=3)
        c, sc = ctx.render(rtow.camera_cpu(aspect=640 / 360), q)
        q.units = 1
        d, sd = ctx.render(rtow.camera_cpu(aspect=640 / 360), q)
        assert np.array_equal(c, d) and sc.segments == sd.segments
        again, _ = ctx.render(cam_s, p)
        assert np.array_equal(first, again)


def test_async_renders_on_two_streams_are_ordered(rtow):
    """two split-chunk renders of one context enqueued on
    two different streams share the chunk buffer; the context orders them
    (the second waits for the first's event), so both images are right."""
    import torch
    with rtow.Context(0) as ctx:
        ctx.upload(rtow.final_scene())
        cam = rtow.camera_cpu(aspect=320 / 180)
        pa = rtow.make_params(320, 180, 200, seed=11, flags=GRID, units=4)
        pb = rtow.make_params(320, 180, 200, seed=12, flags=GRID, units=4)
        want_a, _ = ctx.render(cam, pa)
        want_b, _ = ctx.render(cam, pb)
        dev = torch.device("cuda", 0)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        ta = torch.zeros((180, 320, 3), dtype=torch.float32, device=dev)
        tb = torch.zeros_like(ta)
        torch.cuda.synchronize(dev)
        for _ in range(3):
            ctx.render_async(cam, pa, ta.data_ptr(), s1.cuda_stream)
            ctx.render_async(cam, pb, tb.data_ptr(), s2.cuda_stream)
        torch.cuda.synchronize(dev)
        assert np.array_equal(ta.cpu().numpy(), want_a)
        assert np.array_equal(tb.cpu().numpy(), want_b)


def test_grid_refit_between_async_renders_on_two_streams(rtow, oracle):
    """RT_OPT_GRID_FIT (default on) refits the layer grid in place
    inside render_enqueue, so a render with camera B overwrites the grid
    buffers that camera A's render, still pending on another stream, reads.
    Uploaded with defaults, A (fits 1.11) and B (fits 1.22) alternate on two
    streams with no host sync between them: both images and segment counts
    equal the oracle's, and after each render the context's cell scale is the
    host model's pick for that geometry (rtow.grid_fit).  (The capacity-growth
    branch of the refit is not reached: every candidate is at least as coarse
    as the builder's grid, so it never needs larger buffers.)"""
    import torch
    scene = rtow.final_scene()
    W, H = 320, 180
    cam_a = rtow.camera_cpu(aspect=W / H)
    cam_b = rtow.camera_cpu(lookfrom=(6, 1, 12), aspect=W / H)
    fit_a, fit_b = rtow.grid_fit(scene, cam_a, W, H)[0], rtow.grid_fit(scene, cam_b, W, H)[0]
    assert fit_a != fit_b, (fit_a, fit_b)  # precondition: B's render refits the grid
    pa = rtow.make_params(W, H, 24, seed=31, flags=GRID, units=2)
    pb = rtow.make_params(W, H, 24, seed=32, flags=GRID, units=2)
    want_a, segs_a = kernel_render(scene, cam_a, pa)
    want_b, segs_b = kernel_render(scene, cam_b, pb)
    with rtow.Context(0) as ctx:
        ctx.upload(scene)
        dev = torch.device("cuda", 0)
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        ta = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)
        tb = torch.zeros_like(ta)
        torch.cuda.synchronize(dev)
        ctx.render_async(cam_a, pa, ta.data_ptr(), s1.cuda_stream)
        assert ctx.grid_scale() == pytest.approx(fit_a, abs=1e-12)
        ctx.render_async(cam_b, pb, tb.data_ptr(), s2.cuda_stream)  # refits while A may be pending
        assert ctx.grid_scale() == pytest.approx(fit_b, abs=1e-12)
        torch.cuda.synchronize(dev)
        st_b = ctx.collect_stats()
        assert np.array_equal(ta.cpu().numpy(), want_a)
        assert np.array_equal(tb.cpu().numpy(), want_b)
        assert st_b.segments == segs_b
        # and back to A on the second stream, then B on the first
        for cam, p, t, s, fit, want, segs in ((cam_a, pa, tb, s2, fit_a, want_a, segs_a),
                                              (cam_b, pb, ta, s1, fit_b, want_b, segs_b)):
            ctx.render_async(cam, p, t.data_ptr(), s.cuda_stream)
            assert ctx.grid_scale() == pytest.approx(fit, abs=1e-12)
            torch.cuda.synchronize(dev)
            assert np.array_equal(t.cpu().numpy(), want)
            assert ctx.collect_stats().segments == segs


def test_pilot_first_render_is_asynchronous_and_correct(rtow):
    """The pilot schedule's first render of a geometry enqueues the pilot, the
    device sort and the render without a host sync; the result equals launch
    order, and a different geometry afterwards gets its own order."""
    import torch
    with rtow.Context(0) as ctx:
        ctx.upload(rtow.final_scene())
        dev = torch.device("cuda", 0)
        st = torch.cuda.Stream(dev)
        for (w, h, spp, units) in ((640, 360, 80, 0), (200, 120, 130, 3)):
            cam = rtow.camera_cpu(aspect=w / h)
            want, _ = ctx.render(cam, rtow.make_params(w, h, spp, seed=5, flags=GRID, units=units))
            t = torch.zeros((h, w, 3), dtype=torch.float32, device=dev)
            torch.cuda.synchronize(dev)
            p = rtow.make_params(w, h, spp, seed=5, flags=GRID | rtow.RT_FLAG_PILOT_SCHEDULE, units=units)
            ctx.render_async(cam, p, t.data_ptr(), st.cuda_stream)
            ctx.render_async(cam, p, t.data_ptr(), st.cuda_stream)  # cached order
            torch.cuda.synchronize(dev)
            assert np.array_equal(t.cpu().numpy(), want), (w, h)


def test_lds_resident_grid_equals_global_grid(rtow, gpu_ctx):
    """The layer grid copied into LDS (render_kernel placement kGridLds, the
    default when it fits 17 KB), its cells alone in LDS (kGridCells) and the
    grid read from global memory (RT_OPT_GRID_PLACEMENT) give the same bits,
    with split units and the pilot schedule too."""
    cam = rtow.camera_cpu(aspect=640 / 360)
    outs = []
    for mode in ("global", "lds", "cells"):
        gpu_ctx.upload(rtow.final_scene(), grid_mode=mode)
        for flags, units in ((GRID, 1), (GRID | rtow.RT_FLAG_PILOT_SCHEDULE, 3)):
            outs.append(gpu_ctx.render(cam, rtow.make_params(640, 360, 130, seed=21, flags=flags, units=units)))
    ref, sref = outs[0]
    for img, st in outs[1:]:
        same(ref, sref, img, st)


@pytest.mark.gpu
def test_scene_upload_albedo_domain(rtow):
    """rt_scene_upload takes every finite albedo >= 0 (the reference's
    constructors take any colour, src/cpu/material.h:17,38; above 1 the render
    uses 64-bit pixel sums) and refuses a negative or
    non-finite lambertian / metal albedo with RT_ERR_INVALID, keeping the
    previous scene; a dielectric's albedo is ignored, as the kernel ignores
    it.  An albedo of exactly 1 keeps the 32-bit format (same bits as before)."""
    import dataclasses
    base = rtow.final_scene()
    with rtow.Context(0) as ctx:
        ctx.upload(base)
        cam = rtow.camera_cpu(aspect=16 / 9)
        prm = rtow.make_params(32, 18, 4, seed=3, flags=rtow.RT_FLAG_ACCEL_BVH)
        before, _ = ctx.render(cam, prm)
        lam = int(np.nonzero(base.kind == rtow.RT_LAMBERTIAN)[0][0])
        die = int(np.nonzero(base.kind == rtow.RT_DIELECTRIC)[0][0])
        for bad in (-1e-7, float("nan"), float("inf")):
            alb = base.albedo.copy()
            alb[lam, 1] = bad
            with pytest.raises(rtow.RTError) as ei:
                ctx.upload(dataclasses.replace(base, albedo=alb))
            assert ei.value.status == rtow.RT_ERR_INVALID
        after, _ = ctx.render(cam, prm)
        assert np.array_equal(before, after)  # the previous scene stayed
        alb = base.albedo.copy()
        alb[die] = 7.0  # ignored for a dielectric
        ctx.upload(dataclasses.replace(base, albedo=alb))
        same, _ = ctx.render(cam, prm)
        assert np.array_equal(before, same)
        for hot in (1.0001, 3.0, 1e30):  # accepted: bit-exact vs the oracle
            alb = base.albedo.copy()
            alb[lam] = hot
            sc = dataclasses.replace(base, albedo=alb)
            ctx.upload(sc)
            got, st = ctx.render(cam, prm)
            want, segs = kernel_render(sc, cam, prm)
            assert np.array_equal(got, want) and st.segments == segs, hot
            assert np.isfinite(got).all()


# ---- round 3: the configs at their own sample counts, the sum format's
# ---- headroom, its stochastic rounding, bounded launches, grid placements

@pytest.mark.parametrize("units", [1, 0])
def test_c3_band_at_1000spp_bit_exact_vs_oracle(rtow, gpu_ctx, oracle, units):
    """C3 at its own 1000 spp (F = 22: a sample adds up to 2^22, 1000 of them
    up to 4.19e9 of the uint32's 4.29e9): one full-width 8-row band of the
    7680x4320 frame (rank 0 of the 540-way band split), one wave per tile and
    the automatic split (8 units: the band has 960 tiles), bit-exact vs the
    oracle with equal segments (/root/reference/src/cpu/main.cc:111-123)."""
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=7680 / 4320)
    p = band_params(rtow, 7680, 4320, 1000, 540, 0, seed=310, flags=GRID, units=units)
    assert p.local_rows == 8
    got, st = gpu_ctx.render(cam, p)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs and st.samples == 7680 * 8 * 1000


@pytest.mark.parametrize("mode,units", [("cells", 1), ("cells", 0), ("global", 0)])
def test_c4_scene_at_2000spp_bit_exact_vs_oracle(rtow, gpu_ctx, oracle, mode, units):
    """C4's scene (10 000 spheres), camera (aspect 1) and own 2000 spp (F =
    21), rank 0's first 8-row band of a 64x64 frame split 8 ways (the
    oracle's brute force over 10 004 spheres sizes the frame), with the grid's
    cells in LDS (the automatic placement for this scene) and in global
    memory, one unit and the automatic split: bit-exact vs the oracle."""
    scene = rtow.final_scene(half_extent=50)
    gpu_ctx.upload(scene, grid_mode=mode)
    assert rtow.accel_info(scene, mode)["grid_placement"] == (rtow.RT_GRID_CELLS_LDS if mode == "cells"
                                                              else rtow.RT_GRID_GLOBAL)
    cam = rtow.camera_cpu(aspect=1.0)
    p = band_params(rtow, 64, 64, 2000, 8, 0, rows=8, seed=410, flags=GRID, units=units)
    got, st = gpu_ctx.render(cam, p)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())
    assert st.segments == segs


@pytest.mark.parametrize("half_extent", [11, 50])
def test_grid_cell_scales_render_the_oracle_image(rtow, gpu_ctx, oracle, half_extent):
    """The layer grid's cell size (RT_OPT_GRID_SCALE) is scheduling only: the
    headline scene (grid in LDS) and C4's (cells in LDS) uploaded at the
    builder's scale s0 and at s0 (1 + 0.01 k), k = 3, 7, 15, 30, and with the
    grid's origin shifted by a fraction of a cell (RT_OPT_INTERNAL_GRID_PHASE_X / _Z),
    render the oracle's image bit for bit with equal segments (the lists hold
    every sphere that can win)."""
    scene = rtow.final_scene(half_extent=half_extent)
    W, H = (64, 36) if half_extent == 11 else (64, 64)
    cam = rtow.camera_cpu(aspect=W / H)
    p = band_params(rtow, W, H, 64, 4, 1, rows=8, seed=515, flags=GRID)
    want, segs = kernel_render(scene, cam, p)
    s0 = rtow.accel_info(scene)["grid_scale_milli"] / 1000.0
    try:
        for k, ph in ((0, (0, 0)), (3, (0, 0)), (7, (0, 0)), (15, (0, 0)), (30, (0, 0)), (0, (0.5, 0.25)),
                      (7, (0.75, 0.875))):
            gpu_ctx.upload(scene, grid_mode="auto", grid_scale=s0 * (1.0 + 0.01 * k), grid_phase=ph)
            got, st = gpu_ctx.render(cam, p)
            assert np.array_equal(got, want), (k, ph, int((got != want).sum()))
            assert st.segments == segs, (k, ph)
    finally:
        gpu_ctx.set_option(rtow.RT_OPT_GRID_SCALE, 0)
        gpu_ctx.set_option(rtow.RT_OPT_INTERNAL_GRID_PHASE_X, 0)
        gpu_ctx.set_option(rtow.RT_OPT_INTERNAL_GRID_PHASE_Z, 0)
    for opt, bad in ((rtow.RT_OPT_INTERNAL_GRID_PHASE_X, 1.0), (rtow.RT_OPT_INTERNAL_GRID_PHASE_Z, -0.25)):
        with pytest.raises(rtow.RTError):
            gpu_ctx.set_option(opt, bad)


@pytest.mark.parametrize("spp", [1000, 2000, 2047, 4096])
def test_all_sky_frame_uses_the_sum_headroom_without_wrapping(rtow, gpu_ctx, oracle, spp):
    """A 64x64 frame of sky only (camera looking straight up): under src/cpu
    semantics a sky sample's blue radiance is exactly 1 (s0 + a with s0 = 1 -
    a), so every pixel's blue sum is spp * 2^F -- 4.19e9 at 1000 spp, 4.19e9
    at 2000, 4.29e9 at 2047, within 2^F of the uint32 limit -- and must come
    out as exactly spp, with no wrap; red and green equal the oracle's bits.
    4096 spp runs the stochastic rounding (F = 19)."""
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(lookfrom=(30, 5, 30), lookat=(30, 100, 30.001), vup=(0, 0, 1), vfov=20.0, aspect=1.0,
                          aperture=0.0)
    p = rtow.make_params(64, 64, spp, seed=5, flags=GRID)
    got, st = gpu_ctx.render(cam, p)
    assert st.segments == 64 * 64 * spp  # one segment per sample: all sky
    assert np.all(got[..., 2] == np.float32(spp))
    assert np.all(got[..., :2] <= spp) and np.all(got[..., :2] > 0.5 * spp)
    want, segs = kernel_render(scene, cam, p)
    assert np.array_equal(got, want), int((got != want).sum())


def test_stochastic_rounding_bit_exact_vs_oracle(rtow, gpu_ctx, oracle):
    """spp >= 4096 switches the sums to stochastic rounding (F < 20): the
    kernel's dither draw and rounding equal the oracle's bit for bit, on the
    final scene at 4096 spp, with units 1 and 5 and two bounded launches."""
    scene = rtow.final_scene()
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=32 / 18)
    p = rtow.make_params(32, 18, 4096, seed=44, flags=GRID, units=1)
    want, segs = kernel_render(scene, cam, p)
    for units, budget in ((1, 0), (5, 0), (1, 32 * 18 * 2048)):
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, budget)
        p.units = units
        got, st = gpu_ctx.render(cam, p)
        assert np.array_equal(got, want), (units, budget, int((got != want).sum()))
        assert st.segments == segs and st.launches == (2 if budget else 1)
    gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 0)


def test_strided_ranges_times_sample_ranges_give_the_same_image(rtow, gpu_ctx):
    """A plan with both splits (rt_api.cpp plan_launches): 256x256 at 1000 spp
    under a 2^22 budget would leave 62 spp per wave in sample ranges alone,
    so it runs 4 strided entry ranges x 4 sample ranges of 250 spp; with 3
    units per tile (about 83 spp per wave in each unit's share) as 16 entry
    ranges.  Bit-identical to the one-launch render."""
    gpu_ctx.upload(rtow.final_scene())
    cam = rtow.camera_cpu(aspect=1.0)
    p = rtow.make_params(256, 256, 1000, seed=77, flags=GRID, units=1)
    one, s1 = gpu_ctx.render(cam, p)
    assert s1.launches == 1
    try:
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 1 << 22)
        for units in (1, 3):
            p.units = units
            plan = rtow.launch_plan(p, 1 << 22)
            assert (plan["ranges"], plan["chunks"]) == ((4, 4) if units == 1 else (16, 1)), plan
            img, st = gpu_ctx.render(cam, p)
            assert st.launches == plan["launches"]
            assert np.array_equal(img, one) and st.segments == s1.segments, units
    finally:
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 0)


def test_bounded_launches_give_the_same_image(rtow, gpu_ctx):
    """a render is split into launches of about
    RT_OPT_LAUNCH_SAMPLES samples at most.  C4's rank-0 share (2048 x 16384
    pixels, 10 000 spheres) at 16 spp (too few samples to split) with a
    budget of 2^26 samples runs as 8 strided entry-range launches with all 16
    samples each (float stores, no atomics); with 2 units per tile and a
    2.0e8 budget as 3; with a 2^24 budget as 32.  Every image and segment
    count equals the one-launch render bit for bit.  At the default budget
    (2^35) the headline frame (3840x2160x500 = 4.15e9 samples) stays one
    launch, and C4's full share at 2000 spp (6.7e10) is 2 sample ranges
    (test_host.py test_launch_plan)."""
    scene = rtow.final_scene(half_extent=50)
    gpu_ctx.upload(scene)
    cam = rtow.camera_cpu(aspect=1.0)
    p = band_params(rtow, 16384, 16384, 16, 8, 0, seed=420, flags=GRID, units=1)
    one, s1 = gpu_ctx.render(cam, p)
    assert s1.launches == 1
    for budget, units, launches in ((1 << 26, 1, 8), (2048 * 16384 * 6, 2, 3), (1 << 24, 1, 32)):
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, budget)
        p.units = units
        img, st = gpu_ctx.render(cam, p)
        assert st.launches == launches
        same(one, s1, img, st)
        assert st.kernel_ms / st.launches < 1000.0
    gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, 0)
    with pytest.raises(rtow.RTError):
        gpu_ctx.set_option(rtow.RT_OPT_LAUNCH_SAMPLES, -5)
