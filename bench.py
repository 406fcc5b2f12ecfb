#!/usr/bin/env python3
"""Headline benchmark: Mray/s on the final random-spheres scene, 3840x2160 @ 500 spp,
depth 50 (BASELINE.json `metric`, config 3), on 1..8 MI355X of one node.

One step = one full frame: every rank renders its interleaved row bands
 with the HIP kernel through the C ABI (rt_render_async on a
dedicated torch stream, device-resident frame tile), then rank 0 gathers the
tiles with one RCCL gather over xGMI (rtow_dist.py).  Strong scaling: the frame is fixed, N GPUs
split it.  `value` = closest-hit queries (ray segments) of all ranks per
second of the max-over-ranks wall time / 1e6.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Extra objects on the JSON line:
  roofline     fp32 VALU roofline of the render kernel: executed flops (ray-sphere
               tests x 17 + grid cell steps x 2, counted in-kernel) per launch /
               average launch time from HIP events on the launch stream, against
               157.3 TFLOP/s; plus the VALU issue rate against the wave64 2-cycle
               ceiling at the measured clock, HBM GB/s against 8 TB/s and the
               VALU lane utilisation, from the committed rocprofv3 PMC summary
               of the same kernel (profiles/pmc_traffic_bvh.json)
  cpu_baseline the reference's own src/cpu (oracle/_ref, built from
               /root/reference sources) at C0 (400x225 @ 10 spp): one process
               per host core (up to 16, the box's CPU share) rendering the same
               frame, aggregate Mray/s; the 1-core figure beside it.  Falls back
               to the oracle's fp64 restatement (kind "port")
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ray-tracing-in-one-weekend_amd")
sys.path.insert(0, PKG)

PEAK_FP32_TFLOPS = 157.3      # MI355X vector fp32 (MI355X_MICROARCH.md, chip table)
PEAK_HBM_GBPS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)
N_SIMD = 1024                 # 256 CUs x 4 SIMDs
N_XCD = 8                     # GRBM_GUI_ACTIVE is summed over the 8 XCDs
FLOPS_PER_TEST = 17           # algorithmic flops per ray-sphere test
FLOPS_PER_BOX = 12            # slab test: 6 fma (2 flop) per ray-box test (layer BVH walk)
FLOPS_PER_CELL = 2            # layer grid walk: one compare + one add per DDA cell step
# wave64 VALU issue ceiling: one independent v_fma_f32 per 1.041 ns per SIMD
# with all 64 lanes active (tools/ubench_exec.hip on MI355X), 256 CUs x 4 SIMDs
VALU_ISSUE_PEAK = 1024 / 1.041e-9  # wave instructions per second


# BASELINE.json configs: (width, height, spp, half_extent of the sphere grid).  c2 is the
# headline metric's config and the default; the others are for documentation
# runs (`--preset c3` is what each of 8 GPUs renders 1/8 of, c4 is the
# 10 000-sphere occupancy stress).
PRESETS = {"c1": (1920, 1080, 100, 11), "c2": (3840, 2160, 500, 11),
           "c3": (7680, 4320, 1000, 11), "c4": (16384, 16384, 2000, 50)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", choices=sorted(PRESETS), default="",
                    help="BASELINE config (sets --width/--height/--spp/--half-extent)")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--half-extent", type=int, default=11, help="11: 486 spheres; 50: 10k spheres")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--accel", choices=["scan", "bvh", "layer_bvh"], default="bvh",
                    help="bvh: acceleration structures (default): the final scene is a layer "
                         "scene, so the per-lane layer grid walk; layer_bvh: the wave-uniform "
                         "layer BVH walk instead; scan: brute-force closest hit.  All three give "
                         "the same image (tested on the full headline frame)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse the multi-process path "
                         "on a one-GPU box (tiles staged through host memory)")
    ap.add_argument("--cpu-spp", type=int, default=10, help="spp of the bounded CPU sample (400x225: C0)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="concurrent reference processes for the all-cores figure (0: min(16, cpu count))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pilot", action="store_true",
                    help="launch tiles in index order (no RT_FLAG_PILOT_SCHEDULE)")
    ap.add_argument("--out", default="", help="write the gathered frame as PPM (P6 if .pgm/.p6)")
    a = ap.parse_args()
    if a.preset:
        a.width, a.height, a.spp, a.half_extent = PRESETS[a.preset]
    return a


def _ref_run(harness, spp):
    return subprocess.Popen([harness, "render", "400", "16", "9", str(spp), "50", "final", "0"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)


def cpu_baseline(spp, procs):
    """Reference src/cpu (compiled from /root/reference by oracle/Makefile) at C0
    geometry (400x225, depth 50, `spp` samples): one process on one core, then
    `procs` processes at once (the reference is single-threaded; its threaded
    variant src/cpu-multi-threading is racy and out of scope), each
    rendering the same frame: aggregate segments / wall time."""
    sample = f"final scene 400x225 @ {spp} spp, depth 50 (C0)"
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if os.path.exists(harness):
        def run_many(n):
            t = time.perf_counter()
            ps = [_ref_run(harness, spp) for _ in range(n)]
            segs = 0
            for p in ps:
                _, err = p.communicate(timeout=600)
                if p.returncode != 0:
                    raise RuntimeError(f"ref_harness exit {p.returncode}")
                segs += json.loads(err.decode().strip().splitlines()[-1])["segments"]
            return segs, time.perf_counter() - t
        s1, t1 = run_many(1)
        sn, tn = run_many(procs)
        one = {"value": round(s1 / t1 / 1e6, 4), "cores": 1, "seconds": round(t1, 3)}
        return {"value": round(sn / tn / 1e6, 4), "unit": "Mray/s", "cores": procs, "kind": "reference",
                "seconds": round(tn, 3), "single_core": one,
                "sample": f"{sample}: {procs} concurrent single-threaded processes of the reference "
                          f"src/cpu (g++ -O2), aggregate; single_core = one process alone"}
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    t = time.perf_counter()
    _, segs = oracle_lib.reference_render(400, 16.0 / 9.0, spp)
    dt = time.perf_counter() - t
    return {"value": round(segs / dt / 1e6, 4), "unit": "Mray/s", "cores": 1, "kind": "port",
            "seconds": round(dt, 3), "sample": sample + ", single thread (oracle fp64 restatement)"}


def load_pmc(workload, accel="scan", world=1):
    """The committed rocprofv3 PMC summary of this workload AND this rank share
    (tools/pmc_traffic.py; profiles/pmc_traffic_<accel>.json for the whole
    frame, pmc_traffic_<accel>_w<N>.json for rank 0's 1/N share): HBM bytes and
    VALU wave-instructions per launch.  Returns (summary or {}, reason)."""
    name = "pmc_traffic.json" if accel == "scan" else f"pmc_traffic_{accel}.json"
    if world > 1:
        name = name.replace(".json", f"_w{world}.json")
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}, f"no committed PMC summary for a {world}-way share ({name})"
    if d.get("workload") != workload:
        return {}, f"{name} was collected on another workload ({d.get('workload')!r})"
    if int(d.get("world", 1)) != world:
        return {}, f"{name} was collected on a {d.get('world', 1)}-way share, this line is {world}-way"
    d["path"] = path
    return d, None


def roofline(work, k_avg_s, accel, pmc, pmc_reason, device_sha):
    """The `roofline` object of the JSON line.  work: executed work of one launch
    (RT_FLAG_COUNT_WORK counters of this rank's share); k_avg_s: this run's
    average render time of that share; pmc: the committed PMC summary of the
    SAME share (load_pmc), or {} -- then every counter-derived field is null
    and `pmc_null_reason` says why (counters of another share divided by this
    share's time would be meaningless)."""
    # box_tests counts slab tests (layer BVH) or DDA cell steps (layer grid)
    flops = work["sphere_tests"] * FLOPS_PER_TEST + work["box_tests"] * (
        FLOPS_PER_CELL if accel == "bvh" else FLOPS_PER_BOX)
    achieved = flops / k_avg_s / 1e12
    # the counters are only valid for the device code they were collected on:
    # a summary of other kernel code keeps its name and hash in the line, but
    # every field derived from it is null (Weak 4)
    pmc_fresh = bool(pmc) and pmc.get("device_code_sha16") == device_sha
    pmc_src = os.path.relpath(pmc["path"], ROOT) if pmc.get("path") else None
    if pmc and not pmc_fresh:
        pmc_reason = (f"{pmc_src or 'the PMC summary'} was collected on device code "
                      f"{pmc.get('device_code_sha16')}, this build is {device_sha}: its counters are not used")
        pmc = {}
    valu_insts = pmc.get("valu_insts_per_launch")
    cnt = pmc.get("counters_avg_per_dispatch", {})
    traffic = pmc.get("hbm_bytes_per_launch")
    clock_ghz = (cnt["GRBM_GUI_ACTIVE"] / N_XCD / k_avg_s / 1e9) if cnt.get("GRBM_GUI_ACTIVE") else None
    valu_issue = None
    if valu_insts:
        rate = valu_insts / k_avg_s
        valu_issue = {"achieved": round(rate / 1e9, 1), "unit": "G wave-instr/s",
                      "source": "SQ_INSTS_VALU per launch (committed PMC summary of this share) / this "
                                "run's kernel time"}
        if clock_ghz:
            peak2 = N_SIMD * clock_ghz * 1e9 / 2  # one wave64 VALU instruction per 2 cycles per SIMD
            valu_issue.update({"peak": round(peak2 / 1e9, 1), "frac": round(rate / peak2, 3),
                               "clock_ghz": round(clock_ghz, 3),
                               "peak_basis": "wave64 VALU issue every 2 cycles per SIMD "
                                             "(MI355X_MICROARCH.md) x 1024 SIMDs at the clock from "
                                             "GRBM_GUI_ACTIVE / 8 XCDs / kernel time"})
        valu_issue.update({"peak_ubench": round(VALU_ISSUE_PEAK / 1e9, 1),
                           "frac_ubench": round(rate / VALU_ISSUE_PEAK, 3),
                           "peak_ubench_basis": "dependency-free v_fma_f32 stream, 1.041 ns per "
                                                "wave instruction per SIMD (tools/ubench_exec.hip)"})
    lane_util = None
    if cnt.get("SQ_THREAD_CYCLES_VALU") and cnt.get("SQ_ACTIVE_INST_VALU"):
        lane_util = round(cnt["SQ_THREAD_CYCLES_VALU"] / (64.0 * cnt["SQ_ACTIVE_INST_VALU"]), 3)
    return {"bound": "valu", "achieved": round(achieved, 2), "peak": PEAK_FP32_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
            "traffic": traffic,
            "achieved_basis": "executed work per launch (RT_FLAG_COUNT_WORK frame of this rank's share): "
                              "ray-sphere tests x 17 flop + grid cell steps x 2 flop "
                              "(layer BVH: box tests x 12) / HIP-event kernel time",
            "valu_issue": valu_issue,
            "valu_lane_util": lane_util,
            "valu_lane_util_basis": "SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU): "
                                    "mean active lanes per VALU instruction / 64",
            "hbm": ({"achieved_GBps": round(traffic / k_avg_s / 1e9, 1),
                     "peak_GBps": PEAK_HBM_GBPS,
                     "frac": round(traffic / k_avg_s / 1e9 / PEAK_HBM_GBPS, 5)}
                    if traffic else None),
            "pmc_source": pmc_src,
            "pmc_matches_device_code": pmc_fresh,
            "pmc_null_reason": pmc_reason,
            "culling_speedup": round(work["bf_tests"] / max(1, work["sphere_tests"]), 1),
            "culling_speedup_basis": "brute-force ray-sphere tests (segments x spheres, "
                                     "SURVEY 8d) / tests the walk executes; not a roofline "
                                     "fraction",
            "note": "fp32 VALU-bound (no MFMA, HBM idle): the kernel is control-heavy "
                    "(compares, selects, branches, divergent per-lane walks), so "
                    "valu_issue and valu_lane_util say how close it runs to the issue "
                    "ceiling; frac counts only the algorithmic flops"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("for --gpus N > 1 launch with torch.distributed.run --nproc-per-node N")
    import numpy as np
    import torch
    import torch.distributed as dist
    import rtow
    import rtow_dist

    n_dev = torch.cuda.device_count()
    dev_idx = local_rank % n_dev  # == local_rank on a full node; wraps only for gloo rehearsal
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    W, H, spp = a.width, a.height, a.spp
    workload = f"final random-spheres scene {W}x{H} @ {spp}spp depth {a.depth}"
    if a.half_extent != 11:
        workload += f", sphere grid half-extent {a.half_extent}"
    scene = rtow.final_scene(a.half_extent)
    cam = rtow.camera_cpu(aspect=W / H)
    ctx = rtow.Context(dev_idx)
    ctx.upload(scene)
    params = rtow_dist.partition(W, H, spp, world, rank, a.row_block, max_depth=a.depth)
    params.flags |= rtow.RT_FLAG_KEEP_COUNTERS
    if not a.no_pilot:
        # launch the expensive tiles first: the 4-spp pilot that measures them
        # runs in the first (warmup) frame of this geometry; timed frames reuse
        # the order (include/rt.h RT_FLAG_PILOT_SCHEDULE)
        params.flags |= rtow.RT_FLAG_PILOT_SCHEDULE
    if a.accel in ("bvh", "layer_bvh"):
        params.flags |= rtow.RT_FLAG_ACCEL_BVH
    if a.accel == "layer_bvh":
        params.flags |= rtow.RT_FLAG_LAYER_BVH
    tile = torch.zeros((params.local_rows, W, 3), dtype=torch.float32, device=dev)
    # the step ends like the drop-in CLI's: write_color on the device (src/cpu
    # arithmetic) turns the tile's sums into bytes, and rank 0 gathers the byte
    # tiles (3 B per pixel instead of the 12 of the fp32 sums)
    tile_u8 = torch.zeros((params.local_rows, W, 3), dtype=torch.uint8, device=dev)
    gdev = dev if a.backend == "nccl" else torch.device("cpu")
    gather_list = ([torch.empty(tile_u8.shape, dtype=tile_u8.dtype, device=gdev) for _ in range(world)]
                   if (world > 1 and rank == 0) else None)
    # a dedicated stream: the kernel, the HIP events timing it and the RCCL gather
    # are all ordered on it (torch's default stream would reach the C ABI as NULL)
    stream = torch.cuda.Stream(dev)

    def barrier():
        if world > 1:
            if a.backend == "nccl":
                dist.barrier(device_ids=[dev_idx])
            else:
                dist.barrier()

    def step(i, events=None):
        params.seed = i
        if events is not None:
            events[0].record(stream)
        ctx.render_async(cam, params, tile.data_ptr(), stream.cuda_stream)
        if events is not None:
            events[1].record(stream)
        ctx.tonemap_async(tile.data_ptr(), params.local_rows * W, max(spp, 1), tile_u8.data_ptr(),
                          rtow.RT_TONEMAP_CPU, stream.cuda_stream)
        if events is not None:
            events[2].record(stream)
        if world > 1:
            dist.gather(tile_u8 if a.backend == "nccl" else tile_u8.cpu(), gather_list, dst=0)
        if events is not None:
            events[3].record(stream)

    assert stream.cuda_stream != 0
    first_frame_ms = None
    with torch.cuda.stream(stream):
        # load the kernels (render + pilot builds) on a tiny frame, then time the
        # first headline frame on its own: with the pilot schedule it includes
        # the 4-spp pilot and the device sort of the tile order
        small = rtow.make_params(64, 64, 4, flags=params.flags & ~rtow.RT_FLAG_KEEP_COUNTERS)
        ctx.render_async(cam, small, tile.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        for i in range(a.warmup):
            t_first = time.perf_counter()
            step(1000 + i)
            torch.cuda.synchronize(dev)
            if i == 0:
                first_frame_ms = (time.perf_counter() - t_first) * 1e3
        ctx.reset_stats(stream.cuda_stream)
        evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(4)) for _ in range(a.steps)]

        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i, evs[i])
        torch.cuda.synchronize(dev)
        barrier()
        elapsed = time.perf_counter() - t0
    # the last timed frame's sums and bytes (the work frame below reuses the tile)
    sums_last, u8_last = tile.cpu().numpy(), tile_u8.cpu().numpy()

    st = ctx.collect_stats()
    kernel_ms = [e[0].elapsed_time(e[1]) for e in evs]
    tonemap_ms = [e[1].elapsed_time(e[2]) for e in evs]
    gather_ms = [e[2].elapsed_time(e[3]) for e in evs]
    # executed work per launch: one instrumented frame (RT_FLAG_COUNT_WORK build),
    # same seed as timed step 0, outside the timed region
    wp = rtow_dist.partition(W, H, spp, world, rank, a.row_block, max_depth=a.depth,
                             flags=(params.flags & ~rtow.RT_FLAG_KEEP_COUNTERS) | rtow.RT_FLAG_COUNT_WORK)
    wp.seed = 0
    with torch.cuda.stream(stream):
        ctx.render_async(cam, wp, tile.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize(dev)
    work = ctx.collect_stats()
    local = torch.tensor([float(st.segments), float(st.samples), float(st.wave_steps)],
                         dtype=torch.float64, device=gdev)
    mean = lambda v: sum(v) / len(v)
    # max over ranks: the wall time, and each part of the step (render, write_color, gather)
    t_max = torch.tensor([elapsed, mean(kernel_ms), mean(tonemap_ms), mean(gather_ms)], dtype=torch.float64,
                         device=gdev)
    if world > 1:
        dist.all_reduce(local, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    segments, samples, wave_steps = local.tolist()
    elapsed, render_ms_max, tonemap_ms_max, gather_ms_max = t_max.tolist()

    if rank == 0:
        # assemble the last frame on rank 0 (outside the timed region) and sanity-check it
        if world > 1:
            tiles = torch.stack(gather_list).cpu().numpy()
        else:
            tiles = u8_last[None]
        frame = rtow_dist.assemble(tiles, H, world, a.row_block)
        assert np.isfinite(sums_last).all() and sums_last.max() <= spp + 1e-3
        assert np.array_equal(u8_last, rtow.tonemap(sums_last, max(spp, 1)))
        if a.out:
            rtow.write_ppm(a.out, frame, binary=a.out.endswith((".p6", ".pnm")))

        k_avg_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        value = segments / elapsed / 1e6
        pmc, pmc_reason = load_pmc(workload, a.accel, world)
        roof = roofline({"sphere_tests": work.sphere_tests, "box_tests": work.box_tests,
                         "bf_tests": work.bf_tests}, k_avg_s, a.accel, pmc, pmc_reason, rtow.device_code_sha16())
        out = {
            "metric": "Mray/s (ray segments = closest-hit queries per second), final random-spheres "
                      "scene 3840x2160 @ 500spp depth 50" if not a.preset or a.preset == "c2"
                      else f"Mray/s, {workload}",
            "value": round(value, 2),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic: final random-spheres scene (g++-order mt19937 seed 5489, "
                    f"{scene.n} spheres), src/cpu camera",
            "config": {"workload": workload, "width": W, "height": H, "spp": spp,
                       "max_depth": a.depth, "spheres": scene.n,
                       "parallelism": f"row-interleaved bands of {a.row_block} rows x {world} GPU"
                                      + ((" + RCCL gather of byte tiles" if a.backend == "nccl" else " + gloo gather of byte tiles")
                                         if world > 1 else "")},
            "ms_per_frame": round(elapsed / a.steps * 1e3, 3),
            "msamples_per_s": round(samples / elapsed / 1e6, 2),
            "segments_per_frame": int(segments / a.steps),
            "lane_efficiency": round(segments / (64.0 * wave_steps), 4) if wave_steps else None,
            "kernel_ms_avg_rank0": round(k_avg_s * 1e3, 3),
            "accel": a.accel,
            "grid_cell_scale": round(ctx.grid_scale(), 4) if a.accel == "bvh" else None,
            "grid_cell_scale_note": "the layer grid's cell scale RT_OPT_GRID_FIT fitted to this frame geometry "
                                    "(host model, first frame; DESIGN.md 3.3)",
            "walk": {"bvh": "layer grid (per-lane DDA) + extras scanned", "scan": "brute force",
                     "layer_bvh": "wave-uniform layer BVH + extras scanned"}[a.accel],
            "schedule": "launch order" if a.no_pilot else
                        "pilot (expensive tiles first; 4-spp pilot in the warmup frame)",
            "work_per_launch_rank0": {"segments": work.segments, "sphere_tests": work.sphere_tests,
                                      "box_tests": work.box_tests, "box_hits_own_ray": work.box_hits,
                                      "brute_force_equiv_tests": work.bf_tests},
            "first_frame_ms": round(first_frame_ms, 3) if first_frame_ms is not None else None,
            "first_frame_note": "wall time of the first frame of this geometry on its own, pilot schedule "
                                "included (4-spp pilot + device sort of the tile order); ms_per_step "
                                "reuses the order",
            "step_parts_ms": {"render_max_over_ranks": round(render_ms_max, 3),
                              "write_color_max_over_ranks": round(tonemap_ms_max, 3),
                              "gather_max_over_ranks": round(gather_ms_max, 3),
                              "basis": "HIP events on each rank's launch stream around its render, "
                                       "its device write_color and the RCCL gather of the byte tiles "
                                       "(0 at N = 1); mean over the timed steps, max over ranks"},
            "roofline": roof,
            "cpu_baseline": None,
            "cpu_baseline_note": None if world == 1 else
                                 "measured at N = 1 only (rank 0's host cores would be shared with "
                                 "N render processes); see the N = 1 line",
        }
        if world == 1 and a.no_cpu_baseline:
            out["cpu_baseline_note"] = "skipped (--no-cpu-baseline)"
        if world == 1 and not a.no_cpu_baseline:
            try:
                procs = a.cpu_procs or min(16, os.cpu_count() or 1)
                out["cpu_baseline"] = cpu_baseline(a.cpu_spp, procs)
            except Exception as e:  # the GPU number stands on its own
                out["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
