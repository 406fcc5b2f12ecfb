"""bench.py's JSON line, built on the CPU from the committed PMC summaries
(no GPU): the counter-derived roofline fields are only computed from a
summary of the same rank share, so every line -- N = 1 and the N > 1 lines
the driver records on an 8-GPU node -- carries a plausible clock and
fractions <= 1, or nulls with a reason."""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

WORKLOAD = "final random-spheres scene 3840x2160 @ 500spp depth 50"
WORK = {"sphere_tests": 81_596_426_176, "box_tests": 17_073_404_022, "bf_tests": 5_454_437_042_682}


def _check_fields(roof):
    assert 0 < roof["frac"] <= 1
    vi = roof["valu_issue"]
    assert 1.5 <= vi["clock_ghz"] <= 3.0, vi
    assert 0 < vi["frac"] <= 1 and 0 < vi["frac_ubench"] <= 1
    assert 0 < roof["valu_lane_util"] <= 1
    assert 0 < roof["hbm"]["frac"] <= 1
    assert roof["pmc_null_reason"] is None


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_roofline_fields_only_from_the_same_share(world):
    pmc, reason = bench.load_pmc(WORKLOAD, "bvh", world)
    if world > 1:
        # never the whole frame's counters on a share's line (the round-2 bug:
        # full-frame SQ_INSTS_VALU / GRBM_GUI_ACTIVE over a 1/8 share's time)
        assert not pmc or pmc["world"] == world
    if not pmc:
        roof = bench.roofline(WORK, 0.018, "bvh", pmc, reason, "0" * 16)
        assert reason and roof["pmc_null_reason"] == reason
        assert roof["valu_issue"] is None and roof["valu_lane_util"] is None
        assert roof["hbm"] is None and roof["traffic"] is None
        return
    # the share's own kernel time (the PMC pass's dispatches) as this run's time
    roof = bench.roofline(WORK, pmc["kernel_s_pmc_pass"] * (1.0 if world == 1 else 1.0), "bvh", pmc, None,
                          pmc["device_code_sha16"])
    _check_fields(roof)


def test_simulated_world8_line_never_divides_full_frame_counters_by_a_share_time():
    """A simulated N = 8 line: rank 0's share renders in ~18 ms.  With only the
    whole frame's summary available, the counter fields are null (with a
    reason) instead of a 16.8 GHz clock and fractions above 1."""
    full, _ = bench.load_pmc(WORKLOAD, "bvh", 1)
    assert full and full.get("world", 1) == 1
    k_share = full["kernel_s_pmc_pass"] / 8
    wrong = bench.roofline(WORK, k_share, "bvh", full, None, full["device_code_sha16"])
    assert wrong["valu_issue"]["clock_ghz"] > 3.0  # what the round-2 line would have said
    pmc8, reason = bench.load_pmc(WORKLOAD, "bvh", 8)
    if pmc8:
        share_work = {k: v / 8 for k, v in WORK.items()}
        _check_fields(bench.roofline(share_work, pmc8["kernel_s_pmc_pass"], "bvh", pmc8, None,
                                     pmc8["device_code_sha16"]))
    else:
        assert "8-way" in reason


def test_committed_summaries_name_their_share():
    for path in glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_bvh*.json")):
        d = json.load(open(path))
        w = int(d.get("world", 1))
        assert path.endswith(".json" if w == 1 else f"_w{w}.json"), path
        assert d["workload"] == WORKLOAD


def test_counters_of_other_device_code_are_nulled():
    """A summary collected on other kernel code: the line names it and says
    so, and every counter-derived field is null (Weak 4)."""
    for world in (1, 2, 4, 8):
        pmc, reason = bench.load_pmc(WORKLOAD, "bvh", world)
        if not pmc:
            continue
        roof = bench.roofline(WORK, pmc["kernel_s_pmc_pass"], "bvh", pmc, None, "f" * 16)
        assert roof["pmc_matches_device_code"] is False
        assert roof["pmc_source"] and roof["pmc_source"] in roof["pmc_null_reason"]
        assert "f" * 16 in roof["pmc_null_reason"]
        assert roof["valu_issue"] is None and roof["valu_lane_util"] is None
        assert roof["hbm"] is None and roof["traffic"] is None
        assert 0 < roof["frac"] <= 1  # from the live HIP-event time and the work counters


def test_committed_summaries_carry_the_built_device_code(rtow):
    """Every committed pmc_traffic_bvh*.json (the N = 1, 2, 4, 8 lines' counter
    sources) was collected on the kernel this tree builds: the sha256 of the
    library's device code matches (tools/profile_round.sh,
    tools/profile_shares.sh re-collect them after a kernel change)."""
    sha = rtow.device_code_sha16()
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_bvh*.json")))
    assert len(paths) == 4
    for path in paths:
        assert json.load(open(path))["device_code_sha16"] == sha, os.path.basename(path)
