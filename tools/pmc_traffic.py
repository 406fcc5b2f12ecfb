#!/usr/bin/env python3
"""Summarise rocprofv3 PMC counter CSVs for the render kernel.

    python tools/pmc_traffic.py <dir with *_counter_collection.csv> [...] \
        --workload "<bench workload string>" --out profiles/pmc_traffic.json

Also records SQ_INSTS_VALU (wave instructions per launch) when an SQ pass is
given, for bench.py's VALU issue-rate view.  HBM bytes per launch follow
MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced
streaming read, so the read side is doubled (the render kernel's reads are
scalar/gather loads of a 15 KB scene, so this is an upper bound); WRITE_SIZE
is exact for 16-B/lane stores.  Counters from separate passes are merged by
kernel name and averaged per dispatch.
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict


sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "ray-tracing-in-one-weekend_amd"))
import rtow  # noqa: E402  (device_code_sha16 only: the library is not loaded)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="render_kernel")
    ap.add_argument("--workload", default="")
    ap.add_argument("--world", type=int, default=1,
                    help="the rank share profiled: 1 = the whole frame, N = rank 0's 1/N share "
                         "(bench.py matches a line's world against it)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    # only the full-size dispatches of the kernel: the bench also launches it on
    # a tiny frame to load the code (and the pilot / work-count builds are
    # other kernels), which must not enter the per-launch averages
    rows = []
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                rows += [r for r in csv.DictReader(fh) if a.kernel in r.get("Kernel_Name", "")]
    grid = max((int(r["Grid_Size"]) for r in rows), default=0)
    vals = defaultdict(list)
    dur = {}
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        if int(r["Grid_Size"]) != grid:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[(r["Counter_Name"], r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    # steady state: the first full-size dispatch of a pass is the bench's warmup
    # frame (first touch of the frame tile: its WRITE_SIZE has read up to 2.5x
    # the timed frames'), so it is dropped when later ones exist; median of the rest
    def steady(v):
        v = sorted(v[1:] if len(v) > 1 else v)
        return v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2])
    avg = {k: steady(v) for k, v in vals.items()}
    out = {"kernel": a.kernel, "workload": a.workload, "world": a.world, "grid_size": grid,
           "counters_avg_per_dispatch": avg,
           "dispatches": {k: len(v) for k, v in vals.items()},
           "per_dispatch": dict(vals), "statistic": "median over full-size dispatches after the first (warmup)", "device_code_sha16": rtow.device_code_sha16()}
    g = [dur[k] for k in dur if k[0] == "GRBM_GUI_ACTIVE"]
    if "GRBM_GUI_ACTIVE" in avg and g:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs
        out["clock_ghz_pmc_pass"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / (sum(g) / len(g)) / 1e9, 3)
        out["kernel_s_pmc_pass"] = sum(g) / len(g)  # mean dispatch duration in that pass
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["fetch_bytes"] = avg["FETCH_SIZE"] * 1024
        out["write_bytes"] = avg["WRITE_SIZE"] * 1024
        out["hbm_bytes_per_launch"] = int(2 * out["fetch_bytes"] + out["write_bytes"])
        out["correction"] = "read side x2 (gfx950 FETCH_SIZE half-count), KiB -> bytes"
    if "SQ_INSTS_VALU" in avg:
        out["valu_insts_per_launch"] = int(avg["SQ_INSTS_VALU"])  # wave-level instructions
    s = json.dumps(out, indent=1, sort_keys=True)
    print(s)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
