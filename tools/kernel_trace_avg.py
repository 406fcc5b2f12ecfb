#!/usr/bin/env python3
"""Average duration of the full-size render dispatches in a rocprofv3 kernel
trace (the stats CSV also averages the bench's 64x64 code-loading launch and
the pilot build):  python tools/kernel_trace_avg.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "render_kernel" in r["Kernel_Name"]]
big = max(int(r["Grid_Size_X"]) for r in rows)
d = defaultdict(list)
for r in rows:
    if int(r["Grid_Size_X"]) == big:
        d[r["Kernel_Name"].split("(")[0].replace("void rtk::", "")].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print(f"{k}: {len(v)} full-size dispatches, avg {sum(v) / len(v):.3f} ms, "
          f"steady (after the first) {sum(v[1:]) / max(1, len(v) - 1):.3f} ms")
