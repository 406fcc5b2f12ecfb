#!/usr/bin/env python3
"""Table of the render kernels' register use from `make isa`'s remarks
(build/resource.txt): VGPRs, SGPRs, spills, occupancy, static LDS.

    make -C ray-tracing-in-one-weekend_amd isa >/dev/null; python tools/resource_table.py [filter]
"""
import re
import subprocess
import sys

path = "ray-tracing-in-one-weekend_amd/build/resource.txt"
rows, cur = [], None
for line in open(path):
    m = re.search(r"remark:\s+(.*?)(?: \[-Rpass|$)", line.strip())
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
flt = sys.argv[1] if len(sys.argv) > 1 else "render_kernel"
names = [r["name"] for r in rows]
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if flt not in d:
        continue
    print(f"{d.replace('void rtk::','').replace('(rtk::kparams)',''):60s} V={r.get('VGPRs')} S={r.get('TotalSGPRs')} "
          f"Vspill={r.get('VGPRs Spill')} Sspill={r.get('SGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')} "
          f"lds={r.get('LDS Size [bytes/block]')}")
