#!/usr/bin/env python3
"""Static instruction counts per basic block of one render_kernel instantiation
(A/B inspection of kernel variants; not part of the product).

    python tools/isa_blocks.py <kernel.s> [mangled-name-substring]

Default kernel: the headline build render_kernel<false,false,true,false,true,1,false>.
Prints V (VALU) / S (SALU) / DS / M (VMEM+SMEM) per block and the totals.
"""
import re
import sys

path = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "render_kernelILb0ELb0ELb1ELb0ELb1ELi1ELb0E"
s = open(path).read().split("\n")
start = [i for i, l in enumerate(s) if l.startswith("_Z") and key in l.split(":")[0]][0]
end = [i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end")][0]
blocks, cur = [], None
tot = [0, 0, 0, 0]
for l in s[start:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m or cur is None:
        cur = [m.group(1) if m else "entry", 0, 0, 0, 0, ""]
        blocks.append(cur)
        if m:
            cur[5] = l.split(";", 1)[1].strip() if ";" in l else ""
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    k = 1 if op.startswith("v_") else 2 if op.startswith("s_") else 3 if op.startswith("ds_") else 4
    cur[k] += 1
    tot[k - 1] += 1
for b in blocks:
    print(f"{b[0]:12s} V {b[1]:3d} S {b[2]:3d} DS {b[3]:2d} M {b[4]:2d}  {b[5][:50]}")
print("total V %d S %d DS %d M %d" % tuple(tot))
