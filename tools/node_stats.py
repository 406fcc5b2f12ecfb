#!/usr/bin/env python3
"""Experiment: per-node wave-level test / entry counts of the BVH walk
(instrumented build build/variants/nodestats.so, RT_FLAG_COUNT_WORK), by depth,
and the box tests saved by collapsing internal nodes that waves almost always
enter (collapse X: its test disappears, its children are tested whenever X's
parent is entered: net = tests_X - children * (tests_X - enters_X))."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-in-one-weekend_amd"))


def main():
    w, h, spp = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 16)))
    import rtow
    L = rtow.lib()
    ctx = rtow.Context(0)
    ctx.upload(rtow.final_scene())
    nn = ctypes.c_int(0)
    buf = (ctypes.c_int * (2 * 8 * 4096))()
    n_nodes = L.rt_debug_nodes(ctx._h, buf)
    nodes = np.frombuffer(buf, dtype=np.int32)[: 2 * 8 * n_nodes].reshape(8, n_nodes, 2)
    L.rt_debug_node_stats(ctx._h, 1, None)
    flags = rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_COUNT_WORK
    _, st = ctx.render(rtow.camera_cpu(aspect=w / h), rtow.make_params(w, h, spp, seed=0, flags=flags))
    out = (ctypes.c_ulonglong * (2 * 8 * n_nodes))()
    L.rt_debug_node_stats(ctx._h, 0, out)
    ns = np.frombuffer(out, dtype=np.uint64).reshape(8, n_nodes, 2).astype(np.float64)
    steps = st.wave_steps
    by_depth = {}
    saving = 0.0
    for o in range(8):
        skip = nodes[o, :, 0]
        leaf = nodes[o, :, 1]

        def walk(i, d):
            nonlocal saving
            t, e = ns[o, i]
            bd = by_depth.setdefault(d, [0.0, 0.0, 0])
            bd[0] += t
            bd[1] += e
            bd[2] += 1
            if leaf[i]:
                return
            kids = []
            c = i + 1
            while c < skip[i]:
                kids.append(c)
                c = skip[c]
            if t > 0 and (t - len(kids) * (t - e)) > 0:
                saving += t - len(kids) * (t - e)
            for k in kids:
                walk(k, d + 1)

        i = 0  # the root may be collapsed: walk every top-level sibling
        while i < n_nodes:
            walk(i, 0)
            i = skip[i]
    tot_t = sum(v[0] for v in by_depth.values())
    print(json.dumps({"frame": f"{w}x{h}x{spp}", "n_nodes_per_order": int(n_nodes), "wave_steps": steps,
                      "wave_tests_per_step": round(tot_t / steps, 2),
                      "collapse_saving_per_step_upper": round(saving / steps, 2)}))
    for d in sorted(by_depth):
        t, e, n = by_depth[d]
        print(json.dumps({"depth": d, "nodes": n // 8, "tests_per_step": round(t / steps, 2),
                          "enter_frac": round(e / t, 3) if t else None}))


if __name__ == "__main__":
    main()
