# Per-lane and per-wave (max over walking lanes) distributions of grid cells
# and items visited per walk, headline geometry at 100 spp: experiment build
# build/variants/walkhist.so (rt_read_hist).  Shows whether a wave's walk time
# is set by a few long lanes (work splitting would pay) or by many.
import ctypes, json, os, sys
sys.path.insert(0, 'ray-tracing-in-one-weekend_amd')
os.environ.setdefault("RTOW_LIB", "build/variants/walkhist.so")
import numpy as np
import rtow
ctx = rtow.Context(0)
ctx.upload(rtow.final_scene())
cam = rtow.camera_cpu(aspect=3840 / 2160)
img, st = ctx.render(cam, rtow.make_params(3840, 2160, 100, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH))
h = (ctypes.c_ulonglong * 192)()
assert ctypes.CDLL(rtow.LIB_PATH).rt_read_hist(h) == 0
h = np.array(h, dtype=np.float64)
lane_c, lane_i, wave_c, wave_i = h[0:32], h[32:96], h[96:128], h[128:192]
def stats(x):
    n = x.sum(); v = np.arange(len(x))
    cdf = np.cumsum(x) / n
    return {"n": int(n), "mean": round(float((x * v).sum() / n), 3),
            "p50": int(np.searchsorted(cdf, 0.5)), "p90": int(np.searchsorted(cdf, 0.9)),
            "p99": int(np.searchsorted(cdf, 0.99)), "hist": [int(a) for a in x[:24]]}
print(json.dumps({"segments": st.segments, "wave_steps": st.wave_steps,
                  "lane_cells": stats(lane_c), "lane_items": stats(lane_i),
                  "wave_max_cells": stats(wave_c), "wave_max_items": stats(wave_i)}))
