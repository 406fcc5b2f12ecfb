# Wave-level iteration counts of the layer grid walk on the headline frame
# (RT_FLAG_COUNT_WORK build: box_hits = DDA iterations, root_tests = item iterations).
import sys, json
sys.path.insert(0, 'ray-tracing-in-one-weekend_amd')
import rtow
ctx = rtow.Context(0)
ctx.upload(rtow.final_scene())
cam = rtow.camera_cpu(aspect=3840 / 2160)
p = rtow.make_params(3840, 2160, 500, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_COUNT_WORK)
img, st = ctx.render(cam, p)
ws = st.wave_steps
print(json.dumps({"segments": st.segments, "wave_steps": ws, "lane_cells": st.box_tests,
                  "wave_dda_iters": st.box_hits, "wave_item_iters": st.root_tests,
                  "sphere_tests": st.sphere_tests,
                  "per_wave_step": {"dda": st.box_hits / ws, "items": st.root_tests / ws,
                                    "lane_cells_per_segment": st.box_tests / st.segments}}))
