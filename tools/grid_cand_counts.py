# Grid-walk candidate statistics on the headline frame (experiment build
# build/variants/count.so, RT_COUNT_ITEMS=3: box_hits = wave-level candidate
# sequences in the grid walk, root_tests = lane-level grid candidates,
# box_tests = lane-level cell visits, sphere_tests = lane-level item tests).
import json, os, sys
sys.path.insert(0, 'ray-tracing-in-one-weekend_amd')
os.environ.setdefault("RTOW_LIB", "build/variants/count.so")
import rtow
ctx = rtow.Context(0)
ctx.upload(rtow.final_scene())
cam = rtow.camera_cpu(aspect=3840 / 2160)
p = rtow.make_params(3840, 2160, int(sys.argv[1]) if len(sys.argv) > 1 else 500, seed=0,
                     flags=rtow.RT_FLAG_ACCEL_BVH | rtow.RT_FLAG_COUNT_WORK)
img, st = ctx.render(cam, p)
ws = st.wave_steps
print(json.dumps({"segments": st.segments, "wave_steps": ws, "lane_cells": st.box_tests,
                  "wave_grid_candidate_seqs": st.box_hits, "lane_grid_candidates": st.root_tests,
                  "lane_tests": st.sphere_tests,
                  "per_wave_step": {"grid_cand_seqs": st.box_hits / ws,
                                    "lane_grid_cands_per_segment": st.root_tests / st.segments,
                                    "lane_tests_per_segment": st.sphere_tests / st.segments,
                                    "lane_eff": st.segments / ws / 64}}))
