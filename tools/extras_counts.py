# Candidate sequences of the off-layer "extras" (ground + 3 big spheres) on the
# headline geometry at 100 spp: experiment build build/variants/extcount.so,
# whose kernel counts per extras slot the wave-level root sequences and the
# lanes whose line meets the sphere (rt_read_ext_host).
import ctypes, json, os, sys
sys.path.insert(0, 'ray-tracing-in-one-weekend_amd')
os.environ.setdefault("RTOW_LIB", "build/variants/extcount.so")
import rtow
ctx = rtow.Context(0)
scene = rtow.final_scene()
ctx.upload(scene)
cam = rtow.camera_cpu(aspect=3840 / 2160)
p = rtow.make_params(3840, 2160, 100, seed=0, flags=rtow.RT_FLAG_ACCEL_BVH)
img, st = ctx.render(cam, p)
out = (ctypes.c_ulonglong * 8)()
assert ctypes.CDLL(rtow.LIB_PATH).rt_read_ext_host(out) == 0
ws = st.wave_steps
print(json.dumps({"segments": st.segments, "wave_steps": ws,
                  "wave_seq_per_step": [round(out[j] / ws, 3) for j in range(4)],
                  "lanes_per_seq": [round(out[4 + j] / max(1, out[j]), 1) for j in range(4)],
                  "lane_c_per_segment": [round(out[4 + j] / st.segments, 3) for j in range(4)]}))
