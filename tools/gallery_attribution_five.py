#!/usr/bin/env python3
"""The image20..22 gallery check of tools/image23_attribution.py: the kernel
specification (oracle kernel mode, GPU semantics) and the oracle's restatement of
src/gpu's own fp32 hit arithmetic (rto_gpuref_render, GREF_NAIVE_HIT | GREF_UNNORM)
against gallery/gpu/image20..22.png (five-sphere scene, 1920x1080, 10 spp), two
seeds each.  CPU only.   python tools/gallery_attribution_five.py"""
import sys, ctypes; import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0]=[os.path.join(R,"ray-tracing-in-one-weekend_amd"),os.path.join(R,"tests")]
import numpy as np, rtow, oracle_lib
from test_oracle import IMAGE22, image22_camera, blocks8, gallery_blocks
L=oracle_lib.lib()
L.rto_gpuref_render.argtypes=[ctypes.c_void_p]*3+[ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
scene=rtow.five_scene()
for name in ("image20","image21","image22"):
    cam=image22_camera(rtow,name); g=gallery_blocks(name)
    for mode in (None, 3):
        res=[]
        for seed in (1,2):
            p=rtow.make_params(IMAGE22["width"],IMAGE22["height"],IMAGE22["spp"],seed=seed,flags=rtow.RT_FLAG_GPU_SEMANTICS)
            if mode is None: out,segs=oracle_lib.kernel_render(scene,cam,p)
            else:
                v=scene.view(); out=np.zeros((p.local_rows,p.width,3),np.float32); sg=ctypes.c_ulonglong()
                L.rto_gpuref_render(ctypes.addressof(v),ctypes.addressof(cam),ctypes.addressof(p),mode,out.ctypes.data,ctypes.byref(sg),0); segs=sg.value
            res.append((blocks8(rtow.tonemap(out,IMAGE22["spp"],rtow.RT_TONEMAP_GPU)),segs))
        a,b=res[0][0],res[1][0]
        bias=a.reshape(-1,3).mean(0)-g.reshape(-1,3).mean(0)
        print(name, "spec" if mode is None else "src/gpu restatement", "bias", bias.round(4).tolist(), "err", round(float(np.abs(a-g).mean()),4), "floor", round(float(np.abs(a-b).mean()),4), "segs", res[0][1])
