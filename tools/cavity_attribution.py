#!/usr/bin/env python3
"""Depth-capped paths in the reference's arithmetic and in the fp32 kernel
algorithm ("ground-cut spheres").  For each
random scene (tests/random_scenes.py) at 96x54xSPP: the fp64 restatement of
src/cpu (byte-identical to the reference) with its count of paths ended at
the depth cap (rto_reference_capped: ray_color's depth <= 0, main.cc:16-17),
and the kernel algorithm (oracle kernel mode, 2 seeds) with the same count
(rto_kernel_capped) under the specification, RTO_OPT_FP64_HIT and
RTO_OPT_NO_SAME_EXIT.  CPU only.

Usage: python tools/cavity_attribution.py 11,4,16,15 [SPP=512]
"""
import os, sys, ctypes, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'ray-tracing-in-one-weekend_amd'), os.path.join(ROOT, 'tests')]
import rtow, random_scenes, oracle_lib as ol
L=ol.lib(); L.rto_reference_capped.restype=ctypes.c_ulonglong; L.rto_kernel_capped.restype=ctypes.c_ulonglong
L.rto_kernel_capped.argtypes=[ctypes.c_int]
spp=int(sys.argv[2]) if len(sys.argv)>2 else 512
for case in [int(x) for x in sys.argv[1].split(',')]:
    sc=random_scenes.free_scene(rtow,case)
    img,seg=ol.reference_render_view(sc,96,16/9,spp)
    cap=L.rto_reference_capped()
    print('scene %d ref      segs %d capped %d  (%.3e capped/segment, mean %.4f)'%(case,seg,cap,cap/seg,img.mean()),flush=True)
    cam=rtow.camera_cpu(aspect=16/9)
    for name,opt in (('spec',0),('fp64_hit',ol.RTO_OPT_FP64_HIT),('no_same_exit',ol.RTO_OPT_NO_SAME_EXIT)):
        L.rto_kernel_capped(1)
        segs=0; caps=0
        for seed in (1,2):
            out,_,s=ol._kernel_render_opts(sc,cam,rtow.make_params(96,54,spp,seed=seed),opt,False,0)
            segs+=s
        caps=L.rto_kernel_capped(1)
        print('scene %d %-12s segs %d capped %d  (%.3e capped/segment)  segs/ref %+.2e'%(case,name,segs/2,caps/2,caps/segs,segs/2/seg-1),flush=True)
