#!/usr/bin/env python3
"""Would camera rays walked apart from bounce rays shorten the wave's grid
walk?  (host model, build container)

The layer-grid walk is per lane, so a wave runs as many item / DDA
iterations as its busiest lane needs (tools/wave_walk_sim.py).  Camera rays
of one 8x8 tile are coherent: the spheres any of them can meet inside the
layer slab form a short per-tile list (the tile's lens frustum), which a
wave-uniform scan could test instead of the per-lane walk.  That pays only
if the camera lanes are the ones that make the walk long.  This models the
kernel's waves as wave_walk_sim.py does (64 lanes drawn from one tile's
paths at mixed depths) and counts the wave's iterations over all lanes,
over the bounce lanes alone, and the per-tile frustum list (spheres within
reach + 0.1 of any of 512 camera rays of the tile inside the slab).

    python tools/camera_split_sim.py [--waves 150] [--c4]
"""
import argparse
import math, json, os, sys
import numpy as np
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0]=[os.path.join(ROOT,'ray-tracing-in-one-weekend_amd'),os.path.join(ROOT,'tools')]
import grid_aniso_sim as gs, wave_walk_sim as ws
import rtow
ap=argparse.ArgumentParser(); ap.add_argument('--waves',type=int,default=150); ap.add_argument('--c4',action='store_true'); A=ap.parse_args()
rng=np.random.default_rng(5)
# C4: the 10 001-sphere scene at 16384^2, origins up to oref 86, the cells-in-LDS fit (scale ~1.13)
scene=rtow.final_scene(50 if A.c4 else 11); W,H=(16384,16384) if A.c4 else (3840,2160)
OREF,SCALE=(86.0,1.13) if A.c4 else (64.0,1.11)
cam=rtow.camera_cpu(aspect=W/H)
lay_m=(np.abs(scene.cy-0.2)<1e-6)&(np.abs(scene.radius-0.2)<1e-6)
cx,cz=scene.cx[lay_m].astype(np.float64),scene.cz[lay_m].astype(np.float64)
cn=np.sqrt(cx**2+0.04+cz**2); reach=np.sqrt(0.04+2.0**-19*(cn+OREF)**2)
lay=(cx,cz,reach,0.2-reach.max(),0.2+reach.max())
g0=math.sqrt((cx.max()-cx.min()+0.5)*(cz.max()-cz.min()+0.5)/lay_m.sum())
G=ws.grid(lay,SCALE*g0)
C=np.stack([scene.cx,scene.cy,scene.cz],1).astype(np.float64); R=np.abs(scene.radius.astype(np.float64))
corner,horiz,vert,eye=(np.array(list(getattr(cam,f)),np.float64) for f in ("corner","horiz","vert","eye"))
lu=np.array(list(cam.lens_u)) if hasattr(cam,'lens_u') else None
lu=np.array(list(cam.lens_u),np.float64); lv=np.array(list(cam.lens_v),np.float64)
def cam_rays(tx,ty,n):
    s=(tx*8+rng.random(n)*8)/(W-1); t=(ty*8+rng.random(n)*8)/(H-1)
    rr=np.sqrt(rng.random(n)); ph=2*np.pi*rng.random(n)
    o=eye[None]+(rr*np.cos(ph))[:,None]*lu[None]+(rr*np.sin(ph))[:,None]*lv[None]
    d=corner[None]+s[:,None]*horiz[None]+t[:,None]*vert[None]-o
    d/=np.linalg.norm(d,axis=1,keepdims=True); return o,d
tot={'all':[0,0],'bounce':[0,0],'cam':[0,0]}; lst=[]; ncam=0; nl=0
NW=A.waves
for w in range(NW):
    tx,ty=rng.integers(0,W//8),rng.integers(0,H//8)
    o,d=cam_rays(tx,ty,64)
    segs=[]
    for depth in range(3):
        th,ih=gs.closest(o,d,C,R); segs.append((o.copy(),d.copy(),th.copy(),depth))
        hit=np.isfinite(th)
        if not hit.any(): break
        p=o+np.where(hit,th,0)[:,None]*d
        nrm=np.where(hit[:,None],(p-C[np.maximum(ih,0)])/R[np.maximum(ih,0),None],0)
        u=rng.normal(size=p.shape); u/=np.linalg.norm(u,axis=1,keepdims=True)
        d2=nrm+u; d2/=np.maximum(np.linalg.norm(d2,axis=1,keepdims=True),1e-12)
        o,d=p,np.where(hit[:,None],d2,d)
    pool=[(so[k],sd[k],st[k],dep) for (so,sd,st,dep) in segs for k in range(64) if st[k]>0 and (dep==0 or np.isfinite(segs[0][2][k]))]
    idx=rng.choice(len(pool),64,replace=len(pool)<64)
    lanes=[(ws.cells_of(*pool[k][:3],G),pool[k][3]) for k in idx]
    for key,sel in (('all',lambda dep:True),('bounce',lambda dep:dep>0),('cam',lambda dep:dep==0)):
        L=[c for c,dep in lanes if sel(dep)]
        dd,it=ws.wave_cost(L,1) if L else (0,0)
        tot[key][0]+=dd; tot[key][1]+=it
    ncam+=sum(1 for c,dep in lanes if dep==0); nl+=64
    # primary frustum list: spheres within reach of any of 512 camera rays inside the slab
    o,d=cam_rays(tx,ty,512)
    ylo,yhi=lay[3],lay[4]
    ta=np.maximum(np.minimum((ylo-o[:,1])/d[:,1],(yhi-o[:,1])/d[:,1]),0); tb=np.maximum((ylo-o[:,1])/d[:,1],(yhi-o[:,1])/d[:,1])
    # sample points along each ray in the slab, distance to sphere centres in xz
    ts=ta[:,None]+(tb-ta)[:,None]*np.linspace(0,1,24)[None]
    px=o[:,0,None]+ts*d[:,0,None]; pz=o[:,2,None]+ts*d[:,2,None]
    P=np.stack([px.ravel(),pz.ravel()],1)
    sel=np.zeros(len(cx),bool)
    for k in range(0,len(P),2048):
        dist=np.sqrt((P[k:k+2048,0,None]-cx[None])**2+(P[k:k+2048,1,None]-cz[None])**2)
        sel|=(dist<=reach[None]+0.1).any(0)
    lst.append(sel.sum())
print(json.dumps({'scene':'c4' if A.c4 else 'headline','waves':NW,'cam_lane_frac':ncam/nl,**{k:{'dda':v[0]/NW,'items':v[1]/NW} for k,v in tot.items()},'prim_list_mean':float(np.mean(lst)),'prim_list_p90':float(np.percentile(lst,90)),'prim_list_max':int(np.max(lst))},indent=1))
