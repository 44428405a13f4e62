#!/usr/bin/env python3
"""Offline survey of strip shapes for the blend kernels: (Gaussian, strip)
survivors and blended (Gaussian, pixel) pairs of the bench camera, from the
tools/strip_survey_dump.py export (exact per-pixel alpha >= 1/255 test)."""
import numpy as np, time
import sys
d=np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/strip_survey.npz')
m=d['means2D']; co=d['conic_opacity']; pl=d['point_list']; rg=d['ranges']
W=H=800; gx=50
print(m.shape, co.shape, pl.shape, rg.shape)
ntile=gx*50; rg=rg.reshape(-1,2)
tile_of=np.zeros(len(pl),np.int64)
for t in range(ntile):
    a,b=rg[t]; tile_of[a:b]=t
yy,xx=np.mgrid[0:16,0:16]
xx=xx.reshape(-1).astype(np.float32); yy=yy.reshape(-1).astype(np.float32)
layouts={
 '16x4': (yy//4).astype(int),
 '8x8': ((yy//8)*2+(xx//8)).astype(int),
 '4x16': (xx//4).astype(int),
 '16x8': (yy//8).astype(int),
 '16x16': np.zeros_like(xx).astype(int),
}
res={k:[0,0] for k in layouts}; pairs=0
CH=100000
t0=time.time()
for s in range(0,len(pl),CH):
    g=pl[s:s+CH]; t=tile_of[s:s+CH]
    tx=(t%gx)*16; ty=(t//gx)*16
    px=tx[:,None]+xx[None,:]; py=ty[:,None]+yy[None,:]
    dx=m[g,0][:,None]-px; dy=m[g,1][:,None]-py
    a=co[g,0][:,None]; b=co[g,1][:,None]; c=co[g,2][:,None]; o=co[g,3][:,None]
    power=-0.5*(a*dx*dx+c*dy*dy)-b*dx*dy
    al=np.minimum(0.99,o*np.exp(power))
    ok=(power<=0)&(al>=1/255.)&(px<W)&(py<H)
    pairs+=ok.sum()
    for k,lab in layouts.items():
        for q in range(lab.max()+1):
            res[k][0]+=ok[:,lab==q].any(1).sum()
print('instances',len(pl),'pairs',pairs, time.time()-t0)
for k,v in res.items():
    npx = 256 // (layouts[k].max() + 1)
    print(k,'survivors',v[0],'pixel slots',v[0]*npx,'util',pairs/(v[0]*npx))
