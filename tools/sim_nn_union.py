"""CPU estimate (numpy + the oracle) of how many distinct map points the 27-cell neighbourhoods of
64 / 128 / 256 consecutive stack points hold against their summed candidates (the reuse an LDS-staged
5-NN could buy).  Diagnostic; run from the repo root."""
import sys
import numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R); sys.path.insert(0,os.path.join(R,'oracle'))
import importlib
sg=importlib.import_module('loam_velodyne-1_amd.synthgen')
import oracle_ctypes as oc
def vg(p, leaf):
    if len(p)==0: return p
    k=np.floor(p[:,:3]/leaf).astype(np.int64)
    mn=k.min(0); d=k.max(0)-mn+1
    idx=(k[:,0]-mn[0])+(k[:,1]-mn[1])*d[0]+(k[:,2]-mn[2])*d[0]*d[1]
    o=np.argsort(idx,kind='stable'); idx=idx[o]; p=p[o]
    u,s=np.unique(idx,return_index=True)
    return np.array([p[s[i]:(s[i+1] if i+1<len(s) else len(p))].mean(0) for i in range(len(s))])
prevs,curs=sg.batch_problems(4,base_seed=1000)
for WG in (64,128,256):
  tot=[];
  for i in range(4):
    o=oc.Oracle(oc.default_config(system_delay=1))
    o.scan_registration(prevs[i])
    _,fp=o.scan_registration(prevs[i]); _,fc=o.scan_registration(curs[i])
    for kind,leaf in (("less_sharp",0.2),("less_flat",0.4)):
        m=vg(np.asarray(fp[kind]),leaf); s=vg(np.asarray(fc[kind]),leaf)
        mc=np.floor(m[:,:3]).astype(np.int64)
        from collections import Counter
        cnt=Counter(map(tuple,mc))
        for a in range(0,len(s),WG):
            q=s[a:a+WG]; qc=np.floor(q[:,:3]).astype(np.int64)
            cells=set()
            for c in qc:
                for dx in (-1,0,1):
                    for dy in (-1,0,1):
                        for dz in (-1,0,1): cells.add((c[0]+dx,c[1]+dy,c[2]+dz))
            U=sum(cnt.get(c,0) for c in cells)
            # per-query candidates (27 cells) for comparison
            per=sum(sum(cnt.get((c[0]+dx,c[1]+dy,c[2]+dz),0) for dx in (-1,0,1) for dy in (-1,0,1) for dz in (-1,0,1)) for c in qc)
            tot.append((kind,len(q),len(cells),U,per))
  import collections
  for kind in ("less_sharp","less_flat"):
    t=[x for x in tot if x[0]==kind]
    U=np.array([x[3] for x in t]); per=np.array([x[4] for x in t]); nq=np.array([x[1] for x in t]); nc=np.array([x[2] for x in t])
    print(WG,kind,'runs',len(t),'cells/run mean',nc.mean().round(1),'union pts mean',U.mean().round(1),'p90',np.percentile(U,90),'max',U.max(),'per-query cand (27 cells, no bound) mean',(per/nq).mean().round(1),'reuse',(per.sum()/U.sum()).round(2))
