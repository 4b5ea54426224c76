"""CPU simulation (numpy + the oracle) of the odometry association windows' first round on config-4
problems: points the chunk walk visits per query with the 5 m bound, with the bound from the nearest
neighbour's 27 cells, and with per-category pruning.  Diagnostic; run from the repo root."""
import sys
import numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0,R); sys.path.insert(0,os.path.join(R,'oracle'))
import importlib
sg=importlib.import_module('loam_velodyne-1_amd.synthgen')
import oracle_ctypes as oc
CH=64
def walk_cost(L, c, scan, end, dir, sel, bw, cat=None):
    # points visited by wave_window (chunk pruning by box vs min(25,bw)), returns (pts, boxes)
    n=len(L); pts=0; boxes=0
    rings=L[:,3].astype(int)
    stop=lambda r: r>scan+2 if dir>0 else r<scan-2
    if dir>0:
        j=c+1; hend=min(end,(j+CH-1)//CH*CH)
        if j<hend:
            pts+=hend-j
            if any(stop(r) for r in rings[j:hend]): return pts,boxes
        j=max(j,hend)
        while j<end:
            k=j//CH; lo=L[k*CH:min(end,(k+1)*CH)]
            boxes+=1
            mn=lo[:,:3].min(0); mx=lo[:,:3].max(0)
            g=np.maximum(np.maximum(mn-sel,sel-mx),0); bd=(g*g).sum()
            st=any(stop(r) for r in rings[k*CH:min(end,(k+1)*CH)])
            rr=rings[k*CH:min(end,(k+1)*CH)]
            need=bd<25 and bd<=bw
            if cat is not None:
                b2,b3=cat; need=bd<25 and ((bd<=b2 and rr.min()<=scan) or (bd<=b3 and rr.max()>scan))
            if need or st: pts+=len(lo)
            if st: return pts,boxes
            j=(k+1)*CH
    else:
        j=c-1
        if j<0: return 0,0
        hs=j//CH*CH; pts+=j-hs+1
        if any(stop(r) for r in rings[hs:j+1]): return pts,boxes
        kt=hs//CH-1
        while kt>=0:
            lo=L[kt*CH:(kt+1)*CH]; boxes+=1
            mn=lo[:,:3].min(0); mx=lo[:,:3].max(0)
            g=np.maximum(np.maximum(mn-sel,sel-mx),0); bd=(g*g).sum()
            st=any(stop(r) for r in rings[kt*CH:(kt+1)*CH])
            rr=rings[kt*CH:(kt+1)*CH]
            need=bd<25 and bd<=bw
            if cat is not None:
                b2,b3=cat; need=bd<25 and ((bd<=b2 and rr.max()>=scan) or (bd<=b3 and rr.min()<scan))
            if need or st: pts+=len(lo)
            if st: return pts,boxes
            kt-=1
    return pts,boxes
prevs,curs=sg.batch_problems(3,base_seed=1000)
tot={'base':0,'cell':0,'q':0,'tight':0}
for i in range(3):
    o=oc.Oracle(oc.default_config(system_delay=1))
    o.scan_registration(prevs[i]); _,fp=o.scan_registration(prevs[i]); _,fc=o.scan_registration(curs[i])
    for kind,qk in (("less_sharp","sharp"),("less_flat","flat")):
        L=np.asarray(fp[kind],np.float64); Q=np.asarray(fc[qk],np.float64)
        rings=L[:,3].astype(int); corner=kind=="less_sharp"
        mono=np.all(np.diff(rings)>=0)
        end=min(len(Q),len(L))
        cell=np.floor(L[:,:3]).astype(int)
        for q in Q:
            sel=q[:3]; d=((L[:,:3]-sel)**2).sum(1)
            c=int(np.argmin(d))
            if d[c]>=25: continue
            scan=rings[c]
            # cell candidates: points in 27 cells around sel
            qc=np.floor(sel).astype(int)
            inc=np.all(np.abs(cell-qc)<=1,axis=1)
            idx=np.arange(len(L))
            fw=(idx>c)&(idx<end)&(rings<=scan+2)
            bk=(idx<c)&(rings>=scan-2)
            if corner:
                mem=(fw&(rings>scan))|(bk&(rings<scan)); cb=d[inc&mem].min() if (inc&mem).any() else 25
            else:
                m2=(fw&(rings<=scan))|(bk&(rings>=scan)); m3=(fw&(rings>scan))|(bk&(rings<scan))
                b2=d[inc&m2].min() if (inc&m2).any() else 25; b3=d[inc&m3].min() if (inc&m3).any() else 25
                cb=max(b2,b3); cat=(b2,b3)
            p0=sum(walk_cost(L,c,scan,end,dd,sel,25)[0] for dd in (1,-1))
            p1=sum(walk_cost(L,c,scan,end,dd,sel,cb)[0] for dd in (1,-1))
            p2=p1 if corner else sum(walk_cost(L,c,scan,end,dd,sel,cb,cat)[0] for dd in (1,-1))
            tot['cat']=tot.get('cat',0)+p2
            tot['base']+=p0; tot['cell']+=p1; tot['q']+=1; tot['tight']+= cb<25
        print(i,kind,'mono',mono,tot)
print('window pts/query round0: base',tot['base']/tot['q'],'cell-bound',tot['cell']/tot['q'],'per-category',tot['cat']/tot['q'],'bounded frac',tot['tight']/tot['q'])
