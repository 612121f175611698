import sys, math, numpy as np
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__file__), '..', 'rust-ray-tracing_amd'))
import rt_mi355x as rt
flat = rt.scenes.config_scene(sys.argv[1] if len(sys.argv)>1 else "E").flatten()
C = flat.center; R = flat.radius; n = len(R)
key = np.abs(C).sum(1) + np.abs(R); med = np.median(key)
filt = np.where(key <= 8*med)[0]; exact = np.where(key > 8*med)[0]
# k-d clusters of 16
clusters = []
work = [filt]
while work:
    idx = work.pop()
    if len(idx) <= 16:
        if len(idx): clusters.append(idx)
        continue
    ext = C[idx].max(0) - C[idx].min(0); ax = int(np.argmax(ext))
    m = min(len(idx)-1, (len(idx)+31)//32*16)
    o = np.argsort(C[idx, ax], kind='stable')
    work.append(idx[o[m:]]); work.append(idx[o[:m]])
lo = np.array([ (C[c]-R[c,None]).min(0) for c in clusters]); hi = np.array([(C[c]+R[c,None]).max(0) for c in clusters])
print("clusters", len(clusters), "exact", len(exact))
W, H = (3840, 2160) if (len(sys.argv)<=1 or sys.argv[1] in "DE") else (1920,1080)
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
ulc, vu, vv, ctr = map(np.array, (cam.ulc, cam.vu, cam.vv, cam.center))
rng = np.random.default_rng(1)
def nearest(o, d):
    # brute force nearest sphere hit (root1 only), chunked
    best = np.full(len(o), np.inf); bi = np.full(len(o), -1)
    for s in range(0, n, 2000):
        c = C[s:s+2000]; r2 = R[s:s+2000]**2
        oc = o[:,None,:] - c[None]
        a = (d*d).sum(1)[:,None]; hb = (oc*d[:,None,:]).sum(2); cc = (oc*oc).sum(2) - r2[None]
        disc = hb*hb - a*cc
        with np.errstate(invalid='ignore'):
            t = (-hb - np.sqrt(disc))/a
        t[~(disc>=0)] = np.inf; t[t<0.001] = np.inf
        j = np.argmin(t, 1); tj = t[np.arange(len(o)), j]
        upd = tj < best; best[upd] = tj[upd]; bi[upd] = j[upd] + s
    return best, bi
def clusters_passed(o, d, tmax):
    inv = 1.0/np.where(np.abs(d)<1e-20, 1e-20, d)
    t0 = (lo[None]-o[:,None])*inv[:,None]; t1 = (hi[None]-o[:,None])*inv[:,None]
    tn = np.minimum(t0,t1).max(2); tf = np.maximum(t0,t1).min(2)
    return (tf >= np.maximum(tn,0)) & (tn <= tmax[:,None])
row = int(sys.argv[2]) if len(sys.argv)>2 else int(H*0.62)
col0 = int(sys.argv[3]) if len(sys.argv)>3 else W//2
spp = 512
allo, alld, allpix = [], [], []
for pi in range(16):
    col = col0 + pi
    u = (col + rng.random(spp))/W; v = (row + rng.random(spp))/H
    pc = ulc[None] + vu[None]*u[:,None] + vv[None]*v[:,None]
    d = pc - ctr[None]; d /= np.linalg.norm(d,axis=1)[:,None]
    o = np.repeat(ctr[None], spp, 0)
    t, bi = nearest(o, d)
    hit = bi >= 0
    p = o[hit] + d[hit]*t[hit,None]; nrm = (p - C[bi[hit]]) / R[bi[hit],None]
    z = rng.normal(size=(hit.sum(),3)); z /= np.linalg.norm(z,axis=1)[:,None]
    allo.append(p); alld.append(nrm + z); allpix.append(np.full(hit.sum(), pi))
o = np.concatenate(allo); d = np.concatenate(alld); pix = np.concatenate(allpix)
t, bi = nearest(o, d)
P = clusters_passed(o, d, t)
print("bounced rays", len(o), "mean clusters per ray (to first hit)", P.sum(1).mean())
def union(groups):
    return np.mean([P[g].any(0).sum() for g in groups])
N = len(o) - len(o)%256
nat = [np.arange(s, s+64) for s in range(0, N, 64)]
print("natural order: clusters per 64-ray wave", union(nat))
for name, keyf in [("octant", lambda i: ((d[i,0]>0)*1 + (d[i,1]>0)*2 + (d[i,2]>0)*4)),
                   ("quadrant xz", lambda i: ((d[i,0]>0)*1 + (d[i,2]>0)*2)),
                   ("azimuth 4", lambda i: np.floor((np.arctan2(d[i,2], d[i,0])+np.pi)/(2*np.pi)*4).astype(int)),
                   ("azimuth 4 x elev 2", lambda i: np.floor((np.arctan2(d[i,2], d[i,0])+np.pi)/(2*np.pi)*4).astype(int)*2 + (d[i,1]/np.linalg.norm(d[i],axis=1) > 0.5))]:
    groups = []
    for s in range(0, N, 256):
        i = np.arange(s, s+256); k = keyf(i)
        o_ = i[np.argsort(k, kind='stable')]
        groups += [o_[j:j+64] for j in range(0,256,64)]
    print(name, "sorted in 256: clusters per wave", union(groups))
    groups = []
    for s in range(0, N - N%1024, 1024):
        i = np.arange(s, s+1024); k = keyf(i)
        o_ = i[np.argsort(k, kind='stable')]
        groups += [o_[j:j+64] for j in range(0,1024,64)]
    print(name, "sorted in 1024: clusters per wave", union(groups))
P2 = clusters_passed(o, d, np.full(len(o), np.inf))
print("hit fraction", (bi>=0).mean(), "mean clusters per ray (no hit cull)", P2.sum(1).mean())
print("natural: union no-cull", np.mean([P2[g].any(0).sum() for g in nat]))
# greedy near-first union walk simulation: order clusters by distance of box from wave's first ray origin,
# walk in that order; a lane stops considering clusters whose entry t > its best hit found so far
def walk(g, order):
    best = np.full(len(g), np.inf); walked = 0
    inv = 1.0/np.where(np.abs(d[g])<1e-20, 1e-20, d[g])
    for k in order:
        t0=(lo[k]-o[g])*inv; t1=(hi[k]-o[g])*inv
        tn=np.minimum(t0,t1).max(1); tf=np.maximum(t0,t1).min(1)
        ok=(tf>=np.maximum(tn,0))&(tn<=best)
        if ok.any():
            walked+=1
            # update best with member hits
            for sidx in clusters[k]:
                oc=o[g]-C[sidx]; a=(d[g]**2).sum(1); hb=(oc*d[g]).sum(1); cc=(oc*oc).sum(1)-R[sidx]**2
                disc=hb*hb-a*cc
                with np.errstate(invalid='ignore'): t=(-hb-np.sqrt(disc))/a
                t[~(disc>=0)]=np.inf; t[t<0.001]=np.inf; t[~ok]=np.inf
                best=np.minimum(best,t)
    return walked
import random
idx_order = np.arange(len(clusters))
res_idx=[]; res_near=[]
for g in nat[::4][:24]:
    res_idx.append(walk(g, idx_order))
    cen=(lo+hi)/2; dist=np.linalg.norm(cen-o[g][0],axis=1)
    res_near.append(walk(g, np.argsort(dist)))
print("walk index order", np.mean(res_idx), " near-first", np.mean(res_near))
