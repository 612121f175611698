# Estimate for DESIGN.md §8 (group boxes): config C bounce-1 waves (64 samples of one pixel, Lambertian
# bounces), the k-d clusters of 16 split into 4 spatial groups of 4; counts the clusters a wave walks (some lane
# passes its box, no best-hit cull) and the share of their group boxes some lane passes.
#   python3 tools/group_box_sim.py [C]
import sys, numpy as np
sys.path.insert(0, "rust-ray-tracing_amd")
import rt_mi355x as rt
cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
flat = rt.scenes.config_scene(cfg).flatten()
C = np.asarray(flat.center, float); R = np.abs(np.asarray(flat.radius, float)); n = len(R)
key = np.abs(C).sum(1) + R; med = np.median(key)
big = (key > 8 * med)
small_r = np.median(R)
bigr = R > 3 * small_r
filt = np.where(~big & ~bigr)[0]
def kd(idx, leaf):
    out = []; work = [idx]
    while work:
        i = work.pop()
        if len(i) <= leaf:
            if len(i): out.append(i)
            continue
        ext = C[i].max(0) - C[i].min(0); ax = int(np.argmax(ext))
        m = min(len(i) - 1, (len(i) + 2 * leaf - 1) // (2 * leaf) * leaf)
        o = np.argsort(C[i, ax], kind="stable")
        work.append(i[o[m:]]); work.append(i[o[:m]])
    return out
clusters = kd(filt, 16)
groups = [kd(c, 4) for c in clusters]
def box(ix):
    return (C[ix] - R[ix, None]).min(0), (C[ix] + R[ix, None]).max(0)
cb = [box(c) for c in clusters]
gb = [[box(g) for g in gs] for gs in groups]
def slab(o, d, lo, hi):
    inv = 1.0 / np.where(np.abs(d) < 1e-20, 1e-20, d)
    t0 = (lo - o) * inv; t1 = (hi - o) * inv
    tn = np.minimum(t0, t1).max(1); tf = np.maximum(t0, t1).min(1)
    return (tf >= np.maximum(tn, 0))
W, H = 1920, 1080
cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
ulc, vu, vv, ctr = map(np.array, (cam.ulc, cam.vu, cam.vv, cam.center))
rng = np.random.default_rng(1)
def nearest(o, d):
    best = np.full(len(o), np.inf); bi = np.full(len(o), -1)
    oc = o[:, None, :] - C[None]
    a = (d * d).sum(1)[:, None]; hb = (oc * d[:, None, :]).sum(2); c = (oc * oc).sum(2) - R[None] ** 2
    disc = hb * hb - a * c
    t = (-hb - np.sqrt(np.maximum(disc, 0))) / a
    t = np.where((disc >= 0) & (t > 1e-3), t, np.inf)
    bi = t.argmin(1); best = t.min(1); bi[~np.isfinite(best)] = -1
    return bi, best
walked = 0; gpass = 0; gtot = 0; nw = 0
for w in range(300):
    px = rng.integers(0, W); py = rng.integers(H // 3, H)
    s = np.stack([(px + rng.random(64)) / W, (py + rng.random(64)) / H], 1)
    pc = ulc + s[:, :1] * vu + s[:, 1:] * vv
    d = pc - ctr; d /= np.linalg.norm(d, axis=1, keepdims=True); o = np.repeat(ctr[None], 64, 0)
    bi, bt = nearest(o, d)
    hit = bi >= 0
    if hit.sum() < 8: continue
    p = o[hit] + d[hit] * bt[hit, None]; nrm = (p - C[bi[hit]]) / R[bi[hit], None]
    v = rng.normal(size=(hit.sum(), 3)); v /= np.linalg.norm(v, axis=1, keepdims=True)
    nd = nrm + v; o2 = p; d2 = nd
    nw += 1
    for k in range(len(clusters)):
        lp = slab(o2, d2, *cb[k])
        if not lp.any(): continue
        walked += 1
        for (lo, hi) in gb[k]:
            gtot += 1
            if (slab(o2, d2, lo, hi)).any(): gpass += 1
print(cfg, "waves", nw, "clusters", len(clusters), "walked per wave-sweep", round(walked / nw, 2),
      "group boxes passing (wave union) of walked clusters", round(gpass / max(gtot, 1), 3))
