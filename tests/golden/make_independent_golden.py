#!/usr/bin/env python3
"""Golden vectors from the INDEPENDENT pure-Python restatement of trace_vectorized2
(tests/independent_v2.py, written from the reference source without the C oracle).

They are the oracle's second pin: tests/test_independent_v2.py checks the C oracle's f64 build against
them bit for bit (CPU), and tests/test_gpu_parity.py::test_independent_golden checks the HIP kernel's
fp64 path against them (GPU).  Each case: scene, camera parameters, max_bounces, spp, seed ->
linear f64 + rgb8 + ray segments.

  python tests/golden/make_independent_golden.py     # rewrites tests/golden/independent_v2.npz
  python tests/golden/make_independent_golden.py baseline   # rewrites tests/golden/independent_baseline.npz
  python tests/golden/make_independent_golden.py baseline C_f32 --out /tmp/c.npz   # one case (parallel runs),
  python tests/golden/make_independent_golden.py baseline-merge /tmp/c.npz ...      # then merged in

The baseline set (round 4) pins the BASELINE.json configs at their real sizes: strided pixels of
configs B, C, D and E (full image, camera, sphere count, spp and depth), in f64 (the reference's
arithmetic) and fp32 (the headline path), each pixel -> linear + rgb8 + its ray segments.
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import independent_v2 as iv  # noqa: E402
import rt_mi355x as rt  # noqa: E402

SEED = 0x5EED0001
OUT = os.path.join(HERE, "independent_v2.npz")
MAIN = dict(focal_length=10.0, view_angle=30.0, center=(16.0, 2.0, 18.5), look_at=(0.0, 0.0, 0.0),
            up=(0.0, 1.0, 0.0), defocus_angle=0.0)


def quirk_scene():
    """The reference's edge cases in one small scene: a hollow dielectric (a mirror under Q1), a
    metal with fuzz > 1 (clamped), two identical spheres (the later one wins the tie), and a glass
    sphere around the camera (under Q1 a ray starting inside never hits it)."""
    L, M, D = rt.Lambertian, rt.Metal, rt.Dielectric
    return rt.Scene.from_list([
        rt.Sphere((0.0, -1000.0, 0.0), 1000.0, L((0.5, 0.5, 0.5))),
        rt.Sphere((0.0, 1.0, 0.0), 1.0, D(1.5, True)),
        rt.Sphere((-4.0, 1.0, 0.0), 1.0, M((0.7, 0.6, 0.5), 1.7)),
        rt.Sphere((4.0, 1.0, 0.0), 1.0, L((0.8, 0.1, 0.1))),
        rt.Sphere((4.0, 1.0, 0.0), 1.0, L((0.1, 0.1, 0.8))),
        rt.Sphere((16.0, 2.0, 18.5), 0.5, D(1.5, False)),
    ])


SCENES = {"A": lambda: rt.scenes.config_scene("A"), "S100": lambda: rt.scenes.random_spheres(100),
          "S500": lambda: rt.scenes.config_scene("C"), "Q": quirk_scene}

# name: (scene, W, H, depth, spp, camera overrides)
CASES = {}
for sc in ("A", "S100"):
    for spp in (6, 32, 100):          # (C-1) % 2: 1, 1, 0; spp 6 has a partial last chunk
        for depth in (8, 50):
            CASES[f"{sc.lower()}_spp{spp}_d{depth}"] = (sc, 16, 9, depth, spp, {})
CASES["s500_spp16_d50"] = ("S500", 8, 5, 50, 16, {})                      # config C's scene
CASES["q_spp24_d50"] = ("Q", 16, 9, 50, 24, {})                           # quirks
CASES["q_defocus_spp10_d20"] = ("Q", 8, 5, 20, 10, {"defocus_angle": 2.0})   # disk rejection draws


def camera(W, H, over):
    p = dict(MAIN)
    p.update(over)
    return p, iv.camera_new(W, H, p["focal_length"], p["view_angle"], p["center"], p["look_at"], p["up"],
                            p["defocus_angle"])


OUT_BASELINE = os.path.join(HERE, "independent_baseline.npz")
# name: (config, n pixels, precision); pixels spread over the frame by a golden-ratio stride
BASELINE_CASES = {f"{c}_{p}": (c, n, p) for c, n in (("B", 64), ("C", 64), ("D", 32), ("E", 32)) for p in ("f64", "f32")}


def baseline_pixels(W, H, n):
    step = int(W * H * 0.6180339887498949)
    return [(k * step) % (W * H) for k in range(n)]


def main_baseline(names=None, out=OUT_BASELINE):
    """The baseline cases (all, or the named ones merged into the existing file; out: where to write)."""
    data, meta = {}, {}
    if names is not None and os.path.exists(OUT_BASELINE):
        old = np.load(OUT_BASELINE)
        meta = json.loads(str(old["meta"]))
        data = {k: old[k] for k in old.files if k != "meta"}
    for name, (cfg, n, prec) in BASELINE_CASES.items():
        if names is not None and name not in names:
            continue
        W, H, nsph, spp, depth = rt.scenes.CONFIGS[cfg]
        flat = rt.scenes.config_scene(cfg).flatten()
        p, cam = camera(W, H, {})
        px = baseline_pixels(W, H, n)
        lin, rgb, segs = [], [], []
        t0 = time.time()
        for q in px:   # per pixel, so each pixel's segment count is pinned too
            l, c, s = iv.render(flat, cam, spp, depth, SEED, pixels=[q], prec=prec)
            lin += l
            rgb += c
            segs.append(s)
        print(f"{name}: {W}x{H} {nsph} spheres spp {spp} depth {depth} {prec}: {n} pixels, {sum(segs)} segments, "
              f"{time.time() - t0:.1f} s", flush=True)
        data[f"{name}_lin"] = np.array(lin, dtype=np.float64)
        data[f"{name}_rgb"] = np.array(rgb, dtype=np.uint8)
        data[f"{name}_pix"] = np.array(px, dtype=np.int64)
        data[f"{name}_segs"] = np.array(segs, dtype=np.int64)
        meta[name] = {"config": cfg, "W": W, "H": H, "spheres": nsph, "depth": depth, "spp": spp, "precision": prec,
                      "camera": p, "seed": SEED, "pixels": len(px)}
    data["meta"] = np.array(json.dumps(meta))
    if out != OUT_BASELINE:
        data["computed"] = np.array(json.dumps(sorted(names)))
    np.savez_compressed(out, **data)
    print("wrote", out)


def main():
    data = {}
    meta = {}
    for name, (sc, W, H, depth, spp, over) in CASES.items():
        flat = SCENES[sc]().flatten()
        p, cam = camera(W, H, over)
        t0 = time.time()
        lin, rgb, segs = iv.render(flat, cam, spp, depth, SEED)
        print(f"{name}: {W}x{H} spp {spp} depth {depth}: {segs} segments, {time.time() - t0:.1f} s", flush=True)
        data[f"{name}_lin"] = np.array(lin, dtype=np.float64)
        data[f"{name}_rgb"] = np.array(rgb, dtype=np.uint8)
        meta[name] = {"scene": sc, "W": W, "H": H, "depth": depth, "spp": spp, "camera": p, "seed": SEED,
                      "segments": segs}
    data["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(OUT, **data)
    print("wrote", OUT)


if __name__ == "__main__":
    if sys.argv[1:] == ["baseline"]:
        main_baseline()
    elif sys.argv[1:2] == ["baseline"]:
        # baseline CASE... [--out FILE]: recompute the named cases (e.g. after a change of the fp32 draws:
        # B_f32 C_f32 D_f32 E_f32), keeping the others; one process per case, then merge the outputs with
        # baseline-merge FILE...
        args = sys.argv[2:]
        out = OUT_BASELINE
        if "--out" in args:
            i = args.index("--out")
            out = args[i + 1]
            args = args[:i] + args[i + 2:]
        main_baseline(set(args), out)
    elif sys.argv[1:2] == ["baseline-merge"]:
        # a part file holds the whole set with its own case recomputed: take only that case (named by the
        # part file's "computed" entry) from it
        z = np.load(OUT_BASELINE)
        meta = json.loads(str(z["meta"]))
        data = {k: z[k] for k in z.files if k not in ("meta", "computed")}
        for f in sys.argv[2:]:
            z = np.load(f)
            for name in json.loads(str(z["computed"])):
                meta[name] = json.loads(str(z["meta"]))[name]
                data.update({k: z[k] for k in z.files if k.startswith(name + "_")})
        data["meta"] = np.array(json.dumps(meta))
        np.savez_compressed(OUT_BASELINE, **data)
        print("wrote", OUT_BASELINE)
    else:
        main()
