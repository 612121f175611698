#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle (oracle/).

The reference ships no tests or fixtures and cannot be built here, so these
vectors are produced by the oracle restatement; they pin the oracle against drift (CPU test) and
the HIP kernel against the same numbers (GPU test).  Each case: scene, camera (src/main.rs:51-58
camera at the given resolution), max_bounces, spp, seed, precision -> rgb8 + linear + segments.

  python tests/golden/make_golden.py        # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import rt_mi355x as rt  # noqa: E402
from oracle_bind import oracle_render  # noqa: E402

SEED = 0x5EED0001

# name: (scene, width, height, max_bounces, spp, flags, precision, store_linear)
CASES = {
    "config_a": ("A", 400, 225, 8, 16, 0, "f64", False),          # BASELINE configs[0], RGB8 only
    "config_a_f32": ("A", 400, 225, 8, 16, 0, "f32", False),
    "s100_spp32": ("S100", 64, 36, 50, 32, 0, "f64", True),      # (C-1)%2 == 1
    "s100_spp100": ("S100", 48, 27, 50, 100, 0, "f64", True),    # (C-1)%2 == 0 (Q3's other buffer)
    "s100_spp6": ("S100", 48, 27, 50, 6, 0, "f64", True),        # partial last chunk
    "s100_spp32_f32": ("S100", 64, 36, 50, 32, 0, "f32", True),
    "s100_root2": ("S100", 48, 27, 50, 16, 2, "f64", True),      # quirk Q1 off
    "s500_spp64": ("S500", 32, 18, 50, 64, 0, "f64", True),      # config C's scene
}


def scene_for(tag):
    if tag == "A":
        return rt.scenes.three_spheres().flatten()
    return rt.scenes.random_spheres(int(tag[1:])).flatten()


def render_case(name):
    tag, w, h, depth, spp, flags, prec, store_lin = CASES[name]
    flat = scene_for(tag)
    cam = rt.camera_new_py(w, h, **rt.MAIN_CAMERA)
    rgb, lin, segs, rc = oracle_render(flat, cam, depth, spp, SEED, flags, precision=prec)
    assert rc == 0
    return rgb.reshape(h, w, 3), (lin.reshape(h, w, 3) if store_lin else None), segs


def main():
    for name, case in CASES.items():
        rgb, lin, segs = render_case(name)
        tag, w, h, depth, spp, flags, prec, _ = case
        data = dict(rgb8=rgb, segments=np.uint64(segs), width=w, height=h, max_bounces=depth, spp=spp,
                    flags=flags, precision=prec, scene=tag, seed=np.uint64(SEED))
        if lin is not None:
            data["linear"] = lin
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **data)
        print(name, rgb.shape, segs)


if __name__ == "__main__":
    main()
