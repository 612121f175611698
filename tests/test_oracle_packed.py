"""The reference-shaped CPU baseline (oracle/packed_avx2.h: explicit 4-lane f64 AVX2 packets like
PackedRays<4>, 128x128 tiles through a shared queue, renderer.rs:243-296) computes exactly what the
scalar oracle computes: it only runs the reference's packed path the way the reference runs it, for
bench.py's cpu_baseline.packed timing.  Test infrastructure only."""
import numpy as np
import pytest

import rt_mi355x as rt
from oracle_bind import oracle_render, packed_render

SEED = 0x5EED0001


def test_config_a_bit_identical():
    """BASELINE configs[0] (400x225, the 3-sphere scene, 16 spp, 8 bounces) in full: every pixel equal
    to the scalar oracle's f64 build, bytes and linear values, and the same ray segments."""
    flat = rt.scenes.config_scene("A").flatten()
    cam = rt.camera_new_py(400, 225, **rt.MAIN_CAMERA)
    rgb, lin, segs, pix, rc = packed_render(flat, cam, 8, 16, SEED)
    rgb_o, lin_o, segs_o, rc_o = oracle_render(flat, cam, 8, 16, SEED)
    assert rc == rc_o == 0 and pix == 400 * 225
    assert segs == segs_o
    assert np.array_equal(lin, lin_o) and np.array_equal(rgb, rgb_o)


@pytest.mark.parametrize("spp,depth", [(6, 50), (32, 50), (33, 3), (1, 1)])
def test_random_scene_tiles(spp, depth):
    """A 100-sphere scene on a 70x40 image in 16x16 tiles (ragged edge tiles), spp with partial chunks
    and both values of (C-1)%2; and a subset of the tiles (the rest stays zero)."""
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(70, 40, **rt.MAIN_CAMERA)
    rgb, lin, segs, pix, rc = packed_render(flat, cam, depth, spp, SEED, tile=16)
    rgb_o, lin_o, segs_o, rc_o = oracle_render(flat, cam, depth, spp, SEED)
    assert rc == rc_o and pix == 70 * 40 and segs == segs_o   # spp 1: the partial chunk's sky(0) lanes
    assert np.array_equal(lin, lin_o) and np.array_equal(rgb, rgb_o)   # push channels past 2.0 (rc 3)
    # tiles 1 and 7 of the 5 x 3 grid only
    rgb2, lin2, segs2, pix2, rc2 = packed_render(flat, cam, depth, spp, SEED, tiles=[1, 7], tile=16)
    mask = np.zeros((40, 70), dtype=bool)
    mask[0:16, 16:32] = True
    mask[16:32, 32:48] = True
    m = mask.reshape(-1)
    assert rc2 == rc and pix2 == 2 * 256
    assert np.array_equal(lin2[m], lin_o[m]) and not lin2[~m].any()


def test_config_c_tile():
    """Config C's scene and camera (1920x1080, 500 spheres, depth 50) on one 128x128 tile at 8 spp."""
    flat = rt.scenes.config_scene("C").flatten()
    cam = rt.camera_new_py(1920, 1080, **rt.MAIN_CAMERA)
    tile = 15 * 5 + 7   # a tile over the spheres (15 tiles per row)
    rgb, lin, segs, pix, rc = packed_render(flat, cam, 50, 8, SEED, tiles=[tile])
    r0, c0 = 5 * 128, 7 * 128
    px = np.array([(r0 + r) * 1920 + c0 + c for r in range(128) for c in range(128)], dtype=np.uint32)
    rgb_o, lin_o, segs_o, rc_o = oracle_render(flat, cam, 50, 8, SEED, pixels=px)
    assert rc == rc_o == 0 and pix == 128 * 128 and segs == segs_o
    assert np.array_equal(lin[px], lin_o) and np.array_equal(rgb[px], rgb_o)


def test_bad_arguments():
    flat = rt.scenes.config_scene("A").flatten()
    cam = rt.camera_new_py(40, 20, **rt.MAIN_CAMERA)
    assert packed_render(flat, cam, 8, 0, SEED)[4] == 1            # spp 0
    assert packed_render(flat, cam, 8, 4, SEED, tiles=[9])[4] == 1  # past the 1 x 1 tile grid
