"""GPU tests added in round 2: the fp32 headline against the reference's fp64 arithmetic at the benched
size, fp64 at the 8-GPU configs' sizes, wave-occupancy builds compared bit for bit, the renderer's
scene cache, and the executed-work counters behind the bench's roofline.

fp64 is bit-exact against the oracle's fp64 build (the reference's arithmetic: f64 everywhere,
explicit FMA at /root/reference/src/geometry.rs:434-436,466-468 and src/objects.rs:257), so a GPU
fp64 render stands in for the reference arithmetic on whole frames the CPU oracle cannot render in
test time.
"""
import numpy as np
import pytest

import rt_mi355x as rt
from rt_mi355x import abi
from oracle_bind import oracle_render

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001


def cam_for(w, h):
    return rt.camera_new_py(w, h, **rt.MAIN_CAMERA)


def render(renderer, flat, cam, depth, spp, flags, seed=SEED, tile=None):
    renderer.seed = seed
    renderer.flags = flags
    rgb, lin, st, rc = renderer.render_flat(depth, spp, flat, cam, tile_range=tile, want_linear=True)
    assert rc == 0
    return rgb, lin, st


def spot_check(flat, cam, depth, spp, lin, rows, n_spot, precision):
    """n_spot strided pixels of a (row-strided) render against the oracle, bit for bit."""
    w = cam.image_width
    idx = np.unique((np.arange(n_spot, dtype=np.int64) * 7919) % len(lin))
    px = (rows[idx // w] * w + idx % w).astype(np.uint32)
    _, lin_o, _, rc = oracle_render(flat, cam, depth, spp, SEED, 0, pixels=px, precision=precision)
    assert rc == 0
    bad = np.flatnonzero((lin[idx] != lin_o).any(axis=1))
    assert bad.size == 0, f"{bad.size} of {len(idx)} spot pixels differ, first pixel {px[bad[0]]}"


# ---------------------------------------------------------------- fp32 against fp64 at config C
def test_fp32_tracks_fp64_at_config_c(renderer):
    """north_star's stated fp32 tolerance, at the benched size (config C, 1920x1080, 512 spp).  fp32 draws
    its own Philox2x32 stream (rt_device.hpp rng<T>), so the fp32 frame is an independent estimate of the
    image the fp64 frame estimates: (1) every channel's image mean within 0.5 % of the fp64 frame's, and
    (2) its per-pixel differences from the fp64 frame no larger than those of an fp64 frame of another
    seed (a bias of the fp32 arithmetic would add to them): median |difference| within 3 % and RMSE within
    5 % of the fp64 seed-to-seed values (two million pixels: both ratios of unbiased estimates stay within
    about 1 %)."""
    w, h, _, spp, depth = rt.scenes.CONFIGS["C"]
    flat = rt.scenes.config_scene("C").flatten()
    cam = cam_for(w, h)
    _, l32, _ = render(renderer, flat, cam, depth, spp, abi.RT_FLAG_F32)
    _, l64, _ = render(renderer, flat, cam, depth, spp, 0)
    _, l64b, _ = render(renderer, flat, cam, depth, spp, 0, seed=SEED + 1)
    m32, m64 = l32.mean(axis=0), l64.mean(axis=0)
    assert np.all(np.abs(m32 / m64 - 1.0) < 0.005), (m32, m64)
    rmse = float(np.sqrt(np.mean((l32 - l64) ** 2)))
    noise = float(np.sqrt(np.mean((l64b - l64) ** 2)))
    med = float(np.median(np.abs(l32 - l64)) / np.median(np.abs(l64b - l64)))
    assert rmse < 1.05 * noise, (rmse, noise)
    assert 0.97 < med < 1.03, med
    # recorded by the run (pytest -s)
    print(f"config C: fp32/fp64 channel means {m32 / m64}, rmse fp32-fp64 {rmse:.3e}, "
          f"fp64 seed-to-seed {noise:.3e}, median |diff| ratio {med:.4f}")


# ---------------------------------------------------------------- fp64 at the BASELINE sizes
@pytest.mark.parametrize("config,flags,stride,n_spot", [
    ("B", 0, 1, 512),                    # config B, whole frame, fp64
    ("C", abi.RT_FLAG_F32, 1, 512),      # config C, whole frame (spot-checked more densely than round 1)
    ("C", 0, 1, 512),
    ("D", 0, 1, 512),                    # config D, whole 3840x2160 frame at 1024 spp, fp64
    ("D", abi.RT_FLAG_F32, 8, 512),      # one rank's shard of the 8-GPU partition
    ("E", 0, 8, 256),                    # config E at its real 2048 spp, fp64, one 8-way shard
    ("E", abi.RT_FLAG_F32, 8, 256),
])
def test_baseline_sizes_oracle_spots(renderer, config, flags, stride, n_spot):
    """Every BASELINE config at its full image size, spp and sphere count, in fp64 (the reference's
    arithmetic) and fp32: deterministic across launches, and hundreds of strided pixels bit-identical
    to the oracle (/root/reference/src/renderer.rs:141-176 restated)."""
    w, h, n_sph, spp, depth = rt.scenes.CONFIGS[config]
    flat = rt.scenes.config_scene(config).flatten()
    assert flat.n_spheres == n_sph
    cam = cam_for(w, h)
    tile = rt.parallel.shard_range(w, h, stride, stride // 2) if stride > 1 else None
    rows = np.arange(stride // 2, h, stride) if stride > 1 else np.arange(h)
    rgb, lin, st = render(renderer, flat, cam, depth, spp, flags, tile=tile)
    assert lin.shape == (len(rows) * w, 3)
    assert st.samples == len(rows) * w * spp
    _, lin2, st2 = render(renderer, flat, cam, depth, spp, flags, tile=tile)
    np.testing.assert_array_equal(lin, lin2)
    assert st.ray_segments == st2.ray_segments
    spot_check(flat, cam, depth, spp, lin, rows, n_spot, "f32" if flags & abi.RT_FLAG_F32 else "f64")
    assert 0.2 < lin.mean() < 0.9 and 1.0 < st.ray_segments / st.samples < 4.0


# ---------------------------------------------------------------- occupancy builds, bit for bit
@pytest.mark.parametrize("config,flags,waves", [
    ("C", abi.RT_FLAG_F32, ("4", "5", "6", "7")),   # the whole benched frame; 7 is clamped to 6
    ("B", 0, ("4", "5", "6")),                      # fp64: 6 is clamped to 5
])
def test_wave_builds_bit_identical(renderer, monkeypatch, config, flags, waves):
    """RT_WAVES selects the register-allocation target (waves per SIMD) at every launch; every
    build must give the same linear image, RGB8 bytes and segment count on a whole frame."""
    w, h, _, spp, depth = rt.scenes.CONFIGS[config]
    flat = rt.scenes.config_scene(config).flatten()
    cam = cam_for(w, h)
    ref = None
    for wv in waves:
        monkeypatch.setenv("RT_WAVES", wv)
        rgb, lin, st = render(renderer, flat, cam, depth, spp, flags)
        if ref is None:
            ref = (rgb, lin, st.ray_segments)
        else:
            np.testing.assert_array_equal(lin, ref[1])
            np.testing.assert_array_equal(rgb, ref[0])
            assert st.ray_segments == ref[2]


def test_wave_builds_defocus(renderer, monkeypatch):
    """The defocus-camera (general path) kernels honour RT_WAVES too, with identical results."""
    flat = rt.scenes.random_spheres(100).flatten()
    args = dict(rt.MAIN_CAMERA)
    args["defocus_angle"] = 2.0
    cam = rt.camera_new_py(64, 36, **args)
    outs = []
    for wv in ("4", "5", "6", "7"):
        monkeypatch.setenv("RT_WAVES", wv)
        outs.append(render(renderer, flat, cam, 50, 16, abi.RT_FLAG_F32)[1])
    for o in outs[1:]:
        np.testing.assert_array_equal(outs[0], o)
    _, lin_o, _, _ = oracle_render(flat, cam, 50, 16, SEED, 0, precision="f32")
    np.testing.assert_array_equal(outs[0], lin_o)


# ---------------------------------------------------------------- the renderer's scene cache
def test_two_scenes_in_a_row(renderer):
    """GpuRenderer.render flattens the scene on every call: rendering scene A and then scene B (each a
    fresh temporary FlatScene, so CPython may reuse A's freed address for B's) must draw B."""
    cam = rt.Camera(48, 27, **rt.MAIN_CAMERA)
    a = rt.scenes.three_spheres()
    b = rt.scenes.random_spheres(100)
    renderer.seed, renderer.flags = SEED, 0
    img_a, _ = renderer.render(8, 8, a, cam)
    img_b, _ = renderer.render(8, 8, b, cam)
    img_a2, _ = renderer.render(8, 8, a, cam)
    want_b = oracle_render(b.flatten(), cam.abi, 8, 8, SEED)[0].reshape(27, 48, 3)
    want_a = oracle_render(a.flatten(), cam.abi, 8, 8, SEED)[0].reshape(27, 48, 3)
    np.testing.assert_array_equal(img_b, want_b)
    np.testing.assert_array_equal(img_a, want_a)
    np.testing.assert_array_equal(img_a2, want_a)


# ---------------------------------------------------------------- executed-work counters
def test_work_counters(renderer):
    """The roofline's executed-work counters: depth 1 traces primary rays only (camera sweep, no
    general sweep); deeper renders add general-sweep box, filter and exact tests; the FLOP they
    imply never exceed what the chip can execute in the launch time."""
    flat = rt.scenes.config_scene("C").flatten()
    cam = cam_for(320, 180)
    _, _, s1 = render(renderer, flat, cam, 1, 64, abi.RT_FLAG_F32)
    assert s1.box_groups == s1.filter_groups == s1.exact_tests == 0
    assert s1.cone_tests > 0 and s1.camera_exact_tests > 0
    _, _, s50 = render(renderer, flat, cam, 50, 64, abi.RT_FLAG_F32)
    assert s50.box_groups > 0 and s50.filter_groups > 0 and s50.exact_tests > 0
    f32, f64 = abi.executed_flop(s50, "f32")
    assert f64 == 0 and f32 > 0
    assert f32 / (s50.kernel_ms / 1e3) < 157.3e12
    _, _, d64 = render(renderer, flat, cam, 50, 64, 0)
    g32, g64 = abi.executed_flop(d64, "f64")
    assert g64 > 0 and g32 > 0


# ---------------------------------------------------------------- big scenes: the mega-box level
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_config_e_filter_off_same_image(renderer, monkeypatch, flags):
    """Config E's 10 000 spheres take the four-level general sweep (mega boxes over 4 supers each):
    every box level on and off (RT_FILTER_OFF: every lane degenerate, every box passes) must give the
    oracle's image, pixel for pixel."""
    flat = rt.scenes.config_scene("E").flatten()
    cam = cam_for(24, 14)
    _, lin_on, st_on = render(renderer, flat, cam, 50, 32, flags)
    _, lin_o, segs_o, _ = oracle_render(flat, cam, 50, 32, SEED, 0, precision="f32" if flags else "f64")
    np.testing.assert_array_equal(lin_on, lin_o)
    assert st_on.ray_segments == segs_o
    monkeypatch.setenv("RT_FILTER_OFF", "1")
    _, lin_off, st_off = render(renderer, flat, cam, 50, 32, flags)
    np.testing.assert_array_equal(lin_off, lin_o)
    assert st_off.box_groups > st_on.box_groups and st_off.filter_groups > st_on.filter_groups


def test_launch_size_rule_same_pixels(renderer, monkeypatch):
    """The default occupancy depends on the launch's size (fp32 runs at W5 below kW6PixelsPerWave pixels
    per resident W6 wave, rt_common.hpp; the whole frame of C and its 8-way shards, ~42 pixels per W6
    wave, both run at W6, so this checks the shard path's other work decomposition): the shard's rows must
    equal the same rows of the whole frame, bit for bit, with RT_WAVES unset."""
    monkeypatch.delenv("RT_WAVES", raising=False)
    w, h, _, spp, depth = rt.scenes.CONFIGS["C"]
    flat = rt.scenes.config_scene("C").flatten()
    cam = cam_for(w, h)
    rgb_f, lin_f, _ = render(renderer, flat, cam, depth, spp, abi.RT_FLAG_F32)
    for rank in (0, 5):
        tile = rt.parallel.shard_range(w, h, 8, rank)
        rgb_s, lin_s, st = render(renderer, flat, cam, depth, spp, abi.RT_FLAG_F32, tile=tile)
        rows = np.arange(rank, h, 8)
        np.testing.assert_array_equal(lin_s.reshape(len(rows), w, 3), lin_f.reshape(h, w, 3)[rows])
        np.testing.assert_array_equal(rgb_s.reshape(len(rows), w, 3), rgb_f.reshape(h, w, 3)[rows])


def test_config_e_wave_builds(renderer, monkeypatch):
    """The mega-level kernels at 6 (the fp32 default, kWavesMegaF32) and 5 waves, and the W4 kernel that
    sweeps the same scene from the super boxes: one image, one segment count, the oracle's."""
    flat = rt.scenes.config_scene("E").flatten()
    cam = cam_for(32, 18)
    _, lin_o, segs_o, _ = oracle_render(flat, cam, 50, 16, SEED, 0, precision="f32")
    for wv in (None, "5", "6", "4"):
        if wv is None:
            monkeypatch.delenv("RT_WAVES", raising=False)
        else:
            monkeypatch.setenv("RT_WAVES", wv)
        _, lin, st = render(renderer, flat, cam, 50, 16, abi.RT_FLAG_F32)
        np.testing.assert_array_equal(lin, lin_o, err_msg=f"RT_WAVES={wv}")
        assert st.ray_segments == segs_o


# ---------------------------------------------------------------- vectorized3 (render_vectorized3)
@pytest.mark.parametrize("spp,prec", [(512, 0), (100, abi.RT_FLAG_F32), (1024, abi.RT_FLAG_F32), (130, 0)])
def test_vectorized3_large_spp(renderer, spp, prec):
    """trace_vectorized3's swap partition replayed over many 64-slot passes (P up to 1024), bit-exact
    against the oracle's literal two-pointer loop (ray_tracing.rs:561-607)."""
    flat = rt.scenes.random_spheres(100).flatten()
    cam = cam_for(12, 7)
    rgb, lin, st = render(renderer, flat, cam, 50, spp, abi.RT_FLAG_MODE_VECTORIZED3 | prec)
    rgb_o, lin_o, segs_o, _ = oracle_render(flat, cam, 50, spp, SEED, abi.RT_FLAG_MODE_VECTORIZED3,
                                            precision="f32" if prec else "f64")
    np.testing.assert_array_equal(lin, lin_o)
    np.testing.assert_array_equal(rgb, rgb_o)
    assert st.ray_segments == segs_o


@pytest.mark.parametrize("depth", [60, 200])
def test_vectorized3_long_paths(renderer, depth):
    """Camera inside a glass sphere with root2 allowed: some rays stay trapped for all `depth` bounces,
    so the partition is replayed for up to 200 bounces with survivors in the active chunks."""
    flat = rt.FlatScene(np.array([[16.0, 2.0, 56.5]]), np.array([40.0]), np.array([0], np.uint32),
                        [rt.Dielectric(1.5, False)])
    cam = cam_for(16, 9)
    flags = abi.RT_FLAG_MODE_VECTORIZED3 | abi.RT_FLAG_ROOT2
    _, lin, st = render(renderer, flat, cam, depth, 24, flags)
    _, lin_o, segs_o, _ = oracle_render(flat, cam, depth, 24, SEED, flags)
    np.testing.assert_array_equal(lin, lin_o)
    assert st.ray_segments == segs_o
