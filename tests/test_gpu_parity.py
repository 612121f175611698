"""GPU parity: the HIP megakernel (through the C ABI) against the CPU restatement in oracle/.

Bar: same (seed, pixel, sample) keys -> the kernel follows the oracle's exact arithmetic
(FMA placement, correctly rounded div/sqrt, reference summation order), so the per-pixel
linear colours must be BIT-IDENTICAL in both fp64 and fp32 mode, and RGB8 byte-identical.
Tolerance stated for the record: 0 ulp (we assert array_equal).
"""
import ctypes
import math

import numpy as np
import pytest

import rt_mi355x as rt
from rt_mi355x import abi
from oracle_bind import oracle_render

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001


def cam_for(w, h):
    return rt.camera_new_py(w, h, **rt.MAIN_CAMERA)


def gpu(renderer, flat, cam, depth, spp, seed=SEED, flags=0, tile=None):
    renderer.seed = seed
    renderer.flags = flags
    rgb, lin, st, rc = renderer.render_flat(depth, spp, flat, cam, tile_range=tile, want_linear=True)
    return rgb, lin, st, rc


def assert_parity(renderer, flat, cam, depth, spp, flags=0, seed=SEED):
    prec = "f32" if flags & abi.RT_FLAG_F32 else "f64"
    rgb_g, lin_g, st, rc_g = gpu(renderer, flat, cam, depth, spp, seed, flags)
    rgb_o, lin_o, segs_o, rc_o = oracle_render(flat, cam, depth, spp, seed, flags & ~abi.RT_FLAG_F32,
                                               precision=prec)
    assert rc_g == rc_o
    diff = np.argwhere(lin_g != lin_o)
    assert diff.size == 0, (
        f"{len(diff)} mismatching channels; first pixel {diff[0][0]}: gpu {lin_g[diff[0][0]]} oracle {lin_o[diff[0][0]]}")
    np.testing.assert_array_equal(rgb_g, rgb_o)
    assert st.ray_segments == segs_o
    assert st.samples == cam.image_width * cam.image_height * spp
    return lin_g, st


@pytest.fixture(scope="module")
def scene_a():
    return rt.scenes.config_scene("A").flatten()


@pytest.fixture(scope="module")
def scene_100():
    return rt.scenes.random_spheres(100).flatten()


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_config_a_full(renderer, scene_a, flags):
    """Config A exactly as BASELINE.json names it: 400x225, 3 spheres, 16 spp, 8 bounces."""
    lin, st = assert_parity(renderer, scene_a, cam_for(400, 225), 8, 16, flags)
    assert 0.0 < lin.mean() < 1.0


@pytest.mark.parametrize("spp", [1, 4, 6, 32, 100])
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_random_scene_spp(renderer, scene_100, spp, flags):
    """spp 1/6 exercise partial chunks, 100 has (C-1)%2 == 0 (quirk Q3's other buffer)."""
    assert_parity(renderer, scene_100, cam_for(96, 54), 50, spp, flags)


@pytest.mark.parametrize("depth", [0, 1, 2, 3])
@pytest.mark.parametrize("spp", [6, 8, 12])
def test_depth_edges(renderer, scene_100, depth, spp):
    assert_parity(renderer, scene_100, cam_for(48, 27), depth, spp, 0)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_ROOT2, abi.RT_FLAG_ROOT2 | abi.RT_FLAG_F32])
def test_root2_mode(renderer, scene_100, flags):
    assert_parity(renderer, scene_100, cam_for(64, 36), 50, 16, flags)


def test_empty_scene(renderer):
    """hitables = [] -> every sample misses at bounce 0: pixel = mean sky(primary y)."""
    flat = rt.FlatScene(np.zeros((0, 3)), np.zeros(0), np.zeros(0, np.uint32), [rt.Lambertian((0.5, 0.5, 0.5))])
    lin, st = assert_parity(renderer, flat, cam_for(40, 30), 8, 8, 0)
    assert np.all((lin > 0.5) & (lin <= 1.0)) and st.ray_segments == 40 * 30 * 8


@pytest.mark.parametrize("depth", [2, 50])
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
@pytest.mark.parametrize("spp", [1, 6, 100, 512])
def test_sky_pixels(renderer, spp, flags, depth):
    """Every sample escapes at bounce 0.  With this pinhole camera every pixel's camera candidate list is
    empty, so trace_paths finishes it when it claims it (finish_sky_direct: no slot, no lanes, no
    records); test_sky_pixels_defocus takes finish_pixel's sky path instead.  Partial chunks (1, 6),
    quirk Q3's other buffer (100), config C's spp (512), both precisions."""
    flat = rt.FlatScene(np.zeros((0, 3)), np.zeros(0), np.zeros(0, np.uint32), [rt.Lambertian((0.5, 0.5, 0.5))])
    assert_parity(renderer, flat, cam_for(16, 9), depth, spp, flags)


def test_large_spp(renderer, scene_100):
    assert_parity(renderer, scene_100, cam_for(8, 6), 50, 1024, 0)            # P = 1024, fp64
    assert_parity(renderer, scene_100, cam_for(8, 6), 50, 2048, abi.RT_FLAG_F32)  # two slots per thread


def test_fp64_2048(renderer, scene_100):
    """Config E's spp in fp64 (per-wave scratch has no LDS ceiling)."""
    assert_parity(renderer, scene_100, cam_for(4, 3), 50, 2048, 0)


def test_wide_records(renderer, scene_100):
    """The scratch formats' wide variants (PScratch): more than 32764 positions per pixel take a u32
    position map (u16 entries keep the bounce-0 "white" flag in bit 15), depth > 254 takes u32
    termination bounces.  Both sides of the map's boundary, in both precisions."""
    assert_parity(renderer, scene_100, cam_for(2, 1), 50, 70001, abi.RT_FLAG_F32)   # P = 70004 > 65532
    assert_parity(renderer, scene_100, cam_for(2, 1), 50, 32761, abi.RT_FLAG_F32)   # P = 32764: u16
    assert_parity(renderer, scene_100, cam_for(2, 1), 50, 32765, 0)                 # P = 32768: u32
    assert_parity(renderer, scene_100, cam_for(16, 9), 300, 16, 0)                 # depth 300 > 254


def test_spp_limit(renderer, scene_100):
    with pytest.raises(rt.RtError) as e:
        gpu(renderer, scene_100, cam_for(2, 2), 50, (1 << 20) + 1, flags=abi.RT_FLAG_F32)
    assert e.value.code == abi.RT_ERR_UNSUPPORTED


def test_f32_bounce_limit(renderer, scene_100):
    """fp32 draws Philox2x32 with the counter (pixel, sample | (257 + bounce) << 20): max_bounces up to
    RT_MAX_BOUNCES_F32 renders (bit-exact against the oracle, which has the same limit), one more is
    RT_ERR_UNSUPPORTED; fp64 (Philox4x32, the bounce in its own word) has no such limit."""
    assert_parity(renderer, scene_100, cam_for(2, 1), abi.RT_MAX_BOUNCES_F32, 8, abi.RT_FLAG_F32)
    with pytest.raises(rt.RtError) as e:
        gpu(renderer, scene_100, cam_for(2, 1), abi.RT_MAX_BOUNCES_F32 + 1, 8, flags=abi.RT_FLAG_F32)
    assert e.value.code == abi.RT_ERR_UNSUPPORTED
    assert_parity(renderer, scene_100, cam_for(2, 1), abi.RT_MAX_BOUNCES_F32 + 1, 8, 0)


def test_tile_ranges_compose(renderer, scene_100):
    """Row-interleaved shards (the multi-GPU partition) reassemble the full image bit-exactly."""
    cam = cam_for(64, 36)
    _, full, _, _ = gpu(renderer, scene_100, cam, 50, 16)
    full = full.reshape(36, 64, 3)
    for world in (2, 3):
        for r in range(world):
            rows = len(range(r, 36, world))
            tile = abi.RtTileRange(r, world, rows, 0, 64)
            _, part, _, _ = gpu(renderer, scene_100, cam, 50, 16, tile=tile)
            np.testing.assert_array_equal(part.reshape(rows, 64, 3), full[r::world])
    tile = abi.RtTileRange(5, 1, 7, 11, 20)
    _, part, _, _ = gpu(renderer, scene_100, cam, 50, 16, tile=tile)
    np.testing.assert_array_equal(part.reshape(7, 20, 3), full[5:12, 11:31])


def test_range_error(renderer):
    """albedo > 1 pushes a pixel above 2.0: the reference panics (color.rs:55-57); we return
    RT_ERR_RANGE with the image written, and the oracle flags the same pixels."""
    flat = rt.FlatScene(np.array([[0.0, 0.0, 0.0]]), np.array([5.0]), np.array([0], np.uint32),
                        [rt.Lambertian((9.0, 9.0, 9.0))])
    cam = cam_for(16, 9)
    rgb_g, lin_g, _, rc = gpu(renderer, flat, cam, 4, 8)
    rgb_o, lin_o, _, rc_o = oracle_render(flat, cam, 4, 8, SEED)
    assert rc == abi.RT_ERR_RANGE and rc_o == abi.RT_ERR_RANGE
    np.testing.assert_array_equal(lin_g, lin_o)
    np.testing.assert_array_equal(rgb_g, rgb_o)


def test_invalid_arguments(renderer, scene_100, lib):
    cam = cam_for(8, 6)
    with pytest.raises(rt.RtError) as e:
        gpu(renderer, scene_100, cam, 8, 0)
    assert e.value.code == abi.RT_ERR_INVALID
    bad = rt.FlatScene(np.zeros((1, 3)), np.ones(1), np.array([3], np.uint32), [rt.Lambertian((1, 1, 1))])
    rc = lib.rt_context_set_scene(renderer.ctx, ctypes.byref(bad.abi))
    assert rc == abi.RT_ERR_INVALID
    assert b"material index" in lib.rt_last_error()
    with pytest.raises(rt.RtError):
        gpu(renderer, scene_100, cam, 8, 4, tile=abi.RtTileRange(0, 1, 7, 0, 8))   # 7 rows > 6


def test_one_shot_rt_render(lib, scene_100):
    """rt_render (host in/out) equals the device-resident path."""
    cam = cam_for(32, 18)
    rgb = np.zeros((32 * 18, 3), np.uint8)
    lin = np.zeros((32 * 18, 3), np.float64)
    st = abi.RtStats()
    rc = lib.rt_render(ctypes.byref(scene_100.abi), ctypes.byref(cam), 50, 16, SEED, 0, None,
                       rgb.ctypes.data, lin.ctypes.data, ctypes.byref(st))
    assert rc == abi.RT_OK
    rgb_o, lin_o, segs, _ = oracle_render(scene_100, cam, 50, 16, SEED)
    np.testing.assert_array_equal(lin, lin_o)
    assert st.ray_segments == segs and st.seconds > 0


def test_seed_changes_image(renderer, scene_100):
    cam = cam_for(32, 18)
    _, a, _, _ = gpu(renderer, scene_100, cam, 50, 8, seed=1)
    _, b, _, _ = gpu(renderer, scene_100, cam, 50, 8, seed=2)
    _, c, _, _ = gpu(renderer, scene_100, cam, 50, 8, seed=1)
    assert not np.array_equal(a, b)
    np.testing.assert_array_equal(a, c)


@pytest.mark.parametrize("seeds", [(0, 0x100000001), (0x5EED0001, 0x5EED0001 ^ (7 << 32) ^ 7),
                                   (0x1234, 0x1234 << 32)])
def test_f32_seed_key_uses_all_64_bits(renderer, scene_100, seeds):
    """fp32 keys Philox2x32 with seed lo ^ fmix32(seed hi) (rt_device.hpp rng<float>): seeds that a plain
    lo ^ hi fold sends to one key (0 and (1 << 32) | 1; (a, b) and (a ^ m, b ^ m); swapped halves) render
    different fp32 images, each bit-equal to the oracle's fp32 build."""
    cam = cam_for(32, 18)
    a, _ = assert_parity(renderer, scene_100, cam, 50, 8, abi.RT_FLAG_F32, seed=seeds[0])
    b, _ = assert_parity(renderer, scene_100, cam, 50, 8, abi.RT_FLAG_F32, seed=seeds[1])
    assert not np.array_equal(a, b)


def test_renderer_trait(renderer):
    """GpuRenderer.render mirrors Renderer::render (renderer.rs:38-40)."""
    scene = rt.scenes.three_spheres()
    cam = rt.Camera(40, 30, **rt.MAIN_CAMERA)
    img, stat = renderer.render(8, 16, scene, cam)
    assert img.shape == (30, 40, 3) and img.dtype == np.uint8
    assert stat.pixels_rendered() == 1200 and stat.pixels_per_second() > 0


# ---------------------------------------------------------------- committed golden fixtures
import os  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden_cases():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


@pytest.mark.parametrize("name", sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and not f.startswith("independent")))
def test_golden_fixtures_gpu(renderer, name):
    mg = _golden_cases()
    tag, w, h, depth, spp, flags, prec, _ = mg.CASES[name]
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    flat = mg.scene_for(tag)
    cam = cam_for(w, h)
    f = flags | (abi.RT_FLAG_F32 if prec == "f32" else 0)
    rgb, lin, st, rc = gpu(renderer, flat, cam, depth, spp, int(g["seed"]), f)
    assert rc == 0
    np.testing.assert_array_equal(rgb.reshape(h, w, 3), g["rgb8"])
    assert st.ray_segments == int(g["segments"])
    if "linear" in g:
        np.testing.assert_array_equal(lin.reshape(h, w, 3), g["linear"])


def test_independent_golden(renderer):
    """The HIP kernel's fp64 path against the INDEPENDENT restatement's vectors (tests/independent_v2.py,
    written from the reference source without the C oracle; tests/golden/make_independent_golden.py):
    the oracle's second pin, bit for bit, every case (quirk scene, defocus camera, both (C-1)%2)."""
    import json
    import importlib.util
    spec = importlib.util.spec_from_file_location("mig", os.path.join(GOLDEN, "make_independent_golden.py"))
    mig = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mig)
    z = np.load(os.path.join(GOLDEN, "independent_v2.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    assert len(meta) >= 15
    for name, m in meta.items():
        flat = mig.SCENES[m["scene"]]().flatten()
        cam = rt.camera_new_py(m["W"], m["H"], **m["camera"])
        rgb, lin, st, rc = gpu(renderer, flat, cam, m["depth"], m["spp"], m["seed"], 0)
        assert rc == 0, name
        assert st.ray_segments == m["segments"], name
        np.testing.assert_array_equal(lin, z[f"{name}_lin"], err_msg=name)
        np.testing.assert_array_equal(rgb, z[f"{name}_rgb"], err_msg=name)


def _baseline_cases():
    import json
    import os
    z = np.load(os.path.join(GOLDEN, "independent_baseline.npz"), allow_pickle=False)
    return z, json.loads(str(z["meta"]))


@pytest.mark.parametrize("name", sorted(_baseline_cases()[1]))
def test_independent_baseline_golden(renderer, name):
    """The HIP kernel against the INDEPENDENT restatement at every BASELINE config's real size (B, C, D,
    E: image, camera, sphere count, spp, depth), in fp64 AND fp32 (the headline path): strided pixels,
    each launched as a 1x1 tile of the full frame, bit for bit, ray segments per pixel included
    (tests/golden/independent_baseline.npz, make_independent_golden.py baseline)."""
    z, meta = _baseline_cases()
    m = meta[name]
    flat = rt.scenes.config_scene(m["config"]).flatten()
    cam = rt.camera_new_py(m["W"], m["H"], **m["camera"])
    flags = abi.RT_FLAG_F32 if m["precision"] == "f32" else 0
    lin_all, rgb_all = [], []
    for k, q in enumerate(z[f"{name}_pix"]):
        q = int(q)
        tile = abi.RtTileRange(q // m["W"], 1, 1, q % m["W"], 1)
        rgb, lin, st, rc = gpu(renderer, flat, cam, m["depth"], m["spp"], m["seed"], flags, tile=tile)
        assert rc == 0, (name, q)
        assert st.ray_segments == int(z[f"{name}_segs"][k]), (name, q)
        lin_all.append(lin.reshape(3))
        rgb_all.append(rgb.reshape(3))
    np.testing.assert_array_equal(np.array(lin_all), z[f"{name}_lin"], err_msg=name)
    np.testing.assert_array_equal(np.array(rgb_all), z[f"{name}_rgb"], err_msg=name)


# ---------------------------------------------------------------- BASELINE sizes
@pytest.mark.parametrize("config,flags", [("B", abi.RT_FLAG_F32), ("C", abi.RT_FLAG_F32), ("C", 0)])
def test_full_size_configs(renderer, config, flags):
    """Configs B and C at their full BASELINE sizes: deterministic across launches, the two-shard
    row partition reassembles the frame bit-exactly, and a strided pixel subset is bit-identical
    to the oracle (which cannot render the whole frame in test time)."""
    w, h, n_sph, spp, depth = rt.scenes.CONFIGS[config]
    flat = rt.scenes.config_scene(config).flatten()
    cam = cam_for(w, h)
    rgb, lin, st, rc = gpu(renderer, flat, cam, depth, spp, SEED, flags)
    assert rc == 0
    rgb2, lin2, st2, _ = gpu(renderer, flat, cam, depth, spp, SEED, flags)
    np.testing.assert_array_equal(lin, lin2)
    assert st.ray_segments == st2.ray_segments
    img = lin.reshape(h, w, 3)
    for r in range(2):
        part = gpu(renderer, flat, cam, depth, spp, SEED, flags,
                   tile=rt.parallel.shard_range(w, h, 2, r))[1]
        np.testing.assert_array_equal(part.reshape(-1, w, 3), img[r::2])
    px = (np.arange(48, dtype=np.int64) * 43201) % (w * h)
    _, lin_o, _, _ = oracle_render(flat, cam, depth, spp, SEED, 0, pixels=px.astype(np.uint32),
                                   precision="f32" if flags & abi.RT_FLAG_F32 else "f64")
    np.testing.assert_array_equal(lin[px], lin_o)
    assert 0.2 < lin.mean() < 0.9 and 1.0 < st.ray_segments / (w * h * spp) < 4.0


@pytest.mark.parametrize("w,h,spp,depth,stride,flags", [
    (1280, 720, 4, 3, 1, abi.RT_FLAG_F32),   # 921 600 items: 16/8/4/2/1-item blocks in all 16 partitions
    (1920, 1080, 4, 2, 1, 0),
    (1920, 1080, 4, 2, 7, abi.RT_FLAG_F32),  # a row-strided shard (155 rows)
    (7, 3, 8, 4, 1, abi.RT_FLAG_F32),        # fewer items than partitions: empty partitions
    (1, 1, 4, 4, 1, 0),
])
def test_schedule_covers_every_pixel(renderer, scene_100, w, h, spp, depth, stride, flags):
    """The work schedule (pixel blocks claimed from 16 partition counters, guided block sizes,
    stealing) renders every pixel of the range exactly once: the whole frame is bit-identical to
    the oracle, pixel for pixel, and the sample count is exact."""
    cam = cam_for(w, h)
    tile = rt.parallel.shard_range(w, h, stride, 3 % stride) if stride > 1 else None
    rgb, lin, st, rc = gpu(renderer, scene_100, cam, depth, spp, SEED, flags, tile=tile)
    assert rc == 0
    if tile is None:
        px = None
        n = w * h
    else:
        rows = np.arange(3 % stride, h, stride)
        px = (rows[:, None] * w + np.arange(w)[None, :]).reshape(-1).astype(np.uint32)
        n = len(px)
    assert st.samples == n * spp
    rgb_o, lin_o, segs_o, _ = oracle_render(scene_100, cam, depth, spp, SEED, 0, pixels=px,
                                            precision="f32" if flags & abi.RT_FLAG_F32 else "f64")
    assert lin.shape == lin_o.shape
    bad = np.argwhere((lin != lin_o).any(axis=1))
    assert bad.size == 0, f"{len(bad)} pixels differ, first {bad[0][0]}"
    np.testing.assert_array_equal(rgb, rgb_o)
    assert st.ray_segments == segs_o


# ---------------------------------------------------------------- the CLI (main.rs) end to end
def test_cli_renders_config_a_from_toml(tmp_path):
    """rt-render reads scene.toml, renders on the GPU, writes PNG and PPM (src/main.rs:27-74); the
    pixels equal the committed config-A golden fixture (oracle, same default seed)."""
    import subprocess
    from PIL import Image
    cli = os.path.join(os.path.dirname(GOLDEN), "..", "rust-ray-tracing_amd", "bin", "rt-render")
    (tmp_path / "scene.toml").write_text(rt.scenes.scene_to_toml(rt.scenes.three_spheres()))
    want = np.load(os.path.join(GOLDEN, "config_a.npz"))["rgb8"]
    for out in ("output.png", "output.ppm"):
        r = subprocess.run([cli, "--width", "400", "--height", "225", "--spp", "16", "--bounces", "8", "--out", out],
                           cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "Image Size: 400 x 225" in r.stdout and "Total Pixels: 90000" in r.stdout
        assert "Viewport Top Left Corner: [5.734425819985221, 3.855608886593495, 13.912440284912917]" in r.stdout
        img = np.asarray(Image.open(tmp_path / out).convert("RGB"))
        np.testing.assert_array_equal(img, want)


def test_cli_block_size_prints_per_block_rates(tmp_path):
    """rt-render --block-size 128: TileRenderer's 128x128 blocks (renderer.rs:248-266), one launch each,
    one "complete block (x, y) at R px/s" line per block (renderer.rs:339); the same image."""
    import re
    import subprocess
    cli = os.path.join(os.path.dirname(GOLDEN), "..", "rust-ray-tracing_amd", "bin", "rt-render")
    (tmp_path / "scene.toml").write_text(rt.scenes.scene_to_toml(rt.scenes.three_spheres()))
    want = np.load(os.path.join(GOLDEN, "config_a.npz"))["rgb8"]
    r = subprocess.run([cli, "--width", "400", "--height", "225", "--spp", "16", "--bounces", "8", "--out", "o.ppm",
                        "--block-size", "128"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    blocks = re.findall(r"^Device 0 complete block \((\d+), (\d+)\) at ([0-9.]+) px/s$", r.stdout, flags=re.M)
    assert sorted((int(x), int(y)) for x, y, _ in blocks) == [(x, y) for x in range(4) for y in range(2)]
    assert all(float(v) > 0 for _, _, v in blocks)
    raw = (tmp_path / "o.ppm").read_bytes()
    assert raw.startswith(b"P6")
    np.testing.assert_array_equal(np.frombuffer(raw[-400 * 225 * 3:], np.uint8).reshape(225, 400, 3), want)


@pytest.mark.parametrize("flags,spp", [(abi.RT_FLAG_F32, 2048), (0, 256)])
def test_config_e_scene(renderer, flags, spp):
    """Config E's 10 000-sphere scene (2 500 scalar-load groups per ray) at config E's spp (fp32)."""
    flat = rt.scenes.config_scene("E").flatten()
    assert flat.n_spheres == 10000
    assert_parity(renderer, flat, cam_for(4, 3), 50, spp, flags)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_F32, 0])
@pytest.mark.parametrize("n", [3000, 70000])
def test_mega_walk_shapes(renderer, flags, n):
    """The mega kernels' top level in its other shapes (config E: 40 megas in 10 groups, walked in
    distance tiers).  3 000 spheres: 12 megas in 3 groups.  70 000: 274 megas in 69 groups, more than
    the 16 the walk tests at once, so chunks of 8 groups in index order."""
    flat = rt.scenes.random_spheres(n).flatten()
    assert flat.n_spheres == n
    assert_parity(renderer, flat, cam_for(4, 3), 50, 32, flags)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_F32, 0])
@pytest.mark.parametrize("n", [20, 261, 1029, 2053, 2600, 4100])
def test_layout_padding_shapes(renderer, flags, n):
    """The hierarchy-aligned layout (build_layout) at sphere counts just past its units: 16-sphere
    clusters, 64 (supers), 256 (megas) and 1024 (gigas, scenes over 2048 filtered spheres), so
    children are padded with empty clusters in the middle of the streams; and the big spheres in
    the always-exact group.  Against the oracle in both precisions."""
    flat = rt.scenes.random_spheres(n).flatten()
    assert flat.n_spheres == n
    assert_parity(renderer, flat, cam_for(8, 5), 50, 16, flags)


# ---- semantics modes (tests/test_modes.py pins them on the CPU) ----
MODES = [abi.RT_FLAG_MODE_VECTORIZED, abi.RT_FLAG_MODE_VECTORIZED | abi.RT_FLAG_ROOT2, abi.RT_FLAG_MODE_SCALAR,
         abi.RT_FLAG_MODE_VECTORIZED3, abi.RT_FLAG_MODE_VECTORIZED3 | abi.RT_FLAG_ROOT2]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("prec", [0, abi.RT_FLAG_F32])
def test_modes_config_a(renderer, scene_a, mode, prec):
    assert_parity(renderer, scene_a, cam_for(400, 225), 8, 16, mode | prec)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("spp,depth", [(1, 3), (6, 50), (33, 50), (100, 2), (8, 0), (64, 1)])
@pytest.mark.parametrize("prec", [0, abi.RT_FLAG_F32])
def test_modes_scene_100(renderer, scene_100, mode, spp, depth, prec):
    assert_parity(renderer, scene_100, cam_for(24, 14), depth, spp, mode | prec)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_MODE_VECTORIZED | abi.RT_FLAG_MODE_SCALAR,
                                   abi.RT_FLAG_MODE_VECTORIZED3 | abi.RT_FLAG_MODE_VECTORIZED, 0x20, 0x80000000])
def test_invalid_flag_bits(renderer, scene_a, flags):
    with pytest.raises(abi.RtError) as e:
        gpu(renderer, scene_a, cam_for(8, 4), 8, 4, flags=flags)
    assert e.value.code == abi.RT_ERR_INVALID


@pytest.mark.parametrize("mode,flag", [("scalar", abi.RT_FLAG_MODE_SCALAR), ("vectorized", abi.RT_FLAG_MODE_VECTORIZED),
                                       ("vectorized3", abi.RT_FLAG_MODE_VECTORIZED3)])
def test_cli_modes(tmp_path, mode, flag):
    """rt-render --mode: the PPM bytes equal the oracle's image in that mode."""
    import subprocess
    from PIL import Image
    cli = os.path.join(os.path.dirname(GOLDEN), "..", "rust-ray-tracing_amd", "bin", "rt-render")
    scene = rt.scenes.three_spheres()
    (tmp_path / "scene.toml").write_text(rt.scenes.scene_to_toml(scene))
    r = subprocess.run([cli, "--width", "80", "--height", "45", "--spp", "16", "--bounces", "8", "--mode", mode,
                        "--out", "o.ppm"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    img = np.asarray(Image.open(tmp_path / "o.ppm").convert("RGB")).reshape(-1, 3)
    want, _, _, rc = oracle_render(scene.flatten(), cam_for(80, 45), 8, 16, SEED, flags=flag)
    assert rc == 0
    np.testing.assert_array_equal(img, want)


@pytest.mark.parametrize("config,stride,flags", [("D", 1, abi.RT_FLAG_F32), ("E", 32, abi.RT_FLAG_F32)])
def test_full_size_8gpu_configs(renderer, config, stride, flags):
    """Configs D and E (the 8-GPU rows) at their full image size, one GPU: D renders the whole
    3840x2160 frame at 1024 spp; E (10 000 spheres, 2048 spp) renders every 32nd row (one rank's
    shard of a 32-way row partition).  Deterministic, rank shards compose, oracle spot-check."""
    w, h, n_sph, spp, depth = rt.scenes.CONFIGS[config]
    flat = rt.scenes.config_scene(config).flatten()
    cam = cam_for(w, h)
    tile = rt.parallel.shard_range(w, h, stride, 0) if stride > 1 else None
    rgb, lin, st, rc = gpu(renderer, flat, cam, depth, spp, SEED, flags, tile=tile)
    assert rc == 0
    rows = np.arange(0, h, stride)
    assert lin.shape == (len(rows) * w, 3)
    _, lin2, st2, _ = gpu(renderer, flat, cam, depth, spp, SEED, flags, tile=tile)
    np.testing.assert_array_equal(lin, lin2)
    assert st.ray_segments == st2.ray_segments
    # the first two shards of an 8-way split of those rows are the even/odd rows of the render
    if stride == 1:
        img = lin.reshape(h, w, 3)
        part = gpu(renderer, flat, cam, depth, spp, SEED, flags, tile=rt.parallel.shard_range(w, h, 8, 3))[1]
        np.testing.assert_array_equal(part.reshape(-1, w, 3), img[3::8])
    n_spot = 24 if config == "D" else 8
    idx = (np.arange(n_spot, dtype=np.int64) * 7919) % len(lin)
    px = (rows[idx // w] * w + idx % w).astype(np.uint32)
    _, lin_o, _, _ = oracle_render(flat, cam, depth, spp, SEED, 0, pixels=px,
                                   precision="f32" if flags & abi.RT_FLAG_F32 else "f64")
    np.testing.assert_array_equal(lin[idx], lin_o)
    assert 0.2 < lin.mean() < 0.9


# ---- cameras off the pinhole shortcut (Camera::get_ray's disk draw, ray_tracing.rs:80-86) ----
def _cam(w, h, **kw):
    args = dict(rt.MAIN_CAMERA)
    args.update(kw)
    return rt.camera_new_py(w, h, **args)


@pytest.mark.parametrize("mode", [0] + MODES)
@pytest.mark.parametrize("prec", [0, abi.RT_FLAG_F32])
def test_defocus_camera(renderer, scene_100, mode, prec):
    """defocus_angle > 0: every primary ray has its own origin on the lens disk (rejection
    sampling on stream 1), so the kernel takes the general camera path."""
    assert_parity(renderer, scene_100, _cam(24, 14, defocus_angle=2.0), 50, 12, mode | prec)


@pytest.mark.parametrize("prec", [0, abi.RT_FLAG_F32])
def test_negative_zero_camera_centre(renderer, scene_100, prec):
    """No defocus but a -0.0 in the camera centre: du*dx + dv*dy + center turns -0.0 into +0.0,
    so the host must not take the pinhole shortcut (origin == center) — results stay exact."""
    cam = _cam(24, 14, center=(-0.0, 2.0, 18.5), look_at=(0.0, 0.0, 0.0))
    assert cam.center[0] == 0.0 and math.copysign(1.0, cam.center[0]) < 0
    assert_parity(renderer, scene_100, cam, 50, 12, prec)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_ROOT2, abi.RT_FLAG_MODE_SCALAR,
                                   abi.RT_FLAG_MODE_SCALAR | abi.RT_FLAG_F32, abi.RT_FLAG_ROOT2 | abi.RT_FLAG_F32])
def test_every_primary_ray_hits(renderer, flags):
    """Camera inside a big sphere with both roots allowed: every primary ray hits, so each camera
    batch pushes 64 queue entries and the per-wave queue runs full (the top-up stops at 64 free
    slots).  A small sphere inside adds a second, nearer candidate for some rays."""
    mats = [rt.Lambertian((0.6, 0.5, 0.4)), rt.Metal((0.9, 0.9, 0.9), 0.2)]
    flat = rt.FlatScene(np.array([[16.0, 2.0, 18.5], [0.0, 0.0, 0.0]]), np.array([60.0, 3.0]),
                        np.array([0, 1], np.uint32), mats)
    assert_parity(renderer, flat, cam_for(32, 18), 12, 64, flags)


def test_one_context_two_streams(renderer, scene_100):
    """Renders on one context issued to two different streams without any host sync in between:
    the second waits for the first (shared counter, scratch and camera table), so both images
    equal single renders.  Streams come from the HIP runtime the library already loaded."""
    lib = renderer.lib
    hip = ctypes.CDLL("libamdhip64.so.7")
    cam = cam_for(40, 24)
    renderer.set_scene(scene_100)
    npx = 40 * 24
    want = {}
    for seed in (11, 22):
        renderer.seed = seed
        renderer.flags = abi.RT_FLAG_F32
        want[seed] = renderer.render_flat(50, 32, scene_100, cam, want_linear=True)[1]
    streams = [ctypes.c_void_p(), ctypes.c_void_p()]
    for st in streams:
        assert hip.hipStreamCreate(ctypes.byref(st)) == 0
    bufs = [ctypes.c_void_p(), ctypes.c_void_p()]
    for b in bufs:
        abi.check(lib, lib.rt_device_alloc(renderer.ctx, npx * 3 * 8, ctypes.byref(b)))
    try:
        tr = abi.RtTileRange(0, 1, 24, 0, 40)
        for seed, st, b in zip((11, 22), streams, bufs):
            abi.check(lib, lib.rt_render_async(renderer.ctx, ctypes.byref(cam), 50, 32, seed, abi.RT_FLAG_F32,
                                               ctypes.byref(tr), None, b, st))
        stats = abi.RtStats()
        abi.check(lib, lib.rt_context_collect(renderer.ctx, streams[1], ctypes.byref(stats)))
        for seed, b in zip((11, 22), bufs):
            got = np.empty((npx, 3), dtype=np.float64)
            abi.check(lib, lib.rt_memcpy_d2h(renderer.ctx, got.ctypes.data, b, npx * 3 * 8))
            np.testing.assert_array_equal(got, want[seed])
        assert stats.samples == 2 * npx * 32
    finally:
        for b in bufs:
            lib.rt_device_free(renderer.ctx, b)
        for st in streams:
            hip.hipStreamDestroy(st)


@pytest.mark.parametrize("depth", [60, 63, 64, 65, 200])
@pytest.mark.parametrize("prec", [0, abi.RT_FLAG_F32])
def test_long_paths_replay(renderer, depth, prec):
    """Camera inside a glass sphere, 38 units off its centre, with root2 allowed: rays that meet
    the glass beyond the critical angle are trapped by total internal reflection for all `depth`
    bounces, others escape after a few.  Measured per-pixel K (bounce-loop iterations) at depth
    200: 77 pixels at 2-4, 67 at 200, so the position replay in finish_pixel runs far past 64
    bounces, with long and short paths mixed in one wave.  Depths 63 and 64 take the bit-plane replay
    to its widest comparisons (K = 63: 6 planes, K = 64: 7), 65 the per-bounce loop for K > 64."""
    flat = rt.FlatScene(np.array([[16.0, 2.0, 56.5]]), np.array([40.0]), np.array([0], np.uint32),
                        [rt.Dielectric(1.5, False)])
    lin, st = assert_parity(renderer, flat, cam_for(16, 9), depth, 24, abi.RT_FLAG_ROOT2 | prec)
    # bounce_iters sums each pixel's K = min(depth, longest path + 1); measured: 4224 at depth 60
    assert st.bounce_iters > 9 * 16 * (20 if depth < 100 else 40)


# ---- general-sweep distance filter (nearest_hit / filter_group): never changes a result ----

@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32, abi.RT_FLAG_ROOT2 | abi.RT_FLAG_F32, abi.RT_FLAG_MODE_SCALAR])
def test_filter_off_same_image(renderer, scene_100, flags, monkeypatch):
    """RT_FILTER_OFF=1 sends every general-sweep group through the exact test (the path lanes with
    a degenerate basis take); the image must equal both the filtered one and the oracle."""
    cam = cam_for(64, 36)
    lin_f, _ = assert_parity(renderer, scene_100, cam, 50, 16, flags)
    monkeypatch.setenv("RT_FILTER_OFF", "1")
    lin_x, _ = assert_parity(renderer, scene_100, cam, 50, 16, flags)
    np.testing.assert_array_equal(lin_f, lin_x)


def _transformed(flat, scale, offset):
    return rt.FlatScene(flat.center * scale + offset, flat.radius * scale, flat.material, flat.materials)


@pytest.mark.parametrize("scale,offset", [(1e3, 0.0), (1.0, 3e4), (1e-3, 0.0), (37.0, -2.5e3)])
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_filter_scene_scales(renderer, scene_100, scale, offset, flags):
    """The filter margin scales with (max|c|_1 + |o|_1)^2: far-from-origin and tiny scenes keep
    bit parity (the camera moves with the scene)."""
    flat = _transformed(scene_100, scale, offset)
    kw = dict(rt.MAIN_CAMERA)
    kw["center"] = tuple(np.array(kw["center"]) * scale + offset)
    kw["look_at"] = tuple(np.array(kw["look_at"]) * scale + offset)
    kw["focal_length"] = kw["focal_length"] * scale
    cam = rt.camera_new_py(48, 27, **kw)
    assert_parity(renderer, flat, cam, 50, 8, flags)


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_filter_many_exact_spheres(renderer, flags):
    """Radii spanning six decades: many spheres exceed 8x the median |c|_1 + r and get r2f = +inf
    ("always exact"), the rest share a margin set by the largest of them."""
    rng = np.random.default_rng(11)
    n = 61
    r = 10.0 ** rng.uniform(-2, 4, n)
    dirs = rng.standard_normal((n, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    c = dirs * (r[:, None] + rng.uniform(2.0, 30.0, (n, 1)))
    mats = [rt.Lambertian((0.6, 0.5, 0.4)), rt.Metal((0.8, 0.8, 0.9), 0.05), rt.Dielectric(1.5, False)]
    flat = rt.FlatScene(c, r, rng.integers(0, 3, n).astype(np.uint32), mats)
    cam = rt.camera_new_py(40, 30, 2.0, 60.0, (0.0, 0.0, 0.0), (1.0, 0.2, 0.3), (0.0, 1.0, 0.0), 0.0)
    assert_parity(renderer, flat, cam, 50, 8, flags)


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32, abi.RT_FLAG_MODE_VECTORIZED])
def test_camera_inside_and_on_spheres(renderer, flags):
    """Camera-batch filter under Q1: spheres enclosing the camera (c < 0) and one whose surface
    passes through the camera centre (c == 0 exactly) get sc = +inf -- under Q1 root1 <= 0 for
    them, so the reference never hits them either; the spheres in view keep bit parity."""
    cam_kw = dict(rt.MAIN_CAMERA)
    o = np.array(cam_kw["center"])
    rng = np.random.default_rng(5)
    c = [o, o + np.array([2.0, 0.0, 0.0])]                       # enclosing r=60; on-surface r=2
    r = [60.0, 2.0]
    for _ in range(40):
        p = rng.uniform(-4, 4, 3) * np.array([1, 0.3, 1])
        c.append(p); r.append(rng.uniform(0.2, 0.8))
    mats = [rt.Lambertian((0.7, 0.6, 0.5)), rt.Metal((0.9, 0.9, 0.9), 0.1), rt.Dielectric(1.5, False)]
    mi = np.concatenate([[0, 1], rng.integers(0, 3, 40)]).astype(np.uint32)
    flat = rt.FlatScene(np.array(c), np.array(r), mi, mats)
    lin, st = assert_parity(renderer, flat, cam_for(48, 27), 50, 8, flags)
    assert st.ray_segments > 48 * 27 * 8


# ---- camera-batch cone cull (camera_sweep): never changes a result ----

@pytest.mark.parametrize("w,h,vfov,spp", [(1, 1, 150.0, 100), (3, 2, 150.0, 40), (5, 3, 100.0, 100), (7, 5, 30.0, 36)])
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32, abi.RT_FLAG_MODE_SCALAR | abi.RT_FLAG_F32])
def test_cone_cull_wide_pixels(renderer, scene_100, w, h, vfov, spp, flags):
    """Tiny images with wide fields of view: a pixel spans tens of degrees, so some camera batches
    exceed the cull's 30-degree cone and test every sphere, others cull with a wide cone; spp not a
    multiple of 64 makes batches straddle two pixels (one cone over both)."""
    cam = _cam(w, h, view_angle=vfov)
    assert_parity(renderer, scene_100, cam, 50, spp, flags)


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32, abi.RT_FLAG_ROOT2 | abi.RT_FLAG_F32])
def test_cone_cull_dense_tiny_spheres(renderer, flags):
    """3000 spheres with radii 1e-3..0.1 scattered through the view frustum, many grazing the
    primary rays of neighbouring pixels: the cull's margin must keep every sphere the reference's
    arithmetic hits (bit parity with the oracle, every pixel)."""
    rng = np.random.default_rng(17)
    n = 3000
    o = np.array(rt.MAIN_CAMERA["center"])
    fwd = -o / np.linalg.norm(o)
    up = np.array([0.0, 1.0, 0.0])
    right = np.cross(fwd, up); right /= np.linalg.norm(right)
    up2 = np.cross(right, fwd)
    dist = rng.uniform(3.0, 40.0, n)
    x = rng.uniform(-0.28, 0.28, n) * dist
    y = rng.uniform(-0.16, 0.16, n) * dist
    c = o + dist[:, None] * fwd + x[:, None] * right + y[:, None] * up2
    r = 10.0 ** rng.uniform(-3, -1, n)
    mats = [rt.Lambertian((0.7, 0.6, 0.5)), rt.Metal((0.9, 0.9, 0.9), 0.1), rt.Dielectric(1.5, False)]
    flat = rt.FlatScene(c, r, rng.integers(0, 3, n).astype(np.uint32), mats)
    lin, st = assert_parity(renderer, flat, cam_for(64, 36), 8, 16, flags)
    assert st.ray_segments > 64 * 36 * 16 * 1.05   # some primary rays really hit the cloud


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_pixel_lists_overflow_and_straddle(renderer, flags):
    """Per-pixel camera candidate lists (pixel_list): pixels whose cone passes more spheres than a list
    holds (a file of 12 spheres along the view axis, and pixels crossing it) fall back to the per-batch
    sweep; the rest use their lists, with spp 100 batches straddling two pixels.  Bit parity."""
    o = np.array(rt.MAIN_CAMERA["center"])
    fwd = -o / np.linalg.norm(o)
    c = [o + fwd * (3.0 + 2.5 * k) for k in range(12)]
    r = [0.05 + 0.01 * k for k in range(12)]
    rng = np.random.default_rng(23)
    for _ in range(60):
        c.append(rng.uniform(-6, 6, 3) * np.array([1, 0.4, 1])); r.append(rng.uniform(0.2, 0.9))
    mats = [rt.Lambertian((0.7, 0.6, 0.5)), rt.Metal((0.9, 0.9, 0.9), 0.1), rt.Dielectric(1.5, False)]
    flat = rt.FlatScene(np.array(c), np.array(r), rng.integers(0, 3, len(r)).astype(np.uint32), mats)
    assert_parity(renderer, flat, cam_for(31, 17), 50, 100, flags)


# ---- the benched kernels at their production launch shapes, against the independent restatement ----
PRODUCTION_SHAPES = [
    # (golden case, shards, kernel the launch must run)
    ("C_f32", 1, "trace_paths<float,6,false,0,true,false>"),    # bench.py's headline line
    ("C_f64", 1, "trace_paths<double,4,false,0,true,false>"),   # bench.py's f64 leg
    ("D_f32", 8, "trace_paths<float,6,false,0,true,false>"),    # one rank of the 8-GPU D run
    ("E_f32", 8, "trace_paths<float,6,false,0,true,true>"),     # the mega kernel, one rank of E
    ("E_f64", 8, "trace_paths<double,4,false,0,true,true>"),
]


@pytest.mark.parametrize("name,shards,kernel", PRODUCTION_SHAPES)
def test_production_shapes_vs_independent(renderer, name, shards, kernel, monkeypatch):
    """The kernels bench.py times, launched as bench.py launches them (C: the whole 1920x1080 frame; D and
    E: the 8 row shards of a 3840x2160 frame, bench.py --gpus 8), each compared bit for bit with the
    INDEPENDENT restatement's pixels that fall inside it (tests/golden/independent_baseline.npz: linear
    value and RGB8 bytes; its per-pixel ray segments are pinned by test_independent_baseline_golden).
    rt_stats.kernel_id says which trace_paths instantiation ran, so this pins the timed kernel itself,
    not the small-launch W5 build that 1x1 tiles take; kernel_wg_per_cu says it ran at its occupancy."""
    monkeypatch.delenv("RT_WAVES", raising=False)
    monkeypatch.delenv("RT_FILTER_OFF", raising=False)
    z, meta = _baseline_cases()
    m = meta[name]
    W, H = m["W"], m["H"]
    flat = rt.scenes.config_scene(m["config"]).flatten()
    cam = rt.camera_new_py(W, H, **m["camera"])
    flags = abi.RT_FLAG_F32 if m["precision"] == "f32" else 0
    pix = z[f"{name}_pix"].astype(np.int64)
    got_lin = np.full((len(pix), 3), np.nan)
    got_rgb = np.zeros((len(pix), 3), np.uint8)
    for r in range(shards):
        inside = np.nonzero((pix // W) % shards == r)[0]
        if inside.size == 0:
            continue
        tile = rt.parallel.shard_range(W, H, shards, r) if shards > 1 else None
        rgb, lin, st, rc = gpu(renderer, flat, cam, m["depth"], m["spp"], m["seed"], flags, tile=tile)
        assert rc == 0, (name, r)
        assert abi.kernel_name(st.kernel_id) == kernel, (name, r, abi.kernel_name(st.kernel_id))
        assert st.kernel_wg_per_cu == abi.kernel_info(st.kernel_id)["W"], (name, r, st.kernel_wg_per_cu)
        # compact shard index of frame pixel q: (row // shards) * W + col
        q = pix[inside]
        at = (q // W // shards) * W + q % W
        got_lin[inside] = lin[at]
        got_rgb[inside] = rgb[at]
    np.testing.assert_array_equal(got_lin, z[f"{name}_lin"], err_msg=name)
    np.testing.assert_array_equal(got_rgb, z[f"{name}_rgb"], err_msg=name)


@pytest.mark.parametrize("w,h,spp,flags,waves", [
    (1920, 1080, 512, abi.RT_FLAG_F32, 6),   # big fp32 launch: W6
    (64, 36, 512, abi.RT_FLAG_F32, 5),       # small fp32 launch: W5
    (1920, 1080, 16, 0, 4),                  # fp64: W4
    (64, 36, 16, abi.RT_FLAG_F32 | abi.RT_FLAG_MODE_SCALAR, 6),   # semantics modes: kWavesModes
    (64, 36, 16, abi.RT_FLAG_MODE_VECTORIZED3, 4),
    (64, 36, 16, abi.RT_FLAG_F32 | abi.RT_FLAG_ROOT2, 6),
])
def test_kernel_runs_at_its_occupancy(renderer, scene_100, w, h, spp, flags, waves, monkeypatch):
    """rt_stats.kernel_id / kernel_wg_per_cu: every default kernel pick is resident at the waves per SIMD
    it was built for (LDS and registers within the budget), 4-wave workgroups so W of them per CU."""
    monkeypatch.delenv("RT_WAVES", raising=False)
    _, _, st, rc = gpu(renderer, scene_100, cam_for(w, h), 8, spp, flags=flags)
    assert rc == 0
    k = abi.kernel_info(st.kernel_id)
    assert k["W"] == waves and k["T"] == ("float" if flags & abi.RT_FLAG_F32 else "double"), abi.kernel_name(st.kernel_id)
    assert st.kernel_wg_per_cu == waves
    assert k["camq"]   # pinhole camera, depth >= 1


@pytest.mark.parametrize("flags", [abi.RT_FLAG_F32, 0])
def test_every_wave_override_resident(renderer, scene_100, flags, monkeypatch):
    """RT_WAVES 4..8 (clamped to what each precision's LDS allows: fp32 6, fp64 5), on the pinhole and
    the defocus paths and the mega kernels: each launch's kernel is resident at no less than its own W."""
    flat_e = rt.scenes.config_scene("E").flatten()
    for wv in ("4", "5", "6", "7", "8"):
        monkeypatch.setenv("RT_WAVES", wv)
        for flat, cam in ((scene_100, cam_for(32, 18)), (scene_100, _cam(32, 18, defocus_angle=2.0)), (flat_e, cam_for(8, 6))):
            _, _, st, rc = gpu(renderer, flat, cam, 8, 8, flags=flags)
            assert rc == 0
            k = abi.kernel_info(st.kernel_id)
            # at least its own W (a W4 fp32 build needs few enough registers for 5)
            assert st.kernel_wg_per_cu >= k["W"] and k["W"] <= (6 if flags else 5), (wv, abi.kernel_name(st.kernel_id))


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
@pytest.mark.parametrize("spp", [1, 6, 100, 512])
def test_sky_pixels_defocus(renderer, spp, flags):
    """Every sample escapes at bounce 0 through a defocus camera (no camera batches, no candidate lists):
    each pixel takes finish_pixel's sky path (K = 1 known from the slot's bounce flag: no position map,
    no replay, no colour reads), with several pixels per wave."""
    flat = rt.FlatScene(np.zeros((0, 3)), np.zeros(0), np.zeros(0, np.uint32), [rt.Lambertian((0.5, 0.5, 0.5))])
    _, _, st, _ = gpu(renderer, flat, _cam(16, 9, defocus_angle=2.0), 50, spp, flags=flags)
    assert not abi.kernel_info(st.kernel_id)["camq"] and st.direct_sky_samples == 0
    assert_parity(renderer, flat, _cam(16, 9, defocus_angle=2.0), 50, spp, flags)


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_F32])
def test_mega_scene_whole_image(renderer, flags):
    """Config E's 10 000-sphere scene through the mega kernels on a whole 64x36 image: sky rows finished
    at claim time (finish_sky_direct saves and restores the lane's parked sample/slot word around it
    while other lanes of the wave hold live rays) mixed with hit pixels, several pixels per wave, every
    pixel against the oracle."""
    flat = rt.scenes.config_scene("E").flatten()
    lin, st = assert_parity(renderer, flat, cam_for(64, 36), 50, 16, flags)
    assert abi.kernel_info(st.kernel_id)["mega"]
    assert 0 < st.direct_sky_samples < 64 * 36 * 16   # both kinds of pixel


def test_camera_table_cache_keys(renderer, scene_100, monkeypatch):
    """The per-launch camera tables are cached per precision under (scene, camera centre bits, scalar
    mode, RT_FILTER_OFF).  One context, one scene, every key left and returned to: centre A, B, A;
    scalar then live path; fp32 and fp64 interleaved; RT_FILTER_OFF on and off.  Each render equals the
    oracle's, so no stale table is ever reused."""
    monkeypatch.delenv("RT_FILTER_OFF", raising=False)
    cam_a = cam_for(32, 18)
    cam_b = _cam(32, 18, center=(14.0, 3.0, 17.0))
    seq = [(cam_a, 0, 0), (cam_b, 0, 0), (cam_a, 0, 0),
           (cam_a, abi.RT_FLAG_F32, 0), (cam_b, abi.RT_FLAG_F32, 0), (cam_a, 0, 0),
           (cam_a, abi.RT_FLAG_MODE_SCALAR, 0), (cam_a, 0, 0), (cam_a, abi.RT_FLAG_MODE_SCALAR | abi.RT_FLAG_F32, 0),
           (cam_a, abi.RT_FLAG_F32, 0), (cam_a, abi.RT_FLAG_F32, 1), (cam_a, abi.RT_FLAG_F32, 0), (cam_b, 0, 1),
           (cam_a, 0, 0)]
    renderer.set_scene(scene_100)
    for i, (cam, flags, off) in enumerate(seq):
        if off:
            monkeypatch.setenv("RT_FILTER_OFF", "1")
        else:
            monkeypatch.delenv("RT_FILTER_OFF", raising=False)
        rgb, lin, st, rc = gpu(renderer, scene_100, cam, 50, 8, flags=flags)
        prec = "f32" if flags & abi.RT_FLAG_F32 else "f64"
        _, lin_o, segs_o, _ = oracle_render(scene_100, cam, 50, 8, SEED, flags & ~abi.RT_FLAG_F32, precision=prec)
        np.testing.assert_array_equal(lin, lin_o, err_msg=f"step {i}")
        assert st.ray_segments == segs_o, i
