"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the CPU-side code (SURVEY.md §5 "sanitizers"):
the oracle (oracle/oracle.c, test infrastructure) and the host scene.toml loader (host/toml.hpp,
host/scene.hpp: the C++ side of main.rs:31-39, materials.rs:12-33, objects.rs:38-52).

Each harness (tests/sanitize/) is built with gcc/g++ `-fsanitize=address,undefined
-fno-sanitize-recover=all`, so any report aborts the process with a non-zero status.
* The oracle harness renders a set of small cases (every semantics mode, both precisions, the AVX2 packet
  baseline, partial chunks, depth 0, empty and range-error scenes, listed pixels, 1 and 3 threads); its
  results must be bit-identical to the ordinary -O3 build's (tests/oracle_bind.py).
* The loader harness parses the schema variants, every reference panic case, the BASELINE scenes and ~600
  malformed inputs (truncations, byte mutations, unterminated strings and arrays, deep nesting, huge and
  odd numbers, binary noise); valid files must dump exactly what the Python mirror loads.
No GPU: the loader harness links librt_mi355x.so only for rt_metal_clamp_fuzz / rt_camera_new's host code.
"""
import json
import os
import random
import subprocess

import numpy as np
import pytest

import rt_mi355x as rt
from oracle_bind import oracle_render, packed_render

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=66",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def oracle_san(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("san") / "oracle_san")
    subprocess.run(["gcc", "-std=c11", "-march=x86-64-v3", "-ffp-contract=off", "-fno-math-errno", *SAN, "-o", out,
                    os.path.join(REPO, "tests", "sanitize", "oracle_san.c"), os.path.join(REPO, "oracle", "oracle.c"),
                    "-lm", "-lpthread"], check=True)
    return out


@pytest.fixture(scope="module")
def toml_san(tmp_path_factory):
    lib = os.path.join(REPO, "rust-ray-tracing_amd", "lib")
    if not os.path.exists(os.path.join(lib, "librt_mi355x.so")):
        subprocess.run(["make", "-C", os.path.join(REPO, "rust-ray-tracing_amd")], check=True, capture_output=True)
    out = str(tmp_path_factory.mktemp("san") / "toml_san")
    subprocess.run(["g++", "-std=c++17", *SAN, "-o", out, os.path.join(REPO, "tests", "sanitize", "toml_san.cpp"),
                    "-I" + os.path.join(REPO, "include"), "-L" + lib, "-lrt_mi355x", "-Wl,-rpath," + lib], check=True)
    return out


def _g(v):
    return repr(float(v))


def _case_text(prec, flags, depth, spp, seed, flat, cam, threads, pixels=None):
    px = [] if pixels is None else [int(p) for p in pixels]
    t = [str(x) for x in (prec, flags, depth, spp, seed, cam.image_width, cam.image_height, threads, len(px))]
    for k in ("center", "ulc", "vu", "vv", "du", "dv"):
        t += [_g(v) for v in getattr(cam, k)]
    t += [str(flat.n_spheres), str(len(flat.materials))]
    for c, r, m in zip(flat.center, flat.radius, flat.material):
        t += [_g(c[0]), _g(c[1]), _g(c[2]), _g(r), str(int(m))]
    for m in flat.materials:
        a = m.to_abi()
        t += [str(a.kind), str(a.hollow), _g(a.albedo[0]), _g(a.albedo[1]), _g(a.albedo[2]), _g(a.fuzz), _g(a.ior)]
    return " ".join(t + [str(p) for p in px])


def _cases():
    a = rt.scenes.config_scene("A").flatten()
    s100 = rt.scenes.random_spheres(100).flatten()
    empty = rt.FlatScene(np.zeros((0, 3)), np.zeros(0), np.zeros(0, np.uint32), [rt.Lambertian((0.5, 0.5, 0.5))])
    hot = rt.FlatScene(np.array([[0.0, 0.0, 0.0]]), np.array([5.0]), np.array([0], np.uint32),
                       [rt.Lambertian((9.0, 9.0, 9.0))])
    quirks = rt.FlatScene(np.array([[0.0, 1.0, 0.0], [0.0, 1.0, 0.0], [2.0, 1.0, 0.0], [16.0, 2.0, 18.5]]),
                          np.array([1.0, 1.0, -0.9, 0.5]), np.array([0, 1, 2, 0], np.uint32),
                          [rt.Lambertian((0.5, 0.4, 0.3)), rt.Metal((0.8, 0.8, 0.8), 1.0), rt.Dielectric(1.5, True)])
    cam = lambda w, h, **kw: rt.camera_new_py(w, h, **dict(rt.MAIN_CAMERA, **kw))   # noqa: E731
    cases = [
        (0, 0, 8, 16, 0x5EED0001, a, cam(40, 23), 3, None),
        (1, 0, 8, 16, 0x5EED0001, a, cam(40, 23), 1, None),
        (0, 0, 50, 6, 0x5EED0001, s100, cam(16, 9), 3, None),          # partial chunk, (C-1)%2 == 1
        (1, 0, 50, 100, 0x100000001, s100, cam(4, 3), 2, None),       # (C-1)%2 == 0, fp32 key fold
        (0, 0, 0, 8, 7, s100, cam(8, 5), 1, None),                    # depth 0
        (0, 0x2, 50, 8, 7, s100, cam(8, 5), 1, None),                 # ROOT2
        (0, 0x4, 50, 7, 7, s100, cam(8, 5), 1, None),                 # vectorized
        (1, 0x8, 50, 9, 7, s100, cam(8, 5), 1, None),                 # scalar, fp32
        (0, 0x10, 50, 10, 7, s100, cam(8, 5), 1, None),               # vectorized3
        (0, 0, 8, 8, 3, empty, cam(8, 5), 1, None),
        (0, 0, 4, 8, 3, hot, cam(8, 5), 1, None),                     # range error (rc 3)
        (1, 0, 300, 12, 3, quirks, cam(8, 5), 2, [0, 7, 39, 20]),     # depth > 254, ties, camera inside
        (0, 0, 50, 8, 3, s100, cam(8, 5, defocus_angle=0.6), 1, None),
        (2, 0, 8, 16, 0x5EED0001, a, cam(24, 17), 3, None),           # the AVX2 packet baseline, ragged tiles
    ]
    return cases


def test_oracle_under_asan_ubsan(oracle_san):
    cases = _cases()
    text = f"{len(cases)} " + " ".join(_case_text(*c) for c in cases)
    r = subprocess.run([oracle_san], input=text, capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.split("\n")
    at = 0
    for prec, flags, depth, spp, seed, flat, cam, threads, pixels in cases:
        rc, segs = (int(x) for x in lines[at].split())
        at += 1
        n = (len(pixels) if pixels is not None else cam.image_width * cam.image_height) * 3
        lin = np.array([float.fromhex(v) for v in lines[at:at + n]]).reshape(-1, 3)
        at += n
        if prec == 2:
            _, lin_o, segs_o, _, rc_o = packed_render(flat, cam, depth, spp, seed, tile=8)
        else:
            _, lin_o, segs_o, rc_o = oracle_render(flat, cam, depth, spp, seed, flags,
                                                   pixels=None if pixels is None else np.array(pixels, np.uint32),
                                                   precision="f32" if prec == 1 else "f64")
        assert (rc, segs) == (rc_o, segs_o), (prec, flags, depth, spp)
        np.testing.assert_array_equal(lin, lin_o.reshape(-1, 3))


VALID = {
    "A": rt.scenes.scene_to_toml(rt.scenes.config_scene("A")),
    "B": rt.scenes.scene_to_toml(rt.scenes.config_scene("B")),
}


def _malformed(seed=0x5EED, n=600):
    rng = random.Random(seed)
    base = VALID["A"]
    out = ["", "\x00\x01\x02", "[", "[[", "[[hitables]", "a = ", 'a = "unterminated', "a = [1, 2", "a = {x = 1",
           "a = [" * 2000, "a = {b = " * 500, "a = 1e999999", "a = -0x", "a = 0b102", "a = 1__0", 'a = "\\u00"',
           'a = "\\uD800"', 'a = """x', "a = '''x", "[a]\n[a]\n", "a = 1\na = 2\n", "[[a]]\n[a]\n", "a.b = 1\na = 2",
           "﻿[materials.m]\n", "x = 99999999999999999999999999", "x = 1979-05-27T07:32:00Z", "x = inf\ny = nan",
           "[materials.m]\ntype = 1\n", '[materials.m]\ntype = "metal"\nalbedo = []\n',
           '[materials.m]\ntype = "metal"\nalbedo = [1, 2, 3]\nfuzzy_factor = "x"\n[[hitables]]\ntype = "sphere"\n'
           'center = [0, 0, 0]\nradius = 1\nmaterial = "m"\n']
    for _ in range(n // 3):   # truncations
        out.append(base[:rng.randrange(len(base))])
    for _ in range(n // 3):   # byte mutations
        b = bytearray(base.encode())
        for _ in range(rng.randint(1, 8)):
            b[rng.randrange(len(b))] = rng.choice(b'[]{}"=,.#\n\\ 0123456789aex-+_\'\x00\xff')
        out.append(b.decode("latin-1"))
    for _ in range(n // 3):   # random token soup
        out.append("".join(rng.choice(['[', ']', '{', '}', '"', "'", '=', ',', '.', '\n', 'a', '1', '-', 'e', ' ',
                                       '#', '\\', 'true', '[[hitables]]', '[materials.x]', 'type', '1.5e3'])
                           for _ in range(rng.randint(1, 80))))
    return out


def test_toml_loader_under_asan_ubsan(toml_san, tmp_path):
    from test_host import SCHEMA_VARIANTS, flat_dict, cpp_dict
    files, want = [], []
    for name, text in [("schema", SCHEMA_VARIANTS)] + list(VALID.items()):
        p = tmp_path / f"valid_{name}.toml"
        p.write_text(text)
        files.append(str(p))
        want.append(flat_dict(rt.scene_from_toml(text).flatten()))
    bad = _malformed()
    for i, text in enumerate(bad):
        p = tmp_path / f"bad_{i}.toml"
        p.write_bytes(text.encode("utf-8", "surrogatepass") if isinstance(text, str) else text)
        files.append(str(p))
    r = subprocess.run([toml_san, *files], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(files)
    for line, w in zip(lines, want):
        assert cpp_dict(json.loads(line)) == w
    outcomes = [next(iter(json.loads(ln))) for ln in lines[len(want):]]
    # every malformed input ends in a clean parse error or a reference panic (or, for a mutation that
    # stays valid TOML and a valid scene, a scene)
    assert set(outcomes) <= {"parse_error", "panic", "n_spheres"}
    assert outcomes.count("parse_error") > 100 and outcomes.count("panic") > 10
