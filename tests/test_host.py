"""Host side above the C ABI: scene model, the scene.toml loader (Python mirror and the C++ CLI's),
the synthetic scene generator.  CPU only (the C++ loader runs via `rt-render --dump-scene`)."""
import json
import os
import subprocess

import numpy as np
import pytest

import rt_mi355x as rt
from rt_mi355x import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "rust-ray-tracing_amd", "bin", "rt-render")


def _cli_built():
    if not os.path.exists(CLI):
        subprocess.run(["make", "-C", os.path.join(REPO, "rust-ray-tracing_amd")], check=True, capture_output=True)
    return CLI


def cpp_dump(tmp_path, text):
    p = tmp_path / "scene.toml"
    p.write_text(text)
    r = subprocess.run([_cli_built(), "--scene", str(p), "--dump-scene"], capture_output=True, text=True)
    return r


def flat_dict(flat):
    return {
        "center": list(flat.center.reshape(-1)), "radius": list(flat.radius), "material": list(flat.material),
        "materials": [(a.kind, a.hollow, list(a.albedo), a.fuzz, a.ior) for a in (m.to_abi() for m in flat.materials)],
    }


def cpp_dict(d):
    return {
        "center": d["center"], "radius": d["radius"], "material": d["material"],
        "materials": [(m["kind"], m["hollow"], m["albedo"], m["fuzz"], m["ior"]) for m in d["materials"]],
    }


@pytest.mark.parametrize("config", ["A", "B", "C"])
def test_toml_round_trip_python_and_cpp(tmp_path, config):
    scene = rt.scenes.config_scene(config)
    text = rt.scenes.scene_to_toml(scene)
    want = flat_dict(scene.flatten())
    assert flat_dict(rt.scene_from_toml(text).flatten()) == want
    r = cpp_dump(tmp_path, text)
    assert r.returncode == 0, r.stderr
    assert cpp_dict(json.loads(r.stdout)) == want


SCHEMA_VARIANTS = """
[materials.ground]
type = "Lambertian"            # case-insensitive (materials.rs:22)
albedo = [0.5, 0.5, 0.5]       # array form
[materials.glass]
type = "DIELECTRIC"
index_of_refraction = 1.5
hollow = true
[materials.shiny]
type = "metal"
albedo = {red = 0.7, green = "not a number", blue = 1}   # non-number -> 0.0, int -> float
fuzzy_factor = 7               # clamped to 1 by Metal::new
[materials.unused]
type = "lambertian"
albedo = {red = 1, green = 1, blue = 1}

[[hitables]]
type = "Sphere"
center = {x = 0, y = -1000, z = 0}
radius = 1000                  # integer radius (to_float)
material = "ground"
[[hitables]]
type = "sphere"
center = [0.0, 1.0, 0.0]
radius = 1.0
material = "glass"
[[hitables]]
type = "sphere"
center = [4, 1, 0]
radius = 1e0
material = "shiny"
"""


def test_schema_variants(tmp_path):
    s = rt.scene_from_toml(SCHEMA_VARIANTS)
    f = s.flatten()
    assert f.n_spheres == 3 and len(f.materials) == 3
    assert list(f.radius) == [1000.0, 1.0, 1.0]
    m = f.materials
    assert isinstance(m[0], rt.Lambertian) and m[0].albedo == (0.5, 0.5, 0.5)
    assert isinstance(m[1], rt.Dielectric) and m[1].hollow and m[1].index_of_refraction == 1.5
    assert isinstance(m[2], rt.Metal) and m[2].albedo == (0.7, 0.0, 1.0) and m[2].fuzzy_factor == 1.0
    r = cpp_dump(tmp_path, SCHEMA_VARIANTS)
    assert r.returncode == 0, r.stderr
    assert cpp_dict(json.loads(r.stdout)) == flat_dict(f)


BASE = """
[materials.m]
type = "lambertian"
albedo = [0.5, 0.5, 0.5]
"""


@pytest.mark.parametrize("text,msg", [
    ('[materials.m]\ntype = "plastic"\nalbedo = [1,1,1]\n[[hitables]]\ntype="sphere"\ncenter=[0,0,0]\nradius=1\nmaterial="m"\n',
     "Unknown material type plastic!"),
    (BASE + '[[hitables]]\ntype = "cube"\ncenter=[0,0,0]\nradius=1\nmaterial="m"\n', "Unknown object type cube"),
    (BASE + '[[hitables]]\ntype = "sphere"\ncenter=[0,0,0]\nradius=1\nmaterial="nope"\n', 'material "nope"'),
    (BASE + '[[hitables]]\ntype = "sphere"\ncenter=[0,0]\nradius=1\nmaterial="m"\n', "array.len() >= 3"),
    (BASE + '[[hitables]]\ntype = "sphere"\ncenter=[0,0,0]\nmaterial="m"\n', 'key "radius" missing'),
    (BASE + '[[hitables]]\ntype = "sphere"\ncenter={x=0,y="a",z=0}\nradius=1\nmaterial="m"\n', "None` value (y)"),
    ('[materials.g]\ntype="dielectric"\nindex_of_refraction=1.5\nhollow=1\n[[hitables]]\ntype="sphere"\n'
     'center=[0,0,0]\nradius=1\nmaterial="g"\n', "None` value (hollow)"),
    (BASE, 'key "hitables" missing'),
])
def test_loader_panics_like_the_reference(tmp_path, text, msg):
    with pytest.raises(rt.Panic) as e:
        rt.scene_from_toml(text)
    assert msg in str(e.value)
    r = cpp_dump(tmp_path, text)
    assert r.returncode == 101 and msg in r.stderr, (r.returncode, r.stderr)


def test_cli_bad_toml_and_missing_file(tmp_path):
    r = cpp_dump(tmp_path, "[materials\nfoo = ")
    assert r.returncode == 101 and "Failed parsing scene" in r.stderr
    r = subprocess.run([_cli_built(), "--scene", str(tmp_path / "nope.toml")], capture_output=True, text=True)
    assert r.returncode == 101 and "Can't read scene from file" in r.stderr


def test_scene_flatten_dedups_materials_in_scene_order():
    a, b = rt.Lambertian((1, 0, 0)), rt.Metal((0, 1, 0), 0.1)
    s = rt.Scene.from_list([rt.Sphere((0, 0, 0), 1, b), rt.Sphere((1, 0, 0), 1, a), rt.Sphere((2, 0, 0), 1, b)])
    f = s.flatten()
    assert list(f.material) == [0, 1, 0] and f.materials == [b, a]
    s.add(rt.Sphere((3, 0, 0), 2, a))
    assert s.len() == 4 and list(s.flatten().material) == [0, 1, 0, 1]


def test_generator_is_deterministic():
    f1 = rt.scenes.random_spheres(500).flatten()
    f2 = rt.scenes.random_spheres(500).flatten()
    np.testing.assert_array_equal(f1.center, f2.center)
    assert flat_dict(f1) == flat_dict(f2)
    kinds = [m.kind for m in f1.materials]
    assert kinds.count(abi.RT_LAMBERTIAN) > kinds.count(abi.RT_METAL) > 0
    assert f1.n_spheres == 500 and f1.radius[0] == 1000.0
    assert rt.scenes.random_spheres(10000).flatten().n_spheres == 10000


def test_configs_match_baseline():
    assert rt.scenes.CONFIGS["C"] == (1920, 1080, 500, 512, 50)
    assert rt.scenes.CONFIGS["A"] == (400, 225, 3, 16, 8)
    assert rt.scenes.CONFIGS["E"][2] == 10000 and rt.scenes.CONFIGS["E"][3] == 2048
