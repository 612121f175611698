"""Scene loader for the reference's scene.toml schema (Python mirror; the C++ one is host/scene.hpp).

  get_materials            src/materials.rs:12-19   (type lower-cased; unknown -> panic, :31)
  load_material_from_toml  src/materials.rs:21-33
  get_object_list          src/objects.rs:38-52     (type "sphere" only)
  Sphere::from_table       src/objects.rs:292-299   (material name must exist, :296)
  Vec3::from_toml          src/geometry.rs:190-211  ({x,y,z} or [x,y,z]; non-numbers panic)
  Color::from_toml         src/color.rs:99-123      ({red,green,blue}: non-numbers read 0.0; [r,g,b])
  to_float                 src/toml_utils.rs:2-12   (float or integer)

Where the reference panics, these raise Panic with the reference's message.
"""
import tomli

from .scene import Dielectric, Lambertian, Metal, Scene, Sphere


class Panic(RuntimeError):
    """A reference panic (unwrap on None, panic!, assert!, Index on a missing key)."""


def _index(table, key):
    if key not in table:
        raise Panic(f'index not found: key "{key}" missing from table')
    return table[key]


def _unwrap(v, what):
    if v is None:
        raise Panic(f"called `Option::unwrap()` on a `None` value ({what})")
    return v


def to_float(v):
    if isinstance(v, bool):
        return None
    if isinstance(v, float):
        return v
    if isinstance(v, int):
        return float(v)
    return None


def vec3_from_toml(v):
    if isinstance(v, dict):
        return tuple(_unwrap(to_float(_index(v, k)), k) for k in ("x", "y", "z"))
    if isinstance(v, list):
        if len(v) < 3:
            raise Panic("assertion failed: array.len() >= 3")
        return tuple(_unwrap(to_float(v[i]), "xyz"[i]) for i in range(3))
    return None


def color_from_toml(v):
    if isinstance(v, dict):
        out = []
        for k in ("red", "green", "blue"):
            f = to_float(_index(v, k))
            out.append(0.0 if f is None else f)
        return tuple(out)
    if isinstance(v, list):
        if len(v) < 3:
            raise Panic("assertion failed: array.len() >= 3")
        return tuple(_unwrap(to_float(v[i]), ("red", "green", "blue")[i]) for i in range(3))
    return None


def load_material_from_toml(table):
    ty = _index(table, "type")
    if not isinstance(ty, str):
        raise Panic("called `Option::unwrap()` on a `None` value (type)")
    kind = ty.lower()
    if kind == "lambertian":
        return Lambertian(_unwrap(color_from_toml(_index(table, "albedo")), "albedo"))
    if kind == "metal":
        return Metal(_unwrap(color_from_toml(_index(table, "albedo")), "albedo"),
                     _unwrap(to_float(_index(table, "fuzzy_factor")), "fuzzy_factor"))
    if kind == "dielectric":
        hollow = _index(table, "hollow")
        if not isinstance(hollow, bool):
            raise Panic("called `Option::unwrap()` on a `None` value (hollow)")
        return Dielectric(_unwrap(to_float(_index(table, "index_of_refraction")), "index_of_refraction"), hollow)
    raise Panic(f"Unknown material type {kind}!")


def get_materials(table):
    out = {}
    for key, value in table.items():
        if not isinstance(value, dict):
            raise Panic("called `Option::unwrap()` on a `None` value (material table)")
        out[key] = load_material_from_toml(value)
    return out


def load_object_from_toml(table, materials):
    ty = _index(table, "type")
    if not isinstance(ty, str):
        raise Panic("called `Option::unwrap()` on a `None` value (type)")
    kind = ty.lower()
    if kind != "sphere":
        raise Panic(f"Unknown object type {kind}")
    center = _unwrap(vec3_from_toml(_index(table, "center")), "center")
    radius = _unwrap(to_float(_index(table, "radius")), "radius")
    name = _index(table, "material")
    if not isinstance(name, str):
        raise Panic("called `Option::unwrap()` on a `None` value (material)")
    if name not in materials:
        raise Panic(f'called `Option::unwrap()` on a `None` value (material "{name}")')
    return Sphere(center, radius, materials[name])


def get_object_list(array, materials):
    out = []
    for v in array:
        if not isinstance(v, dict):
            raise Panic("called `Option::unwrap()` on a `None` value (hitable)")
        out.append(load_object_from_toml(v, materials))
    return out


def scene_from_toml(text):
    """src/main.rs:36-43: parse, load materials, then hitables (scene order kept)."""
    data = tomli.loads(text)
    mats = _index(data, "materials")
    if not isinstance(mats, dict):
        raise Panic("called `Option::unwrap()` on a `None` value (materials)")
    hit = _index(data, "hitables")
    if not isinstance(hit, list):
        raise Panic("called `Option::unwrap()` on a `None` value (hitables)")
    return Scene.from_list(get_object_list(hit, get_materials(mats)))


def load_scene(path):
    with open(path, "rb") as f:
        return scene_from_toml(f.read().decode())
