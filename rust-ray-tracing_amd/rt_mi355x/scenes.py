"""Synthetic scenes for the BASELINE.json configs (the reference ships no scene.toml:
`*.toml` is git-ignored at /root/reference/.gitignore:7).

  A  3 spheres, r=1: lambertian (-4,1,0), dielectric ior 1.5 (0,1,0), metal fuzz 0 (4,1,0)
  B  ground + 3 big + 96 small   ("100 random spheres")
  C  ground + 3 big + 496 small  (500 spheres; also D)
  E  ground + 3 big + 9 996 small over a proportionally larger grid (10 000 spheres)

The small spheres follow the "Ray Tracing in One Weekend" final scene: r=0.2 on a jittered
grid, 80 % lambertian (albedo = U*U), 15 % metal (albedo U[0.5,1), fuzz U[0,0.5)), 5 %
dielectric ior 1.5.  Deterministic: numpy PCG64 with a fixed seed per config.
"""
import math

import numpy as np

from .scene import Dielectric, Lambertian, Metal, Scene, Sphere

CONFIGS = {
    # name: (width, height, n_spheres, spp, max_bounces)
    "A": (400, 225, 3, 16, 8),
    "B": (1280, 720, 100, 128, 50),
    "C": (1920, 1080, 500, 512, 50),
    "D": (3840, 2160, 500, 1024, 50),
    "E": (3840, 2160, 10000, 2048, 50),
}

SCENE_SEED = 0x5EED0001


def three_spheres():
    """Config A's 3-sphere scene."""
    return Scene.from_list([
        Sphere((-4.0, 1.0, 0.0), 1.0, Lambertian((0.4, 0.2, 0.1))),
        Sphere((0.0, 1.0, 0.0), 1.0, Dielectric(1.5, False)),
        Sphere((4.0, 1.0, 0.0), 1.0, Metal((0.7, 0.6, 0.5), 0.0)),
    ])


def random_spheres(n_spheres, seed=SCENE_SEED):
    """Ground + 3 big spheres + (n_spheres - 4) small random spheres."""
    assert n_spheres >= 4
    rng = np.random.default_rng(seed)
    objs = [
        Sphere((0.0, -1000.0, 0.0), 1000.0, Lambertian((0.5, 0.5, 0.5))),
        Sphere((0.0, 1.0, 0.0), 1.0, Dielectric(1.5, False)),
        Sphere((-4.0, 1.0, 0.0), 1.0, Lambertian((0.4, 0.2, 0.1))),
        Sphere((4.0, 1.0, 0.0), 1.0, Metal((0.7, 0.6, 0.5), 0.0)),
    ]
    n_small = n_spheres - 4
    g = int(math.ceil(math.sqrt(n_small)))
    big = [(0.0, 1.0, 0.0), (-4.0, 1.0, 0.0), (4.0, 1.0, 0.0)]
    glass = Dielectric(1.5, False)
    for idx in range(n_small):
        a = idx % g - g // 2
        b = idx // g - g // 2
        for _ in range(16):  # keep small spheres out of the big ones (RTIOW's 0.9 clearance)
            cx = a + 0.9 * rng.random()
            cz = b + 0.9 * rng.random()
            if all(math.dist((cx, 0.2, cz), (bx, 0.2, bz)) > 1.2 for bx, _, bz in big):
                break
        choose = rng.random()
        if choose < 0.8:
            mat = Lambertian(tuple(rng.random(3) * rng.random(3)))
        elif choose < 0.95:
            mat = Metal(tuple(0.5 + 0.5 * rng.random(3)), 0.5 * rng.random())
        else:
            mat = glass
        objs.append(Sphere((cx, 0.2, cz), 0.2, mat))
    return Scene.from_list(objs)


def config_scene(name):
    n = CONFIGS[name][2]
    return three_spheres() if name == "A" else random_spheres(n)


def scene_to_toml(scene):
    """Serialise in the reference's scene.toml schema (materials.rs:12-33, objects.rs:38-52)."""
    lines, names = [], {}
    for s in scene.objects:
        if id(s.material) in names:
            continue
        name = f"m{len(names)}"
        names[id(s.material)] = name
        m = s.material
        lines.append(f"[materials.{name}]")
        if isinstance(m, Lambertian):
            lines.append('type = "lambertian"')
            lines.append("albedo = {red = %r, green = %r, blue = %r}" % m.albedo)
        elif isinstance(m, Metal):
            lines.append('type = "metal"')
            lines.append("albedo = {red = %r, green = %r, blue = %r}" % m.albedo)
            lines.append("fuzzy_factor = %r" % m.fuzzy_factor)
        else:
            lines.append('type = "dielectric"')
            lines.append("index_of_refraction = %r" % m.index_of_refraction)
            lines.append("hollow = %s" % ("true" if m.hollow else "false"))
        lines.append("")
    for s in scene.objects:
        lines.append("[[hitables]]")
        lines.append('type = "sphere"')
        lines.append("center = {x = %r, y = %r, z = %r}" % s.center)
        lines.append("radius = %r" % s.radius)
        lines.append('material = "%s"' % names[id(s.material)])
        lines.append("")
    return "\n".join(lines)
