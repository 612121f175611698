"""Host-side scene model mirroring the reference's Scene / Camera / Material surface.

Reference types (file:line):
  Lambertian / Metal / Dielectric   src/materials.rs:41-155   (Metal::new clamps fuzz, :79-88)
  Sphere, Object::Sphere            src/objects.rs:15-19, 203-300
  Scene::{new, from_list, add, len} src/ray_tracing.rs:100-104, 217-229, 308-310
  Camera::new                        src/ray_tracing.rs:27-62

`Scene.flatten()` produces the SoA arrays of the C ABI (include/rt_mi355x.h rt_scene):
spheres in scene order (closest-hit ties resolve to the later sphere, objects.rs:141),
one material-table entry per distinct material object.
"""
import ctypes
import math

import numpy as np

from . import abi


class Material:
    kind = None

    def to_abi(self):
        raise NotImplementedError


class Lambertian(Material):
    """materials.rs:41-69"""
    kind = abi.RT_LAMBERTIAN

    def __init__(self, albedo):
        self.albedo = tuple(float(x) for x in albedo)

    def to_abi(self):
        return abi.RtMaterial(abi.RT_LAMBERTIAN, 0, (ctypes.c_double * 3)(*self.albedo), 0.0, 0.0)

    def __repr__(self):
        return f"Lambertian(albedo={self.albedo})"


class Metal(Material):
    """materials.rs:71-107; the constructor clamps fuzzy_factor to <= 1 (:79-88), not below 0."""
    kind = abi.RT_METAL

    def __init__(self, albedo, fuzzy_factor):
        self.albedo = tuple(float(x) for x in albedo)
        f = float(fuzzy_factor)
        self.fuzzy_factor = f if f < 1.0 else 1.0

    def to_abi(self):
        return abi.RtMaterial(abi.RT_METAL, 0, (ctypes.c_double * 3)(*self.albedo), self.fuzzy_factor, 0.0)

    def __repr__(self):
        return f"Metal(albedo={self.albedo}, fuzzy_factor={self.fuzzy_factor})"


class Dielectric(Material):
    """materials.rs:109-155"""
    kind = abi.RT_DIELECTRIC

    def __init__(self, index_of_refraction, hollow):
        self.index_of_refraction = float(index_of_refraction)
        self.hollow = bool(hollow)

    def to_abi(self):
        return abi.RtMaterial(abi.RT_DIELECTRIC, int(self.hollow), (ctypes.c_double * 3)(0.0, 0.0, 0.0), 0.0,
                              self.index_of_refraction)

    def __repr__(self):
        return f"Dielectric(index_of_refraction={self.index_of_refraction}, hollow={self.hollow})"


class Sphere:
    """objects.rs:203-214"""

    def __init__(self, center, radius, material):
        self.center = tuple(float(x) for x in center)
        self.radius = float(radius)
        self.material = material


class FlatScene:
    """SoA image of a Scene in the C-ABI layout; keeps the ctypes buffers alive."""

    def __init__(self, center, radius, material, materials):
        self.center = np.ascontiguousarray(center, dtype=np.float64).reshape(-1, 3)
        self.radius = np.ascontiguousarray(radius, dtype=np.float64).reshape(-1)
        self.material = np.ascontiguousarray(material, dtype=np.uint32).reshape(-1)
        self.materials = list(materials)
        n = len(self.radius)
        assert self.center.shape[0] == n and self.material.shape[0] == n
        self._mats = (abi.RtMaterial * max(1, len(self.materials)))(*[m.to_abi() for m in self.materials])
        P = ctypes.POINTER
        self.abi = abi.RtScene(
            n, len(self.materials),
            self.center.ctypes.data_as(P(ctypes.c_double)) if n else None,
            self.radius.ctypes.data_as(P(ctypes.c_double)) if n else None,
            self.material.ctypes.data_as(P(ctypes.c_uint32)) if n else None,
            ctypes.cast(self._mats, P(abi.RtMaterial)),
        )

    @property
    def n_spheres(self):
        return len(self.radius)


class Scene:
    """ray_tracing.rs:100-104 / 217-229"""

    def __init__(self, objects=None):
        self.objects = list(objects or [])

    @classmethod
    def from_list(cls, objects):
        return cls(objects)

    def add(self, obj):
        self.objects.append(obj)

    def len(self):
        return len(self.objects)

    def __len__(self):
        return len(self.objects)

    def flatten(self):
        mats, index = [], {}
        mat_idx = []
        for s in self.objects:
            key = id(s.material)
            if key not in index:
                index[key] = len(mats)
                mats.append(s.material)
            mat_idx.append(index[key])
        center = np.array([s.center for s in self.objects], dtype=np.float64).reshape(-1, 3)
        radius = np.array([s.radius for s in self.objects], dtype=np.float64)
        return FlatScene(center, radius, np.array(mat_idx, dtype=np.uint32), mats)


class Camera:
    """Camera::new, ray_tracing.rs:27-62 (computed by the C library in f64)."""

    def __init__(self, image_width, image_height, focal_length, view_angle, center, look_at, up, defocus_angle,
                 lib=None):
        lib = lib or abi.load_library()
        self.abi = abi.RtCamera()
        D3 = ctypes.c_double * 3
        abi.check(lib, lib.rt_camera_new(ctypes.byref(self.abi), int(image_width), int(image_height),
                                         float(focal_length), float(view_angle), D3(*center), D3(*look_at),
                                         D3(*up), float(defocus_angle)))

    @classmethod
    def from_abi(cls, cam):
        obj = cls.__new__(cls)
        obj.abi = cam
        return obj

    def image_width(self):
        return self.abi.image_width

    def image_height(self):
        return self.abi.image_height


def camera_new_py(w, h, focal_length, view_angle, center, look_at, up, defocus_angle):
    """Pure-Python restatement of Camera::new (ray_tracing.rs:27-62), used to fill an RtCamera
    without loading the HIP library (and to cross-check rt_camera_new)."""
    rads = math.pi / 180.0
    aspect = w / h
    vh = math.tan((view_angle * rads) / 2.0) * focal_length * 2.0
    vw = vh * aspect

    def unit(a):
        ln = math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
        return [a[0] / ln, a[1] / ln, a[2] / ln]

    d = unit([look_at[i] - center[i] for i in range(3)])
    wv = [-d[0], -d[1], -d[2]]
    u = unit([up[1] * wv[2] - up[2] * wv[1], up[2] * wv[0] - up[0] * wv[2], up[0] * wv[1] - up[1] * wv[0]])
    v = [wv[1] * u[2] - wv[2] * u[1], wv[2] * u[0] - wv[0] * u[2], wv[0] * u[1] - wv[1] * u[0]]
    dr = focal_length * math.tan((defocus_angle / 2.0) * rads)
    cam = abi.RtCamera()
    cam.image_width, cam.image_height = int(w), int(h)
    for i in range(3):
        cam.center[i] = center[i]
        cam.vu[i] = u[i] * vw
        cam.vv[i] = (-v[i]) * vh
        cam.ulc[i] = ((center[i] - wv[i] * focal_length) - cam.vu[i] / 2.0) - cam.vv[i] / 2.0
        cam.du[i] = u[i] * dr
        cam.dv[i] = v[i] * dr
    return cam


# The camera hard-coded in src/main.rs:51-58.
MAIN_CAMERA = dict(focal_length=10.0, view_angle=30.0, center=(16.0, 2.0, 18.5), look_at=(0.0, 0.0, 0.0),
                   up=(0.0, 1.0, 0.0), defocus_angle=0.0)
