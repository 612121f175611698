"""ctypes mirror of include/rt_mi355x.h (the drop-in C ABI).

The structures below are shared by the product library (lib/librt_mi355x.so) and by the
test-only oracle (oracle/build/liboracle.so), whose structs have the same layout.
"""
import ctypes
import hashlib
import os

u32 = ctypes.c_uint32
u64 = ctypes.c_uint64
f64 = ctypes.c_double

RT_OK = 0
RT_ERR_INVALID = 1
RT_ERR_HIP = 2
RT_ERR_RANGE = 3
RT_ERR_UNSUPPORTED = 4
RT_MAX_BOUNCES_F32 = 3839   # include/rt_mi355x.h: fp32 renders refuse more (RNG counter width)

RT_LAMBERTIAN = 0
RT_METAL = 1
RT_DIELECTRIC = 2

RT_FLAG_F32 = 0x1
RT_FLAG_ROOT2 = 0x2
RT_FLAG_MODE_VECTORIZED = 0x4   # render_vectorized -> trace_vectorized semantics
RT_FLAG_MODE_SCALAR = 0x8       # render -> trace_rays semantics
RT_FLAG_MODE_VECTORIZED3 = 0x10  # render_vectorized3 -> trace_vectorized3 semantics
RT_FLAG_ALL = 0x1F


class RtMaterial(ctypes.Structure):
    _fields_ = [("kind", u32), ("hollow", u32), ("albedo", f64 * 3), ("fuzz", f64), ("ior", f64)]


class RtScene(ctypes.Structure):
    _fields_ = [
        ("n_spheres", u32),
        ("n_materials", u32),
        ("center", ctypes.POINTER(f64)),
        ("radius", ctypes.POINTER(f64)),
        ("material", ctypes.POINTER(u32)),
        ("materials", ctypes.POINTER(RtMaterial)),
    ]


class RtCamera(ctypes.Structure):
    _fields_ = [("image_width", u32), ("image_height", u32)] + [
        (n, f64 * 3) for n in ("center", "ulc", "vu", "vv", "du", "dv")
    ]


class RtTileRange(ctypes.Structure):
    _fields_ = [("row_begin", u32), ("row_step", u32), ("row_count", u32), ("col_begin", u32), ("col_count", u32)]


class RtStats(ctypes.Structure):
    _fields_ = [
        ("seconds", f64),
        ("kernel_ms", f64),
        ("pixels_per_second", f64),
        ("pixels", u64),
        ("samples", u64),
        ("ray_segments", u64),
        ("lane_slots", u64),
        ("bounce_iters", u64),
        ("box_groups", u64),
        ("filter_groups", u64),
        ("exact_tests", u64),
        ("cone_tests", u64),
        ("camera_exact_tests", u64),
        ("direct_sky_samples", u64),
        ("kernel_id", u32),
        ("kernel_wg_per_cu", u32),
    ]


def kernel_info(kernel_id):
    """rt_stats.kernel_id decoded (include/rt_mi355x.h RT_KERNEL_*): the trace_paths instantiation that ran."""
    if kernel_id == 0:
        return None
    return {"T": "double" if kernel_id & 1 else "float", "W": (kernel_id >> 1) & 7, "root2": bool((kernel_id >> 4) & 1),
            "mode": (kernel_id >> 5) & 3, "camq": bool((kernel_id >> 7) & 1), "mega": bool((kernel_id >> 8) & 1)}


def kernel_name(kernel_id):
    """trace_paths<T,W,ROOT2,MODE,CAMQ,MEGA> as rocprofv3 lists it, e.g. trace_paths<float,6,false,0,true,false>."""
    k = kernel_info(kernel_id)
    if k is None:
        return None
    b = lambda v: "true" if v else "false"
    return f"trace_paths<{k['T']},{k['W']},{b(k['root2'])},{k['mode']},{b(k['camq'])},{b(k['mega'])}>"


def lane_utilisation(st):
    """Enabled rays / SIMD lanes issued; pixels finished at claim time hold no lane (rt_stats)."""
    return (st.ray_segments - st.direct_sky_samples) / max(1, st.lane_slots)


# Executed FLOP per lane of one wave-level test (include/rt_mi355x.h); x 64 lanes.
WORK_FLOP_F32 = {"box_groups": 72, "filter_groups": 56, "cone_tests": 23}
WORK_FLOP_T = {"exact_tests": 17, "camera_exact_tests": 8}   # in the render's precision


def executed_flop(st, precision):
    """(fp32 FLOP, fp64 FLOP) the culls and exact tests executed (64 lanes per wave-level test)."""
    f32 = sum(64 * f * getattr(st, k) for k, f in WORK_FLOP_F32.items())
    ft = sum(64 * f * getattr(st, k) for k, f in WORK_FLOP_T.items())
    return (f32 + ft, 0) if precision == "f32" else (f32, ft)


PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RT_MI355X_LIB") or os.path.join(PKG_DIR, "lib", "librt_mi355x.so")

# Every symbol include/rt_mi355x.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "rt_camera_new", "rt_metal_clamp_fuzz", "rt_render", "rt_context_create", "rt_context_destroy",
    "rt_context_set_scene", "rt_render_async", "rt_context_collect", "rt_device_alloc", "rt_device_free",
    "rt_memcpy_d2h", "rt_last_error", "rt_version",
]

_lib = None

# The sources the Makefile hashes into rt_version() ("src=<hash>"), in its order (SRC, then HDR).
KERNEL_SOURCES = ["rt_kernel.hip", "rt_experiments.hpp", "rt_common.hpp", "rt_sweep.hpp", "rt_camera.hpp",
                  "rt_finish.hpp", "rt_trace.hpp", "rt_layout.hpp", "rt_device.hpp"]
SOURCE_FILES = [os.path.join(PKG_DIR, "csrc", f) for f in KERNEL_SOURCES] + \
               [os.path.join(os.path.dirname(PKG_DIR), "include", "rt_mi355x.h")]


def kernel_source_text():
    """The text of every csrc/ file (the one translation unit the library is built from), concatenated:
    tests that pin a constant or a margin formula of the kernel search this."""
    return "\n".join(open(f).read() for f in SOURCE_FILES[:-1])


def source_hash():
    """sha256 (first 12 hex digits) of the kernel sources, as the Makefile computes it."""
    h = hashlib.sha256()
    for f in SOURCE_FILES:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def version_info(lib):
    """rt_version() parsed: {"version": str, "kind": "product" | "experiment" | None, "src_hash": str | None}."""
    v = lib.rt_version().decode()
    kind = "experiment" if " experiment" in v else ("product" if " product" in v else None)
    src = v.split("src=", 1)[1].split()[0] if "src=" in v else None
    return {"version": v, "kind": kind, "src_hash": src}


def load_library(path=None):
    """Load the product library.  Raises (never falls back) when it has not been built, and refuses an
    experiment build (make exp / kstats) unless RT_ALLOW_EXPERIMENT=1 (same-box A/B scripts only)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"rt_mi355x: HIP library not built: {p} (run `make -C rust-ray-tracing_amd`)")
    lib = ctypes.CDLL(p)
    lib.rt_version.restype = ctypes.c_char_p
    if version_info(lib)["kind"] == "experiment" and os.environ.get("RT_ALLOW_EXPERIMENT") != "1":
        raise RuntimeError(f"rt_mi355x: {p} is an experiment build ({lib.rt_version().decode()}); "
                           "set RT_ALLOW_EXPERIMENT=1 for A/B runs")
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    lib.rt_camera_new.argtypes = [P(RtCamera), u32, u32, f64, f64, P(f64), P(f64), P(f64), f64]
    lib.rt_metal_clamp_fuzz.argtypes = [f64]
    lib.rt_metal_clamp_fuzz.restype = f64
    lib.rt_render.argtypes = [P(RtScene), P(RtCamera), u32, u32, u64, u32, P(RtTileRange), vp, vp, P(RtStats)]
    lib.rt_context_create.argtypes = [ctypes.c_int, P(vp)]
    lib.rt_context_destroy.argtypes = [vp]
    lib.rt_context_set_scene.argtypes = [vp, P(RtScene)]
    lib.rt_render_async.argtypes = [vp, P(RtCamera), u32, u32, u64, u32, P(RtTileRange), vp, vp, vp]
    lib.rt_context_collect.argtypes = [vp, vp, P(RtStats)]
    lib.rt_device_alloc.argtypes = [vp, ctypes.c_size_t, P(vp)]
    lib.rt_device_free.argtypes = [vp, vp]
    lib.rt_memcpy_d2h.argtypes = [vp, vp, vp, ctypes.c_size_t]
    lib.rt_last_error.restype = ctypes.c_char_p
    lib.rt_version.restype = ctypes.c_char_p
    if path is None:
        _lib = lib
    return lib


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"rt_mi355x error {code}: {msg}")
        self.code = code


def check(lib, rc, allow=()):
    if rc != RT_OK and rc not in allow:
        raise RtError(rc, lib.rt_last_error().decode())
    return rc
