"""ctypes binding of the test-only oracle (oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

NATIVE_PATH = os.path.join(ORACLE_DIR, "build", "native", "liboracle.so")

_libs = {}


def build_native():
    """Build the -march=native oracle on this host (bench.py's CPU baseline); returns its path or None."""
    r = subprocess.run(["make", "-C", ORACLE_DIR, "native"], capture_output=True, text=True)
    return NATIVE_PATH if r.returncode == 0 and os.path.exists(NATIVE_PATH) else None


def load_oracle(path=None):
    path = path or ORACLE_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = ctypes.CDLL(path)
    vp, u32, u64, f64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
    for name in ("oracle_render_f64", "oracle_render_f32"):
        fn = getattr(lib, name)
        fn.argtypes = [vp, vp, u32, u32, u64, u32, vp, u32, vp, vp, ctypes.POINTER(u64), ctypes.c_int]
        fn.restype = ctypes.c_int
    lib.oracle_camera_new.argtypes = [vp, u32, u32, f64, f64, ctypes.POINTER(f64), ctypes.POINTER(f64),
                                      ctypes.POINTER(f64), f64]
    lib.oracle_philox4x32_10.argtypes = [ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32)]
    lib.oracle_philox2x32_10.argtypes = [ctypes.POINTER(u32), u32, ctypes.POINTER(u32)]
    lib.oracle_sincos2pi_f64.argtypes = [f64, ctypes.POINTER(f64), ctypes.POINTER(f64)]
    lib.oracle_to_u8.argtypes = [ctypes.POINTER(f64), ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int)]
    lib.oracle_get_ray_f64.argtypes = [vp, u32, u32, u32, u64, ctypes.POINTER(f64), ctypes.POINTER(f64)]
    _libs[path] = lib
    return lib


def oracle_render(flat, cam, max_bounces, spp, seed, flags=0, pixels=None, precision="f64", threads=None,
                  lib_path=None):
    """Run the CPU restatement.  flat: rt_mi355x.FlatScene; cam: abi.RtCamera.
    Returns (rgb [n,3] u8, linear [n,3] f64, segments, rc)."""
    lib = load_oracle(lib_path)
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    if pixels is None:
        n = cam.image_width * cam.image_height
        pix_ptr = None
    else:
        pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
        n = len(pixels)
        pix_ptr = pixels.ctypes.data
    rgb = np.zeros((n, 3), dtype=np.uint8)
    lin = np.zeros((n, 3), dtype=np.float64)
    segs = ctypes.c_uint64(0)
    fn = lib.oracle_render_f64 if precision == "f64" else lib.oracle_render_f32
    rc = fn(ctypes.addressof(flat.abi), ctypes.addressof(cam), max_bounces, spp, seed, flags, pix_ptr, n,
            rgb.ctypes.data, lin.ctypes.data, ctypes.byref(segs), threads)
    return rgb, lin, segs.value, rc


def packed_render(flat, cam, max_bounces, spp, seed, tiles=None, tile=128, threads=None, lib_path=None):
    """The reference-shaped CPU baseline (oracle/packed_avx2.h, f64): 4-lane AVX2 packets, tile x tile
    blocks through a shared queue.  tiles: block indices (row-major block grid) or None = all.
    Returns (rgb [W*H,3] u8, linear [W*H,3] f64 -- only the rendered blocks written, segments, pixels, rc)."""
    lib = load_oracle(lib_path)
    fn = lib.packed_render_f64
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    fn.argtypes = [vp, vp, u32, u32, u64, u32, vp, u32, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.c_int]
    fn.restype = ctypes.c_int
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    n = cam.image_width * cam.image_height
    rgb = np.zeros((n, 3), dtype=np.uint8)
    lin = np.zeros((n, 3), dtype=np.float64)
    tptr, nt = None, 0
    if tiles is not None:
        tiles = np.ascontiguousarray(tiles, dtype=np.uint32)
        tptr, nt = tiles.ctypes.data, len(tiles)
    segs, pix = u64(0), u64(0)
    rc = fn(ctypes.addressof(flat.abi), ctypes.addressof(cam), max_bounces, spp, seed, tile, tptr, nt,
            rgb.ctypes.data, lin.ctypes.data, ctypes.byref(segs), ctypes.byref(pix), threads)
    return rgb, lin, segs.value, pix.value, rc
