"""Renderer trait mirror (src/renderer.rs:11-40) backed by the MI355X C ABI.

    trait Renderer { fn render(&self, max_bounces, samples_per_pixel, &Arc<Scene>, &Arc<Camera>)
                     -> (RgbImage, RenderStat) }                       renderer.rs:38-40
    TileRenderer::new(num_threads: Option<NonZeroUsize>, block_size)   renderer.rs:232-241

`GpuRenderer.render` has the same argument meaning and returns (image HxWx3 uint8 numpy array,
RenderStat).  Where the reference panics (Color::to_u8_array's `<= 2.0` assert,
color.rs:55-57; unknown material, materials.rs:31; spp == 0 -> 0/0) this raises RtError.
There is no CPU fallback: the HIP library must be built and a GPU present.
"""
import ctypes
import time

import numpy as np

from . import abi


class RenderStat:
    """renderer.rs:11-34 (+ the GPU work counters)."""

    def __init__(self, duration, pixels_rendered, kernel_ms=0.0, samples=0, ray_segments=0):
        self._duration = float(duration)
        self._pixels = int(pixels_rendered)
        self._pps = self._pixels / self._duration if self._duration > 0 else 0.0
        self.kernel_ms = kernel_ms
        self.samples = samples
        self.ray_segments = ray_segments

    def duration(self):
        return self._duration

    def pixels_rendered(self):
        return self._pixels

    def pixels_per_second(self):
        return self._pps


class Renderer:
    def render(self, max_bounces, samples_per_pixel, scene, camera):
        raise NotImplementedError


class GpuRenderer(Renderer):
    """Drop-in for TileRenderer: renders the whole image on one MI355X via rt_render_async.

    seed: 64-bit key of the counter-based RNG (the reference's thread_rng is unseedable);
    precision: "f64" (reference arithmetic) or "f32"; root2: quirk Q1 off;
    mode: which reference renderer to reproduce — "vectorized2" (the live render_vectorized2,
    default), "vectorized" (render_vectorized), "vectorized3" (render_vectorized3) or "scalar" (render);
    see include/rt_mi355x.h.
    """

    MODES = {"vectorized2": 0, "vectorized": abi.RT_FLAG_MODE_VECTORIZED, "vectorized3": abi.RT_FLAG_MODE_VECTORIZED3,
             "scalar": abi.RT_FLAG_MODE_SCALAR}

    def __init__(self, device=0, seed=0x5EED0001, precision="f64", root2=False, mode="vectorized2", lib=None):
        if mode not in self.MODES:
            raise ValueError(f"unknown mode {mode!r} (one of {sorted(self.MODES)})")
        if precision not in ("f64", "f32"):
            raise ValueError(f"unknown precision {precision!r}")
        self.lib = lib or abi.load_library()
        self.device = device
        self.seed = seed
        self.flags = ((abi.RT_FLAG_F32 if precision == "f32" else 0) | (abi.RT_FLAG_ROOT2 if root2 else 0)
                      | self.MODES[mode])
        self.ctx = ctypes.c_void_p()
        abi.check(self.lib, self.lib.rt_context_create(device, ctypes.byref(self.ctx)))
        self._scene_flat = None   # the FlatScene last uploaded (held, so its identity cannot be reused)

    def close(self):
        if self.ctx:
            self.lib.rt_context_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, flat):
        # rt_context_set_scene frees the previous scene before uploading this one: if the upload fails
        # the context holds no usable scene, so the cache must not point at the previous one either.
        self._scene_flat = None
        abi.check(self.lib, self.lib.rt_context_set_scene(self.ctx, ctypes.byref(flat.abi)))
        # A strong reference, compared with `is`: an id() key could match a new FlatScene that CPython
        # allocated at a freed one's address, and the render would silently use the old spheres.
        self._scene_flat = flat

    def render_flat(self, max_bounces, spp, flat, cam, tile_range=None, want_linear=False):
        """Render with a FlatScene / RtCamera; returns (rgb [n,3] u8, linear [n,3] f64 | None, RtStats, rc)."""
        lib = self.lib
        if self._scene_flat is not flat:
            self.set_scene(flat)
        if tile_range is None:
            tr = abi.RtTileRange(0, 1, cam.image_height, 0, cam.image_width)
        else:
            tr = tile_range
        npx = tr.row_count * tr.col_count
        d_rgb, d_lin = ctypes.c_void_p(), ctypes.c_void_p()
        abi.check(lib, lib.rt_device_alloc(self.ctx, npx * 3, ctypes.byref(d_rgb)))
        try:
            if want_linear:
                abi.check(lib, lib.rt_device_alloc(self.ctx, npx * 3 * 8, ctypes.byref(d_lin)))
            abi.check(lib, lib.rt_render_async(self.ctx, ctypes.byref(cam), max_bounces, spp, self.seed, self.flags,
                                               ctypes.byref(tr), d_rgb, d_lin if want_linear else None, None))
            st = abi.RtStats()
            rc = abi.check(lib, lib.rt_context_collect(self.ctx, None, ctypes.byref(st)), allow=(abi.RT_ERR_RANGE,))
            rgb = np.empty((npx, 3), dtype=np.uint8)
            abi.check(lib, lib.rt_memcpy_d2h(self.ctx, rgb.ctypes.data, d_rgb, npx * 3))
            lin = None
            if want_linear:
                lin = np.empty((npx, 3), dtype=np.float64)
                abi.check(lib, lib.rt_memcpy_d2h(self.ctx, lin.ctypes.data, d_lin, npx * 3 * 8))
        finally:
            lib.rt_device_free(self.ctx, d_rgb)
            if want_linear and d_lin:
                lib.rt_device_free(self.ctx, d_lin)
        return rgb, lin, st, rc

    def render(self, max_bounces, samples_per_pixel, scene, camera):
        t0 = time.perf_counter()
        flat = scene.flatten() if hasattr(scene, "flatten") else scene
        cam = camera.abi if hasattr(camera, "abi") else camera
        rgb, _, st, rc = self.render_flat(max_bounces, samples_per_pixel, flat, cam)
        dt = time.perf_counter() - t0
        if rc == abi.RT_ERR_RANGE:
            raise abi.RtError(rc, "a pixel channel exceeded 2.0 (reference: Color::to_u8_array panics)")
        img = rgb.reshape(cam.image_height, cam.image_width, 3)
        return img, RenderStat(dt, cam.image_width * cam.image_height, st.kernel_ms, st.samples, st.ray_segments)
