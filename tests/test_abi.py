"""The drop-in C ABI (include/rt_mi355x.h): the HIP library loads, exports every declared symbol,
and its struct layouts match what a C compiler sees.  No GPU compute here."""
import ctypes
import os
import re
import subprocess

import pytest

import rt_mi355x as rt
from rt_mi355x import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rt_mi355x.h")


def _ensure_built():
    if not os.path.exists(abi.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(REPO, "rust-ray-tracing_amd")], check=True, capture_output=True)


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(rt_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_abi():
    fns = declared_functions()
    assert sorted(abi.EXPORTED) == fns


def test_library_exports_every_symbol():
    _ensure_built()
    lib = ctypes.CDLL(abi.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_\w+)$", out, flags=re.M))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_only():
    """The fat binary carries exactly one code object, for gfx950 (no CUDA/dual path)."""
    _ensure_built()
    blob = open(abi.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}
    assert b"nvptx" not in blob


C_LAYOUT = r"""
#include <stdio.h>
#include <stddef.h>
#include "rt_mi355x.h"
#define P(T, F) printf(#T "." #F " %zu\n", offsetof(T, F));
int main(void) {
  printf("rt_material %zu\nrt_scene %zu\nrt_camera %zu\nrt_tile_range %zu\nrt_stats %zu\n",
         sizeof(rt_material), sizeof(rt_scene), sizeof(rt_camera), sizeof(rt_tile_range), sizeof(rt_stats));
  P(rt_material, albedo) P(rt_material, fuzz) P(rt_material, ior)
  P(rt_scene, center) P(rt_scene, radius) P(rt_scene, material) P(rt_scene, materials)
  P(rt_camera, center) P(rt_camera, ulc) P(rt_camera, dv)
  P(rt_stats, kernel_ms) P(rt_stats, ray_segments) P(rt_stats, bounce_iters)
  P(rt_stats, camera_exact_tests) P(rt_stats, direct_sky_samples) P(rt_stats, kernel_id) P(rt_stats, kernel_wg_per_cu)
  /* rt_stats.kernel_id's fields: trace_paths<double,4,true,3,true,true> and <float,6,false,0,true,false> */
  printf("id_a %u,%u,%u,%u,%u,%u\n", RT_KERNEL_F64(0x81F9u), RT_KERNEL_WAVES(0x81F9u), RT_KERNEL_ROOT2(0x81F9u),
         RT_KERNEL_MODE(0x81F9u), RT_KERNEL_CAMQ(0x81F9u), RT_KERNEL_MEGA(0x81F9u));
  printf("id_b %u,%u,%u,%u,%u,%u\n", RT_KERNEL_F64(0x808Cu), RT_KERNEL_WAVES(0x808Cu), RT_KERNEL_ROOT2(0x808Cu),
         RT_KERNEL_MODE(0x808Cu), RT_KERNEL_CAMQ(0x808Cu), RT_KERNEL_MEGA(0x808Cu));
  return 0;
}
"""


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text(C_LAYOUT)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.splitlines())
    py = {
        "rt_material": ctypes.sizeof(abi.RtMaterial), "rt_scene": ctypes.sizeof(abi.RtScene),
        "rt_camera": ctypes.sizeof(abi.RtCamera), "rt_tile_range": ctypes.sizeof(abi.RtTileRange),
        "rt_stats": ctypes.sizeof(abi.RtStats),
    }
    for k, v in py.items():
        assert int(got[k]) == v, k
    # the header's RT_KERNEL_* macros and abi.kernel_info decode kernel_id alike
    for tag, kid in (("id_a", 0x81F9), ("id_b", 0x808C)):
        k = abi.kernel_info(kid)
        want = [int(k["T"] == "double"), k["W"], int(k["root2"]), k["mode"], int(k["camq"]), int(k["mega"])]
        assert [int(x) for x in got.pop(tag).split(",")] == want, tag
    assert abi.kernel_name(0x808C) == "trace_paths<float,6,false,0,true,false>"
    assert abi.kernel_name(0x81F9) == "trace_paths<double,4,true,3,true,true>"
    assert abi.kernel_info(0) is None
    for key, val in got.items():
        if "." in key:
            st, field = key.split(".")
            cls = {"rt_material": abi.RtMaterial, "rt_scene": abi.RtScene, "rt_camera": abi.RtCamera,
                   "rt_stats": abi.RtStats}[st]
            assert getattr(cls, field).offset == int(val), key


def test_host_only_entry_points():
    """rt_camera_new / rt_metal_clamp_fuzz / rt_version are pure host code."""
    _ensure_built()
    lib = rt.load_library()
    assert lib.rt_version().startswith(b"rt_mi355x")
    assert lib.rt_metal_clamp_fuzz(5.0) == 1.0 and lib.rt_metal_clamp_fuzz(0.25) == 0.25
    cam = rt.Camera(1920, 1080, **rt.MAIN_CAMERA, lib=lib)
    py = rt.camera_new_py(1920, 1080, **rt.MAIN_CAMERA)
    for f in ("center", "ulc", "vu", "vv", "du", "dv"):
        assert list(getattr(cam.abi, f)) == list(getattr(py, f)), f
    assert list(cam.abi.ulc) == [5.734425819985221, 3.855608886593495, 13.912440284912917]
    D3 = ctypes.c_double * 3
    bad = abi.RtCamera()
    assert lib.rt_camera_new(ctypes.byref(bad), 0, 10, 10.0, 30.0, D3(0, 0, 0), D3(0, 0, 1), D3(0, 1, 0), 0.0) \
        == abi.RT_ERR_INVALID
    assert b"bad argument" in lib.rt_last_error()


def test_no_gpu_fails_loudly():
    """Without a GPU the library reports an error instead of falling back to the CPU."""
    _ensure_built()
    lib = rt.load_library()
    ctx = ctypes.c_void_p()
    rc = lib.rt_context_create(0, ctypes.byref(ctx))
    if rc == abi.RT_OK:
        lib.rt_context_destroy(ctx)
        pytest.skip("GPU present")
    assert rc in (abi.RT_ERR_HIP, abi.RT_ERR_INVALID)
    assert lib.rt_last_error()
    with pytest.raises(rt.RtError):
        rt.GpuRenderer(lib=lib)


def test_header_constants_match_python_mirror():
    """Every RT_* #define in include/rt_mi355x.h has the same value in rt_mi355x.abi."""
    import re
    hdr = open(os.path.join(REPO, "include", "rt_mi355x.h")).read()
    defs = dict(re.findall(r"#define\s+(RT_[A-Z0-9_]+)\s+(0x[0-9A-Fa-f]+|\d+)u?\b", hdr))
    assert {"RT_FLAG_F32", "RT_FLAG_ROOT2", "RT_FLAG_MODE_VECTORIZED", "RT_FLAG_MODE_SCALAR", "RT_FLAG_MODE_VECTORIZED3",
            "RT_FLAG_ALL"} <= set(defs)
    for name, val in defs.items():
        assert getattr(abi, name) == int(val, 0), name


# ---- build kinds (product vs experiment) and the source hash -------------------------------------
CSRC = os.path.join(REPO, "rust-ray-tracing_amd", "csrc")
EXPERIMENTS = os.path.join(CSRC, "rt_experiments.hpp")
EXP_PATCHES = os.path.join(REPO, "tools", "exp")
MAKEFILE = os.path.join(REPO, "rust-ray-tracing_amd", "Makefile")


def _csrc_files():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp")))


def _patches():
    return sorted(os.path.join(EXP_PATCHES, f) for f in os.listdir(EXP_PATCHES) if f.endswith(".patch"))


def test_product_library_reports_its_sources():
    """The default build is a product build, made from the sources in this tree."""
    _ensure_built()
    lib = ctypes.CDLL(abi.LIB_PATH)
    lib.rt_version.restype = ctypes.c_char_p
    v = abi.version_info(lib)
    assert v["kind"] == "product", v
    assert v["src_hash"] == abi.source_hash(), (v, "rebuild: make -C rust-ray-tracing_amd")


def test_every_source_is_hashed():
    """Every csrc/ file is in the source hash (abi.SOURCE_FILES, the Makefile's SRC + HDR)."""
    hashed = {os.path.basename(f) for f in abi.SOURCE_FILES}
    assert set(_csrc_files()) <= hashed, sorted(set(_csrc_files()) - hashed)
    mk = open(MAKEFILE).read()
    for f in _csrc_files():
        assert "csrc/" + f in mk, f


def test_every_experiment_macro_is_refused_by_the_product_build():
    """Each RT_EXP_* (and RT_KSTATS) macro the sources or the experiment patches (tools/exp/) test is in
    the #error list the product build (-DRT_PRODUCT) checks, only rt_experiments.hpp names one among
    the product sources, and the product rule defines RT_PRODUCT and no experiment macro."""
    src = open(EXPERIMENTS).read()
    guard = src[src.index("#if defined(RT_PRODUCT) && (defined("):]
    guard = guard[:guard.index("#error")]
    listed = set(re.findall(r"defined\((RT_EXP_\w+|RT_KSTATS)\)", guard))
    texts = [open(os.path.join(CSRC, f)).read() for f in _csrc_files()] + [open(p).read() for p in _patches()]
    used = set()
    for text in texts:
        used |= set(re.findall(r"#\s*(?:ifdef|ifndef|if\s+!?\s*defined\(|elif\s+defined\()\s*(RT_EXP_\w+|RT_KSTATS)", text))
        used |= set(re.findall(r"defined\((RT_EXP_\w+)\)", text))
    assert used and used <= listed, sorted(used - listed)
    for f in _csrc_files():
        if f != "rt_experiments.hpp":
            assert "RT_EXP_" not in open(os.path.join(CSRC, f)).read(), f
    mk = open(MAKEFILE).read()
    rule = mk[mk.index("$(LIB): $(SRC) $(HDR)"):].split("\n\n")[0]
    assert "-DRT_PRODUCT" in rule and "RT_EXP" not in rule and "RT_EXPERIMENT" not in rule
    assert "RT_EXP" not in mk.split("HIPFLAGS ?=")[1].split("\n")[0]


def test_experiment_patches_apply(tmp_path):
    """The timing-experiment patches (tools/exp/*.patch, applied by `make exp`) apply cleanly to the
    current sources, so an A/B build measures this tree."""
    import shutil
    for f in _csrc_files():
        shutil.copy(os.path.join(CSRC, f), tmp_path / f)
    assert _patches()
    for p in _patches():
        with open(p) as fh:
            r = subprocess.run(["patch", "-s", "-p1", "-d", str(tmp_path)], stdin=fh, capture_output=True, text=True)
        assert r.returncode == 0, (p, r.stdout, r.stderr)


def test_experiment_library_is_refused(tmp_path):
    """rt_mi355x.load_library refuses a library whose rt_version() says "experiment" (make exp / kstats)
    unless RT_ALLOW_EXPERIMENT=1.  A stand-in .so with only rt_version() is enough to check the gate."""
    c = tmp_path / "fake.c"
    c.write_text('const char* rt_version(void) { return "rt_mi355x 0.3 gfx950 experiment src=000000000000"; }\n')
    so = tmp_path / "libfake.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(c)], check=True)
    old = os.environ.pop("RT_ALLOW_EXPERIMENT", None)
    try:
        with pytest.raises(RuntimeError, match="experiment build"):
            abi.load_library(str(so))
    finally:
        if old is not None:
            os.environ["RT_ALLOW_EXPERIMENT"] = old


def test_source_hash_matches_the_makefile_recipe():
    """abi.source_hash() == `cat kernel device-header abi-header | sha256sum | cut -c1-12`."""
    out = subprocess.run("cat " + " ".join(abi.SOURCE_FILES) + " | sha256sum | cut -c1-12", shell=True,
                         capture_output=True, text=True, check=True).stdout.strip()
    assert out == abi.source_hash()
