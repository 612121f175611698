"""The sweep filters never drop a sphere the reference could hit (CPU).

rt_kernel.hip tests every bounced ray against every sphere with a cheap fp32 filter first
(x^2 + y^2 <= r^2 + m in a basis perpendicular to the ray, nearest_hit / filter_group) and runs
the reference's exact sphere test (objects.rs:252-257 / 217-222) only for groups that pass.  This
is only bit-exact if the filter is conservative against the reference's OWN rounding: whenever
the reference computes disc >= 0, the filter must pass.  filter_margin_fuzz.c restates the
kernel's filter arithmetic and the reference's discriminant in all four arithmetic modes and
checks that claim on adversarial near-tangent cases; the margin factor 48 u must also keep a
safety factor over the worst case seen (a first-order error bound gives ~30 u).
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
MARGIN_U = 48.0


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("fuzz") / "filter_margin_fuzz")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out, os.path.join(HERE, "filter_margin_fuzz.c"), "-lm"],
                   check=True)
    return out


def _kernel_src():
    """Every csrc/ source of the library (one translation unit, split by stage)."""
    d = os.path.join(HERE, "..", "rust-ray-tracing_amd", "csrc")
    return "\n".join(open(os.path.join(d, f)).read() for f in sorted(os.listdir(d)) if f.endswith((".hip", ".hpp")))


def test_margin_constant_matches_kernel():
    src = _kernel_src()
    assert "kFilterMargin = 48.0f * 0x1.0p-24f" in src
    assert "KM = 48.0f * 0x1.0p-24f" in open(os.path.join(HERE, "filter_margin_fuzz.c")).read()


@pytest.mark.parametrize("local", [0, 1], ids=["scene", "cluster_local"])
@pytest.mark.parametrize("mode", [0, 1, 2, 3], ids=["f32_packed", "f32_scalar", "f64_packed", "f64_scalar"])
def test_filter_is_conservative(fuzz_bin, mode, local):
    """The sphere filter passes every sphere the reference's arithmetic could hit, in the scene-wide
    frame and (local) in the MEGA kernels' cluster-local frames far from the origin."""
    r = subprocess.run([fuzz_bin, "3000000", str(mode), str(0x9E3779B97F4A7C15 + mode + 17 * local), str(local)],
                       capture_output=True, text=True, timeout=300)
    line = r.stdout.strip()
    fields = line.split()
    misses = int(fields[fields.index("misses") + 1])
    accepted = int(fields[fields.index("ref-accepted") + 1])
    worst = float(fields[fields.index("need") + 1])
    assert r.returncode == 0 and misses == 0, line
    assert accepted > 1000000, line          # the cases really sit on both sides of tangency
    assert worst < MARGIN_U / 4, line        # >= 4x headroom over the worst case found


@pytest.fixture(scope="module")
def cam_fuzz_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("camfuzz") / "cam_filter_fuzz")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out, os.path.join(HERE, "cam_filter_fuzz.c"), "-lm"],
                   check=True)
    return out


def test_cam_margin_constant_matches_kernel():
    src = _kernel_src()
    assert "sqrt(cd) - 0x1.8p-20 * ocn - 1e-20" in src      # 24 u |oc| + 1e-20
    assert "sqrt(c64) - 24 * u * ocn - 1e-20" in open(os.path.join(HERE, "cam_filter_fuzz.c")).read()


@pytest.mark.parametrize("f64", [0, 1], ids=["f32", "f64"])
def test_camera_filter_is_conservative(cam_fuzz_bin, f64):
    """Camera batches under Q1: every valid root1 passes hb' + sc < 0 (margin 24 u; >= 4x headroom)."""
    r = subprocess.run([cam_fuzz_bin, "3000000", str(f64), str(0x5851F42D4C957F2D + f64)], capture_output=True,
                       text=True, timeout=300)
    fields = r.stdout.split()
    misses = int(fields[fields.index("misses") + 1])
    valid = int(fields[fields.index("valid") + 1])
    worst = float(fields[-1])
    assert r.returncode == 0 and misses == 0, r.stdout
    assert valid > 1000000, r.stdout
    assert worst < 24.0 / 4, r.stdout


@pytest.fixture(scope="module")
def cone_fuzz_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("conefuzz") / "cone_cull_fuzz")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out, os.path.join(HERE, "cone_cull_fuzz.c"), "-lm"],
                   check=True)
    return out


def test_cone_margin_constant_matches_kernel():
    src = _kernel_src()
    expr = "sqrt((double)r2 * (1.0 + 0x1.0p-20) + 0x1.0p-18 * wn2) + 0x1.0p-19 * sqrt(wn2) + 1e-30"   # 64 u, 32 u
    assert expr in src
    assert expr.replace("(double)r2 *", "r2t *") in open(os.path.join(HERE, "cone_cull_fuzz.c")).read()
    assert "__builtin_fmaf(__builtin_amdgcn_sqrtf(__uint_as_float(sm)), 1.0f + 0x1.0p-22f, 0x1.0p-21f)" in src
    assert "__builtin_amdgcn_sqrtf(__builtin_fmaf(pz, pz" in src   # p by v_sqrt_f32; the fuzz models +-1 ulp
    # cluster records: rp_k >= rp_i + |c_i - C| for every member (the fuzz also checks this directly)
    assert "rup(R * (1.0 + 0x1.0p-20) + (0x1.0p-9 + 0x1.0p-16) * (wn + R) + 1e-30)" in src
    assert "RR * (1.0 + 0x1.0p-20) + (0x1.0p-9 + 0x1.0p-16) * (Wn + RR) + 1e-30" in \
        open(os.path.join(HERE, "cone_cull_fuzz.c")).read()


@pytest.mark.parametrize("f64", [0, 1], ids=["f32", "f64"])
def test_camera_cone_cull_is_conservative(cone_fuzz_bin, f64):
    """Camera batches: a sphere any ray of the batch hits (Q1, root2 or scalar test) passes the
    wave's cone cull; the worst case found uses at most a quarter of rp - r (>= 4x headroom)."""
    r = subprocess.run([cone_fuzz_bin, "2000000", str(f64), str(0x2545F4914F6CDD1D + f64)], capture_output=True,
                       text=True, timeout=300)
    fields = r.stdout.split()
    misses = int(fields[fields.index("misses") + 1])
    hits = int(fields[fields.index("hits") + 1])
    culled = int(fields[fields.index("culled") + 1])
    worst = float(fields[-1])
    assert r.returncode == 0 and misses == 0, r.stdout
    assert hits > 1000000 and culled > 50000, r.stdout   # both sides of tangency are exercised
    assert worst < 0.25, r.stdout


@pytest.fixture(scope="module")
def pixel_fuzz_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("pixfuzz") / "pixel_cone_fuzz")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out, os.path.join(HERE, "pixel_cone_fuzz.c"), "-lm"],
                   check=True)
    return out


def test_pixel_margin_matches_kernel():
    src = _kernel_src()
    assert "const float margin = (M * 0x1.0p-20f) * __builtin_amdgcn_rsqf(dnc);" in src
    assert "1.0f + 0x1.0p-22f, 0x1.0p-21f + margin));" in src
    fz = open(os.path.join(HERE, "pixel_cone_fuzz.c")).read()
    assert "const float margin = (M * 0x1.0p-20f) * rsq(dnc);" in fz


@pytest.mark.parametrize("f64", [0, 1], ids=["f32", "f64"])
def test_pixel_cone_contains_every_ray(pixel_fuzz_bin, f64):
    """Per-pixel camera cones (pixel_list): every primary ray of the pixel, as computed in T, lies
    inside the cone (worst case well under a quarter of the pixel margin), and every sphere some ray
    of the pixel hits (Q1, root2 or scalar test) passes the cone's cull."""
    r = subprocess.run([pixel_fuzz_bin, "1500000", str(f64), str(0x9E3779B97F4A7C15 + f64)], capture_output=True,
                       text=True, timeout=300)
    fields = r.stdout.split()
    outside = int(fields[fields.index("outside") + 1])
    misses = int(fields[fields.index("misses") + 1])
    hits = int(fields[fields.index("hits") + 1])
    worst = float(fields[-1])
    assert r.returncode == 0 and outside == 0 and misses == 0, r.stdout
    assert hits > 1000000, r.stdout
    assert worst < 0.25, r.stdout


@pytest.fixture(scope="module")
def box_fuzz_bin(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("boxfuzz") / "box_cull_fuzz")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", out, os.path.join(HERE, "box_cull_fuzz.c"), "-lm"],
                   check=True)
    return out


def test_box_margin_constants_match_kernel():
    src = _kernel_src()
    fz = open(os.path.join(HERE, "box_cull_fuzz.c")).read()
    assert "1.0f + __builtin_fmaf(m, qa.f_hir2, pm * qa.f_isr)" in src
    assert "p.f_hir2 = up32(0.5 / r2m)" in src and "p.f_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m))" in src
    assert "1.0f + fmaf(48.0f * 0x1.0p-24f * fmaf(pm, pm, fr2max), up32(0.5 / fr2min), pm * isr)" in fz
    assert "isr = up32(8.0 * 0x1.0p-24 / sqrt((double)fr2min))" in fz
    # the mega kernels' group-local form (lmask): margin factor folded into l_hir2
    assert ("__builtin_fmaf(__builtin_fmaf(pmg, pmg, ql.l_r2max), ql.l_hir2,\n"
            "                                            __builtin_fmaf(pmg, ql.l_isr, 1.0f))") in src
    assert "p.l_hir2 = up32((double)kFilterMargin * 0.5 / r2m);" in src
    assert "p.l_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m));" in src
    assert "fmaf(fmaf(pm, pm, fr2max), up32(48.0 * 0x1.0p-24 * 0.5 / fr2min), fmaf(pm, isr, 1.0f))" in fz
    box = "h * (1.0 + 0x1.0p-20) + 0x1.0p-22 * std::fabs((double)b[a])"
    assert box in src and "hh * (1.0 + 0x1.0p-20) + 0x1.0p-22 * fabs((double)C[a])" in fz
    assert "__builtin_amdgcn_rcpf(fabsf(v) >= 1e-20f ? v : copysignf(1e-20f, v))" in src


@pytest.mark.parametrize("local", [0, 1], ids=["scene", "group_local"])
@pytest.mark.parametrize("f64", [0, 1], ids=["f32", "f64"])
def test_cluster_box_is_conservative(box_fuzz_bin, f64, local):
    """General sweep: a cluster whose member the reference hits (Q1, root2 or scalar test) passes
    the lane's slab test against the cluster box, with a quarter of the margin too (>= 4x headroom);
    in the scene-wide frame and (local) in the MEGA kernels' group frames far from the origin."""
    r = subprocess.run([box_fuzz_bin, "1500000", str(f64), str(0x9E3779B97F4A7C15 ^ (f64 + 7 + 64 * local)), str(local)],
                       capture_output=True, text=True, timeout=300)
    fields = r.stdout.split()
    hits = int(fields[fields.index("hits") + 1])
    culled = int(fields[fields.index("culled") + 1])
    assert r.returncode == 0 and int(fields[fields.index("misses") + 1]) == 0, r.stdout
    assert int(fields[fields.index("quarter-margin-misses") + 1]) == 0, r.stdout
    assert hits > (300000 if local else 500000) and culled > (100000 if local else 200000), r.stdout
