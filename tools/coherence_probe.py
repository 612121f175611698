#!/usr/bin/env python3
"""How coherent are the general sweep's waves?  Renders a row-strided shard of a BASELINE config with the
instrumented library (make kstats: rt_kstats on stderr) at several path depths.  At depth 2 every general
sweep holds bounce-1 rays only (the lanes of a wave then come from the same one or two pixels, so their
origins coincide); at depth 50 the waves mix bounces.  Per general wave-sweep: clusters walked, top box
groups, taken filter groups.  RT_MI355X_LIB=rust-ray-tracing_amd/lib/librt_mi355x_kstats.so RT_ALLOW_EXPERIMENT=1
    python3 tools/coherence_probe.py [config] [row_step] [depths]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import ctypes
    import rt_mi355x as rt
    from rt_mi355x import abi
    cfg, step, depth, prec = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    W, H, nsph, spp, _ = rt.scenes.CONFIGS[cfg]
    flat = rt.scenes.config_scene(cfg).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    r = rt.GpuRenderer(device=0, seed=0x5EED0001, precision=prec)
    tile = abi.RtTileRange(step // 2, step, len(range(step // 2, H, step)), 0, W)
    rgb, lin, st, rc = r.render_flat(depth, spp, flat, cam, tile_range=tile, want_linear=False)
    print(f"STATS segs {st.ray_segments} samples {st.samples} box {st.box_groups} filt {st.filter_groups} "
          f"exact {st.exact_tests} ms {st.kernel_ms:.2f}", flush=True)
    r.close()
    sys.exit(0)

cfg = sys.argv[1] if len(sys.argv) > 1 else "E"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 16
depths = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "2,3,50").split(",")]
prec = sys.argv[4] if len(sys.argv) > 4 else "f32"
for depth in depths:
    p = subprocess.run([sys.executable, __file__, "--child", cfg, str(step), str(depth), prec], capture_output=True,
                       text=True, timeout=300)
    ks = [ln for ln in p.stderr.splitlines() if ln.startswith("rt_kstats")]
    stl = [ln for ln in p.stdout.splitlines() if ln.startswith("STATS")]
    if p.returncode != 0 or not ks or not stl:
        print(f"{cfg} depth {depth}: failed rc={p.returncode}\n{p.stderr[-2000:]}")
        sys.exit(1)
    f = ks[-1].split()
    nums = [int(x) for x in f if x.isdigit()]   # taken, sweeps, clusters, top, cam cand, cam sweeps, finish, lanes
    kv = dict(zip(["taken_groups", "sweeps", "clusters", "top_groups", "cam_candidates", "cam_sweeps", "finish",
                   "filter_lanes"], nums))
    s = stl[-1].split()
    sv = {s[i]: float(s[i + 1]) for i in range(1, len(s) - 1, 2)}
    sw = max(kv.get("sweeps", 1), 1)
    print(f"{cfg} {prec} rows/{step} depth {depth:2d}: {sw} general sweeps, {sv['segs'] / sv['samples']:.3f} segments/sample, "
          f"per sweep: clusters {kv.get('clusters', 0) / sw:.2f}, top groups {kv.get('top_groups', 0) / sw:.2f}, "
          f"taken groups {kv.get('taken_groups', 0) / sw:.2f}, box groups {sv['box'] / sw:.2f}, filter groups "
          f"{sv['filt'] / sw:.2f}, exact {sv['exact'] / sw:.2f}; kernel {sv['ms']:.2f} ms  [{ks[-1]}]", flush=True)
