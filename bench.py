#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X sample loop on BASELINE.json's headline config.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f32|f64] [--config C]

One step = one full frame of config C (1920x1080, 500 spheres, 512 spp, 50 bounces): every rank
renders its row-interleaved shard (rows r, r+N, ...) with the HIP megakernel, then rank 0 gathers
the RGB8 shards over RCCL and re-interleaves them (the north star's tiles + gather; total work is
fixed as N grows -> "scaling": "strong").  Inputs (scene SoA, camera) are resident in HBM before
the timed region.  Rank 0 prints one JSON line.

roofline: the trace kernel is VALU-issue-bound (no MFMA; HBM traffic ~5 % of bandwidth).
  algorithmic FLOP per launch = 17 * n_spheres * ray_segments   (the reference's
  mandatory 17-FLOP sphere test per segment and sphere; segments counted in-kernel), achieved = that /
  average launch duration (HIP events on the launch stream), peak = the packed-FP32 VALU peak for
  both dtypes: fp64 rays also sweep the spheres with the packed-FP32 filters, fp64
  arithmetic is only used on filter candidates.  The filters spend fewer instructions per (ray,
  sphere) than the 17-FLOP test, so this frac is an effective (brute-force-equivalent) rate; the
  physical bound is VALU issue, reported as valu_issue_frac = VALU instructions per launch (PMC,
  profiles/traffic.json) * 4 cycles / (1024 SIMDs * launch time * 2.4 GHz).
cpu_baseline: the CPU restatement (oracle/, f64, 4-lane packets like PackedRays<4>) on this host's
  cores over a bounded strided pixel sample of the same workload.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))

FP32_VALU_PEAK_TF = 157.3   # MI355X_MICROARCH.md chip table (packed FP32 vector)
N_SIMD, CLOCK_HZ = 1024, 2.4e9   # 256 CUs x 4 SIMDs; peak engine clock (one wave64 VALU per 4 cycles)
FLOP_PER_SPHERE_TEST = 17


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0001)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all cores of this process")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--max-spheres", type=int, default=0, help="experiment: truncate the scene (not a bench line)")
    return ap.parse_args()


def cpu_baseline(flat, cam, depth, spp, seed, budget_s, threads):
    """Oracle (CPU restatement, f64) on a strided pixel sample; grows the sample until ~budget_s."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_bind import oracle_render
    W, H = cam.image_width, cam.image_height
    n_all = W * H
    order = (np.arange(n_all, dtype=np.int64) * 7919) % n_all   # 7919 prime, coprime with W*H
    done, t_used, batch, segs = 0, 0.0, 8 * threads, 0
    for _ in range(6):   # a calibration batch, then batches sized to fill the budget
        px = order[done:done + batch].astype(np.uint32)
        if len(px) == 0:
            break
        t0 = time.perf_counter()
        _, _, s, rc = oracle_render(flat, cam, depth, spp, seed, 0, pixels=px, precision="f64", threads=threads)
        t_used += time.perf_counter() - t0
        done += len(px)
        segs += s
        batch = int(1.1 * max(0.0, budget_s - t_used) / (t_used / done))
        if t_used >= 0.95 * budget_s:
            break
    return {
        "value": done * spp / t_used / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} of {n_all} pixels (stride-7919 permutation) x {spp} spp, f64, {t_used:.1f} s",
        "ray_segments_per_sample": segs / (done * spp),
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    import numpy as np
    import torch   # imported before the HIP library so both share one HIP runtime
    import torch.distributed as dist

    # One process per GPU.  RT_BENCH_BACKEND=gloo (rehearsal only: several ranks sharing one GPU,
    # shards staged through host memory) exercises the same partition/gather/assembly code.
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1 or "RANK" in os.environ:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    import rt_mi355x as rt
    from rt_mi355x import abi

    lib = rt.load_library()
    W, H, n_sph, spp, depth = rt.scenes.CONFIGS[args.config]
    scene = rt.scenes.config_scene(args.config)
    if args.max_spheres:
        scene = rt.Scene.from_list(scene.objects[:args.max_spheres])
        n_sph = len(scene.objects)
    flat = scene.flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    flags = abi.RT_FLAG_F32 if args.precision == "f32" else 0

    ctx = ctypes.c_void_p()
    abi.check(lib, lib.rt_context_create(device, ctypes.byref(ctx)))
    abi.check(lib, lib.rt_context_set_scene(ctx, ctypes.byref(flat.abi)))

    from rt_mi355x import parallel
    tile = parallel.shard_range(W, H, world, rank)
    shard = torch.zeros((parallel.rows_max(H, world), W, 3), dtype=torch.uint8, device="cuda")
    gathered = [torch.empty_like(shard) for _ in range(world)] if (world > 1 and rank == 0) else None
    image = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") if rank == 0 else None
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)

    def step():
        abi.check(lib, lib.rt_render_async(ctx, ctypes.byref(cam), depth, spp, args.seed, flags, ctypes.byref(tile),
                                           ctypes.c_void_p(shard.data_ptr()), None, sptr))
        if world > 1:
            if backend == "nccl":   # RCCL over xGMI, device buffers
                dist.gather(shard, gathered, dst=0)
            else:
                host = [g.cpu() for g in gathered] if rank == 0 else None
                dist.gather(shard.cpu(), host, dst=0)
                if rank == 0:
                    for g, h in zip(gathered, host):
                        g.copy_(h)
            if rank == 0:
                parallel.assemble_rows(gathered, H, world, image)
        elif rank == 0:
            image.copy_(shard[:H])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    st = abi.RtStats()
    abi.check(lib, lib.rt_context_collect(ctx, sptr, ctypes.byref(st)), allow=(abi.RT_ERR_RANGE,))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0

    st = abi.RtStats()
    rc = abi.check(lib, lib.rt_context_collect(ctx, sptr, ctypes.byref(st)), allow=(abi.RT_ERR_RANGE,))
    segs = st.ray_segments
    kernel_ms = st.kernel_ms

    red_dev = "cuda" if backend == "nccl" else "cpu"
    stats = torch.tensor([elapsed, float(segs), kernel_ms], dtype=torch.float64, device=red_dev)
    if world > 1:
        t_max = stats[0].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        seg_sum = stats[1].clone()
        dist.all_reduce(seg_sum, op=dist.ReduceOp.SUM)
        elapsed = float(t_max.item())
        segs_total = int(seg_sum.item())
    else:
        segs_total = int(segs)

    if rank == 0:
        samples = W * H * spp * args.steps
        value = samples / elapsed / 1e6
        # roofline on rank 0's own kernel: its algorithmic FLOPs / its average launch duration
        launch_s = (kernel_ms / 1e3) / args.steps
        flop_launch = FLOP_PER_SPHERE_TEST * n_sph * (segs / args.steps)
        achieved = flop_launch / launch_s / 1e12
        peak = FP32_VALU_PEAK_TF
        traffic, valu_insts = None, None
        try:
            with open(args.traffic) as f:
                tr = json.load(f)
            key = f"{args.config}:{args.precision}:{world}"
            traffic = tr.get(key, {}).get("hbm_bytes_per_launch")
            valu_insts = tr.get(key, {}).get("valu_insts_per_launch")
        except (OSError, ValueError):
            pass
        line = {
            "metric": "Msamples/s (pixels×spp/s), 1920×1080·512spp·500 spheres; 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: {W}x{H}, {n_sph} spheres (RTIOW-style, seed 0x5EED0001), "
                            f"{spp} spp, {depth} bounces, camera of src/main.rs:51-58",
                "width": W, "height": H, "spheres": n_sph, "spp": spp, "max_bounces": depth,
                "parallelism": f"row-interleaved image shards x{world}"
                               + ((" + RCCL gather" if backend == "nccl" else f" + {backend} gather (rehearsal)")
                                  if world > 1 else ""),
            },
            "roofline": {
                "bound": "valu",
                "achieved": round(achieved, 3),
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4),
                "traffic": traffic,
                "flop_per_launch": flop_launch,
                "launch_ms": round(launch_s * 1e3, 3),
                "valu_issue_frac": (round(valu_insts * 4 / (N_SIMD * launch_s * CLOCK_HZ), 4)
                                    if valu_insts else None),
            },
            "ray_segments_per_sample": round(segs_total / samples, 5),
            "lane_utilisation": round(st.ray_segments / max(1, st.lane_slots), 4),
            "bounces_per_pixel": round(st.bounce_iters / max(1, st.pixels), 3),
            "range_error": rc == abi.RT_ERR_RANGE,
        }
        if world == 1 and args.cpu_seconds > 0:
            threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
            line["cpu_baseline"] = cpu_baseline(flat, cam, depth, spp, args.seed, args.cpu_seconds, threads)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)

    if rank == 0 and os.environ.get("RT_BENCH_SAVE"):
        import numpy as np
        np.save(os.environ["RT_BENCH_SAVE"], image.cpu().numpy())
    lib.rt_context_destroy(ctx)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
