#!/usr/bin/env python3
"""Benchmark: Msamples/s of the MI355X sample loop on BASELINE.json's headline config.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f32|f64] [--config C]

One step = one full frame of config C (1920x1080, 500 spheres, 512 spp, 50 bounces): every rank
renders its row-interleaved shard (rows r, r+N, ...) with the HIP megakernel, then rank 0 gathers
the RGB8 shards over RCCL and re-interleaves them (the north star's tiles + gather; total work is
fixed as N grows -> "scaling": "strong").  With RCCL the shards are double-buffered: frame k's gather
is issued asynchronously and runs on RCCL's stream under frame k+1's render; frame k is assembled once
its gather is done (--no-overlap: gather, then render the next frame).  The last frame's gather and
assembly are inside the timed region.  Inputs (scene SoA, camera) are resident in HBM before
the timed region.  Rank 0 prints one JSON line.  After the headline leg the same steps run in the
other precision (fp64 = the reference's arithmetic when the headline is fp32), timed the same way,
under the line's "f64" / "f32" key.

roofline: the trace kernel is bound by VALU issue (no MFMA; HBM is not binding).
  executed FLOP per launch = 64 lanes x the FLOP per lane of every wave-level cull and exact test the
  kernel ran (in-kernel counters, rt_stats.box_groups .. camera_exact_tests; per-test FLOP in
  include/rt_mi355x.h), split fp32 / fp64; achieved = that / the average launch duration (HIP events
  around each launch on its stream); peak = 157.3 TF fp32, 78.6 TF fp64 (MI355X vector peaks),
  blended by the FLOP mix; frac = achieved / peak <= 1.  The reference's brute-force work (17 FLOP
  per ray segment and sphere) is reported separately as brute_force_equiv: the culls
  skip most of it, so its "rate" exceeds the chip's peak and says how much work is avoided.
  issue_frac: the VALU pipe's occupancy on a counter, 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / the
  dispatch's SIMD-cycles (VALU quad-cycles, minus those in which two instructions issued together; 1.0 = the
  pipe busy every cycle), and issue_frac_vs_ubench the same against the best VALU-saturating microbenchmark;
  pmc_flop_frac: every FLOP the kernel executes (SQ_INSTS_VALU_FLOPS_FP32/64) at the vector peaks.
  valu_busy and traffic come from rocprofv3 PMC passes of this bench (profiles/pmc.json, with the
  commit and kernel-source hash they were collected at); when that hash is not the loaded library's
  (rt_version() "src=..."), they are reported as null and pmc_source.stale = true.
--gpus N > 1 without a launcher (no RANK in the environment): bench.py starts N ranks itself, as a
  child `python -m torch.distributed.run --nproc-per-node N bench.py ...` (never exec), and exits with
  its return code; a rank whose initialised world size is not --gpus exits non-zero.
--schedule dynamic: instead of one static row shard per rank, the ranks pull chunks (rows j, j+M, ...)
  from a counter in the process group's store, the reference's shared tile channel; every rank writes
  its chunks into a zeroed full frame and one RCCL reduce (sum) assembles the image on rank 0.
cpu_baseline: the CPU restatement (oracle/, f64, 4-lane packets like PackedRays<4>), built
  -march=native on this host, on every core this process may use (affinity, capped by the cgroup's
  CPU quota), over a bounded strided pixel sample of the same workload; cpu_baseline.packed: the
  reference-shaped run of the same path (explicit AVX2 packets, 128x128 tiles through a shared queue)
  over a bounded sample of whole tiles.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rust-ray-tracing_amd"))

PEAK_TF = {"f32": 157.3, "f64": 78.6}   # MI355X vector peaks (MI355X_MICROARCH.md chip table; AMD spec fp64)
FLOP_PER_SPHERE_TEST = 17   # the reference's mandatory test per (segment, sphere)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--other-precision", type=int, default=1, help="also time the other precision (0 = skip)")
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0001)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may use")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc.json"))
    ap.add_argument("--max-spheres", type=int, default=0, help="experiment: truncate the scene (not a bench line)")
    ap.add_argument("--schedule", default="static", choices=["static", "dynamic"],
                    help="static: rank r renders rows r, r+N, ... (one launch); dynamic: ranks pull row-interleaved "
                         "chunks from a shared queue (the reference's tile channel, renderer.rs:248-296)")
    ap.add_argument("--chunks", type=int, default=0, help="dynamic schedule: chunks per frame (0 = 4 x ranks)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="static schedule, nccl: gather each frame before the next render (no double buffering)")
    ap.add_argument("--overlap-gloo", action="store_true",
                    help="rehearsal: the double-buffered gather over gloo (host-staged shards), for one-GPU boxes")
    ap.add_argument("--probe-dist", action="store_true",
                    help="launcher rehearsal: set up the ranks and the process group, print the world, no GPU work")
    return ap.parse_args()


def pmc_fields(pmc, lib_src_hash, source_file):
    """roofline.traffic / valu_busy / pmc_source from a PMC record (tools/pmc_round.py).  The figures
    count only if they were collected from the kernel sources the loaded library was built from:
    otherwise (another hash, or a record without one) they are null and pmc_source.stale is true."""
    keys = ("issue_frac", "issue_frac_vs_ubench", "pmc_flop_frac")
    if not pmc:
        return {"traffic": None, "valu_busy": None, **{k: None for k in keys}, "pmc_source": None}
    stale = pmc.get("src_hash") is None or pmc.get("src_hash") != lib_src_hash
    return {"traffic": None if stale else pmc.get("hbm_bytes_per_launch"),
            "valu_busy": None if stale else pmc.get("valu_busy"),
            **{k: (None if stale else pmc.get(k)) for k in keys},
            "pmc_source": {"file": source_file, "commit": pmc.get("commit"), "src_hash": pmc.get("src_hash"),
                           "library_src_hash": lib_src_hash, "stale": stale, "launch_ms": pmc.get("launch_ms")}}


def self_launch(args):
    """--gpus N > 1 with no launcher around us: run N ranks under torch.distributed.run as a child
    process (one process per GPU, rendezvous on 127.0.0.1) and return its exit code; None when this
    process is already a rank (or N == 1).  Nothing here touches the GPU."""
    if args.gpus <= 1 or "RANK" in os.environ or "WORLD_SIZE" in os.environ:
        return None
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench.py: --gpus {args.gpus}: launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def cpu_share():
    """Cores this process may run on: the affinity set, capped by the cgroup v2 CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, {"nproc": os.cpu_count(), "affinity": aff, "cgroup_cpu_quota": quota, "cpu_model": model}


def cpu_baseline(flat, cam, depth, spp, seed, budget_s, threads, host):
    """Oracle (CPU restatement, f64) on a strided pixel sample; grows the sample until ~budget_s."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_bind
    lib_path = oracle_bind.build_native()
    build = "-O3 -march=native" if lib_path else "-O3 -march=x86-64-v3 (native build failed)"
    W, H = cam.image_width, cam.image_height
    n_all = W * H
    order = (np.arange(n_all, dtype=np.int64) * 7919) % n_all   # 7919 prime, coprime with W*H
    done, t_used, batch, segs = 0, 0.0, 8 * threads, 0
    for _ in range(6):   # a calibration batch, then batches sized to fill the budget
        px = order[done:done + batch].astype(np.uint32)
        if len(px) == 0:
            break
        t0 = time.perf_counter()
        _, _, s, rc = oracle_bind.oracle_render(flat, cam, depth, spp, seed, 0, pixels=px, precision="f64",
                                                threads=threads, lib_path=lib_path)
        t_used += time.perf_counter() - t0
        done += len(px)
        segs += s
        batch = int(1.1 * max(0.0, budget_s - t_used) / (t_used / done))
        if t_used >= 0.95 * budget_s:
            break
    out = {
        "value": done * spp / t_used / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{done} of {n_all} pixels (stride-7919 permutation) x {spp} spp, f64, {t_used:.1f} s",
        "build": build,
        "ray_segments_per_sample": segs / (done * spp),
    }
    out.update(host)
    # The reference-shaped run (oracle/packed_avx2.h): 4-lane f64 AVX2 packets like PackedRays<4>, the frame
    # in 128x128 tiles that every thread pulls from one shared counter (renderer.rs:243-296), on the same
    # cores; a bounded sample of whole tiles spread over the frame (a prime stride over the tile grid),
    # one tile per thread to calibrate, then enough tiles to fill the budget.
    tx, ty = (W + 127) // 128, (H + 127) // 128
    torder = [(k * 37) % (tx * ty) for k in range(tx * ty)]   # 37: coprime with the tile count of every config
    done_t, t_pk, px_pk, segs_pk, n = 0, 0.0, 0, 0, threads
    for _ in range(2):
        tl = torder[done_t:done_t + n]
        if not tl:
            break
        t0 = time.perf_counter()
        _, _, s, npx, rc = oracle_bind.packed_render(flat, cam, depth, spp, seed, tiles=tl, threads=threads,
                                                     lib_path=lib_path)
        t_pk += time.perf_counter() - t0
        done_t += len(tl)
        px_pk += npx
        segs_pk += s
        n = max(threads, int(max(0.0, budget_s - t_pk) / (t_pk / done_t)) // threads * threads)
        if t_pk >= 0.8 * budget_s:
            break
    out["packed"] = {"value": px_pk * spp / t_pk / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
                     "sample": f"{done_t} of {tx * ty} 128x128 tiles ({px_pk} pixels, stride-37 tile order) x {spp} spp, "
                               f"f64, {t_pk:.1f} s",
                     "shape": "explicit 4-lane f64 AVX2 packets (PackedRays<4>), 128x128 tiles through a shared "
                              "queue (renderer.rs:243-296); bit-identical to the scalar port (tests/test_oracle_packed.py)",
                     "ray_segments_per_sample": segs_pk / max(1, px_pk * spp)}
    # BASELINE.json configs[0], the reference's own CPU case, timed in full: 400x225, the 3-sphere
    # scene, 16 spp, 8 bounces, f64, on the same cores (best of 3: it takes well under a second)
    import rt_mi355x as rt
    fa = rt.scenes.config_scene("A").flatten()
    ca = rt.camera_new_py(400, 225, **rt.MAIN_CAMERA)
    best = None
    for _ in range(3):
        t0 = time.perf_counter()
        _, _, sa, _ = oracle_bind.oracle_render(fa, ca, 8, 16, seed, 0, precision="f64", threads=threads,
                                                lib_path=lib_path)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    best_pk = None
    for _ in range(3):
        t0 = time.perf_counter()
        oracle_bind.packed_render(fa, ca, 8, 16, seed, threads=threads, lib_path=lib_path)
        dt = time.perf_counter() - t0
        best_pk = dt if best_pk is None else min(best_pk, dt)
    out["config_a"] = {"value": 400 * 225 * 16 / best / 1e6, "unit": "Msamples/s", "seconds": best,
                       "packed_value": 400 * 225 * 16 / best_pk / 1e6, "packed_seconds": best_pk,
                       "px_per_s": 400 * 225 / best, "cores": threads, "kind": "port",
                       "sample": "all 90000 pixels x 16 spp, 8 bounces, 3-sphere scene, f64 (best of 3)",
                       "ray_segments_per_sample": sa / (400 * 225 * 16)}
    return out


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch   # imported before the HIP library so both share one HIP runtime
    import torch.distributed as dist

    # One process per GPU.  RT_BENCH_BACKEND=gloo (rehearsal only: several ranks sharing one GPU,
    # shards staged through host memory) exercises the same partition/gather/assembly code.
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    if args.probe_dist:
        backend = "gloo"   # the rehearsal exchanges CPU tensors and must not initialise the GPU
    device = 0
    if not args.probe_dist:
        device = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
    if world > 1 or "RANK" in os.environ:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
    dist_on = dist.is_initialized()
    world_init = dist.get_world_size() if dist_on else 1
    if world_init != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the initialised world size is {world_init} "
              f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')}): refusing to report a {world_init}-GPU line as "
              f"{args.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(3)
    if args.probe_dist:
        ranks = [rank]
        if dist_on:
            t = torch.tensor([float(rank)], dtype=torch.float64)
            allr = [torch.empty_like(t) for _ in range(world_init)]
            dist.all_gather(allr, t)
            ranks = [int(a.item()) for a in allr]
        if rank == 0:
            print(json.dumps({"probe_dist": True, "n_gpus": world_init, "gpus_arg": args.gpus,
                              "dist": {"backend": backend if dist_on else None, "world_size_initialised": world_init,
                                       "ranks": ranks}}), flush=True)
        if dist_on:
            dist.destroy_process_group()
        return

    import rt_mi355x as rt
    from rt_mi355x import abi

    lib = rt.load_library()
    vinfo = abi.version_info(lib)
    src_hash = abi.source_hash()
    if vinfo["src_hash"] != src_hash and rank == 0:
        print(f"bench.py: warning: the library was built from sources {vinfo['src_hash']}, the tree holds "
              f"{src_hash} (rebuild with make -C rust-ray-tracing_amd)", file=sys.stderr, flush=True)
    W, H, n_sph, spp, depth = rt.scenes.CONFIGS[args.config]
    scene = rt.scenes.config_scene(args.config)
    if args.max_spheres:
        scene = rt.Scene.from_list(scene.objects[:args.max_spheres])
        n_sph = len(scene.objects)
    flat = scene.flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)

    ctx = ctypes.c_void_p()
    abi.check(lib, lib.rt_context_create(device, ctypes.byref(ctx)))
    abi.check(lib, lib.rt_context_set_scene(ctx, ctypes.byref(flat.abi)))

    from rt_mi355x import parallel
    tile = parallel.shard_range(W, H, world, rank)
    # Two shard buffers (and two gather targets on rank 0): frame k+1 renders into the other buffer while frame k's
    # RCCL gather is in flight (nccl: async gather on RCCL's own stream, waited only before frame k's assembly).
    # --overlap-gloo (rehearsal on one GPU, where RCCL cannot run two ranks): the same pipeline over gloo, each
    # rendered shard staged through a host buffer
    pipelined = world > 1 and ((backend == "nccl" and not args.no_overlap) or (backend == "gloo" and args.overlap_gloo))
    host_pipe = pipelined and backend != "nccl"
    shard = torch.zeros((parallel.rows_max(H, world), W, 3), dtype=torch.uint8, device="cuda")
    gathered = [torch.empty_like(shard) for _ in range(world)] if (world > 1 and rank == 0) else None
    image = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") if rank == 0 else None
    pev = [None]   # the step's events while a pipelined gather completes (ev[2]: after the wait)
    pimage = (image.cpu() if host_pipe else image) if rank == 0 else None
    pipe = parallel.PipelinedGather(lambda: torch.zeros_like(shard, device="cpu" if host_pipe else "cuda"), world, rank,
                                    H, pimage, after_wait=lambda: pev[0][2].record(stream) if pev[0] else None) \
        if pipelined else None
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    dynamic = args.schedule == "dynamic"
    n_chunks = min(args.chunks or 4 * world, H)   # every chunk holds at least one row (rt_render_async
    #                                               rejects an empty range)
    if dynamic:
        store = parallel.default_store() if dist_on else None
        frame = torch.zeros((H, W, 3), dtype=torch.uint8, device="cuda")
        cbufs = [torch.zeros((parallel.rows_max(H, n_chunks), W, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    # dynamic: this leg's claims on this rank, and the events around each chunk's launch (kernel time)
    sched = {"steps": 0, "chunks": 0, "pixels": 0, "kev": []}

    def step_dynamic(flags, ev=None):
        """One frame under the dynamic schedule: claim a chunk, launch it, keep at most two chunks queued
        on the GPU (the host claims the next one only once the one before the last has finished), write
        each into the zeroed frame, then one reduce (sum: every pixel is nonzero on one rank at most)."""
        key = f"rt-bench/{sched['steps']}"
        sched["steps"] += 1
        q = parallel.TileQueue(store, key, n_chunks) if store is not None else None
        frame.zero_()
        if ev:
            ev[0].record(stream)
        pend, k = [], 0
        kev = sched["kev"]
        while True:
            if q is not None:
                j = q.claim()
            else:   # one process: it takes every chunk in order
                j = k if k < n_chunks else None
            if j is None:
                break
            tr = parallel.chunk_range(W, H, n_chunks, j)
            buf = cbufs[k % 2]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            abi.check(lib, lib.rt_render_async(ctx, ctypes.byref(cam), depth, spp, args.seed, flags, ctypes.byref(tr),
                                               ctypes.c_void_p(buf.data_ptr()), None, sptr))
            e1.record(stream)
            kev.append((e0, e1))
            parallel.place_chunk(frame, buf, H, n_chunks, j)
            done = torch.cuda.Event()
            done.record(stream)
            pend.append(done)
            if len(pend) >= 2:
                pend.pop(0).synchronize()
            sched["chunks"] += 1
            sched["pixels"] += tr.row_count * W
            k += 1
        if ev:
            ev[1].record(stream)
        if world > 1:
            if backend == "nccl":
                dist.reduce(frame, dst=0, op=dist.ReduceOp.SUM)
            else:
                host = frame.cpu()
                dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
                if rank == 0:
                    frame.copy_(host)
        if ev:
            ev[2].record(stream)
        if rank == 0:
            image.copy_(frame)
        if ev:
            ev[3].record(stream)

    def flush():
        """Complete the pipelined frame still in flight (its gather, then rank 0's assembly)."""
        if pipe is not None:
            pev[0] = None
            pipe.flush()
            if host_pipe and rank == 0:
                image.copy_(pimage)

    def step(flags, ev=None, k=0):
        if dynamic:
            return step_dynamic(flags, ev)
        if ev:
            ev[0].record(stream)
        buf = pipe.buffer(k) if (pipe is not None and not host_pipe) else shard
        abi.check(lib, lib.rt_render_async(ctx, ctypes.byref(cam), depth, spp, args.seed, flags, ctypes.byref(tile),
                                           ctypes.c_void_p(buf.data_ptr()), None, sptr))
        if ev:
            ev[1].record(stream)
        if pipe is not None:
            if host_pipe:
                pipe.buffer(k).copy_(shard)   # synchronous staging (rehearsal only)
            # frame k's gather starts once its render is done (RCCL's stream waits for this one) and runs under frame
            # k+1's render; frame k-1's gather, issued under this render, is waited for and assembled now
            pev[0] = ev
            if pipe.submit(k) is None and ev:
                ev[2].record(stream)
            if ev:
                ev[3].record(stream)
            return
        if world > 1:
            if backend == "nccl":   # RCCL over xGMI, device buffers
                dist.gather(shard, gathered, dst=0)
            else:
                host = [g.cpu() for g in gathered] if rank == 0 else None
                dist.gather(shard.cpu(), host, dst=0)
                if rank == 0:
                    for g, h in zip(gathered, host):
                        g.copy_(h)
            if ev:
                ev[2].record(stream)
            if rank == 0:
                parallel.assemble_rows(gathered, H, world, image)
        else:
            if ev:
                ev[2].record(stream)
            if rank == 0:
                image.copy_(shard[:H])
        if ev:
            ev[3].record(stream)

    def leg(precision):
        """Warm-up, then exactly args.steps timed steps between barriers; max over ranks."""
        flags = abi.RT_FLAG_F32 if precision == "f32" else 0
        for i in range(args.warmup):
            step(flags, k=i)
        flush()
        torch.cuda.synchronize()
        abi.check(lib, lib.rt_context_collect(ctx, sptr, ctypes.byref(abi.RtStats())), allow=(abi.RT_ERR_RANGE,))
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
        sched["chunks"] = sched["pixels"] = 0
        sched["kev"] = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):
            step(flags, evs[k], k)
        flush()   # the last frame's gather and assembly are inside the timed region
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        st = abi.RtStats()
        rc = abi.check(lib, lib.rt_context_collect(ctx, sptr, ctypes.byref(st)), allow=(abi.RT_ERR_RANGE,))
        phase = [sum(e[i].elapsed_time(e[i + 1]) for e in evs) / args.steps for i in range(3)]   # ms per step
        if dynamic:
            # phase 0 spans the host's claims and its waits for the chunk two back (wall time on the
            # stream); the kernel time is the sum of the chunks' launches
            phase[0] = sum(a.elapsed_time(b) for a, b in sched["kev"]) / args.steps
        pix = sched["pixels"] / args.steps if dynamic else tile.row_count * W   # pixels this rank renders per step
        px_s = pix / (phase[0] / 1e3) if phase[0] > 0 else 0.0   # this rank's px/s (renderer.rs:339)
        mine = [elapsed, phase[0], phase[1], phase[2], float(st.ray_segments), px_s, pix, sched["chunks"] / args.steps]
        if world > 1:
            t = torch.tensor(mine, dtype=torch.float64, device=red_dev)
            allr = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(allr, t)
            per_rank = [a.cpu().tolist() for a in allr]
        else:
            per_rank = [mine]
        return st, rc, per_rank

    def summarize(precision, st, rc, per_rank):
        elapsed = max(r[0] for r in per_rank)
        samples = W * H * spp * args.steps
        launch_s = per_rank[rank][1] / 1e3   # this rank's average launch (render) duration
        f32, f64 = abi.executed_flop(st, precision)
        f32, f64 = f32 / args.steps, f64 / args.steps   # per launch
        t_peak = f32 / (PEAK_TF["f32"] * 1e12) + f64 / (PEAK_TF["f64"] * 1e12)   # seconds at peak
        segs_launch = st.ray_segments / args.steps
        bf = FLOP_PER_SPHERE_TEST * n_sph * segs_launch
        return {
            "value": samples / elapsed / 1e6,
            "ms_per_step": elapsed / args.steps * 1e3,
            "launch_ms": launch_s * 1e3,
            "roofline": {
                "bound": "valu",
                "achieved": (f32 + f64) / launch_s / 1e12,
                "peak": (f32 + f64) / t_peak / 1e12 if t_peak > 0 else PEAK_TF["f32"],
                "unit": "TFLOP/s",
                "frac": t_peak / launch_s,
                "executed_flop_per_launch": {"fp32": f32, "fp64": f64},
                "work_per_launch": {k: getattr(st, k) / args.steps for k in
                                    ("box_groups", "filter_groups", "exact_tests", "cone_tests", "camera_exact_tests")},
                "brute_force_equiv": {"flop_per_launch": bf, "tflops": bf / launch_s / 1e12,
                                      "x_fp32_peak": bf / launch_s / 1e12 / PEAK_TF["f32"]},
            },
            "ray_segments_per_sample": st.ray_segments / max(1.0, per_rank[rank][6] * spp * args.steps),
            "lane_utilisation": abi.lane_utilisation(st),
            "bounces_per_pixel": st.bounce_iters / max(1, st.pixels),
            "range_error": rc == abi.RT_ERR_RANGE,
            "per_rank": per_rank,
        }

    head = summarize(args.precision, *leg(args.precision))
    if rank == 0 and os.environ.get("RT_BENCH_SAVE"):   # the headline precision's frame
        np.save(os.environ["RT_BENCH_SAVE"], image.cpu().numpy())
    other = None
    if args.other_precision:
        op = "f64" if args.precision == "f32" else "f32"
        other = (op, summarize(op, *leg(op)))

    if rank == 0:
        pmc = {}
        try:
            with open(args.pmc) as f:
                pmc = json.load(f).get(f"{args.config}:{args.precision}:{world}", {})
        except (OSError, ValueError):
            pass
        rl = head["roofline"]
        rl.update(pmc_fields(pmc, vinfo["src_hash"], os.path.relpath(args.pmc, REPO)))
        rl["algorithmic_bytes"] = int(head["per_rank"][rank][6]) * 3 + flat.n_spheres * 20   # RGB8 out + the scene (SoA)
        rl["traffic_over_algorithmic"] = (rl["traffic"] / rl["algorithmic_bytes"]) if rl["traffic"] else None
        line = {
            "metric": "Msamples/s (pixels×spp/s), 1920×1080·512spp·500 spheres; 1/2/4/8 GPU",
            "value": round(head["value"], 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(head["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic",
            "config": {
                "workload": f"{args.config}: {W}x{H}, {n_sph} spheres (RTIOW-style, seed 0x5EED0001), "
                            f"{spp} spp, {depth} bounces, camera of src/main.rs:51-58",
                "width": W, "height": H, "spheres": n_sph, "spp": spp, "max_bounces": depth,
                "parallelism": (f"dynamic queue of {n_chunks} row-interleaved chunks over {world} rank(s)"
                                + ((" + RCCL reduce" if backend == "nccl" else f" + {backend} reduce (rehearsal)")
                                   if world > 1 else "")) if dynamic else
                               (f"row-interleaved image shards x{world}"
                                + (((" + RCCL gather, double-buffered under the next frame's render" if pipelined
                                     else " + RCCL gather") if backend == "nccl" else f" + {backend} gather (rehearsal)")
                                   if world > 1 else "")),
                "schedule": args.schedule,
            },
            "roofline": rl,
            "launch_ms": round(head["launch_ms"], 3),
            "ray_segments_per_sample": round(head["ray_segments_per_sample"], 5),
            "lane_utilisation": round(head["lane_utilisation"], 4),
            "bounces_per_pixel": round(head["bounces_per_pixel"], 3),
            "range_error": head["range_error"],
        }
        if other:
            op, o = other
            line[op] = {"value": round(o["value"], 3), "ms_per_step": round(o["ms_per_step"], 3),
                        "launch_ms": round(o["launch_ms"], 3), "roofline_frac": round(o["roofline"]["frac"], 4),
                        "achieved_tflops": round(o["roofline"]["achieved"], 3),
                        "brute_force_equiv_tflops": round(o["roofline"]["brute_force_equiv"]["tflops"], 3),
                        "range_error": o["range_error"]}
        rms = [p[1] for p in head["per_rank"]]
        line["dist"] = {
            "backend": (backend if dist_on else None), "world_size_initialised": world_init,
            "imbalance": round(max(rms) / (sum(rms) / len(rms)), 4) if sum(rms) > 0 else None,   # max / mean render
            "rccl_version": (".".join(map(str, torch.cuda.nccl.version())) if dist_on and backend == "nccl" else None),
            "per_rank": [{"rank": r, "wall_s": round(p[0], 4), "render_ms": round(p[1], 3), "gather_ms": round(p[2], 3),
                          "assemble_ms": round(p[3], 3), "ray_segments": int(p[4]), "px_per_s": round(p[5], 1),
                          "pixels": int(p[6]), "chunks": p[7] if dynamic else None}
                         for r, p in enumerate(head["per_rank"])],
        }
        line["build"] = {"library": vinfo["version"], "source_hash": src_hash,
                         "library_matches_source": vinfo["src_hash"] == src_hash}
        if world == 1 and args.cpu_seconds > 0:
            threads, host = cpu_share()
            threads = args.cpu_threads or threads
            line["cpu_baseline"] = cpu_baseline(flat, cam, depth, spp, args.seed, args.cpu_seconds, threads, host)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)

    lib.rt_context_destroy(ctx)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
