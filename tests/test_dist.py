"""Multi-process partition (the N>1 bench path) on CPU: gloo, world_size 2 and 3.

Each rank renders its row-interleaved shard (rt_mi355x.parallel.shard_range) -- here with the CPU
oracle standing in for the per-GPU kernel -- then shards are gathered to rank 0 exactly as bench.py
does over RCCL, and reassembled.  The image must be bit-identical to a single-process render.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, SPP, DEPTH, SEED = 24, 13, 8, 50, 0x5EED0001


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "rust-ray-tracing_amd"))
    sys.path.insert(0, here)
    import rt_mi355x as rt
    from rt_mi355x import parallel
    from oracle_bind import oracle_render
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    tr = parallel.shard_range(W, H, world, rank)
    rows = list(parallel.shard_rows(H, world, rank))
    pixels = np.array([r * W + c for r in rows for c in range(W)], np.uint32)
    rgb, lin, segs, rc = oracle_render(flat, cam, DEPTH, SPP, SEED, pixels=pixels, threads=2)
    assert tr.row_count == len(rows) and tr.row_step == world and tr.row_begin == rank
    shard = torch.zeros((parallel.rows_max(H, world), W, 3), dtype=torch.float64)
    shard[:len(rows)] = torch.from_numpy(lin.reshape(len(rows), W, 3))
    gathered = [torch.empty_like(shard) for _ in range(world)] if rank == 0 else None
    dist.gather(shard, gathered, dst=0)
    seg_t = torch.tensor([segs], dtype=torch.int64)
    dist.all_reduce(seg_t)
    if rank == 0:
        img = torch.empty((H, W, 3), dtype=torch.float64)
        parallel.assemble_rows(gathered, H, world, img)
        np.savez(out_path, img=img.numpy(), segs=int(seg_t.item()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_shards_gather_bit_identical(tmp_path, world):
    out = str(tmp_path / "img.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    import rt_mi355x as rt
    from oracle_bind import oracle_render
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    _, full, segs, _ = oracle_render(flat, cam, DEPTH, SPP, SEED)
    got = np.load(out)
    np.testing.assert_array_equal(got["img"], full.reshape(H, W, 3))
    assert int(got["segs"]) == segs


def test_partition_covers_every_row_once():
    from rt_mi355x import parallel
    for h in (1, 7, 1080, 2160):
        for world in (1, 2, 3, 4, 8):
            rows = sorted(r for k in range(world) for r in parallel.shard_rows(h, world, k))
            assert rows == list(range(h))
            assert max(len(parallel.shard_rows(h, world, k)) for k in range(world)) == parallel.rows_max(h, world)


def _dyn_worker(rank, world, port, out_path, n_chunks):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "rust-ray-tracing_amd"))
    sys.path.insert(0, here)
    import rt_mi355x as rt
    from rt_mi355x import parallel
    from oracle_bind import oracle_render
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    q = parallel.TileQueue(parallel.default_store(), "test-tiles/0", n_chunks)
    frame = np.zeros((H, W, 3), np.float64)
    segs_total = 0
    while (j := q.claim()) is not None:
        tr = parallel.chunk_range(W, H, n_chunks, j)
        rows = list(parallel.chunk_rows(H, n_chunks, j))
        assert tr.row_begin == j and tr.row_step == n_chunks and tr.row_count == len(rows)
        pixels = np.array([r * W + c for r in rows for c in range(W)], np.uint32)
        _, lin, segs, _ = oracle_render(flat, cam, DEPTH, SPP, SEED, pixels=pixels, threads=1)
        parallel.place_chunk(frame, lin.reshape(len(rows), W, 3), H, n_chunks, j)
        segs_total += segs
    t = torch.from_numpy(frame)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)   # each pixel is nonzero on one rank at most: x + 0 == x
    claimed = torch.zeros(n_chunks, dtype=torch.int64)
    for j in q.claimed:
        claimed[j] += 1
    dist.all_reduce(claimed)
    seg_t = torch.tensor([segs_total], dtype=torch.int64)
    dist.all_reduce(seg_t)
    if rank == 0:
        np.savez(out_path, img=t.numpy(), segs=int(seg_t.item()), claimed=claimed.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_chunks", [(2, 5), (3, 12)])
def test_dynamic_chunk_queue_bit_identical(tmp_path, world, n_chunks):
    """bench.py --schedule dynamic's partition: ranks pull row-interleaved chunks from the process
    group's store (the reference's shared tile channel, renderer.rs:248-296); every chunk is claimed
    exactly once and the reduced frame equals the single-process render bit for bit."""
    out = str(tmp_path / "img.npz")
    mp.spawn(_dyn_worker, args=(world, _free_port(), out, n_chunks), nprocs=world, join=True)
    import rt_mi355x as rt
    from oracle_bind import oracle_render
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    _, full, segs, _ = oracle_render(flat, cam, DEPTH, SPP, SEED)
    got = np.load(out)
    np.testing.assert_array_equal(got["claimed"], np.ones(n_chunks, np.int64))
    np.testing.assert_array_equal(got["img"], full.reshape(H, W, 3))
    assert int(got["segs"]) == segs


def test_chunks_cover_every_row_once():
    from rt_mi355x import parallel
    for h in (1, 7, 1080, 2160):
        for m in (1, 2, 5, 32):
            rows = sorted(r for j in range(m) for r in parallel.chunk_rows(h, m, j))
            assert rows == list(range(h))
            assert all(parallel.chunk_range(17, h, m, j).row_count == len(parallel.chunk_rows(h, m, j)) for j in range(m))


def _pipe_worker(rank, world, port, out_path, frames):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "rust-ray-tracing_amd"))
    sys.path.insert(0, here)
    import rt_mi355x as rt
    from rt_mi355x import parallel
    from oracle_bind import oracle_render
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    rows = list(parallel.shard_rows(H, world, rank))
    pixels = np.array([r * W + c for r in rows for c in range(W)], np.uint32)
    image = torch.zeros((H, W, 3), dtype=torch.float64) if rank == 0 else None
    pipe = parallel.PipelinedGather(lambda: torch.zeros((parallel.rows_max(H, world), W, 3), dtype=torch.float64),
                                    world, rank, H, image)
    got = {}
    for k in range(frames):   # frame k: seed SEED + k, rendered into the buffer frame k-2 used
        _, lin, _, _ = oracle_render(flat, cam, DEPTH, SPP, SEED + k, pixels=pixels, threads=1)
        buf = pipe.buffer(k)
        buf.zero_()
        buf[:len(rows)] = torch.from_numpy(lin.reshape(len(rows), W, 3))
        done = pipe.submit(k)
        assert done == (k - 1 if k > 0 else None)
        if rank == 0 and done is not None:
            got[done] = image.clone().numpy()
    done = pipe.flush()
    assert done == frames - 1 and pipe.flush() is None
    if rank == 0:
        got[done] = image.clone().numpy()
        np.savez(out_path, **{f"f{k}": v for k, v in got.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_pipelined_gather_frames_bit_identical(tmp_path, world):
    """bench.py's double-buffered gather (rt_mi355x.parallel.PipelinedGather): frame k renders while frame k-1's
    async gather completes; every assembled frame (a different seed per frame, so a buffer mix-up would show)
    equals the single-process render of that frame."""
    out = str(tmp_path / "frames.npz")
    frames = 4
    mp.spawn(_pipe_worker, args=(world, _free_port(), out, frames), nprocs=world, join=True)
    import rt_mi355x as rt
    from oracle_bind import oracle_render
    flat = rt.scenes.random_spheres(100).flatten()
    cam = rt.camera_new_py(W, H, **rt.MAIN_CAMERA)
    got = np.load(out)
    assert sorted(got.files) == [f"f{k}" for k in range(frames)]
    for k in range(frames):
        _, full, _, _ = oracle_render(flat, cam, DEPTH, SPP, SEED + k)
        np.testing.assert_array_equal(got[f"f{k}"], full.reshape(H, W, 3))
