"""Image partition across GPUs (one process per GPU) and reassembly on rank 0: a static row
interleave (the default) or a dynamic queue of row-interleaved chunks (below).

The reference splits the image into 128x128 tiles pulled from an MPMC queue by worker threads
(src/renderer.rs:248-296).  Across GPUs the default interleaves rows instead (rank r renders rows
r, r+N, r+2N, ...): every rank gets a statistically identical mix of sky and geometry, so equal
GPUs finish together with one launch each and no queue traffic.  The dynamic schedule keeps the
reference's pull model for unequal or shared GPUs.  Pixels are independent and the RNG is keyed
by the global pixel index, so the assembled image is bit-identical for any N and either schedule.
"""
from . import abi


def shard_rows(height, world, rank):
    """Rows owned by `rank`: range(rank, height, world)."""
    return range(rank, height, world)


def shard_range(width, height, world, rank):
    """rt_tile_range for `rank`'s shard (compact output of len(rows) x width pixels)."""
    rows = shard_rows(height, world, rank)
    return abi.RtTileRange(rank, world, len(rows), 0, width)


def rows_max(height, world):
    """Padded per-rank row count, so every rank sends an equal-sized buffer to the gather."""
    return (height + world - 1) // world


def assemble_rows(shards, height, world, out):
    """Scatter gathered shards back to image rows.  shards[r] is [rows_max, W, C] (padded);
    out is [H, W, C].  Works on numpy arrays and torch tensors alike."""
    for r in range(world):
        nr = len(shard_rows(height, world, r))
        out[r::world] = shards[r][:nr]
    return out


# ---- dynamic schedule: the reference's shared tile queue across GPUs ----------------------------
# TileRenderer::render (src/renderer.rs:243-296) sends every 128x128 block into an unbounded MPMC
# channel once and lets each worker thread pull the next block until the channel is empty, so a slow
# worker simply takes fewer blocks.  Across GPUs the queue is a counter in the process group's store
# (the TCPStore torch.distributed.run sets up): claim() is one atomic add.  A GPU needs far bigger
# work items than a CPU thread (one 128x128 block would leave most of its 6144 resident waves idle),
# so the items are chunks of row-interleaved rows -- chunk j of M is rows j, j+M, j+2M, ... at full
# width -- each a statistically identical 1/M of the frame.  Pixels are independent and the RNG is
# keyed by the global pixel index, so the image is bit-identical whoever renders which chunk.


def chunk_rows(height, n_chunks, j):
    """Rows of chunk j of n_chunks: range(j, height, n_chunks)."""
    return range(j, height, n_chunks)


def chunk_range(width, height, n_chunks, j):
    """rt_tile_range of chunk j (compact output of len(rows) x width pixels)."""
    return abi.RtTileRange(j, n_chunks, len(chunk_rows(height, n_chunks, j)), 0, width)


class TileQueue:
    """A shared work queue of n items over a torch.distributed store (the reference's task channel).

    Every rank builds one with the same key; claim() returns the next unclaimed item index, or None
    once all n are taken (the channel is empty, renderer.rs:281-284).  Each index is handed out
    exactly once across ranks: store.add is atomic on the store's server."""

    def __init__(self, store, key, n):
        self.store, self.key, self.n = store, key, int(n)
        self.claimed = []

    def claim(self):
        j = int(self.store.add(self.key, 1)) - 1
        if j >= self.n:
            return None
        self.claimed.append(j)
        return j


def default_store():
    """The process group's store (the TCPStore of torch.distributed.run's rendezvous)."""
    import torch.distributed.distributed_c10d as c10d
    return c10d._get_default_store()


def place_chunk(frame, chunk, height, n_chunks, j):
    """Write chunk j's compact rows into a full frame [H, W, C] (numpy or torch)."""
    nr = len(chunk_rows(height, n_chunks, j))
    frame[j::n_chunks] = chunk[:nr]
    return frame


# ---- pipelined gather: frame k+1 renders while frame k's shards travel -----------------------------
class PipelinedGather:
    """Double-buffered row-shard gather to rank 0 (bench.py's static schedule over RCCL).

    Frame k renders into buffer(k) (one of two shard buffers); submit(k) issues its gather asynchronously
    (torch.distributed, async_op=True: RCCL runs it on its own stream after the render it depends on, gloo
    in the background) and then completes frame k-1: waits for its gather -- with RCCL the current stream
    waits, the host does not block -- and assembles it into `image` on rank 0.  So frame k's gather overlaps
    frame k+1's render, and a buffer is rendered into again only after its previous gather completed.
    flush() completes the frame still in flight.  Returns of submit/flush: the frame index assembled, or None.
    The reference's renderer collects finished tiles on the main thread while workers keep rendering
    (src/renderer.rs:300-365); this is the same overlap across GPUs."""

    def __init__(self, make_buf, world, rank, height, image, after_wait=None):
        self.world, self.rank, self.height, self.image = world, rank, height, image
        self.bufs = [make_buf(), make_buf()]
        self.gath = [[make_buf() for _ in range(world)] if rank == 0 else None for _ in range(2)]
        self.after_wait = after_wait
        self.pend = None

    def buffer(self, k):
        return self.bufs[k % 2]

    def _finish(self, p):
        w, g, k = p
        w.wait()
        if self.after_wait:
            self.after_wait()
        if self.rank == 0:
            assemble_rows(g, self.height, self.world, self.image)
        return k

    def submit(self, k):
        import torch.distributed as dist
        g = self.gath[k % 2]
        w = dist.gather(self.bufs[k % 2], g if self.rank == 0 else None, dst=0, async_op=True)
        prev, self.pend = self.pend, (w, g, k)
        return self._finish(prev) if prev else None

    def flush(self):
        prev, self.pend = self.pend, None
        return self._finish(prev) if prev else None
