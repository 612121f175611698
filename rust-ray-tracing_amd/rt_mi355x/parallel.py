"""Image partition across GPUs (one process per GPU) and reassembly on rank 0.

The reference splits the image into 128x128 tiles pulled from an MPMC queue by worker threads
(src/renderer.rs:248-296).  Across GPUs we interleave rows instead (rank r renders rows
r, r+N, r+2N, ...): every rank gets a statistically identical mix of sky and geometry, so the
ranks finish together without a dynamic queue.  Pixels are independent and the RNG is keyed by
the global pixel index, so the assembled image is bit-identical for any N.
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
