"""Chunk sharding across GPUs.

Chunks are independent, so a batch of chunks is split into contiguous
chunk-index ranges, one per rank (one process per GPU); each rank encodes /
decodes its own range with the batched kernels and no data-path collective.
Only the timing uses collectives: a barrier before and after, and the max
over ranks of the elapsed time.
"""

from __future__ import annotations

__all__ = ["chunk_range", "aggregate_gibps"]


def chunk_range(nchunks: int, rank: int, world: int) -> "tuple[int, int]":
    """[lo, hi) of the chunks owned by `rank`: rank g gets
    [g*n/world, (g+1)*n/world) (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    if nchunks < 0:
        raise ValueError("nchunks must be >= 0")
    return nchunks * rank // world, nchunks * (rank + 1) // world


def aggregate_gibps(total_bytes: int, max_elapsed_s: float) -> float:
    """Whole-job throughput: bytes processed by all ranks / slowest rank."""
    return total_bytes / (1 << 30) / max_elapsed_s
