"""The N>1 path on CPU: world_size-2 gloo process group exercising the same
helpers bench.py uses on the GPU node (barrier, max over ranks, aggregate
throughput) and the chunk partition of numcodecs_amd.shard (disjoint,
covering, balanced).  No data-path collective exists to test: chunks are
independent."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from numcodecs_amd.shard import aggregate_gibps, chunk_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, nchunks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = chunk_range(nchunks, rank, world)
        ranges = [None] * world
        dist.all_gather_object(ranges, (lo, hi))
        bench.barrier(dist)
        mx = bench.max_over_ranks(dist, float(rank + 1) * 0.5)
        q.put((rank, ranges, mx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nchunks", [8192, 7, 1])
def test_gloo_world2_partition_and_timing(nchunks):
    if torch.cuda.is_available():
        pytest.skip("CPU gloo test")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nchunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, ranges, mx in res:
        assert mx == 1.0  # max over ranks of (0.5, 1.0)
        covered = []
        for lo, hi in ranges:
            covered.extend(range(lo, hi))
        assert covered == list(range(nchunks))
        sizes = [hi - lo for lo, hi in ranges]
        assert max(sizes) - min(sizes) <= 1


def test_chunk_range_and_aggregate():
    assert chunk_range(8192, 0, 8) == (0, 1024)
    assert chunk_range(8192, 7, 8) == (7168, 8192)
    with pytest.raises(ValueError):
        chunk_range(10, 2, 2)
    assert aggregate_gibps(8 * (1 << 30), 2.0) == 4.0
