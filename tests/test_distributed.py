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


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launches_ranks_dry_run(world):
    """`bench.py --gpus N` with no launcher starts N rank processes itself
    (torch.distributed env set per child, gloo here: --dry-run touches no
    GPU); their contiguous ranges cover all 8192 C5 chunks exactly once and
    every rank round-trips a sample of its chunks through the oracle.  N = 8
    rehearses the driver's 8-GPU node: 8 distinct rank processes."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--dry-run",
                        "--cpu-seconds", "0.2", "--cpu-procs", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one line
    d = json.loads(lines[0])
    per = 8192 // world
    assert d["n_ranks"] == world and d["chunks"] == 8192 and d["covered_all"]
    assert [x["range"] for x in d["ranks"]] == [[k * per, (k + 1) * per] for k in range(world)]
    assert len({x["pid"] for x in d["ranks"]}) == world and os.getpid() not in {x["pid"] for x in d["ranks"]}
    assert all(x["ok"] for x in d["ranks"]) and d["max_over_ranks"] == float(world - 1)
    # the N-GPU record the GPU line carries, labelled as a rehearsal
    assert [x["rank"] for x in d["ranks"]] == list(range(world))
    assert all(x["device"] == "cpu" and x["elapsed_s"] > 0 for x in d["ranks"])
    assert d["rehearsal"] is True and d["physical_gpus"] == 0
    assert d["per_gpu_GiBps"] is None and d["frac_of_n_peak"] is None
    assert d["aggregate_GiBps"] > 0
    assert abs(d["per_rank_GiBps"] * world - d["aggregate_GiBps"]) <= 1e-5 * d["aggregate_GiBps"]
    # per-rank GPU-event times exist in the record (none on a CPU rehearsal)
    assert all("gpu_event_s" in x for x in d["ranks"])
    assert d["event_aggregate_GiBps"] is None and "host_minus_event_s" in d
    # the CPU baseline survives N > 1: timed by the launcher parent before
    # the ranks start, handed to rank 0
    cb = d["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] == "port"
    assert cb["parallel_cores"] == 2 and cb["parallel_value"] > 0


def test_bench_torchrun_rank0_times_cpu_baseline():
    """Under torch.distributed.run (WORLD_SIZE set, no launcher file) rank 0
    times the CPU legs itself before joining the process group."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--cpu-seconds", "0.2",
                        "--cpu-procs", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_ranks"] == 2 and d["cpu_baseline"] is not None and d["cpu_baseline"]["cores"] == 1


def test_scaling_fields_physical_gpus():
    """frac_of_n_peak divides by the PHYSICAL GPUs; ranks sharing one device
    are a rehearsal."""
    import bench

    GiB = 1 << 30
    mk = lambda r, pci: {"rank": r, "host": "h", "pci": pci}  # noqa: E731
    four = [mk(r, f"0000:{r:02x}:00") for r in range(4)]
    f = bench.scaling_fields(four, 8e12, 4 * GiB, 1.0, on_gpu=True)
    assert f["physical_gpus"] == 4 and f["rehearsal"] is False
    assert f["aggregate_GiBps"] == 16.0 and f["per_gpu_GiBps"] == 4.0 and f["per_rank_GiBps"] == 4.0
    assert f["frac_of_n_peak"] == 1.0  # 4 x 8e12 B in 1 s over 4 x 8 TB/s
    assert f["event_aggregate_GiBps"] is None  # no per-rank event times given
    timed = [dict(mk(r, f"0000:{r:02x}:00"), gpu_event_s=0.5 + 0.1 * r) for r in range(4)]
    f2 = bench.scaling_fields(timed, 8e12, 4 * GiB, 1.0, on_gpu=True)
    assert f2["event_t_max_s"] == 0.8 and f2["event_aggregate_GiBps"] == 20.0
    assert abs(f2["host_minus_event_s"] - 0.2) < 1e-9
    shared = [mk(r, "0000:03:00") for r in range(2)]
    g = bench.scaling_fields(shared, 8e12, GiB, 2.0, on_gpu=True)
    assert g["physical_gpus"] == 1 and g["rehearsal"] is True
    assert g["aggregate_GiBps"] == 1.0 and g["per_gpu_GiBps"] == 1.0 and g["frac_of_n_peak"] == 1.0


def test_visible_gpu_count_without_hip(monkeypatch):
    """The launcher parent counts GPUs from the visibility variables (or the
    KFD topology), never through torch.cuda / HIP."""
    import bench

    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    assert bench.visible_gpu_count() == (8, "ROCR_VISIBLE_DEVICES")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,3")
    assert bench.visible_gpu_count() == (2, "HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    n, src = bench.visible_gpu_count()
    assert src.startswith("/sys/class/kfd") and n >= 0
    # and the parent never asks torch.cuda
    monkeypatch.setattr(torch.cuda, "device_count", lambda: (_ for _ in ()).throw(AssertionError("HIP call")))
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.launch_ranks(2, dry_run=False)


def test_bench_world_size_mismatch_fails_loudly():
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=root)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
