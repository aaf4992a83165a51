"""Benchmark: Shuffle(4) encode+decode of device-resident 256 MiB fp32 chunks,
plus every other BASELINE.json configuration with its CPU baseline.

Metric (BASELINE.json): "GiB/s encode+decode per GPU, device-resident fp32
chunks (Shuffle, BitRound)", quoted on configs[1]: Shuffle(elementsize=4) on
a 256 MiB float32 chunk per GPU.  One step = Shuffle(4).encode +
Shuffle(4).decode of one chunk (4 rotating buffer sets per GPU so that the
256 MiB Infinity Cache cannot serve a step from the previous one).
value = (bytes into encode + bytes into decode) over all ranks / time of the
slowest rank -- the whole-job aggregate the driver contract asks for; the line
also carries per_gpu_GiBps (= value / physical GPUs, the metric's "per GPU"),
aggregate_GiBps, frac_of_n_peak (HBM reads + writes / (physical GPUs x
8 TB/s)), `ranks` (rank, local rank, host, pid, device, PCI location, UUID,
elapsed) and `rehearsal` (true when ranks share a physical GPU).

    python bench.py [--gpus N --steps K --warmup W] [--no-cpu] [--quick]

--gpus N > 1 without a launcher: bench.py starts N rank processes itself
(before anything touches the GPU), one per GPU (LOCAL_RANK = rank), with the
torch.distributed env set; under torch.distributed.run WORLD_SIZE must equal
N.  Chunks are independent, so ranks share no data: the only collectives are
the timing barrier and the max-over-ranks of the elapsed time.

Printed (rank 0): ONE JSON line with the contract's keys plus
  roofline      the Shuffle(4) encode/decode kernels (2 x 256 MiB of
                algorithmic bytes per launch each) / their mean launch
                duration (a HIP event pair on the launch stream bracketing
                the timed region); peak 8 TB/s; `traffic` = HBM bytes per
                launch from the rocprofv3 PMC summary under profiles/;
  cpu_baseline  the build's own scalar C restatement (oracle/ncoracle.c,
                kind "port") of _shuffle.pyx:11-30 on 1 host core and on P
                processes, bounded sample of the same workload;
  cfg_*         (N = 1) every other BASELINE config on this GPU -- C1, C2 f64,
                C3, C4, C5 on one GPU, a small host->host run -- each with
                GiB/s, the fraction of HBM peak of its kernels (algorithmic
                bytes / event-timed duration) and its CPU baseline at 1 and P
                processes (the same restatement);
  c5_sharded    configs[4]: 8192 x 1 MiB chunks, Shuffle(4) + Fletcher32,
                split over the N ranks by contiguous chunk ranges (strong
                scaling), frac of N x 8 TB/s; the timed decode includes the
                per-step checksum verdict (device compare + one readback).
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MiB = 1 << 20
GiB = 1 << 30
CHUNK = 256 * MiB
PEAK_GBPS = 8000.0  # MI355X HBM3E peak, 8.0 TB/s (MI355X_MICROARCH.md)
METRIC = "GiB/s encode+decode per GPU, device-resident fp32 chunks (Shuffle, BitRound)"


# ---------------------------------------------------------------------------
# ranks
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_count() -> "tuple[int, str]":
    """GPUs a child rank will see, counted WITHOUT any HIP or torch.cuda call
    in this process (the launcher parent must not initialise the GPU before it
    starts the ranks).  The visibility variables win (HIP_VISIBLE_DEVICES
    indexes into ROCR_VISIBLE_DEVICES' set, so the first one set decides);
    otherwise the KFD topology: every node with a nonzero gfx_target_version
    is a GPU.  Returns (count, source)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip():
            return len([x for x in v.split(",") if x.strip()]), var
    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(p) as f:
                for line in f:
                    key, _, val = line.partition(" ")
                    if key == "gfx_target_version" and int(val) != 0:
                        n += 1
        except (OSError, ValueError):
            continue
    return n, "/sys/class/kfd/kfd/topology"


def launch_ranks(n: int, dry_run: bool, extra_env: "dict | None" = None) -> int:
    """Start n rank processes of this script (one per GPU) and wait for them.

    Runs in the parent, which never touches the GPU: devices are counted from
    the visibility variables / KFD topology (visible_gpu_count), not through
    torch.cuda or HIP.  Children get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    as torch.distributed.run would set them.  If a rank fails, the others are
    stopped (they would wait at a barrier forever)."""
    gloo = dry_run or os.environ.get("MCODEC_BENCH_BACKEND") == "gloo"
    if not gloo:
        ndev, src = visible_gpu_count()
        if ndev < n:
            raise SystemExit(f"bench.py --gpus {n}: only {ndev} GPU(s) visible (counted from {src}; "
                             "MCODEC_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MCODEC_BENCH_CHILD="1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [None] * n
    failed_at = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0) and failed_at is None:
                    failed_at = time.time()
        if failed_at is not None and time.time() - failed_at > 30:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.kill()
                    rcs[i] = p.wait()
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return (abs(bad[0]) or 1) if bad else 0


def dist_setup(dry_run: bool):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # RCCL ("nccl") on the GPU node; MCODEC_BENCH_BACKEND=gloo rehearses
        # several ranks on one GPU (device = LOCAL_RANK mod visible devices)
        backend = "gloo" if dry_run else (
            os.environ.get("MCODEC_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo"))
        if not dry_run and torch.cuda.is_available():
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        return dist, rank, world, local
    return None, 0, 1, 0


def barrier(dist):
    if dist is not None:
        if torch.cuda.is_available() and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def max_over_ranks(dist, value: float) -> float:
    if dist is None:
        return value
    on_gpu = torch.cuda.is_available() and dist.get_backend() == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rank_identity(rank: int, local: int, dev) -> dict:
    """Who this rank is and which physical device it drives: the PCI location
    and UUID of the GPU (or "cpu" in a --dry-run rehearsal)."""
    d = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "pid": os.getpid()}
    if dev is None:
        d.update(device="cpu", pci="cpu")
    else:
        p = torch.cuda.get_device_properties(dev)
        d.update(device=f"cuda:{dev.index}", name=p.name,
                 pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
                 uuid=str(getattr(p, "uuid", "")))
    return d


def gather_ranks(dist, mine: dict) -> list:
    if dist is None:
        return [mine]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, mine)
    return out


def scaling_fields(ranks: list, alg_bytes_per_rank: float, counted_bytes_per_rank: float, t_max: float,
                   on_gpu: bool) -> dict:
    """The N-GPU record of one timed workload (north_star: "throughput at
    1/2/4/8 GPUs as absolute GiB/s and as fraction of the aggregate HBM
    roofline").  `counted_bytes_per_rank` are the metric's bytes (bytes into
    encode + decode), `alg_bytes_per_rank` the HBM algorithmic bytes (read +
    write of every launch) each rank moved in the timed region; `t_max` is the
    slowest rank's elapsed time.  Distinct (host, PCI location) pairs are the
    physical GPUs: ranks sharing one (a gloo rehearsal on a one-GPU box) or a
    CPU --dry-run are labelled `rehearsal`, and the roofline is N_physical x
    8 TB/s."""
    world = len(ranks)
    phys = len({(r["host"], r["pci"]) for r in ranks}) if on_gpu else 0
    agg = world * counted_bytes_per_rank / GiB / t_max
    sig = lambda x: float(f"{x:.6g}")  # noqa: E731  (6 significant digits: rehearsal rates are tiny)
    # the same bytes over the slowest rank's GPU-event time (a HIP event pair
    # on its launch stream around its timed steps): the host wall time above
    # also holds the trailing barrier and synchronize, so the gap between the
    # two is barrier skew + launch latency, visible at N = 8
    ev = [r.get("gpu_event_s") for r in ranks]
    ev_max = max(ev) if ev and all(e for e in ev) else None
    return {
        "aggregate_GiBps": sig(agg),
        "per_gpu_GiBps": sig(agg / phys) if phys else None,
        "per_rank_GiBps": sig(agg / world),
        "event_aggregate_GiBps": sig(world * counted_bytes_per_rank / GiB / ev_max) if ev_max else None,
        "event_t_max_s": round(ev_max, 6) if ev_max else None,
        "host_minus_event_s": round(t_max - ev_max, 6) if ev_max else None,
        "n_ranks": world,
        "physical_gpus": phys,
        "rehearsal": (not on_gpu) or phys < world,
        "frac_of_n_peak": round(world * alg_bytes_per_rank / t_max / 1e9 / (phys * PEAK_GBPS), 4) if phys else None,
        "ranks": ranks,
    }


def load_cpu(path: "str | None") -> "dict | None":
    """The CPU baselines the launcher parent timed (MCODEC_BENCH_CPU_JSON)."""
    if not path:
        return None
    with open(path) as f:
        return json.load(f)


def headline_cpu(cpu: "dict | None") -> "dict | None":
    """The line's cpu_baseline: the C2 f32 restatement timed on this box."""
    if not cpu or "C2_f32" not in cpu:
        return None
    c2 = dict(cpu["C2_f32"])
    c2["sample"] = "Shuffle(4) enc+dec: " + c2["sample"]
    return c2


def dry_run(dist, rank: int, world: int, nchunks: int, cpu: "dict | None" = None) -> None:
    """CPU rehearsal of the sharded run (tests/test_distributed.py): every
    rank takes its contiguous C5 chunk range and encodes + verify-decodes a
    sample of its chunks with the oracle, timed between barriers like the GPU
    run; rank 0 prints the same rank / scaling record the GPU line carries,
    labelled a rehearsal.  No GPU is touched."""
    from numcodecs_amd import shard
    from oracle import nporacle as npo

    lo, hi = shard.chunk_range(nchunks, rank, world)
    sample = sorted({lo, (lo + hi) // 2, hi - 1}) if hi > lo else []
    barrier(dist)
    t0 = time.perf_counter()
    ok = True
    for c in sample:
        x = np.random.default_rng(1000 + c).integers(0, 256, 4096, dtype=np.uint8)
        enc = npo.fletcher32_encode(npo.shuffle(x, 4))
        ok &= np.array_equal(npo.unshuffle(npo.fletcher32_decode(enc), 4), x)
    elapsed = time.perf_counter() - t0
    barrier(dist)
    mine = rank_identity(rank, rank, None)
    mine.update(range=[lo, hi], ok=bool(ok), elapsed_s=elapsed, gpu_event_s=None)
    info = gather_ranks(dist, mine)
    t = max_over_ranks(dist, float(rank))
    t_max = max(i["elapsed_s"] for i in info) or 1e-9
    if rank == 0:
        covered = sorted(c for i in info for c in range(*i["range"]))
        line = {"dry_run": True, "max_over_ranks": t, "chunks": nchunks,
                "covered_all": covered == list(range(nchunks)), "cpu_baseline": headline_cpu(cpu)}
        line.update(scaling_fields(info, 2 * 2 * 4096 * 3, 2 * 4096 * 3, t_max, on_gpu=False))
        print(json.dumps(line), flush=True)


# ---------------------------------------------------------------------------
# CPU baselines (the build's restatement; before the GPU is initialised)
# ---------------------------------------------------------------------------
CPU_CONFIGS = {  # config -> (single-core bytes, per-process bytes of the parallel leg)
    "C1": (MiB, MiB),
    "C2_f32": (CHUNK, 32 * MiB),
    "C2_f64": (CHUNK, 32 * MiB),
    "C3": (CHUNK, 32 * MiB),
    "C4": (CHUNK, 32 * MiB),
    "C5": (128 * MiB, 32 * MiB),
}


# the CPU legs an N > 1 run keeps (the headline's C2 f32 and the sharded C5)
CPU_CONFIGS_MULTI = ("C2_f32", "C5")


def cpu_baselines(procs: int, seconds: float, only=None) -> dict:
    from oracle import cpu_baseline as cb

    out = {}
    for cfg, (n1, npar) in CPU_CONFIGS.items():
        if only is not None and cfg not in only:
            continue
        one = cb.single_core(cfg, n1, seconds)
        if procs > 1:
            par = cb.parallel(cfg, procs, npar, seconds)
            one["parallel_value"] = par["value"]
            one["parallel_cores"] = par["cores"]
            one["parallel_sample"] = par["sample"]
        out[cfg] = one
    return out


def _cpu_fields(cpu: "dict | None", cfg: str) -> dict:
    """Flat cpu_* fields of a cfg_* object."""
    c = (cpu or {}).get(cfg)
    if not c:
        return {"cpu_1core_GiBps": None}
    return {"cpu_1core_GiBps": c["value"], "cpu_par_GiBps": c.get("parallel_value"),
            "cpu_par_cores": c.get("parallel_cores"), "cpu_kind": c["kind"]}


# ---------------------------------------------------------------------------
# GPU timing
# ---------------------------------------------------------------------------
def pmc_traffic():
    """HBM bytes per encode launch from the newest profiles/*/pmc_summary.json
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, per launch)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    ks = [d.get("kernels", {}).get(n) for n in ("shuffle_enc", "shuffle_dec")]
    vals = [k.get("hbm_bytes_per_launch") for k in ks if k and k.get("hbm_bytes_per_launch")]
    if not vals:
        return None, None
    return int(sum(vals) / len(vals)), os.path.relpath(files[-1], ROOT)


# the headline kernels as rocprofv3 names them (dispatch defaults for one
# 256 MiB chunk, numcodecs_amd/csrc/mc_shuffle.hip default_variant)
HEADLINE_KERNELS = {"encode": "k_shuffle_enc<4, false, false, false, true, 8>", "decode": "k_shuffle4_dec_pair<true, 2>"}


def trace_roofline():
    """The headline kernels' rocprof averages from the newest
    profiles/*/kernel_stats_headline.csv (the bench under rocprofv3 --stats,
    committed with the round): algorithmic bytes per launch (2 x 256 MiB) /
    average duration / peak, per kernel and for the dominant (slower) one --
    the figure a reader can tie to profiles/, beside this run's event-timed
    `frac` (a different box and run: the two agree within the box spread)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "kernel_stats_headline.csv")))
    if not files:
        return None
    avg = {}
    with open(files[-1]) as f:
        for row in csv.DictReader(f):
            for role, name in HEADLINE_KERNELS.items():
                if name in row["Name"]:
                    avg[role] = float(row["AverageNs"]) * 1e-9
    if len(avg) != 2:
        return None
    per = {role: {"kernel": HEADLINE_KERNELS[role], "avg_us": round(t * 1e6, 2),
                  "frac": round(2 * CHUNK / t / 1e9 / PEAK_GBPS, 4)} for role, t in avg.items()}
    dom = max(per, key=lambda r: avg[r])
    return {"trace_frac": per[dom]["frac"], "trace_kernel": per[dom]["kernel"],
            "trace_file": os.path.relpath(files[-1], ROOT), "trace_kernels": per}


def run_step_timing(args, dev, dist, rank):
    from numcodecs_amd import Shuffle

    codec = Shuffle(4)
    sets = 4
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    ins = [torch.randn(CHUNK // 4, generator=g, device=dev, dtype=torch.float32) for _ in range(sets)]
    encs = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    decs = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    # parity gate before timing: decode(encode(x)) == x on every set
    for i in range(sets):
        codec.encode(ins[i], out=encs[i])
        codec.decode(encs[i], out=decs[i])
        assert torch.equal(decs[i].view(torch.float32), ins[i]), "round trip failed"

    def step(i):
        codec.encode(ins[i % sets], out=encs[i % sets])
        codec.decode(encs[i % sets], out=decs[i % sets])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    # One HIP event pair on the launch stream (torch's current stream) brackets
    # the timed region: per-launch event records would each idle the GPU for
    # ~5 us on ROCm, so the mean launch duration is GPU time / launches (encode
    # and decode move the same 2 x 256 MiB each; rocprofv3 per-kernel averages
    # are in profiles/).
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    ev1.record()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    gpu_ms = ev0.elapsed_time(ev1)
    del ins, encs, decs
    return elapsed, gpu_ms / (2 * args.steps), gpu_ms * 1e-3


def run_c5_sharded(steps, warmup, nchunks, dev, dist, rank, world):
    """configs[4]: nchunks x 1 MiB fp32 chunks, Shuffle(4) + Fletcher32 fused,
    split over ranks by contiguous chunk ranges (shard.chunk_range, no
    collective); one step = encode + verified decode of the rank's chunks:
    the decode's per-chunk (computed, stored) checksum pairs are compared on
    the device and the verdict is read back to the host (one readback per
    step, raising the reference's RuntimeError on a mismatch) INSIDE the
    timed region.  Returns (this rank's elapsed_s, mean launch ms, local
    chunks, GPU-event seconds of the timed steps)."""
    from numcodecs_amd import batch, shard

    lo, hi = shard.chunk_range(nchunks, rank, world)
    b = hi - lo
    g = torch.Generator(device=dev).manual_seed(1000 + lo)
    x = torch.randn((b, MiB // 4), generator=g, device=dev, dtype=torch.float32)
    enc = batch.shuffle_fletcher32_encode_chunks(x, 4)
    dec = torch.empty((b, MiB), dtype=torch.uint8, device=dev)
    batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4, out=dec, check_sums=True)
    assert torch.equal(dec.view(torch.float32), x), "C5 round trip failed"

    def step():
        batch.shuffle_fletcher32_encode_chunks(x, 4, out=enc)
        batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4, out=dec, check_sums=True)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    assert torch.equal(dec.view(torch.float32), x), "C5 round trip failed after timing"
    gpu_ms = ev0.elapsed_time(ev1)
    launch_ms = gpu_ms / (2 * steps)
    del x, enc, dec
    torch.cuda.empty_cache()
    return elapsed, launch_ms, b, gpu_ms * 1e-3


def _timed(fn, sets, reps):
    """Mean seconds per call of fn(i % sets) between HIP events on the launch
    stream, after one warm call per set (every call rotates over `sets`
    buffer sets, so none finds its input left in the Infinity Cache)."""
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % sets)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def _cfg(gibps, t_enc, t_dec, alg_bytes, kernels, cpu, cfg, note=None):
    achieved = alg_bytes / (t_enc + t_dec) / 1e9
    d = {"GiBps": round(gibps, 1), "enc_us": round(t_enc * 1e6, 1), "dec_us": round(t_dec * 1e6, 1),
         "kernel_GBps": round(achieved, 1), "frac": round(achieved / PEAK_GBPS, 4), "kernels": kernels}
    if note:
        d["note"] = note
    d.update(_cpu_fields(cpu, cfg))
    if d.get("cpu_1core_GiBps"):
        d["gpu_over_cpu_1core"] = round(gibps / d["cpu_1core_GiBps"], 1)
    return d


def config_workloads(dev, cpu, sets: int = 4) -> dict:
    """BASELINE.json configs other than the headline, on this GPU, through the
    public codec API (device tensors in, device tensors out)."""
    from numcodecs_amd import BitRound, Delta, FixedScaleOffset, Shuffle, batch

    out = {}
    # C1: one 1 MiB chunk per call (launch-bound: a codec call costs more than
    # the 0.3 us of HBM time); plus the same chunks batched 256 per launch
    x1 = [torch.randn(MiB // 4, device=dev) for _ in range(sets)]
    e1 = [torch.empty(MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    d1 = [torch.empty(MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    sh4 = Shuffle(4)
    t_e = _timed(lambda i: sh4.encode(x1[i], out=e1[i]), sets, 200)
    t_d = _timed(lambda i: sh4.decode(e1[i], out=d1[i]), sets, 200)
    out["cfg_C1"] = _cfg(2 * MiB / GiB / (t_e + t_d), t_e, t_d, 4 * MiB, "k_shuffle_enc<4> / k_shuffle_dec<4>",
                         cpu, "C1", "one 1 MiB chunk per codec call: launch/host-bound, not HBM-bound")
    del x1, e1, d1
    # the same 1 MiB chunks as a Zarr pipeline hands them over: 256 per batched call
    rows = 256
    xb = [torch.randn(rows, MiB // 4, device=dev) for _ in range(sets)]
    eb = [torch.empty(rows, MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    db = [torch.empty(rows, MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    t_be = _timed(lambda i: batch.shuffle_chunks(xb[i], 4, out=eb[i]), sets, 50)
    t_bd = _timed(lambda i: batch.unshuffle_chunks(eb[i], 4, out=db[i]), sets, 50)
    assert torch.equal(db[0].view(torch.float32), xb[0])
    out["cfg_C1"]["batched_256"] = {
        "GiBps": round(2 * rows * MiB / GiB / (t_be + t_bd), 1), "enc_us": round(t_be * 1e6, 1),
        "dec_us": round(t_bd * 1e6, 1), "frac": round(4 * rows * MiB / (t_be + t_bd) / 1e9 / PEAK_GBPS, 4),
        "note": "256 x 1 MiB chunks per batched call (numcodecs_amd.batch.shuffle_chunks / unshuffle_chunks)"}
    del xb, eb, db
    # C2 f64 Shuffle(8)
    sh8 = Shuffle(8)
    x64 = [torch.randn(CHUNK // 8, device=dev, dtype=torch.float64) for _ in range(sets)]
    e64 = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    d64 = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    t_e = _timed(lambda i: sh8.encode(x64[i], out=e64[i]), sets, 20)
    t_d = _timed(lambda i: sh8.decode(e64[i], out=d64[i]), sets, 20)
    assert torch.equal(d64[0].view(torch.float64), x64[0])
    out["cfg_C2_f64"] = _cfg(2 * CHUNK / GiB / (t_e + t_d), t_e, t_d, 4 * CHUNK,
                             "k_shuffle8_enc_pair / k_shuffle8_dec_pair", cpu, "C2_f64")
    del x64, e64, d64
    # C3 BitRound(10) fused with Shuffle(4); decode = unshuffle (+ re-view)
    x32 = [torch.randn(CHUNK // 4, device=dev) for _ in range(sets)]
    pipe = batch.FilterPipeline([BitRound(10), Shuffle(4)])
    enc = [pipe.encode(x) for x in x32]
    dec = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    t_e = _timed(lambda i: pipe.encode(x32[i]), sets, 20)
    t_d = _timed(lambda i: sh4.decode(enc[i], out=dec[i]), sets, 20)
    out["cfg_C3"] = _cfg(2 * CHUNK / GiB / (t_e + t_d), t_e, t_d, 4 * CHUNK,
                         "k_bitround_shuffle4_planes / k_shuffle4_dec_pair", cpu, "C3")
    del x32, enc, dec
    # C4 FSO(f4->i2) -> Delta(i2) -> Shuffle(2), fused kernels
    xc = [1000.0 + 10.0 * torch.rand(CHUNK // 4, device=dev) for _ in range(sets)]
    c4 = batch.FilterPipeline([FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
                               Delta(dtype="<i2"), Shuffle(2)])
    e = [c4.encode(x) for x in xc]
    t_e = _timed(lambda i: c4.encode(xc[i]), sets, 20)
    t_d = _timed(lambda i: c4.decode(e[i]), sets, 20)
    # 1.5 N algorithmic bytes each way (4 B in + 2 B out per element and back)
    out["cfg_C4"] = _cfg(2 * CHUNK / GiB / (t_e + t_d), t_e, t_d, 3 * CHUNK,
                         "k_c4_enc / c4 decode (reduce, sums, apply)", cpu, "C4")
    del xc, e
    torch.cuda.empty_cache()
    # C5 on one GPU: 8192 x 1 MiB, fused Shuffle(4) + Fletcher32 (8 GiB per call)
    nb = 8192
    xb = torch.randn((nb, MiB // 4), device=dev)
    eb = batch.shuffle_fletcher32_encode_chunks(xb, 4)
    db = torch.empty((nb, MiB), dtype=torch.uint8, device=dev)
    t_e = _timed(lambda i: batch.shuffle_fletcher32_encode_chunks(xb, 4, out=eb), 1, 5)
    t_d = _timed(lambda i: batch.fletcher32_unshuffle_decode_chunks(eb, MiB, 4, out=db, check_sums=True), 1, 5)
    assert torch.equal(db.view(torch.float32), xb)
    out["cfg_C5"] = _cfg(2 * nb * MiB / GiB / (t_e + t_d), t_e, t_d, 2 * nb * (2 * MiB + 4),
                         "k_shuffle_f32_enc / k_f32_unshuffle", cpu, "C5",
                         "decode = fused verify + unshuffle, the per-chunk verdict compared on the device and "
                         "read back inside every timed call")
    del xb, eb, db
    torch.cuda.empty_cache()
    return out


def pcie_rates(dev, nbytes: int = GiB) -> dict:
    """Pinned host <-> device copy rates of this box: H2D alone, D2H alone and
    both directions at once on two streams (the bound of a host->host codec
    path, which moves every byte in and out)."""
    h_in = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    h_out = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_out = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            best = t if best is None else min(best, t)
        return best

    def duplex():
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    t_h2d = timed(lambda: d_in.copy_(h_in, non_blocking=True))
    t_d2h = timed(lambda: h_out.copy_(d_out, non_blocking=True))
    t_dup = timed(duplex)
    del h_in, h_out, d_in, d_out
    g = nbytes / GiB
    return {"pcie_h2d_GiBps": round(g / t_h2d, 2), "pcie_d2h_GiBps": round(g / t_d2h, 2),
            "pcie_duplex_GiBps_each_way": round(g / t_dup, 2)}


def end_to_end(dev, cpu, total_gib: int = 1, chunk_bytes: int = 4 * MiB) -> dict:
    """Host -> host rate: pinned H2D + Shuffle(4) kernel + D2H, pipelined over
    H2D / kernel / D2H role streams (batch.host_pipeline).  PCIe-bound: the
    line carries the box's concurrent H2D + D2H rate (pcie_rates), the bound
    of any host->host codec, and the fraction of it reached."""
    from numcodecs_amd import batch

    nchunks = total_gib * GiB // chunk_bytes
    hin = torch.randint(0, 256, (nchunks, chunk_bytes), dtype=torch.uint8).pin_memory()
    henc = torch.empty_like(hin).pin_memory()
    hdec = torch.empty_like(hin).pin_memory()
    batch.host_pipeline(hin, henc, 4, True, slice_chunks=16)
    te = td = None
    for _ in range(3):  # best of three: the host side of the pipeline is noisy
        t0 = time.perf_counter()
        batch.host_pipeline(hin, henc, 4, True, slice_chunks=16)
        t = time.perf_counter() - t0
        te = t if te is None else min(te, t)
        t0 = time.perf_counter()
        batch.host_pipeline(henc, hdec, 4, False, slice_chunks=16)
        t = time.perf_counter() - t0
        td = t if td is None else min(td, t)
    assert torch.equal(hdec, hin)
    del hin, henc, hdec
    res = {"GiBps": round(2 * total_gib / (te + td), 2), "enc_GiBps": round(total_gib / te, 2),
           "dec_GiBps": round(total_gib / td, 2),
           "workload": f"{total_gib} GiB of {chunk_bytes // MiB} MiB chunks, pinned host in/out, Shuffle(4), "
                       "best of 3"}
    res.update(pcie_rates(dev))
    res["frac_of_duplex"] = round(res["GiBps"] / res["pcie_duplex_GiBps_each_way"], 4)
    res.update(_cpu_fields(cpu, "C2_f32"))
    return res


def copy_ceiling(dev, nbytes: int = GiB, reps: int = 10) -> dict:
    """SURVEY §8d's "achievable" line, measured in this run: hipMemcpyAsync
    DtoD (torch's copy_) and libmcodec's nontemporal copy kernel (mc_copy) on
    1 GiB, and the copy calibration of tools/lab/lab_bw.hip (libmcodec_bwcal.so; plain 16-B/lane
    copies, nontemporal loads + stores, the layouts that stream fastest:
    8 vectors per thread one tile per workgroup, 4 per thread on a
    8192-workgroup grid) on 1 GiB and on 4 rotating 256 MiB sets -- the
    headline's working set.  GB/s = read + write bytes / median time;
    ceiling_GBps = the best of them."""
    from numcodecs_amd import _ops

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    st = torch.cuda.current_stream(dev).cuda_stream

    def rate(fn, nb, sets=1, groups=3):
        # back-to-back launches between one event pair, as the headline's
        # mean_launch_ms is measured (round 4: one launch per event pair
        # added the launch ramp and drain to every sample, ~3-5 % of an
        # 85 us copy, and put the ceiling below the kernels it bounds)
        for i in range(sets):
            fn(i)
        ts = []
        for _ in range(groups):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for r in range(reps):
                fn(r % sets)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3 / reps)
        ts.sort()
        return round(2 * nb / ts[len(ts) // 2] / 1e9, 1)

    res = {"hipMemcpyDtoD_1GiB_GBps": rate(lambda i: b.copy_(a), nbytes),
           "mc_copy_1GiB_GBps": rate(lambda i: _ops.copy(a, b, nbytes), nbytes)}
    ins = [a[k * CHUNK:(k + 1) * CHUNK] for k in range(4)]
    outs = [b[k * CHUNK:(k + 1) * CHUNK] for k in range(4)]
    res["mc_copy_256MiB_rot4_GBps"] = rate(lambda i: _ops.copy(ins[i], outs[i], CHUNK), CHUNK, 4)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from lab.lablib import bwcal

        lab = bwcal()
        for u, g in ((8, 0), (4, 8192)):
            res[f"nt_copy_u{u}_g{g}_1GiB_GBps"] = rate(
                lambda i: lab.mc_lab_bw_copy(a.data_ptr(), b.data_ptr(), nbytes, u, g, 3, st), nbytes)
        for u, g in ((8, 0), (4, 8192)):
            res[f"nt_copy_u{u}_g{g}_256MiB_rot4_GBps"] = rate(
                lambda i: lab.mc_lab_bw_copy(ins[i].data_ptr(), outs[i].data_ptr(), CHUNK, u, g, 3, st), CHUNK, 4)
    except (ImportError, OSError, FileNotFoundError) as e:  # built by __graft_entry__.build()
        res["nt_copy_calibration"] = f"unavailable: {e}"
    del a, b, ins, outs
    torch.cuda.empty_cache()
    res["ceiling_GBps"] = max(v for k, v in res.items() if k.endswith("_GBps"))
    return res


def _cpu_rate(fn, nbytes: int, seconds: float = 0.3) -> float:
    """GiB/s of `nbytes` per call of fn() on this host core (one warm call,
    then as many calls as fit in `seconds`)."""
    fn()
    k, t0 = 0, time.perf_counter()
    while True:
        fn()
        k += 1
        t = time.perf_counter() - t0
        if t >= seconds:
            return round(k * nbytes / GiB / t, 3)


def next_rows(dev, sets: int = 3, cpu_seconds: float = 0.3) -> dict:
    """SURVEY §8f's rows on this GPU through their public API (device tensors
    in and out), 256 MiB per call, `sets` rotating buffer sets: each entry has
    enc/dec us, GiB/s of chunk bytes (the metric's definition), its kernels'
    fraction of HBM peak (algorithmic bytes / event-timed duration; a verify
    reads N bytes and syncs once to compare) and a 1-core CPU baseline over a
    64 MiB sample: zlib for CRC32 / Adler32 (the reference's own dependency,
    checksum32.py:95-130), numpy for PackBits / AsType (the reference's own
    code path), the build's C restatement (oracle/) for CRC32C, Fletcher32 and
    the Blosc filters ("port")."""
    import zlib

    from numcodecs_amd import CRC32, CRC32C, Adler32, AsType, Fletcher32, PackBits
    from numcodecs_amd import blosc_shuffle as bsh
    from oracle import blosc as oblosc
    from oracle import nporacle as npo

    N = CHUNK
    sample = np.random.default_rng(0).integers(0, 256, 64 * MiB, dtype=np.uint8)
    xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    out = {}

    def row(name, enc_fn, dec_fn, alg_enc, alg_dec, cpu_gibps, cpu_kind, chunk_bytes=N, reps=10, note=None):
        t_e = _timed(enc_fn, sets, reps)
        t_d = _timed(dec_fn, sets, reps)
        d = {"GiBps": round(2 * chunk_bytes / GiB / (t_e + t_d), 1), "enc_us": round(t_e * 1e6, 1),
             "dec_us": round(t_d * 1e6, 1),
             "enc_frac": round(alg_enc / t_e / 1e9 / PEAK_GBPS, 4), "dec_frac": round(alg_dec / t_d / 1e9 / PEAK_GBPS, 4),
             "cpu_1core_GiBps": cpu_gibps, "cpu_kind": cpu_kind}
        if cpu_gibps:
            d["gpu_over_cpu_1core"] = round(d["GiBps"] / cpu_gibps, 1)
        if note:
            d["note"] = note
        out[name] = d

    for name, codec, cpu_fn, kind in (
            ("CRC32", CRC32(), lambda: zlib.crc32(sample), "reference (zlib.crc32)"),
            ("CRC32C", CRC32C(), lambda: npo.crc32c(sample), "port"),
            ("Adler32", Adler32(), lambda: zlib.adler32(sample), "reference (zlib.adler32)"),
            ("Fletcher32", Fletcher32(), lambda: npo.fletcher32(sample), "port")):
        encs = [codec.encode(x) for x in xs]
        cpu = _cpu_rate(cpu_fn, sample.nbytes, cpu_seconds)
        # CPU: the checksum itself (encode and decode both compute it over N)
        row(name, lambda i, c=codec: c.encode(xs[i]), lambda i, c=codec, e=encs: c.decode(e[i]),
            2 * N + 4, N + 4, cpu, kind, note="decode = one-launch verify + host wait on the verdict")
        del encs
    # PackBits: 256 MiB of bools -> 32 MiB + 1 header byte
    bools = [(x & 1).view(torch.bool) for x in xs]
    pb = PackBits()
    pencs = [pb.encode(b) for b in bools]
    sbool = (sample & 1).astype(bool)
    cpu_pb = _cpu_rate(lambda: np.unpackbits(np.packbits(sbool))[: sbool.size].view(bool), sample.nbytes,
                       cpu_seconds)
    row("PackBits", lambda i: pb.encode(bools[i]), lambda i: pb.decode(pencs[i]), N + N // 8 + 1, N // 8 + 1 + N,
        cpu_pb, "reference (numpy packbits/unpackbits)")
    del bools, pencs
    # AsType f4 -> f8 (encode: decode_dtype f4 to encode_dtype f8) and back
    at = AsType(encode_dtype="<f8", decode_dtype="<f4")
    f4 = [x.view(torch.float32) for x in xs]
    f8 = [at.encode(x) for x in f4]
    s4 = sample.view(np.float32)
    cpu_at = _cpu_rate(lambda: s4.astype(np.float64).astype(np.float32), sample.nbytes, cpu_seconds)
    row("AsType_f4_f8", lambda i: at.encode(f4[i]), lambda i: at.decode(f8[i]), 3 * N, 3 * N, cpu_at,
        "reference (numpy astype)")
    del f8
    # Blosc SHUFFLE / BITSHUFFLE filters, typesize 4, 256 KiB blocks
    for mode, name in ((1, "Blosc_shuffle"), (2, "Blosc_bitshuffle")):
        fw = [bsh.shuffle(x, 4, 256 * 1024, mode) for x in xs]
        small = sample[: 8 * MiB]
        cpu_b = _cpu_rate(lambda m=mode: oblosc.blosc_filter(oblosc.blosc_filter(small, 4, 256 * 1024, m), 4,
                                                             256 * 1024, m, forward=False), small.nbytes,
                          cpu_seconds)
        row(name, lambda i, m=mode: bsh.shuffle(xs[i], 4, 256 * 1024, m),
            lambda i, m=mode, f=fw: bsh.unshuffle(f[i], 4, 256 * 1024, m), 2 * N, 2 * N, cpu_b, "port")
        del fw
    del xs
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline legs")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="timed CPU work per leg and config")
    ap.add_argument("--cpu-procs", type=int, default=min(16, os.cpu_count() or 1),
                    help="processes of the parallel CPU leg (the GPU box's CPU share is 16)")
    ap.add_argument("--quick", action="store_true", help="headline and c5_sharded only (no cfg_* block)")
    ap.add_argument("--c5-chunks", type=int, default=8192)
    ap.add_argument("--c5-steps", type=int, default=5)
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the rank launch and the C5 partition (no GPU)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # the launcher parent never touches the GPU: it times the CPU legs
        # (bounded: the headline's C2 f32 and C5) before it starts the ranks
        # and hands them to rank 0 through a file
        extra = {}
        if not args.no_cpu:
            import tempfile

            cpu = cpu_baselines(args.cpu_procs, args.cpu_seconds, only=CPU_CONFIGS_MULTI)
            fd, path = tempfile.mkstemp(prefix="mcodec_bench_cpu_", suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(cpu, f)
            extra["MCODEC_BENCH_CPU_JSON"] = path
        try:
            rc = launch_ranks(args.gpus, args.dry_run, extra)
        finally:
            if extra:
                os.unlink(extra["MCODEC_BENCH_CPU_JSON"])
        sys.exit(rc)
    world_env = int(env_world or 1)
    if world_env != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world_env}")

    # the CPU legs fork, so they run before anything touches the GPU: at N = 1
    # all of them; at N > 1 the launcher parent's (self-launch) or, under
    # torch.distributed.run, rank 0's own before it joins the process group
    cpu = load_cpu(os.environ.get("MCODEC_BENCH_CPU_JSON"))
    rank_env = int(os.environ.get("RANK", "0"))
    if cpu is None and rank_env == 0 and not args.no_cpu:
        if world_env == 1 and not args.dry_run:
            cpu = cpu_baselines(args.cpu_procs, args.cpu_seconds)
        elif world_env > 1:
            cpu = cpu_baselines(args.cpu_procs, args.cpu_seconds, only=CPU_CONFIGS_MULTI)

    dist, rank, world, local = dist_setup(args.dry_run)
    if args.dry_run:
        dry_run(dist, rank, world, args.c5_chunks, cpu)
        if dist is not None:
            dist.destroy_process_group()
        return
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    ident = rank_identity(rank, local, dev)
    elapsed, launch_ms, gpu_s = run_step_timing(args, dev, dist, rank)
    t = max_over_ranks(dist, elapsed)
    launch_ms = max_over_ranks(dist, launch_ms)
    value = world * args.steps * 2 * CHUNK / GiB / t  # bytes into encode + decode, all ranks
    # headline: 2 x CHUNK into encode + decode per step (the metric's bytes),
    # 4 x CHUNK of HBM reads + writes per step (the roofline's bytes)
    head_ranks = gather_ranks(dist, dict(ident, elapsed_s=round(elapsed, 6), gpu_event_s=round(gpu_s, 6)))
    head_scale = scaling_fields(head_ranks, args.steps * 4 * CHUNK, args.steps * 2 * CHUNK, t, on_gpu=True)

    c5_el, c5_launch_ms, c5_local, c5_gpu_s = run_c5_sharded(args.c5_steps, 1, args.c5_chunks, dev, dist, rank,
                                                              world)
    c5_t = max_over_ranks(dist, c5_el)
    c5_launch_ms = max_over_ranks(dist, c5_launch_ms)
    c5_ranks = gather_ranks(dist, {"rank": rank, "host": ident["host"], "pci": ident["pci"],
                                   "chunks": c5_local, "elapsed_s": round(c5_el, 6),
                                   "gpu_event_s": round(c5_gpu_s, 6)})
    c5_ev_max = max(r["gpu_event_s"] for r in c5_ranks)

    if rank == 0:
        achieved = 2 * CHUNK / (launch_ms * 1e-3) / 1e9  # GB/s per launch
        traffic, traffic_src = pmc_traffic()
        ceiling = copy_ceiling(dev)
        c5_bytes = args.c5_steps * 2 * args.c5_chunks * MiB
        c5_alg = c5_local * (2 * MiB + 4)  # rank 0's chunks per launch: payload in + out (+ footer)
        c5_phys = head_scale["physical_gpus"]
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "value_scope": ("whole-job aggregate over all ranks (the driver contract); per_gpu_GiBps = "
                            "value / physical_gpus is the metric's per-GPU figure (equal at N = 1)"),
            "n_gpus": world,
            "per_gpu_GiBps": head_scale["per_gpu_GiBps"],
            "aggregate_GiBps": head_scale["aggregate_GiBps"],
            "event_aggregate_GiBps": head_scale["event_aggregate_GiBps"],
            "host_minus_event_s": head_scale["host_minus_event_s"],
            "frac_of_n_peak": head_scale["frac_of_n_peak"],
            "physical_gpus": c5_phys,
            "rehearsal": head_scale["rehearsal"],
            "ranks": head_ranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randn fp32 on device, 4 rotating 256 MiB chunk sets per GPU)",
            "config": {
                "workload": "configs[1]: Shuffle(elementsize=4) encode+decode, one 256 MiB fp32 chunk per GPU per step",
                "chunk_bytes": CHUNK,
                "elementsize": 4,
                "parallelism": f"chunk-sharded x{world} (no collective)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_shuffle_enc<4> / k_shuffle4_dec_pair, 2 x 256 MiB per launch",
                "achieved": round(achieved, 1),
                "peak": PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "mean_launch_ms": round(launch_ms, 4),
                "copy_ceiling_GBps": ceiling["ceiling_GBps"],
                "frac_of_copy_ceiling": round(achieved / ceiling["ceiling_GBps"], 4),
                "copy_calibration": ceiling,
                **(trace_roofline() or {"trace_frac": None}),
            },
            "c5_sharded": {
                "GiBps": round(c5_bytes / GiB / c5_t, 1),
                "per_gpu_GiBps": round(c5_bytes / GiB / c5_t / c5_phys, 1),
                "event_GiBps": round(c5_bytes / GiB / c5_ev_max, 1),
                "host_minus_event_s": round(c5_t - c5_ev_max, 6),
                "n_gpus": world,
                "physical_gpus": c5_phys,
                "chunks": args.c5_chunks,
                "steps": args.c5_steps,
                "ms_per_step": round(c5_t / args.c5_steps * 1e3, 3),
                "scaling": "strong",
                "frac_of_n_peak": round(c5_bytes / c5_t / 1e9 * 2 / (c5_phys * PEAK_GBPS), 4),
                "kernel_GBps_rank0": round(c5_alg / (c5_launch_ms * 1e-3) / 1e9, 1),
                "workload": ("configs[4]: 8192 x 1 MiB f32 split into contiguous chunk ranges; timed step = fused "
                             "Shuffle(4)+Fletcher32 encode + fused verify+unshuffle decode with the per-chunk "
                             "verdict compared on the device and read back (raising on a mismatch) every step"),
                "ranks": c5_ranks,
            },
        }
        result["cpu_baseline"] = headline_cpu(cpu)
        if world > 1:
            # the N > 1 line keeps a bounded per-config block: the headline's
            # C2 f32 (rank 0's launches) and the sharded C5, each beside its
            # CPU baseline timed on this node before the ranks started
            t_launch = launch_ms * 1e-3
            result["cfg_C2_f32"] = _cfg(2 * CHUNK / GiB / (2 * t_launch), t_launch, t_launch, 4 * CHUNK,
                                        "k_shuffle_enc<4> / k_shuffle4_dec_pair (rank 0, slowest launch)", cpu,
                                        "C2_f32")
            c5_call = c5_launch_ms * 1e-3
            result["cfg_C5"] = _cfg(2 * c5_local * MiB / GiB / (2 * c5_call), c5_call, c5_call,
                                    2 * c5_alg, "k_shuffle_f32_enc / k_f32_unshuffle (rank 0's chunk range)",
                                    cpu, "C5", f"rank 0's {c5_local} of {args.c5_chunks} chunks per call")
        if world == 1 and not args.quick:
            result.update(config_workloads(dev, cpu))
            result["cfg_e2e"] = end_to_end(dev, cpu)
            result["cfg_next"] = next_rows(dev)
        print(json.dumps(result), flush=True)
    if dist is not None:
        barrier(dist)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
