"""Benchmark: Shuffle(4) encode+decode of device-resident 256 MiB fp32 chunks.

Metric (BASELINE.json): "GiB/s encode+decode per GPU, device-resident fp32
chunks (Shuffle, BitRound)", measured on configs[1]: Shuffle(elementsize=4)
on a 256 MiB float32 chunk per GPU.  One step = Shuffle(4).encode +
Shuffle(4).decode of one chunk (4 rotating buffer sets per GPU so that the
256 MiB Infinity Cache cannot serve a step from the previous one).
value = (bytes into encode + bytes into decode) over all ranks / time.

    python bench.py [--gpus N --steps K --warmup W] [--no-cpu] [--extra]

For N > 1 the driver launches one process per GPU with torch.distributed.run;
chunks are independent, so every rank streams its own chunks (weak scaling)
and the only collectives are the timing barrier and the max-over-ranks of
the elapsed time (no data-path collective).

Printed (rank 0): ONE JSON line with the contract's keys plus
  roofline     -- the Shuffle(4) encode/decode kernels (each moves 2 x 256 MiB
                  of algorithmic bytes per launch) / their mean launch
                  duration, from a HIP event pair on the launch stream
                  bracketing the timed region; peak 8 TB/s; `traffic` = HBM
                  bytes per launch from the rocprofv3 PMC counters committed
                  under profiles/ (null when absent); `achievable` = an
                  on-device 1 GiB DtoD copy measured in the same run (the
                  practical HBM ceiling of SURVEY §8d) and achieved / it;
  cpu_baseline -- the reference's own Cython _doShuffle/_doUnshuffle
                  (src/numcodecs/_shuffle.pyx, compiled from the reference
                  sources into oracle/_ref by oracle/build_ref.sh) on one host
                  core, time-bounded sample of the same workload; falls back to
                  the oracle's C restatement ("port") when _ref is absent.
"""

from __future__ import annotations

import argparse
import glob
import json
import os
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


def dist_setup(n_gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # RCCL ("nccl") on the GPU node; MCODEC_BENCH_BACKEND=gloo rehearses
        # several ranks on one GPU (device = LOCAL_RANK mod visible devices)
        backend = os.environ.get("MCODEC_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
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


def _ref_shuffle_fns():
    """(encode, decode, kind, description) of the CPU Shuffle baseline."""
    try:
        from oracle import refload

        if not os.path.isdir(refload.REF_BUILD) or not glob.glob(os.path.join(refload.REF_BUILD, "_shuffle*.so")):
            raise ImportError
        import importlib.util

        so = glob.glob(os.path.join(refload.REF_BUILD, "_shuffle*.so"))[0]
        spec = importlib.util.spec_from_file_location("numcodecs._shuffle", so)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        do_enc, do_dec = mod._doShuffle, mod._doUnshuffle
        kind = "reference"
        src_desc = "src/numcodecs/_shuffle.pyx _doShuffle/_doUnshuffle compiled from the reference sources (oracle/_ref)"
    except Exception:
        from oracle import nporacle

        def do_enc(a, b, es):
            nporacle.shuffle_into(a, b, es)

        def do_dec(a, b, es):
            nporacle.unshuffle_into(a, b, es)

        src_desc = "oracle/ncoracle.c restatement of _shuffle.pyx:11-30 (-O3, no -march)"
        kind = "port"
    return do_enc, do_dec, kind, src_desc


def _cpu_worker(args):
    """One process of the parallel leg: its own 64 MiB chunk, enc+dec until
    the shared deadline; returns (bytes, seconds)."""
    seed, deadline = args
    do_enc, do_dec, _, _ = _ref_shuffle_fns()
    x = np.random.default_rng(seed).integers(0, 256, 64 * MiB, dtype=np.uint8)
    enc, dec = np.empty_like(x), np.empty_like(x)
    do_enc(x, enc, 4)
    t0 = time.perf_counter()
    n = 0
    while time.time() < deadline or n == 0:
        do_enc(x, enc, 4)
        do_dec(enc, dec, 4)
        n += 1
    return 2 * x.nbytes * n, time.perf_counter() - t0


def cpu_baseline_parallel(procs: int, seconds: float = 5.0):
    """The reference loop in `procs` processes at once (the reference holds the
    GIL, so a Zarr reader scales over processes, not threads).  Forked BEFORE
    the GPU is initialised (never fork or exec after HIP init)."""
    import multiprocessing as mp

    deadline = time.time() + 1.0 + seconds
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(100 + i, deadline) for i in range(procs)])
    total = sum(b for b, _ in res)
    el = max(t for _, t in res)
    return {"value": round(total / GiB / el, 3), "unit": "GiB/s", "cores": procs,
            "sample": f"{procs} processes x Shuffle(4) encode+decode of their own 64 MiB chunk for {el:.1f} s"}


def cpu_baseline(seconds: float = 10.0):
    """Reference Shuffle(4) enc+dec on one core, time-bounded sample."""
    x = np.random.default_rng(0).integers(0, 256, CHUNK, dtype=np.uint8)
    enc = np.empty_like(x)
    dec = np.empty_like(x)
    do_enc, do_dec, kind, src_desc = _ref_shuffle_fns()
    do_enc(x, enc, 4)  # warm
    do_dec(enc, dec, 4)
    assert np.array_equal(dec, x)
    t0 = time.perf_counter()
    n = 0
    while True:
        do_enc(x, enc, 4)
        do_dec(enc, dec, 4)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 3:
            break
    gibps = 2 * CHUNK * n / GiB / el
    return {
        "value": round(gibps, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": f"Shuffle(4) encode+decode of one 256 MiB chunk x {n} ({el:.1f} s), {src_desc}",
    }


def run_step_timing(args, dev, dist, rank, world):
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
    # ~5 us on ROCm (kernel gaps 0 -> 5.8 us in the rocprofv3 trace), so the
    # mean launch duration is GPU time / launches (encode and decode move the
    # same 2 x 256 MiB each; rocprofv3 per-kernel averages are in profiles/).
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
    return elapsed, gpu_ms / (2 * args.steps)


def run_c5_timing(args, dev, dist, rank, world):
    """configs[4]: 8192 x 1 MiB fp32 chunks, Shuffle(4) + Fletcher32 fused,
    sharded over ranks by contiguous chunk ranges (shard.chunk_range, no
    collective); one step = encode + verified decode of the rank's chunks.
    Returns (elapsed_s, mean launch ms, local chunks)."""
    from numcodecs_amd import batch, shard

    lo, hi = shard.chunk_range(args.c5_chunks, rank, world)
    b = hi - lo
    g = torch.Generator(device=dev).manual_seed(1000 + lo)
    x = torch.randn((b, MiB // 4), generator=g, device=dev, dtype=torch.float32)
    enc = batch.shuffle_fletcher32_encode_chunks(x, 4)
    dec = torch.empty((b, MiB), dtype=torch.uint8, device=dev)
    _, status = batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4, out=dec, check_sums=True)
    assert torch.equal(dec.view(torch.float32), x), "C5 round trip failed"

    def step():
        batch.shuffle_fletcher32_encode_chunks(x, 4, out=enc)
        batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4, out=dec, check_sums=False)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    barrier(dist)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the decode's checksum verdicts of the last step: every chunk must match
    _, status = batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4, out=dec, check_sums=True)
    assert torch.equal(dec.view(torch.float32), x), "C5 round trip failed after timing"
    return elapsed, ev0.elapsed_time(ev1) / (2 * args.steps), b


def extra_workloads(dev, sets: int = 4):
    """The other configurations of BASELINE.json, single GPU (reported under
    "extra", not the headline value).  Every timed call rotates over `sets`
    buffer sets, so no call finds its input left in the 256 MiB Infinity Cache
    by the previous one (as in the headline timing)."""
    from numcodecs_amd import BitRound, Delta, FixedScaleOffset, Shuffle, batch

    out = {}

    def timed(fn, reps=20):
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

    # C2 f64 Shuffle(8)
    x64 = [torch.randn(CHUNK // 8, device=dev, dtype=torch.float64) for _ in range(sets)]
    e64 = [Shuffle(8).encode(x) for x in x64]
    d64 = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(sets)]
    t_e = timed(lambda i: Shuffle(8).encode(x64[i], out=e64[i]))
    t_d = timed(lambda i: Shuffle(8).decode(e64[i], out=d64[i]))
    out["C2_shuffle8_f64_encdec_GiBps"] = round(2 * CHUNK / GiB / (t_e + t_d), 1)
    del x64, e64, d64
    # C3 BitRound(10) fused with Shuffle(4); decode = unshuffle (+ re-view)
    x32 = [torch.randn(CHUNK // 4, device=dev) for _ in range(sets)]
    pipe = batch.FilterPipeline([BitRound(10), Shuffle(4)])
    enc = [pipe.encode(x) for x in x32]
    t_e = timed(lambda i: pipe.encode(x32[i]))
    t_d = timed(lambda i: Shuffle(4).decode(enc[i]))
    out["C3_bitround10_shuffle4_encdec_GiBps"] = round(2 * CHUNK / GiB / (t_e + t_d), 1)
    del x32, enc
    # C4 FSO(f4->i2) -> Delta(i2) -> Shuffle(2): fused pipeline, and codec by codec
    xc = [1000.0 + 10.0 * torch.rand(CHUNK // 4, device=dev) for _ in range(sets)]
    fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
    dl = Delta(dtype="<i2")
    sh = Shuffle(2)
    c4 = batch.FilterPipeline([fso, dl, sh])
    e = [c4.encode(x) for x in xc]
    t_e = timed(lambda i: c4.encode(xc[i]))
    t_d = timed(lambda i: c4.decode(e[i]))
    out["C4_fso_delta_shuffle2_fused_encdec_GiBps"] = round(2 * CHUNK / GiB / (t_e + t_d), 1)
    out["C4_fused_encode_us"] = round(t_e * 1e6, 1)
    out["C4_fused_decode_us"] = round(t_d * 1e6, 1)
    t_e = timed(lambda i: sh.encode(dl.encode(fso.encode(xc[i]))))
    t_d = timed(lambda i: fso.decode(dl.decode(sh.decode(e[i]))))
    out["C4_fso_delta_shuffle2_codec_by_codec_encdec_GiBps"] = round(2 * CHUNK / GiB / (t_e + t_d), 1)
    del xc, e
    # C5 batch 8192 x 1 MiB Shuffle(4) + Fletcher32, one GPU (8 GiB per call:
    # nothing survives in the Infinity Cache between calls)
    xb = torch.randint(0, 256, (8192, MiB), dtype=torch.uint8, device=dev)
    eb = batch.shuffle_fletcher32_encode_chunks(xb, 4)
    db = torch.empty_like(xb)
    t_e = timed(lambda i: batch.shuffle_fletcher32_encode_chunks(xb, 4, out=eb), reps=5)
    t_d = timed(lambda i: batch.fletcher32_unshuffle_decode_chunks(eb, MiB, 4, out=db, check_sums=False), reps=5)
    out["C5_batch8192x1MiB_shuffle4_fletcher32_encdec_GiBps"] = round(2 * 8192 * MiB / GiB / (t_e + t_d), 1)
    return out


def next_row_workloads(dev):
    """SURVEY.md §8f next rows (Checksum32 family, PackBits, AsType), single
    GPU, device-resident; GB/s of algorithmic HBM bytes (read + write) so the
    numbers compare with the 8 TB/s peak directly."""
    from numcodecs_amd import AsType, PackBits, batch
    from numcodecs_amd import _ops

    out = {}

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    nb = 2048  # 2048 x 1 MiB chunks = 2 GiB per launch
    xb = torch.randint(0, 256, (nb, MiB), dtype=torch.uint8, device=dev)
    eb = torch.empty((nb, MiB + 4), dtype=torch.uint8, device=dev)
    x1 = torch.randint(0, 256, (CHUNK,), dtype=torch.uint8, device=dev)
    for cid in ("crc32", "crc32c", "adler32"):
        t = timed(lambda: batch.checksum32_chunks(xb, cid))
        out[f"{cid}_batch2048x1MiB_checksum_GBps"] = round(nb * MiB / t / 1e9, 1)
        t = timed(lambda: batch.checksum32_encode_chunks(xb, cid, out=eb))
        out[f"{cid}_batch2048x1MiB_encode_GBps"] = round(2 * nb * MiB / t / 1e9, 1)
        kind = batch._CK_KINDS[cid][0]
        t = timed(lambda: _ops.checksum32(kind, x1, CHUNK, 1, CHUNK, 0))
        out[f"{cid}_256MiB_checksum_GBps"] = round(CHUNK / t / 1e9, 1)
    t = timed(lambda: batch.checksum32_chunks(xb, "jenkins_lookup3"), reps=2)
    out["jenkins_batch2048x1MiB_checksum_GBps"] = round(nb * MiB / t / 1e9, 1)
    del xb, eb
    bools = torch.randint(0, 2, (CHUNK,), dtype=torch.uint8, device=dev).view(torch.bool)
    enc = PackBits().encode(bools)
    t = timed(lambda: PackBits().encode(bools))
    out["packbits_256MiB_encode_GBps"] = round((CHUNK + CHUNK // 8) / t / 1e9, 1)
    t = timed(lambda: PackBits().decode(enc))
    out["packbits_256MiB_decode_GBps"] = round((CHUNK + CHUNK // 8) / t / 1e9, 1)
    from numcodecs_amd import blosc_shuffle as bsh

    x4 = torch.randn(CHUNK // 4, device=dev)
    for mode, name in ((bsh.SHUFFLE, "shuffle"), (bsh.BITSHUFFLE, "bitshuffle")):
        enc4 = bsh.shuffle(x4, 4, 256 * 1024, mode)
        t_e = timed(lambda: bsh.shuffle(x4, 4, 256 * 1024, mode))
        t_d = timed(lambda: bsh.unshuffle(enc4, 4, 256 * 1024, mode))
        out[f"blosc_{name}_f4_256KiB_blocks_enc_GBps"] = round(2 * CHUNK / t_e / 1e9, 1)
        out[f"blosc_{name}_f4_256KiB_blocks_dec_GBps"] = round(2 * CHUNK / t_d / 1e9, 1)
    del x4, enc4
    x64 = torch.randn(CHUNK // 8, device=dev, dtype=torch.float64)
    t = timed(lambda: AsType("<f4", "<f8").encode(x64))
    out["astype_f8_to_f4_256MiB_GBps"] = round(1.5 * CHUNK / t / 1e9, 1)
    return out


def end_to_end(dev, total_gib: int = 2, chunk_bytes: int = 4 * MiB):
    """Host -> host rate: pinned H2D + Shuffle(4) kernel + D2H pipelined over
    H2D / kernel / D2H role streams (batch.host_pipeline); "end_to_end"."""
    from numcodecs_amd import batch

    nchunks = total_gib * GiB // chunk_bytes
    hin = torch.randint(0, 256, (nchunks, chunk_bytes), dtype=torch.uint8).pin_memory()
    henc = torch.empty_like(hin).pin_memory()
    hdec = torch.empty_like(hin).pin_memory()
    res = {}
    for slice_chunks in (16, 32):
        batch.host_pipeline(hin, henc, 4, True, slice_chunks=slice_chunks)
        t0 = time.perf_counter()
        batch.host_pipeline(hin, henc, 4, True, slice_chunks=slice_chunks)
        te = time.perf_counter() - t0
        t0 = time.perf_counter()
        batch.host_pipeline(henc, hdec, 4, False, slice_chunks=slice_chunks)
        td = time.perf_counter() - t0
        assert torch.equal(hdec, hin)
        res[f"slice_{slice_chunks * chunk_bytes // MiB}MiB"] = {
            "encode_GiBps": round(nchunks * chunk_bytes / GiB / te, 2),
            "decode_GiBps": round(nchunks * chunk_bytes / GiB / td, 2),
        }
    # raw PCIe rates for reference: pinned copies alone
    d = torch.empty((nchunks, chunk_bytes), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(hin, non_blocking=True)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    t0 = time.perf_counter()
    henc.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    d2h = time.perf_counter() - t0
    res["pcie_h2d_GiBps"] = round(total_gib / h2d, 2)
    res["pcie_d2h_GiBps"] = round(total_gib / d2h, 2)
    res["workload"] = f"{total_gib} GiB of {chunk_bytes // MiB} MiB chunks in pinned host memory, Shuffle(4), host->host"
    # a Zarr filter chain streamed host -> host (numcodecs_amd.chunks)
    from numcodecs_amd import CRC32, BitRound, Shuffle, chunks

    codecs = [BitRound(10), Shuffle(4), CRC32()]
    x32 = hin.view(torch.float32)
    x32.copy_(torch.randn(x32.shape))
    henc_z = torch.empty((nchunks, chunk_bytes + 4), dtype=torch.uint8).pin_memory()
    out = hdec.view(torch.float32)
    chunks.host_encode_chunks(codecs, x32, henc_z)  # warm-up: allocator pools, lazy init
    chunks.host_decode_chunks(codecs, henc_z, out)
    te = td = float("inf")
    for _ in range(3):  # best of 3 (host-side timing of a PCIe-bound stream)
        t0 = time.perf_counter()
        chunks.host_encode_chunks(codecs, x32, henc_z)
        te = min(te, time.perf_counter() - t0)
        t0 = time.perf_counter()
        chunks.host_decode_chunks(codecs, henc_z, out)
        td = min(td, time.perf_counter() - t0)
    res["zarr_chain_bitround10_shuffle4_crc32"] = {
        "encode_GiBps": round(nchunks * chunk_bytes / GiB / te, 2),
        "decode_GiBps": round(nchunks * chunk_bytes / GiB / td, 2),
    }
    return res


def copy_ceiling(dev, nbytes: int = GiB, reps: int = 10):
    """SURVEY §8d's "achievable" line: on-device DtoD copies of 1 GiB (more
    than the 256 MiB Infinity Cache) timed in this run -- hipMemcpyAsync (via
    torch's copy_) and libmcodec's own nontemporal copy kernel (mc_copy);
    GB/s = read + write bytes / median time of `reps` after a warm-up."""
    from numcodecs_amd import _ops

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)

    def rate(fn):
        fn()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        ts.sort()
        return round(2 * nbytes / ts[len(ts) // 2] / 1e9, 1)

    res = {"hipMemcpyDtoD_GBps": rate(lambda: b.copy_(a)), "mc_copy_GBps": rate(lambda: _ops.copy(a, b, nbytes))}
    del a, b
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=min(16, os.cpu_count() or 1),
                    help="processes of the parallel CPU leg (the GPU box's CPU share is 16)")
    ap.add_argument("--workload", choices=("c2", "c5"), default="c2",
                    help="c2 (default, the metric's config): Shuffle(4) on one 256 MiB chunk per GPU; "
                         "c5: 8192 x 1 MiB chunks + Fletcher32 sharded over the GPUs")
    ap.add_argument("--c5-chunks", type=int, default=8192)
    ap.add_argument("--extra", action="store_true", help="also time C2(f64)/C3/C4/C5 on rank 0")
    ap.add_argument("--e2e", action="store_true", help="also time the host->host pipelined path")
    ap.add_argument("--next", action="store_true",
                    help="also time the SURVEY §8f next rows (checksum32 family, PackBits, AsType)")
    args = ap.parse_args()
    if args.workload == "c5":
        args.no_cpu = True  # the CPU baseline is defined for the metric's workload (c2)

    # the multi-process CPU leg forks, so it runs before anything touches the GPU
    cpu_par = None
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_cpu and args.cpu_procs > 1:
        cpu_par = cpu_baseline_parallel(args.cpu_procs)

    dist, rank, world, local = dist_setup(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    c5 = args.workload == "c5"
    if c5:
        elapsed, launch_ms, local = run_c5_timing(args, dev, dist, rank, world)
    else:
        elapsed, launch_ms = run_step_timing(args, dev, dist, rank, world)
    t = max_over_ranks(dist, elapsed)
    launch_ms = max_over_ranks(dist, launch_ms)
    if c5:  # strong scaling: the 8192 chunks are split over the ranks
        total_bytes = args.steps * 2 * args.c5_chunks * MiB
    else:  # weak scaling: one 256 MiB chunk per rank per step
        total_bytes = world * args.steps * 2 * CHUNK  # bytes into encode + decode, all ranks
    value = total_bytes / GiB / t

    result = None
    if rank == 0:
        achieved = 2 * CHUNK / (launch_ms * 1e-3) / 1e9  # GB/s per launch
        traffic, traffic_src = pmc_traffic()
        ceiling = copy_ceiling(dev)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
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
                "kernel": "k_shuffle_enc<4> / k_shuffle4_dec_pair (Shuffle(4) encode / decode; 2 x 256 MiB algorithmic bytes per launch each)",
                "achieved": round(achieved, 1),
                "peak": PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "mean_launch_ms": round(launch_ms, 4),
                "timing": "HIP events bracketing the timed region on the launch stream / (2 x steps)",
                "achievable": {"what": "on-device DtoD copies of 1 GiB in this run, read+write bytes / time; "
                                       "frac = achieved / the faster copy",
                               **ceiling, "frac": round(achieved / max(ceiling.values()), 4)},
            },
        }
    if rank == 0 and c5:
        per_launch = (local * (MiB + 4) + local * MiB)  # rank 0's chunks: payload in + encoded out
        result["scaling"] = "strong"
        result["data"] = "synthetic (torch.randn fp32 on device, 1 MiB chunks)"
        result["config"] = {
            "workload": f"configs[4]: {args.c5_chunks} x 1 MiB fp32 chunks, Shuffle(4) + Fletcher32 fused encode + "
                        "verified decode, sharded by contiguous chunk ranges",
            "chunks": args.c5_chunks, "chunk_bytes": MiB, "elementsize": 4,
            "parallelism": f"chunk-sharded x{world} (no collective)",
        }
        result["roofline"].update({
            "kernel": "k_shuffle_f32_enc / k_f32_unshuffle (fused Shuffle(4)+Fletcher32, 2N+4 bytes per chunk)",
            "achieved": round(per_launch / (launch_ms * 1e-3) / 1e9, 1),
            "frac": round(per_launch / (launch_ms * 1e-3) / 1e9 / PEAK_GBPS, 4),
            "traffic": None, "traffic_source": None,
        })
        result["roofline"]["achievable"]["frac"] = round(result["roofline"]["achieved"] / max(ceiling.values()), 4)
    if rank == 0 and args.extra:
        result["extra"] = extra_workloads(dev)
    if rank == 0 and args.e2e:
        result["end_to_end"] = end_to_end(dev)
    if rank == 0 and args.next:
        result["next_rows"] = next_row_workloads(dev)
    if rank == 0:
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
            if cpu_par is not None:
                result["cpu_baseline"]["parallel"] = cpu_par
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if dist is not None:
        barrier(dist)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
