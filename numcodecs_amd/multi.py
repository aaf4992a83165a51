"""In-process multi-GPU dispatch of chunk batches.

Chunks are independent: a Zarr read or write of thousands of
chunks can spread its batch over every GPU of the node with no collective
and no data exchange between devices.  The reference's own concurrency model
is the caller's pool (tests/test_shuffle.py:90-109 runs codecs in
multiprocessing / thread pools); here ONE Python caller hands a batch to
:func:`numcodecs_amd.batch.host_pipeline`,
:func:`numcodecs_amd.chunks.host_encode_chunks` / ``host_decode_chunks`` or
:func:`numcodecs_amd.chunks.encode_chunks` / ``decode_chunks`` with
``devices=[...]``, and:

* the rows are cut into contiguous ranges with :func:`shard.chunk_range`
  (device g gets rows [g*B/G, (g+1)*B/G)), so the output keeps the input's
  row order;
* one worker thread per device entry runs the single-device path on its
  range with its own role streams and device ring (the ctypes calls into
  libmcodec and torch's copies release the GIL, so the devices' host work
  and PCIe traffic overlap);
* a device-resident batch is processed where it lives: either as
  per-device resident shards (a list of tensors, one per GPU: each shard
  runs on its own device, on the caller's current stream there, and its
  result stays on that device -- no copy, no host wait;
  :func:`device_shards`), or as ONE tensor whose row ranges run on workers
  of that same device (:func:`device_rows`, the caller's stream).  Naming
  other GPUs for a one-device batch is refused: shipping 7/8 of a batch
  over xGMI and back turns a ~6 TB/s local pass into two transfers at tens
  to low hundreds of GB/s.  ``allow_peer_copy=True`` opts in anyway (each
  range copied to its GPU and the result copied back, ordered by events:
  the caller's stream waits, the host does not);
* checksum mismatches are raised after every worker finished, the first one
  in row order, exactly as the single-device call raises it; any other
  worker exception is re-raised likewise (the first in row order).

The same device may appear several times (``devices=[0, 0]``): its entries
are independent workers, which is how the tests exercise the partition on a
one-GPU box.  Distinct GPUs are untested: nothing here has run on a
multi-GPU node yet.
"""

from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import torch

from . import shard

__all__ = ["normalize_devices", "split_rows", "run_workers", "check_peer_devices", "device_rows", "device_shards",
           "host_rows"]


def normalize_devices(devices) -> "list[torch.device]":
    """A list of HIP devices from ints / strings / torch.device objects."""
    out = []
    for d in devices:
        if isinstance(d, int):
            d = torch.device("cuda", d)
        d = torch.device(d)
        if d.type != "cuda":
            raise ValueError(f"devices must be GPU devices, got {d}")
        if d.index is None:
            d = torch.device("cuda", torch.cuda.current_device())
        out.append(d)
    if not out:
        raise ValueError("devices must name at least one GPU")
    return out


def split_rows(nrows: int, ndev: int) -> "list[tuple[int, int, int]]":
    """(worker, lo, hi) for every worker with a non-empty contiguous row
    range: shard.chunk_range's partition of `nrows` over `ndev` workers."""
    parts = []
    for g in range(ndev):
        lo, hi = shard.chunk_range(nrows, g, ndev)
        if hi > lo:
            parts.append((g, lo, hi))
    return parts


def run_workers(fns) -> list:
    """Run the zero-argument callables `fns` on one thread each; return their
    results in order, or re-raise the first exception in that order after
    every worker has finished (no worker is left running)."""
    if len(fns) == 1:
        return [fns[0]()]
    with ThreadPoolExecutor(max_workers=len(fns), thread_name_prefix="mcodec-dev") as ex:
        futs = [ex.submit(f) for f in fns]
        results, first_exc = [], None
        for f in futs:
            try:
                results.append(f.result())
            except BaseException as e:  # noqa: BLE001 -- re-raised below, in row order
                results.append(None)
                if first_exc is None:
                    first_exc = e
    if first_exc is not None:
        raise first_exc
    return results


def check_peer_devices(home, devices, allow_peer_copy: bool) -> bool:
    """True when `devices` name a GPU other than `home` (the batch's device);
    raises ValueError for that unless `allow_peer_copy`."""
    home = torch.device(home)
    remote = [d for d in devices if d != home]
    if remote and not allow_peer_copy:
        raise ValueError(
            f"devices={[str(d) for d in devices]} names GPUs other than the batch's own ({home}): a device-resident "
            "batch is processed where it lives.  Pass per-device resident shards (a list of tensors, one per GPU) "
            "to use several GPUs, or allow_peer_copy=True to copy row ranges over xGMI and back.")
    return bool(remote)


def device_shards(fn, shards):
    """Apply ``fn(shard) -> (y, extra)`` to per-device resident shards (a
    list of device tensors [b_k, ...], any devices, repeats allowed): one
    worker thread per shard, each on the caller's current stream of the
    shard's device (captured here), so stream order is the only hand-off --
    no copies, no host wait.  Returns ([y_k as [b_k, m] on shard k's
    device], [extra_k]) in shard order."""
    shards = list(shards)
    if not shards:
        raise ValueError("no shards")
    for t in shards:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.dim() < 1:
            raise TypeError("device_shards takes device tensors [b, ...]")
    streams = [torch.cuda.current_stream(t.device) for t in shards]

    def work(k):
        t = shards[k]
        with torch.cuda.device(t.device), torch.cuda.stream(streams[k]):
            y, extra = fn(t)
            return y.reshape(y.shape[0], -1), extra

    res = run_workers([lambda k=k: work(k) for k in range(len(shards))])
    return [r[0] for r in res], [r[1] for r in res]


def device_rows(fn, rows: torch.Tensor, devices, allow_peer_copy: bool = False):
    """Apply the single-device batch function ``fn(rows_on_dev) -> (y, extra)``
    (y a [b, ...] tensor) to the contiguous row ranges of a device batch
    `rows` on `devices`.  Returns (the results gathered in row order on
    `rows`' device as [B, m], the workers' `extra` values in row order).

    Workers on `rows`' own device run on the caller's current stream there.
    Other GPUs are refused unless `allow_peer_copy` (check_peer_devices);
    then each such range is copied to its GPU on a worker stream that waits
    on the caller's stream, processed, and copied back by the caller's thread
    once the caller's stream waits on the worker's completion event (torch's
    cross-device copy orders itself against both devices' current streams):
    no host wait anywhere."""
    devices = normalize_devices(devices)
    home = rows.device
    check_peer_devices(home, devices, allow_peer_copy)
    parts = split_rows(rows.shape[0], len(devices))
    if not parts:
        y, extra = fn(rows)
        return y.reshape(y.shape[0], -1), [extra]
    caller = torch.cuda.current_stream(home)
    ready = torch.cuda.Event()
    ready.record(caller)

    def work(g, lo, hi):
        dev = devices[g]
        if dev == home:
            with torch.cuda.device(home), torch.cuda.stream(caller):
                y, extra = fn(rows[lo:hi])
                return y.reshape(y.shape[0], -1), extra, None
        with torch.cuda.device(dev):
            s = torch.cuda.Stream(device=dev)
            s.wait_event(ready)  # the caller's producers of `rows` are done
            with torch.cuda.stream(s):
                part = rows[lo:hi].to(dev, non_blocking=True)
                y, extra = fn(part)
                y = y.reshape(y.shape[0], -1)
                done = torch.cuda.Event()
                done.record(s)
            return y, extra, done

    res = run_workers([lambda g=g, lo=lo, hi=hi: work(g, lo, hi) for g, lo, hi in parts])
    ys = []
    for (g, lo, hi), (y, _extra, done) in zip(parts, res):
        if done is not None:  # a peer range: back onto the caller's device, in stream order
            src_stream = torch.cuda.current_stream(y.device)
            src_stream.wait_event(done)
            y.record_stream(src_stream)
            with torch.cuda.device(home), torch.cuda.stream(caller):
                y = y.to(home, non_blocking=True)
        ys.append(y)
    with torch.cuda.device(home), torch.cuda.stream(caller):
        out = ys[0] if len(ys) == 1 else torch.cat(ys)
    return out, [r[1] for r in res]


def host_rows(fn, nrows: int, devices) -> list:
    """Run ``fn(device, lo, hi)`` -- a single-device streaming call over host
    rows [lo, hi) -- for every worker's contiguous range, one thread each;
    results in row order (the first exception in row order re-raised)."""
    devices = normalize_devices(devices)
    parts = split_rows(nrows, len(devices))
    return run_workers([lambda g=g, lo=lo, hi=hi: fn(devices[g], lo, hi) for g, lo, hi in parts])
