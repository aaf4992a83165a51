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
* for device-resident batches each range is copied to its device (a peer
  copy over xGMI when it is another GPU), processed there, and the result
  copied back into place on the caller's device;
* checksum mismatches are raised after every worker finished, the first one
  in row order, exactly as the single-device call raises it; any other
  worker exception is re-raised likewise (the first in row order).

The same device may appear several times (``devices=[0, 0]``): its entries
are independent workers with their own streams, which is how the tests
exercise the partition on a one-GPU box.  Nothing here is measured on a
multi-GPU node yet.
"""

from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import torch

from . import shard

__all__ = ["normalize_devices", "split_rows", "run_workers", "device_rows", "host_rows"]


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


def device_rows(fn, rows: torch.Tensor, devices):
    """Apply the single-device batch function ``fn(rows_on_dev) -> (y, extra)``
    (y a [b, ...] tensor) to the contiguous row ranges of a device batch
    `rows` on `devices`.  Returns (the results gathered in row order on
    `rows`' device as [B, m], the workers' `extra` values in row order)."""
    devices = normalize_devices(devices)
    home = rows.device
    parts = split_rows(rows.shape[0], len(devices))
    if not parts:
        y, extra = fn(rows)
        return y.reshape(y.shape[0], -1), [extra]
    caller = torch.cuda.current_stream(home)
    ready = torch.cuda.Event()
    ready.record(caller)

    def work(g, lo, hi):
        dev = devices[g]
        with torch.cuda.device(dev):
            s = torch.cuda.Stream(device=dev)
            s.wait_event(ready)  # the caller's producers of `rows` are done
            with torch.cuda.stream(s):
                part = rows[lo:hi]
                if dev != home:
                    part = part.to(dev, non_blocking=True)
                y, extra = fn(part)
                y = y.reshape(y.shape[0], -1)
                if dev != home:
                    y = y.to(home, non_blocking=True)
                done = torch.cuda.Event()
                done.record(s)
            done.synchronize()
            if dev != home:  # the peer copy may run on the home device's stream
                torch.cuda.current_stream(home).synchronize()
            return y, extra

    res = run_workers([lambda g=g, lo=lo, hi=hi: work(g, lo, hi) for g, lo, hi in parts])
    ys = [r[0] for r in res]
    out = ys[0] if len(ys) == 1 else torch.cat(ys)
    return out, [r[1] for r in res]


def host_rows(fn, nrows: int, devices) -> list:
    """Run ``fn(device, lo, hi)`` -- a single-device streaming call over host
    rows [lo, hi) -- for every worker's contiguous range, one thread each;
    results in row order (the first exception in row order re-raised)."""
    devices = normalize_devices(devices)
    parts = split_rows(nrows, len(devices))
    return run_workers([lambda g=g, lo=lo, hi=hi: fn(devices[g], lo, hi) for g, lo, hi in parts])
