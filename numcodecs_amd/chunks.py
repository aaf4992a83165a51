"""Zarr-style chunk pipelines over many equal-size chunks (SURVEY.md §8f
row 1: the caller around the hot path).

Zarr calls ``codec.encode(chunk)`` once per chunk per filter, host buffer in,
host buffer out.  On a GPU that is launch- and PCIe-bound, so this module
offers the same result for a whole batch:

* :func:`encode_chunks` / :func:`decode_chunks` apply a filter chain (the
  ``filters`` + checksum list of a Zarr array, in encode order) to every row
  of a device batch ``[B, ...]``.  Each step runs batched where its kernel
  allows: elementwise codecs (BitRound, Quantize, FixedScaleOffset, AsType)
  on the flattened batch in one launch, Shuffle and the checksums as batch
  launches, Delta as a batch launch with one scan per chunk; PackBits
  (whose chunk boundaries and header matter) row by row.
* :func:`host_encode_chunks` / :func:`host_decode_chunks` stream host
  chunks through that chain: slices flow through a ring of device buffers on
  three role streams (H2D / kernels / D2H), so both PCIe directions and the
  kernels overlap (:func:`stream_chunks`).

Every row comes out byte-identical to applying the codecs one after another
to that chunk (tests/test_gpu_chunks.py), which the other tests pin to the
reference.
"""

from __future__ import annotations

import math

import torch

from . import _native, batch, multi
from .astype import AsType
from .bitround import BitRound
from .checksum32 import CRC32, CRC32C, Adler32, JenkinsLookup3
from .compat import is_device_tensor, torch_dtype
from .delta import Delta
from .fixedscaleoffset import FixedScaleOffset
from .fletcher32 import Fletcher32, _mismatch
from .quantize import Quantize
from .shuffle import Shuffle

__all__ = ["encode_chunks", "decode_chunks", "stream_chunks", "host_encode_chunks", "host_decode_chunks"]

_ELEMENTWISE = (BitRound, Quantize, FixedScaleOffset, AsType)
_CK32 = (CRC32, CRC32C, Adler32)


def _rows(x: torch.Tensor, b: int) -> torch.Tensor:
    """[B, ...] (or flat B*m) device tensor -> [B, m] uint8 contiguous rows."""
    x = x.contiguous()
    raw = x.view(torch.uint8) if x.numel() else x.new_empty(0, dtype=torch.uint8)
    return raw.reshape(b, -1) if raw.numel() else raw.reshape(b, 0)


def _per_row(fn, x: torch.Tensor) -> torch.Tensor:
    return torch.stack([_rows(fn(x[i]), 1)[0] for i in range(x.shape[0])])


def _raise_first(c, sums, stored):
    bad = torch.nonzero(sums != stored)
    if not bad.numel():
        return
    i = int(bad[0, 0])
    got, exp = int(sums[i]) & 0xFFFFFFFF, int(stored[i]) & 0xFFFFFFFF
    if isinstance(c, Fletcher32):
        raise _mismatch(got, exp)
    if isinstance(c, JenkinsLookup3):
        raise RuntimeError(
            f"The Bob Jenkin's lookup3 checksum of the data ({got}) did not"
            f" match the expected checksum ({exp}).\n"
            "This could be a sign that the data has been corrupted."
        )
    raise RuntimeError(f"Stored and computed {c.codec_id} checksum do not match. Stored: {exp}. Computed: {got}.")


def _verify(c, sums, stored, pending):
    """Check now (one host sync), or queue the comparison when a streaming
    caller collects them (`pending` list) and checks after the last slice."""
    if pending is None:
        _raise_first(c, sums, stored)
    else:
        pending.append((c, sums, stored))


def _fletcher32_decode_rows(rows: torch.Tensor, pending=None) -> torch.Tensor:
    """Fletcher32.decode of every row (fletcher32.pyx:91-115): one pass that
    checksums the payloads, reads the footers and compacts the payloads."""
    b, m = rows.shape
    if m <= 4:
        raise IndexError("Out of bounds on buffer access (axis 0)")
    payload, sums, stored = batch.fletcher32_decode_chunks(rows)
    _verify(Fletcher32(), sums, stored, pending)
    return payload


def _encode_step(c, x: torch.Tensor) -> torch.Tensor:
    b = x.shape[0]
    if isinstance(c, _ELEMENTWISE):
        y = c.encode(x.reshape(-1))
        return y.reshape(b, -1)
    rows = _rows(x, b)
    if isinstance(c, Shuffle):
        return batch.shuffle_chunks(rows, c.elementsize)
    if isinstance(c, _CK32):
        return batch.checksum32_encode_chunks(rows, c.codec_id, location=c.location)
    if isinstance(c, JenkinsLookup3):
        return batch.checksum32_encode_chunks(rows, "jenkins_lookup3", value=c.initval, prefix=c.prefix)
    if isinstance(c, Fletcher32):
        return batch.fletcher32_encode_chunks(rows)
    if isinstance(c, Delta):
        return batch.delta_chunks(rows, c, encode=True)
    return _per_row(c.encode, x)


def _checksum32_decode_rows(c, rows: torch.Tensor, pending=None) -> torch.Tensor:
    """Checksum32.decode of every row (checksum32.py:64-88): one pass that
    checksums each payload, reads the stored value and compacts the payloads
    into an aligned contiguous batch for the next codec."""
    b, m = rows.shape
    if m < 4:
        raise ValueError("Input buffer is too short to contain a 32-bit checksum.")
    if isinstance(c, JenkinsLookup3):
        payload, sums, stored = batch.checksum32_decode_chunks(rows, "jenkins_lookup3", value=c.initval,
                                                               prefix=c.prefix)
    else:
        payload, sums, stored = batch.checksum32_decode_chunks(rows, c.codec_id, location=c.location)
    _verify(c, sums, stored, pending)
    return payload


def _decode_step(c, x: torch.Tensor, pending=None) -> torch.Tensor:
    b = x.shape[0]
    if isinstance(c, _ELEMENTWISE):
        y = c.decode(x.reshape(-1))
        return y.reshape(b, -1)
    rows = _rows(x, b)
    if isinstance(c, Shuffle):
        return batch.unshuffle_chunks(rows, c.elementsize)
    if isinstance(c, (_CK32, JenkinsLookup3)):
        return _checksum32_decode_rows(c, rows, pending)
    if isinstance(c, Fletcher32):
        return _fletcher32_decode_rows(rows, pending)
    if isinstance(c, Delta):
        return batch.delta_chunks(rows, c, encode=False)
    return _per_row(c.decode, x)


def _fused_c4_at(codecs, i):
    """True when codecs[i:i+3] is FixedScaleOffset -> Delta -> Shuffle that the
    fused kernels implement (batch._c4_scalars)."""
    return i + 3 <= len(codecs) and batch._c4_scalars(*codecs[i:i + 3]) is not None


def encode_chunks(codecs, chunks, devices=None, allow_peer_copy=False):
    """Encode every row of the device batch `chunks` ([B, ...], typed as the
    first codec expects) through `codecs` in order; returns [B, m].  A
    FixedScaleOffset -> Delta -> Shuffle run encodes in one fused launch.

    Multi-GPU (numcodecs_amd.multi): `chunks` may be a list of per-device
    resident shards (one tensor per GPU); each is encoded on its own device
    and the list of results is returned, each left on its device.
    ``devices=[...]`` with one tensor splits its row ranges over workers of
    that tensor's device; other GPUs are refused unless
    ``allow_peer_copy=True`` (rows copied over xGMI and back)."""
    codecs = list(codecs)
    if isinstance(chunks, (list, tuple)):
        ys, _ = multi.device_shards(lambda d: (encode_chunks(codecs, d), None), chunks)
        return ys
    if not is_device_tensor(chunks) or chunks.dim() < 1:
        raise TypeError("encode_chunks takes a device tensor [B, ...] or a list of them")
    if devices is not None:
        y, _ = multi.device_rows(lambda d: (encode_chunks(codecs, d), None), chunks, devices, allow_peer_copy)
        return y
    x = chunks.reshape(chunks.shape[0], -1)
    i = 0
    while i < len(codecs):
        if _fused_c4_at(codecs, i):
            y = batch.fso_delta_shuffle_encode_chunks(_rows(x, x.shape[0]), *codecs[i:i + 3])
            if y is not None:
                x = y
                i += 3
                continue
        x = _encode_step(codecs[i], x)
        i += 1
    return x


def decode_chunks(codecs, chunks, _pending=None, devices=None, allow_peer_copy=False):
    """Invert :func:`encode_chunks` (codecs given in encode order); raises
    the codec's RuntimeError if any row's checksum does not match.
    Resident shards / ``devices=[...]``: as for encode_chunks; the checksum
    comparisons of all workers are made after they finish, chain step by
    chain step and row range by row range -- the mismatch the one-device
    call would raise."""
    codecs = list(codecs)
    shards = isinstance(chunks, (list, tuple))
    if not shards and (not is_device_tensor(chunks) or chunks.dim() < 1):
        raise TypeError("decode_chunks takes a device tensor [B, ...] or a list of them")
    if shards or devices is not None:
        def one(d):
            pend = []
            return decode_chunks(codecs, d, pend), pend

        if shards:
            y, pends = multi.device_shards(one, chunks)
        else:
            y, pends = multi.device_rows(one, chunks, devices, allow_peer_copy)
        steps = [[p[k] for p in pends] for k in range(len(pends[0]))] if pends and pends[0] else []
        for step in steps:
            for c, sums, stored in step:
                if _pending is None:
                    _raise_first(c, sums, stored)
                else:
                    _pending.append((c, sums, stored))
        return y
    x = chunks.reshape(chunks.shape[0], -1)
    i = len(codecs)
    while i > 0:
        if i >= 3 and _fused_c4_at(codecs, i - 3):
            y = batch.fso_delta_shuffle_decode_chunks(_rows(x, x.shape[0]), *codecs[i - 3:i])
            if y is not None:
                x = y.view(torch_dtype(codecs[i - 3].dtype))  # typed as FixedScaleOffset.decode returns
                i -= 3
                continue
        x = _decode_step(codecs[i - 1], x, _pending)
        i -= 1
    return x


# ---------------------------------------------------------------------------
# host <-> device streaming
# ---------------------------------------------------------------------------
def _default_slice(host_in: torch.Tensor, host_out: torch.Tensor) -> int:
    """~64 MiB of input rows, rounded down to a row count whose slices start
    64-B aligned in both host tensors: DMA from a pinned range that is only
    4-B aligned runs ~30 GiB/s instead of ~42 (MI355X, 4 MiB + 4-B encoded
    rows, tools/probe_e2e_chain.py)."""
    row_in = host_in.shape[1] * host_in.element_size()
    row_out = host_out.shape[1] * host_out.element_size()
    rows = max(1, (64 << 20) // max(row_in, 1))
    g = math.lcm(64 // math.gcd(row_in, 64), 64 // math.gcd(row_out, 64))
    return max(g, (rows + g // 2) // g * g)


def stream_chunks(host_in: torch.Tensor, host_out: torch.Tensor, fn, slice_chunks: "int | None" = None,
                  nslots: int = 3, device=None) -> None:
    """Run ``fn(dev_in_rows) -> dev_out_rows`` over a [B, n] host batch into
    a [B, m] host batch, slice by slice.

    Slices of `slice_chunks` rows flow through a ring of `nslots` device input
    buffers and three role streams -- H2D copies, kernels (`fn` runs on this
    stream), D2H copies -- ordered by events, so both PCIe directions
    (separate SDMA engines) and the kernels of different slices overlap.  Pin
    both host tensors for asynchronous DMA.  The default slice is ~64 MiB:
    measured on MI355X (tools/probe_e2e.py) 64-128 MiB slices reach 43-44
    GiB/s host->host against 45 GiB/s of concurrent H2D+D2H, 8-16 MiB slices
    ~24 GiB/s.  Returns when host_out is complete.
    """
    _native.require_device()
    if host_in.device.type != "cpu" or host_out.device.type != "cpu":
        raise TypeError("stream_chunks takes CPU tensors (pinned for overlap)")
    if host_in.dim() != 2 or host_out.dim() != 2 or host_in.shape[0] != host_out.shape[0]:
        raise ValueError("host_in [B, n] and host_out [B, m] must have the same number of rows")
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    b, n = host_in.shape
    if b == 0:
        return
    if slice_chunks is None:
        slice_chunks = _default_slice(host_in, host_out)
    slice_chunks = max(1, min(slice_chunks, b))
    nslots = max(1, nslots)
    with torch.cuda.device(device):
        cur = torch.cuda.current_stream(device)
        h2d, comp, d2h = (torch.cuda.Stream(device=device) for _ in range(3))
        dev_in = [torch.empty((slice_chunks, n), dtype=host_in.dtype, device=device) for _ in range(nslots)]
        for s in (h2d, comp, d2h):
            s.wait_stream(cur)  # the ring was allocated on the current stream
        loaded = [torch.cuda.Event() for _ in range(nslots)]
        done = [torch.cuda.Event() for _ in range(nslots)]
        free = [None] * nslots
        outs = [None] * nslots  # keep each slice's output alive until its D2H is done
        for k, lo in enumerate(range(0, b, slice_chunks)):
            hi = min(b, lo + slice_chunks)
            i = k % nslots
            di = dev_in[i][: hi - lo]
            if free[i] is not None:
                h2d.wait_event(free[i])  # the slot's previous D2H has drained it
            with torch.cuda.stream(h2d):
                di.copy_(host_in[lo:hi], non_blocking=True)
                loaded[i].record(h2d)
            comp.wait_event(loaded[i])
            with torch.cuda.stream(comp):
                do = fn(di)
                done[i].record(comp)
            d2h.wait_event(done[i])
            with torch.cuda.stream(d2h):
                host_out[lo:hi].copy_(do, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(d2h)
                free[i] = ev
            do.record_stream(d2h)  # allocated on comp, read by d2h
            outs[i] = do
        d2h.synchronize()
        for s in (h2d, comp):
            s.synchronize()
        cur.wait_stream(d2h)


def _host_rows(x, name):
    if not isinstance(x, torch.Tensor) or x.device.type != "cpu" or x.dim() < 1:
        raise TypeError(f"{name} must be a CPU tensor [B, ...]")
    return x.reshape(x.shape[0], -1)


def host_encode_chunks(codecs, host_in: torch.Tensor, host_out: "torch.Tensor | None" = None,
                       slice_chunks: "int | None" = None, nslots: int = 3, device=None,
                       devices=None) -> torch.Tensor:
    """Encode a batch of host chunks [B, ...] (typed as the first codec
    expects; pin it) through `codecs` on the GPU, streamed; returns the
    [B, m] uint8 host batch (pinned when allocated here).  ``devices=[...]``
    streams contiguous row ranges through those GPUs at once, one worker
    thread and ring each (the host path is PCIe-bound per GPU)."""
    codecs = list(codecs)
    src = _host_rows(host_in, "host_in")
    if devices is not None:
        devs = multi.normalize_devices(devices)
        if host_out is None:
            probe = encode_chunks(codecs, src[:1].to(devs[0]))
            host_out = torch.empty((src.shape[0], _rows(probe, 1).shape[1]), dtype=torch.uint8, pin_memory=True)
        out = _host_rows(host_out, "host_out")
        multi.host_rows(lambda dev, lo, hi: host_encode_chunks(codecs, src[lo:hi], out[lo:hi], slice_chunks, nslots,
                                                               dev), src.shape[0], devs)
        return host_out
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    # encoded row size: run the chain on the first chunk
    probe = encode_chunks(codecs, src[:1].to(device))
    m = _rows(probe, 1).shape[1]
    if host_out is None:
        host_out = torch.empty((src.shape[0], m), dtype=torch.uint8, pin_memory=True)
    out = _host_rows(host_out, "host_out")
    if out.shape != (src.shape[0], m) or out.dtype != torch.uint8:
        raise ValueError(f"host_out must be uint8 [{src.shape[0]}, {m}]")
    stream_chunks(src, out, lambda d: _rows(encode_chunks(codecs, d), d.shape[0]), slice_chunks, nslots, device)
    return host_out


def host_decode_chunks(codecs, host_in: torch.Tensor, host_out: torch.Tensor,
                       slice_chunks: "int | None" = None, nslots: int = 3, device=None,
                       devices=None) -> torch.Tensor:
    """Decode a [B, m] uint8 host batch of encoded chunks through `codecs`
    (given in encode order) into `host_out` ([B, ...] host tensor of the
    decoded chunks' dtype and size); checksums are verified.  ``devices``:
    as for host_encode_chunks (a mismatch is raised after every worker
    finished, the first row range's first)."""
    codecs = list(codecs)
    src = _host_rows(host_in, "host_in")
    out = _host_rows(host_out, "host_out")
    if devices is not None:
        multi.host_rows(lambda dev, lo, hi: host_decode_chunks(codecs, src[lo:hi], out[lo:hi], slice_chunks, nslots,
                                                               dev), src.shape[0], devices)
        return host_out
    pending = []  # checksum comparisons, checked once after the stream (no per-slice host sync)

    def fn(d):
        y = decode_chunks(codecs, d, pending)
        return y.contiguous().reshape(d.shape[0], -1).view(out.dtype) if y.dtype != out.dtype else y.reshape(d.shape[0], -1)

    stream_chunks(src, out, fn, slice_chunks, nslots, device)
    for c, sums, stored in pending:
        _raise_first(c, sums, stored)
    return host_out
