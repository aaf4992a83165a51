"""Batched chunk API and fused filter pipelines.

numcodecs is called by Zarr once per chunk (``codec.encode(chunk)``), which
on a GPU is launch-bound for small chunks (a 1 MiB chunk moves in ~0.3 us at
HBM rate, far less than a kernel launch).  This module adds what the
reference has no counterpart for:

* ``*_chunks`` functions over a ``[B, chunk_bytes]`` batch of equal-size
  chunks in one launch (chunk b at row b; rows may be padded);
* :class:`FilterPipeline`, a Zarr-style filter chain (+ optional checksum)
  that recognises fusable sequences and runs them as single kernels:
  ``BitRound -> Shuffle`` (one pass), ``Shuffle -> Fletcher32`` (one pass,
  checksum of the shuffled bytes computed in registers while they are
  stored), and decodes ``Fletcher32 -> Shuffle`` with the verification fused
  into the unshuffle.  Any other chain runs codec by codec on the device.

Results are identical to applying the reference codecs one after another.
"""

from __future__ import annotations

import numpy as np
import torch

from . import _native, _ops, multi
from ._native import check, lib
from .bitround import BitRound, max_bits
from .compat import device_out_bytes, ensure_contiguous_ndarray, is_device_tensor
from .delta import Delta, check_first_elements, decode_loop_dtype
from .fixedscaleoffset import FixedScaleOffset, _resolve
from .fletcher32 import Fletcher32, _mismatch
from .shuffle import Shuffle

__all__ = [
    "FilterPipeline",
    "fletcher32_chunks",
    "shuffle_chunks",
    "unshuffle_chunks",
    "shuffle_fletcher32_encode_chunks",
    "fletcher32_unshuffle_decode_chunks",
    "encoded_stride",
    "host_pipeline",
    "checksum32_chunks",
    "checksum32_encode_chunks",
    "checksum32_decode_chunks",
    "fletcher32_encode_chunks",
    "fletcher32_decode_chunks",
    "fso_delta_shuffle_encode_chunks",
    "fso_delta_shuffle_decode_chunks",
]

_CK_KINDS = {
    "crc32": (_native.MC_CK_CRC32, 0),
    "crc32c": (_native.MC_CK_CRC32C, 0),
    "adler32": (_native.MC_CK_ADLER32, 1),
    "jenkins_lookup3": (_native.MC_CK_JENKINS, 0),
}


def _as_rows(chunks: torch.Tensor) -> torch.Tensor:
    """[B, ...] device tensor -> [B, row_bytes] uint8 view (rows contiguous)."""
    if not is_device_tensor(chunks):
        raise TypeError("batched chunk functions take a device tensor [B, ...]")
    if chunks.dim() < 1:
        raise ValueError("expected a batch dimension")
    b = chunks.shape[0]
    rows = chunks.reshape(b, -1) if chunks.numel() else chunks.reshape(b, 0)
    if rows.stride(1) != 1:
        raise ValueError("each chunk must be contiguous")
    rows = rows.view(torch.uint8) if rows.element_size() != 1 or rows.dtype != torch.uint8 else rows
    return rows


def encoded_stride(chunk_bytes: int) -> int:
    """Row stride of an encoded batch: payload + 4-byte footer, padded to 256 B
    so that every row stays 16-B aligned for the fused kernels."""
    return (chunk_bytes + 4 + 255) // 256 * 256


def shuffle_chunks(chunks, elementsize, out=None):
    """Shuffle(elementsize).encode of every chunk of a [B, ...] device batch."""
    rows = _as_rows(chunks)
    b, n = rows.shape
    out = torch.empty((b, n), dtype=torch.uint8, device=rows.device) if out is None else _as_rows(out)
    if b and n:
        _ops.shuffle_batch(rows, rows.stride(0), out, out.stride(0), b, n, elementsize, True)
    return out


def unshuffle_chunks(chunks, elementsize, out=None):
    """Shuffle(elementsize).decode of every chunk of a [B, ...] device batch."""
    rows = _as_rows(chunks)
    b, n = rows.shape
    out = torch.empty((b, n), dtype=torch.uint8, device=rows.device) if out is None else _as_rows(out)
    if b and n:
        _ops.shuffle_batch(rows, rows.stride(0), out, out.stride(0), b, n, elementsize, False)
    return out


def delta_chunks(chunks, delta, encode=True, out=None):
    """Delta(dtype, astype).encode (or .decode) of every chunk of a [B, ...]
    device batch, each chunk independently (its own first element / running
    sum), in one launch; returns [B, m] uint8 rows.  Rows are the chunks' raw
    bytes (dtype elements for encode, astype elements for decode)."""
    rows = _as_rows(chunks)
    b, nb = rows.shape
    src_t, dst_t = (delta.dtype, delta.astype) if encode else (delta.astype, delta.dtype)
    if nb % src_t.itemsize:
        raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
    n = nb // src_t.itemsize
    if encode and n == 0 and b:
        raise IndexError("index 0 is out of bounds for axis 0 with size 0")
    if encode and b:
        check_first_elements(rows[:, : src_t.itemsize], delta.dtype, delta.astype)
    loop = None if encode else decode_loop_dtype(delta.astype, delta.dtype)
    m = n * dst_t.itemsize
    out = torch.empty((b, m), dtype=torch.uint8, device=rows.device) if out is None else _as_rows(out)
    if loop is not None:
        # a pair decoded through its loop dtype (delta.decode_loop_dtype):
        # the running sums of every row in `loop`, then one cast of them all
        if b and n:
            sums = delta_chunks(rows, Delta(dtype=loop, astype=delta.astype), encode=False)
            if out.is_contiguous():  # one cast straight into the caller's rows
                _ops.cast(sums, out, b * n, loop, delta.dtype)
            else:
                cast = torch.empty((b, m), dtype=torch.uint8, device=rows.device)
                _ops.cast(sums, cast, b * n, loop, delta.dtype)
                out.copy_(cast)
        return out
    if not encode and b and nb >= _LARGE_ROW and rows.data_ptr() % 16 == 0 and \
            rows.stride(0) % 16 == 0 and out.stride(0) % 16 == 0 and out.data_ptr() % 16 == 0:
        # huge rows: each decoded by the whole chip (mc_delta_decode), not by
        # one workgroup of the row kernel (16 x 64 MiB f4<-i2: 7.6 ms)
        for i in range(b):
            _ops.delta_decode(rows[i], out[i], n, delta.astype, delta.dtype)
        return out
    if b and n:
        _ops.delta_batch(rows, rows.stride(0), out, out.stride(0), b, n, delta.dtype, delta.astype, encode)
    return out


def fletcher32_chunks(chunks, nbytes=None) -> torch.Tensor:
    """Fletcher32 of every chunk (first `nbytes` of each row); int64 [B]."""
    rows = _as_rows(chunks)
    b, n = rows.shape
    nbytes = n if nbytes is None else nbytes
    res = torch.empty(b, dtype=torch.int32, device=rows.device)
    if b:
        _native.require_device()
        with torch.cuda.device(rows.device):
            ws = _ops.workspace(lib.mc_fletcher32_batch_workspace(b, nbytes), rows)
            check(lib.mc_fletcher32_batch(rows.data_ptr(), rows.stride(0), b, nbytes, res.data_ptr(),
                                          ws.data_ptr(), ws.numel(), _ops.stream(rows)),
                  "mc_fletcher32_batch")
    return res.to(torch.int64) & 0xFFFFFFFF


def fletcher32_encode_chunks(chunks, out=None):
    """Fletcher32.encode of every chunk in one pass (fletcher32.pyx:75-89):
    the [B, row_bytes + 4] batch of payload ++ LE32 checksum (or `out`)."""
    rows = _as_rows(chunks)
    b, n = rows.shape
    if n == 0:  # the reference indexes b_mv[0] of an empty view
        raise IndexError("Out of bounds on buffer access (axis 0)")
    out = torch.empty((b, n + 4), dtype=torch.uint8, device=rows.device) if out is None else _as_rows(out)
    if out.shape[0] != b or out.shape[1] < n + 4:
        raise ValueError("output rows must hold chunk_bytes + 4 bytes")
    if b:
        _native.require_device()
        with torch.cuda.device(rows.device):
            ws = _ops.workspace(lib.mc_fletcher32_batch_workspace(b, n), rows)
            check(lib.mc_fletcher32_encode_batch(rows.data_ptr(), rows.stride(0), out.data_ptr(), out.stride(0), b, n,
                                                 ws.data_ptr(), ws.numel(), _ops.stream(rows)),
                  "mc_fletcher32_encode_batch")
    return out


def fletcher32_decode_chunks(chunks):
    """Fletcher32.decode of every encoded row (payload + LE32 footer) in one
    pass: ``(payloads, sums, stored)`` -- the payloads compacted into a fresh
    contiguous [B, row_bytes - 4] batch, the computed and the stored checksums
    (device int32 [B], uint32 bit patterns).  The caller compares and raises
    (fletcher32.pyx:106-113); nothing here syncs the host."""
    rows = _as_rows(chunks)
    b, m = rows.shape
    if m < 4:
        raise IndexError("Out of bounds on buffer access (axis 0)")
    out = torch.empty((b, m - 4), dtype=torch.uint8, device=rows.device)
    pairs = torch.empty((max(b, 1), 2), dtype=torch.int32, device=rows.device)
    if b:
        _native.require_device()
        with torch.cuda.device(rows.device):
            ws = _ops.workspace(lib.mc_fletcher32_batch_workspace(b, m - 4), rows)
            check(lib.mc_fletcher32_decode_batch(rows.data_ptr(), rows.stride(0), out.data_ptr(), m - 4, b, m,
                                                 pairs.data_ptr(), ws.data_ptr(), ws.numel(), _ops.stream(rows)),
                  "mc_fletcher32_decode_batch")
    return out, pairs[:b, 0], pairs[:b, 1]


def checksum32_chunks(chunks, codec_id, nbytes=None, value=None, prefix=None) -> torch.Tensor:
    """`codec_id` checksum ('crc32', 'crc32c', 'adler32', 'jenkins_lookup3')
    of every chunk (first `nbytes` of each row), one launch; int64 [B].
    `value` defaults to the codec's own seed (0, or 1 for adler32); `prefix`
    (jenkins_lookup3 only) is hashed before every chunk."""
    kind, default = _CK_KINDS[codec_id]
    rows = _as_rows(chunks)
    b, n = rows.shape
    nbytes = n if nbytes is None else nbytes
    if b == 0:
        return torch.empty(0, dtype=torch.int64, device=rows.device)
    res = _ops.checksum32(kind, rows, rows.stride(0), b, nbytes, default if value is None else value, prefix)
    return res.to(torch.int64) & 0xFFFFFFFF


def checksum32_encode_chunks(chunks, codec_id, location=None, out=None, value=None, prefix=None):
    """Checksum32.encode of every chunk in one launch: rows of
    ``chunk_bytes + 4`` (checksum at the codec's default location, or
    `location`).  Returns the [B, chunk_bytes + 4] uint8 batch (or `out`)."""
    kind, default = _CK_KINDS[codec_id]
    if location is None:
        location = "end" if codec_id in ("crc32c", "jenkins_lookup3") else "start"
    if location not in ("start", "end") or (codec_id == "jenkins_lookup3" and location != "end"):
        raise ValueError(f"Invalid checksum location: {location}")
    rows = _as_rows(chunks)
    b, n = rows.shape
    out = torch.empty((b, n + 4), dtype=torch.uint8, device=rows.device) if out is None else _as_rows(out)
    if out.shape[1] < n + 4:
        raise ValueError("output rows must hold chunk_bytes + 4 bytes")
    if b:
        loc = _native.MC_CK_START if location == "start" else _native.MC_CK_END
        _ops.checksum32_encode(kind, rows, rows.stride(0), out, out.stride(0), b, n,
                               default if value is None else value, loc, prefix)
    return out


def checksum32_decode_chunks(chunks, codec_id, location=None, value=None, prefix=None):
    """Checksum32.decode of every encoded row in one pass: returns
    ``(payloads, sums, stored)`` -- the [B, row_bytes - 4] payloads compacted
    into a fresh contiguous batch, the computed checksums and the stored ones
    (device int32 [B], uint32 bit patterns).  The caller compares and raises
    (checksum32.py:79-87); nothing here syncs the host."""
    kind, default = _CK_KINDS[codec_id]
    if location is None:
        location = "end" if codec_id in ("crc32c", "jenkins_lookup3") else "start"
    if location not in ("start", "end") or (codec_id == "jenkins_lookup3" and location != "end"):
        raise ValueError(f"Invalid checksum location: {location}")
    rows = _as_rows(chunks)
    b, m = rows.shape
    if m < 4:
        raise ValueError("Input buffer is too short to contain a 32-bit checksum.")
    out = torch.empty((b, m - 4), dtype=torch.uint8, device=rows.device)
    if b == 0:
        z = torch.empty(0, dtype=torch.int32, device=rows.device)
        return out, z, z
    loc = _native.MC_CK_START if location == "start" else _native.MC_CK_END
    sums, stored = _ops.checksum32_decode(kind, rows, rows.stride(0), out if m > 4 else None, m - 4, b, m,
                                          default if value is None else value, loc, prefix)
    return out, sums, stored


def shuffle_fletcher32_encode_chunks(chunks, elementsize, out=None):
    """Per chunk: Shuffle(elementsize).encode then Fletcher32.encode, fused.

    Returns a [B, encoded_stride(chunk_bytes)] uint8 tensor; row b holds the
    chunk_bytes + 4 encoded bytes (the rest of the row is padding).
    """
    rows = _as_rows(chunks)
    b, n = rows.shape
    stride = encoded_stride(n)
    if out is None:
        out = torch.empty((b, stride), dtype=torch.uint8, device=rows.device)
    if b:
        _native.require_device()
        with torch.cuda.device(rows.device):
            ws = _ops.workspace(lib.mc_shuffle_fletcher32_workspace(b, n, elementsize), rows)
            check(lib.mc_shuffle_fletcher32_encode_batch(
                rows.data_ptr(), rows.stride(0), out.data_ptr(), out.stride(0), b, n, elementsize,
                ws.data_ptr(), ws.numel(), _ops.stream(rows)), "mc_shuffle_fletcher32_encode_batch")
    return out


def fletcher32_unshuffle_decode_chunks(encoded, chunk_bytes, elementsize, out=None, check_sums=True):
    """Per chunk: Fletcher32.decode (verify) then Shuffle(elementsize).decode,
    fused.  Raises RuntimeError (the reference's message, first bad chunk) on
    a checksum mismatch when `check_sums`; returns (decoded [B, chunk_bytes],
    status [B, 2] = (computed, stored))."""
    rows = _as_rows(encoded)
    b = rows.shape[0]
    if out is None:
        out = torch.empty((b, chunk_bytes), dtype=torch.uint8, device=rows.device)
    status = torch.empty((b, 2), dtype=torch.int32, device=rows.device)
    if b:
        _native.require_device()
        with torch.cuda.device(rows.device):
            ws = _ops.workspace(lib.mc_shuffle_fletcher32_workspace(b, chunk_bytes, elementsize), rows)
            check(lib.mc_fletcher32_unshuffle_batch(
                rows.data_ptr(), rows.stride(0), out.data_ptr(), out.stride(0), b, chunk_bytes,
                elementsize, status.data_ptr(), ws.data_ptr(), ws.numel(), _ops.stream(rows)),
                "mc_fletcher32_unshuffle_batch")
    if check_sums and b:
        # one compare kernel, one reduction and ONE readback on the good path
        # (int32 equality is the equality of the 32-bit sums)
        bad = status[:, 0] != status[:, 1]
        if bool(bad.any()):
            i = int(bad.nonzero()[0, 0])
            st = status[i].to(torch.int64) & 0xFFFFFFFF
            raise _mismatch(int(st[0]), int(st[1]))
    return out, status


class FilterPipeline:
    """A Zarr-style chain of filters applied in order on encode and in
    reverse on decode, on device tensors, fusing what it can.

    >>> pipe = FilterPipeline([BitRound(10), Shuffle(4)])        # doctest: +SKIP
    >>> enc = pipe.encode(x_f32_on_device)                        # doctest: +SKIP
    """

    def __init__(self, codecs):
        self.codecs = list(codecs)

    # fusable patterns ------------------------------------------------------
    @staticmethod
    def _is_bitround_shuffle(a, b, itemsize):
        return isinstance(a, BitRound) and isinstance(b, Shuffle) and b.elementsize == itemsize

    def encode(self, buf):
        x = buf
        i = 0
        cs = self.codecs
        while i < len(cs):
            c = cs[i]
            nxt = cs[i + 1] if i + 1 < len(cs) else None
            if (
                isinstance(c, BitRound)
                and is_device_tensor(x)
                and x.dtype in (torch.float16, torch.float32, torch.float64)
                and nxt is not None
                and self._is_bitround_shuffle(c, nxt, x.element_size())
            ):
                x = _bitround_shuffle(c, x)
                i += 2
                continue
            if (
                isinstance(c, Shuffle)
                and isinstance(nxt, Fletcher32)
                and is_device_tensor(x)
                and c.elementsize > 1
            ):
                x = _shuffle_fletcher32(c, x)
                i += 2
                continue
            if i + 2 < len(cs) and is_device_tensor(x):
                fused = _fso_delta_shuffle_encode(c, nxt, cs[i + 2], x)
                if fused is not None:
                    x = fused
                    i += 3
                    continue
            x = c.encode(x)
            i += 1
        return x

    def decode(self, buf, out=None):
        from .compat import ndarray_copy

        x = buf
        cs = self.codecs[::-1]
        i = 0
        while i < len(cs):
            c = cs[i]
            nxt = cs[i + 1] if i + 1 < len(cs) else None
            if (
                isinstance(c, Fletcher32)
                and isinstance(nxt, Shuffle)
                and is_device_tensor(x)
                and nxt.elementsize > 1
            ):
                x = _fletcher32_unshuffle(nxt, x)
                i += 2
                continue
            if i + 2 < len(cs) and is_device_tensor(x):
                # the chain's last stage decodes straight into a device `out`
                direct = _c4_direct_out(cs[i + 2], x, out) if i + 3 == len(cs) else None
                fused = _fso_delta_shuffle_decode(cs[i + 2], nxt, c, x, direct)
                if fused is not None:
                    x = fused
                    i += 3
                    if i == len(cs):
                        return out if direct is not None else ndarray_copy(x, out)
                    continue
            if i == len(cs) - 1:
                return c.decode(x, out=out)
            x = c.decode(x)
            i += 1
        return ndarray_copy(x, out)


_C4_FLOATS = ("<f4", "<f8")
_C4_INTS = ("<i2", "<u2", "<i4", "<u4")


def _c4_scalars(fso, delta, sh):
    """Scalars of the fused FSO -> Delta -> Shuffle path, or None when the
    chain is not the one the fused kernels implement (numpy must compute FSO
    encode in the float dtype and decode in float64)."""
    if not (isinstance(fso, FixedScaleOffset) and isinstance(delta, Delta) and isinstance(sh, Shuffle)):
        return None
    d, a = fso.dtype, fso.astype
    if d.str not in _C4_FLOATS or a.str not in _C4_INTS:
        return None
    if delta.dtype != a or delta.astype != a or sh.elementsize != a.itemsize:
        return None
    try:
        t1, off = _resolve(np.subtract, d, fso.offset)
        t2, sc = _resolve(np.multiply, t1, fso.scale)
        t3, sc3 = _resolve(np.true_divide, a, fso.scale)
        t4, off4 = _resolve(np.add, t3, fso.offset)
    except Exception:
        return None
    if t1 != d or t2 != d or t3 != np.float64 or t4 != np.float64:
        return None
    return float(off), float(sc), float(sc3), float(off4)


def _c4_raw(x: torch.Tensor):
    src = ensure_contiguous_ndarray(x)
    return src.view(torch.uint8) if src.numel() else src.new_empty(0, dtype=torch.uint8)


def _fso_delta_shuffle_encode(fso, delta, sh, x):
    sc4 = _c4_scalars(fso, delta, sh)
    if sc4 is None:
        return None
    raw = _c4_raw(x)
    n, rem = divmod(raw.numel(), fso.dtype.itemsize)
    if rem or n == 0 or n % 16 or raw.data_ptr() % 16:
        return None
    off, sc, _, _ = sc4
    out = torch.empty(n * fso.astype.itemsize, dtype=torch.uint8, device=raw.device)
    _native.require_device()
    with torch.cuda.device(raw.device):
        check(lib.mc_fso_delta_shuffle_encode(raw.data_ptr(), out.data_ptr(), n,
                                              _ops.dtype_code(fso.dtype), _ops.dtype_code(fso.astype),
                                              off, sc, _ops.stream(raw)), "mc_fso_delta_shuffle_encode")
    return out


def _c4_direct_out(fso, x, out):
    """The raw bytes of a caller's device `out` when the fused decode of `x`
    can write its result there (compat.device_out_bytes), else None."""
    if out is None or not isinstance(fso, FixedScaleOffset):
        return None
    raw = _c4_raw(x)
    n, rem = divmod(raw.numel(), fso.astype.itemsize)
    return None if rem else device_out_bytes(out, n * fso.dtype.itemsize, raw)


def _fso_delta_shuffle_decode(fso, delta, sh, x, out=None):
    from .compat import torch_dtype

    sc4 = _c4_scalars(fso, delta, sh)
    if sc4 is None:
        return None
    raw = _c4_raw(x)
    n, rem = divmod(raw.numel(), fso.astype.itemsize)
    if rem or n == 0 or n % 16 or raw.data_ptr() % 16:
        return None
    _, _, sc3, off4 = sc4
    if out is None:
        out = torch.empty(n * fso.dtype.itemsize, dtype=torch.uint8, device=raw.device)
    _native.require_device()
    with torch.cuda.device(raw.device):
        ws = _ops.workspace(lib.mc_fso_delta_shuffle_decode_workspace(n), raw)
        st = _ops.stream(raw)
        check(lib.mc_fso_delta_shuffle_decode(raw.data_ptr(), out.data_ptr(), n,
                                              _ops.dtype_code(fso.astype), _ops.dtype_code(fso.dtype),
                                              sc3, off4, ws.data_ptr(), ws.numel(),
                                              _ops.arrival_ticket(raw, st), st),
              "mc_fso_delta_shuffle_decode")
    return out.view(torch_dtype(fso.dtype))


# rows of at least _LARGE_ROW bytes decode row by row with the single-chunk
# (multi-workgroup) decodes -- a row kernel would give each huge row one
# workgroup (1 x 256 MiB of i2 Delta: 28 ms); for the fused FSO/Delta/Shuffle
# chain only when there are at most _FEW_ROWS of them (more fill the chip
# through the segmented batched decode)
_FEW_ROWS = 4
_LARGE_ROW = 16 << 20


def fso_delta_shuffle_encode_chunks(rows, fso, delta, sh):
    """[FixedScaleOffset, Delta, Shuffle(itemsize(astype))] encode of every row
    of a [B, n * itemsize(dtype)] uint8 device batch in one launch
    (mc_fso_delta_shuffle_encode_batch; each row its own Delta); returns the
    [B, n * itemsize(astype)] encoded rows, or None when the chain or the
    layout is not the fused kernels' (the caller then runs codec by codec)."""
    sc4 = _c4_scalars(fso, delta, sh)
    rows = _as_rows(rows)
    b, nb = rows.shape
    if sc4 is None or b == 0 or nb % fso.dtype.itemsize:
        return None
    n = nb // fso.dtype.itemsize
    if n == 0 or n % 16 or rows.data_ptr() % 16 or (b > 1 and rows.stride(0) % 16):
        return None
    off, sc, _, _ = sc4
    out = torch.empty((b, n * fso.astype.itemsize), dtype=torch.uint8, device=rows.device)
    _native.require_device()
    with torch.cuda.device(rows.device):
        check(lib.mc_fso_delta_shuffle_encode_batch(rows.data_ptr(), rows.stride(0), out.data_ptr(), out.stride(0), b,
                                                    n, _ops.dtype_code(fso.dtype), _ops.dtype_code(fso.astype), off,
                                                    sc, _ops.stream(rows)), "mc_fso_delta_shuffle_encode_batch")
    return out


def fso_delta_shuffle_decode_chunks(rows, fso, delta, sh):
    """Inverse of :func:`fso_delta_shuffle_encode_chunks`: every row (or, for
    few large rows, every segment of a row) decoded in a single pass with a
    running carry (mc_fso_delta_shuffle_decode_batch); [B, n * itemsize(dtype)]
    rows, or None when not fusable."""
    sc4 = _c4_scalars(fso, delta, sh)
    rows = _as_rows(rows)
    b, nb = rows.shape
    if sc4 is None or b == 0 or nb % fso.astype.itemsize:
        return None
    n = nb // fso.astype.itemsize
    if n == 0 or n % 16 or rows.data_ptr() % 16 or (b > 1 and rows.stride(0) % 16):
        return None
    _, _, sc3, off4 = sc4
    out = torch.empty((b, n * fso.dtype.itemsize), dtype=torch.uint8, device=rows.device)
    if b <= _FEW_ROWS and nb >= _LARGE_ROW and out.stride(0) % 16 == 0:
        for i in range(b):  # each row alone fills the chip: the single-chunk two-launch decode
            _fso_delta_shuffle_decode(fso, delta, sh, rows[i], out[i])
        return out
    _native.require_device()
    with torch.cuda.device(rows.device):
        ws = _ops.workspace(lib.mc_fso_delta_shuffle_decode_batch_workspace(b, n), rows)
        check(lib.mc_fso_delta_shuffle_decode_batch(rows.data_ptr(), rows.stride(0), out.data_ptr(), out.stride(0), b,
                                                    n, _ops.dtype_code(fso.astype), _ops.dtype_code(fso.dtype), sc3,
                                                    off4, ws.data_ptr(), ws.numel(), _ops.stream(rows)),
              "mc_fso_delta_shuffle_decode_batch")
    return out


def _bitround_shuffle(br: BitRound, x: torch.Tensor) -> torch.Tensor:
    from .compat import numpy_dtype

    dt = numpy_dtype(x.dtype)
    bits = max_bits[str(dt)]
    if br.keepbits > bits:
        raise ValueError("Keepbits too large for given dtype")
    src = x.contiguous().reshape(-1).view(torch.uint8)
    dst = torch.empty_like(src)
    _ops.bitround_shuffle(src, dst, src.numel() // dt.itemsize, dt.itemsize, br.keepbits)
    return dst


def _shuffle_fletcher32(sh: Shuffle, x: torch.Tensor) -> torch.Tensor:
    src = ensure_contiguous_ndarray(x)
    src = src.view(torch.uint8) if src.numel() else src.new_empty(0, dtype=torch.uint8)
    n = src.numel()
    if n == 0:
        raise IndexError("Out of bounds on buffer access (axis 0)")
    if n % sh.elementsize:
        raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
    out = torch.empty(n + 4, dtype=torch.uint8, device=src.device)
    _native.require_device()
    with torch.cuda.device(src.device):
        ws = _ops.workspace(lib.mc_shuffle_fletcher32_workspace(1, n, sh.elementsize), src)
        check(lib.mc_shuffle_fletcher32_encode_batch(src.data_ptr(), n, out.data_ptr(), n + 4, 1, n,
                                                     sh.elementsize, ws.data_ptr(), ws.numel(),
                                                     _ops.stream(src)),
              "mc_shuffle_fletcher32_encode_batch")
    return out


def _fletcher32_unshuffle(sh: Shuffle, x: torch.Tensor) -> torch.Tensor:
    src = ensure_contiguous_ndarray(x)
    src = src.view(torch.uint8) if src.numel() else src.new_empty(0, dtype=torch.uint8)
    if src.numel() <= 4:
        raise IndexError("Out of bounds on buffer access (axis 0)")
    n = src.numel() - 4
    if n % sh.elementsize:
        raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
    out = torch.empty(n, dtype=torch.uint8, device=src.device)
    status = torch.empty(2, dtype=torch.int32, device=src.device)
    _native.require_device()
    with torch.cuda.device(src.device):
        ws = _ops.workspace(lib.mc_shuffle_fletcher32_workspace(1, n, sh.elementsize), src)
        check(lib.mc_fletcher32_unshuffle_batch(src.data_ptr(), n + 4, out.data_ptr(), n, 1, n,
                                                sh.elementsize, status.data_ptr(), ws.data_ptr(),
                                                ws.numel(), _ops.stream(src)),
              "mc_fletcher32_unshuffle_batch")
    v = status.cpu().numpy().view(np.uint32)
    if v[0] != v[1]:
        raise _mismatch(int(v[0]), int(v[1]))
    return out


def host_pipeline(host_in: torch.Tensor, host_out: torch.Tensor, elementsize: int, encode=True,
                  slice_chunks: "int | None" = None, nslots: int = 3, device=None, devices=None) -> None:
    """Shuffle a batch of chunks that lives in (pinned) host memory.

    The Zarr caller's chunks start and end in host memory (a file or socket
    buffer).  ``host_in``/``host_out`` are [B, chunk_bytes] uint8 CPU tensors
    (pin them for asynchronous DMA).  Slices of `slice_chunks` chunks flow
    through a ring of `nslots` device buffer pairs and three role streams --
    one for H2D copies, one for kernels, one for D2H copies -- ordered by
    events, so both PCIe directions (separate SDMA engines) and the kernels
    of different slices overlap.  Returns when host_out is complete.  The
    default slice is ~64 MiB: measured on MI355X (tools/probe_e2e.py) 64-128
    MiB slices reach 43-44 GiB/s host->host against 45 GiB/s of concurrent
    H2D+D2H, while 8-16 MiB slices drop to ~24 GiB/s.

    ``devices=[...]`` splits the rows into contiguous ranges, one worker
    thread and one such ring per entry (numcodecs_amd.multi.host_rows), so
    several GPUs' PCIe links and kernels work on the batch at once.
    """
    _native.require_device()
    if host_in.device.type != "cpu" or host_out.device.type != "cpu":
        raise TypeError("host_pipeline takes CPU tensors (pinned for overlap)")
    if host_in.shape != host_out.shape or host_in.dim() != 2:
        raise ValueError("host_in and host_out must be [B, chunk_bytes] of equal shape")
    if devices is not None:
        multi.host_rows(lambda dev, lo, hi: host_pipeline(host_in[lo:hi], host_out[lo:hi], elementsize, encode,
                                                          slice_chunks, nslots, dev), host_in.shape[0], devices)
        return
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    b, n = host_in.shape
    if b == 0 or n == 0:
        return
    if slice_chunks is None:
        slice_chunks = max(1, (64 << 20) // n)
    slice_chunks = max(1, min(slice_chunks, b))
    nslots = max(1, nslots)
    with torch.cuda.device(device):
        cur = torch.cuda.current_stream(device)
        h2d, comp, d2h = (torch.cuda.Stream(device=device) for _ in range(3))
        dev_in = [torch.empty((slice_chunks, n), dtype=torch.uint8, device=device) for _ in range(nslots)]
        dev_out = [torch.empty((slice_chunks, n), dtype=torch.uint8, device=device) for _ in range(nslots)]
        for s in (h2d, comp, d2h):
            s.wait_stream(cur)  # the ring was allocated on the current stream
        loaded = [torch.cuda.Event() for _ in range(nslots)]
        done = [torch.cuda.Event() for _ in range(nslots)]
        free = [None] * nslots
        for k, lo in enumerate(range(0, b, slice_chunks)):
            hi = min(b, lo + slice_chunks)
            i = k % nslots
            di = dev_in[i][: hi - lo]
            do = dev_out[i][: hi - lo]
            if free[i] is not None:
                h2d.wait_event(free[i])  # the slot's previous D2H has drained it
            with torch.cuda.stream(h2d):
                di.copy_(host_in[lo:hi], non_blocking=True)
                loaded[i].record(h2d)
            comp.wait_event(loaded[i])
            with torch.cuda.stream(comp):
                _ops.shuffle_batch(di, n, do, n, hi - lo, n, elementsize, encode)
                done[i].record(comp)
            d2h.wait_event(done[i])
            with torch.cuda.stream(d2h):
                host_out[lo:hi].copy_(do, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(d2h)
                free[i] = ev
        d2h.synchronize()
        for s in (h2d, comp):
            s.synchronize()
        cur.wait_stream(d2h)
