"""Thin wrappers over the libmcodec entry points (include/mcodec.h).

Each wrapper takes device tensors, calls the C ABI on torch's current stream
for the tensor's device, and raises on a non-zero status.  Nothing here
synchronises except where a result must be inspected on the host
(Fletcher32 verification).
"""

from __future__ import annotations

import contextlib
import ctypes
import math
import threading

import numpy as np
import torch

from . import _native
from ._native import DTYPE_CODES, MC_ARRIVAL_WORDS, check, lib

__all__ = ["dtype_code", "stream", "workspace"]


# numpy's longdouble is the x87 80-bit extended type stored in 16 bytes on
# x86-64 Linux (the platform the reference runs on and the kernels restate:
# csrc/mc_x80.h); anywhere else 'f16' would be another format
_LONGDOUBLE_X87 = np.dtype(np.longdouble).itemsize == 16 and np.finfo(np.longdouble).nmant == 63


def dtype_code(dt) -> int:
    """mc_dtype code of numpy dtype `dt`: bool/int/uint/float (float16 to
    longdouble)/complex (to clongdouble) and timedelta64/datetime64 (any
    unit) of either byte order (a big-endian dtype carries MC_BIG_ENDIAN)."""
    dt = np.dtype(dt)
    code = DTYPE_CODES.get(dt.str)
    if code is not None:
        return code
    key = "m8" if dt.kind == "m" else "M8" if dt.kind == "M" else dt.str[1:]
    code = _native.EXT_CODES.get(key) if is_ext_dtype(dt) else None
    if code is None or (key in ("f16", "c32") and not _LONGDOUBLE_X87):
        raise NotImplementedError(
            f"dtype {dt.str!r} is not supported by the numcodecs_amd device kernels "
            "(bool/int/uint/float/complex/timedelta64/datetime64 only)"
        )
    return code | (_native.MC_BIG_ENDIAN if dt.byteorder == ">" else 0)


def is_ext_dtype(dt) -> bool:
    """complex, timedelta64, datetime64 or longdouble: the dtypes computed by
    mc_ext.hip."""
    dt = np.dtype(dt)
    return dt.kind in "cmM" or (dt.kind == "f" and dt.itemsize == 16)


def is_longdouble(dt) -> bool:
    """longdouble or clongdouble (csrc/mc_x80.h arithmetic)."""
    dt = np.dtype(dt)
    return (dt.kind == "f" and dt.itemsize == 16) or (dt.kind == "c" and dt.itemsize == 32)


# numpy's datetime unit table (datetime.c: NPY_DATETIMEUNIT order and
# _datetime_factors), restated for get_datetime_conversion_factor
_DT_UNITS = ["Y", "M", "W", "D", "h", "m", "s", "ms", "us", "ns", "ps", "fs", "as"]
_DT_FACTORS = [1, 1, 7, 24, 60, 60, 1000, 1000, 1000, 1000, 1000, 1000, 1]
_U64 = (1 << 64) - 1


def _units_factor(big: int, little: int) -> int:
    """get_datetime_units_factor: ticks of unit `little` per unit `big`
    (0 on overflow, as numpy)."""
    f = 1
    for u in range(big, little):
        f = (f * _DT_FACTORS[u]) & _U64
        if f & 0xFF00000000000000:
            return 0
    return f


def datetime_conversion_factor(src, dst) -> "tuple[int, int]":
    """(num, den) of numpy's get_datetime_conversion_factor between the units
    of two timedelta64/datetime64 dtypes (reduced), so that a same-kind cast
    is v*num/den with numpy's floor rounding of negatives (mc_cast_units).
    Generic source units convert with (1, 1); specific -> generic raises
    like numpy."""
    su, sn = np.datetime_data(np.dtype(src))
    du, dn = np.datetime_data(np.dtype(dst))
    if su == "generic":
        return 1, 1
    if du == "generic":
        raise ValueError("Cannot convert from specific units to generic units in NumPy datetimes or timedeltas")
    sb, db = _DT_UNITS.index(su), _DT_UNITS.index(du)
    swapped = sb > db
    lo, hi = (db, sb) if swapped else (sb, db)
    num = den = 1
    if lo != hi:
        ylen = 97 + 400 * 365
        if lo == 0:  # years
            if hi == 1:
                num *= 12
            elif hi == 2:
                num, den = num * ylen, den * 400 * 7
            else:
                num, den = num * ylen * _units_factor(3, hi), den * 400
        elif lo == 1:  # months
            if hi == 2:
                num, den = num * ylen, den * 400 * 12 * 7
            else:
                num, den = num * ylen * _units_factor(3, hi), den * 400 * 12
        else:
            num *= _units_factor(lo, hi)
    num &= _U64
    if num == 0:
        raise OverflowError(
            "Integer overflow while computing the conversion factor between NumPy datetime units "
            f"{_DT_UNITS[lo]} and {_DT_UNITS[hi]}")
    if swapped:
        num, den = den, num
    num, den = (num * sn) & _U64, (den * dn) & _U64
    g = math.gcd(num, den)
    return num // g, den // g


def calendar_cast(from_dt, to_dt):
    """(src_unit, src_num, dst_unit, dst_num) of a datetime64 cast numpy runs
    through its datetimestruct path (years / months on exactly one side:
    csrc/mc_cal.h), else None.  numpy's own conversion-factor errors are
    raised first, as its cast does."""
    f, t = np.dtype(from_dt), np.dtype(to_dt)
    if f.kind != "M" or t.kind != "M" or np.datetime_data(f) == np.datetime_data(t):
        return None
    (fu, fn), (tu, tn) = np.datetime_data(f), np.datetime_data(t)
    if "generic" in (fu, tu) or (fu in ("Y", "M")) == (tu in ("Y", "M")):
        return None
    datetime_conversion_factor(f, t)  # numpy raises its overflow error here too
    return _DT_UNITS.index(fu), fn, _DT_UNITS.index(tu), tn


def time_cast_factor(from_dt, to_dt) -> "tuple[int, int]":
    """The (num, den) mc_cast_units applies for numpy's astype(from -> to):
    a unit conversion between two timedelta64 or two datetime64 dtypes
    (linear units), (1, 1) otherwise (a timedelta <-> datetime cast keeps the
    ticks, as numpy's does).  Calendar conversions of datetime64 between
    years/months and the other units are calendar_cast()'s."""
    f, t = np.dtype(from_dt), np.dtype(to_dt)
    if f.kind not in "mM" or t.kind != f.kind:
        return 1, 1
    if np.datetime_data(f) == np.datetime_data(t):
        return 1, 1
    if calendar_cast(f, t) is not None:
        raise ValueError(f"{f.str!r} -> {t.str!r} is a calendar cast (calendar_cast)")
    return datetime_conversion_factor(f, t)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_capturing = getattr(torch._C, "_cuda_isCurrentStreamCapturing", None) or torch.cuda.is_current_stream_capturing
_cur_device = getattr(torch._C, "_cuda_getDevice", None)  # the current device index


def stream(t: torch.Tensor) -> int:
    """hipStream_t of torch's current stream on `t`'s device (the raw handle
    straight from torch's C++ side: the Python wrapper costs ~4 us a call)."""
    if _raw_stream is not None:
        return _raw_stream(t.get_device())
    return torch.cuda.current_stream(t.device).cuda_stream


def workspace(nbytes: int, like: torch.Tensor) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=like.device)


class _VerifySlot:
    """Per-(thread, device, stream) resources of the one-launch checksum verify: a
    zeroed arrival counter (left zero by every call), a reusable partials
    workspace and a verdict record in mapped, fine-grained pinned host memory
    (mc_verdict_alloc) that the kernel writes {computed, stored, seq} into;
    the host spins on the seq word (mc_verdict_wait) instead of synchronising
    the stream."""

    def __init__(self, device):
        self.device = device
        self.ticket = torch.zeros(MC_ARRIVAL_WORDS, dtype=torch.int32, device=device)
        self.ticket_ptr = self.ticket.data_ptr()
        self.ws = torch.empty(1 << 20, dtype=torch.uint8, device=device)
        self.rec = lib.mc_verdict_alloc()
        if not self.rec:
            raise _native.MCodecError("mc_verdict_alloc failed (mapped pinned host memory)")
        self.rec_np = np.ctypeslib.as_array((ctypes.c_uint32 * 4).from_address(self.rec))
        self.out_ptr = lib.mc_host_device_pointer(self.rec)
        if not self.out_ptr:
            raise _native.MCodecError("the verdict record is not mapped into the device address space")
        self.seq = 0
        self.ws_sizes = {}

    def __del__(self):
        rec, self.rec = getattr(self, "rec", None), None
        if rec:
            try:
                lib.mc_verdict_free(rec)
            except Exception:  # interpreter shutdown
                pass

    def next_seq(self) -> int:
        """The sequence word of the next verify (1 .. 2**32 - 1, never 0)."""
        self.seq = self.seq % 0xFFFFFFFF + 1
        return self.seq

    def read(self, st, seq):
        """(computed, stored) once the kernel published `seq` (0: after a
        stream synchronisation, for kernels that publish no sequence word)."""
        if seq:
            check(lib.mc_verdict_wait(self.rec, seq, st), "mc_verdict_wait")
        else:
            check(lib.mc_stream_synchronize(st), "mc_stream_synchronize")
        return int(self.rec_np[0]), int(self.rec_np[1])

    def workspace_for(self, key, query):
        """The workspace for a verify of `key` = (entry point, sizes...): the
        size query runs once per key."""
        n = self.ws_sizes.get(key)
        if n is None:
            if len(self.ws_sizes) >= 256:  # bounded: many distinct chunk sizes
                self.ws_sizes.clear()
            n = self.ws_sizes[key] = int(query())
        return self.workspace(n)

    def workspace(self, nbytes):
        if self.ws.numel() < nbytes:
            self.ws = torch.empty(max(int(nbytes), 2 * self.ws.numel()), dtype=torch.uint8, device=self.device)
        return self.ws


# slots per thread (threading.local: a slot dies with its thread): two
# threads verifying on the same stream must not share a verdict record, whose
# words the host reads after its own kernel published them
_TLS = threading.local()


def arrival_ticket(t: torch.Tensor, st: int):
    """Device address of the stream's zeroed arrival counter (MC_ARRIVAL_WORDS
    words, left zero by every kernel that takes it; stream order keeps the
    users apart), or None during HIP-graph capture (the callers then take
    their ticket-free schedules)."""
    sl = _verify_slot(t, st)
    return None if sl is None else sl.ticket.data_ptr()


def _verify_slot(t: torch.Tensor, st: int):
    """The stream's verify slot, or None during HIP-graph capture."""
    if _capturing():
        return None
    slots = getattr(_TLS, "slots", None)
    if slots is None:
        slots = _TLS.slots = {}
    key = (t.device.index, st)
    sl = slots.get(key)
    if sl is None:
        sl = slots[key] = _VerifySlot(t.device)
    return sl


_NO_GUARD = contextlib.nullcontext()


def _guard(t: torch.Tensor):
    """Make `t`'s device current for the call (a no-op when it already is)."""
    if t.get_device() == (_cur_device() if _cur_device is not None else torch.cuda.current_device()):
        return _NO_GUARD
    return torch.cuda.device(t.device)


# ---------------------------------------------------------------------------
def copy(src: torch.Tensor, dst: torch.Tensor, nbytes: int) -> None:
    """dst[:nbytes] = src[:nbytes] (raw bytes, same device) through mc_copy:
    the nontemporal vector copy kernel, ~1.4x hipMemcpyAsync DtoD."""
    if nbytes == 0:
        return
    _native.require_device()
    if src.device != dst.device:
        raise ValueError("mc_copy copies within one device")
    with _guard(src):
        check(lib.mc_copy(src.data_ptr(), dst.data_ptr(), nbytes, stream(src)), "mc_copy")


def current_device_index(t: torch.Tensor) -> "int | None":
    """`t`'s device index when it is a HIP tensor on the CURRENT device (the
    case the fast paths handle without a device guard), else None."""
    idx = t.get_device()
    if idx < 0 or _cur_device is None or _raw_stream is None or idx != _cur_device():
        return None
    return idx


def shuffle_ptr(idx: int, src_ptr: int, dst_ptr: int, nbytes: int, es: int, encode: bool) -> None:
    """mc_shuffle / mc_unshuffle on raw device pointers of the current device
    `idx` (torch's current stream there); the caller has validated sizes."""
    fn = lib.mc_shuffle if encode else lib.mc_unshuffle
    rc = fn(src_ptr, dst_ptr, nbytes, es, _raw_stream(idx))
    if rc:
        check(rc, "mc_shuffle" if encode else "mc_unshuffle")


def shuffle(src: torch.Tensor, dst: torch.Tensor, nbytes: int, es: int, encode: bool) -> None:
    _native.require_device()
    if nbytes == 0:
        return
    with _guard(src):
        fn = lib.mc_shuffle if encode else lib.mc_unshuffle
        check(fn(src.data_ptr(), dst.data_ptr(), nbytes, es, stream(src)),
              "mc_shuffle" if encode else "mc_unshuffle")


def shuffle_batch(src, src_stride, dst, dst_stride, nchunks, chunk_bytes, es, encode) -> None:
    _native.require_device()
    with _guard(src):
        fn = lib.mc_shuffle_batch if encode else lib.mc_unshuffle_batch
        check(fn(src.data_ptr(), src_stride, dst.data_ptr(), dst_stride, nchunks, chunk_bytes, es,
                 stream(src)), "mc_(un)shuffle_batch")


def bitround(src, dst, n, itemsize, keepbits) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        check(lib.mc_bitround(src.data_ptr(), dst.data_ptr(), n, itemsize, keepbits, stream(src)),
              "mc_bitround")


def bitround_shuffle(src, dst, n, itemsize, keepbits) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        check(lib.mc_bitround_shuffle(src.data_ptr(), dst.data_ptr(), n, itemsize, keepbits,
                                      stream(src)), "mc_bitround_shuffle")


def delta_encode(src, dst, n, dtype, astype) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        check(lib.mc_delta_encode(src.data_ptr(), dst.data_ptr(), n, dtype_code(dtype),
                                  dtype_code(astype), stream(src)), "mc_delta_encode")


def delta_batch(src, src_stride, dst, dst_stride, nchunks, n, dtype, astype, encode) -> None:
    """Delta encode (dtype -> astype) or decode (astype -> dtype) of nchunks
    chunks of n elements each (byte strides)."""
    _native.require_device()
    if n == 0 or nchunks == 0:
        return
    with _guard(src):
        if encode:
            check(lib.mc_delta_encode_batch(src.data_ptr(), src_stride, dst.data_ptr(), dst_stride, nchunks, n,
                                            dtype_code(dtype), dtype_code(astype), stream(src)),
                  "mc_delta_encode_batch")
        else:
            a, d = dtype_code(astype), dtype_code(dtype)
            ws_n = lib.mc_delta_decode_batch_workspace(nchunks, n, a, d)
            ws = workspace(ws_n, src)
            check(lib.mc_delta_decode_batch_ws(src.data_ptr(), src_stride, dst.data_ptr(), dst_stride, nchunks, n,
                                               a, d, ws.data_ptr(), ws.numel(), stream(src)),
                  "mc_delta_decode_batch_ws")


def delta_decode(src, dst, n, astype, dtype) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        a, d = dtype_code(astype), dtype_code(dtype)
        ws_n = lib.mc_delta_decode_workspace(n, a, d)
        ws = workspace(ws_n, src)
        st = stream(src)
        check(lib.mc_delta_decode(src.data_ptr(), dst.data_ptr(), n, a, d, ws.data_ptr(), ws.numel(),
                                  arrival_ticket(src, st), st), "mc_delta_decode")


def _scalar_args(value, dt):
    """(double, int64) pair carrying `value` in compute dtype `dt`."""
    dt = np.dtype(dt)
    if dt.kind == "f":
        return float(value), 0
    if dt.kind == "b":
        return 0.0, int(bool(value))
    arr = np.asarray(value, dtype=dt)
    if dt.kind == "u" and dt.itemsize == 8:
        return 0.0, int(arr.view(np.int64))
    return 0.0, int(arr)


def _complex_args(value, dt):
    """(re, im, int64) triple carrying `value` in compute dtype `dt`."""
    if np.dtype(dt).kind == "c":
        v = complex(np.asarray(value).astype(dt))
        return v.real, v.imag, 0
    f, i = _scalar_args(value, dt)
    return f, 0.0, i


def _raw_scalar(value, dt):
    """The scalar as numpy holds it in compute dtype `dt` (native bytes, in a
    ctypes buffer that lives for the call)."""
    b = np.asarray(value).astype(np.dtype(dt).newbyteorder("=")).tobytes()
    return ctypes.create_string_buffer(b, max(len(b), 32))


def fso_encode(src, dst, n, dtype, t1, t2, astype, offset_t1, scale_t2) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        if any(is_longdouble(t) for t in (dtype, t1, t2, astype)):
            off, sc = _raw_scalar(offset_t1, t1), _raw_scalar(scale_t2, t2)
            check(lib.mc_fso_encode_raw(src.data_ptr(), dst.data_ptr(), n, dtype_code(dtype), dtype_code(t1),
                                        dtype_code(t2), dtype_code(astype), ctypes.addressof(off),
                                        ctypes.addressof(sc), stream(src)), "mc_fso_encode_raw")
            return
        if any(is_ext_dtype(t) for t in (dtype, t1, t2, astype)):
            ore, oim, oi = _complex_args(offset_t1, t1)
            sre, sim, si = _complex_args(scale_t2, t2)
            check(lib.mc_fso_encode_x(src.data_ptr(), dst.data_ptr(), n, dtype_code(dtype), dtype_code(t1),
                                      dtype_code(t2), dtype_code(astype), ore, oim, oi, sre, sim, si,
                                      stream(src)), "mc_fso_encode_x")
            return
        of, oi = _scalar_args(offset_t1, t1)
        sf, si = _scalar_args(scale_t2, t2)
        check(lib.mc_fso_encode(src.data_ptr(), dst.data_ptr(), n, dtype_code(dtype), dtype_code(t1),
                                dtype_code(t2), dtype_code(astype), of, oi, sf, si, stream(src)),
              "mc_fso_encode")


def fso_decode(src, dst, n, astype, t3, t4, dtype, scale_t3, offset_t4) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        if any(is_longdouble(t) for t in (astype, t3, t4, dtype)):
            sc, off = _raw_scalar(scale_t3, t3), _raw_scalar(offset_t4, t4)
            check(lib.mc_fso_decode_raw(src.data_ptr(), dst.data_ptr(), n, dtype_code(astype), dtype_code(t3),
                                        dtype_code(t4), dtype_code(dtype), ctypes.addressof(sc),
                                        ctypes.addressof(off), stream(src)), "mc_fso_decode_raw")
            return
        if any(is_ext_dtype(t) for t in (astype, t3, t4, dtype)):
            sre, sim, _ = _complex_args(scale_t3, t3)
            ore, oim, _ = _complex_args(offset_t4, t4)
            check(lib.mc_fso_decode_x(src.data_ptr(), dst.data_ptr(), n, dtype_code(astype), dtype_code(t3),
                                      dtype_code(t4), dtype_code(dtype), sre, sim, ore, oim, stream(src)),
                  "mc_fso_decode_x")
            return
        check(lib.mc_fso_decode(src.data_ptr(), dst.data_ptr(), n, dtype_code(astype), dtype_code(t3),
                                dtype_code(t4), dtype_code(dtype), float(scale_t3), float(offset_t4),
                                stream(src)), "mc_fso_decode")


def quantize(src, dst, n, dtype, astype, scale) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        check(lib.mc_quantize(src.data_ptr(), dst.data_ptr(), n, dtype_code(dtype), dtype_code(astype),
                              float(scale), stream(src)), "mc_quantize")


def cast(src, dst, n, from_dt, to_dt) -> None:
    """numpy astype(from_dt -> to_dt) of n elements; timedelta64/datetime64
    unit conversions take numpy's conversion factor (mc_cast_units)."""
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        cal = calendar_cast(from_dt, to_dt)
        if cal is not None:
            check(lib.mc_cast_calendar(src.data_ptr(), dst.data_ptr(), n, dtype_code(from_dt), dtype_code(to_dt),
                                       *cal, stream(src)), "mc_cast_calendar")
            return
        if is_ext_dtype(from_dt) or is_ext_dtype(to_dt):
            num, den = time_cast_factor(from_dt, to_dt)
            check(lib.mc_cast_units(src.data_ptr(), dst.data_ptr(), n, dtype_code(from_dt), dtype_code(to_dt),
                                    num, den, stream(src)), "mc_cast_units")
            return
        check(lib.mc_cast(src.data_ptr(), dst.data_ptr(), n, dtype_code(from_dt), dtype_code(to_dt),
                          stream(src)), "mc_cast")


def fletcher32_encode(src, dst, nbytes) -> None:
    """Payload copy + LE32 footer in one launch (the stream's arrival ticket;
    the two-launch schedule during HIP-graph capture)."""
    _native.require_device()
    with _guard(src):
        st = stream(src)
        sl = _verify_slot(src, st)
        if sl is not None:
            ws = sl.workspace_for(("f32", nbytes), lambda: lib.mc_fletcher32_workspace(nbytes))
            check(lib.mc_fletcher32_encode_fused(src.data_ptr(), dst.data_ptr(), nbytes, ws.data_ptr(), ws.numel(),
                                                 sl.ticket.data_ptr(), st), "mc_fletcher32_encode_fused")
            return
        ws = workspace(lib.mc_fletcher32_workspace(nbytes), src)
        check(lib.mc_fletcher32_encode(src.data_ptr(), dst.data_ptr(), nbytes, ws.data_ptr(),
                                       ws.numel(), st), "mc_fletcher32_encode")


def fletcher32_verify(src, nbytes) -> "tuple[int, int]":
    """(computed, stored) for a buffer of payload + 4-byte footer (syncs):
    one launch writing its verdict into pinned host memory, one stream sync."""
    _native.require_device()
    with _guard(src):
        st = stream(src)
        sl = _verify_slot(src, st)
        if sl is not None:
            ws = sl.workspace_for(("f32", nbytes), lambda: lib.mc_fletcher32_workspace(nbytes))
            seq = sl.next_seq()
            check(lib.mc_fletcher32_verify_fused(src.data_ptr(), nbytes, sl.out_ptr, seq, ws.data_ptr(),
                                                 ws.numel(), sl.ticket.data_ptr(), st), "mc_fletcher32_verify_fused")
            return sl.read(st, seq)
        ws = workspace(lib.mc_fletcher32_workspace(nbytes), src)
        pair = torch.empty(2, dtype=torch.int32, device=src.device)
        check(lib.mc_fletcher32_verify(src.data_ptr(), nbytes, pair.data_ptr(), ws.data_ptr(),
                                       ws.numel(), stream(src)), "mc_fletcher32_verify")
        return _read_pair(pair)


def fletcher32_decode_device(buf: torch.Tensor):
    """Fletcher32.decode of a flat contiguous uint8 device tensor on the
    current device (the Zarr case), host time kept off the GPU's critical
    path: only what the launch needs runs before it (stream, the stream's
    verify slot, the workspace), the payload view is made while the kernel
    runs, and the host then waits on the verdict word.  Returns
    (payload, computed, stored), or None for the general path (other device,
    HIP-graph capture, too short)."""
    n = buf.numel()
    idx = buf.get_device()
    if n <= 4 or _raw_stream is None or _cur_device is None or idx != _cur_device():
        return None
    st = _raw_stream(idx)
    sl = _verify_slot(buf, st)
    if sl is None:
        return None
    ws = sl.workspace_for(("f32", n), lambda: lib.mc_fletcher32_workspace(n))
    seq = sl.next_seq()
    rc = lib.mc_fletcher32_verify_fused(buf.data_ptr(), n, sl.out_ptr, seq, ws.data_ptr(), ws.numel(),
                                        sl.ticket_ptr, st)
    if rc:
        check(rc, "mc_fletcher32_verify_fused")
    payload = buf[: n - 4]  # while the kernel runs
    val, found = sl.read(st, seq)
    return payload, val, found


def checksum32_decode_device(kind, buf: torch.Tensor, init, location):
    """Checksum32.decode (CRC32 / CRC32C / Adler32) of a flat contiguous
    uint8 device tensor on the current device, launch first as
    fletcher32_decode_device: (payload, computed, stored), or None for the
    general path (other device, HIP-graph capture, too short)."""
    n = buf.numel()
    idx = buf.get_device()
    if n <= 4 or _raw_stream is None or _cur_device is None or idx != _cur_device():
        return None
    st = _raw_stream(idx)
    sl = _verify_slot(buf, st)
    if sl is None:
        return None
    ws = sl.workspace_for((kind, n), lambda: lib.mc_checksum32_workspace(kind, 1, n - 4))
    seq = sl.next_seq()
    rc = lib.mc_checksum32_verify_fused(kind, buf.data_ptr(), n, init, None, 0, location, sl.out_ptr, seq,
                                        ws.data_ptr(), ws.numel(), sl.ticket_ptr, st)
    if rc:
        check(rc, "mc_checksum32_verify_fused")
    payload = buf[4:] if location == _native.MC_CK_START else buf[: n - 4]  # while the kernel runs
    val, found = sl.read(st, seq)
    return payload, val, found


def fletcher32(src, nbytes) -> int:
    """Checksum of the first `nbytes` of a device tensor (syncs)."""
    _native.require_device()
    with _guard(src):
        ws = workspace(lib.mc_fletcher32_workspace(nbytes), src)
        out = torch.empty(1, dtype=torch.int32, device=src.device)
        check(lib.mc_fletcher32(src.data_ptr(), nbytes, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                stream(src)), "mc_fletcher32")
        return int(out.cpu().numpy().view(np.uint32)[0])


# ---------------------------------------------------------------------------
def _prefix_dev(prefix, like):
    if prefix is None or len(prefix) == 0:
        return None
    if isinstance(prefix, torch.Tensor):
        return prefix.to(like.device).contiguous().view(torch.uint8)
    return torch.from_numpy(np.frombuffer(bytes(prefix), dtype=np.uint8).copy()).to(like.device)


def checksum32(kind, src, src_stride, nchunks, nbytes, init, prefix=None) -> torch.Tensor:
    """Checksum of `nchunks` rows of `nbytes` at src + c*src_stride -> device int32[nchunks]
    (the uint32 values' bit patterns)."""
    _native.require_device()
    out = torch.empty(max(nchunks, 1), dtype=torch.int32, device=src.device)
    with _guard(src):
        pre = _prefix_dev(prefix, src)
        ws = workspace(lib.mc_checksum32_workspace(kind, nchunks, nbytes), src)
        check(lib.mc_checksum32_batch(kind, src.data_ptr(), src_stride, nchunks, nbytes, init & 0xFFFFFFFF,
                                      pre.data_ptr() if pre is not None else None,
                                      pre.numel() if pre is not None else 0,
                                      out.data_ptr(), ws.data_ptr(), ws.numel(), stream(src)),
              "mc_checksum32_batch")
    return out[:nchunks]


# Single-chunk Checksum32 encodes finish in the tiles launch (one launch: 1 MiB
# CRC32 / Adler32 encode 14.2 / 14.5 -> 10.5 / 8.3 us per call), at every size
# since round 6: with the workgroups' sums riding the arrival atomics
# (CRC: ck_ride_arrive; Adler32: adler_arrive_finish) the one launch beats
# tiles + finalize at 256 MiB by 5-6 us for all three checksums at both
# footer locations (tools/probe_adler_encode.py, 4 rotating sets,
# profiles/r06/probe_ck_encode_sets.jsonl); round 5 had measured Adler32's
# finalize kernel ~3 us faster there and kept chunks >= 16 MiB on it.


def checksum32_encode(kind, src, src_stride, dst, dst_stride, nchunks, nbytes, init, location,
                      prefix=None) -> None:
    """Checksum32.encode of `nchunks` rows into dst rows (LE32 footer at the start or end).
    One chunk of CRC32 / CRC32C / Adler32 runs in one launch (the stream's
    arrival ticket; the tiles-then-finalize schedule during HIP-graph
    capture)."""
    _native.require_device()
    with _guard(src):
        if nchunks == 1 and kind != _native.MC_CK_JENKINS:
            st = stream(src)
            sl = _verify_slot(src, st)
            if sl is not None:
                ws = sl.workspace_for(("ck", kind, nbytes), lambda: lib.mc_checksum32_workspace(kind, 1, nbytes))
                check(lib.mc_checksum32_encode_fused(kind, src.data_ptr(), dst.data_ptr(), nbytes, init & 0xFFFFFFFF,
                                                     None, 0, location, None, ws.data_ptr(), ws.numel(),
                                                     sl.ticket.data_ptr(), st), "mc_checksum32_encode_fused")
                return
        pre = _prefix_dev(prefix, src)
        ws = workspace(lib.mc_checksum32_workspace(kind, nchunks, nbytes), src)
        check(lib.mc_checksum32_encode_batch(kind, src.data_ptr(), src_stride, dst.data_ptr(), dst_stride,
                                             nchunks, nbytes, init & 0xFFFFFFFF,
                                             pre.data_ptr() if pre is not None else None,
                                             pre.numel() if pre is not None else 0, location, None,
                                             ws.data_ptr(), ws.numel(), stream(src)),
              "mc_checksum32_encode_batch")


def checksum32_decode(kind, src, src_stride, dst, dst_stride, nchunks, encoded_bytes, init, location,
                      prefix=None):
    """Checksum32.decode of `nchunks` encoded rows: (sums, stored) device int32[nchunks]
    (uint32 bit patterns); the payloads land compacted in dst rows when dst is given."""
    _native.require_device()
    sums = torch.empty(max(nchunks, 1), dtype=torch.int32, device=src.device)
    stored = torch.empty(max(nchunks, 1), dtype=torch.int32, device=src.device)
    with _guard(src):
        pre = _prefix_dev(prefix, src)
        ws = workspace(lib.mc_checksum32_workspace(kind, nchunks, encoded_bytes - 4), src)
        check(lib.mc_checksum32_decode_batch(kind, src.data_ptr(), src_stride,
                                             dst.data_ptr() if dst is not None else None, dst_stride,
                                             nchunks, encoded_bytes, init & 0xFFFFFFFF,
                                             pre.data_ptr() if pre is not None else None,
                                             pre.numel() if pre is not None else 0, location,
                                             sums.data_ptr(), stored.data_ptr(), ws.data_ptr(), ws.numel(),
                                             stream(src)),
              "mc_checksum32_decode_batch")
    return sums[:nchunks], stored[:nchunks]


def _read_pair(dev: torch.Tensor) -> "tuple[int, int]":
    """Two device uint32 words -> host ints: one async copy into pinned
    memory and a stream sync (no pageable hipMemcpy)."""
    host = torch.empty(2, dtype=torch.int32, pin_memory=True)
    host.copy_(dev, non_blocking=True)
    torch.cuda.current_stream(dev.device).synchronize()
    v = host.numpy().view(np.uint32)
    return int(v[0]), int(v[1])


def checksum32_verify(kind, src, encoded_bytes, init, location, prefix=None) -> "tuple[int, int]":
    """(computed, stored) checksum of ONE encoded buffer (payload + 4 bytes
    at `location`), from one mc_checksum32_decode_batch call (syncs)."""
    _native.require_device()
    with _guard(src):
        pre = _prefix_dev(prefix, src)
        st = stream(src)
        sl = _verify_slot(src, st)
        if sl is not None:  # one launch, verdict into pinned host memory, one host wait
            ws = sl.workspace_for((kind, encoded_bytes),
                                  lambda: lib.mc_checksum32_workspace(kind, 1, encoded_bytes - 4))
            seq = 0 if kind == _native.MC_CK_JENKINS else sl.next_seq()
            check(lib.mc_checksum32_verify_fused(kind, src.data_ptr(), encoded_bytes, init & 0xFFFFFFFF,
                                                 pre.data_ptr() if pre is not None else None,
                                                 pre.numel() if pre is not None else 0, location,
                                                 sl.out_ptr, seq, ws.data_ptr(), ws.numel(),
                                                 sl.ticket.data_ptr(), st), "mc_checksum32_verify_fused")
            return sl.read(st, seq)
        pair = torch.empty(2, dtype=torch.int32, device=src.device)
        ws = workspace(lib.mc_checksum32_workspace(kind, 1, encoded_bytes - 4), src)
        check(lib.mc_checksum32_decode_batch(kind, src.data_ptr(), encoded_bytes, None, 0, 1, encoded_bytes,
                                             init & 0xFFFFFFFF, pre.data_ptr() if pre is not None else None,
                                             pre.numel() if pre is not None else 0, location,
                                             pair.data_ptr(), pair.data_ptr() + 4, ws.data_ptr(), ws.numel(),
                                             stream(src)),
              "mc_checksum32_decode_batch")
        return _read_pair(pair)


def packbits(src, dst, n) -> None:
    _native.require_device()
    with _guard(dst):
        check(lib.mc_packbits(src.data_ptr() if n else None, dst.data_ptr(), n, stream(dst)), "mc_packbits")


def unpackbits_device(src, src_bytes):
    """PackBits.decode of a device buffer without a host round trip before
    the launch: the padding byte is copied to pinned memory ahead of the
    kernel on the same stream, the kernel unpacks all 8 * (src_bytes - 1)
    bits (at most 7 past the end: the returned view drops them), and the
    host waits only for the 1-byte copy.  Returns the uint8 tensor of bools,
    or None when the stream is being captured into a graph."""
    _native.require_device()
    if torch.cuda.is_current_stream_capturing():
        return None
    nmax = 8 * (src_bytes - 1)
    with _guard(src):
        dst = torch.empty(max(nmax, 1), dtype=torch.uint8, device=src.device)
        pad_h = torch.empty(1, dtype=torch.uint8, pin_memory=True)
        pad_h.copy_(src[:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        if nmax:
            check(lib.mc_unpackbits(src.data_ptr(), src_bytes, dst.data_ptr(), nmax, stream(src)), "mc_unpackbits")
        ev.synchronize()
        n = max(nmax - int(pad_h[0]), 0)
    return dst[:n]


def unpackbits(src, src_bytes, dst, n) -> None:
    _native.require_device()
    if n == 0:
        return
    with _guard(src):
        check(lib.mc_unpackbits(src.data_ptr(), src_bytes, dst.data_ptr(), n, stream(src)), "mc_unpackbits")
