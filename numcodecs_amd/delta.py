"""Delta codec (reference: src/numcodecs/delta.py:7-94).

encode: first element, then adjacent differences computed in `dtype` and
cast to `astype` (one fused pass, csrc/mc_elementwise.hip: k_delta_enc).
decode: running sum accumulated in `dtype` (csrc/mc_scan.hip): a parallel
scan for integer/bool dtypes (wrap-around arithmetic, bit-exact), and
numpy's exact left-to-right order for float dtypes.
"""

import numpy as np
import torch

from . import _ops
from .abc import Codec
from .compat import device_out_bytes, empty_like_bytes, finish, ndarray_copy, to_dbuf

__all__ = ["Delta"]


def check_first_elements(firsts, dtype, astype) -> None:
    """delta.py:63 writes ``enc[0] = arr[0]``: a numpy scalar assignment,
    which raises OverflowError (ValueError for NaN) or warns when the first
    element does not fit `astype`, unlike the array cast of the differences.
    Replayed on the host with numpy itself, for casts that are not safe only.
    `firsts` is a device uint8 tensor [..., itemsize] holding first elements."""
    if np.can_cast(dtype, astype, casting="safe"):
        return
    vals = np.frombuffer(firsts.reshape(-1).cpu().numpy().tobytes(), dtype=dtype)
    tmp = np.empty(1, dtype=astype)
    for v in vals:
        tmp[0] = v


def decode_loop_dtype(astype, dtype):
    """np.cumsum(enc, out=dec) (delta.py:80) accepts every numeric pair: it
    accumulates in np.promote_types(astype, dtype) and casts each running
    sum to dtype.  The device decode computes that directly for a float
    dtype (any astype), an integer dtype from an integer/bool astype
    (wrap-around sums: accumulating in the wider integer and casting back is
    the same modulo 2^bits) and bool from bool (logical or); it returns None
    for those.  For the other two families -- a float astype into an
    integer/bool dtype (a float running sum, cast per element) and an
    integer astype into bool (a nonzero test of an integer running sum) --
    it returns the loop dtype L: the decode runs as Delta(L, astype) (a
    supported pair, the running sums exactly as numpy keeps them) followed
    by numpy's cast L -> dtype (mc_cast)."""
    a, d = np.dtype(astype), np.dtype(dtype)
    if d.kind in "iub" and a.kind == "f" or d.kind == "b" and a.kind != "b":
        return np.promote_types(a, d)
    return None


def _dry_run_encode(dtype, astype):
    """delta.py:65-66 on a two-element stand-in: numpy's own errors and
    warnings (e.g. ComplexWarning) for the differences of an extended-dtype
    pair.  The first element's assignment (delta.py:63) depends on its value
    (a timedelta64 scalar may convert through datetime.timedelta): it is
    replayed with the real value by check_first_elements."""
    arr = np.zeros(2, dtype=dtype)
    enc = np.empty_like(arr, dtype=astype)
    enc[1:] = np.diff(arr)


def _dry_run_decode(astype, dtype):
    """delta.py:77-80 on a stand-in: np.cumsum raises numpy's UFuncTypeError
    for a datetime64 dtype (no datetime + datetime loop) or a float astype
    into timedelta64, exactly as the reference does."""
    np.cumsum(np.zeros(2, dtype=astype), out=np.empty(2, dtype=dtype))


_NUMERIC_KINDS = "biufcmM"


def check_numeric(dtype, astype, encode) -> None:
    """A string / bytes / void `dtype` or `astype`: the reference fails inside
    numpy (delta.py:66 np.diff -> UFuncTypeError for the subtract loop;
    delta.py:80 np.cumsum -> numpy's TypeError for add.accumulate), and so
    does this codec, by running the same numpy call on a stand-in."""
    d, a = np.dtype(dtype), np.dtype(astype)
    if d.kind in _NUMERIC_KINDS and a.kind in _NUMERIC_KINDS:
        return
    if encode:
        _dry_run_encode(d, a)
    else:
        _dry_run_decode(a, d)
    raise NotImplementedError(f"Delta({d.str!r}, astype={a.str!r}) is not supported by the numcodecs_amd device "
                              "kernels")


def ext_delta_encode(src, dst, n, dtype, astype) -> None:
    """Delta encode with a complex / timedelta64 / datetime64 / longdouble
    side: the differences in dtype (mc_ext.hip), cast to astype.  A
    timedelta64 / datetime64 pair with a unit change casts the first element
    as numpy's scalar assignment does (delta.py:63: dtype -> astype, numpy's
    astype rules -- a linear unit factor, the calendar path for years /
    months, ticks kept between timedelta and datetime) and the differences
    from timedelta64 in dtype's unit (delta.py:66)."""
    _dry_run_encode(dtype, astype)
    d, a = np.dtype(dtype), np.dtype(astype)
    if d.kind in "mM" and a.kind in "mM" and np.datetime_data(a) != np.datetime_data(d):
        unit, num = np.datetime_data(d)
        diff_dt = np.dtype("m8" if unit == "generic" else f"m8[{num}{unit}]")
        if d.byteorder == ">":
            diff_dt = diff_dt.newbyteorder(">")
        tmp = torch.empty(n * 8, dtype=torch.uint8, device=src.device)
        _ops.delta_encode(src, tmp, n, d, diff_dt)  # timedelta differences in dtype's unit
        if n > 1:
            _ops.cast(tmp[8:], dst[a.itemsize:], n - 1, diff_dt, a)
        _ops.cast(src, dst, 1, d, a)  # enc[0] = arr[0]
        return
    _ops.delta_encode(src, dst, n, d, a)


def ext_delta_decode(src, dst, n, astype, dtype) -> None:
    """Delta decode with a complex / timedelta64 side (mc_ext.hip): numpy's
    timedelta running sums (NaT from the first NaT on) or per-component
    complex running sums.  An astype numpy converts first (another timedelta
    unit) goes through mc_cast_units; an integer dtype from a timedelta
    astype is decoded as timedelta and cast, as numpy's loop does."""
    _dry_run_decode(astype, dtype)
    a, d = np.dtype(astype), np.dtype(dtype)
    if d.kind == "m" and a.kind == "m" and np.datetime_data(a) != np.datetime_data(d):
        tmp = torch.empty(n * 8, dtype=torch.uint8, device=src.device)
        _ops.cast(src, tmp, n, a, d)
        _ops.delta_decode(tmp, dst, n, d, d)
        return
    if a.kind == "m" and d.kind != "m" and not (d.kind == "i" and d.itemsize == 8):
        loop = a.newbyteorder("=")
        tmp = torch.empty(n * 8, dtype=torch.uint8, device=src.device)
        _ops.delta_decode(src, tmp, n, a, loop)
        _ops.cast(tmp, dst, n, loop, d)
        return
    _ops.delta_decode(src, dst, n, a, d)


def decode_two_step(src, dst, n, astype, dtype, loop) -> None:
    """Delta decode of a pair decode_loop_dtype() routes through its loop
    dtype: running sums into a device temporary of `loop`, then cast."""
    tmp = torch.empty(n * loop.itemsize, dtype=torch.uint8, device=src.device)
    _ops.delta_decode(src, tmp, n, astype, loop)
    _ops.cast(tmp, dst, n, loop, dtype)


class Delta(Codec):
    """Store each element as its difference from the previous one (the first
    element as itself), numcodecs id ``delta``.

    `dtype` is the type differences are computed in (and decoded to);
    `astype` (default: `dtype`) is the type they are stored as.  A narrow
    integer `astype` wraps on overflow without any check, as in numcodecs.
    Decoding is the running sum in `dtype` (numpy's ``cumsum`` order).

    >>> import numpy as np, numcodecs_amd
    >>> numcodecs_amd.Delta(dtype='i2', astype='i1').encode(np.arange(100, 120, 2, dtype='i2'))  # doctest: +SKIP
    array([100,   2,   2,   2,   2,   2,   2,   2,   2,   2], dtype=int8)
    """

    codec_id = "delta"

    def __init__(self, dtype, astype=None):
        self.dtype = np.dtype(dtype)
        self.astype = self.dtype if astype is None else np.dtype(astype)
        if self.dtype == np.dtype(object) or self.astype == np.dtype(object):
            raise ValueError("object arrays are not supported")

    def encode(self, buf):
        src = to_dbuf(buf, contiguous=False)
        if src.nbytes % self.dtype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.dtype.itemsize
        if n == 0:  # enc[0] = arr[0] on an empty array (delta.py:63)
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        check_first_elements(src.data[: self.dtype.itemsize], self.dtype, self.astype)
        check_numeric(self.dtype, self.astype, True)
        dst = empty_like_bytes(n * self.astype.itemsize, src)
        if _ops.is_ext_dtype(self.dtype) or _ops.is_ext_dtype(self.astype):
            ext_delta_encode(src.data, dst, n, self.dtype, self.astype)
        else:
            _ops.delta_encode(src.data, dst, n, self.dtype, self.astype)
        return finish(dst, self.astype, (n,), "C", src.host)

    def decode(self, buf, out=None):
        src = to_dbuf(buf, contiguous=False)
        if src.nbytes % self.astype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.astype.itemsize
        check_numeric(self.dtype, self.astype, False)
        ext = _ops.is_ext_dtype(self.dtype) or _ops.is_ext_dtype(self.astype)
        loop = None if ext else decode_loop_dtype(self.astype, self.dtype)
        direct = device_out_bytes(out, n * self.dtype.itemsize, src)
        dst = empty_like_bytes(n * self.dtype.itemsize, src) if direct is None else direct
        if ext:
            ext_delta_decode(src.data, dst, n, self.astype, self.dtype)
        elif loop is None:
            _ops.delta_decode(src.data, dst, n, self.astype, self.dtype)
        elif n:
            decode_two_step(src.data, dst, n, self.astype, self.dtype, loop)
        if direct is not None:
            return out
        return ndarray_copy(finish(dst, self.dtype, (n,), "C", src.host), out)

    def get_config(self):
        return {"id": self.codec_id, "dtype": self.dtype.str, "astype": self.astype.str}

    def __repr__(self):
        r = f"{type(self).__name__}(dtype={self.dtype.str!r}"
        if self.astype != self.dtype:
            r += f", astype={self.astype.str!r}"
        return r + ")"
