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
        dst = empty_like_bytes(n * self.astype.itemsize, src)
        _ops.delta_encode(src.data, dst, n, self.dtype, self.astype)
        return finish(dst, self.astype, (n,), "C", src.host)

    def decode(self, buf, out=None):
        src = to_dbuf(buf, contiguous=False)
        if src.nbytes % self.astype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.astype.itemsize
        loop = decode_loop_dtype(self.astype, self.dtype)
        direct = device_out_bytes(out, n * self.dtype.itemsize, src)
        dst = empty_like_bytes(n * self.dtype.itemsize, src) if direct is None else direct
        if loop is None:
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
