"""Quantize codec (reference: src/numcodecs/quantize.py:9-98).

encode: ``astype(rint(scale * x) / scale)`` computed in `dtype`, with the
power-of-two scale derived on the host exactly as quantize.py:65-73 does;
one fused pass on the GPU (csrc/mc_elementwise.hip).  decode: a cast to
`dtype`, zero-copy when the dtypes are equal, as in the reference.
"""

import math

import numpy as np

from . import _ops
from .abc import Codec
from .compat import (
    device_out_bytes, empty_like_bytes, finish, is_device_tensor, ndarray_copy, numpy_dtype, to_dbuf, torch_dtype,
)

__all__ = ["Quantize", "quantize_scale"]


def quantize_scale(digits) -> float:
    """2**bits with bits the smallest power of two resolving `digits` decimals."""
    precision = 10.0**-digits
    exp = math.log10(precision)
    exp = math.floor(exp) if exp < 0 else math.ceil(exp)
    bits = math.ceil(math.log2(10.0**-exp))
    return 2.0**bits


class Quantize(Codec):
    """Keep about `digits` decimal digits of float data (numcodecs id
    ``quantize``): values are rounded to a multiple of a power-of-two step
    and stored as `astype` (default `dtype`).  Lossy; decode is a cast.
    """

    codec_id = "quantize"

    def __init__(self, digits, dtype, astype=None):
        self.digits = digits
        self.dtype = np.dtype(dtype)
        self.astype = self.dtype if astype is None else np.dtype(astype)
        if self.dtype.kind != "f" or self.astype.kind != "f":
            raise ValueError("only floating point data types are supported")

    def encode(self, buf):
        # ensure_ndarray(buf).view(dtype): the shape is kept (quantize.py:62)
        src = to_dbuf(buf, flatten=False, contiguous=False)
        src_shape = src.shape
        if src.nbytes % self.dtype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.dtype.itemsize
        shape = _view_shape(src_shape, src.dtype.itemsize, self.dtype.itemsize, src.order)
        # the scale is a weak Python float: numpy converts it to `dtype`
        scale = np.asarray(quantize_scale(self.digits), dtype=self.dtype)
        dst = empty_like_bytes(n * self.astype.itemsize, src)
        _ops.quantize(src.data, dst, n, self.dtype, self.astype, float(scale))
        return finish(dst, self.astype, shape, src.order, src.host)

    def decode(self, buf, out=None):
        if is_device_tensor(buf) and numpy_dtype(buf.dtype) == self.astype == self.dtype:
            return ndarray_copy(buf, out)  # astype(copy=False) is the view itself
        src = to_dbuf(buf, flatten=False, contiguous=False)
        if src.nbytes % self.astype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.astype.itemsize
        shape = _view_shape(src.shape, src.dtype.itemsize, self.astype.itemsize, src.order)
        if self.astype == self.dtype:
            dst = src.data
        else:
            direct = device_out_bytes(out, n * self.dtype.itemsize, src)
            dst = empty_like_bytes(n * self.dtype.itemsize, src) if direct is None else direct
            _ops.cast(src.data, dst, n, self.astype, self.dtype)
            if direct is not None:
                return out
        return ndarray_copy(finish(dst, self.dtype, shape, src.order, src.host), out)

    def get_config(self):
        return {
            "id": self.codec_id,
            "digits": self.digits,
            "dtype": self.dtype.str,
            "astype": self.astype.str,
        }

    def __repr__(self):
        r = f"{type(self).__name__}(digits={self.digits}, dtype={self.dtype.str!r}"
        if self.astype != self.dtype:
            r += f", astype={self.astype.str!r}"
        return r + ")"


def _view_shape(shape, old_itemsize, new_itemsize, order):
    """Shape of ``a.view(new_dtype)`` for an array of `shape` (numpy's rule:
    the last axis in memory order is rescaled)."""
    shape = list(shape) or [1]
    if old_itemsize == new_itemsize:
        return tuple(shape)
    axis = 0 if order == "F" and len(shape) > 1 else -1
    shape[axis] = shape[axis] * old_itemsize // new_itemsize
    return tuple(shape)
