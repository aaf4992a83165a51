"""AsType filter (reference: src/numcodecs/astype.py:7-72).

encode: ``ensure_ndarray(buf).view(decode_dtype).astype(encode_dtype)``;
decode: ``view(encode_dtype).astype(decode_dtype)`` copied into `out` when
given.  The cast runs on the GPU with numpy's ``astype`` semantics
(csrc/mc_elementwise.hip ``mc_cast``: wrap-around integer narrowing,
correctly rounded float narrowing, x86-64 results for out-of-range
float -> int); shapes follow numpy's ``view`` rule.
"""

import numpy as np

from . import _ops
from .abc import Codec
from .compat import device_out_bytes, empty_like_bytes, finish, ndarray_copy, to_dbuf
from .quantize import _view_shape

__all__ = ["AsType"]


def _cast(buf, from_dt, to_dt, out=None):
    """The cast, written straight into a device `out` when it can take it
    (then `out` is returned, else the new array)."""
    src = to_dbuf(buf, flatten=False, contiguous=False)
    if from_dt != to_dt and (_ops.is_ext_dtype(from_dt) or _ops.is_ext_dtype(to_dt)):
        # numpy's own errors / ComplexWarning, as astype.py:53,58 raise them,
        # and its result dtype (a cast to generic timedelta64 / datetime64
        # keeps the source unit)
        to_dt = np.zeros(1, dtype=from_dt).astype(to_dt).dtype
    if src.nbytes % from_dt.itemsize:
        raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
    n = src.nbytes // from_dt.itemsize
    shape = _view_shape(src.shape, src.dtype.itemsize, from_dt.itemsize, src.order)
    direct = device_out_bytes(out, n * to_dt.itemsize, src)
    dst = empty_like_bytes(n * to_dt.itemsize, src) if direct is None else direct
    if from_dt == to_dt:
        _ops.copy(src.data, dst, src.nbytes)
    else:  # _ops.cast routes the extended dtypes and the calendar casts itself
        _ops.cast(src.data, dst, n, from_dt, to_dt)
    if direct is not None:
        return out
    return finish(dst, to_dt, shape, src.order, src.host)


class AsType(Codec):
    """Cast chunks from `decode_dtype` to `encode_dtype` on encode and back on
    decode (numcodecs id ``astype``), on the GPU.

    The cast follows numpy's unsafe ``astype``: narrowing an integer wraps,
    narrowing a float rounds to nearest-even, and float values outside the
    integer range give the x86-64 results numpy produces.  A lossy
    `encode_dtype` therefore loses data silently, exactly as in numcodecs.
    """

    codec_id = "astype"

    def __init__(self, encode_dtype, decode_dtype):
        self.encode_dtype = np.dtype(encode_dtype)
        self.decode_dtype = np.dtype(decode_dtype)

    def encode(self, buf):
        return _cast(buf, self.decode_dtype, self.encode_dtype)

    def decode(self, buf, out=None):
        res = _cast(buf, self.encode_dtype, self.decode_dtype, out)
        return res if res is out else ndarray_copy(res, out)

    def get_config(self):
        return {
            "id": self.codec_id,
            "encode_dtype": self.encode_dtype.str,
            "decode_dtype": self.decode_dtype.str,
        }

    def __repr__(self):
        return (
            f"{type(self).__name__}(encode_dtype={self.encode_dtype.str!r}, "
            f"decode_dtype={self.decode_dtype.str!r})"
        )
