"""FixedScaleOffset codec (reference: src/numcodecs/fixedscaleoffset.py:7-130).

encode: ``astype(rint((x - offset) * scale))``; decode:
``dtype(x / scale + offset)``.  Each is one fused pass on the GPU
(csrc/mc_elementwise.hip).  The dtype every step computes in is the one
numpy >= 2 picks (NEP 50: Python scalars are "weak", so a float32 array
minus a Python float stays float32, while integer / Python scalar true
division is float64); it is resolved here on the host by numpy itself on a
one-element stand-in array, and the scalars are converted to that dtype the
way numpy converts them -- so the device arithmetic rounds exactly as the
reference's numpy expression does.
"""

import numpy as np

from . import _ops
from .abc import Codec
from .compat import device_out_bytes, empty_like_bytes, finish, ndarray_copy, to_dbuf

__all__ = ["FixedScaleOffset"]


def _resolve(op, dtype, scalar):
    """Result dtype of ``array(dtype) <op> scalar`` and the scalar in it."""
    probe = np.zeros(1, dtype=dtype)
    res = op(probe, scalar).dtype  # raises like the reference would
    if isinstance(scalar, (np.generic, np.ndarray)):
        val = np.asarray(scalar).astype(res)
    else:
        val = np.asarray(scalar, dtype=res) if res.kind in "fc" else np.asarray(scalar).astype(res)
    return res, val


class FixedScaleOffset(Codec):
    """Fixed scale/offset encoding (numcodecs id ``fixedscaleoffset``), after
    HDF5's scale-offset filter without the bit packing.

    encode: ``astype(round((x - offset) * scale))`` computed in `dtype` (numpy's
    promotion of the Python scalars); decode: ``(y / scale) + offset`` in
    float64, cast back to `dtype`.  `astype` defaults to `dtype`.
    """

    codec_id = "fixedscaleoffset"

    def __init__(self, offset, scale, dtype, astype=None):
        self.offset = offset
        self.scale = scale
        self.dtype = np.dtype(dtype)
        self.astype = self.dtype if astype is None else np.dtype(astype)
        if self.dtype == np.dtype(object) or self.astype == np.dtype(object):
            raise ValueError("object arrays are not supported")

    def encode(self, buf):
        src = to_dbuf(buf, contiguous=False)
        if src.nbytes % self.dtype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.dtype.itemsize
        if _ops.is_ext_dtype(self.dtype) or _ops.is_ext_dtype(self.astype):
            # the reference's expression on a stand-in: numpy's own errors
            # (no rint loop for timedelta64, no multiply for datetime64) and
            # warnings (ComplexWarning on a complex -> real astype)
            np.around((np.zeros(1, dtype=self.dtype) - self.offset) * self.scale).astype(self.astype, copy=False)
        t1, off = _resolve(np.subtract, self.dtype, self.offset)
        t2, sc = _resolve(np.multiply, t1, self.scale)
        dst = empty_like_bytes(n * self.astype.itemsize, src)
        _ops.fso_encode(src.data, dst, n, self.dtype, t1, t2, self.astype, off, sc)
        return finish(dst, self.astype, (n,), "C", src.host)

    def decode(self, buf, out=None):
        src = to_dbuf(buf, contiguous=False)
        if src.nbytes % self.astype.itemsize:
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        n = src.nbytes // self.astype.itemsize
        if _ops.is_ext_dtype(self.dtype) or _ops.is_ext_dtype(self.astype):
            ((np.zeros(1, dtype=self.astype) / self.scale) + self.offset).astype(self.dtype, copy=False)
        t3, sc = _resolve(np.true_divide, self.astype, self.scale)
        t4, off = _resolve(np.add, t3, self.offset)
        direct = device_out_bytes(out, n * self.dtype.itemsize, src)
        dst = empty_like_bytes(n * self.dtype.itemsize, src) if direct is None else direct
        _ops.fso_decode(src.data, dst, n, self.astype, t3, t4, self.dtype, sc, off)
        if direct is not None:
            return out
        return ndarray_copy(finish(dst, self.dtype, (n,), "C", src.host), out)

    def get_config(self):
        return {
            "id": self.codec_id,
            "scale": self.scale,
            "offset": self.offset,
            "dtype": self.dtype.str,
            "astype": self.astype.str,
        }

    def __repr__(self):
        r = (
            f"{type(self).__name__}(scale={self.scale}, offset={self.offset}, "
            f"dtype={self.dtype.str!r}"
        )
        if self.astype != self.dtype:
            r += f", astype={self.astype.str!r}"
        return r + ")"
