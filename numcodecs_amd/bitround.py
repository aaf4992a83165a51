"""BitRound codec (reference: src/numcodecs/bitround.py:9-80).

Round-to-nearest-even on the mantissa bits of the same-width integer view
(wrap-around integer arithmetic), one fused pass on the GPU
(csrc/mc_elementwise.hip: k_bitround) instead of numpy's copy + five passes.
Decoding is a dtype re-view, exactly as in the reference.
"""

import numpy as np
import torch

from . import _ops
from .abc import Codec
from .compat import (
    ensure_ndarray_like,
    finish,
    is_device_tensor,
    ndarray_copy,
    numpy_dtype,
    torch_dtype,
    upload,
)

__all__ = ["BitRound", "max_bits"]

# mantissa bits per float type (bitround.py:9-13)
max_bits = {
    "float16": 10,
    "float32": 23,
    "float64": 52,
}


class BitRound(Codec):
    """Round float mantissas to `keepbits` bits (numcodecs id ``bitround``).

    Round-to-nearest-even on the integer view of each f2/f4/f8 value, so
    the trailing mantissa bits become zero and compress well (Klöwer et al.
    2021).  `keepbits` equal to the dtype's mantissa width is the identity.
    """

    codec_id = "bitround"

    def __init__(self, keepbits: int):
        if keepbits < 0:
            raise ValueError("keepbits must be zero or positive")
        self.keepbits = keepbits

    def _check(self, dtype: np.dtype) -> int:
        if not dtype.kind == "f" or dtype.itemsize > 8:
            raise TypeError("Only float arrays (16-64bit) can be bit-rounded")
        bits = max_bits[str(dtype)]  # KeyError for non-native byte order, as numcodecs
        return bits

    def encode(self, buf):
        a = ensure_ndarray_like(buf)
        device = is_device_tensor(a)
        dtype = numpy_dtype(a.dtype) if device else a.dtype
        bits = self._check(dtype)
        if self.keepbits == bits:
            return a
        if self.keepbits > bits:
            raise ValueError("Keepbits too large for given dtype")
        int_dtype = np.dtype(dtype.str.replace("f", "i"))
        shape = tuple(a.shape)
        if device:
            src = a.contiguous().reshape(-1).view(torch.uint8)  # a.copy(): C order
        else:
            src = upload(np.ascontiguousarray(a))
        n = src.numel() // dtype.itemsize
        dst = torch.empty_like(src)
        _ops.bitround(src, dst, n, dtype.itemsize, self.keepbits)
        return finish(dst, int_dtype, shape, "C", not device)

    def decode(self, buf, out=None):
        buf = ensure_ndarray_like(buf)
        if is_device_tensor(buf):
            dt = np.dtype(numpy_dtype(buf.dtype).str.replace("i", "f"))
            data = buf.view(torch_dtype(dt)) if torch_dtype(dt) is not None else buf
        else:
            dt = np.dtype(buf.dtype.str.replace("i", "f"))
            data = buf.view(dt)
        return ndarray_copy(data, out)
