"""PackBits filter (reference: src/numcodecs/packbits.py:7-82).

encode: booleans -> ``[n_bits_padded] ++ np.packbits(arr)`` (MSB first);
decode: ``np.unpackbits`` minus the padding, as a bool array (copied into
`out` when given).  Both directions are one GPU pass (csrc/mc_bits.hip).
"""

import numpy as np
import torch

from . import _ops
from .abc import Codec
from .compat import download, empty_like_bytes, finish, ndarray_copy, to_dbuf

__all__ = ["PackBits"]


class PackBits(Codec):
    """Booleans to bits, eight per byte, most significant bit first
    (numcodecs id ``packbits``).  The encoded buffer starts with one byte
    holding the number of padding bits in the last byte.
    """

    codec_id = "packbits"

    def encode(self, buf):
        # ensure_ndarray(buf).view(bool).reshape(-1, order='A')
        src = to_dbuf(buf, flatten=True, contiguous=False)
        n = src.nbytes  # one bool per byte
        dst = empty_like_bytes(1 + (n + 7) // 8, src)
        _ops.packbits(src.data, dst, n)
        return finish(dst, np.dtype("u1"), (dst.numel(),), "C", src.host)

    def decode(self, buf, out=None):
        src = to_dbuf(buf, flatten=True, contiguous=False)
        nb = src.nbytes
        if nb == 0:  # enc[0] of an empty array
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        if not src.host:
            dst = _ops.unpackbits_device(src.data, nb)
            if dst is not None:
                return ndarray_copy(dst.view(torch.bool), out)
        pad = int(download(src.data[:1])[0])
        n = max(8 * (nb - 1) - pad, 0)
        dst = empty_like_bytes(n, src)
        _ops.unpackbits(src.data, nb, dst, n)
        if src.host:
            dec = download(dst).view(bool)
        else:
            dec = dst.view(torch.bool)
        return ndarray_copy(dec, out)
