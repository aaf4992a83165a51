"""Shuffle codec (reference: src/numcodecs/shuffle.py:8-61, _shuffle.pyx:11-30).

Byte transpose of the (count, elementsize) byte matrix of a chunk, run by
the gfx950 kernels of libmcodec (csrc/mc_shuffle.hip).
"""

import numpy as np
import torch

from . import _ops
from .abc import Codec
from .compat import (
    _TORCH_TO_NP,
    device_out,
    empty_like_bytes,
    ensure_contiguous_ndarray,
    finish,
    is_device_tensor,
    to_dbuf,
    upload,
)

__all__ = ["Shuffle"]

# tensor dtypes the general path accepts (numpy equivalents exist)
_DEVICE_DTYPES = frozenset(_TORCH_TO_NP)


class Shuffle(Codec):
    """Byte shuffle (numcodecs id ``shuffle``): byte b of every
    `elementsize`-byte element goes to plane b, planes stored one after
    another.  `elementsize` <= 1 copies the bytes unchanged.
    """

    codec_id = "shuffle"

    def __init__(self, elementsize=4):
        self.elementsize = elementsize

    def _run(self, buf, out, encode):
        res = self._run_device(buf, out, encode)
        if res is not None:
            return res
        out = device_out(out)
        src = to_dbuf(buf)  # ensure_contiguous_ndarray semantics (shuffle.py:24)
        nbytes = src.nbytes
        es = self.elementsize
        if es > 1 and nbytes % es != 0:  # shuffle.py:35-36
            raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
        if out is not None and not is_device_tensor(out):
            host_out = ensure_contiguous_ndarray(out)
            if host_out.nbytes < nbytes:
                raise ValueError("output buffer is too small for the shuffled data")
            res = empty_like_bytes(nbytes, src)
        else:
            host_out = None
            if out is not None:
                out_flat = ensure_contiguous_ndarray(out)
                res = out_flat.view(torch.uint8) if out_flat.numel() else out_flat.new_empty(0, dtype=torch.uint8)
                if res.numel() < nbytes:
                    raise ValueError("output buffer is too small for the shuffled data")
                if res.device != src.data.device:
                    raise ValueError("out must be on the same device as the input")
            else:
                res = empty_like_bytes(nbytes, src)
        if es <= 1:  # no shuffling needed (shuffle.py:31-33)
            _ops.copy(src.data, res, nbytes)
        else:
            _ops.shuffle(src.data, res, nbytes, es, encode)
        if host_out is not None:
            tmp = finish(res, np.uint8, (nbytes,), "C", True)
            host_out.view(np.uint8)[:nbytes] = tmp
            return host_out
        if out is not None:
            return ensure_contiguous_ndarray(out)
        return finish(res, np.uint8, (nbytes,), "C", src.host)

    def _run_device(self, buf, out, encode):
        """The common Zarr case on its own short path: a C-contiguous device
        tensor in, a C-contiguous device tensor (or nothing) out, on the
        current device -- the same checks, errors and results as the general
        path below, without its normalisation steps (a 1 MiB chunk's codec
        call is host-bound: BASELINE C1).  None: take the general path."""
        es = self.elementsize
        if not (type(buf) is torch.Tensor and es > 1 and buf.dtype in _DEVICE_DTYPES and buf.is_contiguous()):
            return None
        if out is not None and not (type(out) is torch.Tensor and out.is_cuda and out.is_contiguous()):
            return None
        idx = _ops.current_device_index(buf)
        nbytes = buf.numel() * buf.element_size()
        if idx is None or nbytes == 0:
            return None
        if nbytes % es != 0:  # shuffle.py:35-36
            raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
        if out is None:
            res = torch.empty(nbytes, dtype=torch.uint8, device=buf.device)
        else:
            res = out.reshape(-1)
            if res.numel() * res.element_size() < nbytes:
                raise ValueError("output buffer is too small for the shuffled data")
            if res.get_device() != idx:
                raise ValueError("out must be on the same device as the input")
        _ops.shuffle_ptr(idx, buf.data_ptr(), res.data_ptr(), nbytes, es, encode)
        return res

    def encode(self, buf, out=None):
        return self._run(buf, out, True)

    def decode(self, buf, out=None):
        return self._run(buf, out, False)

    def __repr__(self):
        return f"{type(self).__name__}(elementsize={self.elementsize})"
