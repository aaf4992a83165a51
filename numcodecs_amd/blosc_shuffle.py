"""Blosc's shuffle filters on the GPU.

numcodecs' Blosc codec (blosc.pyx:67-71, 211-326) byte-shuffles or
bit-shuffles every Blosc block before handing it to the compressor, and
inverts that after decompression; the filters themselves are c-blosc's
(shuffle.c / bitshuffle).  This module runs exactly those per-block filters
on device buffers -- the part of the Blosc pipeline that is a data-parallel
transpose -- so that a GPU Blosc pipeline (or a compressor running
elsewhere) can use them.  Compression itself is out of scope.

Semantics (pinned by the reference's fixture/blosc frames, oracle/blosc.py):
blocks of `blocksize` bytes (the last one shorter) are filtered one by one;
SHUFFLE byte-transposes each block's (bsize // typesize, typesize) matrix and
copies its bsize % typesize trailing bytes; BITSHUFFLE bit-transposes blocks
whose element count is a multiple of 8 and copies the others unchanged.
"""

import numpy as np

from . import _native
from ._native import check, lib
from .compat import download, empty_like_bytes, to_dbuf

__all__ = ["NOSHUFFLE", "SHUFFLE", "BITSHUFFLE", "AUTOSHUFFLE", "shuffle", "unshuffle"]

NOSHUFFLE = 0
SHUFFLE = 1
BITSHUFFLE = 2
AUTOSHUFFLE = -1


def _resolve(mode: int, typesize: int) -> int:
    if mode == AUTOSHUFFLE:  # blosc.pyx:270-274
        return BITSHUFFLE if typesize == 1 else SHUFFLE
    if mode not in (NOSHUFFLE, SHUFFLE, BITSHUFFLE):
        raise ValueError(f"invalid shuffle argument; expected -1, 0, 1 or 2, found {mode!r}")
    return mode


def _run(buf, typesize, blocksize, mode, forward):
    if typesize is None:
        typesize = np.asarray(buf).dtype.itemsize if not hasattr(buf, "element_size") else buf.element_size()
    if typesize < 1:
        raise ValueError(f"Cannot use typesize {typesize} less than 1.")
    mode = _resolve(mode, typesize)
    src = to_dbuf(buf)
    if blocksize is None:  # one block spanning the buffer
        blocksize = max(src.nbytes, 1)
    if blocksize < 1:
        raise ValueError("blocksize must be >= 1")
    dst = empty_like_bytes(src.nbytes, src)
    if src.nbytes:
        _native.require_device()
        from ._ops import _guard, stream

        with _guard(src.data):
            check(lib.mc_blosc_filter(src.data.data_ptr(), dst.data_ptr(), src.nbytes, typesize, blocksize,
                                      mode, 1 if forward else 0, stream(src.data)), "mc_blosc_filter")
    return download(dst) if src.host else dst


def shuffle(buf, typesize=None, blocksize=None, mode=SHUFFLE):
    """Filter `buf` as Blosc does before compressing (uint8 result).  typesize
    defaults to the buffer's itemsize, blocksize to the whole buffer."""
    return _run(buf, typesize, blocksize, mode, True)


def unshuffle(buf, typesize, blocksize, mode=SHUFFLE):
    """Invert :func:`shuffle` (Blosc's decompression side)."""
    return _run(buf, typesize, blocksize, mode, False)
