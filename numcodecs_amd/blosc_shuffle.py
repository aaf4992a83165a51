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

Block size: numcodecs' Blosc default is ``blocksize=AUTOBLOCKS`` (0,
blosc.pyx:73,212,301-302), i.e. c-blosc chooses it.  :func:`compute_blocksize`
restates c-blosc 1.x's published ``compute_blocksize`` (blosc.c; c-blosc is an
empty submodule in the reference checkout, so it is restated, not compiled).
Pinned by every fixture/blosc frame written by the current c-blosc (arrays
05-12 of all 13 codec configurations: buffers under L1 = 32 KiB are one
block) and by every frame of the two configurations with a forced blocksize
(256, rounded down to a multiple of the typesize: 255 for typesize 3);
tests/test_oracle_next.py.  The frames of arrays 00-04 were written by an
older c-blosc whose small-buffer rule (128/256-byte blocks) is not restated.
Buffers of >= 32 KiB have no fixture: that branch is parity unpinned.
"""

import numpy as np

from . import _native
from ._native import check, lib
from .compat import download, empty_like_bytes, to_dbuf

__all__ = ["NOSHUFFLE", "SHUFFLE", "BITSHUFFLE", "AUTOSHUFFLE", "AUTOBLOCKS", "compute_blocksize", "shuffle",
           "unshuffle"]

NOSHUFFLE = 0
SHUFFLE = 1
BITSHUFFLE = 2
AUTOSHUFFLE = -1
AUTOBLOCKS = 0  # blosc.pyx:73

# c-blosc 1.x constants (blosc.h / blosc.c)
_L1 = 32 * 1024
_MIN_BUFFERSIZE = 128
_MAX_TYPESIZE = 255
_MAX_SPLITS = 16
_INT_MAX = 2**31 - 1
_MAX_BLOCKSIZE = (_INT_MAX - _MAX_TYPESIZE * 4) // 3
_HCR = ("zlib", "zstd", "lz4hc")  # the high-compression-ratio codecs


def _split_block(cname: str, typesize: int, blocksize: int) -> bool:
    """c-blosc's default split mode (forward-compatible): every codec but
    zstd splits a block into typesize streams when there are at least
    MIN_BUFFERSIZE elements per stream.  (Fixture frames of arrays 09-12 carry
    exactly this split flag: lz4 / zlib / blosclz / snappy split, zstd not.)"""
    return cname != "zstd" and typesize <= _MAX_SPLITS and blocksize // typesize >= _MIN_BUFFERSIZE


def compute_blocksize(nbytes: int, typesize: int, clevel: int = 5, cname: str = "lz4", blocksize: int = 0) -> int:
    """The block size c-blosc uses for a buffer (blosc.c compute_blocksize).

    ``blocksize`` = 0 (AUTOBLOCKS) picks it from the buffer size, codec and
    compression level; a forced size is clamped to [128, MAX_BLOCKSIZE].
    Either way the result never exceeds the buffer and is a multiple of the
    typesize (typesizes above 255 count as 1, as c-blosc treats them)."""
    if typesize > _MAX_TYPESIZE:
        typesize = 1
    if clevel < 0 or clevel > 9:
        raise ValueError(f"clevel must be in 0..9, got {clevel}")
    if nbytes < typesize:
        return 1
    bs = nbytes
    if blocksize:
        bs = min(max(blocksize, _MIN_BUFFERSIZE), _MAX_BLOCKSIZE)
    elif nbytes >= _L1:
        bs = _L1
        if cname in _HCR:
            bs *= 2
        bs = {0: bs // 4, 1: bs // 2, 2: bs, 3: bs * 2, 4: bs * 4, 5: bs * 4}.get(clevel, bs * 8)
        if clevel == 9 and cname in _HCR:
            bs *= 2
        # splittable codecs get larger blocks (one stream per byte of the type)
        if clevel > 0 and _split_block(cname, typesize, bs):
            bs = min(bs, 1 << 18) * typesize
            bs = min(max(bs, 1 << 16), 1 << 20)
    bs = min(bs, nbytes)
    if bs > typesize:
        bs = bs // typesize * typesize
    return bs


def _resolve(mode: int, typesize: int) -> int:
    if mode == AUTOSHUFFLE:  # blosc.pyx:270-274
        return BITSHUFFLE if typesize == 1 else SHUFFLE
    if mode not in (NOSHUFFLE, SHUFFLE, BITSHUFFLE):
        raise ValueError(f"invalid shuffle argument; expected -1, 0, 1 or 2, found {mode!r}")
    return mode


def _run(buf, typesize, blocksize, mode, forward, clevel, cname):
    if typesize is None:
        typesize = np.asarray(buf).dtype.itemsize if not hasattr(buf, "element_size") else buf.element_size()
    if typesize < 1:
        raise ValueError(f"Cannot use typesize {typesize} less than 1.")
    mode = _resolve(mode, typesize)
    src = to_dbuf(buf)
    if blocksize is None:  # one block covering the whole buffer
        blocksize = max(src.nbytes, 1)
    elif blocksize == AUTOBLOCKS:  # c-blosc's choice (numcodecs' default)
        blocksize = max(compute_blocksize(src.nbytes, typesize, clevel, cname), 1)
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


def shuffle(buf, typesize=None, blocksize=AUTOBLOCKS, mode=SHUFFLE, clevel=5, cname="lz4"):
    """Filter `buf` as Blosc does before compressing (uint8 result).  typesize
    defaults to the buffer's itemsize; blocksize to c-blosc's automatic
    choice for `clevel` / `cname` (numcodecs' Blosc defaults: lz4, 5), which
    is what a decoder reads back from the frame header.  An explicit
    blocksize is used exactly as given (the frame header's value); None
    filters the whole buffer as one block."""
    return _run(buf, typesize, blocksize, mode, True, clevel, cname)


def unshuffle(buf, typesize, blocksize=AUTOBLOCKS, mode=SHUFFLE, clevel=5, cname="lz4"):
    """Invert :func:`shuffle` (Blosc's decompression side); pass the frame
    header's blocksize, or AUTOBLOCKS with the compressing side's clevel /
    cname."""
    return _run(buf, typesize, blocksize, mode, False, clevel, cname)
