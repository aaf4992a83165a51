"""32-bit checksum codecs (reference: src/numcodecs/checksum32.py:45-209).

CRC32, CRC32C, Adler32 and JenkinsLookup3 with the reference's framing:
``Checksum32.encode`` returns the little-endian checksum followed by the
payload (``location='start'``) or the payload followed by it (``'end'``), and
``decode`` verifies it and returns the payload, raising the reference's
RuntimeError on a mismatch.  The checksums run on the GPU
(csrc/mc_checksum.hip, mc_crc_bs.hip): CRC32/CRC32C as a generated bit-sliced
XOR network over each loaded dword (no table lookups, since round 3) with
GF(2) tile combination, Adler32 as a weighted parallel reduction, Jenkins lookup3
serially per chunk (its mixing rounds have no parallel form; batches of chunks
run in parallel, see ``numcodecs_amd.batch.checksum32_chunks``).

CRC32C is always available here: the reference defines it only when the
third-party ``google_crc32c`` or ``crc32c`` package is installed
(checksum32.py:19-40, 189-209); the device kernel needs neither.
"""

import numpy as np
import torch

from . import _native, _ops
from .abc import Codec
from .compat import (
    device_out,
    download,
    empty_like_bytes,
    ensure_contiguous_ndarray,
    is_device_tensor,
    ndarray_copy,
    to_dbuf,
)

__all__ = ["CRC32", "CRC32C", "Adler32", "Checksum32", "JenkinsLookup3", "jenkins_lookup3"]

CHECKSUM_LOCATION = ("start", "end")


def _raw(t: torch.Tensor) -> torch.Tensor:
    return t.view(torch.uint8) if t.numel() else t.new_empty(0, dtype=torch.uint8)


def _checksum_of(kind, data, value, prefix=None) -> int:
    """One checksum of a host buffer or device tensor, computed on the GPU."""
    src = to_dbuf(data)
    n = src.nbytes
    res = _ops.checksum32(kind, src.data, n, 1, n, value, prefix)
    return int(download(_raw(res)).view("<u4")[0])


def _buffer_len(buf) -> int:
    if is_device_tensor(buf):
        return buf.numel() * buf.element_size()
    return len(buf)


class Checksum32(Codec):
    """Checksum32 base (checksum32.py:45-92): checksum + payload framing."""

    #: where the checksum is stored, 'start' or 'end' (override in sub-class)
    location = "start"
    _kind: int = -1
    _value: int = 0

    def __init__(self, location=None):
        if location is not None:
            self.location = location
        if self.location not in CHECKSUM_LOCATION:
            raise ValueError(f"Invalid checksum location: {self.location}")

    def _loc(self) -> int:
        return _native.MC_CK_START if self.location == "start" else _native.MC_CK_END

    def encode(self, buf):
        src = to_dbuf(buf)
        n = src.nbytes
        dst = empty_like_bytes(n + 4, src)
        _ops.checksum32_encode(self._kind, src.data, n, dst, n + 4, 1, n, self._value, self._loc())
        return download(dst) if src.host else dst

    def decode(self, buf, out=None):
        if out is None and type(buf) is torch.Tensor and buf.dtype is torch.uint8 and buf.dim() == 1 \
                and buf.is_cuda and buf.is_contiguous():
            # the Zarr case: launch first, host work while the kernel runs
            r = _ops.checksum32_decode_device(self._kind, buf, self._value & 0xFFFFFFFF, self._loc())
            if r is not None:
                payload, checksum, expect = r
                if expect != checksum:
                    raise RuntimeError(
                        f"Stored and computed {self.codec_id} checksum do not match. "
                        f"Stored: {expect}. Computed: {checksum}."
                    )
                return payload
        if _buffer_len(buf) < 4:
            raise ValueError("Input buffer is too short to contain a 32-bit checksum.")
        if out is not None:
            ensure_contiguous_ndarray(out)  # check that out is a valid ndarray
        src = to_dbuf(buf)
        n = src.nbytes
        if n < 4:
            raise ValueError("Input buffer is too short to contain a 32-bit checksum.")
        payload = src.data[4:] if self.location == "start" else src.data[: n - 4]
        checksum, expect = _ops.checksum32_verify(self._kind, src.data, n, self._value, self._loc())
        if expect != checksum:
            raise RuntimeError(
                f"Stored and computed {self.codec_id} checksum do not match. "
                f"Stored: {expect}. Computed: {checksum}."
            )
        if src.host:
            arr = ensure_contiguous_ndarray(buf).view("u1")
            payload_view = arr[4:] if self.location == "start" else arr[:-4]
            return ndarray_copy(payload_view, out)
        return ndarray_copy(payload, out)


class CRC32(Checksum32):
    """Codec add a crc32 checksum to the buffer.

    Parameters
    ----------
    location : 'start' or 'end'
        Where to place the checksum in the buffer.
    """

    codec_id = "crc32"
    location = "start"
    _kind = _native.MC_CK_CRC32
    _value = 0

    @staticmethod
    def checksum(data, value: int = 0) -> int:
        """zlib.crc32(data, value), computed on the GPU."""
        return _checksum_of(_native.MC_CK_CRC32, data, value)


class Adler32(Checksum32):
    """Codec add a adler32 checksum to the buffer.

    Parameters
    ----------
    location : 'start' or 'end'
        Where to place the checksum in the buffer.
    """

    codec_id = "adler32"
    location = "start"
    _kind = _native.MC_CK_ADLER32
    _value = 1

    @staticmethod
    def checksum(data, value: int = 1) -> int:
        """zlib.adler32(data, value), computed on the GPU."""
        return _checksum_of(_native.MC_CK_ADLER32, data, value)


class CRC32C(Checksum32):
    """Codec add a crc32c checksum to the buffer.

    Parameters
    ----------
    location : 'start' or 'end'
        Where to place the checksum in the buffer.
    """

    codec_id = "crc32c"
    location = "end"
    _kind = _native.MC_CK_CRC32C
    _value = 0

    @staticmethod
    def checksum(data, value: int = 0) -> int:
        """CRC-32C (Castagnoli) of data continuing from `value`, on the GPU."""
        return _checksum_of(_native.MC_CK_CRC32C, data, value)


def jenkins_lookup3(data, initval: int = 0) -> int:
    """jenkins.pyx:93-219 -- Bob Jenkins' lookup3 hash (HDF5 variant) of
    `data`, computed on the GPU."""
    return _checksum_of(_native.MC_CK_JENKINS, data, initval)


class JenkinsLookup3(Checksum32):
    """Bob Jenkin's lookup3 checksum with 32-bit output

    This is the HDF5 implementation.  The checksum is concatenated on the end
    of the data bytes when encoded.  At decode time, the checksum is performed
    on the data portion and compared with the four-byte checksum, raising
    RuntimeError if inconsistent.

    Parameters
    ----------
    initval : int
        initial seed passed to the hash algorithm, default: 0
    prefix : int
        bytes prepended to the buffer before evaluating the hash, default: None
    """

    checksum = staticmethod(jenkins_lookup3)
    codec_id = "jenkins_lookup3"

    def __init__(self, initval: int = 0, prefix=None):
        self.initval = initval
        if prefix is None:
            self.prefix = None
        else:
            self.prefix = np.frombuffer(prefix, dtype="uint8")

    def _hash(self, data: torch.Tensor, n: int) -> torch.Tensor:
        return _ops.checksum32(_native.MC_CK_JENKINS, data, n, 1, n, self.initval, self.prefix)

    def encode(self, buf):
        """Return buffer plus 4-byte Bob Jenkin's lookup3 checksum"""
        src = to_dbuf(buf)
        n = src.nbytes
        dst = empty_like_bytes(n + 4, src)
        _ops.checksum32_encode(_native.MC_CK_JENKINS, src.data, n, dst, n + 4, 1, n, self.initval,
                               _native.MC_CK_END, self.prefix)
        if src.host:
            return download(dst).tobytes()
        return dst

    def decode(self, buf, out=None):
        """Check Bob Jenkin's lookup3 checksum, and return buffer without it"""
        src = to_dbuf(buf)
        n = src.nbytes
        if n < 4:  # b[-4:].view('<u4') of fewer than 4 bytes fails in numpy
            raise ValueError("When changing to a larger dtype, its size must be a divisor of the total size")
        val, found = _ops.checksum32_verify(_native.MC_CK_JENKINS, src.data, n, self.initval, _native.MC_CK_END,
                                            self.prefix)
        if val != found:
            raise RuntimeError(
                f"The Bob Jenkin's lookup3 checksum of the data ({val}) did not"
                f" match the expected checksum ({found}).\n"
                "This could be a sign that the data has been corrupted."
            )
        out = device_out(out)
        if out is not None:
            if is_device_tensor(out):
                return ndarray_copy(src.data[: n - 4], out)
            out.view("uint8")[:] = download(src.data[: n - 4]) if not src.host else \
                ensure_contiguous_ndarray(buf).view("uint8")[:-4]
            return out
        if src.host:
            return memoryview(ensure_contiguous_ndarray(buf).view("uint8")[:-4])
        return src.data[: n - 4]
