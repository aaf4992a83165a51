"""Fletcher32 checksum codec (reference: src/numcodecs/fletcher32.pyx:17-115).

The HDF5/netCDF Fletcher-32 (big-endian 16-bit words, 360-word folding)
computed as a parallel reduction on the GPU (csrc/mc_fletcher.hip), with the
4-byte little-endian footer of _utils.pxd:11-24.  encode returns payload +
footer; decode verifies the footer and returns the payload (a view, or a
copy into `out`), raising the reference's RuntimeError on a mismatch.
"""

import torch

from . import _ops
from .abc import Codec
from .compat import (
    device_out,
    download,
    empty_like_bytes,
    ensure_contiguous_ndarray,
    is_device_tensor,
    to_dbuf,
)

__all__ = ["Fletcher32"]

FOOTER_LENGTH = 4


def _mismatch(val, found):
    return RuntimeError(
        f"The fletcher32 checksum of the data ({val}) did not"
        f" match the expected checksum ({found}).\n"
        "This could be a sign that the data has been corrupted."
    )


class Fletcher32(Codec):
    """The fletcher checksum with 16-bit words and 32-bit output

    This is the netCDF4/HDF5 implementation (H5checksum.c), which is not the
    one described on Wikipedia.  The checksum is appended to the data bytes
    when encoding; decoding recomputes it over the data portion and compares
    with the stored footer, raising RuntimeError if inconsistent.
    """

    codec_id = "fletcher32"

    def encode(self, buf):
        """Return buffer plus a footer with the fletcher checksum (4-bytes)."""
        src = to_dbuf(buf)
        nbytes = src.nbytes
        if nbytes == 0:  # the reference indexes the first byte (fletcher32.pyx:79)
            raise IndexError("Out of bounds on buffer access (axis 0)")
        dst = empty_like_bytes(nbytes + FOOTER_LENGTH, src)
        _ops.fletcher32_encode(src.data, dst, nbytes)
        if src.host:
            return download(dst).tobytes()
        return dst

    def decode(self, buf, out=None):
        """Check fletcher checksum, and return buffer without it."""
        if out is None and type(buf) is torch.Tensor and buf.dtype is torch.uint8 and buf.dim() == 1 \
                and buf.is_cuda and buf.is_contiguous():
            # the Zarr case: launch first, host work while the kernel runs
            r = _ops.fletcher32_decode_device(buf)
            if r is not None:
                payload, val, found = r
                if val != found:
                    raise _mismatch(val, found)
                return payload
        src = to_dbuf(buf)
        nbytes = src.nbytes
        if nbytes <= FOOTER_LENGTH:  # fletcher32.pyx:95-99 index out of range
            raise IndexError("Out of bounds on buffer access (axis 0)")
        val, found = _ops.fletcher32_verify(src.data, nbytes)
        if val != found:
            raise _mismatch(val, found)
        payload = src.data[: nbytes - FOOTER_LENGTH]
        out = device_out(out)
        if out is not None:
            if is_device_tensor(out):
                out_flat = ensure_contiguous_ndarray(out)
                out_raw = out_flat.view(torch.uint8) if out_flat.numel() else out_flat.new_empty(0, dtype=torch.uint8)
                # the reference memcpys into `out` unchecked (fletcher32.pyx:107-111);
                # an undersized device buffer must not become an out-of-bounds write
                if out_raw.numel() < payload.numel():
                    raise ValueError(
                        f"cannot copy {payload.numel()} bytes into an output buffer of {out_raw.numel()} bytes"
                    )
                if out_raw.device != payload.device:
                    out_raw[: payload.numel()].copy_(payload)
                else:
                    _ops.copy(payload, out_raw, payload.numel())
                return out
            o = ensure_contiguous_ndarray(out).view("uint8")
            o[: payload.numel()] = download(payload)
            return out
        if src.host:
            # the reference returns a zero-copy memoryview slice of the input
            # (`b_mv[:-FOOTER_LENGTH]`, fletcher32.pyx:113-114)
            return memoryview(ensure_contiguous_ndarray(buf).view("uint8")[:-FOOTER_LENGTH])
        return payload
