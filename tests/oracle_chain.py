"""Apply a numcodecs_amd filter chain with the ORACLE (oracle/, test
infrastructure), one chunk at a time: the checker for the batched, streamed
and graph-replayed pipelines (tests/test_gpu_chunks.py, test_gpu_graphs.py).

Zarr applies a chunk's filters one after another, each codec's output handed
as a buffer to the next (the reference's harness shape, tests/common.py:51-116
of numcodecs); here every step is the oracle's restatement of that codec,
configured from the codec instance (the same attributes get_config exposes).
"""

from __future__ import annotations

import numpy as np

import oracle


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    return np.ascontiguousarray(np.asarray(x)).reshape(-1).view(np.uint8)


def encode_one(codec, x):
    """codec.encode(x) by the oracle (x: numpy array or bytes)."""
    cid = codec.codec_id
    if cid == "bitround":
        return oracle.bitround_encode(np.asarray(x), codec.keepbits)
    if cid == "shuffle":
        return oracle.shuffle(_u8(x), codec.elementsize)
    if cid == "delta":
        return oracle.delta_encode(_u8(x), codec.dtype, codec.astype)
    if cid == "fixedscaleoffset":
        return oracle.fso_encode(_u8(x), codec.offset, codec.scale, codec.dtype, codec.astype)
    if cid == "quantize":
        return oracle.quantize_encode(_u8(x), codec.digits, codec.dtype, codec.astype)
    if cid == "astype":
        return oracle.astype_encode(_u8(x), codec.encode_dtype, codec.decode_dtype)
    if cid == "packbits":
        return oracle.packbits_encode(_u8(x).view(bool))
    if cid == "fletcher32":
        return oracle.fletcher32_encode(_u8(x))
    if cid in ("crc32", "crc32c", "adler32"):
        return oracle.checksum32_encode(cid, _u8(x), codec.location)
    if cid == "jenkins_lookup3":
        pre = None if codec.prefix is None else codec.prefix.tobytes()
        return oracle.jenkins_encode(_u8(x), codec.initval, pre)
    raise NotImplementedError(cid)


def decode_one(codec, x):
    """codec.decode(x) by the oracle."""
    cid = codec.codec_id
    if cid == "bitround":
        return x  # bitround.py:71-80: the integer bits are the float bits
    if cid == "shuffle":
        return oracle.unshuffle(_u8(x), codec.elementsize)
    if cid == "delta":
        return oracle.delta_decode(_u8(x), codec.dtype, codec.astype)
    if cid == "fixedscaleoffset":
        return oracle.fso_decode(_u8(x), codec.offset, codec.scale, codec.dtype, codec.astype)
    if cid == "quantize":
        return oracle.quantize_decode(_u8(x), codec.dtype, codec.astype)
    if cid == "astype":
        return oracle.astype_decode(_u8(x), codec.encode_dtype, codec.decode_dtype)
    if cid == "packbits":
        return oracle.packbits_decode(_u8(x))
    if cid == "fletcher32":
        return oracle.fletcher32_decode(_u8(x))
    if cid in ("crc32", "crc32c", "adler32"):
        return oracle.checksum32_decode(cid, _u8(x), codec.location)
    if cid == "jenkins_lookup3":
        b = _u8(x)
        data = b[:-4]
        pre = None if codec.prefix is None else codec.prefix
        h = oracle.jenkins_lookup3(data if pre is None else np.concatenate([pre, data]), codec.initval)
        if h != int(b[-4:].view("<u4")[0]):
            raise RuntimeError("jenkins_lookup3 checksum mismatch")
        return data
    raise NotImplementedError(cid)


def chain_encode(codecs, row: np.ndarray) -> bytes:
    """The encoded bytes of one chunk: the codecs applied in order."""
    x = row
    for c in codecs:
        x = encode_one(c, x)
    return _u8(x).tobytes()


def chain_decode(codecs, enc) -> bytes:
    """The decoded bytes of one encoded chunk: the codecs in reverse order."""
    x = enc
    for c in codecs[::-1]:
        x = decode_one(c, x)
    return _u8(x).tobytes()
