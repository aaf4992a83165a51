"""Zarr-style chunk pipelines (numcodecs_amd.chunks):
batched encode/decode of [B, chunk] device batches and host-streamed batches
must give, row by row, the bytes of the codecs applied one after another to
that chunk (which the other suites pin to the reference)."""

import numpy as np
import pytest
import torch

from numcodecs_amd import (
    CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, JenkinsLookup3,
    PackBits, Quantize, Shuffle, chunks,
)

pytestmark = pytest.mark.gpu


def _chains():
    return {
        "bitround_shuffle_crc32": ([BitRound(10), Shuffle(4), CRC32()], torch.float32),
        "fso_delta_shuffle_adler32": ([FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
                                       Delta(dtype="<i2"), Shuffle(2), Adler32(location="end")], torch.float32),
        "quantize_shuffle_fletcher32": ([Quantize(3, "<f8", "<f4"), Shuffle(4), Fletcher32()], torch.float64),
        "astype_shuffle_jenkins": ([AsType("<f4", "<f8"), Shuffle(4), JenkinsLookup3(initval=7)], torch.float64),
        "delta_shuffle_crc32c": ([Delta(dtype="<i4"), Shuffle(4), CRC32C()], torch.int32),
        "packbits": ([PackBits()], torch.bool),
    }


def _make(dtype, b, n, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    if dtype == torch.bool:
        return torch.randint(0, 2, (b, n), generator=g, device=device).to(torch.bool)
    if dtype == torch.int32:
        return torch.randint(-1000, 1000, (b, n), generator=g, device=device, dtype=torch.int32)
    return (1000 + 10 * torch.rand((b, n), generator=g, device=device)).to(dtype)


def _seq_encode(codecs, x):
    for c in codecs:
        x = c.encode(x)
    return x.contiguous().view(torch.uint8).reshape(-1)


def _seq_decode(codecs, x):
    for c in codecs[::-1]:
        x = c.decode(x)
    return x.contiguous().view(torch.uint8).reshape(-1)


@pytest.mark.parametrize("name", list(_chains()))
def test_encode_decode_chunks_rowwise(device, name):
    codecs, dtype = _chains()[name]
    x = _make(dtype, 7, 4096 * 3, device, 1)
    enc = chunks.encode_chunks(codecs, x)
    assert enc.shape[0] == 7
    enc_u8 = enc.contiguous().view(torch.uint8).reshape(7, -1)
    for i in range(7):
        assert torch.equal(enc_u8[i], _seq_encode(codecs, x[i])), (name, i)
    dec = chunks.decode_chunks(codecs, enc)
    dec_u8 = dec.contiguous().view(torch.uint8).reshape(7, -1)
    for i in range(7):
        assert torch.equal(dec_u8[i], _seq_decode(codecs, enc[i])), (name, i)


@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "quantize_shuffle_fletcher32", "astype_shuffle_jenkins"])
def test_decode_chunks_detects_corruption(device, name):
    codecs, dtype = _chains()[name]
    x = _make(dtype, 5, 4096, device, 2)
    enc = chunks.encode_chunks(codecs, x).clone()
    enc.view(torch.uint8)[3, 100] ^= 1
    with pytest.raises(RuntimeError):
        chunks.decode_chunks(codecs, enc)


@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "fso_delta_shuffle_adler32", "delta_shuffle_crc32c"])
def test_host_streamed_chunks(device, name):
    codecs, dtype = _chains()[name]
    x = _make(dtype, 23, 4096 * 2, device, 3)
    host = x.cpu().pin_memory()
    enc_host = chunks.host_encode_chunks(codecs, host, slice_chunks=4, nslots=3)
    enc_dev = chunks.encode_chunks(codecs, x).contiguous().view(torch.uint8).reshape(23, -1)
    assert torch.equal(enc_host, enc_dev.cpu())
    out = torch.empty_like(host).pin_memory()
    chunks.host_decode_chunks(codecs, enc_host, out, slice_chunks=5, nslots=2)
    ref = chunks.decode_chunks(codecs, enc_dev).contiguous().view(torch.uint8).reshape(23, -1)
    assert torch.equal(out.view(torch.uint8).reshape(23, -1), ref.cpu())


def test_host_decode_detects_corruption_after_stream(device):
    codecs, dtype = _chains()["bitround_shuffle_crc32"]
    x = _make(dtype, 9, 4096, device, 4)
    enc = chunks.host_encode_chunks(codecs, x.cpu().pin_memory(), slice_chunks=2)
    enc[6, 50] ^= 1
    out = torch.empty((9, 4096), dtype=torch.float32).pin_memory()
    with pytest.raises(RuntimeError, match="crc32 checksum do not match"):
        chunks.host_decode_chunks(codecs, enc, out, slice_chunks=2)
