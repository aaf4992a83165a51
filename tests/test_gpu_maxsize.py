"""Chunks past 4 GiB (byte offsets and element counts beyond 32 bits) through
the device kernels, bit-exact against the oracle on the whole buffer: every
32-bit index, tile count or weight that could overflow shows up here.  The
reference handles such chunks with size_t loops (_shuffle.pyx:11-30,
fletcher32.pyx:24-57) and numpy/zlib."""

import zlib

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, Fletcher32, Shuffle, batch

pytestmark = pytest.mark.gpu

GiB = 1 << 30
N4 = 4 * GiB + 4096 + 12  # ragged: not a multiple of any tile size
N8 = 4 * GiB + 4104


@pytest.fixture(scope="module")
def big(device):
    g = torch.Generator(device=device).manual_seed(4242)
    x = torch.randint(0, 256, (N4,), dtype=torch.uint8, device=device, generator=g)
    return x, x.cpu().numpy()


def test_shuffle4_over_4gib(device, big):
    x, xh = big
    enc = Shuffle(4).encode(x)
    ref = oracle.shuffle(xh, 4)
    assert torch.equal(enc.cpu(), torch.from_numpy(ref))
    del ref
    assert torch.equal(Shuffle(4).decode(enc), x)


def test_shuffle8_over_4gib(device, big):
    x, _ = big
    x8 = x[:N8]
    enc = Shuffle(8).encode(x8)
    ref = oracle.shuffle(x8.cpu().numpy(), 8)
    assert torch.equal(enc.cpu(), torch.from_numpy(ref))
    del ref
    assert torch.equal(Shuffle(8).decode(enc), x8)


def test_fletcher32_over_4gib(device, big):
    x, xh = big
    assert int(batch.fletcher32_chunks(x.view(1, -1))[0]) & 0xFFFFFFFF == oracle.fletcher32(xh)
    enc = Fletcher32().encode(x)
    assert enc.numel() == N4 + 4
    assert int.from_bytes(enc[-4:].cpu().numpy().tobytes(), "little") == oracle.fletcher32(xh)


@pytest.mark.parametrize("cid,fn", [("crc32", zlib.crc32), ("adler32", zlib.adler32)])
def test_checksum32_over_4gib(device, big, cid, fn):
    x, xh = big
    got = int(batch.checksum32_chunks(x.view(1, -1), cid)[0]) & 0xFFFFFFFF
    assert got == fn(memoryview(xh))


def test_delta_i1_decode_over_4gib(device, big):
    """cumsum of > 2^32 int8 values (3-pass scan, > 2^20 tiles): every output
    differs from its predecessor by the input element (mod 256)."""
    x, _ = big
    enc = x.view(torch.int8)
    dec = Delta("|i1").decode(enc).view(torch.int8)
    assert dec.numel() == N4
    assert int(dec[0]) == int(enc[0])
    d = (dec[1:].to(torch.int16) - dec[:-1].to(torch.int16)) & 0xFF
    assert torch.equal(d, enc[1:].to(torch.int16) & 0xFF)
    # and the final value is the total sum of the input mod 256
    total = int(enc.sum(dtype=torch.int64)) & 0xFF
    assert int(dec[-1]) & 0xFF == total
