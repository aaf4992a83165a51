"""mc_copy / mc_copy_rows (the codecs' pass-through copies: Shuffle with
elementsize <= 1, AsType to the same dtype, decode into `out`, Jenkins and
unfiltered Blosc blocks) -- byte-exact for every alignment class and size
around the 32 KiB tile, and through the codecs that use them."""

import ctypes

import numpy as np
import pytest
import torch

from numcodecs_amd import AsType, BitRound, Shuffle, _native, _ops

pytestmark = pytest.mark.gpu

SIZES = [1, 15, 16, 17, 4095, 32767, 32768, 32769, 65536 + 48, (1 << 20) + 3, (16 << 20) + 16]


@pytest.mark.parametrize("soff,doff", [(0, 0), (4, 4), (4, 8), (1, 1), (3, 0), (0, 12)])
def test_copy_sizes_offsets(device, soff, doff):
    for n in SIZES:
        src = torch.randint(0, 256, (n + soff,), dtype=torch.uint8, device=device)
        dst = torch.zeros(n + doff + 16, dtype=torch.uint8, device=device)
        _ops.copy(src[soff:], dst[doff:], n)
        assert torch.equal(dst[doff: doff + n], src[soff:]), (n, soff, doff)
        assert not dst[:doff].any() and not dst[doff + n:].any(), (n, soff, doff)


@pytest.mark.parametrize("width,rows,sstride,dstride", [
    (4096, 7, 4096, 4096), (1000, 37, 1004, 1000), (4100, 5, 4116, 4104), (33, 9, 40, 35), ((1 << 20) + 4, 3, (1 << 20) + 8, (1 << 20) + 4),
])
def test_copy_rows(device, width, rows, sstride, dstride):
    src = torch.randint(0, 256, (rows * sstride,), dtype=torch.uint8, device=device)
    dst = torch.zeros(rows * dstride, dtype=torch.uint8, device=device)
    lib = _native.lib
    rc = lib.mc_copy_rows(src.data_ptr(), sstride, dst.data_ptr(), dstride, width, rows,
                          _ops.stream(src))
    assert rc == 0
    torch.cuda.synchronize()
    s = src.view(rows, sstride)[:, :width]
    d = dst.view(rows, dstride)
    assert torch.equal(d[:, :width], s)
    assert not d[:, width:].any()


def test_copy_invalid_args(device):
    lib = _native.lib
    assert lib.mc_copy(None, None, 0, None) == 0
    assert lib.mc_copy(None, ctypes.c_void_p(16), 5, None) == _native.MC_EINVAL
    assert lib.mc_copy_rows(ctypes.c_void_p(16), 4, ctypes.c_void_p(64), 8, 8, 2, None) == _native.MC_EINVAL


def test_passthrough_codecs_use_the_copy(device):
    x = torch.randn(1 << 20, device=device)
    raw = x.view(torch.uint8)
    assert torch.equal(Shuffle(1).encode(x), raw)
    assert torch.equal(Shuffle(1).decode(Shuffle(1).encode(x)), raw)
    assert torch.equal(AsType("<f4", "<f4").encode(x), x)
    assert torch.equal(BitRound(23).encode(x).view(torch.float32), x)
    out = torch.empty_like(x)
    BitRound(10).decode(BitRound(10).encode(x), out=out)
    ref = BitRound(10).encode(x.cpu().numpy())
    assert np.array_equal(out.cpu().numpy().view("<i4"), np.asarray(ref).view("<i4"))
