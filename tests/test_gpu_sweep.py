"""Randomised parity sweeps on the GPU against the oracle: every element size,
sizes on both sides of every fast-path boundary (tile multiples, count % 4,
count % 16, tails), misaligned device views, every kernel variant, fused
BitRound+Shuffle for f16/f32/f64, and padded batch strides."""

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import BitRound, Shuffle, batch
from tests.helpers import lab_lib

pytestmark = pytest.mark.gpu
RNG = np.random.default_rng(2024)


def _counts():
    base = [1, 2, 3, 4, 5, 15, 16, 17, 255, 1023, 1024, 1025, 4095, 4096, 4097, 4100,
            8192, 16384, 16388, 16400, 32768 + 16, 65536, 65536 + 4]
    return base


@pytest.mark.parametrize("es", [1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16])
def test_shuffle_sizes(device, es):
    for count in _counts():
        x = RNG.integers(0, 256, es * count, dtype=np.uint8)
        xd = torch.from_numpy(x).to(device)
        ref = oracle.shuffle(x, es)
        enc = Shuffle(es).encode(xd)
        assert np.array_equal(enc.cpu().numpy(), ref), (es, count)
        assert torch.equal(Shuffle(es).decode(enc), xd), (es, count)


@pytest.mark.parametrize("es", [2, 4, 8, 16])
def test_shuffle_every_variant(device, es):
    """Every kernel layout (register, LDS-plane, LDS-both, generic, lane-pair,
    big tiles, grouped and pipelined schedules, nt on/off) on sizes with and
    without a tail, through the tuning entry point."""
    st = torch.cuda.current_stream().cuda_stream
    lib = lab_lib()
    variants = [1, 2, 3, 4, 9, 10, 11, 17, 129, 33, 65, 257, 273, 385, 5, 21, 133, 6, 22, 134,
                513, 517, 518, 521, 769]  # | 512: 8x tiles (518 / 769 fall back to valid layouts)
    for count in (4096 * 16 + 64, 16384 * 8, 4096 * 3 + 4, 32768 * 4 + 8):
        n = es * count
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=device)
        ref = oracle.shuffle(x.cpu().numpy(), es)
        for v in variants:
            if (v & 7) == 5 and es not in (4, 8):
                continue
            for grid in (0, 7, 100000):
                y = torch.empty_like(x)
                z = torch.empty_like(x)
                assert lib.mc_lab_shuffle_variant(x.data_ptr(), y.data_ptr(), n, es, 1, v, grid, st) == 0
                assert lib.mc_lab_shuffle_variant(y.data_ptr(), z.data_ptr(), n, es, 0, v, grid, st) == 0
                assert np.array_equal(y.cpu().numpy(), ref), (es, count, v, grid)
                assert torch.equal(z, x), (es, count, v, grid)


def test_shuffle_misaligned_views(device):
    base = torch.randint(0, 256, (8 * 40000 + 64,), dtype=torch.uint8, device=device)
    for es in (2, 4, 8):
        for off in (1, 2, 4, 8, 12):
            x = base[off: off + es * 40000]
            ref = oracle.shuffle(x.cpu().numpy(), es)
            enc = Shuffle(es).encode(x)
            assert np.array_equal(enc.cpu().numpy(), ref), (es, off)
            out = base.new_empty(es * 40000 + 16)[3: 3 + es * 40000]  # misaligned output
            Shuffle(es).decode(enc, out=out)
            assert torch.equal(out, x), (es, off)


@pytest.mark.parametrize("dt,kmax", [("<f2", 10), ("<f4", 23), ("<f8", 52)])
def test_bitround_shuffle_fused(device, dt, kmax):
    es = np.dtype(dt).itemsize
    for count in (4096 * 8, 4096 * 8 + 4, 1000, 65536 * 3, (64 << 20) // es + 32768 * 2 + 4):
        bits = RNG.integers(0, 2**63, count, dtype=np.uint64)
        x = bits.astype({2: np.uint16, 4: np.uint32, 8: np.uint64}[es]).view(dt)
        xd = torch.from_numpy(x.copy()).to(device)
        for k in (0, 3, kmax // 2, kmax - 1, kmax):
            pipe = batch.FilterPipeline([BitRound(k), Shuffle(es)])
            enc = pipe.encode(xd)
            with np.errstate(all="ignore"):
                ref = oracle.shuffle(oracle.bitround_encode(x.copy(), k), es)
            assert np.array_equal(enc.cpu().numpy().view(np.uint8), ref), (dt, count, k)


def test_batch_padded_strides(device):
    b, n = 11, 4096 * 4 * 2
    big = torch.randint(0, 256, (b, n + 256), dtype=torch.uint8, device=device)
    rows = big[:, :n]  # padded row stride
    out = torch.zeros((b, n + 512), dtype=torch.uint8, device=device)[:, :n]
    batch.shuffle_chunks(rows, 4, out=out)
    for c in range(b):
        assert np.array_equal(out[c].cpu().numpy(), oracle.shuffle(rows[c].cpu().numpy(), 4))
    back = batch.unshuffle_chunks(out, 4)
    assert torch.equal(back, rows)


def test_fletcher32_sizes_device(device):
    from numcodecs_amd import Fletcher32

    for n in (1, 2, 3, 15, 16, 17, 359 * 2, 360 * 2, 361 * 2 + 1, 65535 * 2, 65535 * 2 + 1,
              (1 << 20) + 7, (1 << 22) + 16):
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=device)
        enc = Fletcher32().encode(x)
        ref = oracle.fletcher32(x.cpu().numpy())
        assert int.from_bytes(enc[-4:].cpu().numpy().tobytes(), "little") == ref, n
    # all-0xFF and all-zero edge values
    for fill in (0, 255):
        x = torch.full((720 * 7 + 3,), fill, dtype=torch.uint8, device=device)
        enc = Fletcher32().encode(x)
        assert int.from_bytes(enc[-4:].cpu().numpy().tobytes(), "little") == oracle.fletcher32(
            x.cpu().numpy())
