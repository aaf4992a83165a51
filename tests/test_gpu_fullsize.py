"""Full-size configurations of BASELINE.json on the GPU (C1-C5), checked
against SHA-256 digests of the real reference's outputs on the same portable
inputs (tests/golden/fullsize.json, made by tests/golden/make_golden.py) and
through size-independent properties (round trips, per-chunk checksums)."""

import hashlib
import json
import os

import numpy as np
import pytest
import torch

import inputs
import oracle
from numcodecs_amd import BitRound, Delta, FixedScaleOffset, Shuffle, batch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "fullsize.json")) as f:
    FULL = json.load(f)
MiB = 1 << 20


def sha_dev(t: torch.Tensor) -> str:
    return hashlib.sha256(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()


def up(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(a).to(device)


def test_c1_shuffle4_1mib(device):
    x = inputs.f32_wide(1, MiB // 4)
    assert hashlib.sha256(x.tobytes()).hexdigest() == FULL["C1"]["input"]
    xd = up(x, device)
    enc = Shuffle(4).encode(xd)
    assert sha_dev(enc) == FULL["C1"]["shuffle4"]
    assert torch.equal(Shuffle(4).decode(enc).view(torch.float32), xd)


def test_c2_shuffle4_256mib(device):
    x = inputs.f32_wide(2, 256 * MiB // 4)
    assert hashlib.sha256(x.tobytes()).hexdigest() == FULL["C2_f32"]["input"]
    xd = up(x, device)
    del x
    enc = Shuffle(4).encode(xd)
    assert sha_dev(enc) == FULL["C2_f32"]["shuffle4"]
    assert torch.equal(Shuffle(4).decode(enc).view(torch.float32), xd)
    # C3 on the same input: BitRound(10) fused with Shuffle(4)
    fused = batch.FilterPipeline([BitRound(10), Shuffle(4)]).encode(xd)
    assert sha_dev(fused) == FULL["C3"]["bitround10_shuffle4"]
    seq = Shuffle(4).encode(BitRound(10).encode(xd))
    assert torch.equal(fused, seq)


def test_c2_shuffle8_256mib(device):
    x = inputs.f64_wide(3, 256 * MiB // 8)
    assert hashlib.sha256(x.tobytes()).hexdigest() == FULL["C2_f64"]["input"]
    xd = up(x, device)
    del x
    enc = Shuffle(8).encode(xd)
    assert sha_dev(enc) == FULL["C2_f64"]["shuffle8"]
    assert torch.equal(Shuffle(8).decode(enc).view(torch.float64), xd)


def test_c4_fso_delta_shuffle2_256mib(device):
    x = inputs.f32_c4(4, 256 * MiB // 4)
    assert hashlib.sha256(x.tobytes()).hexdigest() == FULL["C4"]["input"]
    xd = up(x, device)
    del x
    fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
    delta = Delta(dtype="<i2")
    e1 = fso.encode(xd)
    assert sha_dev(e1) == FULL["C4"]["fso"]
    e2 = delta.encode(e1)
    assert sha_dev(e2) == FULL["C4"]["delta"]
    e3 = Shuffle(2).encode(e2)
    assert sha_dev(e3) == FULL["C4"]["shuffle2"]
    d = fso.decode(delta.decode(Shuffle(2).decode(e3)))
    assert sha_dev(d) == FULL["C4"]["decoded"]
    # lossy round trip bound: |x - dec| <= 0.5/scale (+ float32 rounding)
    err = (d.view(torch.float32) - xd).abs().max().item()
    assert err <= 0.5e-3 + 1e-4


def _c5_fill(x: torch.Tensor, first_chunk: int):
    """Device twin of inputs.c5_chunk_bytes_formula (int32 wrap-around is
    exact for the bits used)."""
    n = x.shape[1]
    i = torch.arange(n, dtype=torch.int32, device=x.device)
    k = torch.tensor(2654435761 - (1 << 32), dtype=torch.int32, device=x.device)
    base = i * k
    for r in range(x.shape[0]):
        c = first_chunk + r
        x[r] = (((base + c * 40503) >> 13) & 0xFF).to(torch.uint8)


def test_c5_batch_8192x1mib_shuffle_fletcher32(device):
    nchunks = 8192
    x = torch.empty((nchunks, MiB), dtype=torch.uint8, device=device)
    _c5_fill(x, 0)
    for c, ref in FULL["C5"].items():
        c = int(c)
        assert hashlib.sha256(x[c].cpu().numpy().tobytes()).hexdigest() == ref["input"]
    # device formula == host formula on a sample
    assert np.array_equal(x[3].cpu().numpy(), inputs.c5_chunk_bytes_formula(3, MiB))
    enc = batch.shuffle_fletcher32_encode_chunks(x, 4)
    for c, ref in FULL["C5"].items():
        row = enc[int(c), : MiB + 4]
        assert sha_dev(row) == ref["encoded"], c
    # every chunk: checksum of checksums against the oracle on a sample,
    # full verification + exact round trip for all 8192
    dec, status = batch.fletcher32_unshuffle_decode_chunks(enc, MiB, 4)
    st = status.cpu().numpy().view(np.uint32)
    assert (st[:, 0] == st[:, 1]).all()
    for c in (5, 777, 8000):
        assert int(st[c, 0]) == oracle.fletcher32(oracle.shuffle(x[c].cpu().numpy(), 4))
    assert torch.equal(dec, x)
