"""Float Delta decode with rounding events (mc_scan.hip k_fspec_walk): after a
failing element the walker re-bases the speculation on numpy's true value
there and verifies again, tile by tile, instead of finishing the chunk
serially (delta.py:80, np.cumsum(enc, out=dec): one rounding chain).  Every
case here is compared byte for byte with the oracle (numpy's cumsum), for
data families whose chains round every few hundred elements, rounding events
placed at tile edges, in consecutive tiles, many in one tile (the serial
fallback) and on the last element, single chunks and batches of rows.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, _native, _ops, batch
from tests.helpers import delta_decode_both_schedules

pytestmark = pytest.mark.gpu


def _tile(dt):
    return {2: 8192, 4: 4096, 8: 2048}[np.dtype(dt).itemsize]


def _oracle_dec(enc, dt, at=None):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_decode(enc, dt, at or dt)


def _oracle_enc(x, dt, at=None):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_encode(x, dt, at or dt)


def family(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    i = np.arange(n, dtype=np.float64)
    if kind == "sin4096":  # zero crossings, no offset
        return np.sin(2 * np.pi * i / 4096)
    if kind == "sin_noise":
        return np.sin(2 * np.pi * i / 4096) + 1e-3 * rng.standard_normal(n)
    if kind == "randwalk":
        return np.cumsum(rng.standard_normal(n)) * 0.01
    if kind == "sparse":  # mostly zeros, sporadic positive values
        return np.where(rng.random(n) < 0.05, rng.exponential(3.0, n), 0.0)
    if kind == "chirp":
        return np.sin(2 * np.pi * i * i / (2.0 * max(n, 1) * 64))
    if kind == "smallamp":
        return 0.01 * np.sin(2 * np.pi * i / 500) + 1e-4 * rng.standard_normal(n)
    if kind == "randn":
        return rng.standard_normal(n)
    if kind == "smooth":  # every add exact
        return 5000.0 + 100.0 * np.sin(2 * np.pi * i / 65536.0)
    raise ValueError(kind)


FAMILIES = ["sin4096", "sin_noise", "randwalk", "sparse", "chirp", "smallamp", "randn", "smooth"]


def _decode_raw(enc_np, dt, at=None):
    """mc_delta_decode through the C ABI: (decoded, first index that failed
    the apply-time verification)."""
    at = at or dt
    dev = torch.device("cuda", 0)
    n = enc_np.size
    src = torch.from_numpy(np.ascontiguousarray(enc_np)).to(dev)
    dst = torch.empty(n * np.dtype(dt).itemsize, dtype=torch.uint8, device=dev)
    a, d = _ops.dtype_code(at), _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, d)
    first = delta_decode_both_schedules(src, dst, n, a, d, ws_n)
    return dst.cpu().numpy().view(np.dtype(dt)), first


@pytest.mark.parametrize("dt", ["<f4", "<f8", "<f2"])
@pytest.mark.parametrize("kind", FAMILIES)
@pytest.mark.parametrize("n", [4099, 100003, (1 << 20) + 3])
def test_families_single_chunk(device, dt, kind, n):
    x = family(kind, n).astype(dt)
    enc = _oracle_enc(x, dt)
    got, _ = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()


@pytest.mark.parametrize("dt,at", [("<f4", "<i2"), ("<f8", "<f4"), ("<f8", "<i4"), ("<f4", "<f2")])
@pytest.mark.parametrize("kind", ["sin_noise", "randwalk", "randn"])
def test_families_mixed_astype(device, dt, at, kind):
    """astype != dtype: numpy's loop dtype is dtype here (speculative path)."""
    n = 200003
    x = family(kind, n) * (1000.0 if np.dtype(at).kind == "i" else 1.0)
    enc = _oracle_enc(x.astype(dt), dt, at)
    got, _ = _decode_raw(enc, dt, at)
    assert got.tobytes() == _oracle_dec(enc, dt, at).tobytes()


def _events(dt, n, positions, value=0.1):
    """Ramp data (every add exact) with an inexact add at each position."""
    i = np.arange(n, dtype=np.float64)
    step = 0.25 if np.dtype(dt).itemsize > 2 else 1.0 / 1024
    enc = _oracle_enc((1000.0 * step * 4 + step * i).astype(dt), dt)
    for p in positions:
        enc[p] = np.asarray(value, dtype=dt)
    return enc


@pytest.mark.parametrize("dt", ["<f4", "<f8", "<f2"])
def test_events_at_tile_edges_and_last_element(device, dt):
    T = _tile(dt)
    n = 9 * T + 5
    pos = [1, T - 1, T, T + 1, 2 * T - 1, 2 * T, 3 * T + 7, 4 * T - 1, 5 * T, 6 * T, 7 * T, 8 * T + 1, n - 1]
    enc = _events(dt, n, pos)
    got, first = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()
    assert 1 <= first <= n  # nothing can fail before the first event


@pytest.mark.parametrize("dt", ["<f4", "<f8", "<f2"])
def test_events_in_consecutive_tiles(device, dt):
    T = _tile(dt)
    n = 40 * T
    pos = sorted({t * T + (t * 37) % T for t in range(3, 38)})
    enc = _events(dt, n, pos, 0.3)
    got, _ = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("every", [3, 17, 97])
def test_many_events_in_one_tile_serial_fallback(device, dt, every):
    """More re-basings in one tile than the walker allows (FSW_CAP): that
    tile finishes serially, the following ones speculate again."""
    T = _tile(dt)
    n = 12 * T + 11
    pos = list(range(2 * T + 5, 3 * T, every)) + [7 * T + 3, n - 1]
    enc = _events(dt, n, pos, 0.1)
    got, _ = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_nonfinite_after_events(device, dt):
    T = _tile(dt)
    n = 6 * T + 3
    enc = _events(dt, n, [100, T + 5, 2 * T + 9])
    enc[3 * T + 1] = np.inf
    enc[4 * T + 2] = -np.inf  # inf + -inf = NaN from here on
    got, _ = _decode_raw(enc, dt)
    ref = _oracle_dec(enc, dt)
    k = 4 * T + 2
    assert got[:k].tobytes() == ref[:k].tobytes()
    assert np.isnan(got[k:]).all() and np.isnan(ref[k:]).all()


def test_resync_jumps_over_verified_tiles(device):
    """Drift that returns to zero (isolated rounding that the next difference
    undoes): the walker catches up with the apply pass and jumps ahead; the
    output is exact either way."""
    dt = "<f4"
    T = _tile(dt)
    n = 64 * T
    i = np.arange(n, dtype=np.float64)
    x = (1000.0 + 0.25 * i).astype(dt)
    enc = _oracle_enc(x, dt)
    for p in (3 * T + 100, 20 * T + 7, 41 * T + T - 1):
        enc[p] = enc[p] + np.float32(1e-4)   # the add at p rounds ...
        enc[p + 1] = enc[p + 1] - np.float32(1e-4)  # ... and this one takes it back
    got, _ = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8", "<f2"])
@pytest.mark.parametrize("n,pad", [(4099, 0), (70001, 48), (262144, 0)])
def test_batch_rows_families(device, dt, n, pad):
    """mc_delta_decode_batch_ws: one walker per row; smooth rows verify
    (workspace[row] = n), rows with rounding events report where the first
    re-basing happened (< n); every row equals numpy's cumsum."""
    dev = torch.device("cuda", 0)
    it = np.dtype(dt).itemsize
    kinds = FAMILIES * 3
    rows = len(kinds)
    stride = -(-n * it // 16) * 16 + pad
    raw = np.zeros((rows, stride), dtype=np.uint8)
    encs = []
    for r, kind in enumerate(kinds):
        enc = _oracle_enc(family(kind, n, seed=r).astype(dt), dt)
        encs.append(enc)
        raw[r, : n * it] = enc.view(np.uint8)
    src = torch.from_numpy(raw).to(dev)
    dst = torch.zeros_like(src)
    a = _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_batch_workspace(rows, n, a, a)
    ws = torch.zeros(rows, dtype=torch.int64, device=dev)
    _native.check(_native.lib.mc_delta_decode_batch_ws(src.data_ptr(), stride, dst.data_ptr(), stride, rows, n,
                                                       a, a, ws.data_ptr(), ws_n, _ops.stream(src)),
                  "mc_delta_decode_batch_ws")
    got = dst.cpu().numpy()
    fails = ws.cpu().numpy()
    for r in range(rows):
        assert got[r, : n * it].tobytes() == _oracle_dec(encs[r], dt).tobytes(), (r, kinds[r])
        assert not got[r, n * it:].any()
        if kinds[r] == "smooth" and dt != "<f2":
            assert fails[r] == n, (r, fails[r])
        assert 0 <= fails[r] <= n


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_codec_and_batch_api_noisy(device, dt):
    """The codec and batched APIs on noisy zero-crossing data."""
    n = (1 << 18) + 5
    xs = np.stack([family("sin_noise", n, seed=k).astype(dt) for k in range(6)])
    xd = torch.from_numpy(xs).to(device)
    enc = batch.delta_chunks(xd, Delta(dt), encode=True)
    dec = batch.delta_chunks(enc, Delta(dt), encode=False).cpu().numpy()
    for k in range(6):
        assert dec[k].tobytes() == _oracle_dec(_oracle_enc(xs[k], dt), dt).tobytes()
    one = Delta(dt).decode(Delta(dt).encode(xd[2])).cpu().numpy()
    assert one.tobytes() == _oracle_dec(_oracle_enc(xs[2], dt), dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("src_off,dst_off", [(0, 0), (4, 4), (8, 8), (12, 12), (4, 0), (0, 8), (12, 4)])
def test_serial_chain_buffer_offsets(device, dt, src_off, dst_off):
    """Noise decoded by the serial chains with the buffers at every 4-B
    offset: equal offsets modulo 16 take the vector-fed chain
    (mc_scan.h ser_chain_vbc, for f4) with its unaligned head and tail,
    unequal ones the LDS-fed chain; both equal numpy's cumsum bit for bit."""
    es = np.dtype(dt).itemsize
    if src_off % es or dst_off % es:
        pytest.skip("element-aligned offsets only")
    n = 3 * _tile(dt) * 64 + 37  # several walker stretches and a ragged end
    x = family("randn", n, seed=5).astype(dt)
    enc = _oracle_enc(x, dt)
    want = _oracle_dec(enc, dt)
    dev = torch.device("cuda", 0)
    sbuf = torch.zeros(n * es + 64, dtype=torch.uint8, device=dev)
    dbuf = torch.zeros(n * es + 64, dtype=torch.uint8, device=dev)
    sbuf[src_off:src_off + n * es] = torch.from_numpy(enc.view(np.uint8).copy()).to(dev)
    src = sbuf[src_off:src_off + n * es]
    dst = dbuf[dst_off:dst_off + n * es]
    _ops.delta_decode(src, dst, n, dt, dt)
    torch.cuda.synchronize()
    assert dst.cpu().numpy().tobytes() == want.tobytes()
