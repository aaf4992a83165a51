"""Float Delta decode beyond same-type f4/f8: float16 (numpy's half loop:
float32 add rounded to half per step) and mixed dtype/astype,
np.cumsum(enc: astype, out=dec: dtype) (delta.py:69-83).  numpy runs that
accumulate in the loop dtype np.promote_types(astype, dtype) and casts each
running sum to dtype: when the loop dtype is dtype (astype no wider), the
speculative scan (mc_scan.hip, FsT<A, D>) decodes and verifies every
element, data whose every add is exact verify entirely (first-failure word
= n); when it is wider (f8 astype into f4, i4 into f4, ...) the serial chain
accumulates in it.  Bit-identical to the oracle for any data either way.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, _native, _ops, batch
from tests.helpers import delta_decode_both_schedules

pytestmark = pytest.mark.gpu

# (dtype, astype): loop dtype = dtype for the first five, wider for the rest
PAIRS = [("<f2", "<f2"), ("<f8", "<f4"), ("<f4", "<f2"), ("<f8", "<i2"), ("<f8", "<u1"),
         ("<f2", "<f4"), ("<f4", "<f8"), ("<f4", "<i4"), ("<f2", "<i2"), ("<f2", "<f8"), ("<f4", "<i8")]


def _tile(dt):
    return {2: 8192, 4: 4096, 8: 2048}[np.dtype(dt).itemsize]


def _enc(x, dt, at):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_encode(x, dt, at)


def _dec(enc, dt, at):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_decode(enc, dt, at)


def _decode_raw(enc_np, dt, at):
    """mc_delta_decode through the C ABI: (decoded array, first-failure word)."""
    dev = torch.device("cuda", 0)
    n = enc_np.size
    src = torch.from_numpy(enc_np.view(np.uint8).copy()).to(dev)
    dst = torch.empty(n * np.dtype(dt).itemsize, dtype=torch.uint8, device=dev)
    a, d = _ops.dtype_code(at), _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, d)
    ntiles = (n + _tile(dt) - 1) // _tile(dt)
    assert ws_n == ((3 * ntiles + 1) * 8 if _speculative(dt, at) else 0)
    first = delta_decode_both_schedules(src, dst, n, a, d, ws_n)
    return dst.cpu().numpy().view(np.dtype(dt)), first


def _speculative(dt, at):
    """numpy's loop dtype is dtype itself."""
    return np.promote_types(np.dtype(at), np.dtype(dt)) == np.dtype(dt)


def _exact_data(dt, at, n, seed=0):
    """Values whose every difference and every running sum is exact in both
    dtypes: small integers (|x| < 1024, steps < 16)."""
    rng = np.random.default_rng(seed)
    steps = rng.integers(-3, 4, n)
    x = np.clip(np.cumsum(steps), -1000, 1000)
    if np.dtype(at).kind == "u":
        x = np.abs(x) % 200
    return x.astype(dt)


@pytest.mark.parametrize("dt,at", PAIRS)
@pytest.mark.parametrize("n", [1, 7, 8191, 8192, 8193, 100003, (1 << 20) + 3])
def test_exact_data_verifies_whole_chunk(device, dt, at, n):
    x = _exact_data(dt, at, n, n)
    enc = _enc(x, dt, at)
    got, first = _decode_raw(enc, dt, at)
    ref = _dec(enc, dt, at)
    assert got.tobytes() == ref.tobytes(), (dt, at, n)
    assert first == (n if _speculative(dt, at) else None), (dt, at, n, first)


@pytest.mark.parametrize("dt,at", PAIRS)
def test_random_data_bit_exact(device, dt, at):
    """Adds that round (the serial chain takes over at the first one)."""
    rng = np.random.default_rng(7)
    n = 50001
    if np.dtype(at).kind == "f":
        enc = (rng.standard_normal(n) * 3.7).astype(at)
    else:
        info = np.iinfo(np.dtype(at))
        enc = rng.integers(max(info.min, -30000), min(info.max, 30000), n).astype(at)
    got, first = _decode_raw(enc, dt, at)
    assert got.tobytes() == _dec(enc, dt, at).tobytes(), (dt, at)
    assert first is None or first <= n


@pytest.mark.parametrize("pos", [0, 1, 7, 8, 511, 2047, 8191, 8192, 8193, 30000])
def test_f2_rounding_event(device, pos):
    """float16: a step of 0.1 at `pos` among exact integer steps, after which
    adds round: bit-exact (the speculation may verify past the event as long
    as rounding the exact sum agrees with the chain), and the speculation
    held at least up to the event."""
    n = 40000
    enc = _enc(_exact_data("<f2", "<f2", n, 3), "<f2", "<f2")
    enc[pos] = np.float16(0.1)
    got, first = _decode_raw(enc, "<f2", "<f2")
    assert got.tobytes() == _dec(enc, "<f2", "<f2").tobytes()
    assert pos <= first <= n


@pytest.mark.parametrize("dt,at", [("<f2", "<f2"), ("<f8", "<f4"), ("<f4", "<f2"), ("<f2", "<f4"), ("<f4", "<f8")])
@pytest.mark.parametrize("special", ["nan", "inf", "overflow", "subnormal"])
def test_special_values(device, dt, at, special):
    n = 20000
    enc = _enc(_exact_data(dt, at, n, 5), dt, at)
    with np.errstate(all="ignore"):
        if special == "nan":
            enc[9000] = np.nan
        elif special == "inf":
            enc[9000] = np.inf
        elif special == "overflow":  # the running sum leaves the dtype's range
            enc[9000] = np.finfo(np.dtype(at)).max
            enc[9001] = np.finfo(np.dtype(at)).max
        else:
            enc[9000] = np.finfo(np.dtype(at)).smallest_subnormal
    got, first = _decode_raw(enc, dt, at)
    assert got.tobytes() == _dec(enc, dt, at).tobytes(), (dt, at, special)


@pytest.mark.parametrize("dt,at", [("<f2", "<f2"), ("<f8", "<f4"), ("<f4", "<i2"), ("<f4", "<f8"), ("<f2", "<i4")])
def test_codec_and_batch_api(device, dt, at):
    """The public codec (one chunk) and batch.delta_chunks (rows: each row its
    own chain, some exact, some rounding) against the oracle."""
    d = Delta(dtype=dt, astype=at)
    n = 70001
    x = _exact_data(dt, at, n, 11)
    xd = torch.from_numpy(x.view(np.uint8).copy()).to(device)
    enc = d.encode(xd.view(torch.uint8))
    enc_np = _enc(x, dt, at)
    assert enc.cpu().numpy().view(np.uint8).tobytes() == enc_np.view(np.uint8).tobytes()
    dec = d.decode(enc)
    assert dec.cpu().numpy().view(np.uint8).tobytes() == _dec(enc_np, dt, at).view(np.uint8).tobytes()
    rows = 9
    rng = np.random.default_rng(12)
    encs = []
    for r in range(rows):
        e = _enc(_exact_data(dt, at, n, 100 + r), dt, at)
        if r % 3 == 1 and np.dtype(at).kind == "f":
            e[r * 997] = np.asarray(rng.standard_normal(), dtype=at)  # a rounding add somewhere
        encs.append(e)
    eb = torch.from_numpy(np.stack(encs).view(np.uint8).copy()).to(device)
    out = batch.delta_chunks(eb, d, encode=False)
    oh = out.cpu().numpy()
    for r in range(rows):
        assert oh[r].tobytes() == _dec(encs[r], dt, at).view(np.uint8).tobytes(), r
