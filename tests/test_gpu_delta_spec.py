"""Speculative float Delta decode (mc_scan.hip k_fspec_*): one f4/f8 chunk is
decoded by a parallel prefix sum whose every element is checked against
numpy's serial recurrence (delta.py:69-83, np.cumsum); the serial chain
reruns from the first element that fails.  The output must be bit-identical
to the oracle whatever the data, and for smooth data (every add exact) the
whole chunk must verify, so the fix-up launch has nothing to do.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, _native, _ops
from tests.helpers import delta_decode_both_schedules

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(1016)
TILE = 2048  # f8 tile (4 x 16-B vectors x 256 threads); the f4 tile is 4096


def _tile(dt):
    return 4096 if np.dtype(dt).itemsize == 4 else 2048


def _oracle_dec(enc, dt):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_decode(enc, dt, dt)


def _oracle_enc(x, dt):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_encode(x, dt, dt)


def _smooth(dt, n, kind):
    i = np.arange(n, dtype=np.float64)
    if kind == "ramp":
        x = 1000.0 + 0.25 * i
    elif kind == "sine":  # slowly varying, every difference exact (Sterbenz)
        x = 5000.0 + 100.0 * np.sin(2 * np.pi * i / 65536.0)
    else:  # integers stored as floats
        x = np.floor(i / 3.0) - 7.0 * (i % 5)
    return x.astype(dt)


def _decode_raw(enc_np, dt):
    """mc_delta_decode through the C ABI with our own workspace: returns
    (decoded array, first-failure word)."""
    dev = torch.device("cuda", 0)
    n = enc_np.size
    src = torch.from_numpy(enc_np).to(dev)
    dst = torch.empty_like(src)
    a = _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, a)
    ntiles = (n + _tile(dt) - 1) // _tile(dt)
    # totals, prefixes, per-tile failures, first failure
    assert ws_n == (3 * ntiles + 1) * 8
    first = delta_decode_both_schedules(src, dst, n, a, a, ws_n)
    return dst.cpu().numpy(), first


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("kind", ["ramp", "sine", "ints"])
@pytest.mark.parametrize("n", [1, 5, 1025, 2047, 2048, 2049, 4096, 4099, 100003, (1 << 20) + 3])
def test_smooth_data_verifies_whole_chunk(device, dt, kind, n):
    x = _smooth(dt, n, kind)
    enc = _oracle_enc(x, dt)
    got, first_fail = _decode_raw(enc, dt)
    ref = _oracle_dec(enc, dt)
    assert got.tobytes() == ref.tobytes()
    assert first_fail == n, f"speculation failed at {first_fail} of {n}"


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("pos", [0, 1, 2, 3, 4, 5, 1023, 1024, 2047, 2048, 2049, 4095, 4096, 4097, 6143, 50001, 99999, 100002])
def test_rounding_event_mid_chunk(device, dt, pos):
    """An inexact add at `pos`.  Whether the candidates after it still verify
    depends on the data (a later rounding of the exact sum may or may not
    agree with the chain); either way the output must equal numpy's."""
    n = 100003
    enc = _oracle_enc(_smooth(dt, n, "ramp"), dt)
    enc[pos] = np.asarray(0.1, dtype=dt)  # 1000.25*k + 0.1 is not representable
    got, _ = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("special", ["nan", "inf", "-inf", "negzero_first", "negzero_mid", "tiny", "huge"])
def test_special_values(device, dt, special):
    n = 3 * TILE + 17
    enc = _oracle_enc(_smooth(dt, n, "ints"), dt)
    fi = np.finfo(dt)
    if special == "nan":
        enc[4000] = np.nan
    elif special == "inf":
        enc[4001] = np.inf
    elif special == "-inf":
        enc[2048] = -np.inf
    elif special == "negzero_first":
        enc[0] = -0.0
    elif special == "negzero_mid":
        enc[3000] = -0.0
    elif special == "tiny":
        enc[1234] = fi.tiny / 8  # subnormal
    else:  # overflows the running sum
        enc[5000] = fi.max
        enc[5001] = fi.max
    got, _ = _decode_raw(enc, dt)
    ref = _oracle_dec(enc, dt)
    if special == "nan":  # NaN payloads are not pinned (test_gpu_delta.py)
        assert got[:4000].tobytes() == ref[:4000].tobytes()
        assert np.isnan(got[4000:]).all() and np.isnan(ref[4000:]).all()
    else:
        assert got.tobytes() == ref.tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_random_data_falls_back_to_serial(device, dt):
    enc = RNG.normal(0, 1, 3 * TILE * 7 + 5).astype(dt)
    got, first_fail = _decode_raw(enc, dt)
    assert got.tobytes() == _oracle_dec(enc, dt).tobytes()
    assert first_fail < enc.size


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_codec_roundtrip_smooth_4m(device, dt):
    """Delta(dt) encode + decode through the codec API on 4 Mi smooth values."""
    x = _smooth(dt, 1 << 22, "sine")
    xd = torch.from_numpy(x).to(device)
    enc = Delta(dt).encode(xd)
    assert enc.cpu().numpy().tobytes() == _oracle_enc(x, dt).tobytes()
    dec = Delta(dt).decode(enc)
    assert dec.cpu().numpy().tobytes() == x.tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_repeated_calls_reset_failure_word(device, dt):
    """The failure word lives in the workspace: a verified call after a
    failing one (same workspace) must not inherit the old index."""
    dev = torch.device("cuda", 0)
    n = 10 * TILE
    good = _oracle_enc(_smooth(dt, n, "ramp"), dt)
    bad = good.copy()
    bad[7] = np.inf  # non-finite: always a verification failure
    a = _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, a)
    ws = torch.zeros(ws_n // 8, dtype=torch.int64, device=dev)
    for enc in (bad, good, bad, good):
        src = torch.from_numpy(enc).to(dev)
        dst = torch.empty_like(src)
        first = delta_decode_both_schedules(src, dst, n, a, a, ws_n)
        assert dst.cpu().numpy().tobytes() == _oracle_dec(enc, dt).tobytes()
        assert first == (n if enc is good else 7)


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("n,pad", [(1, 0), (2047, 16), (4096, 0), (10007, 48), (70001, 0), (1001, -1)])
def test_batch_rows_mixed(device, dt, n, pad):
    """mc_delta_decode_batch_ws: smooth rows verify entirely (workspace[row] =
    n), rows with rounding or non-finite values finish serially; every row
    equals numpy's cumsum of that row."""
    dev = torch.device("cuda", 0)
    it = np.dtype(dt).itemsize
    rows = 37
    # 16-B aligned row strides take the speculative path; pad = -1 gives an
    # unaligned stride, which takes the serial batch path (output only checked)
    stride = n * it + 4 if pad < 0 else -(-n * it // 16) * 16 + pad
    spec = pad >= 0
    raw = np.zeros((rows, stride), dtype=np.uint8)
    encs, smooth = [], []
    for r in range(rows):
        kind = ("ramp", "sine", "ints", "random", "inf")[r % 5]
        if kind == "random":
            enc = RNG.normal(0, 1, n).astype(dt)
        else:
            enc = _oracle_enc(_smooth(dt, n, "ints" if kind == "inf" else kind), dt)
            if kind == "inf":
                enc[(r * 7919) % n] = np.inf
        encs.append(enc)
        smooth.append(kind in ("ramp", "sine", "ints"))
        raw[r, : n * it] = enc.view(np.uint8)
    src = torch.from_numpy(raw).to(dev)
    dst = torch.zeros_like(src)
    a = _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_batch_workspace(rows, n, a, a)
    assert ws_n == 8 * rows
    ws = torch.zeros(rows, dtype=torch.int64, device=dev)
    _native.check(_native.lib.mc_delta_decode_batch_ws(src.data_ptr(), stride, dst.data_ptr(), stride, rows, n,
                                                       a, a, ws.data_ptr(), ws_n, _ops.stream(src)),
                  "mc_delta_decode_batch_ws")
    got = dst.cpu().numpy()
    fails = ws.cpu().numpy()
    for r in range(rows):
        ref = _oracle_dec(encs[r], dt)
        assert got[r, : n * it].tobytes() == ref.tobytes(), r
        assert not got[r, n * it:].any()  # padding untouched
        if not spec:
            assert fails[r] == 0  # workspace untouched
        elif smooth[r]:
            assert fails[r] == n, (r, fails[r])
        elif n > 2:
            assert fails[r] < n, (r, fails[r])


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_batch_api_smooth_chunks(device, dt):
    """batch.delta_chunks decode (the batched codec path) on smooth chunks."""
    from numcodecs_amd import batch

    n = 1 << 16
    xs = np.stack([_smooth(dt, n, "sine") + np.asarray(k, dtype=dt) for k in range(24)])
    xd = torch.from_numpy(xs).to(device)
    enc = batch.delta_chunks(xd, Delta(dt), encode=True)
    dec = batch.delta_chunks(enc, Delta(dt), encode=False)
    assert dec.cpu().numpy().tobytes() == xs.tobytes()
