"""Delta decode paths on the GPU beyond the reference's own cases
(delta.py:52-83; tests/test_delta.py of numcodecs):

* float dtypes keep numpy's left-to-right rounding order (np.cumsum is one
  dependent add chain): the chain kernel must be bit-exact at every block
  boundary of its double-buffered LDS staging, for every float width, mixed
  astype, non-finite values and unaligned buffers;
* batched Delta (numcodecs_amd.batch.delta_chunks, mc_delta_{en,de}code_batch):
  every chunk of a [B, n] batch is its own Delta, row by row identical to the
  oracle, for padded row strides and odd lengths.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, batch

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(20261016)
# the chain kernel stages 32 KiB per LDS slot: 8192 f4 / 4096 f8 / 8192 f2 values
SIZES = [1, 2, 7, 8, 9, 4095, 4096, 4097, 8191, 8192, 8193, 16385, 100003]


def _float_data(dt, n):
    x = RNG.normal(0, 1, n).astype(dt)
    if n > 50:  # sprinkle non-finite and subnormal values after the start
        x[n // 3] = np.inf
        x[n // 2] = -np.inf
        x[n // 5] = np.finfo(dt).tiny / 4
    return x


def _oracle_dec(enc, dt, astype):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_decode(enc, dt, astype)


def _oracle_enc(x, dt, astype):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_encode(x, dt, astype)


@pytest.mark.parametrize("dt", ["<f2", "<f4", "<f8"])
@pytest.mark.parametrize("n", SIZES)
def test_float_delta_decode_exact(device, dt, n):
    enc = _float_data(dt, n)
    got = Delta(dt).decode(torch.from_numpy(enc).to(device)).cpu().numpy()
    ref = _oracle_dec(enc, dt, dt)
    assert got.tobytes() == ref.tobytes(), (dt, n)


@pytest.mark.parametrize("dt,astype", [("<f8", "<f4"), ("<f8", "<f2"), ("<f4", "<f2"), ("<f8", "<i2"),
                                       ("<f4", "<i4")])
def test_float_delta_decode_mixed_astype(device, dt, astype):
    n = 20011
    enc = RNG.integers(-100, 100, n).astype(astype)
    got = Delta(dt, astype).decode(torch.from_numpy(enc).to(device)).cpu().numpy()
    assert got.tobytes() == _oracle_dec(enc, dt, astype).tobytes()


def test_float_delta_decode_nan_propagates(device):
    enc = RNG.normal(0, 1, 9000).astype("<f4")
    enc[5000] = np.nan
    got = Delta("<f4").decode(torch.from_numpy(enc).to(device)).cpu().numpy()
    ref = _oracle_dec(enc, "<f4", "<f4")
    assert np.array_equal(got[:5000], ref[:5000])
    assert np.isnan(got[5000:]).all() and np.isnan(ref[5000:]).all()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_float_delta_decode_unaligned(device, dt):
    n = 9001
    enc = _float_data(dt, n)
    raw = torch.zeros(enc.nbytes + 1, dtype=torch.uint8, device=device)
    raw[1:] = torch.from_numpy(enc.view(np.uint8)).to(device)
    got = Delta(dt).decode(raw[1:]).cpu().numpy()
    assert got.tobytes() == _oracle_dec(enc, dt, dt).tobytes()


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
def test_float_delta_roundtrip_1m(device, dt):
    """1 Mi elements through encode (parallel differences) and decode (chain)."""
    x = RNG.normal(1000, 5, 1 << 20).astype(dt)
    xd = torch.from_numpy(x).to(device)
    enc = Delta(dt).encode(xd)
    assert enc.cpu().numpy().tobytes() == _oracle_enc(x, dt, dt).tobytes()
    dec = Delta(dt).decode(enc).cpu().numpy()
    assert dec.tobytes() == _oracle_dec(enc.cpu().numpy(), dt, dt).tobytes()


BATCH_CASES = [
    ("<i2", "<i2"), ("<i4", "<i4"), ("|u1", "|u1"), ("<i8", "<i8"), ("<u2", "<u2"), ("|b1", "|b1"),
    ("<i8", "<i4"), ("<i4", "|i1"), ("<f4", "<f4"), ("<f8", "<f8"), ("<f2", "<f2"), ("<f8", "<f4"),
]


def _batch_input(dt, b, n):
    dt = np.dtype(dt)
    if dt.kind == "b":
        return RNG.integers(0, 2, (b, n)).astype(dt)
    if dt.kind in "iu":
        x = RNG.integers(0, 2**63, (b, n), dtype=np.uint64).astype(dt)
        x[:, 0] %= 100  # enc[0] = arr[0] must fit the narrower astype (delta.py:63)
        return x
    return RNG.normal(0, 10, (b, n)).astype(dt)


@pytest.mark.parametrize("dt,astype", BATCH_CASES)
@pytest.mark.parametrize("n", [1, 5, 4096, 10007])
def test_delta_batch_rowwise(device, dt, astype, n):
    b = 13
    x = _batch_input(dt, b, n)
    codec = Delta(dt, astype)
    enc = batch.delta_chunks(torch.from_numpy(x).to(device), codec, encode=True).cpu().numpy()
    for i in range(b):
        assert enc[i].tobytes() == _oracle_enc(x[i], dt, astype).tobytes(), (dt, astype, n, i)
    enc_t = enc.view(np.dtype(astype)) if np.dtype(astype).kind != "b" else enc.view(bool)
    dec = batch.delta_chunks(torch.from_numpy(enc).to(device), codec, encode=False).cpu().numpy()
    for i in range(b):
        assert dec[i].tobytes() == _oracle_dec(enc_t[i], dt, astype).tobytes(), (dt, astype, n, i)


@pytest.mark.parametrize("dt", ["<i2", "<f4"])
def test_delta_batch_padded_strides(device, dt):
    """Rows of a wider buffer (row stride > chunk bytes), output into a padded
    buffer too: only the chunk bytes are read and written."""
    b, n = 9, 3001
    itemsize = np.dtype(dt).itemsize
    x = _batch_input(dt, b, n)
    wide = torch.zeros((b, n * itemsize + 64), dtype=torch.uint8, device=device)
    wide[:, : n * itemsize] = torch.from_numpy(x.view(np.uint8).reshape(b, -1)).to(device)
    rows = wide[:, : n * itemsize]
    out_wide = torch.full((b, n * itemsize + 32), 0xAB, dtype=torch.uint8, device=device)
    out = out_wide[:, : n * itemsize]
    batch.delta_chunks(rows, Delta(dt), encode=True, out=out)
    got = out_wide.cpu().numpy()
    assert (got[:, n * itemsize:] == 0xAB).all()
    for i in range(b):
        assert got[i, : n * itemsize].tobytes() == _oracle_enc(x[i], dt, dt).tobytes()
    dec_wide = torch.full((b, n * itemsize + 16), 0xCD, dtype=torch.uint8, device=device)
    batch.delta_chunks(out, Delta(dt), encode=False, out=dec_wide[:, : n * itemsize])
    dec = dec_wide.cpu().numpy()
    assert (dec[:, n * itemsize:] == 0xCD).all()
    for i in range(b):  # float Delta is lossy (the reference's too): compare with its decode
        enc_i = got[i, : n * itemsize].view(dt)
        assert dec[i, : n * itemsize].tobytes() == _oracle_dec(enc_i, dt, dt).tobytes()
    if np.dtype(dt).kind in "iu":
        assert dec[:, : n * itemsize].tobytes() == x.tobytes()


def test_delta_batch_many_chunks(device):
    """8192 chunks of 1 MiB / 8 rows: grid of thousands of scans."""
    b, n = 2048, 4099
    x = _batch_input("<i4", b, n)
    xd = torch.from_numpy(x).to(device)
    enc = batch.delta_chunks(xd, Delta("<i4"), encode=True)
    dec = batch.delta_chunks(enc, Delta("<i4"), encode=False)
    assert torch.equal(dec.view(torch.int32).reshape(b, n), xd)
    e = enc.cpu().numpy().view("<i4")
    for i in (0, 1, 777, b - 1):
        assert e[i].tobytes() == _oracle_enc(x[i], "<i4", "<i4").tobytes()


@pytest.mark.parametrize("dt,astype,first", [("<i8", "<i4", 2**40), ("<i4", "|i1", 300), ("<f8", "<i2", np.nan),
                                             ("<u2", "|i1", 200), ("<i2", "|u1", -1), ("<i4", "<u2", 70000)])
def test_delta_encode_first_element_assignment(device, dt, astype, first):
    """delta.py:63 `enc[0] = arr[0]` raises where numpy's scalar assignment
    does (the differences are array casts and wrap silently)."""
    x = np.array([first, 1, 2], dtype=dt)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref = oracle.delta_encode(x, dt, astype)
    except (OverflowError, ValueError) as e:
        with pytest.raises(type(e)):
            Delta(dt, astype).encode(torch.from_numpy(x).to(device))
        with pytest.raises(type(e)):
            batch.delta_chunks(torch.from_numpy(np.stack([x[[1, 2, 0]], x])).to(device), Delta(dt, astype))
        return
    assert Delta(dt, astype).encode(torch.from_numpy(x).to(device)).cpu().numpy().tobytes() == ref.tobytes()


@pytest.mark.parametrize("dt,n", [("|i1", 8192 * 300 + 5), ("|u1", 8192 * 16384 + 8192 * 7 + 3), ("<i2", 4096 * 513),
                                  ("<u2", 4096 * 777 + 1), ("<i4", 2048 * 70000 + 9), ("<u4", 17)])
def test_two_launch_int_decode_vs_oracle(device, dt, n):
    """Same-width integer Delta decode, default path (two launches: group
    totals by one 64-bit arrival atomic per 4-tile workgroup, prefixes in the
    apply pass) against the oracle and against the three-pass scan (the ABI
    with no ticket); one group and many, ragged tails, groups of 512 tiles;
    the stream's ticket is left zero."""
    from numcodecs_amd import _native, _ops

    rng = np.random.default_rng(n)
    info = np.iinfo(np.dtype(dt))
    enc = rng.integers(info.min, info.max, n, endpoint=True, dtype=np.dtype(dt))
    src = torch.from_numpy(enc).to(device)
    d = Delta(dtype=dt)
    dec = d.decode(src)
    ref = oracle.delta_decode(enc, dt)
    assert np.array_equal(dec.cpu().numpy().view(np.dtype(dt)), ref)
    a = _ops.dtype_code(dt)
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, a)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=device)
    out = torch.empty_like(src)
    _native.check(_native.lib.mc_delta_decode(src.data_ptr(), out.data_ptr(), n, a, a, ws.data_ptr(), ws_n, None,
                                              _ops.stream(src)), "three-pass")
    assert torch.equal(out.view(torch.uint8), dec.reshape(-1).view(torch.uint8))
    torch.cuda.synchronize()
    assert not _ops._verify_slot(src, _ops.stream(src)).ticket.any()


def _special_floats(dt, n, seed):
    """normal values with NaNs of several payloads (quiet and signalling),
    infinities, signed zeros and subnormals sprinkled in."""
    rng = np.random.default_rng(seed)
    dt = np.dtype(dt)
    x = rng.normal(0, 3, n).astype(dt)
    if n < 4:
        return x
    bits = x.view(np.dtype((">" if dt.byteorder == ">" else "<") + f"u{dt.itemsize}"))
    nan_bits = [0x7FC00001, 0xFFC12345, 0x7F800001] if dt.itemsize == 4 else [
        0x7FF8000000000001, 0xFFF0000000000ABC, 0x7FF0000000000001]
    tiny = np.finfo(dt).tiny
    special = [np.inf, -np.inf, -0.0, 0.0, tiny / 8, -tiny / 3]
    for i, k in enumerate(rng.choice(n, min(n, 24), replace=False)):
        if i % 3 == 0:
            bits[k] = nan_bits[(i // 3) % 3]
        else:
            x[k] = special[i % len(special)]
    return x


@pytest.mark.parametrize("dt", ["<f4", ">f4", "<f8", ">f8"])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 63, 4096, 4097, 65536 + 3, 262144 * 3 + 7])
def test_float_delta_encode_same_type_special_values(device, dt, n):
    """Same-type float Delta encode (the 16-B vector kernel, byte swaps fused
    for big-endian): IEEE differences in dtype, numpy's bytes for NaNs,
    infinities, signed zeros and subnormals, at every tile boundary."""
    x = _special_floats(dt, n, n)

    def enc_bytes(a):  # raw device bytes in (torch holds no big-endian dtypes), bytes out
        out = Delta(dt).encode(torch.from_numpy(a.view(np.uint8).copy()).to(device))
        return out.contiguous().view(torch.uint8).cpu().numpy().tobytes()

    assert enc_bytes(x) == _oracle_enc(x, dt, dt).tobytes(), (dt, n)
    x[0] = -0.0  # the first element is stored as it is (never 0 - x)
    assert enc_bytes(x) == _oracle_enc(x, dt, dt).tobytes(), (dt, n)


@pytest.mark.parametrize("dt", ["<f2", "<f4", "<f8", ">f4"])
@pytest.mark.parametrize("n", [7, 5000, 70001])
def test_float_delta_decode_nan_payloads(device, dt, n):
    """numpy's cumsum keeps the first NaN's payload (x86: the first operand's
    NaN, quieted) and gives inf + -inf the negative default NaN: the device
    decode returns the same bytes."""
    rng = np.random.default_rng(n)
    d = np.dtype(dt)
    x = rng.normal(0, 1, n).astype(d)
    ub = np.dtype((">" if d.byteorder == ">" else "<") + f"u{d.itemsize}")
    pay = {2: [0x7E01, 0xFE35, 0x7C01], 4: [0x7FC00001, 0xFFC12345, 0x7F800001],
           8: [0x7FF8000000000001, 0xFFF0000000000ABC, 0x7FF0000000000001]}[d.itemsize]
    k = max(1, n // 3)
    x.view(ub)[k] = pay[n % 3]
    if n > 10:
        x.view(ub)[k + 1] = pay[(n + 1) % 3]  # a second NaN after the first
    dec = Delta(dt).decode(torch.from_numpy(x.view(np.uint8).copy()).to(device))
    got = dec.contiguous().view(torch.uint8).cpu().numpy().tobytes()
    assert got == _oracle_dec(x, dt, dt).tobytes()
    y = rng.normal(0, 1, n).astype(d)
    y[k] = np.inf
    y[-1] = -np.inf
    dec = Delta(dt).decode(torch.from_numpy(y.view(np.uint8).copy()).to(device))
    assert dec.contiguous().view(torch.uint8).cpu().numpy().tobytes() == _oracle_dec(y, dt, dt).tobytes()


TWO_STEP_PAIRS = [("<i4", "<f4"), ("<i2", "<f8"), ("|b1", "<f4"), ("|u1", "<f2"), ("<i8", "<f8"), (">i4", ">f4"),
                  ("<u2", "<f4"), ("|b1", "<i4"), ("|b1", "|u1"), ("|b1", ">i2"), ("|i1", "<f2")]


def _two_step_input(astype, n, seed):
    rng = np.random.default_rng(seed)
    a = np.dtype(astype)
    if a.kind == "f":
        x = (rng.standard_normal(n) * 2.5).astype(a)
        if n > 40:
            x[n // 4] = np.nan if n % 2 else np.inf
            x[n // 3] = -np.inf
        return x
    info = np.iinfo(a)
    return rng.integers(max(info.min, -3), min(info.max, 3), n, endpoint=True).astype(a)


@pytest.mark.parametrize("dt,astype", TWO_STEP_PAIRS)
@pytest.mark.parametrize("n", [1, 5, 4097, 70001])
def test_delta_decode_through_loop_dtype(device, dt, astype, n):
    """The pairs decoded through their loop dtype (np.promote_types(astype,
    dtype)) and a cast -- a float running sum into integers or bools, an
    integer running sum into bools -- byte-identical to np.cumsum(enc,
    out=dec) (delta.py:80), single chunk and batched rows."""
    enc = _two_step_input(astype, n, n)
    ref = _oracle_dec(enc, dt, astype)
    codec = Delta(dt, astype)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        got = codec.decode(torch.from_numpy(enc.view(np.uint8).copy()).to(device))
    assert got.contiguous().view(torch.uint8).cpu().numpy().tobytes() == ref.tobytes(), (dt, astype, n)
    if n < 70001:
        b = 5
        rows = np.stack([_two_step_input(astype, n, n + k) for k in range(b)])
        dec = batch.delta_chunks(torch.from_numpy(rows.view(np.uint8).reshape(b, -1).copy()).to(device), codec,
                                 encode=False).cpu().numpy()
        for k in range(b):
            assert dec[k].tobytes() == _oracle_dec(rows[k], dt, astype).tobytes(), (dt, astype, n, k)
