"""GPU parity tests: every codec call goes through libmcodec.so's C ABI into
the gfx950 kernels.  Checked against the golden vectors produced by the real
reference (tests/golden/make_golden.py), the reference's backward-compat
fixtures (tests/golden/reference_fixture, byte-exact both ways), its
known-answer tests and the oracle.

Tolerance: none.  Shuffle, Delta and Fletcher32 are integer/byte work and
must be bit-exact; BitRound is integer arithmetic on the bit pattern and is
bit-exact too; FixedScaleOffset and Quantize reproduce numpy's rounding (NEP
50 dtypes, no FMA contraction, correctly rounded division, numpy's
float->half conversion, x86-64 float->int casts) and are also required to
match the reference bit for bit on every vector here -- including NaN, inf,
subnormal and out-of-range inputs.  (The reference's own tests only require
`decimal=digits` agreement for these lossy codecs.)
"""

import itertools
from multiprocessing.pool import ThreadPool

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import BitRound, Delta, FixedScaleOffset, Fletcher32, Quantize, Shuffle, get_codec
from numcodecs_amd import batch
from numcodecs_amd.compat import ensure_bytes
from tests.helpers import (
    check_encode_decode,
    compare_arrays,
    fixture_cases,
    load_vectors,
    vec,
)

pytestmark = pytest.mark.gpu

MANIFEST, DATA = load_vectors()
RNG = np.random.default_rng(42)


def _no_warn():
    return np.errstate(all="ignore")


# ---------------------------------------------------------------------------
# Shuffle (test_shuffle.py)
# ---------------------------------------------------------------------------
SHUFFLE_CODECS = [Shuffle(), Shuffle(elementsize=0), Shuffle(elementsize=4), Shuffle(elementsize=8)]
SHUFFLE_ARRAYS = [
    np.arange(1000, dtype="i4"),
    np.linspace(1000, 1001, 1000, dtype="f8"),
    RNG.normal(loc=1000, scale=1, size=(100, 10)),
    RNG.integers(0, 2, size=1000, dtype=bool).reshape(100, 10, order="F"),
    RNG.choice([b"a", b"bb", b"ccc"], size=1000).reshape(10, 10, 10),
    RNG.integers(0, 2**60, size=1000, dtype="u8").view("M8[ns]"),
    RNG.integers(0, 2**60, size=1000, dtype="u8").view("m8[ns]"),
    RNG.integers(0, 2**25, size=1000, dtype="u8").view("M8[m]"),
    RNG.integers(-(2**63), -(2**63) + 20, size=1000, dtype="i8").view("m8[m]"),
]


@pytest.mark.parametrize("arr", SHUFFLE_ARRAYS)
@pytest.mark.parametrize("codec", SHUFFLE_CODECS)
def test_shuffle_encode_decode(device, arr, codec):
    check_encode_decode(arr, codec)


def test_shuffle_backwards_compatibility(device):
    n = 0
    for arr, _j, config, enc in fixture_cases("shuffle"):
        codec = get_codec(config)
        assert codec.encode(arr).tobytes() == enc
        dec = codec.decode(enc)
        assert ensure_bytes(dec) == arr.tobytes(order="A")
        n += 1
    assert n == 52


def test_shuffle_expected_result(device):
    arr = np.array([0x0001020304050607, 0x08090A0B0C0D0E0F, 0x1011121314151617,
                    0x18191A1B1C1D1E1F], dtype=">u8")
    expected = np.array([0x00081018, 0x01091119, 0x020A121A, 0x030B131B, 0x040C141C,
                         0x050D151D, 0x060E161E, 0x070F171F], dtype="u4")
    enc = Shuffle(elementsize=arr.data.itemsize).encode(arr)
    np.testing.assert_array_equal(np.frombuffer(enc.data, ">u4"), expected)


def test_shuffle_incompatible_elementsize(device):
    with pytest.raises(ValueError):
        Shuffle(elementsize=4).encode(np.arange(1001, dtype="u1"))
    with pytest.raises(ValueError):
        Shuffle(elementsize=4).encode(torch.arange(1001, dtype=torch.uint8, device=device))


def test_shuffle_threadpool(device):
    data = np.arange(1000000)
    enc = Shuffle().encode(data)
    with ThreadPool(5) as pool:
        encs = pool.map(lambda d: Shuffle().encode(d), [data] * 5)
        decs = pool.map(lambda e: Shuffle().decode(e), [enc] * 5)
    assert all(np.array_equal(e, enc) for e in encs)
    assert all(d.nbytes == data.nbytes for d in decs)


def test_shuffle_vectors(device):
    for i, m in enumerate(MANIFEST["shuffle"]):
        x = vec(DATA, "shuffle", i, "input")
        enc = vec(DATA, "shuffle", i, "encoded")
        codec = Shuffle(m["elementsize"])
        assert np.array_equal(codec.encode(x), enc), m
        assert np.array_equal(codec.decode(enc), x), m
        # device tensors in, device tensors out
        xd = torch.from_numpy(x.copy()).to(device)
        ed = codec.encode(xd)
        assert ed.is_cuda and ed.dtype == torch.uint8
        assert np.array_equal(ed.cpu().numpy(), enc), m
        assert torch.equal(codec.decode(ed), xd), m


def test_shuffle_unaligned_device_views(device):
    """Views at odd byte offsets take the generic kernel and stay exact."""
    base = torch.randint(0, 256, (4 * 50000 + 16,), dtype=torch.uint8, device=device)
    for off in (1, 3, 4, 8):
        x = base[off: off + 4 * 50000]
        ref = oracle.shuffle(x.cpu().numpy(), 4)
        assert np.array_equal(Shuffle(4).encode(x).cpu().numpy(), ref)


def test_shuffle_out_argument(device):
    x = np.arange(4096, dtype="<f4")
    out = np.empty(x.nbytes, dtype="u1")
    res = Shuffle(4).encode(x, out=out)
    assert np.shares_memory(res, out)
    assert np.array_equal(out, oracle.shuffle(x, 4))
    xd = torch.from_numpy(x).to(device)
    outd = torch.empty(x.nbytes, dtype=torch.uint8, device=device)
    Shuffle(4).encode(xd, out=outd)
    assert np.array_equal(outd.cpu().numpy(), oracle.shuffle(x, 4))


@pytest.mark.parametrize("es", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("tdt", [torch.uint8, torch.int16, torch.float32, torch.float64, torch.bool])
def test_shuffle_device_short_path(device, es, tdt):
    """The device-tensor short path (Shuffle._run_device) against the oracle,
    and its results, errors and return objects against the general path
    (host staging of the same bytes)."""
    nbytes = 48 * 4096 + 48
    raw = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=device)
    x = raw.view(tdt) if tdt is not torch.bool else (raw & 1).bool()
    host = x.cpu().numpy()
    codec = Shuffle(es)
    assert codec._run_device(x, None, True) is not None  # the short path is the one exercised
    enc = codec.encode(x)
    assert enc.is_cuda and enc.dtype == torch.uint8 and enc.shape == (nbytes,)
    assert np.array_equal(enc.cpu().numpy(), oracle.shuffle(host.view("u1"), es))
    assert np.array_equal(enc.cpu().numpy(), codec.encode(host))
    dec = codec.decode(enc)
    assert torch.equal(dec, raw if tdt is not torch.bool else x.view(torch.uint8))
    # out= of another dtype and shape: returns the flat view of out
    out = torch.empty((nbytes // 4, 4), dtype=torch.uint8, device=device).view(torch.int32)
    res = codec.encode(x, out=out)
    assert res.data_ptr() == out.data_ptr() and res.shape == (out.numel(),) and res.dtype == torch.int32
    assert torch.equal(res.view(torch.uint8), enc)
    big = torch.zeros(nbytes + 64, dtype=torch.uint8, device=device)
    codec.decode(enc, out=big)
    assert torch.equal(big[:nbytes], dec.view(torch.uint8)) and not big[nbytes:].any()
    with pytest.raises(ValueError, match="too small"):
        codec.encode(x, out=torch.empty(nbytes - 1, dtype=torch.uint8, device=device))
    with pytest.raises(ValueError, match="integer multiple"):
        Shuffle(es).encode(raw[: es * 1000 + 1])


def test_shuffle_device_general_path_cases(device):
    """Inputs the short path hands to the general one (F order, an empty
    tensor, elementsize <= 1, a non-contiguous out) keep the reference's
    results and errors."""
    x = torch.randn(64, 48, device=device)
    xf = x.t()  # F-contiguous view
    assert Shuffle(4)._run_device(xf, None, True) is None
    assert np.array_equal(Shuffle(4).encode(xf).cpu().numpy(),
                          oracle.shuffle(np.asfortranarray(xf.cpu().numpy()).reshape(-1, order="A"), 4))
    assert Shuffle(4).encode(torch.empty(0, device=device)).numel() == 0
    assert torch.equal(Shuffle(1).encode(x), x.view(-1).view(torch.uint8))
    with pytest.raises(ValueError):
        Shuffle(4).encode(x, out=torch.empty(2 * x.nbytes, dtype=torch.uint8, device=device)[::2])


# ---------------------------------------------------------------------------
# BitRound (test_bitround.py) -- bit-exact
# ---------------------------------------------------------------------------
def _round(data, keepbits):
    codec = BitRound(keepbits=keepbits)
    return codec.decode(codec.encode(data.copy()))


@pytest.mark.parametrize("dtype", ["float32", "float64", "float16"])
def test_bitround_fixed_points(device, dtype):
    for fill in (0.0, 1.0, -1.0):
        a = np.full((3, 2), fill, dtype=dtype)
        for k in range({"float16": 10, "float32": 23, "float64": 52}[dtype]):
            np.testing.assert_equal(a, _round(a, k))


@pytest.mark.parametrize("dtype", ["float32", "float64"])
def test_bitround_no_rounding_approx_idempotence(device, dtype):
    a = RNG.random((300, 200)).astype(dtype)
    np.testing.assert_equal(a, _round(a, {"float32": 23, "float64": 52}[dtype]))
    ar = _round(a, {"float32": 11, "float64": 18}[dtype])
    np.testing.assert_allclose(a, ar, rtol=np.sqrt(np.finfo(np.float32).eps))
    for k in range(20):
        np.testing.assert_equal(_round(a, k), _round(a, k))


def test_bitround_vectors(device):
    for i, m in enumerate(MANIFEST["bitround"]):
        x = vec(DATA, "bitround", i, "input").view(m["dtype"])
        enc = BitRound(m["keepbits"]).encode(x)
        assert enc.dtype == np.dtype(m["dtype"].replace("f", "i"))
        assert enc.tobytes() == vec(DATA, "bitround", i, "encoded").tobytes(), m
        xd = torch.from_numpy(x.copy()).to(device)
        ed = BitRound(m["keepbits"]).encode(xd)
        assert ed.is_cuda and ed.shape == xd.shape
        assert ed.cpu().numpy().tobytes() == vec(DATA, "bitround", i, "encoded").tobytes(), m
        dd = BitRound(m["keepbits"]).decode(ed)
        assert dd.dtype == xd.dtype


def test_bitround_f_order_and_shape(device):
    a = np.asfortranarray(RNG.random((64, 33)).astype("f4"))
    enc = BitRound(7).encode(a)
    ref = oracle.bitround_encode(a, 7)
    assert enc.shape == ref.shape and enc.flags.c_contiguous == ref.flags.c_contiguous
    assert np.array_equal(enc, ref)


# ---------------------------------------------------------------------------
# Delta (test_delta.py) -- bit-exact
# ---------------------------------------------------------------------------
DELTA_ARRAYS = [
    RNG.integers(0, 1, size=110, dtype="?").reshape(10, 11),
    np.arange(1000, dtype="<i4"),
    np.linspace(1000, 1001, 1000, dtype="<f4").reshape(100, 10),
    RNG.normal(loc=1000, scale=1, size=(10, 10, 10)).astype("<f8"),
    RNG.integers(0, 200, size=1000, dtype="u2").astype("<u2").reshape(100, 10, order="F"),
]


@pytest.mark.parametrize("arr", DELTA_ARRAYS)
def test_delta_encode_decode(device, arr):
    check_encode_decode(arr, Delta(dtype=arr.dtype))


def test_delta_encode_kat(device):
    codec = Delta(dtype="i8", astype="i4")
    actual = codec.encode(np.arange(10, 20, 1, dtype="i8"))
    np.testing.assert_array_equal(np.array([10] + [1] * 9, dtype="i4"), actual)
    assert actual.dtype == np.dtype("i4")


@pytest.mark.parametrize("prefix", ["bool", "int32", "float32", "float64", "uint16"])
def test_delta_backwards_compatibility(device, prefix):
    for arr, _j, config, enc in fixture_cases("delta", prefix):
        codec = get_codec(config)
        assert codec.encode(arr).tobytes() == enc
        assert ensure_bytes(codec.decode(enc)) == arr.tobytes(order="A")


def test_delta_vectors(device):
    for i, m in enumerate(MANIFEST["delta"]):
        x = vec(DATA, "delta", i, "input").view(m["dtype"])
        codec = Delta(m["dtype"], m["astype"])
        enc = codec.encode(x)
        assert enc.tobytes() == vec(DATA, "delta", i, "encoded").tobytes(), m
        dec = codec.decode(vec(DATA, "delta", i, "encoded"))
        assert dec.tobytes() == vec(DATA, "delta", i, "decoded").tobytes(), m


def test_delta_empty_raises(device):
    with pytest.raises(IndexError):
        Delta("<i4").encode(np.zeros(0, "<i4"))


def test_delta_int_scan_many_tiles(device):
    """Wrap-around scan across many 4096-element tiles, all int widths."""
    for dt in ("<i2", "|u1", "<i4", "<u8", "<i8", "|i1", "<u2"):
        x = RNG.integers(0, 2**63, size=300001, dtype=np.uint64).view("<i8").astype(dt)
        codec = Delta(dt)
        with _no_warn():
            enc = oracle.delta_encode(x, dt)
            ref = oracle.delta_decode(enc, dt)
        assert np.array_equal(codec.encode(x), enc), dt
        assert np.array_equal(codec.decode(enc), ref), dt


# ---------------------------------------------------------------------------
# Quantize (test_quantize.py) -- bit-exact against the reference
# ---------------------------------------------------------------------------
Q_ARRAYS = [
    np.linspace(100, 200, 1000, dtype="<f8"),
    RNG.normal(loc=0, scale=1, size=1000).astype("<f8"),
    np.linspace(100, 200, 1000, dtype="<f8").reshape(100, 10),
    np.linspace(100, 200, 1000, dtype="<f8").reshape(100, 10, order="F"),
    np.linspace(100, 200, 1000, dtype="<f8").reshape(10, 10, 10),
]
Q_CODECS = [
    Quantize(digits=-1, dtype="<f8", astype="<f2"),
    Quantize(digits=0, dtype="<f8", astype="<f2"),
    Quantize(digits=1, dtype="<f8", astype="<f2"),
    Quantize(digits=5, dtype="<f8", astype="<f4"),
    Quantize(digits=12, dtype="<f8", astype="<f8"),
]


@pytest.mark.parametrize("arr,codec", list(itertools.product(Q_ARRAYS, Q_CODECS)))
def test_quantize_encode_decode(device, arr, codec):
    check_encode_decode(arr, codec, precision=codec.digits)
    enc = codec.encode(arr)
    with _no_warn():
        ref = oracle.quantize_encode(arr, codec.digits, codec.dtype, codec.astype)
    assert enc.shape == ref.shape and enc.dtype == ref.dtype
    assert enc.tobytes(order="A") == ref.tobytes(order="A")
    np.testing.assert_array_equal(enc, codec.decode(enc))


def test_quantize_backwards_compatibility(device):
    n = 0
    for arr, j, config, enc in fixture_cases("quantize"):
        codec = get_codec(config)
        assert codec.encode(arr).tobytes(order="A") == enc
        dec = codec.decode(enc)
        compare_arrays(arr, dec, precision=codec.digits)
        n += 1
    assert n == 25


def test_quantize_vectors(device):
    for i, m in enumerate(MANIFEST["quantize"]):
        x = vec(DATA, "quantize", i, "input").view(m["dtype"])
        codec = Quantize(m["digits"], m["dtype"], m["astype"])
        assert codec.encode(x).tobytes() == vec(DATA, "quantize", i, "encoded").tobytes(), m
        dec = codec.decode(vec(DATA, "quantize", i, "encoded"))
        assert dec.tobytes() == vec(DATA, "quantize", i, "decoded").tobytes(), m


# ---------------------------------------------------------------------------
# FixedScaleOffset (test_fixedscaleoffset.py) -- bit-exact
# ---------------------------------------------------------------------------
FSO_ARRAYS = [
    np.linspace(1000, 1001, 1000, dtype="<f8"),
    RNG.normal(loc=1000, scale=1, size=1000).astype("<f8"),
    np.linspace(1000, 1001, 1000, dtype="<f8").reshape(100, 10),
    np.linspace(1000, 1001, 1000, dtype="<f8").reshape(100, 10, order="F"),
    np.linspace(1000, 1001, 1000, dtype="<f8").reshape(10, 10, 10),
]
FSO_CODECS = [
    FixedScaleOffset(offset=1000, scale=10, dtype="<f8", astype="<i1"),
    FixedScaleOffset(offset=1000, scale=10**2, dtype="<f8", astype="<i2"),
    FixedScaleOffset(offset=1000, scale=10**6, dtype="<f8", astype="<i4"),
    FixedScaleOffset(offset=1000, scale=10**12, dtype="<f8", astype="<i8"),
    FixedScaleOffset(offset=1000, scale=10**12, dtype="<f8"),
]


@pytest.mark.parametrize("arr,codec", list(itertools.product(FSO_ARRAYS, FSO_CODECS)))
def test_fso_encode_decode(device, arr, codec):
    check_encode_decode(arr, codec, precision=int(np.log10(codec.scale)))


@pytest.mark.parametrize("offset,scale,expected", [
    (1000, 10, [0, 6, 11, 17, 22, 28, 33, 39, 44, 50]),
    (1002.5, 10, [-25, -19, -14, -8, -3, 3, 8, 14, 19, 25]),
    (1000, 0.5, [0, 0, 1, 1, 1, 1, 2, 2, 2, 2]),
])
def test_fso_encode_kat(device, offset, scale, expected):
    codec = FixedScaleOffset(scale=scale, offset=offset, dtype="<f8", astype=np.int16)
    actual = codec.encode(np.linspace(1000, 1005, 10, dtype="<f8"))
    np.testing.assert_array_equal(np.array(expected, dtype=np.int16), actual)
    assert actual.dtype == np.int16


def test_fso_backwards_compatibility(device):
    n = 0
    for arr, _j, config, enc in fixture_cases("fixedscaleoffset"):
        codec = get_codec(config)
        assert codec.encode(arr).tobytes() == enc
        compare_arrays(arr, codec.decode(enc), precision=int(np.log10(codec.scale)))
        n += 1
    assert n == 25


def test_fso_vectors(device):
    for i, m in enumerate(MANIFEST["fso"]):
        x = vec(DATA, "fso", i, "input").view(m["dtype"])
        codec = FixedScaleOffset(m["offset"], m["scale"], m["dtype"], m["astype"])
        assert codec.encode(x).tobytes() == vec(DATA, "fso", i, "encoded").tobytes(), m
        dec = codec.decode(vec(DATA, "fso", i, "encoded"))
        assert dec.tobytes() == vec(DATA, "fso", i, "decoded").tobytes(), m


# ---------------------------------------------------------------------------
# Fletcher32 (test_fletcher32.py) -- bit-exact
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", ["uint8", "int32", "float32"])
def test_fletcher32_with_data(device, dtype):
    data = np.arange(100, dtype=dtype)
    f = Fletcher32()
    arr = np.frombuffer(f.decode(f.encode(data)), dtype=dtype)
    assert (arr == data).all()


def test_fletcher32_error(device):
    enc2 = bytearray(Fletcher32().encode(np.arange(100)))
    enc2[0] += 1
    with pytest.raises(RuntimeError) as e:
        Fletcher32().decode(enc2)
    assert "fletcher32 checksum" in str(e.value)


def test_fletcher32_known(device):
    from tests.test_oracle import KAT_FLETCHER

    out = np.frombuffer(Fletcher32().decode(KAT_FLETCHER), dtype="<i8")
    assert out.tolist() == [1911, -2427, 1897, -2412, 2440, 873, -621, -829, 551, -2118]


def test_fletcher32_out(device):
    data = np.frombuffer(bytearray(b"Hello World"), dtype="uint8")
    f = Fletcher32()
    result = f.encode(data)
    assert f.decode(result, out=data) is data


def test_fletcher32_host_decode_returns_memoryview(device):
    """Host input, no `out`: the reference returns a memoryview slice of the
    input without the footer (`b_mv[:-FOOTER_LENGTH]`, fletcher32.pyx:113-114),
    not a copy -- a memoryview over the caller's own bytes."""
    data = np.arange(100, dtype="<i4")
    enc = bytearray(Fletcher32().encode(data))
    dec = Fletcher32().decode(enc)
    assert type(dec) is memoryview and dec.nbytes == data.nbytes and dec.format == "B"
    assert bytes(dec) == data.tobytes()
    enc[1] = 0x5A  # a write into the input shows through the returned view

    assert dec[1] == 0x5A


def test_fletcher32_device_out_sizes(device):
    """Device `out`: exact and larger buffers receive the payload; an
    undersized one raises ValueError instead of writing out of bounds (the
    reference memcpys unchecked, fletcher32.pyx:107-111)."""
    x = torch.randint(0, 256, (4099,), dtype=torch.uint8, device=device)
    enc = Fletcher32().encode(x)
    exact = torch.empty(4099, dtype=torch.uint8, device=device)
    assert Fletcher32().decode(enc, out=exact) is exact and torch.equal(exact, x)
    big = torch.zeros(5000, dtype=torch.uint8, device=device)
    Fletcher32().decode(enc, out=big)
    assert torch.equal(big[:4099], x) and not big[4099:].any()
    small = torch.zeros(4098, dtype=torch.uint8, device=device)
    with pytest.raises(ValueError):
        Fletcher32().decode(enc, out=small)
    assert not small.any()


def test_fletcher32_vectors(device):
    for i, m in enumerate(MANIFEST["fletcher32"]):
        x = vec(DATA, "fletcher32", i, "input")
        enc = Fletcher32().encode(x)
        assert isinstance(enc, bytes) and enc[:-4] == x.tobytes()
        assert int.from_bytes(enc[-4:], "little") == m["checksum"], m
        xd = torch.from_numpy(x.copy()).to(device)
        ed = Fletcher32().encode(xd)
        assert int.from_bytes(ed[-4:].cpu().numpy().tobytes(), "little") == m["checksum"], m
        assert torch.equal(Fletcher32().decode(ed), xd)


def test_fletcher32_edges(device):
    with pytest.raises(IndexError):
        Fletcher32().encode(b"")
    for n in (0, 3, 4):
        with pytest.raises(IndexError):
            Fletcher32().decode(b"\x00" * n)
    assert Fletcher32().decode(Fletcher32().encode(b"\x07")).tobytes() == b"\x07"


# ---------------------------------------------------------------------------
# batched chunks and fused pipelines
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("es", [2, 4, 8])
def test_batch_shuffle_fletcher32_fused(device, es):
    nchunks, chunk = 37, 4096 * es * 3
    x = torch.randint(0, 256, (nchunks, chunk), dtype=torch.uint8, device=device)
    enc = batch.shuffle_fletcher32_encode_chunks(x, es)
    xh = x.cpu().numpy()
    eh = enc.cpu().numpy()
    for c in range(nchunks):
        ref = oracle.fletcher32_encode(oracle.shuffle(xh[c], es))
        assert eh[c, : chunk + 4].tobytes() == ref, c
    dec, status = batch.fletcher32_unshuffle_decode_chunks(enc, chunk, es)
    assert torch.equal(dec, x)
    st = status.cpu().numpy().view(np.uint32)
    assert (st[:, 0] == st[:, 1]).all()
    # corrupt one byte of chunk 5: its checksum no longer matches
    enc[5, 100] ^= 0x40
    with pytest.raises(RuntimeError, match="fletcher32 checksum"):
        batch.fletcher32_unshuffle_decode_chunks(enc, chunk, es)


def test_batch_fallback_unaligned_chunk(device):
    """Chunk sizes that are not whole tiles use the two-pass path."""
    nchunks, chunk = 9, 4 * 1001
    x = torch.randint(0, 256, (nchunks, chunk), dtype=torch.uint8, device=device)
    enc = batch.shuffle_fletcher32_encode_chunks(x, 4)
    eh = enc.cpu().numpy()
    for c in range(nchunks):
        assert eh[c, : chunk + 4].tobytes() == oracle.fletcher32_encode(oracle.shuffle(x[c].cpu().numpy(), 4))
    dec, _ = batch.fletcher32_unshuffle_decode_chunks(enc, chunk, 4)
    assert torch.equal(dec, x)


def test_batch_shuffle_and_checksums(device):
    x = torch.randint(0, 256, (16, 65536), dtype=torch.uint8, device=device)
    s = batch.shuffle_chunks(x, 4)
    xh = x.cpu().numpy()
    for c in range(16):
        assert np.array_equal(s[c].cpu().numpy(), oracle.shuffle(xh[c], 4))
    assert torch.equal(batch.unshuffle_chunks(s, 4), x)
    sums = batch.fletcher32_chunks(x).cpu().numpy()
    assert [int(v) for v in sums] == [oracle.fletcher32(xh[c]) for c in range(16)]


def test_fletcher32_decode_batches(device):
    """mc_fletcher32_encode_batch / mc_fletcher32_decode_batch: payloads compacted out of rows of every
    alignment (stride payload + 4), computed vs stored footers, a corrupted
    row (fletcher32.pyx:91-115 per row)."""
    for b, n in ((1, 4096), (37, 1000), (16, 65536 + 12), (9, (1 << 20) + 6), (300, 4096 * 3 + 1), (5, 1)):
        for pad in (0, 3, 16):
            rows = torch.randint(0, 256, (b, n + pad), dtype=torch.uint8, device=device)[:, :n]
            host = rows.cpu().numpy()
            wide = torch.zeros((b, n + 4 + pad), dtype=torch.uint8, device=device)
            batch.fletcher32_encode_chunks(rows, out=wide)  # mc_fletcher32_encode_batch into padded rows
            enc = wide[:, : n + 4].cpu().numpy()
            for i in range(b):
                assert enc[i].tobytes() == oracle.fletcher32_encode(host[i]), (b, n, pad, i)
            bad = min(b - 1, 2)
            wide[bad, n // 2] ^= 0x20
            payload, sums, stored = batch.fletcher32_decode_chunks(wide[:, : n + 4])
            exp = host.copy()
            exp[bad, n // 2] ^= 0x20
            assert payload.is_contiguous() and np.array_equal(payload.cpu().numpy(), exp), (b, n, pad)
            assert sums.cpu().numpy().view("<u4").tolist() == [oracle.fletcher32(exp[i]) for i in range(b)]
            assert stored.cpu().numpy().view("<u4").tolist() == [oracle.fletcher32(host[i]) for i in range(b)]
            mism = (sums != stored).cpu().numpy()
            assert mism[bad] and not mism[[i for i in range(b) if i != bad]].any(), (b, n, pad)


def test_pipeline_fusion_matches_sequential(device):
    x = torch.from_numpy(RNG.standard_normal(4096 * 40).astype("f4")).to(device)
    pipe = batch.FilterPipeline([BitRound(10), Shuffle(4), Fletcher32()])
    enc = pipe.encode(x)
    xh = x.cpu().numpy()
    ref = oracle.fletcher32_encode(oracle.shuffle(oracle.bitround_encode(xh, 10), 4))
    assert enc.cpu().numpy().tobytes() == ref
    dec = pipe.decode(enc)
    assert np.array_equal(dec.cpu().numpy().view("f4") if dec.dtype == torch.uint8 else dec.cpu().numpy(),
                          oracle.bitround_encode(xh, 10).view("f4"))


def test_host_pipeline_roundtrip(device):
    """Host-resident chunks: pinned H2D -> kernel -> D2H over 3 streams."""
    b, n = 37, 4096 * 4 * 2
    hin = torch.randint(0, 256, (b, n), dtype=torch.uint8).pin_memory()
    henc = torch.empty_like(hin).pin_memory()
    hdec = torch.empty_like(hin).pin_memory()
    batch.host_pipeline(hin, henc, 4, True, slice_chunks=5)
    xh, eh = hin.numpy(), henc.numpy()
    for c in range(b):  # every row vs the oracle
        assert np.array_equal(eh[c], oracle.shuffle(xh[c], 4)), c
    batch.host_pipeline(henc, hdec, 4, False, slice_chunks=7)
    dh = hdec.numpy()
    for c in range(b):
        assert np.array_equal(dh[c], oracle.unshuffle(eh[c], 4)), c


@pytest.mark.parametrize("codec_id", ["fletcher32", "crc32", "crc32c", "adler32"])
def test_single_chunk_verify_one_launch(device, codec_id):
    """Decode of one device chunk verifies in ONE launch (the checksum's last
    block folds the partials, fletcher32.pyx:91-115 / checksum32.py:72-88)
    and reads its verdict from pinned host memory: sizes around the slice /
    tile boundaries, repeated calls on the stream's ticket (left zero), a
    second stream, and a corrupted byte raising the reference's error."""
    from numcodecs_amd import CRC32, CRC32C, Adler32, _ops

    make = {"fletcher32": Fletcher32, "crc32": CRC32, "crc32c": CRC32C, "adler32": Adler32}[codec_id]
    for n in (1, 15, 16, 4096 * 8 - 3, 32768, 32769, 65536 * 3 + 7, (1 << 22) + 5):
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=device)
        enc = make().encode(x)
        for _ in range(3):
            assert torch.equal(make().decode(enc), x), (codec_id, n)
        ref = oracle.fletcher32_encode(x.cpu().numpy()) if codec_id == "fletcher32" else \
            oracle.checksum32_encode(codec_id, x.cpu().numpy()).tobytes()
        assert enc.cpu().numpy().tobytes() == ref, (codec_id, n)
        bad = enc.clone()
        bad[n // 2 + (4 if codec_id != "fletcher32" and codec_id != "crc32c" else 0)] ^= 0x10
        with pytest.raises(RuntimeError):
            make().decode(bad)
    side = torch.cuda.Stream(device)
    with torch.cuda.stream(side):
        y = torch.randint(0, 256, (100003,), dtype=torch.uint8, device=device)
        assert torch.equal(make().decode(make().encode(y)), y)
    torch.cuda.synchronize()
    for sl in _ops._TLS.slots.values():  # this thread's slots (default + side stream)
        assert not sl.ticket.any()


class _DLPackDeviceArray:
    """A non-torch device array as another library would hand it over: only
    the DLPack producer protocol (ndarray_like.py:39-60 / compat.py:32-33 of
    the reference accept any ndarray-like object as it is)."""

    def __init__(self, t):
        self._t = t

    def __dlpack__(self, stream=None):
        return self._t.__dlpack__()

    def __dlpack_device__(self):
        return self._t.__dlpack_device__()


class _CAIDeviceArray:
    """The same through ``__cuda_array_interface__`` (CuPy-style)."""

    def __init__(self, t):
        self._t = t
        self.__cuda_array_interface__ = t.__cuda_array_interface__


def test_foreign_device_arrays_are_used_in_place(device):
    """Device arrays of other libraries (DLPack / __cuda_array_interface__)
    encode on the device, without a host round trip, to the oracle's bytes."""
    from numcodecs_amd import Delta
    from numcodecs_amd.compat import ensure_ndarray_like

    x = torch.randn(4096 * 3, device=device)
    xh = x.cpu().numpy()
    for wrap in (_DLPackDeviceArray, _CAIDeviceArray):
        obj = wrap(x)
        view = ensure_ndarray_like(obj)
        assert isinstance(view, torch.Tensor) and view.data_ptr() == x.data_ptr()
        enc = Shuffle(4).encode(obj)
        assert isinstance(enc, torch.Tensor) and enc.is_cuda
        assert np.array_equal(enc.cpu().numpy(), oracle.shuffle(xh, 4))
        d = Delta(dtype="<f4")
        assert np.array_equal(d.encode(obj).cpu().numpy().view("<f4"), oracle.delta_encode(xh, "<f4"))


def test_foreign_device_arrays_as_out(device):
    """decode(out=<another library's device array>) writes the result into
    that array's own memory and returns it (a foreign `out` used
    to fall into the host branch of ndarray_copy)."""
    from numcodecs_amd import Delta, FixedScaleOffset

    x = torch.randn(4096 * 3 + 5, device=device)
    xh = x.cpu().numpy()
    for wrap in (_DLPackDeviceArray, _CAIDeviceArray):
        for codec in (Shuffle(4), Delta(dtype="<f4"), FixedScaleOffset(0, 10, "<f4", "<f4")):
            enc = codec.encode(x)
            target = torch.full_like(x, -1.0)
            obj = wrap(target)
            r = codec.decode(enc, out=obj)
            assert r is obj or (isinstance(r, torch.Tensor) and r.data_ptr() == target.data_ptr())
            expect = codec.decode(enc)
            assert torch.equal(target, expect.view(torch.float32).reshape(-1))
            if isinstance(codec, Shuffle):
                assert np.array_equal(target.cpu().numpy(), xh)


def test_checksum_decode_threadpool_same_stream(device):
    """Verified decodes from several threads on the same (default) stream:
    each thread has its own verdict record, so every call reads its own
    verdict (a shared record would be overwritten by the next thread's
    kernel before the first thread read it)."""
    from numcodecs_amd import CRC32, Adler32

    rng = np.random.default_rng(3)
    bufs = [torch.from_numpy(rng.integers(0, 256, 1 << 20, dtype=np.uint8)).to(device) for _ in range(8)]
    for make in (Fletcher32, CRC32, Adler32):
        encs = [make().encode(b) for b in bufs]
        bad = encs[5].clone()
        bad[100] ^= 1

        def work(i):
            if i % 8 == 5:
                try:
                    make().decode(bad)
                except RuntimeError:
                    return "raised"
                return "missed"
            return bool(torch.equal(make().decode(encs[i % 8]), bufs[i % 8]))

        with ThreadPool(6) as pool:
            res = pool.map(work, range(48))
        assert all(r is True for i, r in enumerate(res) if i % 8 != 5), make
        assert all(r == "raised" for i, r in enumerate(res) if i % 8 == 5), make


@pytest.mark.parametrize("codec,dt_in", [
    (Delta(dtype="<i4", astype="<i2"), "<i4"), (Delta(dtype="<f4"), "<f4"),
    (FixedScaleOffset(offset=1000, scale=10, dtype="<f8", astype="<i4"), "<f8"),
    (Quantize(digits=3, dtype="<f8", astype="<f4"), "<f8"),
])
@pytest.mark.parametrize("layout", ["C", "F", "misaligned", "overlap", "host"])
def test_decode_into_device_out(device, codec, dt_in, layout):
    """decode(buf, out=<device tensor>) writes the kernel's result straight
    into `out` when it can (compat.device_out_bytes) and returns `out`; the
    bytes equal decode() followed by ndarray_copy, also for an F-order `out`,
    a misaligned one, one that overlaps the input, and a host input."""
    from numcodecs_amd import compat

    x = (np.arange(6000) % 97 * 1.5).astype(dt_in)
    enc = codec.encode(torch.from_numpy(x).to(device))
    ref = codec.decode(enc).contiguous().view(torch.uint8).reshape(-1)
    nb = ref.numel()
    tdt = compat.torch_dtype(codec.dtype)
    if layout == "C":
        out = torch.empty((60, 100), dtype=tdt, device=device)
    elif layout == "F":
        out = torch.empty((100, 60), dtype=tdt, device=device).t()
    elif layout == "misaligned":
        out = torch.empty(nb + 8, dtype=torch.uint8, device=device)[8:].view(tdt)
    elif layout == "overlap":  # out is the encoded buffer itself when the widths agree
        if enc.element_size() * enc.numel() != nb:
            pytest.skip("widths differ")
        out = enc.view(tdt)
    else:
        out = torch.empty(nb // np.dtype(codec.dtype).itemsize, dtype=tdt, device=device)
        enc = enc.cpu().numpy()
    res = codec.decode(enc, out=out)
    assert res is out
    if layout == "F":
        got = out.t().contiguous().view(torch.uint8).reshape(-1)
    else:
        got = out.contiguous().view(torch.uint8).reshape(-1)
    assert torch.equal(got, ref), (codec, layout)
