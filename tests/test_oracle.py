"""Pin the oracle (CPU) against the reference's own fixtures, its known-answer
tests and the golden vectors generated from the real reference; where the
reference itself is importable (this container), also against it directly.
"""

import json
import os

import numpy as np
import pytest

import oracle
from oracle import nporacle
from tests.helpers import FIXTURE, fixture_cases, load_vectors, vec

MANIFEST, DATA = load_vectors()


def _config_args(config):
    c = dict(config)
    c.pop("id")
    return c


# ---------------------------------------------------------------------------
# reference fixtures: decode reproduces the array, encode reproduces the file
# ---------------------------------------------------------------------------
def test_fixture_shuffle_bytes_exact():
    n = 0
    for arr, j, config, enc in fixture_cases("shuffle"):
        es = config["elementsize"]
        got = oracle.shuffle(arr, es)
        assert got.tobytes() == enc, (j, es)
        dec = oracle.unshuffle(np.frombuffer(enc, "u1"), es)
        assert dec.tobytes() == arr.tobytes(order="A")
        n += 1
    assert n == 52


@pytest.mark.parametrize("prefix", ["bool", "int32", "float32", "float64", "uint16"])
def test_fixture_delta_bytes_exact(prefix):
    cases = list(fixture_cases("delta", prefix))
    assert cases
    for arr, _j, config, enc in cases:
        args = _config_args(config)
        got = oracle.delta_encode(arr, args["dtype"], args["astype"])
        assert got.tobytes() == enc
        dec = oracle.delta_decode(np.frombuffer(enc, "u1"), args["dtype"], args["astype"])
        assert dec.tobytes() == arr.tobytes(order="A")


def test_fixture_quantize_bytes_exact():
    n = 0
    for arr, _j, config, enc in fixture_cases("quantize"):
        a = _config_args(config)
        got = oracle.quantize_encode(arr, a["digits"], a["dtype"], a["astype"])
        assert got.tobytes(order="A") == enc
        n += 1
    assert n == 25


def test_fixture_fso_bytes_exact():
    n = 0
    for arr, _j, config, enc in fixture_cases("fixedscaleoffset"):
        a = _config_args(config)
        got = oracle.fso_encode(arr, a["offset"], a["scale"], a["dtype"], a["astype"])
        assert got.tobytes() == enc
        n += 1
    assert n == 25


# ---------------------------------------------------------------------------
# known-answer tests of the reference suite
# ---------------------------------------------------------------------------
def test_kat_shuffle_big_endian():
    # test_shuffle.py:131-159
    arr = np.array([0x0001020304050607, 0x08090A0B0C0D0E0F, 0x1011121314151617,
                    0x18191A1B1C1D1E1F], dtype=">u8")
    expected = np.array([0x00081018, 0x01091119, 0x020A121A, 0x030B131B, 0x040C141C,
                         0x050D151D, 0x060E161E, 0x070F171F], dtype="u4")
    enc = oracle.shuffle(arr, 8)
    np.testing.assert_array_equal(np.frombuffer(enc.tobytes(), ">u4"), expected)


KAT_FLETCHER = (
    b"w\x07\x00\x00\x00\x00\x00\x00\x85\xf6\xff\xff\xff\xff\xff\xff"
    b"i\x07\x00\x00\x00\x00\x00\x00\x94\xf6\xff\xff\xff\xff\xff\xff"
    b"\x88\t\x00\x00\x00\x00\x00\x00i\x03\x00\x00\x00\x00\x00\x00"
    b"\x93\xfd\xff\xff\xff\xff\xff\xff\xc3\xfc\xff\xff\xff\xff\xff\xff"
    b"'\x02\x00\x00\x00\x00\x00\x00\xba\xf7\xff\xff\xff\xff\xff\xff"
    b"\xfd%\x86d"
)


def test_kat_fletcher32():
    # test_fletcher32.py:25-48
    out = oracle.fletcher32_decode(KAT_FLETCHER)
    assert np.frombuffer(out.tobytes(), "<i8").tolist() == [
        1911, -2427, 1897, -2412, 2440, 873, -621, -829, 551, -2118]
    assert oracle.fletcher32_encode(out)[-4:] == KAT_FLETCHER[-4:]


def test_fletcher32_corruption_raises():
    enc = bytearray(oracle.fletcher32_encode(np.arange(100)))
    enc[0] += 1
    with pytest.raises(RuntimeError, match="fletcher32 checksum"):
        oracle.fletcher32_decode(enc)


@pytest.mark.parametrize("offset,scale,expected", [
    (1000, 10, [0, 6, 11, 17, 22, 28, 33, 39, 44, 50]),
    (1002.5, 10, [-25, -19, -14, -8, -3, 3, 8, 14, 19, 25]),
    (1000, 0.5, [0, 0, 1, 1, 1, 1, 2, 2, 2, 2]),
])
def test_kat_fso(offset, scale, expected):
    # test_fixedscaleoffset.py:39-55
    arr = np.linspace(1000, 1005, 10, dtype="<f8")
    got = oracle.fso_encode(arr, offset, scale, "<f8", np.int16)
    assert got.dtype == np.int16 and got.tolist() == expected


def test_kat_docstrings():
    # delta.py:28-39, quantize.py:23-40, fixedscaleoffset.py:30-62
    x = np.arange(100, 120, 2, dtype="i2")
    y = oracle.delta_encode(x, "i2", "i1")
    assert y.dtype == np.int8 and y.tolist() == [100] + [2] * 9
    assert oracle.delta_decode(y, "i2", "i1").tolist() == x.tolist()
    x = np.linspace(0, 1, 10, dtype="f8")
    assert oracle.quantize_encode(x, 1, "f8").tolist() == [
        0.0, 0.125, 0.25, 0.3125, 0.4375, 0.5625, 0.6875, 0.75, 0.875, 1.0]
    x = np.linspace(1000, 1001, 10, dtype="f8")
    assert oracle.fso_encode(x, 1000, 10, "f8", "u1").tolist() == [0, 1, 2, 3, 4, 6, 7, 8, 9, 10]
    assert oracle.fso_encode(x, 1000, 10**3, "f8", "u2").tolist() == [
        0, 111, 222, 333, 444, 556, 667, 778, 889, 1000]


def test_fletcher32_closed_form_block_independence():
    """The closed form the GPU reduction relies on (mc_fletcher.hip header):
    S1 = sum w, S2 = sum (n - i) w, r(S) = ((S-1) mod 65535) + 1 (0 iff all
    words are zero)."""
    rng = np.random.default_rng(7)
    for n in list(range(0, 40)) + [719, 720, 721, 1440, 5000, 65535 * 2 + 1]:
        for fill in ("rand", "ff", "zero"):
            x = (rng.integers(0, 256, n, dtype=np.uint8) if fill == "rand"
                 else np.full(n, 0xFF if fill == "ff" else 0, np.uint8))
            nw = (n + 1) // 2
            padded = np.concatenate([x, np.zeros(n % 2, np.uint8)])
            w = (padded[0::2].astype(np.int64) << 8) | padded[1::2].astype(np.int64)
            s1 = int(w.sum())
            s2 = int((w * (nw - np.arange(nw))).sum())

            def r(s):
                return 0 if s == 0 else (s - 1) % 65535 + 1

            assert oracle.fletcher32(x) == (r(s2) << 16) | r(s1), (n, fill)


# ---------------------------------------------------------------------------
# golden vectors (expected outputs from the real reference)
# ---------------------------------------------------------------------------
def test_vectors_shuffle():
    for i, m in enumerate(MANIFEST["shuffle"]):
        x = vec(DATA, "shuffle", i, "input")
        enc = vec(DATA, "shuffle", i, "encoded")
        assert np.array_equal(oracle.shuffle(x, m["elementsize"]), enc)
        assert np.array_equal(oracle.unshuffle(enc, m["elementsize"]), x)


def test_vectors_bitround():
    for i, m in enumerate(MANIFEST["bitround"]):
        x = vec(DATA, "bitround", i, "input").view(m["dtype"])
        with np.errstate(all="ignore"):
            got = oracle.bitround_encode(x.copy(), m["keepbits"])
        assert got.tobytes() == vec(DATA, "bitround", i, "encoded").tobytes(), m


def test_vectors_fso():
    for i, m in enumerate(MANIFEST["fso"]):
        x = vec(DATA, "fso", i, "input").view(m["dtype"])
        with np.errstate(all="ignore"):
            enc = oracle.fso_encode(x, m["offset"], m["scale"], m["dtype"], m["astype"])
            dec = oracle.fso_decode(enc, m["offset"], m["scale"], m["dtype"], m["astype"])
        assert enc.tobytes() == vec(DATA, "fso", i, "encoded").tobytes(), m
        assert dec.tobytes() == vec(DATA, "fso", i, "decoded").tobytes(), m


def test_vectors_quantize():
    for i, m in enumerate(MANIFEST["quantize"]):
        x = vec(DATA, "quantize", i, "input").view(m["dtype"])
        with np.errstate(all="ignore"):
            enc = oracle.quantize_encode(x, m["digits"], m["dtype"], m["astype"])
            dec = oracle.quantize_decode(enc, m["dtype"], m["astype"])
        assert enc.tobytes() == vec(DATA, "quantize", i, "encoded").tobytes(), m
        assert dec.tobytes() == vec(DATA, "quantize", i, "decoded").tobytes(), m


def test_vectors_delta():
    for i, m in enumerate(MANIFEST["delta"]):
        x = vec(DATA, "delta", i, "input").view(m["dtype"])
        with np.errstate(all="ignore"):
            enc = oracle.delta_encode(x, m["dtype"], m["astype"])
            dec = oracle.delta_decode(enc, m["dtype"], m["astype"])
        assert enc.tobytes() == vec(DATA, "delta", i, "encoded").tobytes(), m
        assert dec.tobytes() == vec(DATA, "delta", i, "decoded").tobytes(), m


def test_vectors_fletcher32():
    for i, m in enumerate(MANIFEST["fletcher32"]):
        assert oracle.fletcher32(vec(DATA, "fletcher32", i, "input")) == m["checksum"], m


def test_golden_inputs_portable():
    """The full-size inputs regenerate bit-identically (C1 here; C2-C5 use
    the same generators and are checked on the GPU box)."""
    import hashlib

    import inputs

    with open(os.path.join(os.path.dirname(FIXTURE), "fullsize.json")) as f:
        full = json.load(f)
    x1 = inputs.f32_wide(1, inputs.MiB // 4)
    assert hashlib.sha256(x1.tobytes()).hexdigest() == full["C1"]["input"]
    assert hashlib.sha256(oracle.shuffle(x1, 4).tobytes()).hexdigest() == full["C1"]["shuffle4"]


# ---------------------------------------------------------------------------
# direct comparison with the real reference (this container only)
# ---------------------------------------------------------------------------
def _ref():
    from oracle import refload

    if not refload.available():
        pytest.skip("reference sources / oracle/_ref build not present (GPU box)")
    return refload.load()


def test_oracle_matches_reference_random():
    nc = _ref()
    rng = np.random.default_rng(11)
    for es in (2, 3, 4, 8):
        x = rng.integers(0, 256, es * 3001, dtype=np.uint8)
        assert np.array_equal(oracle.shuffle(x, es), nc.Shuffle(es).encode(x))
        assert np.array_equal(oracle.unshuffle(x, es), nc.Shuffle(es).decode(x))
    for n in (1, 2, 3, 100, 721, 10001):
        x = rng.integers(0, 256, n, dtype=np.uint8)
        assert oracle.fletcher32_encode(x) == nc.Fletcher32().encode(x)
    x = rng.standard_normal(5000).astype("f4")
    for k in (0, 3, 10, 22):
        assert np.array_equal(oracle.bitround_encode(x.copy(), k), nc.BitRound(k).encode(x.copy()))


def test_reference_cpu_baseline_importable():
    """oracle/_ref's Cython _doShuffle is what bench.py times as the
    cpu_baseline "reference" leg."""
    _ref()
    import importlib

    mod = importlib.import_module("numcodecs._shuffle")
    x = np.arange(4096, dtype="u1")
    out = np.zeros_like(x)
    mod._doShuffle(x, out, 4)
    assert np.array_equal(out, nporacle.shuffle(x, 4))
