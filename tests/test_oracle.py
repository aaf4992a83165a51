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
    try:
        from oracle import refload
    except ImportError:  # the reference loader stays in the build container (.gpurunignore)
        pytest.skip("reference loader not present (GPU box)")
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


def test_port_equals_reference_cython_loops():
    """bench.py's cpu_baseline times the C restatement (oracle/ncoracle.c),
    never the reference; here (where oracle/_ref exists) the restatement is
    byte-identical to the reference's compiled _doShuffle/_doUnshuffle and
    _fletcher32 on random buffers of every elementsize."""
    _ref()
    import importlib

    mod = importlib.import_module("numcodecs._shuffle")
    rng = np.random.default_rng(5)
    for es in (2, 3, 4, 8, 16):
        x = rng.integers(0, 256, es * 4099, dtype=np.uint8)
        a, b = np.zeros_like(x), np.zeros_like(x)
        mod._doShuffle(x, a, es)
        nporacle.shuffle_into(x, b, es)
        assert np.array_equal(a, b)
        mod._doUnshuffle(x, a, es)
        nporacle.unshuffle_into(x, b, es)
        assert np.array_equal(a, b)


# ---------------------------------------------------------------------------
# the scalar C restatement timed as bench.py's cpu_baseline (oracle/ncoracle.c)
# ---------------------------------------------------------------------------
def test_c_restatement_bitround32_goldens():
    n = 0
    for i, m in enumerate(MANIFEST["bitround"]):
        if m["dtype"] != "<f4":
            continue
        x = vec(DATA, "bitround", i, "input").view("<u4")
        out = np.empty_like(x)
        nporacle.c_bitround32_into(x, out, m["keepbits"])
        assert out.tobytes() == vec(DATA, "bitround", i, "encoded").tobytes(), m
        n += 1
    assert n >= 6


def test_c_restatement_fso_f4_i2_goldens():
    n = 0
    for i, m in enumerate(MANIFEST["fso"]):
        if (m["dtype"], m["astype"]) != ("<f4", "<i2"):
            continue
        x = vec(DATA, "fso", i, "input").view("<f4")
        enc = np.empty(x.size, dtype="<i2")
        nporacle.c_fso_encode_f4_i2_into(x, enc, m["offset"], m["scale"])
        assert enc.tobytes() == vec(DATA, "fso", i, "encoded").tobytes(), m
        dec = np.empty(x.size, dtype="<f4")
        nporacle.c_fso_decode_i2_f4_into(enc, dec, m["offset"], m["scale"])
        exp = oracle.fso_decode(enc, m["offset"], m["scale"], "<f4", "<i2")
        assert dec.tobytes() == exp.tobytes(), m
        n += 1
    assert n == 2


def test_c_restatement_fso_decode_every_int16():
    """(enc / scale) + offset in float64 -> float32 for all 65536 int16 values."""
    enc = np.arange(-32768, 32768, dtype="<i2")
    for offset, scale in ((1000, 1e3), (1000.1, 1000.0), (-3.5, 0.1), (0, 7)):
        dec = np.empty(enc.size, dtype="<f4")
        nporacle.c_fso_decode_i2_f4_into(enc, dec, offset, scale)
        assert dec.tobytes() == oracle.fso_decode(enc, offset, scale, "<f4", "<i2").tobytes()


def test_c_restatement_delta_i2_goldens_and_wrap():
    i = next(k for k, m in enumerate(MANIFEST["delta"]) if (m["dtype"], m["astype"]) == ("<i2", "<i2"))
    x = vec(DATA, "delta", i, "input").view("<i2")
    enc = np.empty_like(x)
    nporacle.c_delta_encode_i2_into(x, enc)
    assert enc.tobytes() == vec(DATA, "delta", i, "encoded").tobytes()
    dec = np.empty_like(x)
    nporacle.c_delta_decode_i2_into(enc, dec)
    assert np.array_equal(dec, x)
    w = np.array([32767, -32768, 5, -32768, 32767, 0], dtype="<i2")
    e2 = np.empty_like(w)
    nporacle.c_delta_encode_i2_into(w, e2)
    assert e2.tobytes() == oracle.delta_encode(w, "<i2").tobytes()


def test_c_restatement_c4_chain_sha():
    """The CPU baseline's C4 chain (FSO f4->i2, Delta i2, Shuffle 2, and back)
    reproduces the reference's outputs on the full-size C4 input (256 MiB
    f32, tests/golden/inputs.py), by the SHA-256 digests make_golden.py took
    from the real reference."""
    import hashlib

    from tests.golden import inputs

    with open(os.path.join(os.path.dirname(__file__), "golden", "fullsize.json")) as f:
        full = json.load(f)["C4"]
    sha = lambda a: hashlib.sha256(a.tobytes()).hexdigest()  # noqa: E731
    x = inputs.f32_c4(4, 64 << 20)
    assert sha(x) == full["input"]
    t1 = np.empty(x.size, dtype="<i2")
    t2 = np.empty_like(t1)
    nporacle.c_fso_encode_f4_i2_into(x, t1, 1000, 1e3)
    assert sha(t1) == full["fso"]
    nporacle.c_delta_encode_i2_into(t1, t2)
    assert sha(t2) == full["delta"]
    enc = np.empty(t2.nbytes, dtype="u1")
    nporacle.shuffle_into(t2, enc, 2)
    assert sha(enc) == full["shuffle2"]
    nporacle.unshuffle_into(enc, t1, 2)
    nporacle.c_delta_decode_i2_into(t1, t2)
    dec = np.empty_like(x)
    nporacle.c_fso_decode_i2_f4_into(t2, dec, 1000, 1e3)
    assert sha(dec) == full["decoded"]


def test_cpu_baseline_workloads_roundtrip():
    """Every bench cpu_baseline workload decodes to the oracle's answer."""
    from oracle import cpu_baseline

    for cfg, nbytes in (("C1", 1 << 20), ("C2_f32", 1 << 20), ("C2_f64", 1 << 20), ("C3", 1 << 20),
                        ("C4", 1 << 20), ("C5", 2 << 20)):
        w = cpu_baseline.Workload(cfg, nbytes, seed=3)
        w.step()
        w.verify()


def test_oracle_chain_roundtrip():
    """tests/oracle_chain.py (the pipeline tests' checker): each chain's oracle
    encode decodes back to the input, and the checksum steps catch a flipped
    byte -- on CPU, no device involved."""
    from numcodecs_amd import (
        CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, JenkinsLookup3,
        PackBits, Quantize, Shuffle,
    )
    from tests import oracle_chain

    rng = np.random.default_rng(11)
    f4 = (1000 + 10 * rng.random(3001)).astype("<f4")
    f8 = f4.astype("<f8")
    i4 = rng.integers(-1000, 1000, 3001).astype("<i4")
    cases = [
        ([BitRound(23), Shuffle(4), CRC32()], f4, True),
        ([FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"), Delta(dtype="<i2"), Shuffle(2),
          Adler32(location="end")], f4, False),
        ([Quantize(3, "<f8", "<f4"), Shuffle(4), Fletcher32()], f8, False),
        ([AsType("<f4", "<f8"), Shuffle(4), JenkinsLookup3(initval=7)], f8, True),
        ([Delta(dtype="<i4"), Shuffle(4), CRC32C()], i4, True),
        ([PackBits()], rng.integers(0, 2, 77).astype(bool), True),
    ]
    for codecs, x, exact in cases:
        enc = oracle_chain.chain_encode(codecs, x)
        dec = np.frombuffer(oracle_chain.chain_decode(codecs, enc), dtype=x.dtype)
        if exact:
            assert np.array_equal(dec, x), codecs
        else:
            assert np.allclose(dec, x, atol=1e-2), codecs
        if codecs[-1].codec_id in ("crc32", "crc32c", "adler32", "fletcher32", "jenkins_lookup3"):
            bad = bytearray(enc)
            bad[len(bad) // 2] ^= 1
            with pytest.raises(RuntimeError):
                oracle_chain.chain_decode(codecs, bytes(bad))
