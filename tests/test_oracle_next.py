"""Pin the oracle for the §8f next-row codecs (Checksum32 family, AsType,
PackBits) against the reference's own fixtures (fixture/{crc32,crc32c,adler32,
astype,packbits}), its known-answer tests (test_jenkins.py:8-71,
packbits.py/astype.py docstrings) and, where the reference is importable
here, against the reference's compiled jenkins.pyx and Python modules.
"""

import os
import zlib
from glob import glob

import numpy as np
import pytest

import oracle
try:  # the reference loader stays in this container (.gpurunignore)
    from oracle import refload
except ImportError:  # GPU box
    refload = None
from tests.helpers import FIXTURE, fixture_cases

RNG = np.random.default_rng(77)


def _args(config):
    c = dict(config)
    c.pop("id")
    return c


@pytest.mark.parametrize("codec_id,count", [("crc32", 13), ("adler32", 13), ("crc32c", 13)])
def test_fixture_checksum32_bytes_exact(codec_id, count):
    n = 0
    for arr, _j, config, enc in fixture_cases(codec_id):
        loc = _args(config).get("location")
        got = oracle.checksum32_encode(codec_id, arr, loc)
        assert got.tobytes() == enc, (codec_id, _j)
        dec = oracle.checksum32_decode(codec_id, np.frombuffer(enc, "u1"), loc)
        assert dec.tobytes() == arr.tobytes(order="A")
        n += 1
    assert n == count


def test_fixture_checksum32_corruption_detected():
    for arr, _j, _config, enc in fixture_cases("crc32"):
        bad = bytearray(enc)
        bad[len(bad) // 2] ^= 1
        with pytest.raises(RuntimeError):
            oracle.checksum32_decode("crc32", np.frombuffer(bytes(bad), "u1"))
        break


@pytest.mark.parametrize("prefix", ["f", "i"])
def test_fixture_astype_bytes_exact(prefix):
    cases = list(fixture_cases("astype", prefix))
    assert cases
    for arr, _j, config, enc in cases:
        a = _args(config)
        got = oracle.astype_encode(arr, a["encode_dtype"], a["decode_dtype"])
        assert got.tobytes(order="A") == enc
        dec = oracle.astype_decode(np.frombuffer(enc, a["encode_dtype"]), a["encode_dtype"], a["decode_dtype"])
        if prefix == "i":
            assert dec.tobytes() == arr.tobytes(order="A")
        else:  # f8 -> f4 -> f8 is lossy; the fixture's stored bytes are the reference
            assert np.array_equal(dec, arr.reshape(-1, order="A").astype("<f4").astype("<f8"))


def test_fixture_packbits_bytes_exact():
    n = 0
    for arr, _j, _config, enc in fixture_cases("packbits"):
        assert oracle.packbits_encode(arr).tobytes() == enc
        dec = oracle.packbits_decode(np.frombuffer(enc, "u1"))
        assert np.array_equal(dec, arr.reshape(-1, order="A"))
        n += 1
    assert n == 4


def test_kat_jenkins():
    """test_jenkins.py:8-71."""
    j = oracle.jenkins_lookup3
    assert j(b"", 0) == 0xDEADBEEF
    assert j(b"", 0xDEADBEEF) == 0xBD5B7DDE
    assert j(b"Four score and seven years ago", 0) == 0x17770551
    assert j(b"Four score and seven years ago", 1) == 0xCD628161
    assert j(b"jenkins", 0) == 202276345
    s = b"Four score and seven years ago"
    assert oracle.jenkins_encode(s)[-4:] == b"\x51\x05\x77\x17"
    assert oracle.jenkins_encode(s, initval=1230)[-4:] == b"\xd7Z\xe2\x0e"
    h = [0]
    for _ in range(9):
        v = j(b"", h[-1])
        assert v not in h
        h.append(v)


def test_kat_crc32c_check_value():
    # the CRC-32C catalogue check value of "123456789"
    assert oracle.crc32c(b"123456789") == 0xE3069283
    assert oracle.crc32c(b"") == 0


def test_kat_packbits_docstring():
    """packbits.py:13-21."""
    x = np.array([True, False, False, True], dtype=bool)
    assert oracle.packbits_encode(x).tolist() == [4, 144]
    assert oracle.packbits_decode(np.array([4, 144], "u1")).tolist() == [True, False, False, True]


def test_kat_astype_docstring():
    """astype.py:27-38."""
    x = np.arange(100, 120, 2, dtype=np.int8)
    y = oracle.astype_decode(x, "i1", "i2")
    assert y.dtype == np.int16 and y.tolist() == list(range(100, 120, 2))
    assert oracle.astype_encode(y, "i1", "i2").dtype == np.int8


def test_crc32c_streaming_and_split():
    """crc32c(a ++ b) == crc32c(b, crc32c(a)) -- the `value` continuation the
    device combine relies on."""
    for n in (0, 1, 7, 100, 4099):
        d = RNG.integers(0, 256, n, dtype=np.uint8).tobytes()
        for cut in (0, n // 3, n):
            assert oracle.crc32c(d[cut:], oracle.crc32c(d[:cut])) == oracle.crc32c(d)
        assert oracle.crc32(d[n // 2:], oracle.crc32(d[: n // 2])) == zlib.crc32(d)


@pytest.mark.skipif(refload is None or not refload.available(), reason="reference not importable here")
def test_oracle_matches_reference_jenkins_astype_packbits():
    nc = refload.load()
    for n in (0, 1, 11, 12, 13, 24, 25, 100, 1000, 4097):
        d = RNG.integers(0, 256, n, dtype=np.uint8)
        for init in (0, 1, 0xDEADBEEF, 1230):
            assert nc.jenkins_lookup3(d, init) == oracle.jenkins_lookup3(d, init)
    for n in (0, 1, 7, 8, 9, 1001):
        x = RNG.integers(0, 2, n).astype(bool)
        assert np.array_equal(nc.PackBits().encode(x), oracle.packbits_encode(x))
    for enc_dt, dec_dt in (("<f4", "<f8"), ("<i2", "<i4"), ("<u1", "<f8"), ("<i4", "<f4")):
        x = (RNG.standard_normal(257) * 1e5).astype(dec_dt)
        assert np.array_equal(nc.AsType(enc_dt, dec_dt).encode(x), oracle.astype_encode(x, enc_dt, dec_dt))


# ---------------------------------------------------------------------------
# Blosc shuffle framing (oracle/blosc.py) pinned by fixture/blosc frames
# ---------------------------------------------------------------------------
def _blosc_cases():
    from oracle import blosc

    for arr, j, config, frame in fixture_cases("blosc"):
        flags, ts, bs, blocks = (None, None, None, None)
        try:
            flags, ts, bs, blocks = blosc.frame_filtered_blocks(frame)
        except NotImplementedError:
            continue
        yield arr, j, config, flags, ts, bs, blocks


def test_fixture_blosc_filters_bytes_exact():
    from oracle import blosc

    counts = {1: 0, 2: 0, 0: 0}
    for arr, _j, config, flags, ts, bs, blocks in _blosc_cases():
        raw = arr.tobytes(order="A")
        if blocks is None:  # memcpyed frame: stored raw
            continue
        mode = 2 if flags & blosc.BLOSC_DOBITSHUFFLE else 1 if flags & blosc.BLOSC_DOSHUFFLE else 0
        if config["shuffle"] in (1, 2):
            assert mode == config["shuffle"] or (ts == 1 and mode == 0)
        filtered = b"".join(blocks)
        if mode == 0:
            assert filtered == raw
        else:
            assert blosc.blosc_filter(raw, ts, bs, mode) == filtered, (_j, ts, bs, mode)
            assert blosc.blosc_filter(filtered, ts, bs, mode, forward=False) == raw
        counts[mode] += 1
    assert counts == {0: 16, 1: 55, 2: 13}, counts  # 84 LZ4 frames walked


def test_blosc_filter_roundtrip_edges():
    from oracle import blosc

    for ts in (1, 2, 3, 4, 8, 16):
        for n in (0, 1, 7, 64, 1000, 4099):
            raw = RNG.integers(0, 256, n * ts + (n % 3), dtype=np.uint8).tobytes()
            for bs in (8 * ts, 255, 4096):
                for mode in (1, 2):
                    enc = blosc.blosc_filter(raw, ts, bs, mode)
                    assert len(enc) == len(raw)
                    assert blosc.blosc_filter(enc, ts, bs, mode, forward=False) == raw


def test_blosc_compute_blocksize_pinned_by_fixture_headers():
    """numcodecs_amd.blosc_shuffle.compute_blocksize (c-blosc's
    compute_blocksize restated; host logic, no device) against the blocksize
    in every fixture/blosc frame header it covers: the frames the current
    c-blosc wrote (arrays 05-12, automatic blocksize) and every frame with a
    forced blocksize.  Arrays 00-04 with an automatic blocksize were written
    by an older c-blosc (128/256-byte blocks for <= 8 KB buffers) and are
    reported, not matched."""
    from numcodecs_amd.blosc_shuffle import compute_blocksize
    from oracle import blosc

    checked = old = 0
    ncodecs = len(glob(os.path.join(FIXTURE, "blosc", "codec.*")))
    for k, (arr, j, config, frame) in enumerate(fixture_cases("blosc")):
        i = k // ncodecs  # the array index (arrays outer, codecs inner)
        flags, ts, nbytes, bs, _cb = blosc.frame_header(frame)
        got = compute_blocksize(nbytes, ts, config["clevel"], config["cname"], config["blocksize"])
        if config["blocksize"] == 0 and i <= 4:
            old += 1
            continue
        assert got == bs, (i, j, config, ts, nbytes, bs, got)
        checked += 1
    assert checked == 8 * 11 + 13 * 2 and old == 5 * 11


def test_blosc_compute_blocksize_rules():
    """The branches the fixtures cannot reach (buffers >= 32 KiB): c-blosc's
    published rule, parity unpinned (c-blosc is absent here)."""
    from numcodecs_amd.blosc_shuffle import compute_blocksize

    MiB = 1 << 20
    assert compute_blocksize(256 * MiB, 4, 5, "lz4") == 524288  # L1 x 4 = 128 KiB, split: x typesize
    assert compute_blocksize(256 * MiB, 4, 5, "zstd") == 262144  # HCR x 2, never split
    assert compute_blocksize(256 * MiB, 4, 9, "zlib") == 1 << 20  # HCR, clevel 9, split, capped at 1 MiB
    assert compute_blocksize(256 * MiB, 4, 0, "lz4") == 8192  # clevel 0: L1 / 4, no split at clevel 0
    assert compute_blocksize(256 * MiB, 32, 5, "lz4") == 131072  # typesize > 16: no split
    assert compute_blocksize(256 * MiB, 3, 1, "blosclz") == 65535  # 16 KiB x 3, raised to 64 KiB, multiple of 3
    assert compute_blocksize(100, 300, 5, "lz4") == 100  # typesize > 255 counts as 1
    assert compute_blocksize(3, 4, 5, "lz4") == 1  # fewer bytes than one element
    assert compute_blocksize(10000, 4, 5, "lz4", 64) == 128  # forced sizes are at least 128
    with pytest.raises(ValueError):
        compute_blocksize(100, 4, 10)
