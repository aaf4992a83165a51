"""Property-based parity fuzzing on the GPU (hypothesis, derandomized so the
GPU run is reproducible): random sizes, dtypes, parameters and bit patterns
through every codec's device path, byte-compared with the oracle (numpy /
zlib / the C restatement of the reference's Cython), which tests/test_oracle*
pin to the reference itself.  Complements the fixed vectors with the
combinations nobody wrote down: odd lengths around every tile size, every
elementsize 1..17, keepbits over the whole range, NaN/inf/subnormal patterns.
"""

import warnings

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

import oracle
from numcodecs_amd import (
    CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, JenkinsLookup3, PackBits,
    Quantize, Shuffle,
)

pytestmark = pytest.mark.gpu

FUZZ = settings(max_examples=150, deadline=None, derandomize=True, database=None,
                suppress_health_check=list(HealthCheck))

# sizes that straddle the tile sizes of the kernels (4096 / 16384 elements,
# 64 KiB checksum tiles) plus small odd ones
SIZES = st.one_of(st.integers(0, 64), st.integers(4000, 4200), st.integers(16300, 16500),
                  st.integers(65000, 66000), st.integers(0, 200_000))


def _raw(seed: int, nbytes: int) -> np.ndarray:
    return np.random.default_rng(seed).integers(0, 256, nbytes, dtype=np.uint8)


def _dev(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _quiet():
    w = warnings.catch_warnings()
    w.__enter__()
    warnings.simplefilter("ignore")
    return w


@FUZZ
@given(n=SIZES, es=st.integers(1, 17), seed=st.integers(0, 2**32 - 1))
def test_fuzz_shuffle(device, n, es, seed):
    x = _raw(seed, n * es)
    xd = _dev(x, device)
    enc = Shuffle(es).encode(xd)
    assert enc.cpu().numpy().tobytes() == oracle.shuffle(x, es).tobytes()
    assert torch.equal(Shuffle(es).decode(enc), xd)


def _float_bits(seed, n, dtype):
    """random bit patterns (every class: NaN payloads, inf, subnormals, +-0)."""
    dt = np.dtype(dtype)
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
    b[: min(n, 8)] = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, np.finfo(dt).tiny / 2],
                              dtype=dt)[: min(n, 8)]
    return b


@FUZZ
@given(n=SIZES, dt=st.sampled_from(["<f2", "<f4", "<f8"]), seed=st.integers(0, 2**32 - 1), data=st.data())
def test_fuzz_bitround(device, n, dt, seed, data):
    maxb = {"<f2": 10, "<f4": 23, "<f8": 52}[dt]
    k = data.draw(st.integers(0, maxb - 1))
    x = _float_bits(seed, n, dt)
    enc = BitRound(k).encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == oracle.bitround_encode(x, k).tobytes()


DELTA_TYPES = [("<i2", "<i2"), ("<i4", "<i4"), ("<i8", "<i8"), ("|u1", "|u1"), ("<u4", "<u4"), ("|b1", "|b1"),
               ("<i4", "<i2"), ("<f4", "<f4"), ("<f8", "<f8"), ("<f2", "<f2"), ("<f8", "<f4")]


@FUZZ
@given(n=st.integers(1, 50_000), types=st.sampled_from(DELTA_TYPES), seed=st.integers(0, 2**32 - 1))
def test_fuzz_delta(device, n, types, seed):
    dt, at = types
    d = np.dtype(dt)
    rng = np.random.default_rng(seed)
    if d.kind == "f":
        x = rng.normal(0, 100, n).astype(d)
    elif d.kind == "b":
        x = rng.integers(0, 2, n).astype(bool)
    else:
        x = rng.integers(0, 256, n * d.itemsize, dtype=np.uint8).view(d).copy()
        x[0] = 7  # delta.py:63 enc[0] = arr[0] must fit astype
    codec = Delta(dt, at)
    w = _quiet()
    try:
        ref_enc = oracle.delta_encode(x, dt, at)
        ref_dec = oracle.delta_decode(ref_enc, dt, at)
    finally:
        w.__exit__(None, None, None)
    enc = codec.encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == ref_enc.tobytes()
    assert codec.decode(enc).cpu().numpy().tobytes() == ref_dec.tobytes()


@FUZZ
@given(n=SIZES, digits=st.integers(-2, 12), dt=st.sampled_from(["<f4", "<f8"]),
       at=st.sampled_from(["<f2", "<f4", "<f8"]), seed=st.integers(0, 2**32 - 1))
def test_fuzz_quantize(device, n, digits, dt, at, seed):
    x = (np.random.default_rng(seed).normal(0, 1000, n)).astype(dt)
    w = _quiet()
    try:
        ref = oracle.quantize_encode(x, digits, dt, at)
    finally:
        w.__exit__(None, None, None)
    enc = Quantize(digits, dt, at).encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == ref.tobytes()


@FUZZ
@given(n=SIZES, dt=st.sampled_from(["<f4", "<f8"]), at=st.sampled_from(["|i1", "<i2", "<i4", "<i8", "|u1", "<u2"]),
       offset=st.floats(-1e4, 1e4, allow_nan=False), scale=st.floats(1e-3, 1e4, allow_nan=False),
       seed=st.integers(0, 2**32 - 1))
def test_fuzz_fixedscaleoffset(device, n, dt, at, offset, scale, seed):
    info = np.iinfo(at)
    rng = np.random.default_rng(seed)
    # in-range data (out-of-range casts are covered by the fixed vectors)
    x = (offset + rng.uniform(max(info.min, -1e15), min(info.max, 1e15), n) / scale * 0.99).astype(dt)
    codec = FixedScaleOffset(offset=offset, scale=scale, dtype=dt, astype=at)
    w = _quiet()
    try:
        ref_enc = oracle.fso_encode(x, offset, scale, dt, at)
        ref_dec = oracle.fso_decode(ref_enc, offset, scale, dt, at)
    finally:
        w.__exit__(None, None, None)
    enc = codec.encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == ref_enc.tobytes()
    assert codec.decode(enc).cpu().numpy().tobytes() == ref_dec.tobytes()


@FUZZ
@given(n=st.integers(1, 300_000), seed=st.integers(0, 2**32 - 1), off=st.integers(0, 15))
def test_fuzz_fletcher32(device, n, seed, off):
    x = _raw(seed, n + off)
    xd = _dev(x, device)[off:]  # misaligned views too
    enc = Fletcher32().encode(xd)
    assert enc.cpu().numpy().tobytes() == oracle.fletcher32_encode(x[off:])
    assert torch.equal(Fletcher32().decode(enc), xd)


@FUZZ
@given(n=st.integers(0, 300_000), seed=st.integers(0, 2**32 - 1), off=st.integers(0, 15),
       cid=st.sampled_from(["crc32", "crc32c", "adler32"]), loc=st.sampled_from(["start", "end"]))
def test_fuzz_checksum32(device, n, seed, off, cid, loc):
    x = _raw(seed, n + off)
    codec = {"crc32": CRC32, "crc32c": CRC32C, "adler32": Adler32}[cid](location=loc)
    enc = codec.encode(_dev(x, device)[off:])
    assert enc.cpu().numpy().tobytes() == oracle.checksum32_encode(cid, x[off:], loc).tobytes()
    assert np.array_equal(codec.decode(enc).cpu().numpy(), x[off:])


FUZZ_BIG = settings(max_examples=40, deadline=None, derandomize=True, database=None,
                    suppress_health_check=list(HealthCheck))


@FUZZ_BIG
@given(tiles=st.integers(1, 2100), rem=st.integers(-8, 8), seed=st.integers(0, 2**32 - 1),
       off=st.sampled_from([0, 0, 4, 8, 1]), cid=st.sampled_from(["crc32", "crc32c", "adler32"]),
       loc=st.sampled_from(["start", "end"]), flip=st.integers(0, 2**40))
@example(tiles=2049, rem=4, seed=1, off=0, cid="crc32", loc="start", flip=123456789)
@example(tiles=1025, rem=-3, seed=2, off=1, cid="crc32c", loc="end", flip=987654321)
@example(tiles=513, rem=0, seed=3, off=4, cid="adler32", loc="start", flip=5)
@example(tiles=2100, rem=8, seed=4, off=8, cid="crc32c", loc="start", flip=2**39)
def test_fuzz_checksum32_one_launch(device, tiles, rem, seed, off, cid, loc, flip):
    """The one-launch encode and verify (the workgroups' sums riding the
    arrival atomics) over chunks of up to ~2100 tiles of 64 KiB with ragged
    ends, aligned and misaligned, at both locations; a flipped payload bit
    must fail the verify with the reference's error."""
    n = max(1, tiles * 65536 + rem)
    x = _raw(seed, n + off)
    codec = {"crc32": CRC32, "crc32c": CRC32C, "adler32": Adler32}[cid](location=loc)
    xd = _dev(x, device)[off:]
    enc = codec.encode(xd)
    ref = oracle.checksum32_encode(cid, x[off:], loc)
    assert enc.cpu().numpy().tobytes() == ref.tobytes()
    assert torch.equal(codec.decode(enc), xd)
    big = torch.empty(enc.numel() + 16, dtype=torch.uint8, device=device)
    view = big[off: off + enc.numel()]
    view.copy_(enc)
    k = (4 if loc == "start" else 0) + flip % n
    view[k] ^= 1 << (flip % 8)
    with pytest.raises(RuntimeError, match="checksum do not match"):
        codec.decode(view)


@FUZZ
@given(n=st.integers(0, 20_000), seed=st.integers(0, 2**32 - 1), initval=st.integers(0, 2**32 - 1),
       prefix=st.one_of(st.none(), st.binary(min_size=0, max_size=13)))
def test_fuzz_jenkins(device, n, seed, initval, prefix):
    x = _raw(seed, n)
    enc = JenkinsLookup3(initval=initval, prefix=prefix).encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == oracle.jenkins_encode(x, initval, prefix)


@FUZZ
@given(n=SIZES, seed=st.integers(0, 2**32 - 1))
def test_fuzz_packbits(device, n, seed):
    x = np.random.default_rng(seed).integers(0, 2, n).astype(bool)
    enc = PackBits().encode(_dev(x, device))
    ref = oracle.packbits_encode(x)
    assert enc.cpu().numpy().tobytes() == ref.tobytes()
    assert PackBits().decode(enc).cpu().numpy().tobytes() == x.tobytes()


@FUZZ
@given(n=SIZES, pair=st.sampled_from([("<f4", "<f8"), ("<f2", "<f4"), ("<f8", "<f2"), ("<i2", "<i8"),
                                      ("<f4", "<i4"), ("|u1", "<f8"), ("<i8", "<f4")]),
       seed=st.integers(0, 2**32 - 1))
def test_fuzz_astype(device, n, pair, seed):
    enc_t, dec_t = pair
    d = np.dtype(dec_t)
    rng = np.random.default_rng(seed)
    x = rng.normal(0, 1e3, n).astype(d) if d.kind == "f" else rng.integers(-100, 100, n).astype(d)
    w = _quiet()
    try:
        ref = oracle.astype_encode(x, enc_t, dec_t)
    finally:
        w.__exit__(None, None, None)
    enc = AsType(enc_t, dec_t).encode(_dev(x, device))
    assert enc.cpu().numpy().tobytes() == ref.tobytes()
