"""The device kernels' longdouble ('<f16', x87 80-bit extended) arithmetic
(numcodecs_amd/csrc/mc_x80.h) against numpy's own longdouble results on the
build machine: the same header compiled for the host (tests/native/
host_check.hip -> libhostcheck.so), fed random and special operands -- zeros,
denormals, pseudo-denormals, unnormals, pseudo-infinities / pseudo-NaNs, quiet
and signalling NaNs with payloads, infinities, integers and halfway values,
values around 2^63 / 2^64 and the int/float range limits.  Results are
compared on the 10 value bytes of each element (numpy leaves the 6 padding
bytes of a computed longdouble as whatever the output buffer held).

Reference: numpy's longdouble ufunc loops and casts, which the reference's
Delta / Quantize / FixedScaleOffset / AsType (delta.py:52-83,
quantize.py:60-82, fixedscaleoffset.py:83-113, astype.py:47-59) call."""

import ctypes
import os

import numpy as np
import pytest

from numcodecs_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "_build", "libhostcheck.so")

pytestmark = pytest.mark.skipif(np.finfo(np.longdouble).nmant != 63,
                                reason="numpy's longdouble is not x87 extended on this machine")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (__graft_entry__.build())")
    lib = ctypes.CDLL(LIB)
    P, N, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    for f, args in (("x80h_binop", [I, P, P, P, N]), ("x80h_rint", [P, P, N]), ("x80h_from", [I, P, P, N]),
                    ("x80h_to", [I, P, P, N])):
        getattr(lib, f).restype = ctypes.c_int
        getattr(lib, f).argtypes = args
    lib.calh_convert.restype = ctypes.c_int
    lib.calh_convert.argtypes = [P, P, N, I, ctypes.c_int64, I, ctypes.c_int64]
    return lib


def ld(m, se):
    """longdouble array from significand / sign+exponent words."""
    m = np.asarray(m, dtype=np.uint64).reshape(-1)
    se = np.broadcast_to(np.asarray(se, dtype=np.uint16), m.shape)
    b = np.zeros((m.size, 16), np.uint8)
    b[:, :8] = m.view(np.uint8).reshape(-1, 8)
    b[:, 8:10] = np.ascontiguousarray(se).view(np.uint8).reshape(-1, 2)
    return b.reshape(-1).view(np.longdouble)


def value_bytes(a):
    return np.ascontiguousarray(a).view(np.uint8).reshape(-1, 16)[:, :10]


def operands(rng, n):
    """n longdoubles mixing every class x87 distinguishes."""
    J = np.uint64(1 << 63)
    parts = []
    k = n // 16
    r64 = lambda: rng.integers(0, 1 << 63, k, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, k, dtype=np.uint64)
    sgn = lambda: rng.integers(0, 2, k, dtype=np.uint16) << np.uint16(15)
    # normals over the whole range and near 1
    parts.append(ld(r64() | J, sgn() | rng.integers(1, 0x7fff, k, dtype=np.uint16)))
    parts.append(ld(r64() | J, sgn() | rng.integers(16383 - 70, 16383 + 70, k, dtype=np.uint16)))
    parts.append(ld(r64() | J, sgn() | rng.integers(16383 - 3, 16383 + 3, k, dtype=np.uint16)))
    # short significands (exact sums / integers / halves)
    short = (rng.integers(0, 1 << 12, k, dtype=np.uint64) << np.uint64(51)) | J
    parts.append(ld(short, sgn() | rng.integers(16383 - 4, 16383 + 66, k, dtype=np.uint16)))
    # denormals, pseudo-denormals, tiny normals
    parts.append(ld(r64() >> rng.integers(1, 64, k, dtype=np.uint64), sgn()))
    parts.append(ld(r64() | J, sgn()))
    parts.append(ld(r64() | J, sgn() | rng.integers(1, 80, k, dtype=np.uint16)))
    # huge
    parts.append(ld(r64() | J, sgn() | rng.integers(0x7fff - 80, 0x7fff, k, dtype=np.uint16)))
    # unnormals, pseudo-inf / pseudo-NaN
    parts.append(ld(r64() >> np.uint64(1), sgn() | rng.integers(1, 0x7fff, k, dtype=np.uint16)))
    parts.append(ld(r64() >> rng.integers(1, 3, k, dtype=np.uint64), sgn() | np.uint16(0x7fff)))
    # infinities, quiet / signalling NaNs
    parts.append(ld(np.full(k, J, np.uint64), sgn() | np.uint16(0x7fff)))
    parts.append(ld(r64() | J | np.uint64(1 << 62), sgn() | np.uint16(0x7fff)))
    sn = (r64() & np.uint64((1 << 62) - 1)) | J
    sn[sn == J] |= np.uint64(1)
    parts.append(ld(sn, sgn() | np.uint16(0x7fff)))
    # zeros
    parts.append(ld(np.zeros(k, np.uint64), sgn()))
    # around the integer limits
    lim = np.array([2.0 ** e for e in (7, 8, 15, 16, 31, 32, 63, 64)], np.longdouble)
    near = lim[rng.integers(0, lim.size, k)] * np.where(rng.integers(0, 2, k) == 1, 1, -1).astype(np.longdouble)
    near += rng.integers(-3, 4, k).astype(np.longdouble) * np.where(rng.integers(0, 2, k) == 1, 0.5, 1).astype(np.longdouble)
    parts.append(near)
    # integers and halves
    parts.append(rng.integers(-(1 << 20), 1 << 20, k).astype(np.longdouble) / 2)
    a = np.concatenate(parts)
    return a[rng.permutation(a.size)]


def call(fn, *args):
    rc = fn(*args)
    assert rc == 0


@pytest.mark.parametrize("op", ["add", "sub", "mul", "div"])
def test_binops_vs_numpy(lib, op):
    rng = np.random.default_rng(["add", "sub", "mul", "div"].index(op))
    n = 1 << 16
    a, b = operands(rng, n), operands(rng, n)
    # operand pairs with close exponents (cancellation) and swapped duplicates
    b[: n // 8] = a[: n // 8] * (1 + rng.standard_normal(n // 8).astype(np.longdouble) * 2.0 ** -40)
    b[n // 8: n // 4] = a[n // 4: 3 * n // 8]
    with np.errstate(all="ignore"):
        want = {"add": np.add, "sub": np.subtract, "mul": np.multiply, "div": np.true_divide}[op](a, b)
    got = np.empty_like(a)
    call(lib.x80h_binop, ["add", "sub", "mul", "div"].index(op), a.ctypes.data, b.ctypes.data,
         got.ctypes.data, a.size)
    bad = np.nonzero((value_bytes(got) != value_bytes(want)).any(axis=1))[0]
    assert bad.size == 0, [(value_bytes(a[i:i + 1]).tobytes().hex(), value_bytes(b[i:i + 1]).tobytes().hex(),
                            value_bytes(got[i:i + 1]).tobytes().hex(), value_bytes(want[i:i + 1]).tobytes().hex())
                           for i in bad[:5]]


def test_rint_vs_numpy(lib):
    rng = np.random.default_rng(7)
    a = operands(rng, 1 << 16)
    with np.errstate(all="ignore"):
        want = np.rint(a)
    got = np.empty_like(a)
    call(lib.x80h_rint, a.ctypes.data, got.ctypes.data, a.size)
    bad = np.nonzero((value_bytes(got) != value_bytes(want)).any(axis=1))[0]
    assert bad.size == 0, [(value_bytes(a[i:i + 1]).tobytes().hex(), value_bytes(got[i:i + 1]).tobytes().hex(),
                            value_bytes(want[i:i + 1]).tobytes().hex()) for i in bad[:5]]


REAL = ["?", "i1", "i2", "i4", "i8", "u1", "u2", "u4", "u8", "f2", "f4", "f8"]


@pytest.mark.parametrize("dt", REAL)
def test_cast_to_vs_numpy(lib, dt):
    rng = np.random.default_rng(REAL.index(dt))
    a = operands(rng, 1 << 16)
    with np.errstate(all="ignore"):
        want = a.astype(dt)
    got = np.empty_like(want)
    call(lib.x80h_to, _native.DTYPE_CODES[np.dtype(dt).str], a.ctypes.data, got.ctypes.data, a.size)
    bad = np.nonzero(got.view(np.uint8).reshape(a.size, -1) != want.view(np.uint8).reshape(a.size, -1))[0]
    assert bad.size == 0, [(value_bytes(a[i:i + 1]).tobytes().hex(), got[i:i + 1].tobytes().hex(),
                            want[i:i + 1].tobytes().hex()) for i in bad[:5]]


@pytest.mark.parametrize("dt", REAL)
def test_cast_from_vs_numpy(lib, dt):
    rng = np.random.default_rng(100 + REAL.index(dt))
    size = np.dtype(dt).itemsize
    src = rng.integers(0, 256, (1 << 16) * size, dtype=np.uint8).view(dt)
    if dt == "?":
        src = rng.integers(0, 2, 1 << 16).astype("?")
    if np.dtype(dt).kind == "f":  # specials: NaN payloads, infinities, denormals
        bits = src.view(f"u{size}")
        bits[::7] &= np.array((1 << (8 * size - 1)) | ((1 << {2: 5, 4: 8, 8: 11}[size]) - 1) << {2: 10, 4: 23, 8: 52}[size] |
                              1, dtype=f"u{size}")
    want = src.astype(np.longdouble)
    got = np.empty_like(want)
    call(lib.x80h_from, _native.DTYPE_CODES[np.dtype(dt).str], src.ctypes.data, got.ctypes.data, src.size)
    bad = np.nonzero((value_bytes(got) != value_bytes(want)).any(axis=1))[0]
    assert bad.size == 0, [(src[i:i + 1].tobytes().hex(), value_bytes(got[i:i + 1]).tobytes().hex(),
                            value_bytes(want[i:i + 1]).tobytes().hex()) for i in bad[:5]]


def test_special_pairs_vs_numpy(lib):
    """Every ordered pair of a crafted set of specials (NaNs with equal and
    different significands of both signs, SNaN vs QNaN, rejected formats,
    infinities, zeros, denormals, pseudo-denormals, the extremes) through all
    four operations: the x87 NaN-selection and invalid rules."""
    J, Q = 1 << 63, 1 << 62
    vals = [(J | Q | 5, 0x7fff), (J | Q | 5, 0xffff), (J | Q | 9, 0x7fff), (J | Q, 0xffff), (J | 5, 0x7fff),
            (J | 5, 0xffff), (J | 9, 0xffff), (J, 0x7fff), (J, 0xffff), (0, 0), (0, 0x8000), (1, 0), (J | 3, 0),
            (J | 3, 0x8000), ((1 << 62), 0x3fff), (Q, 0x7fff), (5, 0x7fff), (J, 1), ((1 << 64) - 1, 0x7ffe),
            ((1 << 64) - 1, 0xfffe), (J, 0x3fff), (J | 1, 0xbfff), (J | Q, 0x4000)]
    x = ld([v[0] for v in vals], [v[1] for v in vals])
    a = np.repeat(x, x.size)
    b = np.tile(x, x.size)
    for i, f in enumerate((np.add, np.subtract, np.multiply, np.true_divide)):
        with np.errstate(all="ignore"):
            want = f(a, b)
        got = np.empty_like(a)
        call(lib.x80h_binop, i, a.ctypes.data, b.ctypes.data, got.ctypes.data, a.size)
        bad = np.nonzero((value_bytes(got) != value_bytes(want)).any(axis=1))[0]
        assert bad.size == 0, (f.__name__, [(value_bytes(a[j:j + 1]).tobytes().hex(),
                                             value_bytes(b[j:j + 1]).tobytes().hex(),
                                             value_bytes(got[j:j + 1]).tobytes().hex(),
                                             value_bytes(want[j:j + 1]).tobytes().hex()) for j in bad[:6]])


UNITS = ["Y", "M", "W", "D", "h", "m", "s", "ms", "us", "ns", "ps", "fs", "as"]
# ticks per day of the linear units (for a realistic range of dates)
PER_DAY = {"W": 1 / 7, "D": 1, "h": 24, "m": 1440, "s": 86400, "ms": 86400e3, "us": 86400e6, "ns": 86400e9,
           "ps": 86400e12, "fs": 86400e15, "as": 86400e18}


def _cal_pairs():
    out = []
    for s in UNITS:
        for d in UNITS:
            if s == d or (s in "YM") == (d in "YM"):
                continue
            for sn, dn in ((1, 1), (3, 1), (1, 5), (2, 7)):
                src, dst = np.dtype(f"M8[{sn}{s}]"), np.dtype(f"M8[{dn}{d}]")
                try:
                    np.zeros(1, src).astype(dst)
                except (OverflowError, ValueError, TypeError):
                    continue
                out.append((s, sn, d, dn))
    return out


@pytest.mark.parametrize("s,sn,d,dn", _cal_pairs())
def test_calendar_cast_vs_numpy(lib, s, sn, d, dn):
    """mc_cal.h's calendar cast against numpy's datetime64 astype: NaT,
    negative ticks, dates from -30000 to 30000 (within the range numpy's
    int64 arithmetic holds for the unit)."""
    rng = np.random.default_rng(UNITS.index(s) * 100 + UNITS.index(d))
    if s == "Y":
        span = 30000
    elif s == "M":
        span = 30000 * 12
    else:
        span = min(30000 * 365 * PER_DAY[s], 2 ** 62)
        if d in "YM" and s in ("fs", "as"):
            span = 2 ** 62
    span = int(span // sn)
    v = rng.integers(-span, span, 4096, dtype=np.int64)
    v[:8] = [0, -1, 1, np.iinfo(np.int64).min, 11, -11, 12, -13]
    src = v.view(f"M8[{sn}{s}]")
    with np.errstate(all="ignore"):
        want = src.astype(f"M8[{dn}{d}]").view(np.int64)
    got = np.empty_like(v)
    call(lib.calh_convert, v.ctypes.data, got.ctypes.data, v.size, UNITS.index(s), sn, UNITS.index(d), dn)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(v[i]), int(got[i]), int(want[i])) for i in bad[:6]]
