"""Host logic of the extended dtypes (CPU only, no kernels).

* ``_ops.datetime_conversion_factor`` restates numpy's
  get_datetime_conversion_factor; applied with numpy's cast rule
  (v*num/den, floor for negatives, wrap-around products, NaT kept) -- the
  arithmetic mc_cast_units does on the device -- it must reproduce numpy's
  own astype between every pair of timedelta64 units (and datetime64 linear
  units), multiples included;
* ``_ops.dtype_code`` maps complex / timedelta / datetime dtypes of either
  byte order to the include/mcodec.h codes;
* codecs raise numpy's errors for the combinations the reference refuses
  before any device work (dry runs of the reference's expressions).
"""

import numpy as np
import pytest

from numcodecs_amd import _native, _ops

UNITS = ["Y", "M", "W", "D", "h", "m", "s", "ms", "us", "ns", "ps", "fs", "as"]
NAT = np.iinfo(np.int64).min


def _ticks():
    rng = np.random.default_rng(3)
    t = np.concatenate([
        np.array([0, 1, -1, 7, -7, 999, -1001, 2**31, -(2**40) - 3, 2**62, -(2**62), NAT, NAT + 1,
                  np.iinfo(np.int64).max], dtype=np.int64),
        rng.integers(-(10**12), 10**12, 200),
        rng.integers(-(2**63), 2**63 - 1, 50, dtype=np.int64),
    ])
    return t


def _apply(t, num, den):
    """mc_cast_units' arithmetic (x_scale_ticks in mc_ext.hip) in Python
    integers: int64 wrap-around product, C division (toward zero)."""
    def wrap(v):
        v &= (1 << 64) - 1
        return v - (1 << 64) if v >> 63 else v

    def cdiv(a, b):
        q = abs(a) // b
        return q if a >= 0 else -q

    out = []
    for v in t.tolist():
        if v == NAT:
            out.append(NAT)
            continue
        m = wrap(v * num)
        out.append(wrap(cdiv(wrap(m - (den - 1)), den)) if v < 0 else wrap(cdiv(m, den)))
    return np.array(out, dtype=np.int64)


@pytest.mark.parametrize("kind", ["m8", "M8"])
def test_conversion_factor_reproduces_numpy(kind):
    t = _ticks()
    with np.errstate(all="ignore"):
        for a in UNITS:
            for b in UNITS:
                if kind == "M8" and (a in "YM") != (b in "YM"):
                    continue  # calendar conversions: mc_cast_calendar (tests/test_x80.py)
                src, dst = np.dtype(f"{kind}[{a}]"), np.dtype(f"{kind}[{b}]")
                try:
                    want = t.view(src).astype(dst).view(np.int64)
                except OverflowError as e:  # numpy's factor overflows: the same error here
                    with pytest.raises(OverflowError) as ei:
                        _ops.time_cast_factor(src, dst)
                    assert str(ei.value) == str(e)
                    continue
                num, den = _ops.time_cast_factor(src, dst)
                got = _apply(t, num, den)
                if kind == "M8" and a in "YM" and a != b:
                    # numpy's calendar loop for years <-> months: linear except
                    # where the product overflows int64 (not the wrap-around)
                    ok = np.abs(t) < 2**58
                    assert np.array_equal(got[ok], want[ok]), (a, b)
                else:
                    assert np.array_equal(got, want), (a, b, num, den)


@pytest.mark.parametrize("a,b", [("5s", "2ms"), ("3D", "7h"), ("10us", "s"), ("2Y", "3M"), ("4W", "6D")])
def test_conversion_factor_multiples(a, b):
    t = _ticks()
    src, dst = np.dtype(f"m8[{a}]"), np.dtype(f"m8[{b}]")
    num, den = _ops.datetime_conversion_factor(src, dst)
    with np.errstate(all="ignore"):
        want = t.view(src).astype(dst).view(np.int64)
    assert np.array_equal(_apply(t, num, den), want)


def test_generic_units():
    assert _ops.time_cast_factor("m8", "m8[s]") == (1, 1)
    with pytest.raises(ValueError):
        _ops.datetime_conversion_factor("m8[s]", "m8")
    assert _ops.time_cast_factor("m8[s]", "M8[ms]") == (1, 1)  # cross-kind: ticks kept
    with pytest.raises(ValueError):  # the calendar path is mc_cast_calendar's
        _ops.time_cast_factor("M8[Y]", "M8[D]")
    assert _ops.calendar_cast("M8[Y]", "M8[3D]") == (0, 1, 3, 3)
    assert _ops.calendar_cast("M8[2h]", "M8[M]") == (4, 2, 1, 1)
    assert _ops.calendar_cast("M8[Y]", "M8[M]") is None  # linear (x12)
    assert _ops.calendar_cast("m8[Y]", "m8[D]") is None  # timedelta: linear
    assert _ops.calendar_cast("M8", "M8[Y]") is None  # generic
    with pytest.raises(OverflowError):  # numpy's factor check comes first
        _ops.calendar_cast("M8[Y]", "M8[as]")


def test_dtype_codes():
    assert _ops.dtype_code("<c8") == _native.MC_C8
    assert _ops.dtype_code(">c16") == _native.MC_C16 | _native.MC_BIG_ENDIAN
    assert _ops.dtype_code("<m8[ns]") == _native.MC_TD8
    assert _ops.dtype_code("<m8") == _native.MC_TD8
    assert _ops.dtype_code(">M8[D]") == _native.MC_DT8 | _native.MC_BIG_ENDIAN
    assert _ops.dtype_code("<f4") == 10
    with pytest.raises(NotImplementedError):
        _ops.dtype_code("S3")
    with pytest.raises(NotImplementedError):
        _ops.dtype_code("V8")
    if np.finfo(np.longdouble).nmant == 63:  # x87 longdouble (round 6)
        assert _ops.dtype_code("<f16") == _native.MC_F16L
        assert _ops.dtype_code(">c32") == _native.MC_C32 | _native.MC_BIG_ENDIAN


def test_header_codes_match():
    import os

    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                            "mcodec.h")).read()
    for name in ("MC_C8", "MC_C16", "MC_TD8", "MC_DT8"):
        assert f"{name} = {getattr(_native, name)}," in hdr
