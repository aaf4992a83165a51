"""Generate tests/golden/ld.npz and ld.json: the inputs the reference
computes that rounds 1-5 refused --

  * longdouble / clongdouble ('<f16' / '<c32', x87 80-bit extended on x86-64)
    on Delta, Quantize, FixedScaleOffset and AsType, with the specials x87
    distinguishes (+-0, infinities, quiet and signalling NaNs with payloads,
    denormals, pseudo-denormals, unnormals, pseudo-NaNs, the extremes);
  * datetime64 Delta with a unit change (the first element cast as a
    datetime, the differences as timedeltas) and the calendar datetime64
    AsType casts (years / months <-> the linear units);
  * the errors numpy raises for string / bytes / void dtypes on Delta and
    FixedScaleOffset.

Expected outputs come from the REAL reference (/root/reference/src/numcodecs:
delta.py:52-83, quantize.py:60-82, fixedscaleoffset.py:83-113,
astype.py:46-58) imported through oracle/refload.py in the build container
(never on the GPU box; only these data files travel):

    python tests/golden/make_golden_ld.py

numpy leaves the 6 padding bytes of a computed longdouble as whatever the
output buffer held, so the tests compare the 10 value bytes of each
longdouble (tests/helpers.py::ld_value_view).  Fixtures are data (inputs and
expected outputs), not reference source.
"""

from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import inputs  # noqa: E402

warnings.simplefilter("ignore", RuntimeWarning)
from oracle import refload  # noqa: E402

nc = refload.load()

assert np.finfo(np.longdouble).nmant == 63, "x87 longdouble expected"

arrays: dict[str, np.ndarray] = {}
manifest: dict[str, list] = {}
NAT = np.iinfo(np.int64).min


def b(a) -> np.ndarray:
    a = np.asarray(a)
    return np.frombuffer(a.tobytes(order="A"), dtype=np.uint8).copy()


def add(family, meta, **arrs):
    cases = manifest.setdefault(family, [])
    i = len(cases)
    for k, v in arrs.items():
        arrays[f"{family}__{i}__{k}"] = b(v)
    cases.append(meta)


def run(fn):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            return fn(), None
        except Exception as e:  # the reference's error is the expected result
            base = next(c.__name__ for c in type(e).__mro__ if c.__module__ == "builtins")
            return None, [type(e).__name__, base, str(e)]


def unif(seed, n):
    return (inputs.words(seed, n) >> np.uint64(40)).astype(np.float64) * 2.0**-24


def ld_bits(m, se):
    m = np.asarray(m, dtype=np.uint64).reshape(-1)
    se = np.broadcast_to(np.asarray(se, dtype=np.uint16), m.shape)
    out = np.zeros((m.size, 16), np.uint8)
    out[:, :8] = m.view(np.uint8).reshape(-1, 8)
    out[:, 8:10] = np.ascontiguousarray(se).view(np.uint8).reshape(-1, 2)
    return out.reshape(-1).view(np.longdouble)


J, Q = 1 << 63, 1 << 62
LD_SPECIALS = ld_bits(
    [0, 0, J, J, J | Q, J | Q | 12345, J | 777, J | Q | 5, 1, (1 << 62) + 3, J | 9, (1 << 62), 5, (1 << 64) - 1,
     (1 << 64) - 1, J, J, J | 1],
    [0, 0x8000, 0x7fff, 0xffff, 0xffff, 0x7fff, 0x7fff, 0xffff, 0, 0x8000, 0, 0x3fff, 0x7fff, 0x7ffe, 0xfffe, 1,
     0x3fff, 0xbffe])


def ld_vals(seed, n, kind):
    """longdouble data: 'ramp' (exact sums), 'noise' (rounding on every add),
    'special' (noise with every x87 special class planted), 'smallint'"""
    if kind == "ramp":
        x = np.arange(n, dtype=np.longdouble) * np.longdouble(0.125) - 1000
    elif kind == "smallint":
        x = ((inputs.words(seed, n) % np.uint64(2001)).astype(np.int64) - 1000).astype(np.longdouble)
    else:
        w = inputs.words(seed, n)
        # full 64-bit significands, exponents over +-40 around 1
        x = ld_bits(w | np.uint64(J), ((inputs.words(seed + 7, n) % np.uint64(81)).astype(np.uint16) + 16383 - 40)
                    | ((w & np.uint64(1)).astype(np.uint16) << np.uint16(15)))
        if kind == "special":
            for j, v in enumerate(LD_SPECIALS):
                x[(j * 97 + 3) % n] = v
    return x


seed = 61000

# --------------------------------------------------------------------------
# Delta (delta.py:52-83)
# --------------------------------------------------------------------------
delta_cases = [
    ("<f16", "<f16", "ramp", 9001), ("<f16", "<f16", "noise", 6001), ("<f16", "<f16", "special", 4099),
    ("<f16", "<f16", "ramp", 5), (">f16", ">f16", "noise", 3001), ("<f16", ">f16", "special", 2001),
    ("<f16", "<f8", "noise", 4001), ("<f8", "<f16", "noise", 4001), ("<f4", "<f16", "noise", 4001),
    ("<f16", "<f4", "special", 3001), ("<f16", "<f2", "ramp", 3001), ("<f2", "<f16", "ramp", 2001),
    ("<i4", "<f16", "smallint", 4001), ("<f16", "<i2", "smallint", 4001), ("<i8", "<f16", "smallint", 2001),
    ("<f16", "<i8", "special", 2001), ("<u2", "<f16", "smallint", 2001), ("|b1", "<f16", "bools", 1001),
    ("<f16", "|b1", "special", 1001), ("<c32", "<c32", "noise", 3001), ("<c32", "<c32", "special", 2001),
    ("<c8", "<c32", "noise", 2001), ("<c32", "<c16", "noise", 2001), ("<f16", "<c32", "noise", 2001),
    ("<c32", "<f16", "noise", 2001), ("<c16", "<f16", "noise", 2001), (">c32", "<c32", "noise", 1001),
    ("<m8[s]", "<f16", "ticks", 1001),
    # datetime64 with a unit change (delta.py:63 the datetime, :66 the timedeltas)
    ("<M8[D]", "<m8[s]", "dates", 4001), ("<M8[s]", "<M8[ms]", "dates", 4001), ("<M8[D]", "<M8[Y]", "dates", 2001),
    ("<M8[s]", "<m8[D]", "dates", 2001), ("<M8[M]", "<M8[D]", "dates", 2001), (">M8[s]", "<M8[ms]", "dates", 2001),
    ("<m8[D]", "<M8[s]", "ticks", 2001), ("<M8[h]", "<M8[M]", "dates", 2001), ("<M8[ms]", ">m8[us]", "dates", 2001),
    ("<M8[Y]", "<M8[D]", "dates", 1001), ("<M8[3D]", "<M8[W]", "dates", 1001),
    # numpy refuses these (the reference raises from np.diff / np.cumsum)
    ("|S3", "|S3", "bytes", 9), ("<U2", "<U2", "str", 9), ("|V4", "|V4", "void", 9), ("<f4", "|S4", "noise", 9),
]
for dt, at, kind, n in delta_cases:
    seed += 1
    d = np.dtype(dt)
    if kind in ("ticks", "dates"):
        t = np.cumsum((inputs.words(seed, n) % np.uint64(2001)).astype(np.int64) - 1000)
        if kind == "dates":
            t += {"Y": 30, "M": 360, "W": 1500, "D": 11000}.get(np.datetime_data(d)[0], 10**9)
        t[n // 3] = NAT
        t[n // 2] = NAT
        x = t.view(np.dtype(d.str.replace(">", "<"))).astype(d)
    elif kind == "bytes":
        x = np.array([b"ab", b"c", b"", b"xyz"] * 2 + [b"q"], dtype=d)
    elif kind == "str":
        x = np.array(["ab", "c", "", "x"] * 2 + ["q"], dtype=d)
    elif kind == "void":
        x = np.frombuffer(inputs.words(seed, n).tobytes()[: 4 * n], dtype=d).copy()
    elif kind == "bools":
        x = (inputs.words(seed, n) % np.uint64(3)) == 0
    elif d.kind == "c":
        re, im = ld_vals(seed, n, kind), ld_vals(seed + 1, n, "ramp" if kind == "special" else kind)
        if d.itemsize < 32:  # a complex64/128 input: narrow components
            ct = np.float32 if d.itemsize == 8 else np.float64
            x = (re.astype(ct) + 1j * im.astype(ct)).astype(d)
        else:
            x = np.empty(n, d)
            x.real, x.imag = re, im
    elif d.kind in "iub":
        x = ld_vals(seed, n, "smallint").astype(d)
    else:
        x = ld_vals(seed, n, kind)
        if d.itemsize < 16:
            x = x.astype(d)
        x = x.astype(d)
    codec = nc.Delta(dtype=dt, astype=at)
    meta = {"dtype": dt, "astype": at, "kind": kind, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ld_delta", meta, input=x)
        continue
    assert enc.dtype == np.dtype(at)
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ld_delta", meta, input=x, encoded=enc)
    else:
        assert dec.dtype == d
        add("ld_delta", meta, input=x, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# Quantize (quantize.py:60-82)
# --------------------------------------------------------------------------
for dt, at, digits, kind in (("<f16", "<f16", 3, "noise"), ("<f16", "<f16", 1, "special"), ("<f16", "<f8", 5, "noise"),
                             ("<f16", "<f4", 2, "special"), ("<f16", "<f2", 1, "noise"), ("<f8", "<f16", 4, "noise"),
                             ("<f4", "<f16", 2, "noise"), (">f16", ">f16", 3, "noise"), ("<f16", "<f16", 30, "noise"),
                             ("<f16", "<f16", 0, "ramp")):
    seed += 1
    n = 3001
    x = ld_vals(seed, n, kind) * np.longdouble(37.5)
    x = x.astype(dt)
    codec = nc.Quantize(digits=digits, dtype=dt, astype=at)
    meta = {"dtype": dt, "astype": at, "digits": digits, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ld_quantize", meta, input=x)
        continue
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ld_quantize", meta, input=x, encoded=enc)
    else:
        add("ld_quantize", meta, input=x, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# FixedScaleOffset (fixedscaleoffset.py:83-113)
# --------------------------------------------------------------------------
BIG = 2**60 + 1  # a Python int only a longdouble holds exactly
for dt, at, off, sc, kind in (
        ("<f16", "<i2", 1000, 10, "ramp"), ("<f16", "<f16", 1000.5, 1e3, "noise"), ("<f16", "<f16", 1, 10, "special"),
        ("<f8", "<f16", 1000, 7.0, "noise"), ("<i4", "<f16", 100, 4, "smallint"), ("<f16", "<u1", 3, 0.5, "ramp"),
        ("<f16", "<i8", BIG, 3, "noise"), ("<f16", "<f16", BIG, 1, "ramp"), (">f16", ">i4", 2, 1e2, "noise"),
        ("<f16", "<f4", 2, 1e2, "special"), ("<c32", "<c32", 1, 10, "noise"), ("<c32", "<c32", 1 + 2j, 10 - 1j, "noise"),
        ("<c32", "<c32", 3, 0.1 + 0.7j, "special"), ("<f16", "<c32", 1000, 7.0, "noise"), ("<c32", "<i2", 1000, 10, "ramp"),
        ("<c16", "<c32", 0.25, 3.0, "noise"), ("<f16", "|b1", 1, 10, "special"), ("|S3", "|S3", 1, 10, "bytes"),
        ("<U2", "<i2", 1, 10, "str")):
    seed += 1
    n = 2001
    d = np.dtype(dt)
    if kind == "bytes":
        x = np.array([b"ab", b"c"] * 4, dtype=d)
    elif kind == "str":
        x = np.array(["ab", "c"] * 4, dtype=d)
    elif d.kind == "c":
        x = np.empty(n, d)
        re = ld_vals(seed, n, kind)
        im = ld_vals(seed + 1, n, "ramp" if kind == "special" else kind)
        if d.itemsize < 32:
            ct = np.float32 if d.itemsize == 8 else np.float64
            re, im = re.astype(ct), im.astype(ct)
        x.real, x.imag = re, im
    elif d.kind in "iu":
        x = ld_vals(seed, n, "smallint").astype(d) + 1000
    else:
        x = (ld_vals(seed, n, kind) + off).astype(d)
    codec = nc.FixedScaleOffset(offset=off, scale=sc, dtype=dt, astype=at)
    meta = {"dtype": dt, "astype": at, "offset": [off.real, off.imag] if isinstance(off, complex) else off,
            "scale": [sc.real, sc.imag] if isinstance(sc, complex) else sc, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ld_fso", meta, input=x)
        continue
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ld_fso", meta, input=x, encoded=enc)
    else:
        add("ld_fso", meta, input=x, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# AsType (astype.py:46-58): encode_dtype, decode_dtype
# --------------------------------------------------------------------------
REAL = ["|b1", "|i1", "<i2", "<i4", "<i8", "|u1", "<u2", "<u4", "<u8", "<f2", "<f4", "<f8"]
a_cases = [("<f16", t) for t in REAL] + [(t, "<f16") for t in REAL] + [
    ("<f16", "<f16"), (">f16", "<f16"), ("<f16", ">f16"), ("<c32", "<c8"), ("<c16", "<c32"), ("<c32", "<f16"),
    ("<f16", "<c32"), ("<c32", "<f8"), ("<f8", "<c32"), ("<c32", "|b1"), ("<c32", ">c32"), ("<m8[ns]", "<f16"),
    ("<f16", "<m8[ns]"), ("<f16", "<M8[s]"),
    # calendar datetime64 casts (numpy's datetimestruct path)
    ("<M8[Y]", "<M8[D]"), ("<M8[D]", "<M8[Y]"), ("<M8[M]", "<M8[s]"), ("<M8[ns]", "<M8[M]"), ("<M8[2Y]", "<M8[3D]"),
    ("<M8[W]", "<M8[M]"), ("<M8[Y]", ">M8[h]"), ("<M8[M]", "<M8[W]"), ("<M8[5M]", "<M8[us]"), ("<M8[ms]", "<M8[Y]"),
]
for et, dt in a_cases:
    seed += 1
    n = 1001
    d = np.dtype(dt)
    if d.kind == "M":
        unit = np.datetime_data(d)[0]
        span = {"Y": 20000, "M": 240000, "W": 10**6, "D": 7 * 10**6}.get(unit, 2**50)
        t = (inputs.words(seed, n) % np.uint64(2 * span)).astype(np.int64) - span
        t[:6] = [0, -1, 1, NAT, 11, -13]
        x = t.view(np.dtype(d.str.replace(">", "<"))).astype(d)
    elif d.kind == "m":
        x = ((inputs.words(seed, n) % np.uint64(10**12)).astype(np.int64) - 5 * 10**11).view(d)
        x[3] = np.timedelta64("NaT")
    elif d.kind == "c":
        x = np.empty(n, d)
        re, im = ld_vals(seed, n, "special"), ld_vals(seed + 1, n, "noise")
        if d.itemsize < 32:
            ct = np.float32 if d.itemsize == 8 else np.float64
            re, im = re.astype(ct), im.astype(ct)
        x.real, x.imag = re, im
    elif d.kind == "f" and d.itemsize == 16:
        x = ld_vals(seed, n, "special") * np.longdouble(1e3)
        x[-40:] = np.array([2.0**e for e in range(-20, 20)], np.longdouble) + np.longdouble(0.5)
        x[-80:-40] = -np.array([2.0**e for e in range(-20, 20)], np.longdouble) - np.longdouble(0.5)
        x[-120:-80] = np.array([2.0**e for e in (7, 8, 15, 16, 31, 32, 63, 64)] * 5, np.longdouble)
        x = x.astype(d)
    elif d.kind == "f":
        x = (1e6 * (unif(seed, n) - 0.5)).astype(d)
        bits = x.view(f"u{d.itemsize}")
        x[:8] = [0.5, -0.5, 1.5, -1.7, np.nan, np.inf, -np.inf, -0.0]
        bits[8::13] |= np.array((1 << (8 * d.itemsize - 1)) - 1, f"u{d.itemsize}") ^ np.array(
            1 << {2: 9, 4: 22, 8: 51}[d.itemsize], f"u{d.itemsize}")  # NaNs with payloads, some signalling
    elif d.kind == "b":
        x = (inputs.words(seed, n) % np.uint64(2)) == 0
    else:
        x = inputs.words(seed, n).view(np.int64).astype(d)
    codec = nc.AsType(encode_dtype=et, decode_dtype=dt)
    meta = {"encode_dtype": et, "decode_dtype": dt, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ld_astype", meta, input=x)
        continue
    meta["encoded_dtype"] = enc.dtype.str
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ld_astype", meta, input=x, encoded=enc)
    else:
        meta["decoded_dtype"] = dec.dtype.str
        add("ld_astype", meta, input=x, encoded=enc, decoded=dec)

np.savez_compressed(os.path.join(HERE, "ld.npz"), **arrays)
with open(os.path.join(HERE, "ld.json"), "w") as f:
    json.dump(manifest, f, indent=1, sort_keys=True)
print({k: len(v) for k, v in manifest.items()}, sum(a.nbytes for a in arrays.values()), "bytes")
for fam, cases in manifest.items():
    for c in cases:
        if "encode_error" in c or "decode_error" in c:
            print(fam, {k: v for k, v in c.items() if k not in ("n",)})
