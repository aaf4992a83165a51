"""Generate tests/golden/ext.npz and ext.json: the extended dtypes of the
arithmetic codecs -- complex64/complex128, timedelta64 and datetime64 -- on
Delta, FixedScaleOffset and AsType, plus the errors the reference raises for
the combinations numpy refuses.

Expected outputs come from the REAL reference (/root/reference/src/numcodecs:
delta.py:52-83, fixedscaleoffset.py:83-113, astype.py:46-58) imported through
oracle/refload.py in the build container; the arithmetic is numpy's
(complex loops per component, timedelta NaT propagation, datetime unit
casts).  Run here (the reference never travels to the GPU box; only these
data files do):

    python tests/golden/make_golden_ext.py

Fixtures are data (inputs and expected outputs), not reference source.
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

arrays: dict[str, np.ndarray] = {}
manifest: dict[str, list] = {}
NAT = np.iinfo(np.int64).min
I64MAX = np.iinfo(np.int64).max


def b(a) -> np.ndarray:
    a = np.asarray(a)
    return np.frombuffer(a.tobytes(order="A"), dtype=np.uint8).copy()


def add(family, meta, **arrs):
    cases = manifest.setdefault(family, [])
    i = len(cases)
    for k, v in arrs.items():
        arrays[f"{family}__{i}__{k}"] = b(v)
    cases.append(meta)


def unif(seed, n):
    """24-bit uniforms in [0, 1), exact"""
    return (inputs.words(seed, n) >> np.uint64(40)).astype(np.float64) * 2.0**-24


def ticks(seed, n, kind):
    """int64 ticks: 'walk' (small steps), 'wide' (raw words), with NaT and
    overflow placements"""
    w = inputs.words(seed, n)
    if kind == "walk":
        t = np.cumsum((w % np.uint64(2001)).astype(np.int64) - 1000) + 10**12
    else:
        t = w.view(np.int64).copy()
    return t


def complex_vals(seed, n, kind, ft):
    """complex test data: 'ramp' (every Delta add exact), 'noise' (rounding
    events), 'special' (NaN / inf / -0 / subnormal components)"""
    if kind == "ramp":
        re = -1000.0 + 0.125 * np.arange(n)
        im = 500.0 - 0.25 * np.arange(n)
    elif kind == "noise":
        re = 100.0 * unif(seed, n) - 50.0
        im = 1e3 * unif(seed + 1, n)
    else:
        re = 10.0 * unif(seed, n) - 5.0
        im = 10.0 * unif(seed + 1, n) - 5.0
        sp = np.array([np.nan, np.inf, -np.inf, -0.0, 0.0, 1e-310 if ft == np.float64 else 1e-40, 3.4e38])
        for j, v in enumerate(sp):
            re[(j * 97 + 3) % n] = v
            im[(j * 61 + 11) % n] = v
        re[n // 2] = np.nan
        im[n // 2 + 1] = -np.inf
    return re.astype(ft) + 1j * im.astype(ft)


def run(fn):
    """(result, None) or (None, (exception type name, isinstance TypeError/ValueError..., message))"""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            return fn(), None
        except Exception as e:  # the reference's error is the expected result
            base = next(c.__name__ for c in type(e).__mro__ if c.__module__ == "builtins")
            return None, [type(e).__name__, base, str(e)]


seed = 9000
# --------------------------------------------------------------------------
# Delta (delta.py:52-83)
# --------------------------------------------------------------------------
delta_cases = []
# timedelta64: NaT placements (first / mid / last), overflow into INT64_MIN
for dt in ("<m8[ns]", "<m8[s]", ">m8[ns]", "<m8"):
    for kind, n in (("walk", 17001), ("nat_first", 4099), ("nat_mid", 20001), ("nat_last", 4099),
                    ("overflow", 9), ("tiny", 3)):
        if dt != "<m8[ns]" and kind in ("nat_last", "overflow", "tiny"):
            continue
        delta_cases.append((dt, dt, kind, n))
for dt, at, kind, n in (("<m8[ns]", "<i8", "nat_mid", 9001), ("<m8[ns]", "<i4", "small", 9001),
                        ("<m8[ns]", "<i2", "small", 6001), ("<m8[ns]", "<i2", "walk", 101), ("<m8[us]", "<m8[ns]", "nat_mid", 6001),
                        ("<m8[ns]", "<m8[us]", "nat_mid", 6001), ("<m8[D]", "<f8", "walk", 4001),
                        ("<i8", "<m8[ns]", "nat_mid", 6001), ("<m8[ns]", ">m8[ns]", "nat_mid", 6001),
                        ("<m8[ms]", "<i8", "overflow", 9), ("<i4", "<m8[ns]", "walk", 4001),
                        ("<M8[D]", "<M8[D]", "nat_mid", 6001), ("<M8[ns]", "<M8[ns]", "walk", 6001),
                        ("<M8[s]", "<i8", "walk", 4001), ("<M8[ns]", "<m8[ns]", "nat_mid", 4001),
                        ("<m8[ns]", "<u8", "walk", 101), ("<M8[D]", ">M8[D]", "nat_first", 101)):
    delta_cases.append((dt, at, kind, n))
# complex: per-component differences / running sums
for dt in ("<c8", "<c16", ">c8", ">c16"):
    for kind, n in (("ramp", 20001), ("noise", 9001), ("special", 4099), ("ramp", 7)):
        if dt[0] == ">" and n > 20000:
            continue
        delta_cases.append((dt, dt, kind, n))
for dt, at, kind, n in (("<c16", "<c8", "ramp", 17001), ("<c8", "<c16", "noise", 9001),
                        ("<c8", "<f4", "noise", 6001), ("<f4", "<c8", "ramp", 6001),
                        ("<c8", "<i2", "ramp", 6001), ("<i2", "<c8", "intvals", 6001),
                        ("<c16", "<i4", "ramp", 6001), ("<f8", "<c16", "noise", 6001),
                        ("<c8", "<f8", "noise", 4001), ("<c16", "<f2", "ramp", 4001),
                        ("<i4", "<c8", "intvals", 4001), ("<c8", "|b1", "special", 1001),
                        ("|b1", "<c8", "bools", 1001), ("<c16", ">c8", "special", 4099)):
    delta_cases.append((dt, at, kind, n))

for dt, at, kind, n in delta_cases:
    seed += 1
    d = np.dtype(dt)
    if d.kind in "mM":
        t = ticks(seed, n, "wide" if kind == "overflow" else "walk")
        if kind == "small":
            t -= 10**12
            t[0] = 12
        if kind == "nat_first":
            t[0] = NAT
        elif kind == "nat_mid":
            t[n // 3] = NAT
            t[n // 3 + 1] = NAT
            t[2 * n // 3] = NAT
        elif kind == "nat_last":
            t[-1] = NAT
        elif kind == "overflow":
            t[:] = [I64MAX - 3, 1, 1, 1, 1, -5, 7, NAT + 1, 2][:n]
        elif kind == "tiny":
            t[:] = [1, 2, NAT][:n]
        x = t.view(np.dtype(d.str.replace(">", "<"))).astype(d)
    elif d.kind == "c":
        x = complex_vals(seed, n, kind, np.float32 if d.itemsize == 8 else np.float64).astype(d)
    elif d.kind == "b":
        x = (inputs.words(seed, n) % np.uint64(3)) == 0
    elif kind == "intvals":
        x = ((inputs.words(seed, n) % np.uint64(2001)).astype(np.int64) - 1000).astype(d)
    elif d.kind in "iu":
        x = (ticks(seed, n, "walk") - 10**12).astype(d)
        if kind == "nat_mid":
            x[n // 3] = NAT
    else:
        x = complex_vals(seed, n, kind, np.float64).real.astype(d)
    codec = nc.Delta(dtype=dt, astype=at)
    enc, enc_err = run(lambda: codec.encode(x))
    meta = {"dtype": dt, "astype": at, "kind": kind, "n": n}
    if enc_err:
        meta["encode_error"] = enc_err
        add("ext_delta", meta, input=x)
        continue
    assert enc.dtype == np.dtype(at)
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ext_delta", meta, input=x, encoded=enc)
    else:
        assert dec.dtype == d
        add("ext_delta", meta, input=x, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# FixedScaleOffset (fixedscaleoffset.py:83-113)
# --------------------------------------------------------------------------
fso_cases = [
    ("<c8", "<c8", 1, 10, "special"), ("<c8", "<i2", 1000, 10, "ramp"), ("<c16", "<c8", 1000.5, 1e3, "noise"),
    ("<c8", "<f4", 2, 1e2, "special"), ("<f8", "<c16", 1000, 7.0, "noise"), ("<c16", "<i4", 1000, 1e4, "special"),
    ("<c8", "<c16", 0.25, 3.0, "noise"), ("<c16", "<c16", 1 + 2j, 10 - 1j, "noise"),
    ("<c8", "<c8", 1 + 2j, 10 - 1j, "special"), ("<c16", "<c16", 3, 0.1 + 0.7j, "special"),
    (">c8", ">c8", 1, 10, "noise"), ("<c16", ">i2", 1000, 10, "ramp"), ("<i2", "<c8", 100, 4, "ramp"),
    ("<c8", "|b1", 1, 10, "special"), ("<c16", "<c16", 0, 0j, "noise"),
    ("<m8[ns]", "<m8[ns]", 1, 10, "ramp"), ("<m8[ns]", "<i8", 1, 10, "ramp"),
    ("<M8[ns]", "<M8[ns]", 1, 10, "ramp"), ("<m8[s]", "<f8", 0, 1.5, "ramp"),
]
for dt, at, off, sc, kind in fso_cases:
    seed += 1
    n = 3001
    d = np.dtype(dt)
    if d.kind == "c":
        x = (off if not isinstance(off, complex) else 0) + complex_vals(seed, n, kind,
                                                                         np.float32 if d.itemsize == 8 else np.float64)
        x = x.astype(d)
    elif d.kind in "mM":
        x = ticks(seed, n, "walk").view(np.dtype(d.str)).astype(d)
    else:
        x = (off + 5 * np.sin(np.arange(n) / 50.0)).astype(d) if d.kind == "f" else (
            (inputs.words(seed, n) % np.uint64(500)).astype(np.int64) + 100).astype(d)
    codec = nc.FixedScaleOffset(offset=off, scale=sc, dtype=dt, astype=at)
    meta = {"dtype": dt, "astype": at, "offset": [off.real, off.imag] if isinstance(off, complex) else off,
            "scale": [sc.real, sc.imag] if isinstance(sc, complex) else sc, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ext_fso", meta, input=x)
        continue
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ext_fso", meta, input=x, encoded=enc)
    else:
        add("ext_fso", meta, input=x, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# AsType (astype.py:46-58): encode_dtype, decode_dtype
# --------------------------------------------------------------------------
a_cases = [
    ("<c8", "<c16"), ("<c16", "<c8"), ("<f4", "<c8"), ("<c8", "<f8"), ("<i2", "<c8"), ("<c16", "<i4"),
    ("<c8", "|b1"), ("|b1", "<c8"), ("<c8", "<f2"), ("<f2", "<c8"), (">c8", "<c16"), ("<c16", ">c16"),
    ("<c16", "<u8"), ("<i8", "<c16"),
    ("<m8[ns]", "<i8"), ("<i8", "<m8[ns]"), ("<i2", "<m8[ns]"), ("<m8[ns]", "<u4"), ("<f8", "<m8[ns]"),
    ("<m8[ns]", "<f8"), ("<f2", "<m8[s]"), ("<m8[s]", "<f4"), ("|b1", "<m8[ns]"), ("<m8[ns]", "|b1"),
    ("<c8", "<m8[ns]"), ("<m8[ns]", "<c16"), ("<u8", "<m8[s]"),
    ("<m8[us]", "<m8[ns]"), ("<m8[ns]", "<m8[us]"), ("<m8[D]", "<m8[Y]"), ("<m8[Y]", "<m8[D]"),
    ("<m8[W]", "<m8[M]"), ("<m8[2ms]", "<m8[5s]"), ("<m8[ps]", "<m8[ns]"), ("<m8[s]", "<m8"),
    ("<M8[s]", "<M8[ns]"), ("<M8[ns]", "<M8[s]"), ("<M8[D]", "<M8[h]"), ("<M8[D]", "<M8[W]"),
    ("<M8[ns]", "<m8[ns]"), ("<m8[ns]", "<M8[ns]"), ("<M8[s]", "<m8[D]"), ("<M8[D]", "<i4"), ("<i8", "<M8[D]"),
    ("<M8[ns]", "<f8"), (">m8[ns]", "<m8[ns]"), ("<m8[ns]", ">m8[us]"), (">M8[s]", ">M8[ms]"),
    ("<M8[M]", "<M8[Y]"),
]
for et, dt in a_cases:
    seed += 1
    n = 1001
    d = np.dtype(dt)
    if d.kind in "mM":
        t = ticks(seed, n, "wide")
        t[:8] = [0, 1, -1, NAT, I64MAX, NAT + 1, 2**62, -(2**62)]
        t[8:200] = ticks(seed + 1, 192, "walk") - 10**12
        t[200:600] = ticks(seed + 2, 400, "walk") % 100000 - 50000
        x = t.view(np.dtype(d.str.replace(">", "<"))).astype(d)
    elif d.kind == "c":
        x = complex_vals(seed, n, "special", np.float32 if d.itemsize == 8 else np.float64).astype(d)
        x[:6] = [1.5 + 2j, -7.75 - 0.5j, 3e9 + 1j, -1e19 + 0j, 2.0**63 + 0j, 255.5 - 3j]
    elif d.kind == "f":
        x = (1e6 * (unif(seed, n) - 0.5)).astype(d)
        x[:8] = [0.5, -0.5, 1.5, -1.7, np.nan, np.inf, -np.inf, 1e19 if d.itemsize > 2 else 6e4]
    elif d.kind == "b":
        x = (inputs.words(seed, n) % np.uint64(2)) == 0
    else:
        x = inputs.words(seed, n).view(np.int64).astype(d)
    codec = nc.AsType(encode_dtype=et, decode_dtype=dt)
    meta = {"encode_dtype": et, "decode_dtype": dt, "n": n}
    enc, enc_err = run(lambda: codec.encode(x))
    if enc_err:
        meta["encode_error"] = enc_err
        add("ext_astype", meta, input=x)
        continue
    meta["encoded_dtype"] = enc.dtype.str
    dec, dec_err = run(lambda: codec.decode(enc))
    if dec_err:
        meta["decode_error"] = dec_err
        add("ext_astype", meta, input=x, encoded=enc)
    else:
        meta["decoded_dtype"] = dec.dtype.str
        add("ext_astype", meta, input=x, encoded=enc, decoded=dec)

np.savez_compressed(os.path.join(HERE, "ext.npz"), **arrays)
with open(os.path.join(HERE, "ext.json"), "w") as f:
    json.dump(manifest, f, indent=1, sort_keys=True)
print({k: len(v) for k, v in manifest.items()}, sum(a.nbytes for a in arrays.values()), "bytes")
for fam, cases in manifest.items():
    for c in cases:
        if "encode_error" in c or "decode_error" in c:
            print(fam, {k: v for k, v in c.items() if k not in ("n",)})
