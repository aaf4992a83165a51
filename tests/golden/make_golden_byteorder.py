"""Generate tests/golden/byteorder.npz and byteorder.json: non-native
(big-endian) byte-order cases of Delta, FixedScaleOffset, Quantize and AsType.

Expected outputs come from the REAL reference (/root/reference/src/numcodecs:
delta.py:52-83, fixedscaleoffset.py:83-113, quantize.py:60-82,
astype.py:46-58) imported through oracle/refload.py in the build container;
the arithmetic is numpy's, which computes big-endian arrays in native
registers and stores them byte-swapped.  Run here (the reference never
travels to the GPU box; only these data files do):

    python tests/golden/make_golden_byteorder.py

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
from oracle import refload  # noqa: E402

nc = refload.load()

arrays: dict[str, np.ndarray] = {}
manifest: dict[str, list] = {}


def b(a) -> np.ndarray:
    a = np.asarray(a)
    return np.frombuffer(a.tobytes(order="A"), dtype=np.uint8).copy()


def add(family, meta, **arrs):
    cases = manifest.setdefault(family, [])
    i = len(cases)
    for k, v in arrs.items():
        arrays[f"{family}__{i}__{k}"] = b(v)
    cases.append(meta)


def ramp(n, step=0.125, start=-1000.0):
    """exact dyadic ramp (every Delta add is exact)"""
    return start + step * np.arange(n, dtype=np.float64)


def tri_noise(seed, n, amp=10.0, noise=0.5):
    """a dyadic triangle wave plus 24-bit uniforms: rounding events in f4/f2"""
    w = inputs.words(seed, n)
    u = (w >> np.uint64(40)).astype(np.float64) * 2.0**-24
    i = np.arange(n, dtype=np.int64) % 4096
    tri = np.abs(i.astype(np.float64) / 2048.0 - 1.0)
    return amp * tri + noise * (u - 0.5)


def ints(seed, n, dt):
    dt = np.dtype(dt)
    w = inputs.words(seed, n)
    return w.view(np.int64).astype(dt.newbyteorder("="), casting="unsafe")


seed = 7000
# --------------------------------------------------------------------------
# Delta (delta.py:52-83)
# --------------------------------------------------------------------------
delta_cases = []
for dt, at in (("f4", "f4"), ("f8", "f8"), ("f2", "f2")):
    for bo_d, bo_a in ((">", ">"), (">", "<"), ("<", ">")):
        for kind, n in (("ramp", 17001), ("tri", 17001), ("wide", 4097), ("tiny", 5)):
            if dt == "f2" and kind == "wide":
                continue
            if (bo_d, bo_a) != (">", ">") and kind in ("wide", "tiny"):
                continue
            delta_cases.append((bo_d + dt, bo_a + at, kind, n))
for dt, at, kind, n in ((">f8", ">f4", "ramp", 9001), (">f4", ">i2", "intvals", 17001),
                        (">f8", ">i4", "intvals", 6001), (">f4", "<f8", "ramp", 6001)):
    delta_cases.append((dt, at, kind, n))
for t in ("i2", "i4", "i8", "u2", "u4", "u8"):
    delta_cases.append((">" + t, ">" + t, "int", 17001))
    delta_cases.append((">" + t, ">" + t, "int", 7))
for dt, at in ((">i2", "<i2"), ("<i2", ">i2"), (">i4", ">i2"), (">i8", ">i4"), (">u2", ">i2"), (">i4", "<i8")):
    delta_cases.append((dt, at, "int_small", 9001))

for dt, at, kind, n in delta_cases:
    seed += 1
    d = np.dtype(dt)
    if kind == "ramp":
        x = ramp(n)
    elif kind == "tri":
        x = tri_noise(seed, n) if d.kind == "f" and d.itemsize < 8 else tri_noise(seed, n) * 1.0001
    elif kind == "wide":
        x = inputs.f32_wide(seed, n).astype(np.float64) if d.itemsize == 4 else inputs.f64_wide(seed, n)
    elif kind == "tiny":
        x = np.array([1.5, -2.25, 1e30 if d.itemsize > 2 else 1000.0, -0.0, 3.0])[:n]
    elif kind == "intvals":
        x = (inputs.words(seed, n) % np.uint64(2001)).astype(np.float64) - 1000.0
    elif kind == "int":
        x = ints(seed, n, d)
    else:  # int_small: values whose first element fits any astype here
        x = (inputs.words(seed, n) % np.uint64(6001)).astype(np.int64) - 10000
        x[0] = 17
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xa = np.asarray(x).astype(d)
        codec = nc.Delta(dtype=dt, astype=at)
        enc = codec.encode(xa)
        dec = codec.decode(enc)
    assert enc.dtype == np.dtype(at) and dec.dtype == d
    add("bo_delta", {"dtype": dt, "astype": at, "kind": kind, "n": n}, input=xa, encoded=enc, decoded=dec)

# --------------------------------------------------------------------------
# FixedScaleOffset (fixedscaleoffset.py:83-113)
# --------------------------------------------------------------------------
fso_cases = [
    (">f8", ">i2", 1000, 10, 17001), (">f4", ">i2", 1000, 1e3, 17001), (">f4", "<i2", 1000, 1e3, 6001),
    ("<f4", ">i2", 1000, 1e3, 6001), (">f8", ">i4", 1000.5, 1e4, 6001), (">f8", ">u2", 1000, 10, 6001),
    (">f8", ">f8", 1000, 7.0, 6001), (">i4", ">i2", 1000, 2, 6001), (">f8", ">i8", 0.25, 1e6, 6001),
    (">f2", ">i2", 100, 4.0, 6001), (">f4", ">u1", 1000, 10, 6001), ("<f8", ">i4", 1000, 1e4, 6001),
]
for dt, at, off, sc, n in fso_cases:
    seed += 1
    d = np.dtype(dt)
    x = off + tri_noise(seed, n, amp=20.0 if d.itemsize > 2 else 5.0, noise=2.0)
    if d.kind == "i":
        x = np.rint(x)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xa = x.astype(d)
        codec = nc.FixedScaleOffset(offset=off, scale=sc, dtype=dt, astype=at)
        enc = codec.encode(xa)
        dec = codec.decode(enc)
    add("bo_fso", {"dtype": dt, "astype": at, "offset": off, "scale": sc, "n": n}, input=xa, encoded=enc,
        decoded=dec)

# --------------------------------------------------------------------------
# Quantize (quantize.py:60-82)
# --------------------------------------------------------------------------
q_cases = [(">f8", ">f4", 3), (">f4", ">f4", 2), (">f8", ">f2", 1), (">f4", "<f4", 3), ("<f8", ">f2", 2),
           (">f2", ">f2", 1), (">f8", ">f8", 5), ("<f4", ">f4", 4)]
for dt, at, digits in q_cases:
    seed += 1
    n = 6001
    x = 100.0 * tri_noise(seed, n, amp=3.0, noise=1.0) - 150.0
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xa = x.astype(dt)
        codec = nc.Quantize(digits=digits, dtype=dt, astype=at)
        enc = codec.encode(xa)
        dec = codec.decode(enc)
    add("bo_quantize", {"dtype": dt, "astype": at, "digits": digits, "n": n}, input=xa, encoded=enc,
        decoded=dec)

# --------------------------------------------------------------------------
# AsType (astype.py:46-58): encode_dtype, decode_dtype
# --------------------------------------------------------------------------
a_cases = [(">f4", ">f8"), ("<f4", ">f8"), (">f8", "<f4"), (">i2", ">i4"), (">u2", "<f8"), (">f4", "<f4"),
           (">i8", ">f8"), (">f2", ">f4"), (">i4", ">f4"), ("<i2", ">i2"), (">u4", ">i8")]
for et, dt in a_cases:
    seed += 1
    n = 6001
    d = np.dtype(dt)
    x = 300.0 * tri_noise(seed, n, amp=3.0, noise=1.0) - 450.0
    if d.kind in "iu":
        x = np.rint(np.abs(x) if d.kind == "u" else x)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xa = x.astype(d)
        codec = nc.AsType(encode_dtype=et, decode_dtype=dt)
        enc = codec.encode(xa)
        dec = codec.decode(enc)
    add("bo_astype", {"encode_dtype": et, "decode_dtype": dt, "n": n}, input=xa, encoded=enc, decoded=dec)

np.savez_compressed(os.path.join(HERE, "byteorder.npz"), **arrays)
with open(os.path.join(HERE, "byteorder.json"), "w") as f:
    json.dump(manifest, f, indent=1, sort_keys=True)
print({k: len(v) for k, v in manifest.items()}, sum(a.nbytes for a in arrays.values()), "bytes")
