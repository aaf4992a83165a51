"""Generate tests/golden/vectors.npz, vectors.json and fullsize.json.

Expected outputs come from the REAL reference: zarr-developers/numcodecs'
own hot-path sources under /root/reference/src/numcodecs, with its Cython
extensions compiled from those sources into oracle/_ref/ (oracle/build_ref.sh)
and imported through oracle/refload.py.  Run in the build container (the
reference never travels to the GPU box; only these data files do):

    make -C oracle && python tests/golden/make_golden.py

Fixtures are data (inputs and expected outputs), not reference source.
"""

from __future__ import annotations

import hashlib
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
    """raw bytes of an array/bytes as uint8"""
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8).copy()
    a = np.asarray(a)
    return np.frombuffer(a.tobytes(order="A"), dtype=np.uint8).copy()


def add(family, meta, **arrs):
    cases = manifest.setdefault(family, [])
    i = len(cases)
    for k, v in arrs.items():
        arrays[f"{family}__{i}__{k}"] = v
    cases.append(meta)


def rand_bytes(seed, n):
    return inputs.words(seed, (n + 7) // 8).view(np.uint8)[:n].copy()


# --------------------------------------------------------------------------
# Shuffle (shuffle.py, _shuffle.pyx)
# --------------------------------------------------------------------------
seed = 100
for es in (2, 3, 4, 5, 8, 16):
    for count in (1, 7, 1000, 4097, 4096 * 2 + 3, 16384):
        x = rand_bytes(seed, es * count)
        seed += 1
        enc = nc.Shuffle(es).encode(x)
        add("shuffle", {"elementsize": es, "nbytes": int(x.nbytes)}, input=x, encoded=b(enc))

# --------------------------------------------------------------------------
# BitRound (bitround.py) -- encoded integer patterns
# --------------------------------------------------------------------------
SPECIAL = {
    "float16": [0x0000, 0x8000, 0x7C00, 0xFC00, 0x7E00, 0x7C01, 0xFDFF, 0x0001, 0x03FF, 0x0400,
                0x7BFF, 0xFBFF, 0x3C00, 0xBC00, 0x3555, 0x7FFF, 0xFFFF, 0x07FF, 0x4001],
    "float32": [0x00000000, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00000, 0x7F800001, 0xFFBFFFFF,
                0x00000001, 0x007FFFFF, 0x00800000, 0x7F7FFFFF, 0xFF7FFFFF, 0x3F800000, 0xBF800000,
                0x7FFFFFFF, 0xFFFFFFFF, 0x3EAAAAAB, 0x00FFFFFF, 0x4B7FFFFF],
    "float64": [0x0, 0x8000000000000000, 0x7FF0000000000000, 0xFFF0000000000000, 0x7FF8000000000000,
                0x7FF0000000000001, 0x0000000000000001, 0x000FFFFFFFFFFFFF, 0x0010000000000000,
                0x7FEFFFFFFFFFFFFF, 0x3FF0000000000000, 0xBFF0000000000000, 0x7FFFFFFFFFFFFFFF,
                0xFFFFFFFFFFFFFFFF, 0x3FD5555555555555],
}
KEEP = {"float16": [0, 1, 3, 5, 9], "float32": [0, 1, 5, 10, 11, 16, 22],
        "float64": [0, 1, 10, 18, 23, 40, 51]}
for dt, ks in KEEP.items():
    idt = {"float16": np.uint16, "float32": np.uint32, "float64": np.uint64}[dt]
    special = np.array(SPECIAL[dt], dtype=np.uint64).astype(idt)
    rnd = inputs.words(200 + len(dt), 4093).astype(idt)  # all bit patterns, odd length
    x = np.concatenate([special, rnd]).view(dt)
    for k in ks:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            enc = nc.BitRound(k).encode(x.copy())
        add("bitround", {"dtype": np.dtype(dt).str, "keepbits": k}, input=b(x), encoded=b(enc))

# --------------------------------------------------------------------------
# FixedScaleOffset (fixedscaleoffset.py) -- encode and decode
# --------------------------------------------------------------------------
c4 = inputs.f32_c4(4, 4096)
edge32 = np.array([1000.0, 1000.0005, 999.9995, 1032.767, 1032.768, 967.232, 967.2315, 1040.4,
                   1e10, -1e10, np.inf, -np.inf, np.nan, 0.0, -0.0, 1000.0015, 1000.0025],
                  dtype=np.float32)
lin8 = np.linspace(1000, 1001, 1000, dtype="<f8")
nrm8 = (1000.0 + (inputs.words(301, 1000) >> np.uint64(11)).astype(np.float64) * 2.0**-53 - 0.5)
FSO_CASES = [
    (1000, 1000, "<f4", "<i2", np.concatenate([c4, edge32])),
    (1000.1, 1000.0, "<f4", "<i2", c4),
    (1000, 10, "<f8", "<i1", lin8),
    (1000, 10, "<f8", "<u1", lin8),
    (1000, 100, "<f8", "<i2", nrm8),
    (1000, 10**6, "<f8", "<i4", lin8),
    (1000, 10**12, "<f8", "<i8", lin8),
    (1000, 10**12, "<f8", "<f8", lin8),
    (1002.5, 10, "<f8", "<i2", np.linspace(1000, 1005, 10, dtype="<f8")),
    (1000, 0.5, "<f8", "<i2", np.linspace(1000, 1005, 10, dtype="<f8")),
    (0, 1, "<f4", "<u2", np.array([0.5, 1.5, 2.5, -1.0, 65535.4, 70000.0, -0.4], dtype="<f4")),
    (1000, 1000, "<f8", "<u4", np.array([1000.5, 999.0, 5e6, -3.0, 1e20], dtype="<f8")),
    (1000, 1000, "<f8", "<u8", np.array([1000.5, 999.0, 5e12, -3.0, 1e20, 2e16], dtype="<f8")),
    (100, 10, "<i4", "<i4", np.arange(-50, 50, dtype="<i4") * 1000),
    (1.5, 2, "<i4", "<f8", np.arange(-50, 50, dtype="<i4")),
    (10, 3, "<i2", "<i2", np.arange(-20000, 20000, 997, dtype="<i2")),
    (0.5, 4, "<f2", "<i2", np.array([0.1, 0.5, 1.0, 1.3, 100.7, -3.2, 65000.0], dtype="<f2")),
    (1000, 1000, "<f4", "<f4", c4[:512]),
    (1000, 1000, "<f4", "<f2", c4[:512]),
]
for off, sc, dt, at, x in FSO_CASES:
    codec = nc.FixedScaleOffset(offset=off, scale=sc, dtype=dt, astype=at)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        enc = codec.encode(x)
        dec = codec.decode(enc)
    add("fso", {"offset": off, "scale": sc, "dtype": dt, "astype": at},
        input=b(x), encoded=b(enc), decoded=b(dec))

# --------------------------------------------------------------------------
# Quantize (quantize.py)
# --------------------------------------------------------------------------
qx8 = np.concatenate([
    np.linspace(100, 200, 257, dtype="<f8"),
    (inputs.words(401, 512) >> np.uint64(11)).astype(np.float64) * 2.0**-53 * 8 - 4,
    np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e300, -1e-300, 5e-324, 65504.0, 65520.0], dtype="<f8"),
])
Q_CASES = [(d, "<f8", at) for d in (-1, 0, 1, 2, 3, 5, 7, 12) for at in ("<f2", "<f4", "<f8")]
Q_CASES += [(d, "<f4", at) for d in (0, 1, 3, 6) for at in ("<f2", "<f4", "<f8")]
Q_CASES += [(d, "<f2", at) for d in (0, 1, 2) for at in ("<f2", "<f4")]
for d, dt, at in Q_CASES:
    x = qx8.astype(dt)
    codec = nc.Quantize(digits=d, dtype=dt, astype=at)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        enc = codec.encode(x)
        dec = codec.decode(enc)
    add("quantize", {"digits": d, "dtype": dt, "astype": at},
        input=b(x), encoded=b(enc), decoded=b(dec))

# --------------------------------------------------------------------------
# Delta (delta.py)
# --------------------------------------------------------------------------
w = inputs.words(501, 5000)
D_CASES = [
    ("<i2", "<i2", (w % np.uint64(65536)).astype(np.uint16).view("<i2")),
    ("<i2", "<i1", np.arange(100, 120, 2, dtype="<i2")),
    ("|b1", "|b1", (w % np.uint64(2)).astype(bool)),
    ("|u1", "|u1", (w % np.uint64(256)).astype(np.uint8)),
    ("|i1", "|i1", (w % np.uint64(256)).astype(np.uint8).view("i1")),
    ("<u2", "<u2", (w % np.uint64(65536)).astype("<u2")),
    ("<i4", "<i4", (w % np.uint64(2**32)).astype(np.uint32).view("<i4")),
    ("<i4", "<i2", np.cumsum((w % np.uint64(100)).astype("<i4"))),
    ("<i8", "<i4", np.arange(10, 20, 1, dtype="<i8")),
    ("<i8", "<i8", w.view("<i8")),
    ("<u8", "<u8", w.astype("<u8")),
    ("<u4", "<u4", (w >> np.uint64(32)).astype("<u4")),
    ("<f4", "<f4", inputs.f32_c4(502, 5000)),
    ("<f8", "<f8", 1000.0 + (w >> np.uint64(11)).astype(np.float64) * 2.0**-53),
    ("<f2", "<f2", (inputs.f32_c4(503, 3000) - 1000.0).astype("<f2")),
    ("<f8", "<f4", np.linspace(0, 1, 1000, dtype="<f8")),
    ("<f4", "<f4", np.linspace(1000, 1001, 1000, dtype="<f4")),
]
for dt, at, x in D_CASES:
    codec = nc.Delta(dtype=dt, astype=at)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        enc = codec.encode(x)
        dec = codec.decode(enc)
    add("delta", {"dtype": dt, "astype": at}, input=b(x), encoded=b(enc), decoded=b(dec))

# --------------------------------------------------------------------------
# Fletcher32 (fletcher32.pyx)
# --------------------------------------------------------------------------
F_CASES = [(n, "rand") for n in (1, 2, 3, 5, 15, 16, 17, 31, 719, 720, 721, 1440, 1441, 4096,
                                 65537, (1 << 20) + 3)]
F_CASES += [(n, "ff") for n in (2, 720, 721, 4096, 65537)] + [(1024, "zero"), (7, "zero")]
for n, kind in F_CASES:
    if kind == "rand":
        x = rand_bytes(600 + n % 1000, n)
    elif kind == "ff":
        x = np.full(n, 0xFF, dtype=np.uint8)
    else:
        x = np.zeros(n, dtype=np.uint8)
    enc = nc.Fletcher32().encode(x)
    add("fletcher32", {"nbytes": n, "kind": kind, "checksum": int.from_bytes(enc[-4:], "little")},
        input=x)

np.savez_compressed(os.path.join(HERE, "vectors.npz"), **arrays)
with open(os.path.join(HERE, "vectors.json"), "w") as f:
    json.dump(manifest, f, indent=1, sort_keys=True)

# --------------------------------------------------------------------------
# full-size configurations: SHA-256 of inputs and reference outputs
# --------------------------------------------------------------------------
def sha(a) -> str:
    return hashlib.sha256(b(a).tobytes() if not isinstance(a, bytes) else a).hexdigest()


full = {}
x1 = inputs.f32_wide(1, inputs.MiB // 4)
full["C1"] = {"input": sha(x1), "shuffle4": sha(nc.Shuffle(4).encode(x1))}
x2 = inputs.f32_wide(2, 256 * inputs.MiB // 4)
full["C2_f32"] = {"input": sha(x2), "shuffle4": sha(nc.Shuffle(4).encode(x2))}
full["C3"] = {"bitround10_shuffle4": sha(nc.Shuffle(4).encode(nc.BitRound(10).encode(x2)))}
del x2
x3 = inputs.f64_wide(3, 256 * inputs.MiB // 8)
full["C2_f64"] = {"input": sha(x3), "shuffle8": sha(nc.Shuffle(8).encode(x3))}
del x3
x4 = inputs.f32_c4(4, 256 * inputs.MiB // 4)
fso = nc.FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
e1 = fso.encode(x4)
e2 = nc.Delta(dtype="<i2").encode(e1)
e3 = nc.Shuffle(2).encode(e2)
d3 = fso.decode(nc.Delta(dtype="<i2").decode(nc.Shuffle(2).decode(e3)))
full["C4"] = {"input": sha(x4), "fso": sha(e1), "delta": sha(e2), "shuffle2": sha(e3), "decoded": sha(d3)}
del x4, e1, e2, e3, d3
c5 = {}
for c in (0, 1, 17, 4095, 8191):
    xc = inputs.c5_chunk_bytes_formula(c, inputs.MiB)
    enc = nc.Fletcher32().encode(nc.Shuffle(4).encode(xc))
    c5[str(c)] = {"input": sha(xc), "encoded": sha(enc), "checksum": int.from_bytes(enc[-4:], "little")}
full["C5"] = c5
with open(os.path.join(HERE, "fullsize.json"), "w") as f:
    json.dump(full, f, indent=1, sort_keys=True)
print("cases:", {k: len(v) for k, v in manifest.items()}, "arrays:", len(arrays))
