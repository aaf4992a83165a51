"""CPU: the oracle restatement (oracle/nporacle.py) pinned against the
big-endian goldens that the real reference produced
(tests/golden/make_golden_byteorder.py), and the byte-order dtype codes of
the C ABI (include/mcodec.h MC_BIG_ENDIAN) as the Python layer maps them."""

import json
import os

import numpy as np
import pytest

import oracle.nporacle as npo

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "byteorder.json")) as _f:
    MANIFEST = json.load(_f)
DATA = np.load(os.path.join(GOLDEN, "byteorder.npz"))


def vec(fam, i, key):
    return DATA[f"{fam}__{i}__{key}"]


def _b(a):
    return np.asarray(a).tobytes(order="A")


def test_manifest_covers_the_verdict_dtypes():
    """'>f4', '>f8', '>i2', '>i4', '>u2' and mixed-order pairs are present."""
    pairs = {(m["dtype"], m["astype"]) for m in MANIFEST["bo_delta"]}
    assert {(">f4", ">f4"), (">f8", ">f8"), (">i2", ">i2"), (">i4", ">i4"), (">u2", ">u2"),
            (">f4", "<f4"), ("<f4", ">f4")} <= pairs
    fso = {(m["dtype"], m["astype"]) for m in MANIFEST["bo_fso"]}
    assert {(">f8", ">i2"), (">f4", ">i2")} <= fso
    assert {(m["dtype"], m["astype"]) for m in MANIFEST["bo_quantize"]} >= {(">f8", ">f4")}
    assert {(m["encode_dtype"], m["decode_dtype"]) for m in MANIFEST["bo_astype"]} >= {(">f4", ">f8")}


@pytest.mark.parametrize("i", range(len(MANIFEST["bo_delta"])))
def test_oracle_delta(i):
    m = MANIFEST["bo_delta"][i]
    x = vec("bo_delta", i, "input")
    assert _b(npo.delta_encode(x, m["dtype"], m["astype"])) == vec("bo_delta", i, "encoded").tobytes()
    assert _b(npo.delta_decode(vec("bo_delta", i, "encoded"), m["dtype"], m["astype"])) == \
        vec("bo_delta", i, "decoded").tobytes()


@pytest.mark.parametrize("i", range(len(MANIFEST["bo_fso"])))
def test_oracle_fso(i):
    m = MANIFEST["bo_fso"][i]
    with np.errstate(all="ignore"):
        enc = npo.fso_encode(vec("bo_fso", i, "input"), m["offset"], m["scale"], m["dtype"], m["astype"])
        dec = npo.fso_decode(vec("bo_fso", i, "encoded"), m["offset"], m["scale"], m["dtype"], m["astype"])
    assert _b(enc) == vec("bo_fso", i, "encoded").tobytes()
    assert _b(dec) == vec("bo_fso", i, "decoded").tobytes()


@pytest.mark.parametrize("i", range(len(MANIFEST["bo_quantize"])))
def test_oracle_quantize(i):
    m = MANIFEST["bo_quantize"][i]
    with np.errstate(all="ignore"):
        enc = npo.quantize_encode(vec("bo_quantize", i, "input"), m["digits"], m["dtype"], m["astype"])
        dec = npo.quantize_decode(vec("bo_quantize", i, "encoded"), m["dtype"], m["astype"])
    assert _b(enc) == vec("bo_quantize", i, "encoded").tobytes()
    assert _b(dec) == vec("bo_quantize", i, "decoded").tobytes()


@pytest.mark.parametrize("i", range(len(MANIFEST["bo_astype"])))
def test_oracle_astype(i):
    m = MANIFEST["bo_astype"][i]
    with np.errstate(all="ignore"):
        enc = npo.astype_encode(vec("bo_astype", i, "input"), m["encode_dtype"], m["decode_dtype"])
        dec = npo.astype_decode(vec("bo_astype", i, "encoded"), m["encode_dtype"], m["decode_dtype"])
    assert _b(enc) == vec("bo_astype", i, "encoded").tobytes()
    assert _b(dec) == vec("bo_astype", i, "decoded").tobytes()


def test_dtype_codes_carry_the_byte_order_flag():
    from numcodecs_amd import _native
    from numcodecs_amd._ops import dtype_code

    assert _native.MC_BIG_ENDIAN == 32
    for s in ("i2", "i4", "i8", "u2", "u4", "u8", "f2", "f4", "f8"):
        assert dtype_code(">" + s) == dtype_code("<" + s) | 32
    for s in ("i1", "u1", "b1"):  # numpy has no byte order for 1-byte types
        assert dtype_code(">" + s) == dtype_code("<" + s) == dtype_code("|" + s)
    assert dtype_code(">c8") == dtype_code("<c8") | 32  # extended dtypes (round 5)
    with pytest.raises(NotImplementedError):
        dtype_code("|S4")
    with open(os.path.join(os.path.dirname(GOLDEN), "..", "include", "mcodec.h")) as f:
        assert "#define MC_BIG_ENDIAN 32" in f.read()
