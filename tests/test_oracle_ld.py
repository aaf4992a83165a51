"""The oracle (oracle/nporacle.py: the reference's numpy expressions restated)
reproduces the reference's own outputs for the round-6 inputs
(tests/golden/ld.npz, made by tests/golden/make_golden_ld.py from the real
reference): longdouble / clongdouble on Delta, Quantize, FixedScaleOffset
and AsType, datetime64 Delta with unit changes and the calendar AsType
casts, and numpy's errors for string / void dtypes.  Longdoubles are compared
on their 10 value bytes (tests/helpers.py::value_mask)."""

import json
import os
import warnings

import numpy as np
import pytest

from oracle import nporacle
from tests.helpers import same_values

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "ld.json")) as _f:
    MANIFEST = json.load(_f)

pytestmark = pytest.mark.skipif(np.finfo(np.longdouble).nmant != 63, reason="x87 longdouble goldens")

CASES = [(fam, i) for fam in ("ld_delta", "ld_quantize", "ld_fso", "ld_astype") for i in range(len(MANIFEST[fam]))]


@pytest.fixture(scope="module")
def data():
    return np.load(os.path.join(GOLDEN, "ld.npz"))


def _scalar(v):
    return complex(v[0], v[1]) if isinstance(v, list) else v


def _ops(fam, m):
    if fam == "ld_delta":
        return (lambda x: nporacle.delta_encode(x, m["dtype"], m["astype"]),
                lambda e: nporacle.delta_decode(e, m["dtype"], m["astype"]), m["dtype"], m["astype"])
    if fam == "ld_quantize":
        return (lambda x: nporacle.quantize_encode(x, m["digits"], m["dtype"], m["astype"]),
                lambda e: nporacle.quantize_decode(e, m["dtype"], m["astype"]), m["dtype"], m["astype"])
    if fam == "ld_fso":
        o, s = _scalar(m["offset"]), _scalar(m["scale"])
        return (lambda x: nporacle.fso_encode(x, o, s, m["dtype"], m["astype"]),
                lambda e: nporacle.fso_decode(e, o, s, m["dtype"], m["astype"]), m["dtype"], m["astype"])
    return (lambda x: nporacle.astype_encode(x, m["encode_dtype"], m["decode_dtype"]),
            lambda e: nporacle.astype_decode(e, m["encode_dtype"], m["decode_dtype"]), m["decode_dtype"],
            m["encode_dtype"])


@pytest.mark.parametrize("case", CASES, ids=[f"{f}-{i}" for f, i in CASES])
def test_oracle_matches_reference_goldens(data, case):
    fam, i = case
    m = MANIFEST[fam][i]
    enc_fn, dec_fn, d_in, d_enc = _ops(fam, m)
    x = data[f"{fam}__{i}__input"].view(d_in)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if "encode_error" in m:
            with pytest.raises(Exception) as ei:
                enc_fn(x)
            assert type(ei.value).__name__ == m["encode_error"][0]
            return
        enc = enc_fn(x)
        want = data[f"{fam}__{i}__encoded"]
        assert same_values(enc.tobytes(), want.tobytes(), enc.dtype), "encode"
        e = want.view(m.get("encoded_dtype", d_enc))
        if "decode_error" in m:
            with pytest.raises(Exception) as ei:
                dec_fn(e)
            assert type(ei.value).__name__ == m["decode_error"][0]
            return
        dec = dec_fn(e)
    assert same_values(dec.tobytes(), data[f"{fam}__{i}__decoded"].tobytes(), dec.dtype), "decode"
