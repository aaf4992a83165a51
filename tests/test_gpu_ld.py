"""Round 6 inputs on the GPU, against the real reference's outputs
(tests/golden/ld.npz / ld.json, tests/golden/make_golden_ld.py):

  * longdouble / clongdouble ('<f16' / '<c32', the x87 80-bit extended type
    numpy uses on x86-64) on Delta, Quantize, FixedScaleOffset and AsType --
    csrc/mc_x80.h on the device: every x87 operation and cast bit-exact,
    specials included (signalling / quiet NaN payloads, denormals,
    pseudo-denormals, unnormals, pseudo-NaNs, infinities, +-0);
  * datetime64 Delta with a unit change and the calendar AsType casts
    (csrc/mc_cal.h, numpy's datetimestruct path);
  * numpy's errors for string / bytes / void dtypes (delta.py:66 np.diff,
    fixedscaleoffset.py:87 the subtraction).

Bar: byte-identical on the bytes numpy defines (a computed longdouble's 6
padding bytes are whatever numpy's output buffer held: tests/helpers.py::
value_mask), the same exception type and message.  Larger sizes are checked
against the oracle (numpy on the box's host) on random bit patterns."""

import json
import os
import warnings

import numpy as np
import pytest
import torch

from numcodecs_amd import AsType, Delta, FixedScaleOffset, Quantize
from oracle import nporacle
from tests.helpers import same_values

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(np.finfo(np.longdouble).nmant != 63, reason="x87 longdouble host")]

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "ld.json")) as _f:
    MANIFEST = json.load(_f)
_DATA = None


def data():
    global _DATA
    if _DATA is None:
        _DATA = np.load(os.path.join(GOLDEN, "ld.npz"))
    return _DATA


def vec(family, i, key):
    return data()[f"{family}__{i}__{key}"]


def raw(x) -> bytes:
    if isinstance(x, torch.Tensor):
        return x.contiguous().view(-1).view(torch.uint8).cpu().numpy().tobytes()
    return np.asarray(x).tobytes(order="A")


def _scalar(v):
    return complex(v[0], v[1]) if isinstance(v, list) else v


def _codec(family, meta):
    if family == "ld_delta":
        return Delta(dtype=meta["dtype"], astype=meta["astype"])
    if family == "ld_quantize":
        return Quantize(digits=meta["digits"], dtype=meta["dtype"], astype=meta["astype"])
    if family == "ld_fso":
        return FixedScaleOffset(offset=_scalar(meta["offset"]), scale=_scalar(meta["scale"]), dtype=meta["dtype"],
                                astype=meta["astype"])
    return AsType(encode_dtype=meta["encode_dtype"], decode_dtype=meta["decode_dtype"])


def _dtypes(family, meta):
    if family == "ld_astype":
        return np.dtype(meta["decode_dtype"]), np.dtype(meta["encoded_dtype"] if "encoded_dtype" in meta
                                                       else meta["encode_dtype"])
    return np.dtype(meta["dtype"]), np.dtype(meta["astype"])


def _check_error(err, fn):
    name, base, msg = err
    with pytest.raises(Exception) as ei:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            fn()
    e = ei.value
    assert type(e).__name__ == name, (type(e), e)
    assert any(c.__name__ == base for c in type(e).__mro__)
    assert str(e) == msg


CASES = [(fam, i) for fam in ("ld_delta", "ld_quantize", "ld_fso", "ld_astype") for i in range(len(MANIFEST[fam]))]


def _id(c):
    fam, i = c
    m = MANIFEST[fam][i]
    if fam == "ld_astype":
        return f"{fam}-{m['encode_dtype']}<-{m['decode_dtype']}-{i}"
    return f"{fam}-{m['dtype']}-{m['astype']}-{m.get('kind', m.get('digits', ''))}-{i}"


def _device_input(x: np.ndarray, dev):
    t = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).copy()).to(dev)
    if x.dtype.str in ("<c8", "<c16"):
        return t.view(torch.complex64 if x.dtype.itemsize == 8 else torch.complex128)
    if x.dtype.str in ("<f2", "<f4", "<f8"):
        return t.view({"<f2": torch.float16, "<f4": torch.float32, "<f8": torch.float64}[x.dtype.str])
    return t


def _string_astype(meta):
    # numpy formats floats as strings here (delta.py:66 into an 'S' array):
    # not a per-element float filter; the build refuses it loudly
    return np.dtype(meta.get("astype", "f")).kind in "SUV" and np.dtype(meta.get("dtype", "f")).kind not in "SUV"


@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("case", CASES, ids=[_id(c) for c in CASES])
def test_vs_reference(device, case, where):
    fam, i = case
    meta = MANIFEST[fam][i]
    codec = _codec(fam, meta)
    d_in, d_enc = _dtypes(fam, meta)
    x = vec(fam, i, "input").view(d_in)
    feed = (lambda a: _device_input(a, device)) if where == "device" else (lambda a: a)
    if "encode_error" in meta:
        _check_error(meta["encode_error"], lambda: codec.encode(feed(x)))
        return
    if _string_astype(meta):
        with pytest.raises(NotImplementedError):
            codec.encode(feed(x))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # ComplexWarning, as the reference emits it
        enc = codec.encode(feed(x))
    if where == "host":
        assert enc.dtype == d_enc
    assert same_values(raw(enc), vec(fam, i, "encoded").tobytes(), d_enc), "encode"
    e = feed(vec(fam, i, "encoded").view(d_enc))
    if "decode_error" in meta:
        _check_error(meta["decode_error"], lambda: codec.decode(e))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        dec = codec.decode(e)
    d_out = np.dtype(meta.get("decoded_dtype", d_in))
    if where == "host":
        assert dec.dtype == d_out
    assert same_values(raw(dec), vec(fam, i, "decoded").tobytes(), d_out), "decode"


def _ld_random(rng, n):
    """random 80-bit patterns: every class x87 distinguishes, weighted to
    normals around 1"""
    w = rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    e = rng.integers(16383 - 70, 16383 + 70, n).astype(np.uint16)
    e[::5] = rng.integers(0, 0x8000, e[::5].size).astype(np.uint16)
    e[::11] = 0x7fff
    m = w | np.uint64(1 << 63)
    m[::7] = w[::7]  # J clear: denormals / unnormals / pseudo-NaNs
    e |= (rng.integers(0, 2, n).astype(np.uint16) << np.uint16(15))
    b = np.zeros((n, 16), np.uint8)
    b[:, :8] = m.view(np.uint8).reshape(-1, 8)
    b[:, 8:10] = e.view(np.uint8).reshape(-1, 2)
    return b.reshape(-1).view(np.longdouble)


@pytest.mark.parametrize("t", ["|b1", "|i1", "<i2", "<i4", "<i8", "|u1", "<u2", "<u4", "<u8", "<f2", "<f4", "<f8",
                               ">f8", "<c8", "<c16", "<m8[s]", ">f16", "<c32"])
def test_astype_random_bits_vs_oracle(device, t):
    """AsType both ways between longdouble and `t` on 1 Mi random 80-bit
    patterns (and random `t` bit patterns): the device casts against numpy's
    on the box's host."""
    rng = np.random.default_rng(abs(hash(t)) % 2**32)
    n = 1 << 20
    x = _ld_random(rng, n)
    codec = AsType(encode_dtype=t, decode_dtype="<f16")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = nporacle.astype_encode(x, t, "<f16")
        got = codec.encode(_device_input(x, device))
    assert same_values(raw(got), want.tobytes(), want.dtype)
    dt = np.dtype(t)
    if dt.kind in "fc":
        y = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
    elif dt.kind == "b":
        y = rng.integers(0, 2, n).astype("?")
    else:
        y = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = nporacle.astype_decode(y, t, "<f16")
        got = codec.decode(_device_input(y, device))
    assert same_values(raw(got), want.tobytes(), want.dtype)


@pytest.mark.parametrize("op", ["fso_f16_i4", "fso_f16_f16", "quant_f16", "quant_f8_f16", "fso_dec_i2_f16"])
def test_elementwise_random_bits_vs_oracle(device, op):
    """FixedScaleOffset / Quantize over 1 Mi random longdouble patterns (NaN
    payloads, denormals, rejected encodings) against numpy on the host."""
    rng = np.random.default_rng(["fso_f16_i4", "fso_f16_f16", "quant_f16", "quant_f8_f16", "fso_dec_i2_f16"].index(op))
    n = 1 << 20
    x = _ld_random(rng, n)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        if op == "fso_f16_i4":
            c, want = FixedScaleOffset(7, 1e3, "<f16", "<i4"), nporacle.fso_encode(x, 7, 1e3, "<f16", "<i4")
        elif op == "fso_f16_f16":
            c, want = FixedScaleOffset(0.1, 3.0, "<f16"), nporacle.fso_encode(x, 0.1, 3.0, "<f16")
        elif op == "quant_f16":
            c, want = Quantize(3, "<f16"), nporacle.quantize_encode(x, 3, "<f16")
        elif op == "quant_f8_f16":
            x = rng.standard_normal(n) * 1e3
            c, want = Quantize(2, "<f8", "<f16"), nporacle.quantize_encode(x, 2, "<f8", "<f16")
        else:
            x = rng.integers(-30000, 30000, n).astype("<i2")
            c, want = FixedScaleOffset(3, 7.0, "<f16", "<i2"), nporacle.fso_decode(x, 3, 7.0, "<f16", "<i2")
            got = c.decode(_device_input(x, device))
            assert same_values(raw(got), want.tobytes(), want.dtype)
            return
        got = c.encode(_device_input(x, device))
    assert same_values(raw(got), want.tobytes(), want.dtype)


@pytest.mark.parametrize("dt,at", [("<f16", "<f16"), ("<f8", "<f16"), ("<f16", "<f4"), ("<i8", "<f16"),
                                   ("<c32", "<c32")])
def test_delta_chain_vs_oracle(device, dt, at):
    """Delta encode + the longdouble running-sum decode on 2 Mi elements of
    noise (a rounding event on nearly every add) against numpy's cumsum."""
    rng = np.random.default_rng(5)
    n = 2 << 20
    d = np.dtype(dt)
    if d.kind == "c":
        x = np.empty(n, d)
        x.real = rng.standard_normal(n).astype(np.longdouble) * np.longdouble(1e3)
        x.imag = rng.standard_normal(n).astype(np.longdouble) / np.longdouble(3)
    elif d.kind == "i":
        x = rng.integers(-(1 << 40), 1 << 40, n).astype(d)
    else:
        x = (rng.standard_normal(n).astype(np.longdouble) / np.longdouble(7)).astype(d)
    c = Delta(dt, astype=at)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want_enc = nporacle.delta_encode(x, dt, at)
        enc = c.encode(_device_input(x, device))
        assert same_values(raw(enc), want_enc.tobytes(), want_enc.dtype), "encode"
        want = nporacle.delta_decode(want_enc, dt, at)
        dec = c.decode(_device_input(want_enc, device))
    assert same_values(raw(dec), want.tobytes(), want.dtype), "decode"


@pytest.mark.parametrize("pair", [("M8[Y]", "M8[D]"), ("M8[ns]", "M8[M]"), ("M8[3M]", "M8[2W]"), ("M8[h]", "M8[Y]")])
def test_calendar_cast_random_vs_numpy(device, pair):
    """Calendar datetime64 casts on 1 Mi ticks spanning +-20000 years."""
    src, dst = np.dtype(pair[0]), np.dtype(pair[1])
    rng = np.random.default_rng(9)
    unit = np.datetime_data(src)[0]
    span = {"Y": 20000, "M": 240000}.get(unit, 6 * 10**17 if unit == "h" else 2**62)
    t = rng.integers(-span, span, 1 << 20)
    t[::1000] = np.iinfo(np.int64).min
    x = t.view(src)
    want = x.astype(dst)
    got = AsType(encode_dtype=dst.str, decode_dtype=src.str).encode(_device_input(x, device))
    assert raw(got) == want.tobytes()
