"""Extended dtypes on the arithmetic codecs, on the GPU: complex64 /
complex128, timedelta64 and datetime64 on Delta, FixedScaleOffset and AsType
(delta.py:52-83, fixedscaleoffset.py:83-113, astype.py:46-58).

Expected results: tests/golden/ext.npz / ext.json, produced by the real
reference (tests/golden/make_golden_ext.py) -- bytes and dtypes of every
encode and decode, or the exception type and message the reference raises
(numpy's UFuncTypeError for a datetime64 Delta decode, TypeError for
FixedScaleOffset on timedelta64, ...).  Bar: byte-identical, same errors.

Device tensors cannot carry timedelta/datetime (torch has no such dtype):
device inputs are raw uint8 bytes and device results of those dtypes are raw
bytes (compat.finish); complex device results are complex tensors.
"""

import json
import os
import warnings

import numpy as np
import pytest
import torch

from numcodecs_amd import AsType, Delta, FixedScaleOffset

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLDEN, "ext.json")) as _f:
    MANIFEST = json.load(_f)
_DATA = None


def data():
    global _DATA
    if _DATA is None:
        _DATA = np.load(os.path.join(GOLDEN, "ext.npz"))
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
    if family == "ext_delta":
        return Delta(dtype=meta["dtype"], astype=meta["astype"])
    if family == "ext_fso":
        return FixedScaleOffset(offset=_scalar(meta["offset"]), scale=_scalar(meta["scale"]), dtype=meta["dtype"],
                                astype=meta["astype"])
    return AsType(encode_dtype=meta["encode_dtype"], decode_dtype=meta["decode_dtype"])


def _dtypes(family, meta):
    if family == "ext_astype":
        return np.dtype(meta["decode_dtype"]), np.dtype(meta["encode_dtype"])
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


CASES = [(fam, i) for fam in ("ext_delta", "ext_fso", "ext_astype") for i in range(len(MANIFEST[fam]))]


def _id(c):
    fam, i = c
    m = MANIFEST[fam][i]
    if fam == "ext_astype":
        return f"{fam}-{m['encode_dtype']}<-{m['decode_dtype']}-{i}"
    return f"{fam}-{m['dtype']}-{m['astype']}-{m.get('kind', '')}{m['n']}-{i}"


def _device_input(x: np.ndarray, dev):
    """A device tensor of the input: complex as a complex tensor, the rest
    (timedelta/datetime, big-endian) as raw bytes."""
    t = torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).copy()).to(dev)
    if x.dtype.str in ("<c8", "<c16"):
        return t.view(torch.complex64 if x.dtype.itemsize == 8 else torch.complex128)
    return t


@pytest.mark.parametrize("case", CASES, ids=[_id(c) for c in CASES])
def test_device_vs_reference(device, case):
    fam, i = case
    meta = MANIFEST[fam][i]
    codec = _codec(fam, meta)
    d_in, d_enc = _dtypes(fam, meta)
    x = vec(fam, i, "input").view(d_in)
    if "encode_error" in meta:
        _check_error(meta["encode_error"], lambda: codec.encode(_device_input(x, device)))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # ComplexWarning, as the reference emits it
        enc = codec.encode(_device_input(x, device))
    assert raw(enc) == vec(fam, i, "encoded").tobytes(), "encode"
    e = _device_input(vec(fam, i, "encoded").view(d_enc), device)
    if "decode_error" in meta:
        _check_error(meta["decode_error"], lambda: codec.decode(e))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        dec = codec.decode(e)
    assert raw(dec) == vec(fam, i, "decoded").tobytes(), "decode"


@pytest.mark.parametrize("case", CASES, ids=[_id(c) for c in CASES])
def test_host_vs_reference(device, case):
    """numpy arrays of the dtype in (staged through the device), numpy arrays
    of the reference's dtype out."""
    fam, i = case
    meta = MANIFEST[fam][i]
    codec = _codec(fam, meta)
    d_in, d_enc = _dtypes(fam, meta)
    x = vec(fam, i, "input").view(d_in)
    if "encode_error" in meta:
        _check_error(meta["encode_error"], lambda: codec.encode(x))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        enc = codec.encode(x)
    assert enc.dtype == np.dtype(meta.get("encoded_dtype", d_enc))
    assert raw(enc) == vec(fam, i, "encoded").tobytes()
    e = vec(fam, i, "encoded").view(d_enc)
    if "decode_error" in meta:
        _check_error(meta["decode_error"], lambda: codec.decode(e))
        return
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        dec = codec.decode(e)
    assert dec.dtype == np.dtype(meta.get("decoded_dtype", d_in))
    assert raw(dec) == vec(fam, i, "decoded").tobytes()


def test_complex_warning_like_reference(device):
    """A complex -> real cast warns with numpy's ComplexWarning (astype.py:53
    emits it through numpy), on device input too."""
    x = torch.tensor([1 + 2j, 3 - 1j], dtype=torch.complex64, device=device)
    with pytest.warns(np.exceptions.ComplexWarning):
        out = AsType(encode_dtype="<f4", decode_dtype="<c8").encode(x)
    assert out.cpu().tolist() == [1.0, 3.0]


def test_datetime_calendar_cast_like_numpy(device):
    """datetime64 calendar conversions (years/months <-> days; round 6:
    csrc/mc_cal.h) give numpy's dates (the reference's astype.py:53 is
    numpy's astype), both ways."""
    x = np.array([0, 1, -1, 30, -2000, np.iinfo(np.int64).min, 7], dtype="i8").view("M8[Y]")
    c = AsType(encode_dtype="M8[D]", decode_dtype="M8[Y]")
    enc = c.encode(x)
    assert enc.dtype == np.dtype("M8[D]") and enc.tobytes() == x.astype("M8[D]").tobytes()
    assert c.decode(enc).tobytes() == x.tobytes()


@pytest.mark.parametrize("dt", ["<c8", "<c16"])
def test_large_complex_delta_round_trip(device, dt):
    """32 MiB complex chunks: the per-component decode takes the speculative
    float scan (exact-add ramp: the round trip is the identity)."""
    n = (32 << 20) // np.dtype(dt).itemsize
    k = torch.arange(n, dtype=torch.float64, device=device)
    ft = torch.float32 if dt == "<c8" else torch.float64
    x = torch.complex((k * 0.125 - 1000).to(ft), (500 - k * 0.25).to(ft))
    c = Delta(dt)
    enc = c.encode(x)
    dec = c.decode(enc)
    assert torch.equal(dec.view(-1), x)


def test_large_timedelta_nat_round_trip(device):
    """64 MiB timedelta64 chunk with NaT mid-chunk: the decode equals numpy's
    (the prefix up to the NaT, NaT after it)."""
    n = 8 << 20
    g = torch.Generator(device="cpu").manual_seed(11)
    steps = torch.randint(-1000, 1000, (n,), generator=g, dtype=torch.int64)
    t = torch.cumsum(steps, 0).numpy()
    t[n // 2 + 17] = np.iinfo(np.int64).min
    x = t.view("m8[ns]")
    c = Delta("<m8[ns]")
    enc = c.encode(x)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = np.cumsum(np.diff(x, prepend=np.timedelta64(0, "ns")))
    dec = c.decode(enc)
    assert dec.dtype == x.dtype
    assert dec.tobytes() == want.tobytes()


# signalling / quiet NaN payloads through casts that only change byte order
# (the value kernel's float -> double -> float round trip would
# quiet them; numpy's byte-swapping astype keeps every bit).  Expected: numpy
# itself (the reference's astype.py:53,58 is numpy's astype).
_NAN_BITS = {
    "f2": [0x7C01, 0xFC01, 0x7E00, 0x7D55, 0x3C00, 0x0001],
    "f4": [0x7F800001, 0xFF800001, 0x7FC00000, 0x7FA5A5A5, 0x3F800000, 0x00000001],
    "f8": [0x7FF0000000000001, 0xFFF0000000000001, 0x7FF8000000000000, 0x7FF5A5A5A5A5A5A5,
           0x3FF0000000000000, 0x0000000000000001],
}


@pytest.mark.parametrize("t", ["f2", "f4", "f8"])
@pytest.mark.parametrize("pair", [("<", ">"), (">", "<")])
@pytest.mark.parametrize("offset", [0, 1])
def test_byte_order_cast_keeps_nan_payloads(device, t, pair, offset):
    src_dt, dst_dt = np.dtype(pair[0] + t), np.dtype(pair[1] + t)
    bits = np.array(_NAN_BITS[t] * 700, dtype=f"u{src_dt.itemsize}")
    x = np.frombuffer(bits.astype(bits.dtype.newbyteorder(pair[0])).tobytes(), dtype=src_dt)
    want = x.astype(dst_dt).tobytes()
    raw_in = torch.from_numpy(np.frombuffer(b"\0" * offset + x.tobytes(), dtype=np.uint8).copy()).to(device)
    got = AsType(encode_dtype=dst_dt.str, decode_dtype=src_dt.str).encode(raw_in[offset:])
    assert raw(got) == want


@pytest.mark.parametrize("t", ["f4", "f8"])
def test_delta_decode_first_element_nan_payload(device, t):
    """np.cumsum's first output is the first input cast to dtype: a
    signalling NaN there keeps its payload (later sums quiet it, as x86
    does)."""
    for at, dt in ((">" + t, "<" + t), ("<" + t, ">" + t), (">" + t, ">" + t)):
        bits = np.array(_NAN_BITS[t][:1] + [_NAN_BITS[t][4]] * 5, dtype=f"u{np.dtype(t).itemsize}")
        enc = np.frombuffer(bits.astype(bits.dtype.newbyteorder(at[0])).tobytes(), dtype=at)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            want = np.cumsum(enc, out=np.empty(len(enc), dtype=dt)).tobytes()
        got = Delta(dtype=dt, astype=at).decode(enc)
        assert raw(got) == want, (at, dt)


@pytest.mark.parametrize("at", ["<f4", ">f4", ">f2", "<f2", ">f8"])
def test_complex_decode_from_real_astype_with_nans(device, at):
    """Delta(complex64, astype=a real float of either byte order) decode of
    data with NaNs (a big-endian astype's NaN inputs were tested
    on their raw bytes): bytes identical to numpy's cumsum (the reference's
    delta.py:80), computed on the host beside the run.  numpy's complex NaN
    choice is pinned to the goldens' numpy (mc_ext.hip
    x_complex_cumsum_keeps_second_nan)."""
    n = 5000
    rng = np.random.default_rng(8)
    x = (rng.standard_normal(n) * 10).astype(np.dtype(at).newbyteorder("="))
    x[[3, 17, 1000, 1001, 4000]] = np.nan
    x[[50, 2000]] = [np.inf, -np.inf]
    enc = x.astype(at)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = np.cumsum(enc, out=np.empty(n, "<c8")).tobytes()
    got = Delta(dtype="<c8", astype=at).decode(enc)
    assert raw(got) == want
