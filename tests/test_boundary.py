"""The drop-in boundary, on CPU: registry, configs, reprs, equality, argument
errors (reference tests: test_registry.py, test_shuffle.py:53-77,
test_bitround.py:75-81, test_delta.py:42-61, test_quantize.py:117-132,
test_fixedscaleoffset.py:195-214), and the C ABI: libmcodec.so loads and
exports every entry point include/mcodec.h declares (no compute without a
GPU)."""

import ctypes
import os
import re

import numpy as np
import pytest

import numcodecs_amd
from numcodecs_amd import (
    BitRound,
    Delta,
    FixedScaleOffset,
    Fletcher32,
    Quantize,
    Shuffle,
    UnknownCodecError,
    get_codec,
)
from numcodecs_amd import _native
from tests.helpers import check_config, check_repr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mcodec.h")


def test_registry_ids():
    assert set(numcodecs_amd.codec_registry) == {
        "shuffle", "bitround", "delta", "quantize", "fixedscaleoffset", "fletcher32",
        "crc32", "crc32c", "adler32", "jenkins_lookup3", "astype", "packbits"}


def test_registry_errors():
    with pytest.raises(UnknownCodecError, match="foo"):
        get_codec({"id": "foo"})
    assert issubclass(UnknownCodecError, ValueError)
    assert str(UnknownCodecError("'x'")) == "codec not available: ''x''"


def test_get_codec_argument_not_modified():
    arg = {"id": "shuffle", "elementsize": 8}
    before = dict(arg)
    assert get_codec(arg) == Shuffle(8)
    assert arg == before


def test_register_codec_replaces():
    class MyShuffle(Shuffle):
        pass

    numcodecs_amd.register_codec(MyShuffle, "myshuffle")
    try:
        assert isinstance(get_codec({"id": "myshuffle", "elementsize": 2}), MyShuffle)
    finally:
        numcodecs_amd.codec_registry.pop("myshuffle")


@pytest.mark.parametrize("codec", [
    Shuffle(), Shuffle(elementsize=8), BitRound(10), Delta(dtype="<i4", astype="<i2"),
    Quantize(digits=2, dtype="<f8", astype="<f2"),
    FixedScaleOffset(dtype="<f8", astype="<i4", scale=10, offset=100), Fletcher32(),
    FixedScaleOffset(offset=1000.5, scale=1e3, dtype="<f4", astype="<i2"),
])
def test_config_roundtrip(codec):
    check_config(codec)


def test_configs_match_reference_shapes():
    assert Shuffle().get_config() == {"id": "shuffle", "elementsize": 4}
    assert BitRound(3).get_config() == {"id": "bitround", "keepbits": 3}
    assert Delta("i8", "i4").get_config() == {"id": "delta", "dtype": "<i8", "astype": "<i4"}
    assert Quantize(1, "f8").get_config() == {"id": "quantize", "digits": 1, "dtype": "<f8",
                                              "astype": "<f8"}
    assert FixedScaleOffset(1000, 10, "f8", "u1").get_config() == {
        "id": "fixedscaleoffset", "scale": 10, "offset": 1000, "dtype": "<f8", "astype": "|u1"}
    assert Fletcher32().get_config() == {"id": "fletcher32"}


@pytest.mark.parametrize("stmt", [
    "Shuffle(elementsize=0)", "Shuffle(elementsize=4)", "Shuffle(elementsize=16)",
    "Delta(dtype='<i4', astype='<i2')", "Delta(dtype='<f8')",
    "Quantize(digits=2, dtype='<f8', astype='<f2')",
    "FixedScaleOffset(scale=10, offset=100, dtype='<f8', astype='<i4')",
    "BitRound(keepbits=10)", "Fletcher32()",
])
def test_repr(stmt):
    check_repr(stmt)


def test_eq():
    assert Shuffle() == Shuffle()
    assert Shuffle(elementsize=16) != Shuffle()
    assert Delta("<i4") != Delta("<i4", "<i2")
    assert Fletcher32() == Fletcher32()
    assert Shuffle() != "shuffle"


def test_constructor_errors():
    with pytest.raises(ValueError):
        BitRound(-1)
    with pytest.raises(ValueError):
        Delta(dtype=object)
    with pytest.raises(ValueError):
        Delta(dtype="i8", astype=object)
    with pytest.raises(ValueError):
        Quantize(digits=2, dtype="i4")
    with pytest.raises(ValueError):
        Quantize(digits=2, dtype=object)
    with pytest.raises(ValueError):
        Quantize(digits=2, dtype="f8", astype=object)
    with pytest.raises(ValueError):
        FixedScaleOffset(dtype=object, astype="i4", scale=10, offset=100)
    with pytest.raises(ValueError):
        FixedScaleOffset(dtype="f8", astype=object, scale=10, offset=100)


def test_encode_argument_errors_before_device():
    """Errors the reference raises from argument checks come first, also on a
    machine without a GPU (test_bitround.py:75-81, test_shuffle.py:162-166)."""
    with pytest.raises(ValueError):
        BitRound(keepbits=99).encode(np.array([0], dtype="float32"))
    with pytest.raises(TypeError):
        BitRound(keepbits=10).encode(np.array([0]))
    with pytest.raises(KeyError):
        BitRound(keepbits=3).encode(np.array([0], dtype=">f4"))
    x = np.ones(3, "f4")
    assert BitRound(23).encode(x) is x  # keepbits == max: the input itself


def test_no_device_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(_native.MCodecError, match="no CPU fallback"):
        Shuffle(4).encode(np.arange(16, dtype="i4"))
    with pytest.raises(_native.MCodecError):
        Fletcher32().encode(b"abcd")


def _header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char \*|void \*|void)\s*(mc_\w+)\s*\(", src, re.M)))


def test_header_declares_extern_c_and_plain_types():
    src = open(HEADER).read()
    assert 'extern "C"' in src
    assert "torch" not in re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    assert len(_header_functions()) >= 25


def test_library_exports_every_header_symbol():
    assert os.path.exists(_native.lib_path), "build with __graft_entry__.build()"
    handle = ctypes.CDLL(_native.lib_path)
    missing = [f for f in _header_functions() if not hasattr(handle, f)]
    assert not missing, missing
    # and the Python binding knows every one of them (argtypes table)
    assert set(_header_functions()) == set(_native.EXPORTED)
    assert handle.mc_abi_version() == 2


def test_library_host_queries_need_no_gpu():
    lib = _native.lib
    assert lib.mc_strerror(-22) == b"invalid argument"
    assert lib.mc_fletcher32_workspace(1 << 20) >= 12
    assert lib.mc_delta_decode_workspace(1 << 20, 2, 2) >= ((1 << 20) // 4096) * 8  # tile totals (+ group offsets)
    # float f4/f8: tile totals + tile prefixes + the first-failure word of the
    # speculative scan (16 KiB of output per tile) for every float dtype and
    # any numeric astype but bool
    # float: tile totals, tile prefixes, per-tile first failures (the walker), the first failure
    assert lib.mc_delta_decode_workspace(100, 10, 10) == 4 * 8
    assert lib.mc_delta_decode_workspace(1 << 20, 10, 10) == (3 * 256 + 1) * 8
    assert lib.mc_delta_decode_workspace(1 << 20, 11, 11) == (3 * 512 + 1) * 8
    assert lib.mc_delta_decode_workspace(1 << 20, 9, 9) == (3 * 128 + 1) * 8
    assert lib.mc_delta_decode_workspace(1 << 20, 10, 11) == (3 * 512 + 1) * 8  # astype f4 -> dtype f8
    assert lib.mc_delta_decode_workspace(100, 2, 10) == 4 * 8  # astype i2 -> dtype f4
    assert lib.mc_delta_decode_workspace(100, 0, 10) == 0  # bool astype: serial
    assert lib.mc_delta_decode_batch_workspace(7, 100, 10, 10) == 7 * 8
    assert lib.mc_delta_decode_batch_workspace(7, 100, 9, 11) == 7 * 8
    assert lib.mc_delta_decode_batch_workspace(7, 100, 2, 2) == 0


# ---- §8f next-row codecs: config surface (no device needed) ----------------
@pytest.mark.parametrize("stmt", [
    "CRC32(location='start')", "CRC32(location='end')", "Adler32(location='start')",
    "Adler32(location='end')", "CRC32C(location='start')", "CRC32C(location='end')",
    "AsType(encode_dtype='<f4', decode_dtype='<f8')", "AsType(encode_dtype='<i2', decode_dtype='<i4')",
    "PackBits()", "JenkinsLookup3(initval=0, prefix=None)", "JenkinsLookup3(initval=1230, prefix=None)",
])
def test_next_codecs_repr(stmt):
    check_repr(stmt)


def test_next_codecs_config():
    from numcodecs_amd import CRC32, CRC32C, Adler32, AsType, JenkinsLookup3, PackBits

    for c in (CRC32(), CRC32(location="end"), Adler32(), CRC32C(), CRC32C(location="start"),
              AsType("<f4", "<f8"), PackBits(), JenkinsLookup3(), JenkinsLookup3(initval=5)):
        check_config(c)
    assert CRC32().get_config() == {"id": "crc32"}
    assert CRC32C().location == "end" and CRC32().location == "start"
    assert AsType("f4", "f8").get_config() == {"id": "astype", "encode_dtype": "<f4", "decode_dtype": "<f8"}
    for cls in (CRC32, Adler32, CRC32C):
        with pytest.raises(ValueError):
            cls(location="foo")
    assert JenkinsLookup3(prefix=b"ab").prefix.tolist() == [97, 98]


def test_is_ndarray_like_mirrors_reference_protocol():
    """ndarray_like.py:39-64: the structural NDArrayLike check."""
    import numpy as np

    from numcodecs_amd.compat import is_ndarray_like

    assert is_ndarray_like(np.zeros(3))
    assert not is_ndarray_like(b"abc")
    assert not is_ndarray_like(bytearray(3))
    assert not is_ndarray_like(memoryview(b"abc"))


def test_delta_decode_pairs():
    """np.cumsum(enc, out=dec) (delta.py:80) accepts every numeric pair (it
    accumulates in promote_types(astype, dtype)); the device decodes float
    dtypes, integer-from-integer (wrap-around) and bool-from-bool directly,
    and the two other families through their loop dtype and a cast."""
    import itertools

    from numcodecs_amd.delta import decode_loop_dtype

    ts = ["|b1", "|i1", "<i2", ">i4", "<i8", "|u1", ">u2", "<u4", "<u8", "<f2", ">f4", "<f8"]
    for a, d in itertools.product(ts, ts):
        ka, kd = np.dtype(a).kind, np.dtype(d).kind
        two_step = (kd in "iub" and ka == "f") or (kd == "b" and ka != "b")
        loop = decode_loop_dtype(a, d)
        if two_step:
            assert loop == np.promote_types(a, d) and loop.isnative, (a, d)
        else:
            assert loop is None, (a, d)
