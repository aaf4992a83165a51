"""Numpy + C restatement of the numcodecs hot path -- TEST INFRASTRUCTURE ONLY.

Every function names the reference lines it restates (paths under
src/numcodecs/ of zarr-developers/numcodecs).  Inputs are host buffers
(numpy arrays or bytes-like); outputs mirror what the reference returns.
"""

from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libncoracle.so")
_lib = None


def _c():
    """Load (building on first use) the C restatement oracle/ncoracle.c."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.run(["make", "-s", "-C", _HERE, "_build/libncoracle.so"], check=True)
        lib = ctypes.CDLL(_LIB_PATH)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        lib.nco_shuffle.argtypes = [vp, vp, sz, sz]
        lib.nco_unshuffle.argtypes = [vp, vp, sz, sz]
        lib.nco_shuffle_batch.argtypes = [vp, vp, sz, sz, sz]
        lib.nco_unshuffle_batch.argtypes = [vp, vp, sz, sz, sz]
        lib.nco_fletcher32.argtypes = [vp, sz]
        lib.nco_fletcher32.restype = ctypes.c_uint32
        lib.nco_jenkins_lookup3.argtypes = [vp, sz, ctypes.c_uint32]
        lib.nco_jenkins_lookup3.restype = ctypes.c_uint32
        lib.nco_crc32c.argtypes = [vp, sz, ctypes.c_uint32]
        lib.nco_crc32c.restype = ctypes.c_uint32
        lib.nco_bitround32.argtypes = [vp, vp, sz, ctypes.c_int]
        lib.nco_fso_encode_f4_i2.argtypes = [vp, vp, sz, ctypes.c_float, ctypes.c_float]
        lib.nco_fso_decode_i2_f4.argtypes = [vp, vp, sz, ctypes.c_double, ctypes.c_double]
        lib.nco_delta_encode_i2.argtypes = [vp, vp, sz]
        lib.nco_delta_decode_i2.argtypes = [vp, vp, sz]
        _lib = lib
    return _lib


def _bytes_view(buf) -> np.ndarray:
    """Flat uint8 view of a contiguous buffer (compat.py:120-150 semantics)."""
    if isinstance(buf, np.ndarray):
        a = buf
        if a.dtype.kind in "Mm":
            a = a.view("i8")
        if not (a.flags.c_contiguous or a.flags.f_contiguous):
            raise ValueError("an array with contiguous memory is required")
        return a.reshape(-1, order="A").view("u1")
    return np.frombuffer(memoryview(buf), dtype="u1")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# --------------------------------------------------------------------------
# Shuffle: _shuffle.pyx:11-30, shuffle.py:23-58
# --------------------------------------------------------------------------
def shuffle(buf, elementsize: int) -> np.ndarray:
    """Shuffle(elementsize).encode(buf) -> uint8 array (shuffle.py:40-48)."""
    src = np.ascontiguousarray(_bytes_view(buf))
    out = np.zeros(src.nbytes, dtype="u1")
    if elementsize <= 1:
        out[:] = src
        return out
    if src.nbytes % elementsize != 0:
        raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
    if src.nbytes:
        _c().nco_shuffle(_ptr(src), _ptr(out), src.nbytes, elementsize)
    return out


def unshuffle(buf, elementsize: int) -> np.ndarray:
    """Shuffle(elementsize).decode(buf) -> uint8 array (shuffle.py:50-58)."""
    src = np.ascontiguousarray(_bytes_view(buf))
    out = np.zeros(src.nbytes, dtype="u1")
    if elementsize <= 1:
        out[:] = src
        return out
    if src.nbytes % elementsize != 0:
        raise ValueError("Shuffle buffer is not an integer multiple of elementsize")
    if src.nbytes:
        _c().nco_unshuffle(_ptr(src), _ptr(out), src.nbytes, elementsize)
    return out


# --------------------------------------------------------------------------
# Fletcher32: fletcher32.pyx:24-115, _utils.pxd:11-24
# --------------------------------------------------------------------------
def fletcher32(buf) -> int:
    """_fletcher32 over the raw bytes (fletcher32.pyx:24-57)."""
    src = np.ascontiguousarray(_bytes_view(buf))
    if src.nbytes == 0:
        return 0
    return int(_c().nco_fletcher32(_ptr(src), src.nbytes))


def fletcher32_encode(buf) -> bytes:
    """payload + LE32 checksum footer (fletcher32.pyx:75-89)."""
    src = _bytes_view(buf)
    if src.nbytes == 0:  # the reference indexes b_mv[0] of an empty view
        raise IndexError("Out of bounds on buffer access (axis 0)")
    return src.tobytes() + int(fletcher32(src)).to_bytes(4, "little")


def fletcher32_decode(buf) -> np.ndarray:
    """Verify the footer and return the payload view (fletcher32.pyx:91-115)."""
    b = _bytes_view(buf)
    if b.nbytes <= 4:
        raise IndexError("Out of bounds on buffer access (axis 0)")
    val = fletcher32(b[:-4])
    found = int.from_bytes(b[-4:].tobytes(), "little")
    if val != found:
        raise RuntimeError(
            f"The fletcher32 checksum of the data ({val}) did not"
            f" match the expected checksum ({found}).\n"
            "This could be a sign that the data has been corrupted."
        )
    return b[:-4]


# --------------------------------------------------------------------------
# BitRound: bitround.py:9-80
# --------------------------------------------------------------------------
MAX_BITS = {"float16": 10, "float32": 23, "float64": 52}


def bitround_encode(a: np.ndarray, keepbits: int):
    """bitround.py:45-69 -- round the mantissa on the same-width int view."""
    if not a.dtype.kind == "f" or a.dtype.itemsize > 8:
        raise TypeError("Only float arrays (16-64bit) can be bit-rounded")
    bits = MAX_BITS[str(a.dtype)]
    int_dtype = np.dtype(a.dtype.str.replace("f", "i"))
    if keepbits == bits:
        return a
    if keepbits > bits:
        raise ValueError("Keepbits too large for given dtype")
    b = a.copy().view(int_dtype)
    maskbits = bits - keepbits
    all_set = np.array(-1, dtype=int_dtype)
    mask = (all_set >> maskbits) << maskbits
    b += ((b >> maskbits) & 1) + ((1 << (maskbits - 1)) - 1)
    b &= mask
    return b


def bitround_decode(enc: np.ndarray) -> np.ndarray:
    """bitround.py:71-80 -- re-view the integers as floats."""
    return enc.view(np.dtype(enc.dtype.str.replace("i", "f")))


# --------------------------------------------------------------------------
# Delta: delta.py:52-83
# --------------------------------------------------------------------------
def delta_encode(buf, dtype, astype=None) -> np.ndarray:
    """enc[0] = x[0]; enc[1:] = np.diff(x) (delta.py:52-67)."""
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    arr = np.asarray(buf).view(dtype).reshape(-1, order="A")
    enc = np.empty_like(arr, dtype=astype)
    enc[0] = arr[0]
    enc[1:] = np.diff(arr)
    return enc


def delta_decode(buf, dtype, astype=None) -> np.ndarray:
    """np.cumsum(enc, out=dec) accumulated in dtype (delta.py:69-83)."""
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    enc = np.asarray(buf).view(astype).reshape(-1, order="A")
    dec = np.empty_like(enc, dtype=dtype)
    np.cumsum(enc, out=dec)
    return dec


# --------------------------------------------------------------------------
# Quantize: quantize.py:60-82
# --------------------------------------------------------------------------
def quantize_scale(digits: int) -> float:
    """The power-of-two scale of quantize.py:65-73."""
    precision = 10.0**-digits
    exp = math.log10(precision)
    exp = math.floor(exp) if exp < 0 else math.ceil(exp)
    bits = math.ceil(math.log2(10.0**-exp))
    return 2.0**bits


def quantize_encode(buf, digits, dtype, astype=None) -> np.ndarray:
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    arr = np.asarray(buf).view(dtype)
    scale = quantize_scale(digits)
    enc = np.around(scale * arr) / scale
    return enc.astype(astype, copy=False)


def quantize_decode(buf, dtype, astype=None) -> np.ndarray:
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    return np.asarray(buf).view(astype).astype(dtype, copy=False)


# --------------------------------------------------------------------------
# FixedScaleOffset: fixedscaleoffset.py:83-113
# --------------------------------------------------------------------------
def fso_encode(buf, offset, scale, dtype, astype=None) -> np.ndarray:
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    arr = np.asarray(buf).view(dtype).reshape(-1, order="A")
    enc = np.around((arr - offset) * scale)
    return enc.astype(astype, copy=False)


def fso_decode(buf, offset, scale, dtype, astype=None) -> np.ndarray:
    dtype = np.dtype(dtype)
    astype = dtype if astype is None else np.dtype(astype)
    enc = np.asarray(buf).view(astype).reshape(-1, order="A")
    dec = (enc / scale) + offset
    return dec.astype(dtype, copy=False)


# --------------------------------------------------------------------------
# Checksum32 family: checksum32.py:45-209, jenkins.pyx:93-325
# --------------------------------------------------------------------------
def crc32(buf, value: int = 0) -> int:
    """CRC32.checksum (checksum32.py:106-111) = zlib.crc32 -- the reference's
    own dependency (CPython's zlib module) is the oracle here."""
    import zlib

    return zlib.crc32(_bytes_view(buf), value) & 0xFFFFFFFF


def adler32(buf, value: int = 1) -> int:
    """Adler32.checksum (checksum32.py:125-130) = zlib.adler32."""
    import zlib

    return zlib.adler32(_bytes_view(buf), value) & 0xFFFFFFFF


def crc32c(buf, value: int = 0) -> int:
    """CRC32C.checksum (checksum32.py:203-209); C restatement in ncoracle.c."""
    a = np.ascontiguousarray(_bytes_view(buf))
    return int(_c().nco_crc32c(_ptr(a), a.nbytes, value & 0xFFFFFFFF))


def jenkins_lookup3(buf, initval: int = 0) -> int:
    """jenkins.pyx:93-219; C restatement in ncoracle.c."""
    a = np.ascontiguousarray(_bytes_view(buf))
    return int(_c().nco_jenkins_lookup3(_ptr(a), a.nbytes, initval & 0xFFFFFFFF))


CHECKSUMS = {"crc32": crc32, "adler32": adler32, "crc32c": crc32c}
DEFAULT_LOCATION = {"crc32": "start", "adler32": "start", "crc32c": "end"}


def checksum32_encode(codec_id: str, buf, location=None) -> np.ndarray:
    """Checksum32.encode (checksum32.py:56-70): LE32 checksum + payload."""
    arr = _bytes_view(buf)
    location = location or DEFAULT_LOCATION[codec_id]
    cs = np.array([CHECKSUMS[codec_id](arr)], dtype="<u4").view("u1")
    return np.concatenate([cs, arr] if location == "start" else [arr, cs])


def checksum32_decode(codec_id: str, buf, location=None) -> np.ndarray:
    """Checksum32.decode (checksum32.py:72-88): verify, return the payload."""
    arr = _bytes_view(buf)
    location = location or DEFAULT_LOCATION[codec_id]
    stored, payload = (arr[:4], arr[4:]) if location == "start" else (arr[-4:], arr[:-4])
    if int(stored.view("<u4")[0]) != CHECKSUMS[codec_id](payload):
        raise RuntimeError("checksum mismatch")
    return payload


def jenkins_encode(buf, initval=0, prefix=None) -> bytes:
    """JenkinsLookup3.encode (checksum32.py:160-167)."""
    arr = _bytes_view(buf)
    data = arr if prefix is None else np.concatenate([np.frombuffer(prefix, "u1"), arr])
    return arr.tobytes() + np.array([jenkins_lookup3(data, initval)], "<u4").tobytes()


# --------------------------------------------------------------------------
# AsType (astype.py:46-58), PackBits (packbits.py:33-82)
# --------------------------------------------------------------------------
def astype_encode(buf, encode_dtype, decode_dtype) -> np.ndarray:
    return np.asarray(buf).view(np.dtype(decode_dtype)).astype(np.dtype(encode_dtype))


def astype_decode(buf, encode_dtype, decode_dtype) -> np.ndarray:
    return np.asarray(buf).view(np.dtype(encode_dtype)).astype(np.dtype(decode_dtype))


def packbits_encode(buf) -> np.ndarray:
    arr = np.asarray(buf).view(bool).reshape(-1, order="A")
    n = arr.size
    enc = np.empty(n // 8 + (1 if n % 8 else 0) + 1, dtype="u1")
    enc[0] = (8 - n % 8) if n % 8 else 0
    enc[1:] = np.packbits(arr)
    return enc


def packbits_decode(buf) -> np.ndarray:
    enc = np.asarray(buf).view("u1").reshape(-1, order="A")
    pad = int(enc[0])
    dec = np.unpackbits(enc[1:])
    if pad:
        dec = dec[:-pad]
    return dec.view(bool)


# --------------------------------------------------------------------------
# CPU baseline helpers (bench.py cpu_baseline leg)
# --------------------------------------------------------------------------
def shuffle_into(src: np.ndarray, dst: np.ndarray, elementsize: int) -> None:
    _c().nco_shuffle(_ptr(src), _ptr(dst), src.nbytes, elementsize)


def unshuffle_into(src: np.ndarray, dst: np.ndarray, elementsize: int) -> None:
    _c().nco_unshuffle(_ptr(src), _ptr(dst), src.nbytes, elementsize)


# C restatements of the numpy-expressed codecs (ncoracle.c), into caller
# buffers; pinned bit-exact against the numpy restatements above and the
# goldens by tests/test_oracle.py.
def c_bitround32_into(src: np.ndarray, dst: np.ndarray, keepbits: int) -> None:
    """bitround.py:62-68, float32 (0 <= keepbits < 23)."""
    _c().nco_bitround32(_ptr(src), _ptr(dst), src.nbytes // 4, keepbits)


def c_fso_encode_f4_i2_into(src: np.ndarray, dst: np.ndarray, offset, scale) -> None:
    """fixedscaleoffset.py:91-97, '<f4' -> '<i2' (NEP 50: float32 compute,
    offset/scale rounded to float32)."""
    _c().nco_fso_encode_f4_i2(_ptr(src), _ptr(dst), src.nbytes // 4, float(np.float32(offset)),
                              float(np.float32(scale)))


def c_fso_decode_i2_f4_into(src: np.ndarray, dst: np.ndarray, offset, scale) -> None:
    """fixedscaleoffset.py:107-110, '<i2' -> '<f4' through float64."""
    _c().nco_fso_decode_i2_f4(_ptr(src), _ptr(dst), src.nbytes // 2, float(scale), float(offset))


def c_delta_encode_i2_into(src: np.ndarray, dst: np.ndarray) -> None:
    """delta.py:63-66, '<i2'."""
    _c().nco_delta_encode_i2(_ptr(src), _ptr(dst), src.nbytes // 2)


def c_delta_decode_i2_into(src: np.ndarray, dst: np.ndarray) -> None:
    """delta.py:80 (np.cumsum in int16), '<i2'."""
    _c().nco_delta_decode_i2(_ptr(src), _ptr(dst), src.nbytes // 2)


def c_fletcher32(src: np.ndarray) -> int:
    """fletcher32.pyx:24-57 over a contiguous uint8 array."""
    return int(_c().nco_fletcher32(_ptr(src), src.nbytes))
