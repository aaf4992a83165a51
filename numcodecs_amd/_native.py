"""ctypes binding of libmcodec.so (the C ABI declared in include/mcodec.h).

The library is a plain C-ABI shared object built by hipcc for gfx950
(numcodecs_amd/csrc/Makefile).  It is bound to the HIP runtime that torch has
already loaded: torch is imported first, so the library's NEEDED
``libamdhip64.so.7`` resolves (by soname) to torch's copy and both share one
runtime, one device context and torch's streams.

There is no CPU fallback anywhere in the product path: if the library is
missing, or no HIP device is visible, every codec call raises.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must precede the dlopen below (shared HIP runtime)

__all__ = [
    "DTYPE_CODES",
    "MCodecError",
    "lib",
    "lib_path",
    "check",
    "available",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
lib_path = os.environ.get("NUMCODECS_AMD_LIB", os.path.join(_HERE, "_lib", "libmcodec.so"))

# mc_dtype codes (include/mcodec.h)
DTYPE_CODES = {
    "|b1": 0,
    "|i1": 1,
    "<i2": 2,
    "<i4": 3,
    "<i8": 4,
    "|u1": 5,
    "<u2": 6,
    "<u4": 7,
    "<u8": 8,
    "<f2": 9,
    "<f4": 10,
    "<f8": 11,
}
# big-endian (non-native) byte order: MC_BIG_ENDIAN OR'd into the code of a
# multi-byte dtype (include/mcodec.h); the kernels reverse each element's
# bytes in registers (numpy normalises '>i1' / '>u1' / '>b1' to '|')
MC_BIG_ENDIAN = 32
DTYPE_CODES.update({">" + k[1:]: v | MC_BIG_ENDIAN for k, v in DTYPE_CODES.items() if k[0] == "<"})
# extended dtypes (round 5): complex64/128, and timedelta64 / datetime64 of
# any unit (the codes carry no unit: int64 ticks; unit casts take numpy's
# conversion factor, see numcodecs_amd._ops.datetime_conversion_factor)
MC_C8, MC_C16, MC_TD8, MC_DT8 = 12, 13, 14, 15
# round 6: numpy's longdouble / clongdouble ('<f16' / '<c32', the x87 80-bit
# extended type of x86-64)
MC_F16L, MC_C32 = 16, 17
EXT_CODES = {"c8": MC_C8, "c16": MC_C16, "m8": MC_TD8, "M8": MC_DT8, "f16": MC_F16L, "c32": MC_C32}

MC_OK = 0
MC_EINVAL = -22
MC_ENOSPC = -28
MC_EPROTO = -71
MC_ARRIVAL_WORDS = 2080  # include/mcodec.h: 64 shard lines + a top line
MC_EHIP_BASE = -1000


class MCodecError(RuntimeError):
    """A libmcodec entry point returned a non-zero status."""


_c_size = ctypes.c_size_t
_c_int = ctypes.c_int
_c_vp = ctypes.c_void_p
_c_double = ctypes.c_double
_c_i64 = ctypes.c_int64
_c_u32 = ctypes.c_uint32

# mc_checksum_kind / mc_checksum_location (include/mcodec.h)
MC_CK_CRC32, MC_CK_CRC32C, MC_CK_ADLER32, MC_CK_JENKINS = 0, 1, 2, 3
MC_CK_START, MC_CK_END = 0, 1

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGNATURES = {
    "mc_abi_version": [],
    "mc_strerror": [_c_int],
    "mc_device_count": [],
    "mc_shuffle": [_c_vp, _c_vp, _c_size, _c_size, _c_vp],
    "mc_unshuffle": [_c_vp, _c_vp, _c_size, _c_size, _c_vp],
    "mc_shuffle_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_size, _c_vp],
    "mc_unshuffle_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_size, _c_vp],
    "mc_bitround": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_vp],
    "mc_bitround_shuffle": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_vp],
    "mc_delta_encode": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_vp],
    "mc_delta_decode_workspace": [_c_size, _c_int, _c_int],
    "mc_delta_decode": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_vp, _c_size, _c_vp, _c_vp],
    "mc_delta_encode_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_vp],
    "mc_delta_decode_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_vp],
    "mc_delta_decode_batch_workspace": [_c_size, _c_size, _c_int, _c_int],
    "mc_delta_decode_batch_ws": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_vp, _c_size,
                                 _c_vp],
    "mc_fso_encode": [
        _c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int,
        _c_double, _c_i64, _c_double, _c_i64, _c_vp,
    ],
    "mc_fso_decode": [
        _c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int, _c_double, _c_double, _c_vp,
    ],
    "mc_quantize": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_double, _c_vp],
    "mc_cast": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_vp],
    "mc_cast_units": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_i64, _c_i64, _c_vp],
    "mc_fso_encode_x": [
        _c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int,
        _c_double, _c_double, _c_i64, _c_double, _c_double, _c_i64, _c_vp,
    ],
    "mc_fso_decode_x": [
        _c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int, _c_double, _c_double, _c_double, _c_double, _c_vp,
    ],
    "mc_fso_encode_raw": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "mc_fso_decode_raw": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_int, _c_vp, _c_vp, _c_vp],
    "mc_cast_calendar": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_int, _c_i64, _c_int, _c_i64, _c_vp],
    "mc_fletcher32_workspace": [_c_size],
    "mc_fletcher32": [_c_vp, _c_size, _c_vp, _c_vp, _c_size, _c_vp],
    "mc_fletcher32_encode": [_c_vp, _c_vp, _c_size, _c_vp, _c_size, _c_vp],
    "mc_fletcher32_encode_fused": [_c_vp, _c_vp, _c_size, _c_vp, _c_size, _c_vp, _c_vp],
    "mc_fletcher32_verify": [_c_vp, _c_size, _c_vp, _c_vp, _c_size, _c_vp],
    "mc_fletcher32_verify_fused": [_c_vp, _c_size, _c_vp, _c_u32, _c_vp, _c_size, _c_vp, _c_vp],
    "mc_fletcher32_batch_workspace": [_c_size, _c_size],
    "mc_fletcher32_batch": [_c_vp, _c_size, _c_size, _c_size, _c_vp, _c_vp, _c_size, _c_vp],
    "mc_fletcher32_encode_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_vp, _c_size, _c_vp],
    "mc_fletcher32_decode_batch": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_vp, _c_vp, _c_size, _c_vp],
    "mc_shuffle_fletcher32_workspace": [_c_size, _c_size, _c_size],
    "mc_shuffle_fletcher32_encode_batch": [
        _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_size, _c_vp, _c_size, _c_vp,
    ],
    "mc_fletcher32_unshuffle_batch": [
        _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_size, _c_vp, _c_vp, _c_size, _c_vp,
    ],
    "mc_fso_delta_shuffle_encode": [_c_vp, _c_vp, _c_size, _c_int, _c_int, _c_double, _c_double, _c_vp],
    "mc_fso_delta_shuffle_decode_workspace": [_c_size],
    "mc_fso_delta_shuffle_encode_batch": [
        _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_double, _c_double, _c_vp,
    ],
    "mc_fso_delta_shuffle_decode_batch_workspace": [_c_size, _c_size],
    "mc_fso_delta_shuffle_decode_batch": [
        _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_double, _c_double, _c_vp, _c_size,
        _c_vp,
    ],
    "mc_fso_delta_shuffle_decode": [
        _c_vp, _c_vp, _c_size, _c_int, _c_int, _c_double, _c_double, _c_vp, _c_size, _c_vp, _c_vp,
    ],
    "mc_checksum32_workspace": [_c_int, _c_size, _c_size],
    "mc_checksum32_batch": [
        _c_int, _c_vp, _c_size, _c_size, _c_size, _c_u32, _c_vp, _c_size, _c_vp, _c_vp, _c_size, _c_vp,
    ],
    "mc_checksum32_encode_batch": [
        _c_int, _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_u32, _c_vp, _c_size, _c_int,
        _c_vp, _c_vp, _c_size, _c_vp,
    ],
    "mc_checksum32_decode_batch": [
        _c_int, _c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_u32, _c_vp, _c_size, _c_int,
        _c_vp, _c_vp, _c_vp, _c_size, _c_vp,
    ],
    "mc_checksum32_encode_fused": [
        _c_int, _c_vp, _c_vp, _c_size, _c_u32, _c_vp, _c_size, _c_int, _c_vp, _c_vp, _c_size, _c_vp, _c_vp,
    ],
    "mc_checksum32_verify_fused": [
        _c_int, _c_vp, _c_size, _c_u32, _c_vp, _c_size, _c_int, _c_vp, _c_u32, _c_vp, _c_size, _c_vp, _c_vp,
    ],
    "mc_stream_synchronize": [_c_vp],
    "mc_host_device_pointer": [_c_vp],
    "mc_verdict_alloc": [],
    "mc_verdict_free": [_c_vp],
    "mc_verdict_wait": [_c_vp, _c_u32, _c_vp],
    "mc_packbits": [_c_vp, _c_vp, _c_size, _c_vp],
    "mc_copy": [_c_vp, _c_vp, _c_size, _c_vp],
    "mc_copy_rows": [_c_vp, _c_size, _c_vp, _c_size, _c_size, _c_size, _c_vp],
    "mc_blosc_filter": [_c_vp, _c_vp, _c_size, _c_size, _c_size, _c_int, _c_int, _c_vp],
    "mc_unpackbits": [_c_vp, _c_size, _c_vp, _c_size, _c_vp],
}
_RESTYPES = {
    "mc_host_device_pointer": ctypes.c_void_p,
    "mc_verdict_alloc": ctypes.c_void_p,
    "mc_verdict_free": None,
    "mc_strerror": ctypes.c_char_p,
    "mc_delta_decode_workspace": ctypes.c_size_t,
    "mc_delta_decode_batch_workspace": ctypes.c_size_t,
    "mc_fletcher32_workspace": ctypes.c_size_t,
    "mc_fletcher32_batch_workspace": ctypes.c_size_t,
    "mc_shuffle_fletcher32_workspace": ctypes.c_size_t,
    "mc_fso_delta_shuffle_decode_workspace": ctypes.c_size_t,
    "mc_fso_delta_shuffle_decode_batch_workspace": ctypes.c_size_t,
    "mc_checksum32_workspace": ctypes.c_size_t,
}

EXPORTED = tuple(_SIGNATURES)

_lock = threading.Lock()
_lib = None
_load_error: Exception | None = None


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(lib_path):
            _load_error = MCodecError(
                f"libmcodec.so not found at {lib_path}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C numcodecs_amd/csrc)"
            )
            raise _load_error
        handle = ctypes.CDLL(lib_path)
        missing = []
        for name, argtypes in _SIGNATURES.items():
            try:
                fn = getattr(handle, name)
            except AttributeError:
                missing.append(name)
                continue
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        if missing:
            _load_error = MCodecError(f"libmcodec.so is missing symbols: {missing}")
            raise _load_error
        _lib = handle
        return _lib


class _LibProxy:
    """Attribute access loads the library on first use (import stays cheap)."""

    def __getattr__(self, name):
        # only reached on the first access of `name`: the function object is
        # then cached on the proxy (a plain attribute hit per call afterwards)
        fn = getattr(_load(), name)
        self.__dict__[name] = fn
        return fn


lib = _LibProxy()


def check(status: int, what: str = "mcodec") -> None:
    """Raise MCodecError for a non-zero libmcodec status."""
    if status != MC_OK:
        msg = lib.mc_strerror(status)
        msg = msg.decode() if msg else "unknown"
        raise MCodecError(f"{what} failed with status {status}: {msg}")


def available() -> bool:
    """True when the library loads and a HIP device is visible to it."""
    try:
        _load()
    except Exception:
        return False
    return torch.cuda.is_available()


_device_ok = False


def require_device() -> None:
    """Fail loudly when there is no HIP device: no CPU fallback exists."""
    global _device_ok
    if _device_ok:
        return
    _load()
    if torch.cuda.is_available():
        _device_ok = True
    else:
        raise MCodecError(
            "numcodecs_amd requires a HIP device (MI355X/gfx950); none is visible. "
            "There is no CPU fallback in the product path."
        )


def stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream on `device` (as an int)."""
    return torch.cuda.current_stream(device).cuda_stream
