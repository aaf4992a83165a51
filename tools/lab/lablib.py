"""ctypes binding of libmcodec_lab.so -- LAB ONLY (tools/, tests of the
rejected / sweep schedules).  The lab library is the product objects plus
tools/lab/*.hip; the product (numcodecs_amd, include/mcodec.h) never loads it.
"""

from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- the HIP runtime must be torch's (see numcodecs_amd/_native.py)

LAB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_build", "libmcodec_lab.so")

_V, _S, _I, _D = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_double
_SIGS = {
    "mc_lab_shuffle_variant": ([_V, _V, _S, _S, _I, _I, _I, _V], _I),
    "mc_lab_shuffle_batch_variant": ([_V, _S, _V, _S, _S, _S, _S, _I, _I, _I, _V], _I),
    "mc_lab_delta_decode_batch_variant": ([_V, _S, _V, _S, _S, _S, _I, _I, _I, _V], _I),
    "mc_lab_c4_decode_workspace": ([_S], _S),
    "mc_lab_c4_decode_variant": ([_V, _V, _S, _I, _I, _D, _D, _V, _S, _I, _V], _I),
    "mc_lab_delta_dec1p_state_bytes": ([_S, _I], _S),
    "mc_lab_c4_dec1p_state_bytes": ([_S, _I], _S),
    "mc_lab_delta_dec1p": ([_V, _V, _S, _I, _V, ctypes.c_uint, _V, _V], _I),
    "mc_lab_c4_dec1p": ([_V, _V, _S, _I, _I, _D, _D, _V, ctypes.c_uint, _V, _V], _I),
    "mc_lab_rocprim_scan_workspace": ([_S, _I], _S),
    "mc_lab_rocprim_scan": ([_V, _V, _S, _I, _V, _S, _V], _I),
    "mc_lab_shuffle4_enc": ([_V, _V, _S, _I, _V], _I),
    "mc_lab_bw_copy": ([_V, _V, _S, _I, _I, _I, _V], _I),
    "mc_lab_bitround_shuffle_variant": ([_V, _V, _S, _I, _I, _I, _I, _V], _I),
    "mc_lab_chain": ([_V, _V, _V, _I, _I, _I, _V], _I),
    "mc_lab_chain_g": ([_V, _V, _V, _I, _I, _I, _V, _V, _V], _I),
    "mc_lab_chain64": ([_V, _V, _V, _I, _I, _I, _V, _V, _V], _I),
    "mc_lab_stream": ([_V, _V, _S, _I, _I, _S, _S, _I, _V, _V], _I),
    "mc_lab_crc": ([_I, _V, _S, _I, _I, _I, ctypes.c_uint, _V, _V], _I),
    "mc_lab_crc_product": ([_I, _V, _S, _I, ctypes.c_uint, _V, _V], _I),
}
_lib = None
_bwcal = None
BWCAL_PATH = os.path.join(os.path.dirname(LAB_PATH), "libmcodec_bwcal.so")


def bwcal():
    """The copy calibration alone (`make -C tools/lab bwcal`: lab_bw.hip, the
    one lab entry bench.py's copy ceiling needs; it travels to the GPU box,
    the full lab library does not)."""
    global _bwcal
    if _bwcal is None:
        if not os.path.exists(BWCAL_PATH):
            raise FileNotFoundError(f"{BWCAL_PATH} missing: build it with `make -C tools/lab bwcal`")
        lib = ctypes.CDLL(BWCAL_PATH)
        args, res = _SIGS["mc_lab_bw_copy"]
        lib.mc_lab_bw_copy.argtypes = args
        lib.mc_lab_bw_copy.restype = res
        _bwcal = lib
    return _bwcal


def lab():
    """The loaded lab library (built by `make -C tools/lab`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LAB_PATH):
            raise FileNotFoundError(f"{LAB_PATH} missing: build it with `make -C tools/lab`")
        lib = ctypes.CDLL(LAB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
    return _lib
