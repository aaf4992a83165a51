"""Shared checks, restating the behaviour of the reference's test harness
(tests/common.py:31-243 of numcodecs) for numcodecs_amd codecs."""

from __future__ import annotations

import array
import json
import os
from glob import glob

import numpy as np
from numpy.testing import assert_array_almost_equal, assert_array_equal

import numcodecs_amd
from numcodecs_amd import get_codec
from numcodecs_amd.compat import ensure_bytes, ensure_ndarray

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURE = os.path.join(GOLDEN, "reference_fixture")


def compare_arrays(arr, res, precision=None):
    """common.py:31-48: view `res` as arr.dtype, reshape, compare."""
    res = np.asarray(ensure_ndarray(res)).view(arr.dtype)
    res = res.reshape(arr.shape, order="F" if arr.flags.f_contiguous else "C")
    if precision is None:
        assert_array_equal(arr, res)
    else:
        assert_array_almost_equal(arr, res, decimal=precision)


def check_encode_decode(arr, codec, precision=None):
    """common.py:51-116: round trip through every buffer flavour."""
    enc = codec.encode(arr)
    compare_arrays(arr, codec.decode(enc), precision)
    raw = arr.tobytes(order="A")
    for buf in (raw, bytearray(raw), array.array("b", raw)):
        enc = codec.encode(buf)
        compare_arrays(arr, codec.decode(enc), precision)
    enc_bytes = ensure_bytes(enc)
    for buf in (enc_bytes, bytearray(enc_bytes), array.array("b", enc_bytes),
                np.frombuffer(enc_bytes, dtype="u1")):
        compare_arrays(arr, codec.decode(buf), precision)
    out = np.empty_like(arr)
    codec.decode(enc_bytes, out=out)
    compare_arrays(arr, out, precision)
    out = bytearray(arr.nbytes)
    codec.decode(enc_bytes, out=out)
    compare_arrays(arr, out, precision)


def check_config(codec):
    """common.py:154-158."""
    config = json.loads(json.dumps(codec.get_config()))
    assert codec == get_codec(config)


def check_repr(stmt):
    """common.py:161-165 (names resolved in numcodecs_amd)."""
    ns = {name: getattr(numcodecs_amd, name) for name in numcodecs_amd.__all__}
    assert repr(eval(stmt, ns)) == stmt


def load_fixture_array(fn):
    return np.load(fn, allow_pickle=False)


def fixture_cases(codec_id, prefix=None):
    """Yield (arr, j, config, encoded_bytes) for every stored fixture file
    (common.py:168-243 layout: array.NN.npy, codec.MM/config.json,
    codec.MM/encoded.NN.dat).  Read-only: nothing is ever written."""
    d = os.path.join(FIXTURE, codec_id, prefix) if prefix else os.path.join(FIXTURE, codec_id)
    for arr_fn in sorted(glob(os.path.join(d, "array.*.npy"))):
        i = int(arr_fn.split(".")[-2])
        arr = load_fixture_array(arr_fn)
        for codec_dir in sorted(glob(os.path.join(d, "codec.*"))):
            j = int(codec_dir.split(".")[-1])
            with open(os.path.join(codec_dir, "config.json")) as f:
                config = json.load(f)
            with open(os.path.join(codec_dir, f"encoded.{i:02d}.dat"), "rb") as f:
                enc = f.read()
            yield arr, j, config, enc


def load_vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        manifest = json.load(f)
    data = np.load(os.path.join(GOLDEN, "vectors.npz"), allow_pickle=False)
    return manifest, data


def vec(data, family, i, key):
    return data[f"{family}__{i}__{key}"]


def lab_lib():
    """libmcodec_lab.so (tools/lab): the product objects plus the measured and
    rejected alternative schedules, which these tests keep byte-identical."""
    import sys

    tools = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    import pytest
    from lab.lablib import LAB_PATH, lab

    check_lab_build()
    if not os.path.exists(LAB_PATH):  # optional: the product never needs it
        pytest.skip(f"lab library not built ({LAB_PATH}); `make -C tools/lab`")
    return lab()


def check_lab_build():
    """Fail (not skip) when __graft_entry__.build() recorded a failed lab build."""
    import pytest

    marker = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "_build",
                          "LAB_BUILD_FAILED")
    if os.path.exists(marker):
        with open(marker) as f:
            pytest.fail(f"the lab library failed to build: {f.read().strip()}")


def value_mask(dtype, nbytes: int) -> np.ndarray:
    """Boolean byte mask of the bytes numpy defines for `nbytes` of `dtype`:
    every byte, except the 6 padding bytes of each longdouble (component),
    which numpy leaves as whatever its output buffer held ('<f16' bytes
    10-15, '>f16' bytes 0-5; '<c32' / '>c32' per 16-byte component)."""
    dt = np.dtype(dtype)
    mask = np.ones(nbytes, dtype=bool)
    if (dt.kind == "f" and dt.itemsize == 16) or (dt.kind == "c" and dt.itemsize == 32):
        m = mask.reshape(-1, 16)
        if dt.byteorder == ">":
            m[:, :6] = False
        else:
            m[:, 10:] = False
    return mask


def same_values(got: bytes, want: bytes, dtype) -> bool:
    """got == want on the bytes numpy defines for `dtype` (value_mask)."""
    if len(got) != len(want):
        return False
    g = np.frombuffer(got, dtype=np.uint8)
    w = np.frombuffer(want, dtype=np.uint8)
    m = value_mask(dtype, len(g))
    return bool(np.array_equal(g[m], w[m]))


def delta_decode_both_schedules(src, dst, n, a, d, ws_n):
    """mc_delta_decode of device bytes `src` into `dst` twice: with a fresh
    arrival ticket (the product's schedule: the float decode's tile prefixes
    folded into its reduce pass) and without one (the HIP-graph-capture
    schedule, k_fspec_pre).  Both must give the same bytes (numpy's); the
    ticket must be left zero.  The first-failure word (the workspace's last
    word; the ticket schedule's is returned, None without a workspace) is
    where the speculation's candidates first missed, and the two schedules
    add the tile prefixes in different orders, so on inexact data they may
    miss at different tiles -- but a chunk that verifies entirely under one
    verifies under the other."""
    import torch

    from numcodecs_amd import _native, _ops

    out, words = [], []
    for with_ticket in (True, False):
        ws = torch.zeros(max(ws_n // 8, 1), dtype=torch.int64, device=src.device)
        ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=src.device)
        dst.fill_(0xA5 if dst.dtype == torch.uint8 else 0)
        _native.check(_native.lib.mc_delta_decode(src.data_ptr(), dst.data_ptr(), n, a, d,
                                                  ws.data_ptr() if ws_n else None, ws_n,
                                                  ticket.data_ptr() if with_ticket else None, _ops.stream(src)),
                      "mc_delta_decode")
        torch.cuda.synchronize()
        assert int(ticket.abs().sum()) == 0, "arrival ticket not left zero"
        out.append(dst.cpu().numpy().tobytes())
        words.append(int(ws[-1].item()) if ws_n else None)
    assert out[0] == out[1], "ticket / ticket-free schedules differ"
    assert (words[0] == n) == (words[1] == n), words
    return words[0]
