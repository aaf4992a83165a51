"""Every non-default schedule of the product kernels, checked against the
oracle (run by tests/test_gpu_sched.py in ONE child process).

The product library reads no environment: its schedule parameters
(numcodecs_amd/csrc/mc_sched.h) are fixed at the measured defaults.  The lab
library (tools/lab, the product objects + tools/lab/lab_sched.hip) can
change them, so this script runs the public codecs on top of the lab library
(NUMCODECS_AMD_LIB set by the parent), walks every field through its
alternative values with mc_lab_set_sched, and compares each result with the
oracle byte for byte.  Prints one JSON line: {"ok": bool, "cases": [...]}.
"""

from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from numcodecs_amd import (  # noqa: E402
    CRC32,
    CRC32C,
    Adler32,
    Delta,
    FixedScaleOffset,
    Fletcher32,
    Shuffle,
    _native,
    batch,
    chunks,
)
from tests import oracle_chain  # noqa: E402

dev = torch.device("cuda:0")
lab = ctypes.CDLL(_native.lib_path)  # the same handle the codecs use
lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, ctypes.c_int]
lab.mc_lab_set_sched.restype = ctypes.c_int
rng = np.random.default_rng(7)


def _h(t):
    return t.contiguous().view(torch.uint8).reshape(-1).cpu().numpy().tobytes()


def check_copy():
    x = rng.integers(0, 256, (1 << 22) + 5, dtype=np.uint8)
    out = _h(Shuffle(1).encode(torch.from_numpy(x).to(dev)))  # es <= 1: mc_copy
    return out == x.tobytes()


def check_checksums():
    ok = True
    for n in ((1 << 22) + 7, 3 << 20, 1000):
        x = rng.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(dev)
        for codec, cid in ((CRC32(), "crc32"), (CRC32C(), "crc32c"), (Adler32(), "adler32")):
            enc = codec.encode(xd)
            ok &= _h(enc) == oracle.checksum32_encode(cid, x).tobytes()
            ok &= _h(codec.decode(enc)) == x.tobytes()
    rows = torch.from_numpy(rng.integers(0, 256, (6, 1 << 20), dtype=np.uint8)).to(dev)
    for cid in ("crc32", "crc32c", "adler32"):
        enc = batch.checksum32_encode_chunks(rows, cid)
        eh = enc.cpu().numpy()
        for i in range(6):
            ok &= eh[i].tobytes() == oracle.checksum32_encode(cid, rows[i].cpu().numpy()).tobytes()
        dec, sums, stored = batch.checksum32_decode_chunks(enc, cid)
        ok &= bool(torch.equal(dec, rows)) and bool(torch.equal(sums, stored))
    return ok


def check_fletcher32():
    ok = True
    for n in ((1 << 22) + 6, 1 << 24, 999):
        x = rng.integers(0, 256, n, dtype=np.uint8)
        xd = torch.from_numpy(x).to(dev)
        enc = Fletcher32().encode(xd)
        ok &= _h(enc) == oracle.fletcher32_encode(x)
        ok &= _h(Fletcher32().decode(enc)) == x.tobytes()
    rows = torch.from_numpy(rng.integers(0, 256, (5, 1 << 20), dtype=np.uint8)).to(dev)
    enc = batch.fletcher32_encode_chunks(rows)
    eh = enc.cpu().numpy()
    for i in range(5):
        ok &= eh[i][: (1 << 20) + 4].tobytes() == oracle.fletcher32_encode(rows[i].cpu().numpy())
    dec, sums, stored = batch.fletcher32_decode_chunks(enc)
    ok &= bool(torch.equal(dec, rows)) and bool(torch.equal(sums, stored))
    return ok


_C4 = [FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"), Delta(dtype="<i2"), Shuffle(2)]


def check_c4_batch():
    b, n = 8, (1 << 21) + 96
    xh = (1000.0 + rng.uniform(-15, 15, (b, n))).astype("<f4")
    enc = chunks.encode_chunks(_C4, torch.from_numpy(xh).to(dev))
    eh = enc.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    dh = chunks.decode_chunks(_C4, enc).contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    return all(dh[i].tobytes() == oracle_chain.chain_decode(_C4, eh[i].tobytes()) for i in range(b))


def check_delta_int():
    ok = True
    for dt in ("<i1", "<i2", "<i4", "<i8"):
        n = (1 << 24) // np.dtype(dt).itemsize + 3
        x = rng.integers(-100, 100, n).astype(dt)
        d = Delta(dtype=dt)
        enc = d.encode(torch.from_numpy(x).to(dev))
        ok &= _h(enc) == oracle.delta_encode(x, dt).tobytes()
        ok &= _h(d.decode(enc)) == oracle.delta_decode(oracle.delta_encode(x, dt), dt).tobytes()
    return ok


def check_delta_same_type():
    """k_delta_enc_same: every width, both byte orders, integers and floats"""
    ok = check_delta_int()
    for dt in ("<f4", ">f4", "<f8", ">i2", ">i8"):
        d = np.dtype(dt)
        n = (1 << 22) // d.itemsize + 5
        x = (rng.standard_normal(n) * 100).astype(d)
        enc = Delta(dtype=dt).encode(torch.from_numpy(x.view(np.uint8).copy()).to(dev))
        ok &= _h(enc) == oracle.delta_encode(x, dt).tobytes()
    return ok


def check_delta_float():
    ok = True
    for dt in ("<f4", "<f8"):
        n = (1 << 20) + 3
        x = (np.arange(n) * 0.25).astype(dt)  # every add exact: the speculation verifies
        y = rng.standard_normal(1 << 16).astype(dt)  # rounding from the start
        for v in (x, y):
            enc = oracle.delta_encode(v, dt)
            got = Delta(dtype=dt).decode(torch.from_numpy(np.ascontiguousarray(enc)).to(dev))
            ok &= _h(got) == oracle.delta_decode(enc, dt).tobytes()
    return ok


def check_fso():
    ok = True
    for scale in (1e3, 7.0, 0.1):
        x = rng.integers(-32768, 32768, 1 << 20).astype("<i2")
        f = FixedScaleOffset(offset=3, scale=scale, dtype="<f4", astype="<i2")
        got = f.decode(torch.from_numpy(x).to(dev))
        ok &= _h(got) == oracle.fso_decode(x, 3, scale, "<f4", "<i2").tobytes()
    return ok


def check_bitround_shuffle():
    """BitRound(k) + Shuffle(4) of one large chunk for every keepbits (each
    plane split of the mask) against the oracle."""
    from numcodecs_amd import BitRound, batch

    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(8 << 20, generator=g, dtype=torch.float32)
    xh = x.numpy()
    xd = x.to(dev)
    ok = True
    for k in (0, 1, 7, 8, 9, 10, 15, 16, 22):
        got = batch.FilterPipeline([BitRound(k), Shuffle(4)]).encode(xd)
        ok &= _h(got) == oracle.shuffle(oracle.bitround_encode(xh, k), 4).tobytes()
    return ok


# field -> (alternative values, check)
PLAN = {
    "copy_u": ([8], check_copy),
    "copy_grid": ([64, 2048], check_copy),
    "ck_k": ([4, 8, 16], check_checksums),
    "ck_kcopy": ([4, 16], check_checksums),
    "ck_grid": ([256, 1024], check_checksums),
    "ck_grid_copy": ([128, 4096], check_checksums),
    "f32_unroll": ([1, 4, 8], check_fletcher32),
    "f32_ntld": ([0], check_fletcher32),
    "f32_fused_grid": ([256, 65536], check_fletcher32),
    "f32_slice_kb": ([4, 128], check_fletcher32),
    "c4_group_mi": ([1, 4], check_c4_batch),
    "delta_enc_vec": ([0], check_delta_int),
    "dscan": ([0], check_delta_int),
    "dscan_nt": ([0, 1, 3], check_delta_int),
    "fspec": ([0], check_delta_float),
    "fastdiv": ([0], check_fso),
    "crc_lds": ([1], check_checksums),
    "delta_enc_dv": ([8], check_delta_same_type),
    "br_planes": ([0], check_bitround_shuffle),
    "ck_fused_plain": ([1], check_checksums),
}


def main():
    cases = []
    for field, (values, fn) in PLAN.items():
        default = lab.mc_lab_set_sched(field.encode(), 0)
        lab.mc_lab_set_sched(field.encode(), default)
        assert default != -(1 << 31), field
        for v in [default] + values:
            lab.mc_lab_set_sched(field.encode(), v)
            try:
                ok = bool(fn())
                err = None
            except Exception as e:  # noqa: BLE001
                ok, err = False, f"{type(e).__name__}: {e}"
            torch.cuda.synchronize()
            cases.append({"field": field, "value": v, "default": v == default, "ok": ok, "error": err})
            print(f"{field}={v}: {'ok' if ok else 'FAIL ' + str(err)}", file=sys.stderr, flush=True)
        lab.mc_lab_set_sched(field.encode(), default)
    print(json.dumps({"ok": all(c["ok"] for c in cases), "cases": cases}), flush=True)


if __name__ == "__main__":
    main()
