"""The one-launch CRC verify (ride finish, round 6) of 256 MiB + 4 bytes at
location "start" through the lab library's copy of
mc_checksum32_verify_fused, over the checksum-only grid cap (sched field
ck_grid): back-to-back launches (10 between one event pair) and single
launches (event pair around each, stream idle before), interleaved rounds.
One JSON line per (kind, grid).

Usage: python tools/probe_ck_verify_grid6.py   (CK_ADLER=1: Adler32 instead;
CK_KSWEEP=1: 16, 32 and 64 KiB tiles)"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import _native  # noqa: E402

lab = _lab()
V, S, I, U = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32
lab.mc_checksum32_verify_fused.argtypes = [I, V, S, U, V, S, I, V, U, V, S, V, V]
lab.mc_checksum32_verify_fused.restype = I
lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, I]
lab.mc_lab_set_sched.restype = I
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
NB = 256 * MiB + 4
bufs = [torch.randint(0, 256, (NB,), dtype=torch.uint8, device=dev) for _ in range(2)]
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)
rec = torch.zeros(4, dtype=torch.int32, device=dev)


def ver(kind, i):
    rc = lab.mc_checksum32_verify_fused(kind, bufs[i].data_ptr(), NB, 0, None, 0, _native.MC_CK_START,
                                        rec.data_ptr(), 0, ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
    assert rc == 0, rc


def b2b(fn, reps=10):
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        fn(r % 2)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def single(fn, reps=10):
    ts = []
    for r in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(r % 2)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


KINDS = ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C"))
GRIDS = (512, 768, 1024, 1536, 2048)
KS = (0,)  # ck_k: 0 = the product's tile size
if os.environ.get("CK_ADLER") == "1":  # Adler32's one-launch verify over its grid cap
    KINDS = ((_native.MC_CK_ADLER32, "Adler32"),)
    GRIDS = (512, 1024, 2048, 4096)
if os.environ.get("CK_KSWEEP") == "1":  # 16 / 32 KiB tiles too (fewer registers: 4 / 3 waves per SIMD)
    GRIDS = (512, 768, 1024)
    KS = (4, 8, 16)
    if os.environ.get("CK_ADLER") == "1":
        GRIDS, KS = (1024, 2048, 4096), (8, 16)
res = {}
ref = {}
for rnd in range(4):
    for kind, name in KINDS:
        for g, kk in [(g, kk) for g in GRIDS for kk in KS]:
            lab.mc_lab_set_sched(b"ck_grid", g)
            lab.mc_lab_set_sched(b"ck_k", kk)
            ver(kind, 0)
            torch.cuda.synchronize()
            got = tuple(int(v) for v in rec[:2].cpu())
            assert ref.setdefault(name, got) == got, (name, g)
            res.setdefault((name, g, kk, "b2b"), []).append(b2b(lambda i: ver(kind, i)))
            res.setdefault((name, g, kk, "single"), []).append(single(lambda i: ver(kind, i)))
lab.mc_lab_set_sched(b"ck_grid", 0)
lab.mc_lab_set_sched(b"ck_k", 16)
for (name, g, kk, mode), ts in res.items():
    ts.sort()
    print(json.dumps({"probe": "ck_verify_grid6", "kind": name, "ck_grid": g, "ck_k": kk or 16, "mode": mode,
                      "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}), flush=True)
assert not ticket.any()
