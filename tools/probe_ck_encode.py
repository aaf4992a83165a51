"""The one-launch CRC32 / CRC32C encode (payload copy + footer, 256 MiB)
through the lab library's copy of mc_checksum32_encode_fused, with the
payload stores nontemporal or plain (sched field ck_fused_plain) at both
footer locations: "start" puts the payload at dst + 4 (dword-aligned stores
either way), "end" at the 16-B aligned dst.  Interleaved rounds, outputs
compared with the product library's.  One JSON line per case.

Usage: python tools/probe_ck_encode.py   (CK_SWEEP=1: the copying pass's tile
size x grid instead; CK_SWEEP_K4=1: 16 / 32 KiB tiles x 768-1536 workgroups)"""
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
lab.mc_checksum32_encode_fused.argtypes = [I, V, V, S, U, V, S, I, V, V, S, V, V]
lab.mc_checksum32_encode_fused.restype = I
lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, I]
lab.mc_lab_set_sched.restype = I
lib = _native.lib
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
N = 256 * MiB
srcs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(2)]
dsts = [torch.empty(N + 4, dtype=torch.uint8, device=dev) for _ in range(2)]
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)


def enc(L, kind, loc, i):
    rc = L.mc_checksum32_encode_fused(kind, srcs[i].data_ptr(), dsts[i].data_ptr(), N, 0, None, 0, loc, None,
                                      ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
    assert rc == 0, rc


def timed(fn, reps=10):
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        fn(r % 2)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


SWEEP = os.environ.get("CK_SWEEP") == "1"
KCS, GRIDS = (8, 16), (512, 1024, 2048)
if os.environ.get("CK_SWEEP_K4") == "1":  # 16 KiB tiles (four waves per SIMD) against 32 KiB
    SWEEP, KCS, GRIDS = True, (4, 8), (768, 1024, 1536)
if SWEEP:  # tile size and grid of the copying pass, nontemporal stores
    res = {}
    for rnd in range(3):
        for kind, name in ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C")):
            for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
                for kc in KCS:
                    for g in GRIDS:
                        lab.mc_lab_set_sched(b"ck_kcopy", kc)
                        lab.mc_lab_set_sched(b"ck_grid_copy", g)
                        t = timed(lambda i: enc(lab, kind, loc, i))
                        res.setdefault((name, loc_name, kc, g), []).append(t)
    lab.mc_lab_set_sched(b"ck_kcopy", 8)
    lab.mc_lab_set_sched(b"ck_grid_copy", 1024)
    for (name, loc_name, kc, g), ts in res.items():
        ts.sort()
        print(json.dumps({"probe": "ck_encode_sweep", "kind": name, "location": loc_name, "ck_kcopy": kc,
                          "ck_grid_copy": g, "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}),
              flush=True)
    sys.exit(0)

res = {}
for rnd in range(5):
    for kind, name in ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C")):
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            for plain in (0, 1):
                assert lab.mc_lab_set_sched(b"ck_fused_plain", plain) != -2 ** 31
                t = timed(lambda i: enc(lab, kind, loc, i))
                res.setdefault((name, loc_name, plain), []).append(t)
                if rnd == 0:
                    enc(lab, kind, loc, 0)
                    got = dsts[0].clone()
                    enc(lib, kind, loc, 0)
                    assert torch.equal(got, dsts[0]), (name, loc_name, plain)
lab.mc_lab_set_sched(b"ck_fused_plain", 0)
for (name, loc_name, plain), ts in res.items():
    ts.sort()
    print(json.dumps({"probe": "ck_encode", "kind": name, "location": loc_name, "plain_stores": plain,
                      "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}), flush=True)
assert not ticket.any()
