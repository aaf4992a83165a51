"""Fletcher32's one-launch verify of 256 MiB + 4 bytes through the lab
library's copy of mc_fletcher32_verify_fused over its schedule fields
(f32_fused_grid x f32_slice_kb), back-to-back and single launches,
interleaved rounds.  One JSON line per setting.

Usage: python tools/probe_f32_verify_sched.py"""
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
lab.mc_fletcher32_verify_fused.argtypes = [V, S, V, U, V, S, V, V]
lab.mc_fletcher32_verify_fused.restype = I
lab.mc_fletcher32_workspace.argtypes = [S]
lab.mc_fletcher32_workspace.restype = S
lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, I]
lab.mc_lab_set_sched.restype = I
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
NB = 256 * MiB + 4
bufs = [torch.randint(0, 256, (NB,), dtype=torch.uint8, device=dev) for _ in range(2)]
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(64 * MiB, dtype=torch.uint8, device=dev)
rec = torch.zeros(4, dtype=torch.int32, device=dev)


def ver(i):
    rc = lab.mc_fletcher32_verify_fused(bufs[i].data_ptr(), NB, rec.data_ptr(), 0, ws.data_ptr(), ws.numel(),
                                        ticket.data_ptr(), st)
    assert rc == 0, rc


def b2b(reps=10):
    ver(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        ver(r % 2)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def single(reps=10):
    ts = []
    for r in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ver(r % 2)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


assert lab.mc_fletcher32_workspace(NB - 4) <= ws.numel()
res, ref = {}, None
for rnd in range(4):
    for g in (1024, 2048, 4096, 8192):
        for kb in (16, 32, 64):
            lab.mc_lab_set_sched(b"f32_fused_grid", g)
            lab.mc_lab_set_sched(b"f32_slice_kb", kb)
            ver(0)
            torch.cuda.synchronize()
            got = tuple(int(v) for v in rec[:2].cpu())
            ref = ref or got
            assert got == ref, (g, kb)
            res.setdefault((g, kb, "b2b"), []).append(b2b())
            res.setdefault((g, kb, "single"), []).append(single())
lab.mc_lab_set_sched(b"f32_fused_grid", 4096)
lab.mc_lab_set_sched(b"f32_slice_kb", 32)
for (g, kb, mode), ts in res.items():
    ts.sort()
    print(json.dumps({"probe": "f32_verify_sched", "f32_fused_grid": g, "f32_slice_kb": kb, "mode": mode,
                      "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}), flush=True)
assert not ticket.any()
