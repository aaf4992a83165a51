"""The int16 Delta decode's reduce pass over 256 MiB (tools/lab/lab_dscan_reduce.hip):
one workgroup per 4 tiles (the product's shape) against a persistent grid
that prefetches the next group, back-to-back launches, interleaved rounds;
tile and group totals compared.  One JSON line per variant.

Usage: python tools/probe_dscan_reduce.py"""
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
V, S, I, U = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
lab.mc_lab_dscan_reduce.argtypes = [V, S, V, V, I, U, V]
lab.mc_lab_dscan_reduce.restype = I
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
N = 256 << 20
srcs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(2)]
ntiles = N // 8192
ws = torch.zeros(ntiles + 64, dtype=torch.int32, device=dev)
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)


def run(persist, grid, i):
    rc = lab.mc_lab_dscan_reduce(srcs[i].data_ptr(), N, ws.data_ptr(), ticket.data_ptr(), persist, grid, st)
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


VARIANTS = [(0, 0)] + [(1, g) for g in (768, 1024, 1536, 1792, 2048, 3584)]
run(0, 0, 0)
torch.cuda.synchronize()
ref = ws.clone()
res = {}
for rnd in range(5):
    for p, g in VARIANTS:
        if rnd == 0:
            ws.zero_()
            run(p, g, 0)
            torch.cuda.synchronize()
            assert torch.equal(ws, ref), (p, g)
        res.setdefault((p, g), []).append(b2b(lambda i: run(p, g, i)))
for (p, g), ts in res.items():
    ts.sort()
    print(json.dumps({"probe": "dscan_reduce", "persistent": p, "grid": g or ntiles // 4,
                      "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}), flush=True)
assert not ticket.any()
