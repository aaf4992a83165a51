"""Shuffle(4) / Shuffle(8) on 256 MiB: the default schedules against the same
layouts with default-policy (temporal) loads and stores (V_NO_NT = 8), via
tools/lab's mc_lab_shuffle_variant; 4 rotating buffer sets, event-timed,
two interleaved rounds; outputs checked against the default variant.  One
JSON line of GB/s (read + write bytes)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import _ops  # noqa: E402

lab = _lab()
fn = lab.mc_lab_shuffle_variant
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
               ctypes.c_int, ctypes.c_void_p]
fn.restype = ctypes.c_int
dev = torch.device("cuda:0")
N = 256 << 20
sets = 4
ins = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(sets)]
outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(sets)]
st = _ops.stream(ins[0])
CASES = {  # (es, encode): variants (first = the library default)
    (8, 1): [5, 13, 21, 29, 133, 141],
    (8, 0): [21, 29, 5, 13],
    (4, 1): [129, 137, 257, 265, 17, 25],
    (4, 0): [21, 29, 5, 13],
}
res = {}
ref = {}
for rnd in range(2):
    for (es, enc), vs in CASES.items():
        for v in vs:
            def run(i):
                rc = fn(ins[i].data_ptr(), outs[i].data_ptr(), N, es, enc, v, 0, st)
                assert rc == 0, (es, enc, v, rc)
            for i in range(sets):
                run(i)
            torch.cuda.synchronize()
            key = (es, enc)
            h = outs[0][:: 4093].clone()
            if key not in ref:
                ref[key] = h
            ok = bool(torch.equal(h, ref[key]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for r in range(20):
                run(r % sets)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            res.setdefault(f"es{es}_{'enc' if enc else 'dec'}_v{v}", []).append(
                {"GBps": round(2 * N / us / 1e3, 1), "ok": ok})
print(json.dumps(res), flush=True)
