"""The one-launch CRC verify at 256 MiB with the stored word at either end
(mc_checksum32_verify_fused): which loads of the few bytes outside the whole
tiles (the stored word, a tail past the tiles) cost the kernel time.  One
JSON line per case (median / best of 5 x 10 back-to-back launches).

Usage: python tools/probe_ck_tail.py"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from numcodecs_amd import _native  # noqa: E402

lib = _native.lib
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
buf = torch.randint(0, 256, (256 * MiB + 64 * 1024,), dtype=torch.uint8, device=dev)
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)
rec = torch.zeros(4, dtype=torch.int32, device=dev)


def timed(fn, reps=10, groups=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(groups):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return round(ts[len(ts) // 2], 2), round(ts[0], 2)


for kind, name in ((_native.MC_CK_CRC32C, "CRC32C"),):
    for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
        for enc in (256 * MiB + 4, 256 * MiB, 256 * MiB + 16, 256 * MiB + 20, 256 * MiB + 21):
            def ver():
                rc = lib.mc_checksum32_verify_fused(kind, buf.data_ptr(), enc, 0, None, 0, loc, rec.data_ptr(), 0,
                                                    ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
                assert rc == 0, rc
            med, best = timed(ver)
            print(json.dumps({"probe": "ck_tail", "kind": name, "location": loc_name, "encoded": enc,
                              "us_med": med, "us_best": best}), flush=True)
