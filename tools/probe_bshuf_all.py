"""Blosc BITSHUFFLE filter, 256 MiB, 256 KiB blocks, typesize 1/2/4/8:
encode / decode µs (HIP events, 3 rotating buffers, best of 3 x 10) and the
fraction of 8 TB/s for 2N bytes; round trip checked.
Usage: python tools/probe_bshuf_all.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import blosc_shuffle as bsh  # noqa: E402

N = 256 << 20
dev = torch.device("cuda:0")
xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(3)]


def timed(fn):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(10):
            fn(i % 3)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) * 100.0
        best = t if best is None else min(best, t)
    return best


for ts in (1, 2, 4, 8):
    fw = [bsh.shuffle(x, ts, 256 * 1024, bsh.BITSHUFFLE) for x in xs]
    ok = torch.equal(bsh.unshuffle(fw[0], ts, 256 * 1024, bsh.BITSHUFFLE).view(torch.uint8).reshape(-1), xs[0])
    te = timed(lambda i: bsh.shuffle(xs[i], ts, 256 * 1024, bsh.BITSHUFFLE))
    td = timed(lambda i: bsh.unshuffle(fw[i], ts, 256 * 1024, bsh.BITSHUFFLE))
    print(json.dumps({"probe": "bitshuffle", "typesize": ts, "enc_us": round(te, 1), "dec_us": round(td, 1),
                      "enc_frac": round(2 * N / (te * 1e-6) / 8e12, 4), "dec_frac": round(2 * N / (td * 1e-6) / 8e12, 4),
                      "round_trip": ok}), flush=True)
