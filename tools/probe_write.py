"""Write-dominated streams on 256 MiB: torch's fill (a write-only kernel)
against PackBits decode (N/8 read + N written) through the public API and
the bare C ABI, event-timed medians over rotating buffers.  One JSON line."""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import PackBits  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(3)]
bools = torch.randint(0, 2, (N,), dtype=torch.bool, device=dev)
enc = PackBits().encode(bools)
st = torch.cuda.current_stream().cuda_stream


def timed(fn, reps=20):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    ts = []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(reps):
            fn(i % 3)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return round(statistics.median(ts), 2)


res = {"fill_us": timed(lambda i: outs[i].fill_(7))}
res["fill_TBps"] = round(N / res["fill_us"] / 1e6, 3)
res["unpack_abi_us"] = timed(lambda i: lib.mc_unpackbits(enc.data_ptr(), enc.numel(), outs[i].data_ptr(), N, st))
res["unpack_TBps"] = round((N + N // 8) / res["unpack_abi_us"] / 1e6, 3)
ok = bool(torch.equal(outs[0].view(torch.bool), bools))
res["ok"] = ok
print(json.dumps(res), flush=True)
