"""Where does the host-streamed Zarr-chain decode spend its time?  Times the
device-only encode_chunks / decode_chunks of one 64 MiB slice and the
streamed host versions.  python tools/probe_chunks.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, BitRound, Shuffle, chunks  # noqa: E402

MiB = 1 << 20
dev = torch.device("cuda:0")
codecs = [BitRound(10), Shuffle(4), CRC32()]
x = torch.randn(15, MiB, device=dev)  # 15 x 4 MiB f32 chunks
res = {}


def wall(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


enc = chunks.encode_chunks(codecs, x)
res["dev_encode_ms"] = round(wall(lambda: chunks.encode_chunks(codecs, x)), 3)
res["dev_decode_ms"] = round(wall(lambda: chunks.decode_chunks(codecs, enc)), 3)
pending = []
res["dev_decode_deferred_ms"] = round(wall(lambda: chunks.decode_chunks(codecs, enc, pending)), 3)
for c in (codecs[::-1]):
    pass
# per step
x1 = enc
steps = {}
for c in codecs[::-1]:
    f = (lambda c=c, x1=x1: chunks._decode_step(c, x1, []))
    steps[type(c).__name__] = round(wall(f), 3)
    x1 = chunks._decode_step(c, x1, [])
res["decode_steps_ms"] = steps
hx = x.cpu().pin_memory().reshape(15, -1)
big = hx.repeat(32, 1).pin_memory()  # 480 chunks = 1.9 GiB
t0 = time.perf_counter()
henc = chunks.host_encode_chunks(codecs, big)
res["host_encode_GiBps"] = round(big.numel() * 4 / (1 << 30) / (time.perf_counter() - t0), 2)
out = torch.empty_like(big).pin_memory()
t0 = time.perf_counter()
chunks.host_decode_chunks(codecs, henc, out)
res["host_decode_GiBps"] = round(big.numel() * 4 / (1 << 30) / (time.perf_counter() - t0), 2)
print(json.dumps(res), flush=True)
