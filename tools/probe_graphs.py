"""Eager chunk pipeline vs its HIP-graph replay (numcodecs_amd.graphs) on
small batches, where issuing the kernels from Python dominates.  One JSON
line: microseconds per encode / decode of the whole batch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, BitRound, Shuffle, chunks  # noqa: E402
from numcodecs_amd.graphs import GraphChain  # noqa: E402

dev = torch.device("cuda:0")
codecs = [BitRound(10), Shuffle(4), CRC32()]
res = {}
for b, n in ((16, 16384), (64, 65536), (256, 262144)):
    x = torch.randn((b, n), device=dev)
    enc = chunks.encode_chunks(codecs, x)
    ge = GraphChain(codecs, x, "encode")
    gd = GraphChain(codecs, enc, "decode")

    def t(fn, reps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    key = f"{b}x{n * 4 // 1024}KiB"
    res[key] = {
        "eager_encode_us": round(t(lambda: chunks.encode_chunks(codecs, x)), 1),
        "graph_encode_us": round(t(lambda: ge()), 1),  # input written into ge.input by the producer
        "eager_decode_us": round(t(lambda: chunks.decode_chunks(codecs, enc)), 1),
        "graph_decode_us": round(t(lambda: gd()), 1),
    }
print(json.dumps(res), flush=True)
