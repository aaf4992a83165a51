"""JenkinsLookup3 on the GPU: one 16 MiB chunk (one serial chain) and a batch
of 2048 x 1 MiB chunks (one chain per chunk), public API on device tensors,
encode + decode verified against the oracle; ms per call (HIP events).
Usage: python tools/probe_jenkins.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from numcodecs_amd import JenkinsLookup3, chunks  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(3)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


codec = JenkinsLookup3()
small = torch.randint(0, 256, (65536 + 7,), dtype=torch.uint8, generator=g)
ok = codec.encode(small.to(dev)).cpu().numpy().tobytes() == oracle.jenkins_encode(small.numpy())
x = torch.randint(0, 256, (16 << 20,), dtype=torch.uint8, generator=g).to(dev)
t1 = timed(lambda: codec.encode(x), 3)
print(json.dumps({"probe": "jenkins", "case": "one 16 MiB chunk", "encode_ms": round(t1, 2), "oracle_ok_64KiB": ok,
                  "GBps": round((16 << 20) / (t1 * 1e-3) / 1e9, 3)}), flush=True)
rows = torch.randint(0, 256, (2048, 1 << 20), dtype=torch.uint8, generator=g).to(dev)
t2 = timed(lambda: chunks.encode_chunks([codec], rows), 3)
print(json.dumps({"probe": "jenkins", "case": "2048 x 1 MiB batch", "encode_ms": round(t2, 3),
                  "GBps": round(2048 * (1 << 20) / (t2 * 1e-3) / 1e9, 2)}), flush=True)
