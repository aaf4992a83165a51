"""Blosc BITSHUFFLE kernels alone (typesize 4 and 8, 256 KiB blocks, 256 MiB),
a few launches each -- the program rocprofv3 --pmc / --kernel-trace passes run.
Usage: python tools/probe_bshuf.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import blosc_shuffle as bsh  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
N = 256 << 20
x = torch.randint(0, 256, (N,), dtype=torch.uint8, device="cuda:0")
for ts in (4, 8):
    fw = bsh.shuffle(x, ts, 256 * 1024, bsh.BITSHUFFLE)
    for _ in range(reps):
        bsh.shuffle(x, ts, 256 * 1024, bsh.BITSHUFFLE)
        bsh.unshuffle(fw, ts, 256 * 1024, bsh.BITSHUFFLE)
torch.cuda.synchronize()
print("done", flush=True)
