"""Host-side cost of one codec call on a small device chunk: wall time per
call and a cProfile of the Python path (where the ~14 us go)."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Shuffle  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(16384, device=dev)
out = torch.empty(65536, dtype=torch.uint8, device=dev)
c = Shuffle(4)
for _ in range(100):
    c.encode(x, out=out)
torch.cuda.synchronize()
N = 2000
t0 = time.perf_counter()
for _ in range(N):
    c.encode(x, out=out)
torch.cuda.synchronize()
print(f"encode(out=) {1e6 * (time.perf_counter() - t0) / N:.1f} us/call")
t0 = time.perf_counter()
for _ in range(N):
    c.encode(x)
torch.cuda.synchronize()
print(f"encode() {1e6 * (time.perf_counter() - t0) / N:.1f} us/call")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    c.encode(x)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
print(s.getvalue())
