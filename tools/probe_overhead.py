"""Host-side cost of one codec call on a small device chunk, layer by layer:
the bare ctypes call into libmcodec (pointers precomputed), _ops.shuffle,
and Shuffle.encode/decode(out=) through the public API; plus a cProfile of
the public path (where the microseconds go)."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Shuffle, _ops  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(262144, device=dev)  # 1 MiB (BASELINE C1)
out = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
back = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
c = Shuffle(4)
N = 4000


def rate(name, f):
    for _ in range(200):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        f()
    torch.cuda.synchronize()
    print(f"{name:32s} {1e6 * (time.perf_counter() - t0) / N:6.2f} us/call", flush=True)


xp, op, st = x.data_ptr(), out.data_ptr(), _ops.stream(x)
rate("ctypes mc_shuffle", lambda: lib.mc_shuffle(xp, op, 1 << 20, 4, st))
rate("_ops.stream", lambda: _ops.stream(x))
rate("_ops.shuffle", lambda: _ops.shuffle(x, out, 1 << 20, 4, True))
rate("Shuffle.encode(x, out=)", lambda: c.encode(x, out=out))
rate("Shuffle.decode(e, out=)", lambda: c.decode(out, out=back))
rate("Shuffle.encode(x)", lambda: c.encode(x))
assert torch.equal(back.view(torch.float32), x)
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    c.encode(x, out=out)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(20)
print(s.getvalue())
