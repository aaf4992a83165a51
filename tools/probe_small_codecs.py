"""Host cost of one codec call per codec on a 1 MiB device chunk (the C1 chunk
size), against the bare launch of a libmcodec kernel: wall time per call of
encode and decode through the public API, back to back (the GPU work per call
is ~0.3 us of HBM time, so this is the host path).  One JSON line, then a
cProfile of the slowest codec's encode+decode."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import (  # noqa: E402
    CRC32, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, Quantize, Shuffle, _ops)
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(262144, device=dev) + 1000.0  # 1 MiB f4
N = 2000


def per_call(f):
    for _ in range(100):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        f()
    torch.cuda.synchronize()
    return round(1e6 * (time.perf_counter() - t0) / N, 2)


out = {}
o8 = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
xp, op, st = x.data_ptr(), o8.data_ptr(), _ops.stream(x)
out["bare_launch_us"] = per_call(lambda: lib.mc_shuffle(xp, op, 1 << 20, 4, st))
codecs = {
    "shuffle4": Shuffle(4),
    "bitround10": BitRound(10),
    "delta_f4": Delta(dtype="<f4"),
    "delta_i2": Delta(dtype="<i2"),
    "fso_f4_i2": FixedScaleOffset(offset=1000, scale=10, dtype="<f4", astype="<i2"),
    "quantize3": Quantize(digits=3, dtype="<f4"),
    "astype_f8": AsType(encode_dtype="<f8", decode_dtype="<f4"),
    "fletcher32": Fletcher32(),
    "crc32": CRC32(),
    "adler32": Adler32(),
}
xi2 = (torch.arange(524288, device=dev) % 1000).to(torch.int16)
for name, c in codecs.items():
    src = xi2 if name == "delta_i2" else x
    enc = c.encode(src)
    out[name] = {"enc_us": per_call(lambda: c.encode(src)), "dec_us": per_call(lambda: c.decode(enc))}
print(json.dumps(out), flush=True)
worst = max((k for k in codecs), key=lambda k: out[k]["enc_us"] + out[k]["dec_us"])
c = codecs[worst]
src = xi2 if worst == "delta_i2" else x
enc = c.encode(src)
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    c.decode(c.encode(src))
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(worst, s.getvalue())
