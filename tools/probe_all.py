"""Every codec's device path on one 256 MiB chunk (3 rotating buffer sets so
no call finds its input in the 256 MiB Infinity Cache): encode / decode time
and the achieved rate of algorithmic HBM bytes (read + write) against the
8 TB/s peak.  One JSON line per codec; used for DESIGN.md's codec table."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import (  # noqa: E402
    CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, JenkinsLookup3, PackBits,
    Quantize, Shuffle,
)

dev = torch.device("cuda:0")
MiB = 1 << 20
N = 256 * MiB
SETS = 3
PEAK = 8000.0


def timed(fn, reps=12):
    for i in range(SETS):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % SETS)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def row(name, codec, make, enc_bytes, dec_bytes, decode=True):
    xs = [make() for _ in range(SETS)]
    encs = [codec.encode(x) for x in xs]
    te = timed(lambda i: codec.encode(xs[i]))
    r = {"codec": name, "encode_us": round(te * 1e6, 1), "encode_GBps": round(enc_bytes / te / 1e9, 1),
         "encode_frac": round(enc_bytes / te / 1e9 / PEAK, 3)}
    if decode:
        td = timed(lambda i: codec.decode(encs[i]))
        r.update({"decode_us": round(td * 1e6, 1), "decode_GBps": round(dec_bytes / td / 1e9, 1),
                  "decode_frac": round(dec_bytes / td / 1e9 / PEAK, 3)})
    print(json.dumps(r), flush=True)
    del xs, encs
    torch.cuda.empty_cache()


# ~0.5 s of back-to-back kernels first: the first rows otherwise run while
# the clock is still ramping
_w = torch.empty(N, dtype=torch.uint8, device=dev)
_o = torch.empty_like(_w)
for _ in range(2000):
    Shuffle(4).encode(_w, out=_o)
torch.cuda.synchronize()
del _w, _o

f4 = lambda: torch.randn(N // 4, device=dev)  # noqa: E731
f8 = lambda: torch.randn(N // 8, device=dev, dtype=torch.float64)  # noqa: E731
u8 = lambda: torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)  # noqa: E731
row("Shuffle(4) f4", Shuffle(4), f4, 2 * N, 2 * N)
row("Shuffle(8) f8", Shuffle(8), f8, 2 * N, 2 * N)
row("Shuffle(2) i2", Shuffle(2), lambda: torch.randint(-9, 9, (N // 2,), dtype=torch.int16, device=dev), 2 * N, 2 * N)
row("BitRound(10) f4", BitRound(10), f4, 2 * N, 0, decode=False)  # decode is a view
row("Delta(<i4)", Delta("<i4"), lambda: torch.randint(-9, 9, (N // 4,), dtype=torch.int32, device=dev), 2 * N, 2 * N)
row("Delta(<i2)", Delta("<i2"), lambda: torch.randint(-9, 9, (N // 2,), dtype=torch.int16, device=dev), 2 * N, 2 * N)
row("FixedScaleOffset(1000, 1e3, <f4 -> <i2)", FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
    lambda: 1000 + 10 * torch.rand(N // 4, device=dev), 1.5 * N, 1.5 * N)
row("Quantize(3, <f4)", Quantize(3, "<f4"), f4, 2 * N, 0, decode=False)  # decode is a view
row("Quantize(3, <f8 -> <f4)", Quantize(3, "<f8", "<f4"), f8, 1.5 * N, 1.5 * N)
row("AsType(<f4, <f8)", AsType("<f4", "<f8"), f8, 1.5 * N, 1.5 * N)
row("Fletcher32", Fletcher32(), u8, 2 * N + 4, N + 4)
row("CRC32", CRC32(), u8, 2 * N + 4, N + 4)
row("CRC32C", CRC32C(), u8, 2 * N + 4, N + 4)
row("Adler32", Adler32(), u8, 2 * N + 4, N + 4)
row("PackBits", PackBits(), lambda: torch.randint(0, 2, (N,), dtype=torch.uint8, device=dev).view(torch.bool),
    1.125 * N, 1.125 * N)
row("JenkinsLookup3 (one 16 MiB chunk)", JenkinsLookup3(), lambda: u8()[: 16 * MiB].clone(), 2 * 16 * MiB,
    16 * MiB, decode=True)
