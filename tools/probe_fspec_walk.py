"""Float Delta decode with rounding events: the walker (k_fspec_walk) on one
256 MiB chunk and on 2048 x 1 MiB rows, per data family; rotating buffers,
HIP events on the launch stream; one JSON line.  The first call of each case
is checked byte for byte against numpy's cumsum (the oracle's expression).

    python tools/probe_fspec_walk.py [f2|f4|f8] [MiB] [quick]   (KINDS=smooth,randn,... to select)
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, batch  # noqa: E402
from tests.test_gpu_delta_walk import family  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "f4"
mib = int(sys.argv[2]) if len(sys.argv) > 2 else 256
quick = len(sys.argv) > 3 and sys.argv[3] == "quick"  # single chunk only, no batches
npdt = np.dtype("<" + dt)
tdt = {"f2": torch.float16, "f4": torch.float32, "f8": torch.float64}[dt]
dev = torch.device("cuda", 0)
codec = Delta("<" + dt)


def timed(fn, reps):
    fn(0)
    torch.cuda.synchronize()
    ts = []
    for r in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(r)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


out = {"dtype": dt, "MiB": mib}
n = mib * (1 << 20) // npdt.itemsize
KINDS = os.environ.get("KINDS", "smooth,sin4096,sin_noise,randwalk,chirp,sparse,smallamp,randn").split(",")
for kind in KINDS:
    t0 = time.time()
    x = family(kind, n).astype(npdt)
    enc_h = np.empty_like(x)
    enc_h[0] = x[0]
    np.subtract(x[1:], x[:-1], out=enc_h[1:])
    ref = np.cumsum(enc_h, dtype=npdt)
    encs = [torch.from_numpy(enc_h).to(dev) for _ in range(2)]
    dst = torch.empty_like(encs[0])
    codec.decode(encs[0], out=dst)
    ok = dst.cpu().numpy().tobytes() == ref.tobytes()
    reps = 3 if kind in ("randn",) else 5
    us = timed(lambda r: codec.decode(encs[r % 2], out=dst), reps)
    out[kind] = {"us": round(us, 1), "GBps_2N": round(2 * n * npdt.itemsize / us / 1e3, 2), "ok": ok}
    print(kind, out[kind], round(time.time() - t0, 1), "s", file=sys.stderr, flush=True)
    del encs, dst
# batches: 2048 x 1 MiB (fewer for the random rows)
rows_n = (1 << 20) // npdt.itemsize
for kind, rows in [] if quick else (("smooth", 2048), ("sin_noise", 2048), ("randwalk", 2048), ("randn", 512)):
    xs = np.stack([family(kind, rows_n, seed=k % 16).astype(npdt) for k in range(16)])
    enc_h = np.empty_like(xs)
    enc_h[:, 0] = xs[:, 0]
    np.subtract(xs[:, 1:], xs[:, :-1], out=enc_h[:, 1:])
    ref = np.cumsum(enc_h, axis=1, dtype=npdt)
    e = torch.from_numpy(enc_h).to(dev).repeat(rows // 16, 1)
    d = batch.delta_chunks(e, codec, encode=False)
    ok = d[:16].cpu().numpy().tobytes() == ref.tobytes() and d[-16:].cpu().numpy().tobytes() == ref.tobytes()
    us = timed(lambda r: batch.delta_chunks(e, codec, encode=False), 3)
    out[f"batch_{rows}x1MiB_{kind}"] = {"us": round(us, 1), "GBps_2N": round(2 * rows * (1 << 20) / us / 1e3, 2),
                                       "ok": ok}
    print(kind, "batch", out[f"batch_{rows}x1MiB_{kind}"], file=sys.stderr, flush=True)
    del e, d
print(json.dumps(out), flush=True)
