"""Single-chunk checksum decode through the public API (the call syncs: its
verdict decides between returning and raising): Fletcher32, CRC32, Adler32 of
one 256 MiB device chunk, 3 rotating buffers, wall time per call; GB/s of the
N + 4 algorithmic bytes.  One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, Adler32, Fletcher32  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
out = {}
for name, cls in (("fletcher32", Fletcher32), ("crc32", CRC32), ("adler32", Adler32)):
    c = cls()
    encs = [c.encode(torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)) for _ in range(3)]
    for e in encs:
        c.decode(e)
    torch.cuda.synchronize()
    reps = 30
    t0 = time.perf_counter()
    for i in range(reps):
        c.decode(encs[i % 3])
    t = (time.perf_counter() - t0) / reps
    out[f"{name}_256MiB_decode_us"] = round(t * 1e6, 1)
    out[f"{name}_256MiB_decode_frac"] = round((N + 4) / t / 8e12, 3)
    del encs
print(json.dumps(out), flush=True)
