"""Checksum32 kernel tuning probe: one config per process (the knobs are read
once per process).  python tools/probe_ck.py  -> one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import batch, _ops  # noqa: E402

MiB = 1 << 20


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


dev = torch.device("cuda:0")
xb = torch.randint(0, 256, (2048, MiB), dtype=torch.uint8, device=dev)
eb = torch.empty((2048, MiB + 4), dtype=torch.uint8, device=dev)
x1 = xb.view(-1)[: 256 * MiB]
res = {"K": os.environ.get("MCODEC_CK_K"), "grid": os.environ.get("MCODEC_CK_GRID")}
for cid in ("crc32", "adler32"):
    kind = batch._CK_KINDS[cid][0]
    res[cid + "_batch"] = round(2048 * MiB / timed(lambda: batch.checksum32_chunks(xb, cid)) / 1e9, 1)
    res[cid + "_enc"] = round(2 * 2048 * MiB / timed(lambda: batch.checksum32_encode_chunks(xb, cid, out=eb)) / 1e9, 1)
    res[cid + "_256MiB"] = round(256 * MiB / timed(lambda: _ops.checksum32(kind, x1, 256 * MiB, 1, 256 * MiB, 0)) / 1e9, 1)
print(json.dumps(res), flush=True)
