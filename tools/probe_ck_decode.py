"""Batched checksum decode kernels on 64 x 4 MiB rows: the one-pass
decode (checksum + stored footer + payload compaction) for 16-B aligned
and 4-B aligned row strides, against the checksum alone.  Rotates 4 buffer
sets (past the 256 MiB Infinity Cache); us per call, median of 20."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from numcodecs_amd import batch  # noqa: E402

MiB = 1 << 20
B, N = 64, 4 * MiB


def timeit(fn, sets, reps=60):
    for i in range(4):
        fn(sets[i % len(sets)])
    ts = []
    for r in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn(sets[r % len(sets)])
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


res = {}
for kind in os.environ.get("PROBE_ONLY", "crc32,adler32,fletcher32").split(","):
    for pad, loc in ((12, "end"), (0, "end"), (0, "start")):
        if kind == "fletcher32" and loc == "start":
            continue
        sets = []
        for _ in range(4):
            w = torch.randint(0, 256, (B, N + 4 + pad), dtype=torch.uint8, device="cuda")
            sets.append(w[:, : N + 4])
        if kind == "fletcher32":
            fn = lambda x: batch.fletcher32_decode_chunks(x)  # noqa: E731
        else:
            fn = lambda x, k=kind, lc=loc: batch.checksum32_decode_chunks(x, k, location=lc)  # noqa: E731
        res[f"{kind}_decode_stride{N + 4 + pad}_{loc}"] = timeit(fn, sets)
    al = [torch.randint(0, 256, (B, N), dtype=torch.uint8, device="cuda") for _ in range(4)]
    if kind == "fletcher32":
        res[f"{kind}_sum_aligned"] = timeit(lambda x: batch.fletcher32_chunks(x), al)
    else:
        res[f"{kind}_sum_aligned"] = timeit(lambda x, k=kind: batch.checksum32_chunks(x, k), al)
        res[f"{kind}_encode_aligned"] = timeit(lambda x, k=kind: batch.checksum32_encode_chunks(x, k), al)
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("MCODEC_")}, **res}))
