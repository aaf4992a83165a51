"""Single-chunk integer Delta decode (the same-width dscan path) for i1..i8
on 128 MiB and 256 MiB, 4 rotating buffers; run under rocprofv3
--kernel-trace --stats for the per-kernel split (reduce / sums / apply)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from numcodecs_amd import Delta  # noqa: E402

res = {}
for dt, tdt in (("|i1", torch.int8), ("<i2", torch.int16), ("<i4", torch.int32), ("<i8", torch.int64)):
    for nbytes in (128 << 20, 256 << 20):
        n = nbytes // torch.tensor([], dtype=tdt).element_size()
        xs = [torch.randint(-100, 100, (n,), dtype=tdt, device="cuda") for _ in range(4)]
        codec = Delta(dt)
        for x in xs:
            codec.decode(x)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(20):
            codec.decode(xs[r % 4])
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        res[f"{dt}_{nbytes >> 20}MiB_us"] = round(us, 1)
        res[f"{dt}_{nbytes >> 20}MiB_GBps_2N"] = round(2 * nbytes / us / 1e3, 1)
        del xs
print(json.dumps(res))
