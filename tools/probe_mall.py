"""Does the three-pass C4 decode's re-read of the encoded planes come from the
Infinity Cache when the chunk is small?  Runs the (three-pass) product decode on chunks of 4..64 Mi elements, 4 rotating
sets, under rocprofv3 --kernel-trace; the reduce pass reads 2n bytes, the
apply pass re-reads 2n and writes 4n.  Compare the apply pass's bytes/time
across sizes (tools: rocprof stats, grouped by grid size).
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mall -o m -- python3 tools/probe_mall.py
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, batch  # noqa: E402

dev = torch.device("cuda:0")
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
pipe = batch.FilterPipeline([fso, Delta(dtype="<i2"), Shuffle(2)])
res = {}
for log2n in (22, 23, 24, 25, 26):
    n = 1 << log2n
    sets = 4
    xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
    es = [pipe.encode(x) for x in xs]
    for i in range(sets):
        pipe.decode(es[i])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for i in range(reps):
        pipe.decode(es[i % sets])
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps
    res[f"n=2^{log2n}"] = {"decode_us": round(t * 1e3, 2), "GBps_6n": round(6 * n / (t * 1e-3) / 1e9, 1)}
    del xs, es
print(json.dumps(res), flush=True)
