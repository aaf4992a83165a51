"""Fletcher32.decode of one 256 MiB device chunk through the public API:
wall time per call, alone and after CRC32 decodes ran in the same process
(the two probes tools/probe_verify_overhead.py and probe_verify_ck.py
disagreed: 58 vs 70 us).  One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, Fletcher32  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]


def wall(fn, sets, reps=30):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i % sets)
    return round((time.perf_counter() - t0) / reps * 1e6, 1)


out = {}
f = Fletcher32()
fe = [f.encode(x) for x in xs]
out["f32_first_3sets"] = wall(lambda i: f.decode(fe[i]), 3)
out["f32_first_4sets"] = wall(lambda i: f.decode(fe[i]), 4)
c = CRC32()
ce = [c.encode(x) for x in xs]
out["crc32_4sets"] = wall(lambda i: c.decode(ce[i]), 4)
out["f32_after_crc_4sets"] = wall(lambda i: f.decode(fe[i]), 4)
del ce
torch.cuda.empty_cache()
out["f32_after_free_4sets"] = wall(lambda i: f.decode(fe[i]), 4)
print(json.dumps(out), flush=True)
