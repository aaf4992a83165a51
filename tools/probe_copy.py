"""mc_copy against hipMemcpyAsync DtoD (torch copy_) at 256 MiB and 1 GiB,
4 rotating buffer pairs, median of 20; GB/s = read + write bytes / time."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from numcodecs_amd import _ops  # noqa: E402

res = {"env": {k: v for k, v in os.environ.items() if k.startswith("MCODEC_COPY")}}
for nb in (256 << 20, 1 << 30):
    nsets = 4 if nb <= 256 << 20 else 2
    bufs = [(torch.ones(nb, dtype=torch.uint8, device="cuda"), torch.empty(nb, dtype=torch.uint8, device="cuda"))
            for _ in range(nsets)]
    for name, fn in (("hipMemcpy", lambda a, b: b.copy_(a)), ("mc_copy", lambda a, b: _ops.copy(a, b, nb))):
        for i in range(nsets):
            fn(*bufs[i])
        ts = []
        for r in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn(*bufs[r % nsets])
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        ts.sort()
        res[f"{name}_{nb >> 20}MiB_GBps"] = round(2 * nb / ts[10] / 1e9, 1)
    del bufs
print(json.dumps(res))
