"""Per-call latency of the codec API on small chunks (configs[0]: Shuffle(4)
on a 1 MiB fp32 chunk): device tensor in/out, numpy in/out (staged through
the GPU), and the reference CPU loop on the same chunk.  One JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from numcodecs_amd import Shuffle  # noqa: E402

dev = torch.device("cuda:0")
MiB = 1 << 20
res = {}
for nbytes in (64 << 10, MiB, 16 * MiB):
    x = torch.randn(nbytes // 4, device=dev)
    xh = x.cpu().numpy()
    c = Shuffle(4)
    out_e = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out_d = torch.empty(nbytes, dtype=torch.uint8, device=dev)

    def dev_step():
        c.decode(c.encode(x, out=out_e), out=out_d)

    for _ in range(20):
        dev_step()
    torch.cuda.synchronize()
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        dev_step()
    torch.cuda.synchronize()
    t_dev = (time.perf_counter() - t0) / reps
    for _ in range(5):
        c.decode(c.encode(xh))
    reps_h = 50
    t0 = time.perf_counter()
    for _ in range(reps_h):
        c.decode(c.encode(xh))
    t_host = (time.perf_counter() - t0) / reps_h
    k = f"{nbytes >> 10}KiB"
    res[f"{k}_device_encdec_us"] = round(t_dev * 1e6, 1)
    res[f"{k}_device_encdec_GiBps"] = round(2 * nbytes / (1 << 30) / t_dev, 2)
    res[f"{k}_numpy_encdec_us"] = round(t_host * 1e6, 1)
    res[f"{k}_numpy_encdec_GiBps"] = round(2 * nbytes / (1 << 30) / t_host, 2)
    try:
        sys.path.insert(0, ROOT)
        import bench

        do_enc, do_dec, kind, _ = bench._ref_shuffle_fns()
        raw = xh.view(np.uint8)
        e, d = np.empty_like(raw), np.empty_like(raw)
        t0 = time.perf_counter()
        for _ in range(20):
            do_enc(raw, e, 4)
            do_dec(e, d, 4)
        res[f"{k}_cpu_{kind}_encdec_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
    except Exception as ex:  # noqa: BLE001
        res["cpu_error"] = str(ex)
print(json.dumps(res), flush=True)
