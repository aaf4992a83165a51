"""Host<->device transfer and host->host pipeline probe (pinned memory).

    python tools/probe_e2e.py            (also run with HSA_ENABLE_SDMA=0)
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import batch  # noqa: E402

GiB = 1 << 30
MiB = 1 << 20


def t_of(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    dev = torch.device("cuda:0")
    total = 2 * GiB
    chunk = 4 * MiB
    n = total // chunk
    ha = torch.randint(0, 256, (n, chunk), dtype=torch.uint8).pin_memory()
    hb = torch.empty_like(ha).pin_memory()
    da = torch.empty((n, chunk), dtype=torch.uint8, device=dev)
    db = torch.empty_like(da)
    res = {"env_HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA")}
    res["h2d_GiBps"] = round(2 / t_of(lambda: da.copy_(ha, non_blocking=True)), 2)
    res["d2h_GiBps"] = round(2 / t_of(lambda: hb.copy_(db, non_blocking=True)), 2)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():
        with torch.cuda.stream(s1):
            da.copy_(ha, non_blocking=True)
        with torch.cuda.stream(s2):
            hb.copy_(db, non_blocking=True)
        s1.synchronize()
        s2.synchronize()

    res["duplex_each_GiBps"] = round(2 / t_of(duplex), 2)
    for ns in (2, 3, 4):
        for sl in (2, 4, 16, 32):
            t = t_of(lambda: batch.host_pipeline(ha, hb, 4, True, slice_chunks=sl, nslots=ns))
            res[f"pipe_slots{ns}_slice{sl * chunk // MiB}MiB_GiBps"] = round(2 / t, 2)
    print(json.dumps(res), flush=True)
    tag = "nosdma" if os.environ.get("HSA_ENABLE_SDMA") == "0" else "sdma"
    with open(os.path.join("gpurun_out", f"probe_e2e_{tag}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
