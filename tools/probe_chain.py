"""The serial float chain's instruction schedules (tools/lab/lab_chain.hip):
one wave, lane 0 runs numpy's add chain over an 8192-value LDS buffer
`reps` times; elements/s from HIP events and s_memtime ticks per element.

Usage: python tools/probe_chain.py  -> gpurun_out/probe_chain.json
"""

import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

NAMES = {0: "register-only", 1: "product (fsw_chain)", 2: "strict interleave", 3: "reads only", 4: "DPP-fed adds",
         5: "rot G16 NS4", 6: "rot G16 NS8", 7: "rot G32 NS4", 8: "rot G16 NS4 ld-first", 9: "rot G8 NS8",
         10: "rot G16 NS8 ld-first", 11: "SGPR-fed, no stores", 12: "SGPR-fed, LDS stores",
         13: "SGPR-fed, global stores", 14: "LDS-fed, global stores", 15: "SGPR-fed, lane-gathered stores",
         16: "SGPR-fed x4 waves, split stores", 17: "SGPR-fed x2 waves, split stores",
         18: "SGPR-fed x8 waves, split stores", 19: "SGPR-fed, every 16th group stored",
         20: "SGPR-fed, 4-B global stores", 21: "SGPR-fed, stores one group late",
         22: "SGPR-fed, all-lane stores one group late", 23: "SGPR-fed, all-lane stores",
         24: "LDS-fed all lanes, LDS stores", 25: "LDS-fed all lanes, global stores"}


def main():
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    init = (torch.arange(64, device=dev, dtype=torch.float32) * 1e-3)
    out = torch.empty(4, device=dev)
    cyc = torch.zeros(2, dtype=torch.int64, device=dev)
    n, reps = 8192, 64
    gin = torch.randn(n, device=dev)
    gout = torch.zeros(n, device=dev)

    def run(kind, r=reps):
        if kind < 11 or kind == 24:
            return lab.mc_lab_chain(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, r, kind, st)
        return lab.mc_lab_chain_g(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, r, kind, gin.data_ptr(),
                                  gout.data_ptr(), st)

    # the global-output kinds must write numpy's float32 cumsum of gin
    bad = []
    want = np.cumsum(gin.cpu().numpy())
    for kind in (13, 15, 16, 17, 18, 20, 21, 22, 23):
        gout.zero_()
        assert run(kind, 1) == 0
        torch.cuda.synchronize()
        if not np.array_equal(gout.cpu().numpy().view(np.uint32), want.view(np.uint32)):
            bad.append(kind)
    print("chain correctness failures:", bad, flush=True)
    # f64 kinds (round 5): correctness of the stored kinds, then timing
    n64 = 4096
    gin64 = torch.randn(n64, device=dev, dtype=torch.float64)
    gout64 = torch.zeros(n64, device=dev, dtype=torch.float64)
    init64 = torch.arange(64, device=dev, dtype=torch.float64) * 1e-3
    out64 = torch.empty(4, device=dev, dtype=torch.float64)

    def run64(kind, r=reps):
        return lab.mc_lab_chain64(init64.data_ptr(), out64.data_ptr(), cyc.data_ptr(), n64, r, kind,
                                  gin64.data_ptr(), gout64.data_ptr(), st)

    want64 = np.cumsum(gin64.cpu().numpy())
    bad64 = []
    for kind in (42, 43, 44):
        gout64.zero_()
        assert run64(kind, 1) == 0
        torch.cuda.synchronize()
        if not np.array_equal(gout64.cpu().numpy().view(np.uint64), want64.view(np.uint64)):
            bad64.append(kind)
    print("f64 chain correctness failures:", bad64, flush=True)
    for rnd in range(3):
        for kind, name in ((40, "f64 register-only"), (41, "f64 SGPR-fed, no stores"),
                           (42, "f64 SGPR-fed, all-lane stores"), (43, "f64 LDS-fed, lane-0 global stores"),
                           (44, "f64 SGPR-fed, lane-0 global stores")):
            assert run64(kind) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert run64(kind) == 0
            e1.record()
            e1.synchronize()
            t = e0.elapsed_time(e1) * 1e-3
            el = n64 * reps
            print(json.dumps({"round": rnd, "kind": kind, "name": name, "Melem_per_s": round(el / t / 1e6, 1),
                              "ticks_per_elem": round(int(cyc[0].item()) / el, 3), "us": round(t * 1e6, 1)}),
                  flush=True)
    rows = []
    for rnd in range(3):
        for kind in NAMES:
            assert run(kind) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert run(kind) == 0
            e1.record()
            e1.synchronize()
            t = e0.elapsed_time(e1) * 1e-3
            el = n * reps
            rows.append({"round": rnd, "kind": kind, "name": NAMES[kind], "Melem_per_s": round(el / t / 1e6, 1),
                         "ticks_per_elem": round(int(cyc[0].item()) / el, 3), "us": round(t * 1e6, 1)})
            print(json.dumps(rows[-1]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_chain.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
