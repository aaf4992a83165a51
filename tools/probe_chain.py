"""The serial float chain's instruction schedules (tools/lab/lab_chain.hip):
one wave, lane 0 runs numpy's add chain over an 8192-value LDS buffer
`reps` times; elements/s from HIP events and s_memtime ticks per element.

Usage: python tools/probe_chain.py  -> gpurun_out/probe_chain.json
"""

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

NAMES = {0: "register-only", 1: "product (fsw_chain)", 2: "strict interleave", 3: "reads only", 4: "DPP-fed adds"}


def main():
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    init = (torch.arange(64, device=dev, dtype=torch.float32) * 1e-3)
    out = torch.empty(4, device=dev)
    cyc = torch.zeros(2, dtype=torch.int64, device=dev)
    n, reps = 8192, 64
    rows = []
    for rnd in range(3):
        for kind in NAMES:
            assert lab.mc_lab_chain(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, reps, kind, st) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lab.mc_lab_chain(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, reps, kind, st) == 0
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
