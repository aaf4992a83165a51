"""The SGPR-fed serial chain streaming a large buffer from HBM
(tools/lab/lab_chain.hip k_lab_stream: the lab's ser_chain_sgpr + ser_prefetch
and the product's ser_chain_vbc): group size x prefetch windows -> Melem/s and ticks/element.

Usage: python tools/probe_stream.py [MiB]  (one JSON line per configuration)
"""

import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

CONFIGS = {
    # ser_chain_sgpr: (SG, l2 window, scalar-cache window, prefetch wave)
    0: [(32, 32768, 0, 1), (40, 32768, 0, 1)],
    1: [(16, 32768, 0, 1), (20, 32768, 0, 1)],
    # ser_chain_vbc: (SG, l2 window, depth D, prefetch wave)
    2: [(32, 0, 6, 0), (32, 32768, 6, 1), (32, 0, 4, 0), (24, 0, 8, 0), (16, 0, 12, 0)],
    3: [(16, 0, 6, 0), (16, 32768, 6, 1), (12, 0, 8, 0), (8, 0, 12, 0)],
}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    cyc = torch.zeros(2, dtype=torch.int64, device=dev)
    for kind in (0, 2, 1, 3):
        dt = torch.float32 if kind in (0, 2) else torch.float64
        n = (mib << 20) // (4 if kind in (0, 2) else 8)
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(n, device=dev, dtype=dt, generator=g)
        y = torch.empty_like(x)
        want = np.cumsum(x.cpu().numpy())
        for sg, l2a, ka, pf in CONFIGS[kind]:
            rc = lab.mc_lab_stream(x.data_ptr(), y.data_ptr(), n, kind, sg, l2a, ka, pf, cyc.data_ptr(), st)
            assert rc == 0, rc
            torch.cuda.synchronize()
            ok = bool(np.array_equal(y.cpu().numpy(), want))
            best = None
            for _ in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert lab.mc_lab_stream(x.data_ptr(), y.data_ptr(), n, kind, sg, l2a, ka, pf, cyc.data_ptr(),
                                         st) == 0
                e1.record()
                e1.synchronize()
                t = e0.elapsed_time(e1) * 1e-3
                best = t if best is None else min(best, t)
            print(json.dumps({"probe": "stream", "dtype": "f4" if kind in (0, 2) else "f8",
                              "chain": "sgpr" if kind < 2 else "vbc", "MiB": mib, "sg": sg, "l2_ahead": l2a,
                              ("k_ahead" if kind < 2 else "depth"): ka, "prefetch": pf, "ok": ok,
                              "Melem_per_s": round(n / best / 1e6, 1),
                              "ticks_per_elem": round(int(cyc[0].item()) / n, 3),
                              "ms_256MiB": round(best * 1e3 * 256 / mib, 1)}), flush=True)


if __name__ == "__main__":
    main()
