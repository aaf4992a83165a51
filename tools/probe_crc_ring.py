"""The bit-sliced CRC checksum-only tile pass (256 MiB): the product kernel
against lab variants with a deeper register ring and/or per-wave partials
(tools/lab/lab_crc.hip).  Partials checked against the product kernel of the
same tile size; one JSON line per configuration (best of 3 x 10 launches).

Usage: python tools/probe_crc_ring.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

N = 256 << 20
dev = torch.device("cuda:0")
lab = _lab()
st = torch.cuda.current_stream().cuda_stream
x = torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) * 100.0  # us per launch
        best = t if best is None else min(best, t)
    return best


for kind in (0, 1):
    ref = {}
    for K in (16, 8):
        total = N // (K * 4096)
        p = torch.zeros(total, dtype=torch.int32, device=dev)
        for grid in (2048, 1024):
            t = timed(lambda: lab.mc_lab_crc_product(kind, x.data_ptr(), N, K, grid, p.data_ptr(), st))
            print(json.dumps({"probe": "crc_ring", "kind": kind, "variant": "product", "K": K, "grid": grid,
                              "us": round(t, 2)}), flush=True)
        ref[K] = p.clone()
    for K, R, wavep in ((16, 2, 1), (16, 2, 0), (8, 3, 1), (8, 3, 0), (8, 4, 1), (8, 2, 1)):
        total = N // (K * 4096)
        p = torch.zeros(total * (4 if wavep else 1), dtype=torch.int32, device=dev)
        for grid in (2048, 1024, 768, 512):
            rc = lab.mc_lab_crc(kind, x.data_ptr(), N, K, R, wavep, grid, p.data_ptr(), st)
            assert rc == 0, rc
            torch.cuda.synchronize()
            got = p.view(total, 4) if wavep else p.view(total, 1)
            red = got[:, 0]
            for w in range(1, got.shape[1]):
                red = torch.bitwise_xor(red, got[:, w])
            ok = bool(torch.equal(red, ref[K]))
            t = timed(lambda: lab.mc_lab_crc(kind, x.data_ptr(), N, K, R, wavep, grid, p.data_ptr(), st))
            print(json.dumps({"probe": "crc_ring", "kind": kind, "variant": "lab", "K": K, "R": R,
                              "wave_partials": wavep, "grid": grid, "ok": ok, "us": round(t, 2)}), flush=True)
