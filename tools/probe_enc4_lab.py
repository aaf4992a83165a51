"""Shuffle(4) encode schedules of tools/lab/lab_shuffle4.hip against the
product's encode (lab variant 129 = V_REG | V_BIG4, the default), the lane-pair
and V_WIDE layouts, the product decode, and the copy calibration
(tools/lab/lab_bw.hip), interleaved rounds in one process, 4 rotating
256 MiB buffer sets (no Infinity-Cache reuse between calls).

Usage: python tools/probe_enc4_lab.py [rounds]  -> gpurun_out/probe_enc4_lab.json
"""

import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

MiB = 1 << 20


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    n = 256 * MiB
    sets = 4
    ins = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(sets)]
    cfgs = [("prod_enc", 129), ("prod_dec", 21), ("pair_big4_enc", 133), ("wide_big4_enc", 134)]
    cfgs += [(f"lab{k}", k) for k in range(10)]
    cfgs += [(f"copy_u{u}_nt{nt}_g{g}", (u, nt, g)) for u, nt, g in
             ((4, 3, 0), (4, 3, 2048), (4, 3, 4096), (4, 3, 8192), (4, 3, 16384), (8, 3, 0), (8, 3, 8192),
              (4, 1, 8192), (4, 0, 8192))]
    cfgs += [("mc_copy", None), ("hipMemcpy", None)]
    lib = None

    def run(c, i):
        name, arg = c
        s, d = ins[i], outs[i]
        if name.startswith("prod") or name.endswith("big4_enc"):
            enc = 0 if name == "prod_dec" else 1
            rc = lab.mc_lab_shuffle_variant(s.data_ptr(), d.data_ptr(), n, 4, enc, arg, 0, st)
        elif name.startswith("lab"):
            rc = lab.mc_lab_shuffle4_enc(s.data_ptr(), d.data_ptr(), n, arg, st)
        elif name.startswith("copy_"):
            u, nt, g = arg
            rc = lab.mc_lab_bw_copy(s.data_ptr(), d.data_ptr(), n, u, g, nt, st)
        elif name == "mc_copy":
            rc = lab.mc_copy(s.data_ptr(), d.data_ptr(), n, st)
        else:
            d.copy_(s)
            rc = 0
        assert rc == 0, (name, rc)

    import ctypes

    lab.mc_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    iters = 30
    res = {c[0]: [] for c in cfgs}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for c in cfgs:
            for i in range(2):
                run(c, i % sets)
            e0.record()
            for i in range(iters):
                run(c, i % sets)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / iters * 1e-3
            res[c[0]].append((t * 1e6, 2 * n / t / 1e9))
        print(f"round {r} done", flush=True)
    # correctness of every shuffle against torch's transpose
    x = ins[0]
    ref = x.view(n // 4, 4).t().contiguous().view(-1)
    bad = []
    for name, arg in cfgs:
        if not (name.startswith("lab") or name.endswith("_enc")):
            continue
        outs[0].zero_()
        if name.startswith("lab"):
            if arg == 7:
                continue  # not a shuffle (access-pattern ceiling)
            assert lab.mc_lab_shuffle4_enc(x.data_ptr(), outs[0].data_ptr(), n, arg, st) == 0
        else:
            assert lab.mc_lab_shuffle_variant(x.data_ptr(), outs[0].data_ptr(), n, 4, 1, arg, 0, st) == 0
        if not torch.equal(outs[0], ref):
            bad.append(name)
    print("correctness failures:", bad, flush=True)
    out = {"bad": bad, "rows": []}
    for name, v in res.items():
        us = [a for a, _ in v]
        gb = [b for _, b in v]
        row = {"cfg": name, "us_med": round(statistics.median(us), 2), "us_min": round(min(us), 2),
               "GBps_med": round(statistics.median(gb), 1), "GBps_max": round(max(gb), 1)}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_enc4_lab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
