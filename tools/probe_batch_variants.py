"""Shuffle(4) encode of 256 MiB as 256 rows of 1 MiB (BASELINE C1 batched)
and as 64 rows of 4 MiB, every encode layout through the lab's batched
entry point, one workgroup per tile (or the stated cap), 4 rotating sets,
HIP events; outputs checked against the product default.

    python tools/probe_batch_variants.py  -> gpurun_out/probe_batch_variants.json
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
V_REG, V_PAIR, V_NO_NT, V_BIG, V_BIG4, V_BIG8, G2, G4 = 1, 5, 8, 16, 128, 512, 32, 64
ES = int(os.environ.get("ES", "4"))
V_WIDE = 6
VARIANTS8 = [(0, 0), (V_PAIR, 0), (V_PAIR | V_BIG, 0), (V_PAIR | V_BIG4, 0), (V_REG, 0), (V_REG | V_BIG, 0),
             (V_REG | V_BIG4, 0), (V_REG | V_BIG8, 0), (V_WIDE, 0), (V_WIDE | V_BIG, 0)]
VARIANTS = [(0, 0), (V_REG | V_BIG8, 0), (V_REG | V_BIG4, 0), (V_REG | V_BIG, 0), (V_REG, 0), (V_PAIR | V_BIG8, 0),
            (V_PAIR | V_BIG4, 0), (V_PAIR | V_BIG, 0), (V_REG | V_BIG8 | V_NO_NT, 0), (V_REG | V_BIG8, 1024),
            (V_REG | V_BIG8, 512), (V_REG | V_BIG4 | G2, 1024), (V_REG | V_BIG | G4, 1024), (V_REG | V_BIG4, 2048)]


def main():
    lab = _lab()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    sets, n = 4, 256 * MiB
    ins = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(sets)]
    rows_out = []
    global VARIANTS
    if ES == 8:
        VARIANTS = VARIANTS8
    for rows in (256, 64):
        m = n // rows

        def run(v, cap, i):
            return lab.mc_lab_shuffle_batch_variant(ins[i].data_ptr(), m, outs[i].data_ptr(), m, rows, m, ES, 1, v, cap,
                                                    st)

        assert run(0, 0, 0) == 0
        torch.cuda.synchronize()
        ref = outs[0].clone()
        times = {vc: [] for vc in VARIANTS}
        bad = []
        for vc in VARIANTS:
            if run(*vc, 0) != 0:
                bad.append(vc)
                continue
            torch.cuda.synchronize()
            if not torch.equal(ref, outs[0]):
                bad.append(vc)
        for _ in range(3):
            for vc in VARIANTS:
                if vc in bad:
                    continue
                for i in range(sets):
                    run(*vc, i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for r in range(20):
                    run(*vc, r % sets)
                e1.record()
                e1.synchronize()
                times[vc].append(e0.elapsed_time(e1) * 1e3 / 20)
        for vc in VARIANTS:
            if vc in bad:
                rows_out.append({"rows": rows, "variant": vc[0], "cap": vc[1], "bad": True})
            else:
                us = statistics.median(times[vc])
                rows_out.append({"es": ES, "rows": rows, "variant": vc[0], "cap": vc[1], "us": round(us, 2),
                                 "TBps": round(2 * n / us / 1e6, 3)})
            print(json.dumps(rows_out[-1]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_batch_variants.json"), "w") as f:
        json.dump(rows_out, f, indent=1)


if __name__ == "__main__":
    main()
