"""Shuffle(4) encode layouts on 256 MiB, interleaved rounds in one process:
the default (V_REG | V_BIG4 = 129), 16-B plane stores (V_WIDE = 6, | V_BIG 22,
| V_BIG4 134) and the lane-pair stores (V_PAIR | V_BIG4 = 133); every layout
checked against torch's transpose first.  One JSON line of TB/s (2N / time)."""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

lab = _lab()
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
N = 256 << 20
VARS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "129,6,22,134,133".split(","))]
ins = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]
outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(4)]
ref = ins[0].view(N // 4, 4).t().contiguous().view(-1)
ok = {}
for v in VARS:
    assert lab.mc_lab_shuffle_variant(ins[0].data_ptr(), outs[0].data_ptr(), N, 4, 1, v, 0, st) == 0
    torch.cuda.synchronize()
    ok[v] = bool(torch.equal(outs[0], ref))
res = {v: [] for v in VARS}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(7):
    for v in VARS:
        for i in range(2):
            lab.mc_lab_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), N, 4, 1, v, 0, st)
        e0.record()
        for i in range(20):
            lab.mc_lab_shuffle_variant(ins[i % 4].data_ptr(), outs[i % 4].data_ptr(), N, 4, 1, v, 0, st)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(2 * N / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e12)
print(json.dumps({str(v): {"ok": ok[v], "TBps_med": round(statistics.median(x), 3), "TBps_max": round(max(x), 3),
                           "us_med": round(2 * N / statistics.median(x) / 1e6, 1)} for v, x in res.items()}), flush=True)
