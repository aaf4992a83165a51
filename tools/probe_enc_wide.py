"""Shuffle layouts on 256 MiB, interleaved rounds in one process (default:
es = 4 encode: V_REG | V_BIG4 = 129, 16-B plane stores V_WIDE = 6, | V_BIG 22,
| V_BIG4 134, lane-pair stores V_PAIR | V_BIG4 = 133); every layout checked
against torch's transpose first.  One JSON line of TB/s (2N / time).

    python tools/probe_enc_wide.py [variants] [es] [enc|dec]"""
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
ES = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ENC = 0 if len(sys.argv) > 3 and sys.argv[3] == "dec" else 1
ins = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]
outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(4)]
shuf = ins[0].view(N // ES, ES).t().contiguous().view(-1)
src0 = ins[0] if ENC else shuf
ref = shuf if ENC else ins[0]
ok = {}
for v in VARS:
    assert lab.mc_lab_shuffle_variant(src0.data_ptr(), outs[0].data_ptr(), N, ES, ENC, v, 0, st) == 0
    torch.cuda.synchronize()
    ok[v] = bool(torch.equal(outs[0], ref))
res = {v: [] for v in VARS}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(7):
    for v in VARS:
        for i in range(2):
            lab.mc_lab_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), N, ES, ENC, v, 0, st)
        e0.record()
        for i in range(20):
            lab.mc_lab_shuffle_variant(ins[i % 4].data_ptr(), outs[i % 4].data_ptr(), N, ES, ENC, v, 0, st)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(2 * N / (e0.elapsed_time(e1) / 20 * 1e-3) / 1e12)
print(json.dumps({str(v): {"ok": ok[v], "TBps_med": round(statistics.median(x), 3), "TBps_max": round(max(x), 3),
                           "us_med": round(2 * N / statistics.median(x) / 1e6, 1)} for v, x in res.items()}), flush=True)
