"""The vendor library's single-pass scan against the product's Delta decode.

    python tools/probe_rocprim_scan.py

rocprim::inclusive_scan (decoupled look-back, tools/lab/lab_rocprim.hip) of
a 256 MiB chunk of u1/u2/u4 words against Delta(<i1/<i2/<i4).decode through
the public codec API (the two-launch scan), 4 rotating buffer sets; the two
outputs are checked equal (wrap-around sums).  One JSON line; GB/s =
algorithmic bytes (read + write) / time.
"""

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import Delta, _ops  # noqa: E402

lab = _lab()
MiB = 1 << 20
dev = torch.device("cuda:0")
sets = 4
out = {}


def timed(fn, reps=20):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % sets)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for es, dt in ((1, "<i1"), (2, "<i2"), (4, "<i4")):
    nb = 256 * MiB
    n = nb // es
    srcs = [torch.randint(-100, 100, (nb,), dtype=torch.int8, device=dev).view(torch.uint8) for _ in range(sets)]
    dsts = [torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(sets)]
    wsb = lab.mc_lab_rocprim_scan_workspace(n, es)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    st = _ops.stream(srcs[0])

    def rp(i):
        assert lab.mc_lab_rocprim_scan(srcs[i].data_ptr(), dsts[i].data_ptr(), n, es, ws.data_ptr(), wsb, st) == 0

    t_rp = timed(rp)
    ref = dsts[0].clone()
    d = Delta(dtype=dt)
    t_api = timed(lambda i: d.decode(srcs[i], out=dsts[i]))
    assert torch.equal(ref, dsts[0]), dt
    out[dt] = {"rocprim_us": round(t_rp, 1), "rocprim_GBps": round(2 * nb / t_rp / 1e3, 1),
               "product_us": round(t_api, 1), "product_GBps": round(2 * nb / t_api / 1e3, 1),
               "rocprim_ws_bytes": wsb}
    del srcs, dsts
    torch.cuda.empty_cache()
print(json.dumps(out))
