"""Phase timeline of the single-pass scans (lab trace buffer): where does a
partition's time go?  C4 decode (64 Mi elements) and Delta(i2) 256 MiB.

    python tools/trace_scan1p.py > gpurun_out/trace_scan1p.json

Per partition (wall_clock64 ticks, 100 MHz): ticket, staged (aggregate
published), look-back resolved, emit start, emitted; summarised as medians /
percentiles of the phase lengths and of the wait between staged and
resolved, plus the kernel's own duration.
"""

import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, _ops, batch  # noqa: E402

lab = _lab()
dev = torch.device("cuda:0")
TICK_US = 0.01  # wall_clock64 runs at 100 MHz


def summarise(tr, npart, elapsed_ms):
    t = tr[:npart].astype(np.int64)
    t0 = t[:, 0].min()
    ticket, staged, resolved, emit0, emit1 = (t[:, i] - t0 for i in range(5))
    ok = (emit1 > 0) & (resolved > 0)
    q = lambda a: {k: round(float(np.percentile(a[ok], p)) * TICK_US, 2) for k, p in (("p10", 10), ("p50", 50), ("p90", 90), ("max", 100))}  # noqa: E731
    return {
        "npart": int(npart), "kernel_ms": round(elapsed_ms, 4),
        "span_us": round(float(emit1.max()) * TICK_US, 1),
        "stage_us(ticket->published)": q(staged - ticket),
        "wait_us(published->resolved)": q(resolved - staged),
        "emit_us": q(emit1 - emit0),
        "first_ticket_us": round(float(ticket.min()) * TICK_US, 2),
        "last_emit_us": round(float(emit1.max()) * TICK_US, 2),
        "workgroups": int(len(np.unique(t[:, 5]))),
    }


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


out = {}
# C4
n = 64 << 20
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
codecs = [fso, Delta(dtype="<i2"), Shuffle(2)]
pipe = batch.FilterPipeline(codecs)
x = 1000.0 + 10.0 * torch.rand(n, device=dev)
enc = pipe.encode(x).view(torch.uint8).reshape(-1)
ref = pipe.decode(enc).view(torch.uint8).reshape(-1)
_, _, sc3, off4 = batch._c4_scalars(*codecs)
a, d = _ops.dtype_code("<i2"), _ops.dtype_code("<f4")
nb = lab.mc_lab_c4_dec1p_state_bytes(n, a)
npart = (nb - 16) // 8
state = torch.zeros(nb, dtype=torch.uint8, device=dev)
outb = torch.empty_like(ref)
trace = torch.zeros(8 * npart, dtype=torch.int64, device=dev)
for rep in range(3):
    trace.zero_()
    ms = timed(lambda: lab.mc_lab_c4_dec1p(enc.data_ptr(), outb.data_ptr(), n, a, d, sc3, off4, state.data_ptr(),
                                           1 << 14, trace.data_ptr(), _ops.stream(enc)))
assert torch.equal(outb, ref)
out["c4"] = summarise(trace.view(npart, 8).cpu().numpy(), npart, ms)
# Delta(i2) 256 MiB
n = 128 << 20
dl = Delta("<i2")
xi = torch.randint(-100, 100, (n,), dtype=torch.int16, device=dev)
e2 = dl.encode(xi)
y = torch.empty_like(xi)
nb = lab.mc_lab_delta_dec1p_state_bytes(n, 2)
npart = (nb - 16) // 8
state = torch.zeros(nb, dtype=torch.uint8, device=dev)
trace = torch.zeros(8 * npart, dtype=torch.int64, device=dev)
for rep in range(3):
    trace.zero_()
    ms = timed(lambda: lab.mc_lab_delta_dec1p(e2.data_ptr(), y.data_ptr(), n, 2, state.data_ptr(), 1 << 14,
                                              trace.data_ptr(), _ops.stream(e2)))
assert torch.equal(y, xi)
out["delta_i2"] = summarise(trace.view(npart, 8).cpu().numpy(), npart, ms)
# same kernel without the trace writes
ms = timed(lambda: lab.mc_lab_delta_dec1p(e2.data_ptr(), y.data_ptr(), n, 2, state.data_ptr(), 1 << 14, None,
                                          _ops.stream(e2)))
out["delta_i2_untraced_ms"] = round(ms, 4)
print(json.dumps(out, indent=1))
