"""One-launch lagged C4 decode (tools/lab/lab_mall.hip, mc_lab_c4_decode_1l)
against the product decode: n = 64 Mi (and a ragged size), 4 rotating
buffer sets, several lags (tile pairs); bytes checked against the product.
One JSON line of event-timed us per call."""

import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, _ops, batch  # noqa: E402

lab = _lab()
fn = lab.mc_lab_c4_decode_1l
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint32, ctypes.c_void_p]
fn.restype = ctypes.c_int
lab.mc_lab_c41_state_bytes.argtypes = [ctypes.c_size_t]
lab.mc_lab_c41_state_bytes.restype = ctypes.c_size_t

dev = torch.device("cuda:0")
sets = 4
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
_, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
ticket = torch.zeros(2080, dtype=torch.int32, device=dev)
epoch = [0]


def timed(f, reps=20):
    for i in range(sets):
        f(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        f(i % sets)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


out = {}
for n in (64 << 20, (64 << 20) - 4096 * 3 - 16, 4096 * 37 + 16):
    xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
    encs = [pipe.encode(x) for x in xs]
    ref = [pipe.decode(e).view(torch.int32).clone() for e in encs]
    ys = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(sets)]
    state = torch.zeros(lab.mc_lab_c41_state_bytes(n), dtype=torch.uint8, device=dev)
    st = _ops.stream(xs[0])
    key = f"n={n}"
    out[key] = {"product_us": timed(lambda i: pipe.decode(encs[i]))}
    for lag in (2048, 4096, 6144, 8192):
        def run(i, lag=lag):
            epoch[0] += 1
            rc = fn(encs[i].data_ptr(), ys[i].data_ptr(), n, sc3, off4, state.data_ptr(), state.numel(),
                    ticket.data_ptr(), lag, epoch[0], st)
            assert rc == 0, rc
        for i in range(sets):
            run(i)
        ok = all(bool(torch.equal(ys[i].view(torch.int32), ref[i])) for i in range(sets))
        out[key][f"lag{lag}"] = {"us": timed(run), "ok": ok, "ticket_zero": not bool(ticket.any())}
    del xs, encs, ref, ys
print(json.dumps(out), flush=True)
