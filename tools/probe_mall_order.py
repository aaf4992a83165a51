"""C4 decode (FSO f4 <- Delta i2 <- Shuffle(2), n = 64 Mi) with the two
passes in the same or opposite tile orders and nt / default-policy loads
(tools/lab/lab_mall.hip, flags 0..15), 4 rotating buffer sets; each flag's
bytes checked against the product decode.  One JSON line; run under
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mallo -o m -- python3 tools/probe_mall_order.py
for the per-pass kernel times (template arguments <REV, NT>)."""

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
from numcodecs_amd._native import lib  # noqa: E402

lab = _lab()
fn = lab.mc_lab_c4_decode_mall
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
fn.restype = ctypes.c_int

dev = torch.device("cuda:0")
n = 64 << 20
sets = 4
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
encs = [pipe.encode(x) for x in xs]
ref = pipe.decode(encs[0]).view(torch.int32).clone()
_, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
ws = torch.empty(lib.mc_fso_delta_shuffle_decode_workspace(n), dtype=torch.uint8, device=dev)
ys = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(sets)]
st = _ops.stream(xs[0])


def run(i, flags):
    rc = fn(encs[i].data_ptr(), ys[i].data_ptr(), n, sc3, off4, ws.data_ptr(), ws.numel(), flags, st)
    assert rc == 0, rc


out = {}
for flags in range(16):
    run(0, flags)
    ok = bool(torch.equal(ys[0].view(torch.int32), ref))
    for i in range(sets):
        run(i, flags)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for i in range(reps):
        run(i % sets, flags)
    e1.record()
    torch.cuda.synchronize()
    out[f"flags{flags}"] = {"us": round(e0.elapsed_time(e1) / reps * 1e3, 1), "ok": ok}
print(json.dumps(out), flush=True)
