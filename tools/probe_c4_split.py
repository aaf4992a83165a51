"""Two-launch C4 decode with a per-tile load policy (tools/lab/lab_mall.hip,
mc_lab_c4_decode_split): the reduce pass reads tiles below a split point with
the default policy (kept in the Infinity Cache for the apply pass) and the
rest nontemporally; the apply pass likewise with its own split.  FSO f4 <-
Delta i2 <- Shuffle(2), n = 64 Mi, 4 rotating buffer sets, bytes checked
against the product decode.  One JSON line of event-timed us per call."""

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
fn = lab.mc_lab_c4_decode_split
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
               ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
fn.restype = ctypes.c_int
lab.mc_lab_c4_2l_workspace.argtypes = [ctypes.c_size_t]
lab.mc_lab_c4_2l_workspace.restype = ctypes.c_size_t

dev = torch.device("cuda:0")
sets = 4
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
_, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
ticket = torch.zeros(64 * 32 + 64, dtype=torch.int32, device=dev)


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


n = 64 << 20
ntiles = n // 4096
xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
encs = [pipe.encode(x) for x in xs]
ref = [pipe.decode(e).view(torch.int32).clone() for e in encs]
ys = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(sets)]
ws = torch.empty(lab.mc_lab_c4_2l_workspace(n), dtype=torch.uint8, device=dev)
st = _ops.stream(xs[0])
out = {}
for rep in range(2):
    out[f"product_{rep}"] = timed(lambda i: pipe.decode(encs[i], out=ys[i]))
    for rf in (1.0, 0.75, 0.625, 0.5, 0.375, 0.0):
        for af in (1.0, rf, 0.0):
            r_split, a_split = int(rf * ntiles), int(af * ntiles)

            def run(i, r_split=r_split, a_split=a_split):
                rc = fn(encs[i].data_ptr(), ys[i].data_ptr(), n, sc3, off4, ws.data_ptr(), ws.numel(),
                        ticket.data_ptr(), r_split, a_split, st)
                assert rc == 0, rc
            for y in ys:
                y.zero_()
            us = timed(run)
            ok = all(bool(torch.equal(ys[i].view(torch.int32), ref[i])) for i in range(sets))
            out[f"r{rf}_a{af}_{rep}"] = {"us": us, "ok": ok}
print(json.dumps(out), flush=True)
