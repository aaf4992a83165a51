"""Two-stream slab pipeline for the C4 decode (tools/lab/lab_mall.hip,
mc_lab_c4_decode_2s): reduce of slab k+1 on the caller's stream overlaps the
apply of slab k on a side stream, against the product's two-launch decode and
the one-stream slab loop (mc_lab_c4_decode_2l).  FSO f4 <- Delta i2 <-
Shuffle(2), n = 64 Mi, 4 rotating buffer sets; every setting's bytes are
checked against the product.  One JSON line of event-timed us per call."""

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
f2l = lab.mc_lab_c4_decode_2l
f2l.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
f2l.restype = ctypes.c_int
f2s = lab.mc_lab_c4_decode_2s
f2s.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                ctypes.c_void_p, ctypes.c_void_p]
f2s.restype = ctypes.c_int
lab.mc_lab_c4_2l_workspace.argtypes = [ctypes.c_size_t]
lab.mc_lab_c4_2l_workspace.restype = ctypes.c_size_t

dev = torch.device("cuda:0")
sets = 4
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
_, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
ticket = torch.zeros(64 * 32 + 64, dtype=torch.int32, device=dev)
side = torch.cuda.Stream(device=dev)


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
for n in (64 << 20, (64 << 20) - 4096 * 3 - 16):
    xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
    encs = [pipe.encode(x) for x in xs]
    ref = [pipe.decode(e).view(torch.int32).clone() for e in encs]
    ys = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(sets)]
    ws = torch.empty(lab.mc_lab_c4_2l_workspace(n), dtype=torch.uint8, device=dev)
    st = _ops.stream(xs[0])
    key = f"n={n}"
    res = out[key] = {}
    for rep in range(2):
        res[f"product_{rep}"] = timed(lambda i: pipe.decode(encs[i]))
        for flags in (6 | 1 << 4, 6 | 2 << 4):
            for slabs in (1, 2):
                def run(i, flags=flags, slabs=slabs):
                    rc = f2l(encs[i].data_ptr(), ys[i].data_ptr(), n, sc3, off4, ws.data_ptr(), ws.numel(),
                             ticket.data_ptr(), flags, slabs, st)
                    assert rc == 0, rc
                for y in ys:
                    y.zero_()
                us = timed(run)
                ok = all(bool(torch.equal(ys[i].view(torch.int32), ref[i])) for i in range(sets))
                res[f"2l_f{flags}_s{slabs}_{rep}"] = {"us": us, "ok": ok}
            for slabs in (2, 4, 8, 16):
                for window in (0, 1, 2):
                    if window >= slabs:
                        continue
                    def run(i, flags=flags, slabs=slabs, window=window):
                        rc = f2s(encs[i].data_ptr(), ys[i].data_ptr(), n, sc3, off4, ws.data_ptr(), ws.numel(),
                                 ticket.data_ptr(), flags, slabs, window, st, side.cuda_stream)
                        assert rc == 0, rc
                    for y in ys:
                        y.zero_()
                    us = timed(run)
                    ok = all(bool(torch.equal(ys[i].view(torch.int32), ref[i])) for i in range(sets))
                    res[f"2s_f{flags}_s{slabs}_w{window}_{rep}"] = {
                        "us": us, "ok": ok, "ticket_zero": not bool(ticket.any())}
        print(json.dumps({key: res}), flush=True)
    del xs, encs, ref, ys
print(json.dumps(out), flush=True)
