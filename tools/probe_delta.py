"""Delta decode rates on MI355X (device-resident):
  * float Delta single chunk (one dependent add chain, numpy order)
  * batched Delta decode/encode, one scan per chunk (2048 x 1 MiB)
  * integer single-chunk 3-pass scan, for comparison
Prints one JSON line."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, batch  # noqa: E402

dev = torch.device("cuda", 0)
MiB = 1 << 20


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


out = {}
for dt, tdt, n in (("<f4", torch.float32, 16 * MiB), ("<f8", torch.float64, 8 * MiB), ("<f2", torch.float16, 16 * MiB)):
    x = torch.randn(n, device=dev).to(tdt)
    c = Delta(dt)
    t = timed(lambda: c.decode(x), reps=2)
    out[f"float_chain_{dt[1:]}_{n * x.element_size() // MiB}MiB_GBps"] = round(n * x.element_size() / t / 1e9, 3)
    out[f"float_chain_{dt[1:]}_Melem_per_s"] = round(n / t / 1e6, 1)
b = 2048
for dt, tdt in (("<i2", torch.int16), ("<i4", torch.int32), ("<f4", torch.float32), ("<f8", torch.float64)):
    x = (torch.randn((b, MiB // torch.tensor([], dtype=tdt).element_size()), device=dev) * 100).to(tdt)
    c = Delta(dt)
    enc = batch.delta_chunks(x, c, encode=True)
    dec = torch.empty_like(enc)
    te = timed(lambda: batch.delta_chunks(x, c, encode=True, out=enc))
    td = timed(lambda: batch.delta_chunks(enc, c, encode=False, out=dec))
    assert torch.equal(dec, x.view(torch.uint8).reshape(b, -1)) or dt[1] == "f"
    out[f"batch{b}x1MiB_{dt[1:]}_encode_GBps"] = round(2 * b * MiB / te / 1e9, 1)
    out[f"batch{b}x1MiB_{dt[1:]}_decode_GBps"] = round(2 * b * MiB / td / 1e9, 1)
sets = 3  # rotating buffer sets: no call finds its input in the Infinity Cache
for dt, tdt in (("|i1", torch.int8), ("<i2", torch.int16), ("<i4", torch.int32), ("<i8", torch.int64)):
    es = torch.tensor([], dtype=tdt).element_size()
    c = Delta(dt)
    encs = [c.encode((torch.randn(256 * MiB // es, device=dev) * 100).to(tdt)) for _ in range(sets)]
    k = [0]

    def dec():
        i = k[0] % sets
        k[0] += 1
        c.decode(encs[i])

    td = timed(dec, reps=6)
    out[f"single256MiB_{dt[1:]}_decode_GBps"] = round(2 * 256 * MiB / td / 1e9, 1)
# float-chain schedules (lab: mc_lab_delta_decode_batch_variant)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd._native import check  # noqa: E402
lib = _lab()
from numcodecs_amd._ops import dtype_code  # noqa: E402
import numpy as np  # noqa: E402

st = torch.cuda.current_stream().cuda_stream
for dt, tdt in (("<f4", torch.float32), ("<f8", torch.float64)):
    code = dtype_code(np.dtype(dt))
    es = torch.tensor([], dtype=tdt).element_size()
    for rows, nbytes in ((1, 64 * MiB), (2048, MiB)):
        n = nbytes // es
        x = torch.randn((rows, n), device=dev).to(tdt)
        y = torch.empty_like(x)
        ref = None
        for v in range(6):
            f = lambda: check(lib.mc_lab_delta_decode_batch_variant(x.data_ptr(), n * es, y.data_ptr(), n * es, rows, n,
                                                                  code, code, v, st), "variant")
            t = timed(f, reps=2)
            if ref is None:
                ref = y.clone()
            assert torch.equal(y.view(torch.uint8), ref.view(torch.uint8)), (dt, rows, v)
            out[f"chain_{dt[1:]}_{rows}x{nbytes // MiB}MiB_v{v}_GBps"] = round(rows * nbytes / t / 1e9, 3)
print(json.dumps(out), flush=True)
