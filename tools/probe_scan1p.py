"""Single-pass vs three-pass integer scans on one 256 MiB chunk (MI355X).

    python tools/probe_scan1p.py            # default schedule (single pass)
    MCODEC_SCAN1P=0 python tools/probe_scan1p.py   # the three-pass scans

Times, through the public codec API with 4 rotating buffer sets (no call finds
its input in the Infinity Cache): Delta(<i1/<i2/<i4) decode of a 256 MiB
chunk, and the fused C4 decode (FSO f4<-i2 <- Delta(i2) <- Shuffle(2), 64 Mi
elements); each checked against the codec-by-codec / three-pass bytes.  One
JSON line; GB/s = algorithmic bytes (read + write) / time.
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, batch  # noqa: E402

MiB = 1 << 20
dev = torch.device("cuda:0")
sets = 4
out = {"MCODEC_SCAN1P": os.environ.get("MCODEC_SCAN1P", "1")}


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
    return e0.elapsed_time(e1) / reps * 1e-3


for name, tdt, dt in (("i1", torch.int8, "|i1"), ("i2", torch.int16, "<i2"), ("i4", torch.int32, "<i4")):
    es = torch.tensor([], dtype=tdt).element_size()
    n = 256 * MiB // es
    d = Delta(dt)
    xs = [torch.randint(-100, 100, (n,), dtype=tdt, device=dev) for _ in range(sets)]
    encs = [d.encode(x) for x in xs]
    ok = all(torch.equal(d.decode(encs[i]), xs[i]) for i in range(sets))
    t = timed(lambda i: d.decode(encs[i]))
    out[f"delta_{name}_256MiB_decode_us"] = round(t * 1e6, 1)
    out[f"delta_{name}_256MiB_decode_GBps"] = round(2 * 256 * MiB / t / 1e9, 1)
    out[f"delta_{name}_ok"] = ok
    del xs, encs

n = 64 << 20
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
es_ = [pipe.encode(x) for x in xs]
ref = fso.decode(dl.decode(sh.decode(es_[0])))
out["c4_ok"] = bool(torch.equal(pipe.decode(es_[0]).view(torch.int32), ref.view(torch.int32)))
t_dec = timed(lambda i: pipe.decode(es_[i]))
t_enc = timed(lambda i: pipe.encode(xs[i]))
out["c4_decode_us"] = round(t_dec * 1e6, 1)
out["c4_decode_GBps"] = round(6 * n / t_dec / 1e9, 1)
out["c4_encode_us"] = round(t_enc * 1e6, 1)
out["c4_encdec_GiBps"] = round(2 * 4 * n / (1 << 30) / (t_dec + t_enc), 1)
print(json.dumps(out), flush=True)
