"""Product three-pass vs lab single-pass integer scans on one 256 MiB chunk.

    python tools/probe_scan1p.py

Times, with 4 rotating buffer sets (no call finds its input in the Infinity
Cache): Delta(<i1/<i2/<i4) decode of a 256 MiB chunk and the fused C4 decode
(FSO f4<-i2 <- Delta(i2) <- Shuffle(2), 64 Mi elements), through the public
codec API (product: three passes) and through the lab's single pass
(tools/lab/lab_scan1p.hip); each checked against the codec-by-codec bytes.
One JSON line; GB/s = algorithmic bytes (read + write) / time.
"""

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
    st = torch.zeros(lab.mc_lab_delta_dec1p_state_bytes(n, es), dtype=torch.uint8, device=dev)
    ys = [torch.empty_like(x) for x in xs]
    one = lambda i: lab.mc_lab_delta_dec1p(encs[i].data_ptr(), ys[i].data_ptr(), n, es, st.data_ptr(),  # noqa: E731
                                           1 << 14, None, _ops.stream(encs[i]))
    t1 = timed(one)
    out[f"delta_{name}_256MiB_single_pass_us"] = round(t1 * 1e6, 1)
    out[f"delta_{name}_single_pass_ok"] = all(torch.equal(ys[i], xs[i]) for i in range(sets))
    del ys
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
_, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
a, d = _ops.dtype_code("<i2"), _ops.dtype_code("<f4")
st = torch.zeros(lab.mc_lab_c4_dec1p_state_bytes(n, a), dtype=torch.uint8, device=dev)
ys = [torch.empty_like(x) for x in xs]
t1 = timed(lambda i: lab.mc_lab_c4_dec1p(es_[i].data_ptr(), ys[i].data_ptr(), n, a, d, sc3, off4, st.data_ptr(),
                                         1 << 14, None, _ops.stream(xs[i])))
out["c4_single_pass_decode_us"] = round(t1 * 1e6, 1)
out["c4_single_pass_ok"] = bool(torch.equal(ys[0].view(torch.int32), ref.view(torch.int32)))
print(json.dumps(out), flush=True)
