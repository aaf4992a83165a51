"""C4 decode/encode with 4 rotating buffer sets (so no call finds its input in
the 256 MiB Infinity Cache from a previous call); knobs are read once per
process (MCODEC_C4_LOADS).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, batch  # noqa: E402

n = 64 << 20
dev = torch.device("cuda:0")
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
pipe = batch.FilterPipeline([fso, Delta(dtype="<i2"), Shuffle(2)])
sets = 4
xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(sets)]
es = [pipe.encode(x) for x in xs]
outs = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(sets)]
ref = fso.decode(Delta(dtype="<i2").decode(Shuffle(2).decode(es[0])))
ok = bool(torch.equal(pipe.decode(es[0]).view(torch.int32), ref.view(torch.int32)))


def timed(fn, reps=40):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % sets)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t_dec = timed(lambda i: pipe.decode(es[i]))
t_enc = timed(lambda i: pipe.encode(xs[i]))
print(json.dumps({"loads": os.environ.get("MCODEC_C4_LOADS", "0"),
                  "ok": ok, "dec_us": round(t_dec * 1e3, 1), "enc_us": round(t_enc * 1e3, 1),
                  "encdec_GiBps": round(2 * 4 * n / (1 << 30) / ((t_dec + t_enc) / 1e3), 1)}), flush=True)
