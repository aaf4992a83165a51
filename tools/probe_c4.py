"""C4 decode variant probe (MCODEC_C4_VARIANT is read once per process):
times the fused FSO->Delta->Shuffle(2) decode and checks it against the
codec-by-codec decode.   MCODEC_C4_VARIANT=3 python tools/probe_c4.py [n]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
dev = torch.device("cuda:0")
x = 1000.0 + 10.0 * torch.rand(n, device=dev)
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
e = pipe.encode(x)
ref = fso.decode(dl.decode(sh.decode(e)))
got = pipe.decode(e)
ok = bool(torch.equal(got.view(-1).view(torch.int32), ref.view(-1).view(torch.int32)))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t_dec = timed(lambda: pipe.decode(e)) if n >= (16 << 20) else None
t_enc = timed(lambda: pipe.encode(x)) if n >= (16 << 20) else None
print(json.dumps({"variant": os.environ.get("MCODEC_C4_VARIANT", "0"), "n": n, "ok": ok,
                  "dec_ms": t_dec, "enc_ms": t_enc,
                  "encdec_GiBps": round(2 * 4 * n / (1 << 30) / ((t_dec + t_enc) / 1e3), 1) if t_dec else None}),
      flush=True)
