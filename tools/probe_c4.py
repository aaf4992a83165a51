"""C4 decode schedule probe: times the fused FSO->Delta->Shuffle(2) decode
(variant 0 = the product schedule through the codec API, 1-7 the lab's
schedules, tools/lab/lab_c4.hip) and checks it against the codec-by-codec
decode.   python tools/probe_c4.py [n] [variant]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
dev = torch.device("cuda:0")
x = 1000.0 + 10.0 * torch.rand(n, device=dev)
fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
dl, sh = Delta(dtype="<i2"), Shuffle(2)
pipe = batch.FilterPipeline([fso, dl, sh])
e = pipe.encode(x)
ref = fso.decode(dl.decode(sh.decode(e)))
if variant:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from lab.lablib import lab as _lab  # noqa: E402
    from numcodecs_amd import _ops  # noqa: E402

    lab = _lab()
    _, _, sc3, off4 = batch._c4_scalars(fso, dl, sh)
    raw = e.view(torch.uint8).reshape(-1)
    outb = torch.empty(4 * n, dtype=torch.uint8, device=dev)
    ws = _ops.workspace(lab.mc_lab_c4_decode_workspace(n), raw)

    def lab_decode():
        assert lab.mc_lab_c4_decode_variant(raw.data_ptr(), outb.data_ptr(), n, _ops.dtype_code("<i2"),
                                            _ops.dtype_code("<f4"), sc3, off4, ws.data_ptr(), ws.numel(),
                                            variant, _ops.stream(raw)) == 0
        return outb.view(torch.float32)
    decode = lab_decode
else:
    def decode():
        return pipe.decode(e)
got = decode()
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


t_dec = timed(decode) if n >= (16 << 20) else None
t_enc = timed(lambda: pipe.encode(x)) if n >= (16 << 20) else None
print(json.dumps({"variant": variant, "n": n, "ok": ok,
                  "dec_ms": t_dec, "enc_ms": t_enc,
                  "encdec_GiBps": round(2 * 4 * n / (1 << 30) / ((t_dec + t_enc) / 1e3), 1) if t_dec else None}),
      flush=True)
