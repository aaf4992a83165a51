"""Batched Shuffle(4) encode/decode of 256 MiB as B rows of 256/B MiB
(batch.shuffle_chunks / unshuffle_chunks), B = 1 .. 4096, 4 rotating buffer
sets, HIP events: does the row size change the kernels' rate?

    python tools/probe_batch_rows.py  -> one JSON line per row count
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import batch  # noqa: E402

MiB = 1 << 20


def timed(fn, sets, reps=20):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        fn(r % sets)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    sets = 4
    rows_list = [int(x) for x in os.environ.get("ROWS", "1,4,16,64,256,1024,4096").split(",")]
    xs = [torch.randn(64 * MiB, device=dev) for _ in range(sets)]
    es = [torch.empty(256 * MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    ds = [torch.empty(256 * MiB, dtype=torch.uint8, device=dev) for _ in range(sets)]
    out = []
    for b in rows_list:
        m = 256 * MiB // b
        xv = [x.view(b, m // 4) for x in xs]
        ev = [e.view(b, m) for e in es]
        dv = [d.view(b, m) for d in ds]
        te = timed(lambda i: batch.shuffle_chunks(xv[i], 4, out=ev[i]), sets)
        td = timed(lambda i: batch.unshuffle_chunks(ev[i], 4, out=dv[i]), sets)
        ok = bool(torch.equal(dv[0].view(torch.float32).reshape(-1), xs[0]))
        out.append({"rows": b, "row_MiB": m / MiB, "enc_us": round(te, 1), "dec_us": round(td, 1),
                    "enc_TBps": round(512 * MiB / te / 1e6, 3), "dec_TBps": round(512 * MiB / td / 1e6, 3), "ok": ok})
        print(json.dumps(out[-1]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_batch_rows.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
