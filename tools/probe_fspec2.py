"""Float Delta decode of one 256 MiB-of-output chunk for float16 and mixed
dtype/astype pairs: the speculative scan (default) against the serial chain
(MCODEC_FSPEC=0 in a child), on data whose every add is exact (small
integers, which verify entirely).  Rotating buffers, event-timed median;
one JSON line.  Usage: python tools/probe_fspec2.py"""
import json
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta  # noqa: E402

TD = {"<f2": torch.float16, "<f4": torch.float32, "<f8": torch.float64, "<i2": torch.int16}


def time_decode(dt, at, out_bytes, reps=7, rot=3):
    dev = torch.device("cuda", 0)
    n = out_bytes // np.dtype(dt).itemsize
    g = torch.Generator(device=dev).manual_seed(1)
    steps = torch.randint(-3, 4, (n,), device=dev, generator=g, dtype=torch.int32)
    x = (torch.cumsum(steps, 0) % 1000).to(TD[dt])
    codec = Delta(dtype=dt, astype=at)
    encs = [codec.encode(x) for _ in range(rot)]
    torch.cuda.synchronize()
    ts = []
    for r in range(reps):
        e = encs[r % rot]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        codec.decode(e)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    us = float(np.median(ts))
    alg = n * (np.dtype(dt).itemsize + np.dtype(at).itemsize)
    return {"us": round(us, 1), "GBps_alg": round(alg / us / 1e3, 2)}


def main():
    if len(sys.argv) > 1:  # child: one measurement
        dt, at, nb = sys.argv[1], sys.argv[2], int(sys.argv[3])
        print(json.dumps(time_decode(dt, at, nb)), flush=True)
        return
    out = {}
    for dt, at, nb in (("<f2", "<f2", 256 << 20), ("<f8", "<f4", 256 << 20), ("<f4", "<f2", 256 << 20),
                       ("<f8", "<i2", 256 << 20), ("<f4", "<f4", 256 << 20)):
        key = f"{dt}<-{at}"
        out[key] = {"speculative": time_decode(dt, at, nb)}
        if dt == "<f4" and at == "<f4":
            continue
        env = dict(os.environ, MCODEC_FSPEC="0", NUMCODECS_AMD_LIB=os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libmcodec_lab.so"))
        r = subprocess.run([sys.executable, __file__, dt, at, str(16 << 20)], capture_output=True, text=True,
                           env=env, timeout=300)
        out[key]["serial_16MiB"] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
