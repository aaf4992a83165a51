"""Float Delta decode of one chunk: speculative scan (default) vs the serial
chain (the lab library's fspec = 0 schedule in a child), smooth data (every add exact) and random
data (verification fails early, serial fix-up).  Rotating buffers; prints one
JSON line.  Usage: python tools/probe_fspec.py"""
import json
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta  # noqa: E402


def time_decode(dt, n, kind, reps=10, rot=3):
    dev = torch.device("cuda", 0)
    i = torch.arange(n, device=dev, dtype=torch.float64)
    if kind == "smooth":
        x = (5000.0 + 100.0 * torch.sin(2 * np.pi * i / 65536.0)).to(getattr(torch, {"<f4": "float32", "<f8": "float64"}[dt]))
    else:
        x = torch.randn(n, device=dev, dtype=getattr(torch, {"<f4": "float32", "<f8": "float64"}[dt]))
    codec = Delta(dt)
    encs = [codec.encode(x) for _ in range(rot)]
    dec = codec.decode(encs[0])
    assert kind != "smooth" or torch.equal(dec, x)
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
    nbytes = n * np.dtype(dt).itemsize
    return {"us": round(us, 1), "GBps_2N": round(2 * nbytes / us / 1e3, 2)}


def time_batch(dt, rows, n, kind, reps=5):
    from numcodecs_amd import batch

    dev = torch.device("cuda", 0)
    tdt = getattr(torch, {"<f4": "float32", "<f8": "float64"}[dt])
    i = torch.arange(n, device=dev, dtype=torch.float64)
    if kind == "smooth":
        x = (5000.0 + 100.0 * torch.sin(2 * np.pi * i / 65536.0)).to(tdt).repeat(rows, 1)
    else:
        x = torch.randn(rows, n, device=dev, dtype=tdt)
    codec = Delta(dt)
    enc = batch.delta_chunks(x, codec, encode=True)
    dec = batch.delta_chunks(enc, codec, encode=False)
    assert kind != "smooth" or torch.equal(dec.view(tdt), x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        batch.delta_chunks(enc, codec, encode=False, out=dec)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    us = float(np.median(ts))
    return {"us": round(us, 1), "GBps_2N": round(2 * x.numel() * x.element_size() / us / 1e3, 2)}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "serial":
        import ctypes

        from numcodecs_amd import _native

        # serial chain only: a lab-library schedule (the product reads no environment)
        assert ctypes.CDLL(_native.lib_path).mc_lab_set_sched(b"fspec", 0) != -(1 << 31)
        out = {}
        for dt in ("<f4", "<f8"):
            out[f"serial_{dt}_16MiB_smooth"] = time_decode(dt, (16 << 20) // np.dtype(dt).itemsize, "smooth", reps=3)
            out[f"serial_{dt}_batch2048x1MiB_smooth"] = time_batch(dt, 2048, (1 << 20) // np.dtype(dt).itemsize, "smooth", reps=2)
        print(json.dumps(out))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "batchrandom":  # rocprofv3: spec vs serial kernels, random rows
        print(json.dumps({dt: time_batch(dt, 2048, (1 << 20) // np.dtype(dt).itemsize, "random", reps=2)
                          for dt in ("<f4",)}))
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "prof":  # the smooth 256 MiB cases only (rocprofv3)
        print(json.dumps({dt: time_decode(dt, (256 << 20) // np.dtype(dt).itemsize, "smooth") for dt in ("<f4", "<f8")}))
        sys.exit(0)
    # the serial leg runs in a child started before this process touches the GPU
    lab = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libmcodec_lab.so")
    r = subprocess.run([sys.executable, __file__, "serial"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, NUMCODECS_AMD_LIB=lab))
    out = json.loads(r.stdout.strip().splitlines()[-1])
    for dt in ("<f4", "<f8"):
        for mib in (16, 256):
            out[f"spec_{dt}_{mib}MiB_smooth"] = time_decode(dt, (mib << 20) // np.dtype(dt).itemsize, "smooth")
        out[f"spec_{dt}_16MiB_random"] = time_decode(dt, (16 << 20) // np.dtype(dt).itemsize, "random", reps=3)
        for kind in ("smooth", "random"):
            out[f"spec_{dt}_batch2048x1MiB_{kind}"] = time_batch(dt, 2048, (1 << 20) // np.dtype(dt).itemsize, kind,
                                                                 reps=2 if kind == "random" else 5)
    print(json.dumps(out))
