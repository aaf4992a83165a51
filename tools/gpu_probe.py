"""First-contact probe on a MI355X box: runtime binding, shuffle correctness
against torch's own transpose, and a variant x grid sweep of the shuffle
kernels (device-resident buffers, rotating sets to defeat the 256 MiB MALL).

Usage: python tools/gpu_probe.py [--quick]
"""

import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "numcodecs_amd", "_lib", "libmcodec.so"))
V = ctypes.c_void_p
S = ctypes.c_size_t
I = ctypes.c_int
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402  (the sweep entry points live in the lab library)

lab = _lab()
lib.mc_device_count.restype = I


def maps():
    with open("/proc/self/maps") as f:
        return sorted({l.split()[-1] for l in f if "amdhip64" in l or "hsa-runtime" in l})


def main():
    quick = "--quick" in sys.argv
    dev = torch.device("cuda:0")
    torch.cuda.init()
    print("torch", torch.__version__, "hip", torch.version.hip, torch.cuda.get_device_name(0))
    print("mc_device_count", lib.mc_device_count())
    print("runtime libs mapped:", maps())
    st = torch.cuda.current_stream().cuda_stream

    # correctness vs torch transpose
    g = torch.Generator(device=dev).manual_seed(0)
    bad = 0
    for es in (2, 3, 4, 8, 16, 5):
        for nbytes in (es * 1000, es * 4096 * 3 + es * 100, es * 4096 * 16, 1 << 22, es * 12345):
            if nbytes % es:
                continue
            count = nbytes // es
            x = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g)
            ref = x.view(count, es).t().contiguous().view(-1)
            for var in (0, 1, 2, 3, 4, 9, 10, 11):
                y = torch.empty_like(x)
                rc = lab.mc_lab_shuffle_variant(x.data_ptr(), y.data_ptr(), nbytes, es, 1, var, 0, st)
                z = torch.empty_like(x)
                rc2 = lab.mc_lab_shuffle_variant(y.data_ptr(), z.data_ptr(), nbytes, es, 0, var, 0, st)
                torch.cuda.synchronize()
                ok = rc == 0 and rc2 == 0 and torch.equal(y, ref) and torch.equal(z, x)
                if not ok:
                    bad += 1
                    print("MISMATCH es", es, "nbytes", nbytes, "var", var, rc, rc2,
                          torch.equal(y, ref), torch.equal(z, x))
    print("correctness failures:", bad)

    # bandwidth sweep: 256 MiB chunks, 4 rotating buffer sets
    N = 256 << 20
    sets = 4
    ins = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev, generator=g) for _ in range(sets)]
    outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(sets)]
    iters = 10 if quick else 20
    results = []

    def timeit(fn):
        for i in range(3):
            fn(i % sets)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i % sets)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e-3

    t = timeit(lambda i: outs[i].copy_(ins[i]))
    print(f"D2D copy 256MiB: {t*1e3:.3f} ms  {2*N/t/1e9:.1f} GB/s")
    results.append({"op": "copy", "ms": t * 1e3, "GBps": 2 * N / t / 1e9})
    for es in (4, 8, 2):
        for enc in (1, 0):
            for var in (1, 2, 3, 9, 10, 11):
                for grid in ((0, 4096, 8192, 16384) if not quick else (0,)):
                    def fn(i, es=es, enc=enc, var=var, grid=grid):
                        rc = lab.mc_lab_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), N, es, enc, var, grid, st)
                        assert rc == 0, rc
                    t = timeit(fn)
                    r = {"es": es, "enc": enc, "var": var, "grid": grid, "ms": round(t * 1e3, 4),
                         "GBps": round(2 * N / t / 1e9, 1)}
                    results.append(r)
                    print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe.json"), "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
