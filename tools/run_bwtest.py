"""Run the HBM calibration kernels of tools/bwtest.hip on cuda:0.

Usage: python tools/run_bwtest.py   (expects tools/_build/libbwtest.so; build
with: hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -shared -fPIC
tools/bwtest.hip -o tools/_build/libbwtest.so)
"""

import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libbwtest.so"))
lib.bw_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                        ctypes.c_int, ctypes.c_void_p]

NAMES = {0: "copy U4", 1: "copy U4 ntst", 2: "copy U4 ntld+ntst", 3: "copy U1", 4: "copy U8",
         5: "copy U8 ntst", 6: "copy U2", 7: "copy U4 ntld", 8: "read U4", 9: "write U4",
         10: "write U4 ntst"}


def main():
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    N = 256 << 20
    sets = 4
    ins = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(sets)]
    iters = 30
    res = []
    for var in NAMES:
        for grid in (512, 1024, 2048, 4096, 8192, 16384, 65536):
            def fn(i):
                assert lib.bw_copy(ins[i].data_ptr(), outs[i].data_ptr(), N, var, grid, st) == 0
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
            t = e0.elapsed_time(e1) / iters * 1e-3
            nb = N if var >= 8 else 2 * N
            r = {"kernel": NAMES[var], "grid": grid, "us": round(t * 1e6, 2), "GBps": round(nb / t / 1e9, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bwtest.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
