"""A/B of the same-type Delta encode kernel (k_delta_enc_same): 4 or 8
16-B vectors per thread (mc_sched.delta_enc_dv, set through the lab
library), 256 MiB per dtype and byte order, rotating buffers, HIP events on
the launch stream; every variant's output checked against the first.

    python tools/probe_delta_enc_dv.py  -> one JSON line per case
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import _ops  # noqa: E402


def main():
    lab = _lab()
    lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lab.mc_lab_set_sched.restype = ctypes.c_int
    lab.mc_delta_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    nbytes = 256 << 20
    srcs = [torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev) for _ in range(3)]
    dsts = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(3)]
    dv0 = lab.mc_lab_set_sched(b"delta_enc_dv", 4)
    rows = []
    dvs = [int(v) for v in os.environ.get("DVS", "4,8,4,8").split(",")]
    pairs = [p.split(":") for p in os.environ.get("PAIRS", "|u1:|u1,<i2:<i2,>i2:>i2,<i4:<i4,<f4:<f4,>f4:>f4,<f8:<f8,>f8:>f8").split(",")]
    for dt, at in pairs:
        code, acode = _ops.dtype_code(dt), _ops.dtype_code(at)
        n = nbytes // int(dt[-1])
        ref = None
        for dv in dvs:
            lab.mc_lab_set_sched(b"delta_enc_dv", dv)
            for i in range(3):
                assert lab.mc_delta_encode(srcs[i].data_ptr(), dsts[i].data_ptr(), n, code, acode, st) == 0
            torch.cuda.synchronize()
            if ref is None:
                ref = dsts[0].clone()
            ok = bool(torch.equal(ref, dsts[0]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 30
            e0.record()
            for r in range(reps):
                lab.mc_delta_encode(srcs[r % 3].data_ptr(), dsts[r % 3].data_ptr(), n, code, acode, st)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            rows.append({"dtype": dt, "astype": at, "dv": dv, "us": round(us, 2), "GBps": round(2 * nbytes / us / 1e3, 1), "ok": ok})
            print(json.dumps(rows[-1]), flush=True)
    lab.mc_lab_set_sched(b"delta_enc_dv", dv0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_delta_enc_dv.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
