"""Where does a single-chunk checksum decode spend its time?  One 256 MiB
device chunk, 3 rotating buffers, Fletcher32:

  sync_idle_us      mc_stream_synchronize on an idle stream
  kernel_us         the fused verify kernel alone, back-to-back launches
                    timed with HIP events (no host wait per call)
  raw_sync_us       ctypes launch + mc_stream_synchronize per call
  raw_wait_us       ctypes launch + mc_verdict_wait (spin on the seq word)
  api_us            Fletcher32().decode through the public API

    python tools/probe_verify_overhead.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Fletcher32, _ops  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
c = Fletcher32()
encs = [c.encode(torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)) for _ in range(3)]
st = _ops.stream(encs[0])
sl = _ops._verify_slot(encs[0], st)
ws = sl.workspace(lib.mc_fletcher32_workspace(N + 4))
out = {}
reps = 50


def wall(fn):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i % 3)
    return (time.perf_counter() - t0) / reps * 1e6


def launch(i, seq=0):
    lib.mc_fletcher32_verify_fused(encs[i].data_ptr(), N + 4, sl.out_ptr, seq, ws.data_ptr(), ws.numel(),
                                   sl.ticket.data_ptr(), st)


out["sync_idle_us"] = round(wall(lambda i: lib.mc_stream_synchronize(st)), 2)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for i in range(reps):
    launch(i % 3)
e1.record()
torch.cuda.synchronize()
out["kernel_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)


def raw_sync(i):
    launch(i)
    lib.mc_stream_synchronize(st)


out["raw_sync_us"] = round(wall(raw_sync), 2)



def raw_wait(i):
    seq = sl.next_seq()
    launch(i, seq)
    assert lib.mc_verdict_wait(sl.rec, seq, st) == 0


out["raw_wait_us"] = round(wall(raw_wait), 2)
out["api_us"] = round(wall(lambda i: c.decode(encs[i])), 2)


def launch_only(i):
    launch(i)


# host-side pieces of the public decode, each timed alone
from numcodecs_amd.compat import to_dbuf  # noqa: E402


def per_call(fn, n=2000):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t0) / n * 1e6, 3)


e = encs[0]
out["py_capturing_us"] = per_call(torch.cuda.is_current_stream_capturing)
out["py_current_device_us"] = per_call(torch.cuda.current_device)
out["py_stream_us"] = per_call(lambda: _ops.stream(e))
out["py_to_dbuf_us"] = per_call(lambda: to_dbuf(e))
out["py_slice_us"] = per_call(lambda: e[: N])
out["py_workspace_query_us"] = per_call(lambda: lib.mc_fletcher32_workspace(N + 4))
out["py_verify_slot_us"] = per_call(lambda: _ops._verify_slot(e, st))
out["py_data_ptr_us"] = per_call(lambda: e.data_ptr())
out["grid_env"] = os.environ.get("MCODEC_F32_FUSED_GRID", "default")
t0 = time.perf_counter()
for i in range(reps):
    launch_only(i % 3)
out["host_launch_us"] = round((time.perf_counter() - t0) / reps * 1e6, 2)
torch.cuda.synchronize()
print(json.dumps(out), flush=True)
