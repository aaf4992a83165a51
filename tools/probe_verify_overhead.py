"""Where does a single-chunk checksum decode spend its time?  One 256 MiB
device chunk, 3 rotating buffers, for Fletcher32, CRC32, CRC32C and Adler32:

  kernel_us         the fused verify kernel alone, back-to-back launches
                    timed with HIP events (no host wait per call)
  host_launch_us    CPU time of the ctypes launch call itself
  raw_sync_us       ctypes launch + mc_stream_synchronize per call
  raw_wait_us       ctypes launch + mc_verdict_wait (spin on the seq word)
  api_us            Codec().decode through the public API

    python tools/probe_verify_overhead.py  -> one JSON line per codec
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, CRC32C, Adler32, Fletcher32, _native, _ops  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
reps = 50


def wall(fn):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i % 3)
    return (time.perf_counter() - t0) / reps * 1e6


def probe(name, codec):
    encs = [codec.encode(torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)) for _ in range(3)]
    st = _ops.stream(encs[0])
    sl = _ops._verify_slot(encs[0], st)
    if name == "fletcher32":
        ws = sl.workspace(lib.mc_fletcher32_workspace(N + 4))

        def launch(i, seq=0):
            lib.mc_fletcher32_verify_fused(encs[i].data_ptr(), N + 4, sl.out_ptr, seq, ws.data_ptr(), ws.numel(),
                                           sl.ticket.data_ptr(), st)
    else:
        kind, loc = codec._kind, codec._loc()
        ws = sl.workspace(lib.mc_checksum32_workspace(kind, 1, N))

        def launch(i, seq=0):
            lib.mc_checksum32_verify_fused(kind, encs[i].data_ptr(), N + 4, codec._value, None, 0, loc,
                                           sl.out_ptr, seq, ws.data_ptr(), ws.numel(), sl.ticket.data_ptr(), st)

    out = {"codec": name}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(3):
        launch(i)
    torch.cuda.synchronize()
    e0.record()
    for i in range(reps):
        launch(i % 3)
    e1.record()
    torch.cuda.synchronize()
    out["kernel_us"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    t0 = time.perf_counter()
    for i in range(reps):
        launch(i % 3)
    out["host_launch_us"] = round((time.perf_counter() - t0) / reps * 1e6, 2)
    torch.cuda.synchronize()

    def raw_sync(i):
        launch(i)
        lib.mc_stream_synchronize(st)

    def raw_wait(i):
        seq = sl.next_seq()
        launch(i, seq)
        assert lib.mc_verdict_wait(sl.rec, seq, st) == 0

    out["raw_sync_us"] = round(wall(raw_sync), 2)
    out["raw_wait_us"] = round(wall(raw_wait), 2)
    out["api_us"] = round(wall(lambda i: codec.decode(encs[i])), 2)
    out["api_minus_kernel_us"] = round(out["api_us"] - out["kernel_us"], 2)
    print(json.dumps(out), flush=True)
    return out


def main():
    rows = [probe(n, c) for n, c in (("fletcher32", Fletcher32()), ("crc32", CRC32()), ("crc32c", CRC32C()),
                                     ("adler32", Adler32()))]
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/probe_verify_overhead.json", "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
