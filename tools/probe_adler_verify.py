"""Single-chunk Adler32 / CRC32 verify of 256 MiB (+4 checksum bytes at the
start, the codecs' default location): kernel time of the one-launch verify
(mc_checksum32_verify_fused with a ticket) and of the two-launch schedule
(ticket NULL: tiles + finalize), event-timed over back-to-back launches, and
the public-API decode wall time.  One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, Adler32, _native, _ops  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
out = {}
for name, cls, kind in (("adler32", Adler32, _native.MC_CK_ADLER32), ("crc32", CRC32, _native.MC_CK_CRC32)):
    c = cls()
    encs = [c.encode(torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)) for _ in range(4)]
    st = _ops.stream(encs[0])
    sl = _ops._verify_slot(encs[0], st)
    ws = sl.workspace(lib.mc_checksum32_workspace(kind, 1, N))
    init = 1 if kind == _native.MC_CK_ADLER32 else 0
    pair = torch.zeros(2, dtype=torch.int32, device=dev)
    res = {}
    for label, tk in (("fused_us", sl.ticket.data_ptr()), ("two_launch_us", None)):
        def launch(i, tk=tk):
            _native.check(lib.mc_checksum32_verify_fused(kind, encs[i].data_ptr(), N + 4, init, None, 0,
                                                         _native.MC_CK_START, pair.data_ptr(), 0, ws.data_ptr(),
                                                         ws.numel(), tk, st), "verify")
        for i in range(4):
            launch(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(20):
            launch(r % 4)
        e1.record()
        torch.cuda.synchronize()
        res[label] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    for i in range(4):
        c.decode(encs[i])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(20):
        c.decode(encs[r % 4])
    res["api_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
    out[name] = res
    del encs
print(json.dumps(out), flush=True)
