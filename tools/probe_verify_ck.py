"""Single-chunk CRC32 / Adler32 / Fletcher32 decode wall time per call
through the public API, 256 MiB, for 3 and 4 rotating buffer sets and both
checksum locations; plus the raw one-launch verify + host wait, and the
verify with a stream synchronisation instead (seq = 0).  One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, Adler32, Fletcher32, _native, _ops  # noqa: E402
from numcodecs_amd._native import lib  # noqa: E402

dev = torch.device("cuda:0")
N = 256 << 20
out = {}


def wall(fn, sets, reps=30):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i % sets)
    return round((time.perf_counter() - t0) / reps * 1e6, 1)


xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]
for name, mk in (("crc32_start", lambda: CRC32()), ("crc32_end", lambda: CRC32(location="end")),
                 ("adler32_start", lambda: Adler32()), ("fletcher32", lambda: Fletcher32())):
    c = mk()
    encs = [c.encode(x) for x in xs]
    out[name] = {"api_3sets_us": wall(lambda i: c.decode(encs[i]), 3), "api_4sets_us": wall(lambda i: c.decode(encs[i]), 4)}
    if name.startswith("crc32"):
        st = _ops.stream(encs[0])
        sl = _ops._verify_slot(encs[0], st)
        loc = _native.MC_CK_START if name.endswith("start") else _native.MC_CK_END
        ws = sl.workspace(lib.mc_checksum32_workspace(_native.MC_CK_CRC32, 1, N))

        def raw(i, seq_on=True):
            seq = sl.next_seq() if seq_on else 0
            _native.check(lib.mc_checksum32_verify_fused(_native.MC_CK_CRC32, encs[i].data_ptr(), N + 4, 0, None, 0,
                                                         loc, sl.out_ptr, seq, ws.data_ptr(), ws.numel(),
                                                         sl.ticket.data_ptr(), st), "verify")
            if seq:
                _native.check(lib.mc_verdict_wait(sl.rec, seq, st), "wait")
            else:
                _native.check(lib.mc_stream_synchronize(st), "sync")

        out[name]["raw_wait_us"] = wall(lambda i: raw(i, True), 4)
        out[name]["raw_sync_us"] = wall(lambda i: raw(i, False), 4)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(20):
            _native.check(lib.mc_checksum32_verify_fused(_native.MC_CK_CRC32, encs[i % 4].data_ptr(), N + 4, 0, None,
                                                         0, loc, sl.out_ptr, 0, ws.data_ptr(), ws.numel(),
                                                         sl.ticket.data_ptr(), st), "verify")
        e1.record()
        torch.cuda.synchronize()
        out[name]["kernel_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    del encs
print(json.dumps(out), flush=True)
