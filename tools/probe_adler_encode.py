"""Adler32 encode of one 256 MiB chunk (payload copy + footer) in one launch
(ticket: the workgroups' sums ride the arrival atomics) against tiles +
finalize (NULL ticket), both footer locations, 4 rotating buffer sets as
bench.py times them; outputs compared.  One JSON line per case.

Usage: python tools/probe_adler_encode.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from numcodecs_amd import _native  # noqa: E402

lib = _native.lib
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
N = 256 * MiB
SETS = 4
srcs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(SETS)]
dsts = [torch.empty(N + 4, dtype=torch.uint8, device=dev) for _ in range(SETS)]
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(lib.mc_checksum32_workspace(_native.MC_CK_ADLER32, 1, N) + 16, dtype=torch.uint8, device=dev)


def enc(kind, loc, tk, i):
    rc = lib.mc_checksum32_encode_fused(kind, srcs[i].data_ptr(), dsts[i].data_ptr(), N, 1, None, 0, loc, None,
                                        ws.data_ptr(), ws.numel(), tk, st)
    assert rc == 0, rc


def timed(fn, reps=20):
    for i in range(SETS):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        fn(r % SETS)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


res = {}
for rnd in range(5):
    for kind, name in ((_native.MC_CK_ADLER32, "Adler32"), (_native.MC_CK_CRC32, "CRC32"),
                       (_native.MC_CK_CRC32C, "CRC32C")):
        for loc_name, loc in (("start", _native.MC_CK_START), ("end", _native.MC_CK_END)):
            outs = {}
            for sched, tk in (("one_launch", ticket.data_ptr()), ("two_launch", None)):
                res.setdefault((name, loc_name, sched), []).append(timed(lambda i: enc(kind, loc, tk, i)))
                if rnd == 0:
                    enc(kind, loc, tk, 0)
                    outs[sched] = dsts[0].clone()
            if rnd == 0:
                assert torch.equal(outs["one_launch"], outs["two_launch"]), (name, loc_name)
for (name, loc_name, sched), ts in res.items():
    ts.sort()
    print(json.dumps({"probe": "ck_encode_sets", "kind": name, "location": loc_name, "schedule": sched,
                      "sets": SETS, "us_med": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2)}), flush=True)
assert not ticket.any()
