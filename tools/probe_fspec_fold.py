"""A/B of the speculative float Delta decode's two schedules on one box:
mc_delta_decode with an arrival ticket (tile prefixes folded into the reduce
pass: reduce_g + apply + walk) against without (reduce + k_fspec_pre + apply
+ walk), 256 MiB of smooth f4 (every tile verifies), 4 rotating buffer sets,
HIP events around 20 calls per round, rounds interleaved.
    python tools/probe_fspec_fold.py [rounds]   -> one JSON line"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, _native, _ops  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    n = (256 << 20) // 4
    sets = 4
    xs = [(torch.arange(n, device=dev, dtype=torch.float64) * 0.25 % 4096.0).float() for _ in range(sets)]
    encs = [Delta("<f4").encode(x).view(torch.uint8) for x in xs]
    outs = [torch.empty(n * 4, dtype=torch.uint8, device=dev) for _ in range(sets)]
    a = _ops.dtype_code("<f4")
    ws_n = _native.lib.mc_delta_decode_workspace(n, a, a)
    ws = torch.zeros(ws_n, dtype=torch.uint8, device=dev)
    ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def call(i, tk):
        rc = _native.lib.mc_delta_decode(encs[i].data_ptr(), outs[i].data_ptr(), n, a, a, ws.data_ptr(), ws_n,
                                         ticket.data_ptr() if tk else None, st)
        assert rc == 0, rc

    for tk in (True, False):  # warm + parity
        for i in range(sets):
            call(i, tk)
            assert torch.equal(outs[i].view(torch.float32), xs[i])
    res = {"ticket_us": [], "pre_us": []}
    for _ in range(rounds):
        for tk, key in ((True, "ticket_us"), (False, "pre_us")):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for k in range(20):
                call(k % sets, tk)
            e1.record()
            torch.cuda.synchronize()
            res[key].append(round(e0.elapsed_time(e1) * 1e3 / 20, 2))
    res["ticket_med"] = sorted(res["ticket_us"])[len(res["ticket_us"]) // 2]
    res["pre_med"] = sorted(res["pre_us"])[len(res["pre_us"]) // 2]
    assert int(ticket.abs().sum()) == 0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
