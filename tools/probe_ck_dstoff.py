"""CRC32 / CRC32C / Adler32 256 MiB encode (tiles + finalize) with the payload
copy written at dst + off, off = 0, 4, 8, 12, 16 (16-B aligned copies take
nontemporal 16-B stores, 4-B aligned ones plain 16-B stores).
Usage: python tools/probe_ck_dstoff.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import _native, _ops, batch  # noqa: E402

N = 256 << 20
dev = torch.device("cuda:0")
xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(3)]
outs = [torch.empty(N + 64, dtype=torch.uint8, device=dev) for _ in range(3)]
lib = _native.lib
st = _ops.stream(xs[0])


def timed(fn):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(10):
            fn(i % 3)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) * 100.0
        best = t if best is None else min(best, t)
    return best


for name in ("crc32", "crc32c", "adler32"):
    kind = batch._CK_KINDS[name][0]
    ws_n = lib.mc_checksum32_workspace(kind, 1, N)
    ws = torch.empty(max(ws_n, 16), dtype=torch.uint8, device=dev)
    res = {}
    for off in (0, 4, 8, 12, 16):
        def two(i, off=off):
            rc = lib.mc_checksum32_encode_batch(kind, xs[i].data_ptr(), N, outs[i].data_ptr() + off, N + 4, 1, N, 0,
                                                None, 0, _native.MC_CK_END, None, ws.data_ptr(), ws.numel(), st)
            assert rc == 0, rc
        res[off] = round(timed(two), 1)
    print(json.dumps({"probe": "ck_encode_dst_offset", "codec": name, "us_by_offset": res}), flush=True)
