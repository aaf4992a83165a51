"""Where the one-launch CRC verify's finish goes (verdict r5 item 5): the
product entry point (mc_checksum32_verify_fused, location "start", 16-B
aligned buffer, verdict in mapped host memory) timed at 256 MiB + 4 encoded
bytes (4097 tiles of 64 KiB: the stored word makes one 4-byte tile) and at
256 MiB (4096 tiles), and the lab restatement with wall_clock64() stamps
(tools/lab/lab_ck_stamp.hip: round 5's finish) broken down per phase; then
the 256 MiB encode (payload copy + footer) in one launch (ticket) against
the two-launch schedule (tiles + k_ck_finalize).  One JSON line per
measurement.

Usage: python tools/probe_ck_stamp.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402
from numcodecs_amd import _native  # noqa: E402

import ctypes  # noqa: E402

lib = _native.lib
lab = _lab()
lab.mc_lab_crc_verify_stamp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
lab.mc_lab_crc_verify_stamp.restype = ctypes.c_int
dev = torch.device("cuda:0")
st = torch.cuda.current_stream().cuda_stream
MiB = 1 << 20
buf = torch.randint(0, 256, (256 * MiB + 4,), dtype=torch.uint8, device=dev)
ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
ws = torch.empty(8 * MiB, dtype=torch.uint8, device=dev)
rec = lib.mc_verdict_alloc()
out_ptr = lib.mc_host_device_pointer(rec)
rec_np = np.ctypeslib.as_array((ctypes.c_uint32 * 4).from_address(rec))
seq = [0]


def nxt():
    seq[0] = seq[0] % 0xFFFFFFFF + 1
    return seq[0]


def timed(fn, reps=10, groups=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(groups):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return round(ts[len(ts) // 2], 2), round(ts[0], 2)


def product(kind, nbytes):
    rc = lib.mc_checksum32_verify_fused(kind, buf.data_ptr(), nbytes, 0, None, 0, _native.MC_CK_START, out_ptr,
                                        nxt(), ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
    assert rc == 0, rc


def stamped(kind, nbytes, grid, stamps):
    rc = lab.mc_lab_crc_verify_stamp(kind, buf.data_ptr(), nbytes, 0, out_ptr, nxt(), ws.data_ptr(),
                                     ticket.data_ptr(), grid, stamps.data_ptr(), st)
    assert rc == 0, rc


for kind, name in ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C")):
    for nbytes in (256 * MiB + 4, 256 * MiB):
        med, best = timed(lambda: product(kind, nbytes))
        product(kind, nbytes)
        torch.cuda.synchronize()
        ref = (int(rec_np[0]), int(rec_np[1]))
        print(json.dumps({"probe": "ck_stamp", "what": "product", "kind": name, "encoded": nbytes,
                          "tiles": -(-nbytes // 65536), "us_med": med, "us_best": best}), flush=True)
        for grid in (2048,):
            stamps = torch.zeros(4 * grid + 8, dtype=torch.int64, device=dev)
            med, best = timed(lambda: stamped(kind, nbytes, grid, stamps))
            stamped(kind, nbytes, grid, stamps)
            torch.cuda.synchronize()
            got = (int(rec_np[0]), int(rec_np[1]))
            s = stamps.cpu().numpy().astype(np.int64)
            blk = s[: 4 * grid].reshape(grid, 4)
            ls = s[4 * grid:]
            t0 = blk[:, 0].min()
            us = lambda v: round(float(v - t0) / 100.0, 2)  # noqa: E731  (100 MHz ticks)
            loop = blk[:, 1] - t0
            order = np.argsort(blk[:, 1])
            print(json.dumps({
                "probe": "ck_stamp", "what": "lab_stamped", "kind": name, "encoded": nbytes, "grid": grid,
                "ok": got == ref, "us_med": med, "us_best": best,
                "start_max_us": us(blk[:, 0].max()),
                "loop_done_us": {"p50": round(float(np.percentile(loop, 50)) / 100, 2),
                                 "p99": round(float(np.percentile(loop, 99)) / 100, 2),
                                 "max": us(blk[:, 1].max()), "max_block": int(order[-1]),
                                 "second_max": us(blk[order[-2], 1])},
                "drain_us_max": round(float((blk[:, 2] - blk[:, 1]).max()) / 100, 2),
                "drain_us_p50": round(float(np.percentile(blk[:, 2] - blk[:, 1], 50)) / 100, 2),
                "arrive_us_max": round(float((blk[:, 3] - blk[:, 2]).max()) / 100, 2),
                "arrive_us_p50": round(float(np.percentile(blk[:, 3] - blk[:, 2], 50)) / 100, 2),
                "last_arrival_done_us": us(blk[:, 3].max()),
                "last_block": {"tables": us(ls[0]), "loads": us(ls[1]), "fold": us(ls[2]), "finish": us(ls[3]),
                               "published": us(ls[4])},
            }), flush=True)

# the verdict's cost: no seq word (nothing published), and the record in device memory
dev_rec = torch.zeros(4, dtype=torch.int32, device=dev)
for kind, name in ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C")):
    for what, optr, sq in (("host_record_seq", out_ptr, None), ("host_record_noseq", out_ptr, 0),
                           ("device_record_noseq", dev_rec.data_ptr(), 0)):
        def ver():
            rc = lib.mc_checksum32_verify_fused(kind, buf.data_ptr(), 256 * MiB + 4, 0, None, 0,
                                                _native.MC_CK_START, optr, nxt() if sq is None else sq,
                                                ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
            assert rc == 0, rc
        med, best = timed(ver)
        print(json.dumps({"probe": "ck_stamp", "what": "verify_record", "kind": name, "record": what,
                          "us_med": med, "us_best": best}), flush=True)

dst = torch.empty(256 * MiB + 4, dtype=torch.uint8, device=dev)
outd = torch.zeros(4, dtype=torch.int32, device=dev)
for kind, name in ((_native.MC_CK_CRC32, "CRC32"), (_native.MC_CK_CRC32C, "CRC32C")):
    n = 256 * MiB
    res = {}
    for sched, tk in (("one_launch", ticket.data_ptr()), ("two_launch", None)):
        def enc():
            rc = lib.mc_checksum32_encode_fused(kind, buf.data_ptr(), dst.data_ptr(), n, 0, None, 0,
                                                _native.MC_CK_START, outd.data_ptr(), ws.data_ptr(), ws.numel(),
                                                tk, st)
            assert rc == 0, rc
        med, best = timed(enc)
        torch.cuda.synchronize()
        res[sched] = (int(outd[0].item()) & 0xFFFFFFFF, dst[:4].cpu().numpy().tobytes())
        print(json.dumps({"probe": "ck_stamp", "what": "encode", "kind": name, "schedule": sched, "bytes": n,
                          "us_med": med, "us_best": best}), flush=True)
    assert res["one_launch"] == res["two_launch"], res
assert not ticket.any()
