"""Round-5 probe: the 256 MiB CRC32 / CRC32C encode as one launch (arrival
before the last tile's payload stores) against tiles + finalize, and the
Blosc BITSHUFFLE filter (typesize 4 / 8, 256 KiB blocks, 32x32 transposes)
-- HIP events, 3 rotating buffer sets, one JSON line each; correctness of the
one-launch encode against the two-launch one checked first."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import _native, _ops, batch  # noqa: E402
from numcodecs_amd import blosc_shuffle as bsh  # noqa: E402

MiB = 1 << 20
N = 256 * MiB
SETS = 3
dev = torch.device("cuda:0")
xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(SETS)]
outs = [torch.empty(N + 4, dtype=torch.uint8, device=dev) for _ in range(SETS)]


def timed(fn, reps=10):
    for i in range(SETS):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % SETS)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


lib = _native.lib
st = _ops.stream(xs[0])
for name in ("crc32", "crc32c"):
    kind = batch._CK_KINDS[name][0]
    ws_n = lib.mc_checksum32_workspace(kind, 1, N)
    ws = torch.empty(max(ws_n, 16), dtype=torch.uint8, device=dev)
    ticket = torch.zeros(_native.MC_ARRIVAL_WORDS, dtype=torch.int32, device=dev)
    init = 0

    def fused(i):
        rc = lib.mc_checksum32_encode_fused(kind, xs[i].data_ptr(), outs[i].data_ptr(), N, init, None, 0,
                                            _native.MC_CK_END, None, ws.data_ptr(), ws.numel(), ticket.data_ptr(), st)
        assert rc == 0, rc

    def two(i):
        rc = lib.mc_checksum32_encode_batch(kind, xs[i].data_ptr(), N, outs[i].data_ptr(), N + 4, 1, N, init, None, 0,
                                            _native.MC_CK_END, None, ws.data_ptr(), ws.numel(), st)
        assert rc == 0, rc

    two(0)
    torch.cuda.synchronize()
    ref = outs[0].clone()
    outs[0].zero_()
    fused(0)
    torch.cuda.synchronize()
    ok = torch.equal(ref, outs[0])
    t_f, t_2 = timed(fused), timed(two)
    print(json.dumps({"probe": f"{name}_encode_256MiB", "fused_us": round(t_f, 1), "two_launch_us": round(t_2, 1),
                      "fused_frac": round((2 * N + 4) / (t_f * 1e-6) / 1e9 / 8000, 4), "same_bytes": ok}), flush=True)

for ts in (4, 8):
    fw = [bsh.shuffle(x, ts, 256 * 1024, bsh.BITSHUFFLE) for x in xs]
    back = bsh.unshuffle(fw[0], ts, 256 * 1024, bsh.BITSHUFFLE)
    ok = torch.equal(back.view(torch.uint8).reshape(-1), xs[0])
    t_e = timed(lambda i: bsh.shuffle(xs[i], ts, 256 * 1024, bsh.BITSHUFFLE))
    t_d = timed(lambda i: bsh.unshuffle(fw[i], ts, 256 * 1024, bsh.BITSHUFFLE))
    print(json.dumps({"probe": f"blosc_bitshuffle_ts{ts}_256MiB", "enc_us": round(t_e, 1), "dec_us": round(t_d, 1),
                      "enc_frac": round(2 * N / (t_e * 1e-6) / 1e9 / 8000, 4),
                      "dec_frac": round(2 * N / (t_d * 1e-6) / 1e9 / 8000, 4), "round_trip": ok}), flush=True)
