"""Shuffle tile-size sweep (round 4): the product layouts with 1x..8x tiles
(mc_shuffle.hip V_BIG / V_BIG4 / V_BIG8), one workgroup per tile as the
product launches them (lab max_blocks 0; before round 4's fix that meant a
2048-workgroup cap), for es = 2, 4, 8, encode and
decode, the BitRound-fused encode, the lab encodes of lab_shuffle4.hip and
the copy calibration -- interleaved rounds, 4 rotating 256 MiB buffer sets.

Usage: python tools/probe_shuffle_tiles.py [rounds]  -> gpurun_out/probe_shuffle_tiles.json
"""

import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

MiB = 1 << 20
V_REG, V_PAIR, V_BIG, V_BIG4, V_BIG8 = 1, 5, 16, 128, 512


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    n = 256 * MiB
    sets = 4
    ins = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(sets)]
    cfgs = []
    for es, enc, variants in (
        (4, 1, (V_REG | V_BIG4, V_REG | V_BIG8, V_PAIR | V_BIG4, V_PAIR | V_BIG8)),
        (4, 0, (V_PAIR | V_BIG, V_PAIR | V_BIG4, V_PAIR | V_BIG8, V_REG | V_BIG4, V_REG | V_BIG8)),
        (8, 1, (V_PAIR, V_PAIR | V_BIG, V_PAIR | V_BIG4, V_PAIR | V_BIG8)),
        (8, 0, (V_PAIR | V_BIG, V_PAIR | V_BIG4, V_PAIR | V_BIG8)),
        (2, 1, (V_REG | V_BIG4, V_REG | V_BIG8)),
        (2, 0, (V_REG | V_BIG4, V_REG | V_BIG8)),
    ):
        for v in variants:
            cfgs.append((f"es{es}_{'enc' if enc else 'dec'}_v{v}", ("shuffle", es, enc, v)))
    for v in (V_REG | V_BIG4, V_REG | V_BIG8):
        cfgs.append((f"bitround10_es4_enc_v{v}", ("bitround", 4, 1, v)))
    for v in (V_PAIR, V_PAIR | V_BIG4, V_PAIR | V_BIG8):
        cfgs.append((f"bitround10_es8_enc_v{v}", ("bitround", 8, 1, v)))
    for k in (8, 18, 19):
        cfgs.append((f"lab{k}", ("lab", 4, 1, k)))
    cfgs.append(("copy_u8_nt3_g0", ("copy", 8, 3, 0)))
    cfgs.append(("mc_copy_u4", ("mc_copy", 4, 0, 0)))
    cfgs.append(("mc_copy_u8", ("mc_copy", 8, 0, 0)))
    cfgs.append(("copy_u4_nt3_g8192", ("copy", 4, 3, 8192)))

    def run(c, i):
        kind, a, b, v = c[1]
        s, d = ins[i], outs[i]
        if kind == "shuffle":
            rc = lab.mc_lab_shuffle_variant(s.data_ptr(), d.data_ptr(), n, a, b, v, 0, st)
        elif kind == "bitround":
            rc = lab.mc_lab_bitround_shuffle_variant(s.data_ptr(), d.data_ptr(), n // a, a, 10, v, 0, st)
        elif kind == "lab":
            rc = lab.mc_lab_shuffle4_enc(s.data_ptr(), d.data_ptr(), n, v, st)
        elif kind == "mc_copy":
            lab.mc_lab_set_sched(b"copy_u", a)
            rc = lab.mc_copy(s.data_ptr(), d.data_ptr(), n, st)
        else:
            rc = lab.mc_lab_bw_copy(s.data_ptr(), d.data_ptr(), n, a, v, b, st)
        assert rc == 0, (c, rc)

    import ctypes

    lab.mc_lab_set_sched.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lab.mc_lab_set_sched.restype = ctypes.c_int
    lab.mc_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    copy_u0 = lab.mc_lab_get_sched(b"copy_u")
    iters = 30
    res = {c[0]: [] for c in cfgs}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for c in cfgs:
            for i in range(2):
                run(c, i % sets)
            e0.record()
            for i in range(iters):
                run(c, i % sets)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / iters * 1e-3
            res[c[0]].append((t * 1e6, 2 * n / t / 1e9))
        print(f"round {r} done", flush=True)
    lab.mc_lab_set_sched(b"copy_u", copy_u0)
    # every shuffle layout against torch's transpose (and back)
    x = ins[0]
    bad = []
    for name, (kind, es, enc, v) in cfgs:
        if kind != "shuffle":
            continue
        ref = x.view(n // es, es).t().contiguous().view(-1)
        src, want = (x, ref) if enc else (ref, x)
        outs[0].zero_()
        assert lab.mc_lab_shuffle_variant(src.data_ptr(), outs[0].data_ptr(), n, es, enc, v, 0, st) == 0
        if not torch.equal(outs[0], want):
            bad.append(name)
    print("correctness failures:", bad, flush=True)
    out = {"bad": bad, "rows": []}
    for name, v in res.items():
        us = [a for a, _ in v]
        gb = [b for _, b in v]
        row = {"cfg": name, "us_med": round(statistics.median(us), 2), "us_min": round(min(us), 2),
               "GBps_med": round(statistics.median(gb), 1), "GBps_max": round(max(gb), 1)}
        out["rows"].append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_shuffle_tiles.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
