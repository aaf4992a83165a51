"""Every encode layout for the Shuffle(4) encode with BitRound(10) fused
(C3; ONLY=br10_es4), the plain Shuffle(4) encode (ONLY=shuf_es4) and the
Shuffle(8) encode (C2 f64; ONLY=shuf_es8), one workgroup per tile as the
product launches them (the pipelined layouts on their 2048 cap), 256 MiB, 4
rotating buffer sets, interleaved rounds, HIP events; every variant's
output compared with the product default's.

    python tools/probe_enc_variants.py [rounds]  -> gpurun_out/probe_enc_variants.json
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402

V_REG, V_WIDE, V_PAIR, V_NO_NT, V_BIG, V_BIG4, V_PIPE, V_BIG8 = 1, 6, 5, 8, 16, 128, 256, 512
V_PAIR_LDS = 7  # round 5: lane pairs + LDS-staged 16-B plane stores (es = 8)
LAYOUTS = {
    4: [V_REG | V_BIG8, V_REG | V_BIG4, V_REG | V_BIG, V_REG, V_REG | V_PIPE | V_BIG4, V_REG | V_PIPE | V_BIG,
        V_PAIR | V_BIG8, V_PAIR | V_BIG4, V_PAIR | V_BIG, V_PAIR, V_WIDE | V_BIG, V_WIDE | V_BIG4,
        V_REG | V_BIG8 | V_NO_NT, V_PAIR | V_BIG4 | V_NO_NT],
    8: [V_PAIR, V_PAIR_LDS, V_PAIR_LDS | V_BIG, V_PAIR_LDS | V_BIG4, V_PAIR_LDS | V_NO_NT,
        V_PAIR | V_BIG, V_PAIR | V_BIG4, V_PAIR | V_BIG8, V_REG, V_REG | V_BIG, V_REG | V_BIG4, V_REG | V_BIG8,
        V_REG | V_PIPE, V_REG | V_PIPE | V_BIG, V_WIDE, V_WIDE | V_BIG, V_WIDE | V_BIG4, V_PAIR | V_NO_NT,
        V_REG | V_NO_NT, V_REG | V_BIG4 | V_NO_NT],
}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    lab = _lab()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    n = 256 << 20
    sets = 4
    # DATA=randn: the bench's inputs (float64 / float32 normal samples), else random bytes
    if os.environ.get("DATA") == "randn":
        ins = [torch.randn(n // 8, device=dev, dtype=torch.float64).view(torch.uint8) for _ in range(sets)]
    else:
        ins = [torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(sets)]
    only = os.environ.get("ONLY")
    cfgs = ([("br10_es4", 4, True, v) for v in LAYOUTS[4]] + [("shuf_es4", 4, False, v) for v in LAYOUTS[4]] +
            [("shuf_es8", 8, False, v) for v in LAYOUTS[8]])
    if only:
        cfgs = [c for c in cfgs if c[0] == only]

    def run(c, i):
        _, es, br, v = c
        # one workgroup per tile (the product's large-buffer grid); the
        # software-pipelined persistent layouts loop on the 2048-workgroup cap
        mb = -1 if v & V_PIPE else 0
        if br:
            return lab.mc_lab_bitround_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), n // es, es, 10, v, mb, st)
        return lab.mc_lab_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), n, es, 1, v, mb, st)

    refs, bad, times = {}, [], {c: [] for c in cfgs}
    for c in cfgs:
        rc = run(c, 0)
        if rc != 0:
            bad.append((c[0], c[3], "rc", rc))
            continue
        torch.cuda.synchronize()
        key = c[0]
        if key not in refs:
            refs[key] = outs[0].clone()
        elif not torch.equal(refs[key], outs[0]):
            bad.append((c[0], c[3], "mismatch"))
    print("bad:", bad, flush=True)
    live = [c for c in cfgs if not any(b[0] == c[0] and b[1] == c[3] for b in bad)]
    for _ in range(rounds):
        for c in live:
            for i in range(sets):
                run(c, i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for r in range(reps):
                run(c, r % sets)
            e1.record()
            e1.synchronize()
            times[c].append(e0.elapsed_time(e1) * 1e3 / reps)
    rows = []
    for c in live:
        us = statistics.median(times[c])
        rows.append({"cfg": c[0], "data": os.environ.get("DATA", "bytes"), "variant": c[3], "us_med": round(us, 2), "us_min": round(min(times[c]), 2),
                     "GBps": round(2 * n / us / 1e3, 1)})
        print(json.dumps(rows[-1]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_enc_variants.json"), "w") as f:
        json.dump({"rows": rows, "bad": bad}, f, indent=1)


if __name__ == "__main__":
    main()
