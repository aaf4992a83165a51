"""Shuffle(4) encode/decode variant sweep at several chunk sizes, interleaved
rounds in one process (guide §5.4 rule 24), against the nt copy calibration."""

import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "numcodecs_amd", "_lib", "libmcodec.so"))
bw = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libbwtest.so"))
V, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
sys.path.insert(0, os.path.join(ROOT, "tools"))
from lab.lablib import lab as _lab  # noqa: E402  (the sweep entry points live in the lab library)

lab = _lab()
bw.bw_copy.argtypes = [V, V, S, I, I, V]


def main():
    es = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    MiB = 1 << 20
    sizes = [256 * MiB]
    sets = 4
    cap = max(sizes)
    ins = [torch.randint(0, 256, (cap,), dtype=torch.uint8, device=dev) for _ in range(sets)]
    outs = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(sets)]
    iters, rounds = 30, 5
    cfgs = []
    for n in sizes:
        cfgs.append(("copy-nt", n, None, None, 8192))
        for enc in (1, 0):
            variants = [int(v) for v in os.environ.get("PROBE_VARIANTS", "1,17,129,2,3").split(",")]
            grids = [int(g) for g in os.environ.get("PROBE_GRIDS", "0,1024,4096,8192,16384,32768").split(",")]
            for var, grid in [(v, g) for v in variants for g in grids]:
                cfgs.append(("shuffle", n, enc, var, grid))
    res = {c: [] for c in cfgs}

    def run(c, i):
        kind, n, enc, var, grid = c
        if kind == "copy-nt":
            assert bw.bw_copy(ins[i].data_ptr(), outs[i].data_ptr(), n, 2, grid, st) == 0
        else:
            assert lab.mc_lab_shuffle_variant(ins[i].data_ptr(), outs[i].data_ptr(), n, es, enc, var, grid, st) == 0

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
            res[c].append(2 * c[1] / t / 1e9)
    # correctness of every config against torch's transpose
    bad = []
    x = ins[0]
    for c in cfgs:
        kind, n, enc, var, grid = c
        if kind != "shuffle":
            continue
        y = torch.empty(n, dtype=torch.uint8, device=dev)
        src = x[:n] if enc else x[:n].view(n // es, es).t().contiguous().view(-1)
        assert lab.mc_lab_shuffle_variant(src.data_ptr(), y.data_ptr(), n, es, enc, var, grid, st) == 0
        ref = x[:n].view(n // es, es).t().contiguous().view(-1) if enc else x[:n]
        if not torch.equal(y, ref):
            bad.append(c)
    print("correctness failures:", bad, flush=True)
    out = []
    for c, v in res.items():
        d = {"kind": c[0], "MiB": round(c[1] / MiB, 3), "enc": c[2], "var": c[3], "grid": c[4],
             "GBps_med": round(statistics.median(v), 1), "GBps_max": round(max(v), 1)}
        out.append(d)
        print(json.dumps(d), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", f"probe_enc_es{es}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
