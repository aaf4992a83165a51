"""Float Delta decode on noise-like data: the speculative path with the
walker (fspec=1, the product default) against the serial chain alone
(fspec=0), each in a child process on the lab library, two interleaved
rounds.  One f4 chunk of MiB (default 64) per family, HIP-event timed,
median of 3; outputs checked against numpy's cumsum.

    python tools/probe_walk_vs_chain.py [MiB]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAB = os.path.join(ROOT, "tools", "_build", "libmcodec_lab.so")
FAMS = ("randn", "chirp", "smallamp", "sparse", "sin_noise", "randwalk")


def child(mib):
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from numcodecs_amd import Delta
    from tests.test_gpu_delta_walk import family

    dev = torch.device("cuda", 0)
    n = mib * (1 << 20) // 4
    codec = Delta("<f4")
    res = {}
    for kind in FAMS:
        x = family(kind, n).astype("<f4")
        enc = np.empty_like(x)
        enc[0] = x[0]
        np.subtract(x[1:], x[:-1], out=enc[1:])
        ref = np.cumsum(enc, dtype="<f4")
        e = torch.from_numpy(enc).to(dev)
        d = torch.empty_like(e)
        codec.decode(e, out=d)
        ok = d.cpu().numpy().tobytes() == ref.tobytes()
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            codec.decode(e, out=d)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        res[kind] = {"ms": round(float(np.median(ts)), 2), "ok": ok}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "child":
        child(int(sys.argv[2]))
        sys.exit(0)
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    for rnd in range(2):
        out = {"MiB": mib}
        for fspec in (1, 0):
            env = dict(os.environ, MCODEC_FSPEC=str(fspec), NUMCODECS_AMD_LIB=LAB)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child", str(mib)], env=env,
                               capture_output=True, text=True, timeout=400)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            out["walker" if fspec else "chain"] = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps(out), flush=True)
