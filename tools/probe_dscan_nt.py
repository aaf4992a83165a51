"""Same-width integer Delta decode of 256 MiB (i1 / i2 / i4) through the
public API into a device out, 4 rotating buffer sets, event-timed; run once
per MCODEC_DSCAN_NT setting (0-3: nontemporal loads in the reduce / apply
pass) in child processes, outputs compared with the first setting's.  One
JSON line."""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    from numcodecs_amd import Delta

    dev = torch.device("cuda:0")
    res = {}
    for dt, tdt in (("<i1", torch.int8), ("<i2", torch.int16), ("<i4", torch.int32)):
        n = (256 << 20) // torch.tensor([], dtype=tdt).element_size()
        c = Delta(dtype=dt)
        encs = [torch.randint(-100, 100, (n,), dtype=tdt, device=dev) for _ in range(4)]
        outs = [torch.empty(n, dtype=tdt, device=dev) for _ in range(4)]
        for i in range(4):
            c.decode(encs[i], out=outs[i])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(40):
            c.decode(encs[r % 4], out=outs[r % 4])
        e1.record()
        torch.cuda.synchronize()
        res[dt] = {"us": round(e0.elapsed_time(e1) / 40 * 1e3, 1),
                   "check": int(outs[0].view(torch.uint8)[:: 4097].sum().item())}
        del encs, outs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child()
        sys.exit(0)
    out = {}
    for rep in range(2):
        for m in (0, 1, 2, 3):
            env = dict(os.environ, MCODEC_DSCAN_NT=str(m), NUMCODECS_AMD_LIB=os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libmcodec_lab.so"))
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True,
                               text=True, timeout=120)
            if r.returncode:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            out[f"nt{m}_{rep}"] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(out), flush=True)
