"""CRC32 / Adler32 encode of one 256 MiB device chunk through the public API
(payload copy + checksum, two launches at this size) under the checksum
kernels' knobs MCODEC_CK_KCOPY (tiles of K x 4 KiB) and MCODEC_CK_GRID_COPY
(persistent grid), each setting in a child process; 4 rotating buffers,
event-timed.  One JSON line of us per call."""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    from numcodecs_amd import CRC32, Adler32

    dev = torch.device("cuda:0")
    N = 256 << 20
    xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]
    res = {}
    for name, c in (("crc32", CRC32()), ("adler32", Adler32())):
        for i in range(4):
            c.encode(xs[i])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(20):
            c.encode(xs[r % 4])
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child()
        sys.exit(0)
    out = {}
    for rnd in range(2):
        for k in (4, 8, 16):
            for g in (512, 1024, 2048, 4096):
                env = dict(os.environ, MCODEC_CK_KCOPY=str(k), MCODEC_CK_GRID_COPY=str(g), NUMCODECS_AMD_LIB=os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libmcodec_lab.so"))
                r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env,
                                   capture_output=True, text=True, timeout=120)
                if r.returncode:
                    print(r.stderr[-2000:], file=sys.stderr)
                    sys.exit(r.returncode)
                out.setdefault(f"K{k}_G{g}", []).append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(json.dumps(out), flush=True)
