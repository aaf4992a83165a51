"""One-launch CRC32 / CRC32C / Adler32 verify of one 256 MiB device chunk
through the public API (decode), under the lab library's checksum grid knob
MCODEC_CK_GRID (persistent workgroups of the checksum-only pass; product
default 2048), each setting in a child process; 4 rotating buffers,
event-timed, µs per decode.  One JSON line per round."""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    from numcodecs_amd import CRC32, CRC32C, Adler32

    dev = torch.device("cuda:0")
    N = 256 << 20
    res = {}
    for name, c in (("crc32", CRC32()), ("crc32c", CRC32C()), ("adler32", Adler32())):
        encs = [c.encode(torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev)) for _ in range(4)]
        for i in range(4):
            c.decode(encs[i])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for r in range(20):
            c.decode(encs[r % 4])
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / 20 * 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child()
        sys.exit(0)
    lab = os.path.join(ROOT, "tools", "_build", "libmcodec_lab.so")
    for rnd in range(2):
        out = {}
        for g in (256, 512, 768, 1024, 1536, 2048, 4096):
            env = dict(os.environ, MCODEC_CK_GRID=str(g), NUMCODECS_AMD_LIB=lab)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env,
                               capture_output=True, text=True, timeout=120)
            if r.returncode:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            out[f"G{g}"] = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps({"probe": "ck_verify_grid", "round": rnd, "us": out}), flush=True)
