"""A/B of the CRC32 / CRC32C tile fold: bit-sliced XOR network (crc_lds=0,
the product default) against the LDS slicing-by-16 tables (crc_lds=1), each
setting in a child process on the lab library, two interleaved rounds.

Per setting, event-timed through the public API on 4 rotating 256 MiB device
buffers (no call finds its input in the Infinity Cache):
  verify  -- CRC32(C).decode of one 256 MiB chunk (one-launch verify, K = 16)
  encode  -- CRC32(C).encode of one 256 MiB chunk (checksum + payload copy, K = 8)
  batch   -- batch.checksum32_decode_chunks over 256 x 1 MiB rows
One JSON line per round: {setting: {name: us per call}}."""
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LAB = os.path.join(ROOT, "tools", "_build", "libmcodec_lab.so")


def timed(fn, reps=20):
    for i in range(4):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for r in range(reps):
        fn(r % 4)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps * 1e3, 1)


def child():
    sys.path.insert(0, ROOT)
    from numcodecs_amd import CRC32, CRC32C, batch

    dev = torch.device("cuda:0")
    N = 256 << 20
    xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(4)]
    res = {}
    for name, c, cid in (("crc32", CRC32(), "crc32"), ("crc32c", CRC32C(), "crc32c")):
        encs = [c.encode(x) for x in xs]
        res[f"{name}_verify"] = timed(lambda i: c.decode(encs[i]))
        res[f"{name}_encode"] = timed(lambda i: c.encode(xs[i]))
        rows = [x.view(256, 1 << 20) for x in xs]
        erows = [batch.checksum32_encode_chunks(r, cid) for r in rows]
        res[f"{name}_batch256x1M"] = timed(lambda i: batch.checksum32_decode_chunks(erows[i], cid))
        del encs, erows
    print(json.dumps(res), flush=True)


SETTINGS = {
    "bitsliced": {},
    "lds_tables": {"MCODEC_CRC_LDS": "1"},
    "bs_grid256": {"MCODEC_CK_GRID": "256", "MCODEC_CK_GRID_COPY": "256"},
    "bs_grid512": {"MCODEC_CK_GRID": "512", "MCODEC_CK_GRID_COPY": "512"},
    "bs_grid768": {"MCODEC_CK_GRID": "768", "MCODEC_CK_GRID_COPY": "768"},
    "bs_grid1024": {"MCODEC_CK_GRID": "1024", "MCODEC_CK_GRID_COPY": "1024"},
    "bs_grid2048": {"MCODEC_CK_GRID": "2048", "MCODEC_CK_GRID_COPY": "2048"},
    "bs_k8": {"MCODEC_CK_K": "8"},
    "bs_k8_grid768": {"MCODEC_CK_K": "8", "MCODEC_CK_GRID": "768"},
    "bs_k8_grid1024": {"MCODEC_CK_K": "8", "MCODEC_CK_GRID": "1024"},
    "bs_k8_grid2048": {"MCODEC_CK_K": "8", "MCODEC_CK_GRID": "2048"},
    "bs_grid4096": {"MCODEC_CK_GRID": "4096", "MCODEC_CK_GRID_COPY": "4096"},
    "bs_kcopy16_grid512": {"MCODEC_CK_KCOPY": "16", "MCODEC_CK_GRID_COPY": "512"},
    "bs_gridcopy512": {"MCODEC_CK_GRID_COPY": "512"},
    "bs_gridcopy768": {"MCODEC_CK_GRID_COPY": "768"},
    "bs_kcopy16": {"MCODEC_CK_KCOPY": "16"},
}

if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
        sys.exit(0)
    names = sys.argv[1:] or ["bitsliced", "lds_tables"]
    for rnd in range(2):
        out = {}
        for name in names:
            env = dict(os.environ, NUMCODECS_AMD_LIB=LAB, **SETTINGS[name])
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env,
                               capture_output=True, text=True, timeout=240)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            out[name] = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps(out), flush=True)
