"""CRC32 (or CRC32C) decode of one 256 MiB device chunk, 20 calls over 4
rotating buffers, for rocprofv3 kernel traces and PMC passes of the one-launch
verify kernel.  Usage: python tools/probe_crc_verify.py [crc32|crc32c] [encode]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import CRC32, CRC32C  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "crc32"
enc_mode = len(sys.argv) > 2 and sys.argv[2] == "encode"
c = CRC32() if kind == "crc32" else CRC32C()
xs = [torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device="cuda") for _ in range(4)]
encs = [c.encode(x) for x in xs]
torch.cuda.synchronize()
for r in range(20):
    if enc_mode:
        c.encode(xs[r % 4])
    else:
        c.decode(encs[r % 4])
torch.cuda.synchronize()
print("ok", kind, "encode" if enc_mode else "verify")
