"""Host-streamed Zarr chain (BitRound(10) -> Shuffle(4) -> CRC32) throughput
on 512 x 4 MiB pinned chunks, and what the checksum adds: host->host encode
/ decode through chunks.host_*_chunks, the device-only decode of 64 chunks,
and plain H2D copies of 4 MiB+4-B rows (64-B aligned slices) vs 4 MiB rows."""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from numcodecs_amd import CRC32, BitRound, Fletcher32, Shuffle, chunks  # noqa: E402

MiB = 1 << 20
n, cb = 512, 4 * MiB


def h2d_rate(host, rows_per_slice=16):
    dev = torch.empty((rows_per_slice, host.shape[1]), dtype=host.dtype, device="cuda")
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for lo in range(0, host.shape[0], rows_per_slice):
            dev.copy_(host[lo:lo + rows_per_slice], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    return host.numel() * host.element_size() / dt / 2**30


x = torch.randn((n, cb // 4)).pin_memory()
for name, codecs in (("crc32_start", [BitRound(10), Shuffle(4), CRC32()]),
                     ("crc32_end", [BitRound(10), Shuffle(4), CRC32(location="end")]),
                     ("fletcher32", [BitRound(10), Shuffle(4), Fletcher32()]),
                     ("no_crc", [BitRound(10), Shuffle(4)])):
    enc = chunks.host_encode_chunks(codecs, x)
    out = torch.empty_like(x).pin_memory()
    chunks.host_decode_chunks(codecs, enc, out)
    tds = []
    for sl in (None, None, None):
        t0 = time.perf_counter()
        chunks.host_decode_chunks(codecs, enc, out, slice_chunks=sl)
        tds.append(time.perf_counter() - t0)
    print(name, "decode GiB/s runs", [round(n * cb / t / 2**30, 1) for t in tds])
    td = min(tds)
    t0 = time.perf_counter()
    chunks.host_encode_chunks(codecs, x, enc)
    te = time.perf_counter() - t0
    dev = enc[:64].cuda()
    chunks.decode_chunks(codecs, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        chunks.decode_chunks(codecs, dev)
    torch.cuda.synchronize()
    tdd = (time.perf_counter() - t0) / 10
    print(name, "enc GiB/s", round(n * cb / te / 2**30, 1), "dec GiB/s", round(n * cb / td / 2**30, 1),
          "device decode 64x4MiB us", round(tdd * 1e6, 1), "H2D of encoded rows GiB/s", round(h2d_rate(enc), 1),
          flush=True)
print("H2D of 4 MiB rows GiB/s", round(h2d_rate(x.view(torch.uint8).reshape(n, cb)), 1))
