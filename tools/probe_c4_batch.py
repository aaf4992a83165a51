"""Batched FSO(f4->i2) -> Delta(i2) -> Shuffle(2) over B chunks (Zarr chunk
pipeline): the fused batch kernels (chunks.encode_chunks / decode_chunks)
against the same chain codec by codec (chunks._encode_step per codec),
2048 x 1 MiB and 256 x 4 MiB of f32; event-timed, rotating 2 buffer sets.
GB/s over the algorithmic 1.5 N per direction.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, chunks  # noqa: E402

dev = torch.device("cuda:0")
codecs = [FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"), Delta(dtype="<i2"), Shuffle(2)]


def timed(fn, sets=2, reps=10):
    for i in range(sets):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % sets)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def seq_encode(x):
    for c in codecs:
        x = chunks._encode_step(c, x)
    return x


def seq_decode(x):
    for c in codecs[::-1]:
        x = chunks._decode_step(c, x)
    return x


out = {}
for b, mib in ((2048, 1), (256, 4), (16, 64), (1, 256)):
    n = mib * (1 << 20) // 4
    xs = [1000.0 + 10.0 * torch.rand((b, n), device=dev) for _ in range(2)]
    encs = [chunks.encode_chunks(codecs, x) for x in xs]
    assert torch.equal(seq_encode(xs[0]).view(torch.uint8), encs[0].view(torch.uint8))
    assert torch.equal(seq_decode(encs[0]).contiguous().view(torch.uint8),
                       chunks.decode_chunks(codecs, encs[0]).contiguous().view(torch.uint8))
    alg = 1.5 * b * n * 4
    r = {}
    for name, fn in (("fused_enc", lambda i: chunks.encode_chunks(codecs, xs[i])),
                     ("fused_dec", lambda i: chunks.decode_chunks(codecs, encs[i])),
                     ("seq_enc", lambda i: seq_encode(xs[i])),
                     ("seq_dec", lambda i: seq_decode(encs[i]))):
        t = timed(fn)
        r[name + "_us"] = round(t * 1e6, 1)
        r[name + "_GBps"] = round(alg / t / 1e9, 1)
    out[f"{b}x{mib}MiB"] = r
    del xs, encs
print(json.dumps(out), flush=True)
