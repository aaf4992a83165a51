"""One BASELINE configuration's encode OR decode, for rocprofv3 (one process
per config and direction, so every libmcodec dispatch in the trace belongs to
that operation).

    python tools/prof_configs.py CONFIG {enc|dec} [reps]

Setup (input generation, and for `dec` the encode that produces the input)
and WARM calls run first; then `reps` calls of the operation through the
public codec API, rotating over 4 buffer sets (no call finds its input in the
Infinity Cache), bracketed by two torch.cuda._sleep marker kernels
("spin_kernel"): tools/prof_summary.py attributes every dispatch between the
markers (by dispatch id) to the operation.

Configs and their algorithmic HBM bytes per call:
  C2_f32   Shuffle(4), 256 MiB f32                    2N each way
  C2_f64   Shuffle(8), 256 MiB f64                    2N
  C3       BitRound(10)+Shuffle(4) fused / unshuffle  2N
  C4       FSO(f4->i2) -> Delta(i2) -> Shuffle(2)     1.5N each way (N = f32 bytes)
  C5       8192 x 1 MiB Shuffle(4)+Fletcher32          2N + 4 per chunk
  D_i2     Delta(<i2), 256 MiB                        2N each way
  F32      Fletcher32, 256 MiB (decode: public API)   enc 2N + 4, dec N + 4
  CRC32    CRC32, 256 MiB (decode: public API)        enc 2N + 4, dec N + 4
  CRC32C / ADLER32   as CRC32
  PACKBITS PackBits, 256 MiB of bools                 enc N + N/8 + 1, dec N/8 + 1 + N
  ASTYPE   AsType(<f8 <- <f4), 256 MiB of f4          3N each way
  BLOSC_S / BLOSC_B  Blosc SHUFFLE / BITSHUFFLE filter, typesize 4,
           256 KiB blocks, 256 MiB                    2N each way
  FSO_LE / FSO_BE    FixedScaleOffset(1000, 1e3, f4 -> i2), '<f4'->'<i2' and
           '>f4'->'>i2', 256 MiB of f4                1.5N each way
  DF4_LE / DF4_BE    Delta('<f4') / Delta('>f4'), 256 MiB of smooth f4
           (speculative decode)                       2N each way
  DI2_BE   Delta('>i2'), 256 MiB                      2N each way
"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import (  # noqa: E402
    CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, PackBits, Shuffle, batch,
)
from numcodecs_amd import blosc_shuffle as bsh  # noqa: E402

MiB = 1 << 20
N = 256 * MiB
WARM = 2
SETS = 4


def config(name, dev):
    """(encode(i), decode(i), alg_bytes_enc, alg_bytes_dec) over SETS buffer sets."""
    if name in ("C2_f32", "C2_f64", "C3"):
        es = 8 if name == "C2_f64" else 4
        xs = [torch.randn(N // es, device=dev, dtype=torch.float64 if es == 8 else torch.float32)
              for _ in range(SETS)]
        sh = Shuffle(es)
        enc_op = batch.FilterPipeline([BitRound(10), sh]) if name == "C3" else None
        encs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(SETS)]
        decs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(SETS)]
        for i in range(SETS):
            if enc_op:
                encs[i] = enc_op.encode(xs[i])
            else:
                sh.encode(xs[i], out=encs[i])
        e = (lambda i: enc_op.encode(xs[i])) if enc_op else (lambda i: sh.encode(xs[i], out=encs[i]))
        return e, lambda i: sh.decode(encs[i], out=decs[i]), 2 * N, 2 * N
    if name == "C4":
        n = N // 4
        fso = FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
        pipe = batch.FilterPipeline([fso, Delta(dtype="<i2"), Shuffle(2)])
        xs = [1000.0 + 10.0 * torch.rand(n, device=dev) for _ in range(SETS)]
        encs = [pipe.encode(x) for x in xs]
        return (lambda i: pipe.encode(xs[i])), (lambda i: pipe.decode(encs[i])), 6 * n, 6 * n
    if name == "C5":
        nb = 8192
        xb = torch.randn((nb, MiB // 4), device=dev)
        eb = batch.shuffle_fletcher32_encode_chunks(xb, 4)
        db = torch.empty((nb, MiB), dtype=torch.uint8, device=dev)
        alg = nb * (2 * MiB + 4)
        return ((lambda i: batch.shuffle_fletcher32_encode_chunks(xb, 4, out=eb)),
                (lambda i: batch.fletcher32_unshuffle_decode_chunks(eb, MiB, 4, out=db, check_sums=False)), alg, alg)
    if name == "D_i2":
        d = Delta("<i2")
        xs = [torch.randint(-100, 100, (N // 2,), dtype=torch.int16, device=dev) for _ in range(SETS)]
        encs = [d.encode(x) for x in xs]
        return (lambda i: d.encode(xs[i])), (lambda i: d.decode(encs[i])), 2 * N, 2 * N
    if name in ("F32", "CRC32", "CRC32C", "ADLER32"):
        c = {"F32": Fletcher32, "CRC32": CRC32, "CRC32C": CRC32C, "ADLER32": Adler32}[name]()
        xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(SETS)]
        encs = [c.encode(x) for x in xs]
        return (lambda i: c.encode(xs[i])), (lambda i: c.decode(encs[i])), 2 * N + 4, N + 4
    if name == "PACKBITS":
        pb = PackBits()
        xs = [torch.randint(0, 2, (N,), dtype=torch.uint8, device=dev).view(torch.bool) for _ in range(SETS)]
        encs = [pb.encode(x) for x in xs]
        return (lambda i: pb.encode(xs[i])), (lambda i: pb.decode(encs[i])), N + N // 8 + 1, N // 8 + 1 + N
    if name == "ASTYPE":
        at = AsType(encode_dtype="<f8", decode_dtype="<f4")
        xs = [torch.randn(N // 4, device=dev) for _ in range(SETS)]
        encs = [at.encode(x) for x in xs]
        return (lambda i: at.encode(xs[i])), (lambda i: at.decode(encs[i])), 3 * N, 3 * N
    if name in ("BLOSC_S", "BLOSC_B"):
        mode = 1 if name == "BLOSC_S" else 2
        xs = [torch.randint(0, 256, (N,), dtype=torch.uint8, device=dev) for _ in range(SETS)]
        encs = [bsh.shuffle(x, 4, 256 * 1024, mode) for x in xs]
        return ((lambda i: bsh.shuffle(xs[i], 4, 256 * 1024, mode)),
                (lambda i: bsh.unshuffle(encs[i], 4, 256 * 1024, mode)), 2 * N, 2 * N)
    if name in ("FSO_LE", "FSO_BE"):
        bo = "<" if name == "FSO_LE" else ">"
        f = FixedScaleOffset(offset=1000, scale=1e3, dtype=bo + "f4", astype=bo + "i2")
        xs = [(1000.0 + 10.0 * torch.rand(N // 4, device=dev)) for _ in range(SETS)]
        if bo == ">":  # the same values stored big-endian (raw device bytes)
            xs = [x.view(torch.int32).view(torch.uint8).view(-1, 4).flip(1).contiguous().view(-1) for x in xs]
        encs = [f.encode(x) for x in xs]
        return (lambda i: f.encode(xs[i])), (lambda i: f.decode(encs[i])), 3 * N // 2, 3 * N // 2
    if name in ("DF4_LE", "DF4_BE", "DI2_BE"):
        if name == "DI2_BE":
            d, es = Delta(">i2"), 2
            xs = [torch.randint(-100, 100, (N // 2,), dtype=torch.int16, device=dev).view(torch.uint8)
                  for _ in range(SETS)]
        else:
            bo = "<" if name == "DF4_LE" else ">"
            d, es = Delta(bo + "f4"), 4
            xs = [(torch.arange(N // 4, device=dev, dtype=torch.float64) * 0.25 % 4096.0).float() for _ in range(SETS)]
            if bo == ">":
                xs = [x.view(torch.uint8).view(-1, 4).flip(1).contiguous().view(-1) for x in xs]
        encs = [d.encode(x) for x in xs]
        return (lambda i: d.encode(xs[i])), (lambda i: d.decode(encs[i])), 2 * N, 2 * N
    raise SystemExit(f"unknown config {name}")


def main():
    name, direction = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    dev = torch.device("cuda:0")
    enc, dec, ab_enc, ab_dec = config(name, dev)
    op = enc if direction == "enc" else dec
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(WARM):
        op(i % SETS)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)  # marker: the measured dispatches follow
    e0.record()
    for i in range(reps):
        op(i % SETS)
    e1.record()
    torch.cuda._sleep(1000)  # marker: end of the measured dispatches
    torch.cuda.synchronize()
    print(json.dumps({"config": name, "direction": direction, "reps": reps,
                      "alg_bytes_per_call": ab_enc if direction == "enc" else ab_dec,
                      "event_us_per_call": round(e0.elapsed_time(e1) / reps * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
