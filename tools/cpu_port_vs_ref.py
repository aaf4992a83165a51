"""Time the build's C restatement (oracle/ncoracle.c, bench.py's cpu_baseline)
against the reference's own compiled loops and numpy expressions, in THIS
container only (the reference never travels to the GPU box).

    python tools/cpu_port_vs_ref.py > profiles/r02/cpu_port_vs_ref.json

For each hot loop: best-of-5 wall time on 64 MiB of input, one core.
  shuffle/unshuffle   reference _shuffle.pyx (Cython -O3, oracle/_ref) vs nco_shuffle
  fletcher32          reference fletcher32.pyx encode vs nco_fletcher32 (+ memcpy)
  bitround(10) f4     reference bitround.py (numpy) vs nco_bitround32
  fso f4->i2 enc/dec  reference fixedscaleoffset.py (numpy) vs nco_fso_*
  delta i2 enc/dec    reference delta.py (numpy) vs nco_delta_*_i2
"""

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import nporacle as npo  # noqa: E402
from oracle import refload  # noqa: E402

MiB = 1 << 20


def best(fn, reps=5):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    nc = refload.load()
    import importlib

    sh = importlib.import_module("numcodecs._shuffle")
    nbytes = 64 * MiB
    rng = np.random.default_rng(0)
    x = rng.standard_normal(nbytes // 4, dtype=np.float32)
    u8 = x.view(np.uint8)
    out = np.empty_like(u8)
    res = {}

    def row(name, t_ref, t_port, nb):
        res[name] = {"reference_GiBps": round(nb / t_ref / (1 << 30), 3),
                     "port_GiBps": round(nb / t_port / (1 << 30), 3),
                     "port_over_reference": round(t_ref / t_port, 3)}

    for es in (4, 8):
        row(f"shuffle{es}_encode", best(lambda: sh._doShuffle(u8, out, es)),
            best(lambda: npo.shuffle_into(u8, out, es)), nbytes)
        row(f"shuffle{es}_decode", best(lambda: sh._doUnshuffle(u8, out, es)),
            best(lambda: npo.unshuffle_into(u8, out, es)), nbytes)
    f = nc.Fletcher32()
    row("fletcher32_encode", best(lambda: f.encode(u8)),
        best(lambda: (np.copyto(out, u8), npo.c_fletcher32(u8))), nbytes)
    b = np.empty(x.size, dtype="<u4")
    row("bitround10_f4_encode", best(lambda: nc.BitRound(10).encode(x)),
        best(lambda: npo.c_bitround32_into(x, b, 10)), nbytes)
    xc = (1000 + 10 * np.sin(np.arange(x.size) / 651.9)).astype(np.float32)
    fso = nc.FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2")
    e2 = np.empty(x.size, dtype="<i2")
    d4 = np.empty(x.size, dtype="<f4")
    enc = fso.encode(xc)
    row("fso_f4_i2_encode", best(lambda: fso.encode(xc)),
        best(lambda: npo.c_fso_encode_f4_i2_into(xc, e2, 1000, 1e3)), nbytes)
    row("fso_f4_i2_decode", best(lambda: fso.decode(enc)),
        best(lambda: npo.c_fso_decode_i2_f4_into(enc, d4, 1000, 1e3)), nbytes)
    dl = nc.Delta(dtype="<i2")
    denc = dl.encode(enc)
    row("delta_i2_encode", best(lambda: dl.encode(enc)),
        best(lambda: npo.c_delta_encode_i2_into(enc, e2)), enc.nbytes)
    row("delta_i2_decode", best(lambda: dl.decode(denc)),
        best(lambda: npo.c_delta_decode_i2_into(denc, e2)), enc.nbytes)
    res["_note"] = ("one core of this container (8 vCPU Xeon); 64 MiB of input per call, best of 5; "
                    "reference = its Cython compiled by oracle/build_ref.sh (-O3, no -march) or its numpy "
                    "expressions (numpy 2.2.6); port = oracle/ncoracle.c -O3 -ffp-contract=off, no -march")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
