"""Throughput of the longdouble paths (csrc/mc_x80.h) through the public
codecs: Delta('<f16') decode (one x87 add chain, k_ld_chain) and encode, and
FixedScaleOffset / Quantize / AsType on '<f16', for 32 MiB (2 Mi elements)
of noisy data; outputs checked against numpy.  One JSON line (us per call,
ns per element)."""
import json
import os
import sys
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import AsType, Delta, FixedScaleOffset, Quantize  # noqa: E402
from oracle import nporacle  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    n = 2 << 20
    rng = np.random.default_rng(1)
    x = rng.standard_normal(n).astype(np.longdouble) / np.longdouble(7)
    xd = torch.from_numpy(x.view(np.uint8).copy()).to(dev)
    out = {"n": n}
    d = Delta("<f16")
    enc = d.encode(xd)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        want = nporacle.delta_decode(nporacle.delta_encode(x, "<f16"), "<f16")
    assert np.array_equal(d.decode(enc).cpu().numpy().reshape(-1, 16)[:, :10], want.view(np.uint8).reshape(-1, 16)[:, :10])
    out["delta_dec_us"] = round(timed(lambda: d.decode(enc)), 1)
    out["delta_enc_us"] = round(timed(lambda: d.encode(xd)), 1)
    fso = FixedScaleOffset(0.5, 1e3, "<f16", "<i4")
    out["fso_enc_us"] = round(timed(lambda: fso.encode(xd)), 1)
    q = Quantize(3, "<f16")
    out["quantize_enc_us"] = round(timed(lambda: q.encode(xd)), 1)
    a = AsType("<f8", "<f16")
    out["astype_enc_us"] = round(timed(lambda: a.encode(xd)), 1)
    out["delta_dec_ns_per_elem"] = round(out["delta_dec_us"] * 1e3 / n, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
