import os, sys, warnings
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np, torch
import oracle
from test_gpu_delta_spec2 import _decode_raw, _dec
rng = np.random.default_rng(7)
n = 50001
for dt, at in [("<f2", "<f4"), ("<f2", "<f8"), ("<f4", "<f8"), ("<f2", "<f2"), ("<f8","<f4")]:
    enc = (rng.standard_normal(n) * 3.7).astype(at)
    got, first = _decode_raw(enc, dt, at)
    ref = _dec(enc, dt, at)
    bad = np.nonzero(got.view(np.uint8 if got.itemsize == 1 else f"u{got.itemsize}") != ref.view(f"u{ref.itemsize}"))[0]
    print(dt, at, "first_fail_word", first, "nbad", bad.size, "first_bad", bad[:5].tolist(),
          "got", got[bad[:3]].tolist() if bad.size else None, "ref", ref[bad[:3]].tolist() if bad.size else None,
          "enc", enc[bad[:3]].tolist() if bad.size else None, "prev_ref", ref[bad[:3]-1].tolist() if bad.size else None, flush=True)
