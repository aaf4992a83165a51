"""Debug: c16 'special' Delta decode mismatch against the goldens."""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from numcodecs_amd import Delta
G = "tests/golden"
man = json.load(open(f"{G}/ext.json"))
D = np.load(f"{G}/ext.npz")
for i, m in enumerate(man["ext_delta"]):
    if m["kind"] != "special" or "c16" not in m["dtype"]:
        continue
    enc = D[f"ext_delta__{i}__encoded"].view(m["astype"])
    want = D[f"ext_delta__{i}__decoded"].view(m["dtype"])
    got = Delta(m["dtype"], m["astype"]).decode(enc)
    gb = got.view(np.uint64).reshape(-1, 2); wb = want.view(np.uint64).reshape(-1, 2)
    bad = np.nonzero((gb != wb).any(1))[0]
    print(m, "bad", len(bad), bad[:8])
    for j in bad[:4]:
        print(j, [hex(v) for v in gb[j]], [hex(v) for v in wb[j]], "enc", enc[max(j-1,0):j+1])
    # real-part plane alone through the real f8 decode
    er = np.ascontiguousarray(enc.real.astype("<f8"))
    wr = np.cumsum(er)
    gr = Delta("<f8").decode(er)
    print("real plane f8 decode bad:", np.nonzero(gr.view(np.uint64) != wr.view(np.uint64))[0][:8])
    ei = np.ascontiguousarray(enc.imag.astype("<f8"))
    gi = Delta("<f8").decode(ei)
    print("imag plane f8 decode bad:", np.nonzero(gi.view(np.uint64) != np.cumsum(ei).view(np.uint64))[0][:8])
