import json, torch, sys, os
sys.path.insert(0, os.getcwd())
from numcodecs_amd import PackBits
dev = torch.device("cuda:0")
N = 256 << 20
sets = 4
bools = [torch.randint(0, 2, (N,), dtype=torch.uint8, device=dev).view(torch.bool) for _ in range(sets)]
encs = [PackBits().encode(b) for b in bools]
for i in range(sets):
    assert torch.equal(PackBits().decode(encs[i]), bools[i])
def timed(fn, reps=20):
    for i in range(sets): fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps): fn(i % sets)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3
td = timed(lambda i: PackBits().decode(encs[i]))
te = timed(lambda i: PackBits().encode(bools[i]))
print(json.dumps({"decode_us": round(td*1e6,1), "decode_GBps": round(9*N/8/td/1e9,1), "encode_us": round(te*1e6,1), "encode_GBps": round(9*N/8/te/1e9,1)}))
