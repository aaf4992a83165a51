import torch, sys, os
sys.path.insert(0, os.getcwd())
from numcodecs_amd import CRC32, Adler32, Fletcher32
x = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device="cuda")
for c in (CRC32(), Adler32(), Fletcher32()):
    e = c.encode(x)
    for _ in range(10):
        c.decode(e)
torch.cuda.synchronize()
