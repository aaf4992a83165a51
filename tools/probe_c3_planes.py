"""A/B of the C3 encode (BitRound(10) + Shuffle(4), one 256 MiB f32 chunk):
the plane-masked kernel (k_bitround_shuffle4_planes, mc_sched.br_planes = 1,
the product default) against the element-masked k_shuffle_enc<4, true>
(br_planes = 0), and the plain Shuffle(4) encode beside them -- one process
on the lab library (mc_lab_set_sched between rounds), 4 rotating buffer sets,
HIP events around 20 calls, 7 interleaved rounds; outputs checked equal.
    NUMCODECS_AMD_LIB=tools/_build/libmcodec_lab.so python tools/probe_c3_planes.py"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from numcodecs_amd import _native, _ops  # noqa: E402


def main():
    lib = _native.lib
    set_sched = lib.mc_lab_set_sched
    set_sched.argtypes = [ctypes.c_char_p, ctypes.c_int]
    set_sched.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    n = (256 << 20) // 4
    sets = 4
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randn(n, generator=g, device=dev) for _ in range(sets)]
    ys = [torch.empty(n * 4, dtype=torch.uint8, device=dev) for _ in range(sets)]
    st = _ops.stream(xs[0])

    def br(i):
        assert lib.mc_bitround_shuffle(xs[i].data_ptr(), ys[i].data_ptr(), n, 4, 10, st) == 0

    def sh(i):
        assert lib.mc_shuffle(xs[i].data_ptr(), ys[i].data_ptr(), n * 4, 4, st) == 0

    outs = {}
    for v in (0, 1):
        assert set_sched(b"br_planes", v) != -2**31
        br(0)
        torch.cuda.synchronize()
        outs[v] = ys[0].clone()
    assert torch.equal(outs[0], outs[1]), "plane-masked and element-masked encodes differ"

    def timed(fn):
        for i in range(sets):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for k in range(20):
            fn(k % sets)
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / 20, 2)

    res = {"planes_us": [], "elements_us": [], "shuffle4_us": []}
    for _ in range(7):
        set_sched(b"br_planes", 1)
        res["planes_us"].append(timed(br))
        set_sched(b"br_planes", 0)
        res["elements_us"].append(timed(br))
        res["shuffle4_us"].append(timed(sh))
    set_sched(b"br_planes", 1)
    # the encode layouts (mc_shuffle.hip variants) with the plane mask where
    # the layout has it (register layouts, 128 / 64 KiB tiles)
    lab_var = lib.mc_lab_bitround_shuffle_variant
    lab_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                        ctypes.c_int, ctypes.c_void_p]
    lab_var.restype = ctypes.c_int
    variants = {"reg_128k": 513, "reg_64k": 129, "reg_32k": 17, "reg_64k_g2": 129 | 32, "pipe_64k": 385,
                "pair_128k": 517}
    for name, v in variants.items():
        def fn(i, v=v):
            assert lab_var(xs[i].data_ptr(), ys[i].data_ptr(), n, 4, 10, v, 0, st) == 0
        fn(0)
        torch.cuda.synchronize()
        assert torch.equal(ys[0], outs[1]), name
        res[f"var_{name}_us"] = sorted(timed(fn) for _ in range(5))[2]
    for k in ("planes_us", "elements_us", "shuffle4_us"):
        res[k.replace("_us", "_med")] = sorted(res[k])[3]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
