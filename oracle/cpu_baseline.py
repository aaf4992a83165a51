"""CPU baseline workloads -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

The build's own scalar C restatement of the reference's hot path
(oracle/ncoracle.c, -O3, no -march, like the reference's release build,
src/numcodecs/meson.build:245-254), timed on the host cores of the GPU box for
every BASELINE.json configuration.  Nothing of the reference travels to the
GPU box: the loops are restated, and pinned bit-exact against the reference's
goldens in this container (tests/test_oracle.py).

Each workload mirrors the reference's per-codec call structure (one output
buffer per codec, as numcodecs allocates one per encode/decode):

  C1 / C2  Shuffle(es).encode + decode ........ _shuffle.pyx:11-30
  C3       BitRound(10) then Shuffle(4); decode = unshuffle (BitRound.decode
           is a re-view) ......................... bitround.py:62-68
  C4       FixedScaleOffset(1000, 1e3, f4->i2) -> Delta(i2) -> Shuffle(2) and
           back ................................... fixedscaleoffset.py:91-110,
                                                    delta.py:63-80
  C5       per 1 MiB chunk: Shuffle(4) then Fletcher32.encode (payload copy +
           checksum footer); decode = checksum verify + unshuffle
                                                    fletcher32.pyx:24-115

value = bytes into encode + bytes into decode (uncompressed chunk bytes) /
wall time, i.e. the GPU metric's definition.
"""

from __future__ import annotations

import os
import time

import numpy as np

from . import nporacle as npo

MiB = 1 << 20
GiB = 1 << 30


def _touch(a: np.ndarray) -> np.ndarray:
    a.view(np.uint8).fill(0)  # fault the pages in before timing
    return a


def _c4_input(n: int, seed: int) -> np.ndarray:
    """SURVEY §8d's C4 data: 1000 + 10 sin(2 pi i / 4096) + U(-0.5, 0.5),
    built from a 64 Ki-element period (the codec's cost is data-independent)."""
    rng = np.random.default_rng(seed)
    per = 1 << 16
    i = np.arange(per)
    base = (1000.0 + 10.0 * np.sin(2 * np.pi * i / 4096) + rng.uniform(-0.5, 0.5, per)).astype(np.float32)
    return np.resize(base, n)


class Workload:
    """One configuration on `nbytes` of input: step() = encode + decode once."""

    def __init__(self, config: str, nbytes: int, seed: int = 0):
        self.config = config
        self.nbytes = nbytes
        rng = np.random.default_rng(seed)
        u8 = lambda k: _touch(np.empty(k, dtype=np.uint8))  # noqa: E731
        if config in ("C1", "C2_f32", "C3"):
            self.x = rng.standard_normal(nbytes // 4, dtype=np.float32)
        elif config == "C2_f64":
            self.x = rng.standard_normal(nbytes // 8)
        elif config == "C4":
            self.x = _c4_input(nbytes // 4, seed)
        elif config == "C5":
            self.x = rng.standard_normal(nbytes // 4, dtype=np.float32).reshape(-1, MiB // 4)
        else:
            raise ValueError(config)
        if config == "C4":
            n = nbytes // 4
            self.t_fso = _touch(np.empty(n, dtype="<i2"))
            self.t_delta = _touch(np.empty(n, dtype="<i2"))
            self.enc = u8(2 * n)
            self.d_unsh = u8(2 * n)
            self.d_delta = _touch(np.empty(n, dtype="<i2"))
            self.dec = _touch(np.empty(n, dtype="<f4"))
        elif config == "C5":
            self.tmp = u8(MiB)
            self.enc = u8(MiB + 4)
            self.dec = _touch(np.empty_like(self.x))
        else:
            self.tmp = u8(nbytes)
            self.enc = u8(nbytes)
            self.dec = _touch(np.empty_like(self.x))

    @property
    def bytes_per_step(self) -> int:
        return 2 * self.nbytes

    def step(self) -> None:
        c = self.config
        if c in ("C1", "C2_f32"):
            npo.shuffle_into(self.x, self.enc, 4)
            npo.unshuffle_into(self.enc, self.dec, 4)
        elif c == "C2_f64":
            npo.shuffle_into(self.x, self.enc, 8)
            npo.unshuffle_into(self.enc, self.dec, 8)
        elif c == "C3":
            npo.c_bitround32_into(self.x, self.tmp, 10)
            npo.shuffle_into(self.tmp, self.enc, 4)
            npo.unshuffle_into(self.enc, self.dec, 4)
        elif c == "C4":
            npo.c_fso_encode_f4_i2_into(self.x, self.t_fso, 1000, 1e3)
            npo.c_delta_encode_i2_into(self.t_fso, self.t_delta)
            npo.shuffle_into(self.t_delta, self.enc, 2)
            npo.unshuffle_into(self.enc, self.d_unsh, 2)
            npo.c_delta_decode_i2_into(self.d_unsh, self.d_delta)
            npo.c_fso_decode_i2_f4_into(self.d_delta, self.dec, 1000, 1e3)
        else:  # C5: chunk by chunk
            enc, tmp = self.enc, self.tmp
            for r in range(self.x.shape[0]):
                row = self.x[r]
                npo.shuffle_into(row, tmp, 4)  # Shuffle(4).encode
                enc[:MiB] = tmp  # Fletcher32.encode: memcpy + footer
                enc[MiB:] = np.frombuffer(npo.c_fletcher32(tmp).to_bytes(4, "little"), np.uint8)
                payload = enc[:MiB]  # Fletcher32.decode: verify, view
                if npo.c_fletcher32(payload) != int.from_bytes(enc[MiB:].tobytes(), "little"):
                    raise RuntimeError("fletcher32 mismatch in the CPU baseline")
                npo.unshuffle_into(payload, self.dec[r], 4)  # Shuffle(4).decode

    def verify(self) -> None:
        """The decoded chunk equals the input (C3/C4 are lossy: compare with
        the oracle's numpy restatement of the lossy step instead)."""
        if self.config == "C3":
            exp = npo.bitround_encode(self.x, 10).view(np.float32)
        elif self.config == "C4":
            exp = npo.fso_decode(npo.fso_encode(self.x, 1000, 1e3, "<f4", "<i2"), 1000, 1e3, "<f4", "<i2")
        else:
            exp = self.x
        if not np.array_equal(self.dec.view(exp.dtype).reshape(exp.shape), exp):
            raise AssertionError(f"CPU baseline {self.config} round trip differs from the oracle")


def time_workload(w: Workload, seconds: float, deadline: float | None = None):
    """Run steps until `seconds` elapsed (or the wall-clock deadline); returns
    (bytes, elapsed seconds, steps).  At least one step is timed."""
    t0 = time.perf_counter()
    steps = 0
    while True:
        w.step()
        steps += 1
        el = time.perf_counter() - t0
        if deadline is not None:
            if time.time() >= deadline:
                break
        elif el >= seconds:
            break
    return w.bytes_per_step * steps, el, steps


def single_core(config: str, nbytes: int, seconds: float) -> dict:
    """One process, one core: warm-up step (checked against the oracle), then
    timed steps for about `seconds`."""
    w = Workload(config, nbytes, seed=1)
    w.step()
    w.verify()
    b, el, steps = time_workload(w, seconds)
    return {"value": round(b / GiB / el, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{steps} x encode+decode of {nbytes // MiB} MiB ({el:.1f} s), oracle/ncoracle.c -O3"}


def _par_worker(config, nbytes, seed, seconds, barrier, q):
    w = Workload(config, nbytes, seed)
    w.step()
    barrier.wait()  # every process has set up: the timed legs overlap
    b, el, _ = time_workload(w, seconds)
    q.put((b, el))


def parallel(config: str, procs: int, nbytes: int, seconds: float) -> dict:
    """`procs` processes at once, each streaming its own `nbytes` chunk set
    (numcodecs holds the GIL in its loops, so a Zarr reader scales over
    processes, not threads); aggregate = all bytes / the slowest process.
    Forked: call before anything touches the GPU."""
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    barrier = ctx.Barrier(procs)
    q = ctx.Queue()
    ps = [ctx.Process(target=_par_worker, args=(config, nbytes, 100 + i, seconds, barrier, q))
          for i in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=600) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        if p.exitcode != 0:
            raise RuntimeError(f"CPU baseline worker failed ({p.exitcode})")
    total = sum(b for b, _ in res)
    el = max(t for _, t in res)
    return {"value": round(total / GiB / el, 3), "unit": "GiB/s", "cores": procs, "kind": "port",
            "sample": f"{procs} processes x encode+decode of their own {nbytes // MiB} MiB for {el:.1f} s"}
