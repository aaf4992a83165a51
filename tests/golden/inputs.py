"""Portable synthetic inputs for the parity tests and the goldens.

Values are built from raw PCG64 words (``bit_generator.random_raw``, a stream
numpy keeps stable across versions) with integer and exactly-rounded float
operations only -- no transcendental functions, whose last bits depend on the
host CPU's SIMD dispatch -- so this container and the GPU box produce
byte-identical inputs.

Configs (BASELINE.json):
  C1  1 MiB f32, seed 1                      Shuffle(4)
  C2  256 MiB f32 seed 2 (Shuffle(4)); 256 MiB f64 seed 3 (Shuffle(8))
  C3  = C2 f32 input                         BitRound(10) -> Shuffle(4)
  C4  256 MiB f32 ~ 1000 +- 10.5, seed 4     FSO(1000, 1e3, f4->i2) -> Delta(i2) -> Shuffle(2)
  C5  8192 x 1 MiB f32, chunk c from seed 1000 + c   Shuffle(4) -> Fletcher32
"""

from __future__ import annotations

import numpy as np

MiB = 1 << 20


def words(seed: int, n: int) -> np.ndarray:
    """n raw 64-bit PCG64 outputs."""
    return np.random.PCG64(seed).random_raw(n).astype(np.uint64, copy=False)


def f32_wide(seed: int, n: int) -> np.ndarray:
    """float32 with random sign/mantissa and biased exponent in [100, 154):
    values from ~1e-8 to ~1e8, every mantissa bit exercised."""
    w = words(seed, n)
    sign = (w >> np.uint64(63)).astype(np.uint32) << np.uint32(31)
    exp = ((w >> np.uint64(23)) % np.uint64(54) + np.uint64(100)).astype(np.uint32) << np.uint32(23)
    mant = (w & np.uint64(0x7FFFFF)).astype(np.uint32)
    return (sign | exp | mant).view(np.float32)


def f64_wide(seed: int, n: int) -> np.ndarray:
    """float64 with random sign/mantissa and biased exponent in [990, 1058)."""
    w = words(seed, n)
    sign = (w >> np.uint64(63)) << np.uint64(63)
    w2 = words(seed + 0x5EED, n)
    exp = ((w2 % np.uint64(68)) + np.uint64(990)) << np.uint64(52)
    mant = w & np.uint64((1 << 52) - 1)
    return (sign | exp | mant).view(np.float64)


def f32_c4(seed: int, n: int) -> np.ndarray:
    """1000 + 10*tri(i/4096) + U(-0.5, 0.5): |(x - 1000) * 1e3| <= 10500 < 32767.

    Every step is exact in float64 (24-bit uniforms, dyadic triangle wave),
    then one correctly rounded cast to float32."""
    w = words(seed, n)
    u = (w >> np.uint64(40)).astype(np.float64) * 2.0**-24  # [0, 1), 24 bits
    i = np.arange(n, dtype=np.int64) % 4096
    tri = np.abs(i.astype(np.float64) / 2048.0 - 1.0)  # [0, 1], dyadic
    return (1000.0 + 10.0 * tri + (u - 0.5)).astype(np.float32)


def c5_chunk(chunk: int, chunk_bytes: int = MiB) -> np.ndarray:
    """C5 chunk `chunk` as float32 (seed 1000 + chunk)."""
    return f32_wide(1000 + chunk, chunk_bytes // 4)


def c5_chunk_bytes_formula(chunk: int, nbytes: int) -> np.ndarray:
    """Cheap deterministic chunk bytes computable identically in torch on the
    device (used to fill the 8 GiB C5 batch without a host upload):
    byte[i] = ((i * 2654435761 + chunk * 40503) >> 13) & 0xff."""
    i = np.arange(nbytes, dtype=np.int64)
    return (((i * 2654435761 + chunk * 40503) >> 13) & 0xFF).astype(np.uint8)
