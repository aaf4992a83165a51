#!/usr/bin/env python3
"""Generate mc_crc_bs.h: bit-sliced CRC32 / CRC32C tile folds (no table lookups).

What the kernel needs per lane (mc_checksum.hip, k_ck_tiles): for the K 16-B
vectors v[0..K-1] a lane reads at byte offsets k*STEP (STEP = 4096) of its
virtual message, the raw register (zero init, no inversion)

    acc = raw(0, v[0] ++ zeros(STEP-16) ++ v[1] ++ ... ++ v[K-1] ++ zeros(STEP-16))

-- the value the slicing-by-16 LDS tables produce today.  raw(0, .) is linear
over GF(2), and with the reflected representation (bit 31 = x^0, bit 0 =
x^31) message bit q of an N-byte message contributes x^(8N - 1 - q + 32) mod P.
Dword j of the lane (byte offset o_j, bit s = message bit 8*o_j + s) therefore
contributes  d_j[s] * x^(31-s) * z_j  with  z_j = x^(8 (N - o_j)) mod P.

Bit-slice over s: the 32 bit positions of a dword are 32 independent streams.
Stream s accumulates H_s = XOR_j d_j[s] * z_j, a field element; store it
transposed, as 32 words W_i whose bit s is coefficient i of H_s.  Then

    W_i = XOR of the data dwords D_j whose z_j has coefficient i set

-- plain XORs of whole loaded dwords, no transpose, no lookups -- and

    acc = XOR_s x^(31-s) H_s = XOR_i x^i * W_i      (W_i read as a polynomial:
                                                      bit s <-> x^(31-s))

which is a 31-step Horner with multiply-by-x (shift + conditional poly).

The XOR network uses the method of four Russians over the 4 dwords of each
vector (11 XORs build a group's 15 non-zero combinations) and accumulates two
groups per 3-input XOR (v_bitop3_b32 0x96, which the compiler does not form
from a^b^c by itself).  Every function is checked here against a bytewise CRC
on random inputs before the header is written.

Usage:  python3 gen_crc_bs.py [out.h]     (default: mc_crc_bs.h next to this file)
"""

import os
import random
import sys

POLYS = {"crc32": 0xEDB88320, "crc32c": 0x82F63B78}
STEP = 4096
KS = (4, 8, 16)
ONE = 0x80000000  # x^0 in the reflected representation


def gf_mul(a, b, poly):
    p = 0
    for i in range(32):
        if a & (ONE >> i):
            p ^= b
        b = (b >> 1) ^ poly if b & 1 else b >> 1
    return p


def xpow(e, poly):
    r, base = ONE, 0x40000000  # x^1
    while e:
        if e & 1:
            r = gf_mul(r, base, poly)
        base = gf_mul(base, base, poly)
        e >>= 1
    return r


def raw(c, data, poly):
    """Reflected CRC register update, no pre/post inversion."""
    for byte in data:
        c ^= byte
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
    return c


def mulx(a, poly):
    return (a >> 1) ^ (poly if a & 1 else 0)


def columns(K, poly):
    """z_j for the lane's dwords j = 4k + w (offset k*STEP + 4w of N = K*STEP)."""
    n = K * STEP
    return [xpow(8 * (n - (k * STEP + 4 * w)), poly) for k in range(K) for w in range(4)]


def model(dwords, K, poly):
    """The bit-sliced computation in Python (what the emitted code does)."""
    z = columns(K, poly)
    W = [0] * 32
    for i in range(32):
        for j, zj in enumerate(z):
            if zj & (ONE >> i):
                W[i] ^= dwords[j]
    acc = W[31]
    for i in range(30, -1, -1):
        acc = mulx(acc, poly) ^ W[i]
    return acc


def reference(dwords, K, poly):
    msg = bytearray()
    for k in range(K):
        for w in range(4):
            msg += dwords[4 * k + w].to_bytes(4, "little")
        msg += bytes(STEP - 16)
    return raw(0, msg, poly)


def emit(name, K, poly):
    z = columns(K, poly)
    J = 4 * K
    lines = [f"MC_DEV uint32_t {name}(const mc_u32x4 *__restrict__ v) {{"]
    for k in range(K):
        lines.append(f"  const uint32_t d{4*k} = v[{k}].x, d{4*k+1} = v[{k}].y, "
                     f"d{4*k+2} = v[{k}].z, d{4*k+3} = v[{k}].w;")
    # pattern of output i in group g: bit b set when dword 4g+b feeds W_i
    pat = [[sum(1 << b for b in range(4) if z[4 * g + b] & (ONE >> i)) for g in range(K)] for i in range(32)]
    nops = 0

    def combos(g):
        nonlocal nops
        need = {pat[i][g] for i in range(32)} - {0}
        names = {}
        for m in (1, 2, 4, 8):
            names[m] = f"d{4*g + m.bit_length() - 1}"
        order = sorted(need, key=lambda m: bin(m).count("1"))  # pairs first
        out = []

        def get(m):  # triples: one X3 of singles; the quad: pair ^ pair
            nonlocal nops
            if m in names:
                return names[m]
            bits = [b for b in range(4) if m >> b & 1]
            nm = f"c{g}_{m}"
            if len(bits) == 2:
                out.append(f"  const uint32_t {nm} = {get(1 << bits[0])} ^ {get(1 << bits[1])};")
            elif len(bits) == 3:
                out.append(f"  const uint32_t {nm} = X3({get(1 << bits[0])}, {get(1 << bits[1])}, {get(1 << bits[2])});")
            else:
                out.append(f"  const uint32_t {nm} = {get(3)} ^ {get(12)};")
            nops += 1
            names[m] = nm
            return nm
        for m in order:
            get(m)
        return names, out

    started = [False] * 32
    for g0 in range(0, K, 2):
        gs = [g for g in (g0, g0 + 1) if g < K]
        tables = []
        for g in gs:
            names, out = combos(g)
            lines += out
            tables.append((g, names))
        for i in range(32):
            terms = [names[pat[i][g]] for g, names in tables if pat[i][g]]
            if not started[i]:
                if not terms:
                    continue
                started[i] = True
                expr = terms[0] if len(terms) == 1 else f"{terms[0]} ^ {terms[1]}"
                nops += len(terms) - 1
                lines.append(f"  uint32_t w{i} = {expr};")
            elif len(terms) == 2:
                lines.append(f"  w{i} = X3(w{i}, {terms[0]}, {terms[1]});")
                nops += 1
            elif len(terms) == 1:
                lines.append(f"  w{i} ^= {terms[0]};")
                nops += 1
    for i in range(32):
        if not started[i]:
            lines.append(f"  const uint32_t w{i} = 0;")
    lines.append(f"  uint32_t acc = w31;")
    for i in range(30, -1, -1):
        lines.append(f"  acc = MULX_XOR(acc, w{i}, 0x{poly:08X}u);")
    lines.append("  return acc;")
    lines.append("}")
    return lines, nops


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "mc_crc_bs.h")
    rng = random.Random(1234)
    body = []
    stats = []
    for pname, poly in POLYS.items():
        for K in KS:
            for trial in range(6):
                d = [rng.getrandbits(32) for _ in range(4 * K)]
                if trial == 0:
                    d = [0] * (4 * K)
                    d[rng.randrange(4 * K)] = 1 << rng.randrange(32)
                assert model(d, K, poly) == reference(d, K, poly), (pname, K, trial)
            name = f"crc_bs_{pname}_k{K}"
            lines, nops = emit(name, K, poly)
            stats.append(f"//   {name}: {nops} XOR-network ops + 31 Horner steps for {16 * K} bytes per lane")
            body += lines + [""]
    hdr = [
        "// mc_crc_bs.h -- GENERATED by gen_crc_bs.py; do not edit.",
        "// Bit-sliced CRC32 / CRC32C tile folds for k_ck_tiles (mc_checksum.hip):",
        "// acc = raw(0, v[0] ++ zeros(4080) ++ ... ++ v[K-1] ++ zeros(4080)) with no",
        "// table lookups (derivation in gen_crc_bs.py).  Checked against a bytewise",
        "// CRC on random inputs by the generator.",
    ] + stats + [
        "#pragma once",
        "#include \"mc_common.h\"",
        "",
        "#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)",
        "// a * x mod P (reflected) xor w: shift, sign-extended low bit & poly, xor3",
        "#define MULX_XOR(a, w, poly) X3((a) >> 1, (uint32_t)__builtin_amdgcn_sbfe((int)(a), 0, 1) & (poly), (w))",
        "",
    ] + body + ["#undef MULX_XOR", "#undef X3", ""]
    with open(out, "w") as f:
        f.write("\n".join(hdr))
    print("\n".join(stats))


if __name__ == "__main__":
    main()
