"""Blosc shuffle framing restated in numpy -- TEST INFRASTRUCTURE ONLY.

SURVEY.md §8f row 2: Blosc's byte-shuffle and bit-shuffle filters as they
act on each Blosc block (blosc.pyx:67-71 SHUFFLE/BITSHUFFLE/AUTOSHUFFLE,
:211-326 compress/decompress).  The algorithms live in the third-party c-blosc
library (its submodule is empty in the reference checkout, so it is absent
here): c-blosc 1.x shuffle.c ``shuffle``/``bitshuffle`` and the bitshuffle
library's ``bshuf_trans_bit_elem``, restated from their published behaviour
and pinned ONLY by the reference's ``fixture/blosc`` frames: this module
also carries a minimal Blosc1 frame walker and an LZ4 block decoder (the
published LZ4 block format) so that the frames' shuffled block bytes can be
recovered and compared byte for byte.  Pinned facts (tests/test_oracle_next.py):

* a block of ``bsize`` bytes holds ``E = bsize // typesize`` elements;
* byte shuffle: the (E, typesize) byte matrix is transposed; the
  ``bsize % typesize`` trailing bytes are copied;
* bit shuffle: if E % 8 == 0, bit k (LSB = 0) of byte j of element i goes to
  bit (i % 8) of byte i // 8 of bit-plane ``8*j + k`` (planes of E/8 bytes,
  ordered byte-major); otherwise the whole block is copied unchanged
  (fixture/blosc codec.05 array.04: typesize 3, E = 85 and 65);
* blocks: the buffer is cut into ``blocksize``-byte blocks, the last one
  shorter; each is filtered on its own.
"""

from __future__ import annotations

import struct

import numpy as np

BLOSC_DOSHUFFLE = 0x1
BLOSC_MEMCPYED = 0x2
BLOSC_DOBITSHUFFLE = 0x4
BLOSC_NOSPLIT = 0x10
LZ4_FORMAT = 1  # flags >> 5


def lz4_block_decompress(src: bytes, usize: int) -> bytes:
    """LZ4 block format: sequences of token, literals, 2-byte offset, match."""
    out = bytearray()
    i, n = 0, len(src)
    while i < n:
        tok = src[i]
        i += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        out += src[i:i + lit]
        i += lit
        if i >= n:
            break
        off = src[i] | (src[i + 1] << 8)
        i += 2
        ml = tok & 15
        if ml == 15:
            while True:
                b = src[i]
                i += 1
                ml += b
                if b != 255:
                    break
        ml += 4
        st = len(out) - off
        for k in range(ml):  # overlapping copies are byte-serial by definition
            out.append(out[st + k])
    if len(out) != usize:
        raise ValueError(f"lz4 block decoded to {len(out)} bytes, expected {usize}")
    return bytes(out)


def frame_header(frame: bytes):
    """(flags, typesize, nbytes, blocksize, cbytes) of a Blosc1 frame."""
    flags, ts = frame[2], frame[3]
    nbytes, bs, cbytes = struct.unpack("<III", frame[4:16])
    return flags, ts, nbytes, bs, cbytes


def frame_filtered_blocks(frame: bytes):
    """The still-shuffled bytes of every block of an LZ4 (or memcpyed)
    Blosc1 frame: (flags, typesize, blocksize, [block bytes]), or blocks=None
    for memcpyed frames (stored raw, no filter applied)."""
    flags, ts, nbytes, bs, _ = frame_header(frame)
    if flags & BLOSC_MEMCPYED:
        return flags, ts, bs, None
    if flags >> 5 != LZ4_FORMAT:
        raise NotImplementedError("only LZ4 frames are walked by the oracle")
    nblocks = (nbytes + bs - 1) // bs
    starts = struct.unpack(f"<{nblocks}I", frame[16:16 + 4 * nblocks])
    blocks = []
    for bi, s in enumerate(starts):
        bsize = bs if (bi < nblocks - 1 or nbytes % bs == 0) else nbytes % bs
        split = not (flags & BLOSC_NOSPLIT) and bsize == bs and ts <= 16 and bsize // ts >= 128
        nsplit = ts if split else 1
        neb = bsize // nsplit
        p, out = s, b""
        for _ in range(nsplit):
            cb = struct.unpack("<i", frame[p:p + 4])[0]
            p += 4
            out += frame[p:p + cb] if cb == neb else lz4_block_decompress(frame[p:p + cb], neb)
            p += cb
        blocks.append(out)
    return flags, ts, bs, blocks


# ---------------------------------------------------------------------------
# the filters, per block and per buffer
# ---------------------------------------------------------------------------
def byteshuffle_block(blk: bytes, ts: int) -> bytes:
    e = len(blk) // ts
    body = np.frombuffer(blk, np.uint8)[: e * ts].reshape(e, ts).T.tobytes()
    return body + blk[e * ts:]


def byteunshuffle_block(blk: bytes, ts: int) -> bytes:
    e = len(blk) // ts
    body = np.frombuffer(blk, np.uint8)[: e * ts].reshape(ts, e).T.tobytes()
    return body + blk[e * ts:]


def bitshuffle_block(blk: bytes, ts: int) -> bytes:
    e = len(blk) // ts
    if e % 8:
        return bytes(blk)
    x = np.frombuffer(blk, np.uint8)[: e * ts].reshape(e, ts)
    bits = np.unpackbits(x[..., None], axis=-1, bitorder="little")  # (e, ts, 8)
    planes = bits.transpose(1, 2, 0).reshape(ts * 8, e)
    return np.packbits(planes, axis=1, bitorder="little").tobytes() + blk[e * ts:]


def bitunshuffle_block(blk: bytes, ts: int) -> bytes:
    e = len(blk) // ts
    if e % 8:
        return bytes(blk)
    planes = np.frombuffer(blk, np.uint8)[: e * ts].reshape(ts * 8, e // 8)
    bits = np.unpackbits(planes, axis=1, bitorder="little").reshape(ts, 8, e)
    x = np.packbits(bits.transpose(2, 0, 1), axis=-1, bitorder="little").reshape(e, ts)
    return x.tobytes() + blk[e * ts:]


_FILTERS = {
    (1, True): byteshuffle_block, (1, False): byteunshuffle_block,
    (2, True): bitshuffle_block, (2, False): bitunshuffle_block,
}


def blosc_filter(buf, typesize: int, blocksize: int, mode: int, forward: bool = True) -> bytes:
    """Apply mode 1 (SHUFFLE) / 2 (BITSHUFFLE) block by block."""
    raw = bytes(np.ascontiguousarray(np.frombuffer(memoryview(buf), np.uint8)))
    fn = _FILTERS[(mode, forward)]
    return b"".join(fn(raw[p:p + blocksize], typesize) for p in range(0, len(raw), blocksize))
