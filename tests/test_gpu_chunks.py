"""Zarr-style chunk pipelines (numcodecs_amd.chunks / batch, SURVEY.md §8f
row 1) pinned to the ORACLE row by row: every row of a batched, host-streamed
or padded-stride batch must equal the oracle's codecs applied one after
another to that chunk (tests/oracle_chain.py; the reference harness shape is
tests/common.py:51-116 of numcodecs), encode and decode."""

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import (
    CRC32, CRC32C, Adler32, AsType, BitRound, Delta, FixedScaleOffset, Fletcher32, JenkinsLookup3,
    PackBits, Quantize, Shuffle, batch, chunks, multi,
)
from tests import oracle_chain

pytestmark = pytest.mark.gpu


def _chains():
    return {
        "bitround_shuffle_crc32": ([BitRound(10), Shuffle(4), CRC32()], torch.float32),
        "fso_delta_shuffle_adler32": ([FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
                                       Delta(dtype="<i2"), Shuffle(2), Adler32(location="end")], torch.float32),
        "quantize_shuffle_fletcher32": ([Quantize(3, "<f8", "<f4"), Shuffle(4), Fletcher32()], torch.float64),
        "astype_shuffle_jenkins": ([AsType("<f4", "<f8"), Shuffle(4), JenkinsLookup3(initval=7)], torch.float64),
        "delta_shuffle_crc32c": ([Delta(dtype="<i4"), Shuffle(4), CRC32C()], torch.int32),
        "bitround_shuffle_fletcher32": ([BitRound(12), Shuffle(4), Fletcher32()], torch.float32),
        "delta_i8_i2_shuffle_crc32": ([Delta(dtype="<i8", astype="<i2"), Shuffle(2), CRC32(location="end")],
                                      torch.int64),
        "packbits": ([PackBits()], torch.bool),
    }


def _make(dtype, b, n, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    if dtype == torch.bool:
        return torch.randint(0, 2, (b, n), generator=g, device=device).to(torch.bool)
    if dtype in (torch.int32, torch.int64):
        return torch.randint(-1000, 1000, (b, n), generator=g, device=device, dtype=dtype)
    return (1000 + 10 * torch.rand((b, n), generator=g, device=device)).to(dtype)


def _rows_u8(t, b):
    return t.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()


@pytest.mark.parametrize("name", list(_chains()))
@pytest.mark.parametrize("n", [4096 * 3, 1000, 77])
def test_encode_decode_chunks_vs_oracle(device, name, n):
    """encode_chunks / decode_chunks: every row equals the oracle chain; the
    chunk lengths cover whole tiles, ragged tails and a tiny chunk."""
    codecs, dtype = _chains()[name]
    b = 7
    x = _make(dtype, b, n, device, 1)
    xh = x.cpu().numpy()
    enc = chunks.encode_chunks(codecs, x)
    assert enc.shape[0] == b
    enc_u8 = _rows_u8(enc, b)
    for i in range(b):
        ref = oracle_chain.chain_encode(codecs, xh[i])
        assert enc_u8[i].tobytes() == ref, (name, n, i)
    dec = chunks.decode_chunks(codecs, enc)
    dec_u8 = _rows_u8(dec, b)
    for i in range(b):
        ref = oracle_chain.chain_decode(codecs, enc_u8[i].tobytes())
        assert dec_u8[i].tobytes() == ref, (name, n, i)


@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "quantize_shuffle_fletcher32", "astype_shuffle_jenkins"])
def test_decode_chunks_detects_corruption(device, name):
    codecs, dtype = _chains()[name]
    x = _make(dtype, 5, 4096, device, 2)
    enc = chunks.encode_chunks(codecs, x).clone()
    enc.view(torch.uint8)[3, 100] ^= 1
    with pytest.raises(RuntimeError):
        oracle_chain.chain_decode(codecs, enc.view(torch.uint8)[3].cpu().numpy().tobytes())
    with pytest.raises(RuntimeError):
        chunks.decode_chunks(codecs, enc)


@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "fso_delta_shuffle_adler32", "delta_shuffle_crc32c",
                                  "bitround_shuffle_fletcher32"])
def test_host_streamed_chunks_vs_oracle(device, name):
    """host_encode_chunks / host_decode_chunks (pinned slices through a ring of
    device buffers on three streams): every row equals the oracle chain."""
    codecs, dtype = _chains()[name]
    b = 23
    x = _make(dtype, b, 4096 * 2, device, 3)
    host = x.cpu().pin_memory()
    xh = host.numpy()
    enc_host = chunks.host_encode_chunks(codecs, host, slice_chunks=4, nslots=3)
    eh = enc_host.numpy()
    for i in range(b):
        assert eh[i].tobytes() == oracle_chain.chain_encode(codecs, xh[i]), (name, i)
    out = torch.empty_like(host).pin_memory()
    chunks.host_decode_chunks(codecs, enc_host, out, slice_chunks=5, nslots=2)
    oh = out.view(torch.uint8).reshape(b, -1).numpy()
    for i in range(b):
        assert oh[i].tobytes() == oracle_chain.chain_decode(codecs, eh[i].tobytes()), (name, i)


def test_host_decode_detects_corruption_after_stream(device):
    codecs, dtype = _chains()["bitround_shuffle_crc32"]
    x = _make(dtype, 9, 4096, device, 4)
    enc = chunks.host_encode_chunks(codecs, x.cpu().pin_memory(), slice_chunks=2)
    enc[6, 50] ^= 1
    out = torch.empty((9, 4096), dtype=torch.float32).pin_memory()
    with pytest.raises(RuntimeError, match="crc32 checksum do not match"):
        chunks.host_decode_chunks(codecs, enc, out, slice_chunks=2)


# ---------------------------------------------------------------------------
# batch-level entry points on padded rows (row stride > row bytes) and on
# checksum rows of n + 4 bytes (4-B aligned when n % 4 == 0, unaligned else)
# ---------------------------------------------------------------------------
def _padded(device, b, n, pad, seed):
    """[b, n] uint8 view of a [b, n + pad] buffer (padding bytes random)."""
    g = torch.Generator(device=device).manual_seed(seed)
    big = torch.randint(0, 256, (b, n + pad), generator=g, device=device, dtype=torch.uint8)
    return big[:, :n]


@pytest.mark.parametrize("n,pad", [(4096 * 4, 256), (4096 * 4, 4), (1000, 24), (65536 + 12, 4)])
@pytest.mark.parametrize("es", [2, 4, 8])
def test_shuffle_chunks_padded_vs_oracle(device, n, pad, es):
    if n % es:
        pytest.skip("Shuffle of a ragged element count is covered by the codec tests")
    x = _padded(device, 9, n, pad, 5)
    assert x.stride(0) == n + pad
    xh = x.cpu().numpy()
    out_big = torch.zeros((9, n + 8), dtype=torch.uint8, device=device)
    enc = batch.shuffle_chunks(x, es, out=out_big[:, :n])
    eh = out_big.cpu().numpy()
    for i in range(9):
        assert eh[i, :n].tobytes() == oracle.shuffle(xh[i], es).tobytes(), (n, pad, es, i)
        assert not eh[i, n:].any(), "padding written"
    dec = batch.unshuffle_chunks(enc, es)
    dh = dec.cpu().numpy()
    for i in range(9):
        assert dh[i].tobytes() == oracle.unshuffle(eh[i, :n], es).tobytes()


@pytest.mark.parametrize("n,pad", [(4096 * 4, 256), (4096, 4), (1002, 6), (3, 1)])
def test_checksum_rows_padded_vs_oracle(device, n, pad):
    """Fletcher32 / CRC32 / CRC32C / Adler32 batch encode into rows of n + 4
    bytes (stride n + 4: 4-B aligned rows when n % 4 == 0) from padded input
    rows; decode of those rows compacts the payloads; every row vs oracle."""
    b = 11
    x = _padded(device, b, n, pad, 6)
    xh = x.cpu().numpy()
    out = batch.fletcher32_encode_chunks(x)
    assert out.stride(0) == n + 4
    oh = out.cpu().numpy()
    for i in range(b):
        assert oh[i].tobytes() == oracle.fletcher32_encode(xh[i]), (n, i)
    payloads, sums, stored = batch.fletcher32_decode_chunks(out)
    ph = payloads.cpu().numpy()
    assert torch.equal(sums, stored)
    for i in range(b):
        assert ph[i].tobytes() == xh[i].tobytes()
    for cid in ("crc32", "crc32c", "adler32"):
        for loc in ("start", "end"):
            out = batch.checksum32_encode_chunks(x, cid, location=loc)
            oh = out.cpu().numpy()
            for i in range(b):
                assert oh[i].tobytes() == oracle.checksum32_encode(cid, xh[i], loc).tobytes(), (cid, loc, n, i)
            payloads, sums, stored = batch.checksum32_decode_chunks(out, cid, location=loc)
            assert torch.equal(sums, stored), (cid, loc)
            ph = payloads.cpu().numpy()
            for i in range(b):
                assert ph[i].tobytes() == oracle.checksum32_decode(cid, oh[i], loc).tobytes()


@pytest.mark.parametrize("dt,at", [("<i2", "<i2"), ("<i4", "<i4"), ("<i8", "<i2"), ("<f4", "<f4"), ("<u2", "<u2")])
def test_delta_chunks_padded_vs_oracle(device, dt, at):
    """batch.delta_chunks on padded rows: each row its own Delta (first
    element + running sum), delta.py:52-83, vs the oracle."""
    d = Delta(dtype=dt, astype=at)
    b, n = 6, 3001
    isz, asz = np.dtype(dt).itemsize, np.dtype(at).itemsize
    rng = np.random.default_rng(7)
    if np.dtype(dt).kind == "f":
        vals = np.cumsum(rng.integers(-4, 5, (b, n))).reshape(b, n).astype(dt)  # exact steps
    else:
        vals = rng.integers(-100, 100, (b, n)).astype(dt)
    big = torch.zeros((b, n * isz + 40), dtype=torch.uint8, device=device)
    big[:, : n * isz] = torch.from_numpy(vals.view(np.uint8).reshape(b, -1)).to(device)
    x = big[:, : n * isz]
    enc = batch.delta_chunks(x, d, encode=True)
    eh = enc.cpu().numpy()
    for i in range(b):
        assert eh[i].tobytes() == oracle.delta_encode(vals[i], dt, at).tobytes(), (dt, at, i)
    ebig = torch.zeros((b, n * asz + 24), dtype=torch.uint8, device=device)
    ebig[:, : n * asz] = enc
    dec = batch.delta_chunks(ebig[:, : n * asz], d, encode=False)
    dh = dec.cpu().numpy()
    for i in range(b):
        assert dh[i].tobytes() == oracle.delta_decode(eh[i], dt, at).tobytes(), (dt, at, i)


@pytest.mark.parametrize("es", [2, 4, 8])
def test_shuffle_fletcher32_fused_rows_vs_oracle(device, es):
    """The fused Shuffle + Fletcher32 batch (rows padded to encoded_stride)
    and its fused verify + unshuffle: every row vs the oracle."""
    b, n = 9, 8192 * es
    x = _padded(device, b, n, 64, 8)
    xh = x.cpu().numpy()
    enc = batch.shuffle_fletcher32_encode_chunks(x, es)
    assert enc.stride(0) == batch.encoded_stride(n)
    eh = enc.cpu().numpy()
    for i in range(b):
        ref = oracle.fletcher32_encode(oracle.shuffle(xh[i], es))
        assert eh[i, : n + 4].tobytes() == ref, (es, i)
    dec, status = batch.fletcher32_unshuffle_decode_chunks(enc, n, es)
    dh = dec.cpu().numpy()
    for i in range(b):
        assert dh[i].tobytes() == oracle.unshuffle(oracle.fletcher32_decode(eh[i, : n + 4]), es).tobytes()



@pytest.mark.parametrize("dt,at,scale", [("<f4", "<i2", 1e3), ("<f8", "<u4", 1e6), ("<f4", "<i4", 3.7)])
@pytest.mark.parametrize("n,b", [(4096 * 3, 5), (4096 * 64 + 48, 3), (16, 9)])
def test_fused_c4_batch_vs_oracle(device, dt, at, scale, n, b):
    """[FixedScaleOffset, Delta, Shuffle] over a batch runs the fused batched
    kernels (one launch each way, a single-pass row decode); every row vs the
    oracle chain, and the public batch functions on padded rows."""
    codecs = [FixedScaleOffset(offset=1000, scale=scale, dtype=dt, astype=at), Delta(dtype=at),
              Shuffle(np.dtype(at).itemsize)]
    rng = np.random.default_rng(n + b)
    xh = (1000.0 + rng.uniform(-15, 15, (b, n))).astype(dt)
    x = torch.from_numpy(xh).to(device)
    assert batch.fso_delta_shuffle_encode_chunks(x.view(torch.uint8), *codecs) is not None  # the fused path applies
    enc = chunks.encode_chunks(codecs, x)
    eh = enc.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    for i in range(b):
        assert eh[i].tobytes() == oracle_chain.chain_encode(codecs, xh[i]), i
    dec = chunks.decode_chunks(codecs, enc)
    assert dec.dtype == x.dtype
    dh = dec.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    for i in range(b):
        assert dh[i].tobytes() == oracle_chain.chain_decode(codecs, eh[i].tobytes()), i
    # padded rows (16-B multiple strides) through the batch functions
    pad_in = torch.zeros((b, n * np.dtype(dt).itemsize + 64), dtype=torch.uint8, device=device)
    pad_in[:, : n * np.dtype(dt).itemsize] = x.view(torch.uint8)
    e2 = batch.fso_delta_shuffle_encode_chunks(pad_in[:, : n * np.dtype(dt).itemsize], *codecs)
    assert torch.equal(e2, enc.view(torch.uint8).reshape(b, -1))
    pad_enc = torch.zeros((b, e2.shape[1] + 32), dtype=torch.uint8, device=device)
    pad_enc[:, : e2.shape[1]] = e2
    d2 = batch.fso_delta_shuffle_decode_chunks(pad_enc[:, : e2.shape[1]], *codecs)
    assert torch.equal(d2, dec.contiguous().view(torch.uint8).reshape(b, -1))


@pytest.mark.parametrize("b,n", [(1, 4096 * 40 + 16), (3, 4096 * 7 + 32), (40, 4096 * 2)])
def test_fused_c4_batch_segments_vs_oracle(device, b, n):
    """Few chunks: the batched decode cuts each chunk into segments (a first
    pass of segment totals); every row still equals the oracle."""
    from numcodecs_amd._native import lib

    codecs = [FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"), Delta(dtype="<i2"), Shuffle(2)]
    assert lib.mc_fso_delta_shuffle_decode_batch_workspace(b, n) > 0  # segmented
    rng = np.random.default_rng(b * n)
    xh = (1000.0 + rng.uniform(-15, 15, (b, n))).astype("<f4")
    enc = chunks.encode_chunks(codecs, torch.from_numpy(xh).to(device))
    eh = enc.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    dh = chunks.decode_chunks(codecs, enc).contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    for i in range(b):
        assert dh[i].tobytes() == oracle_chain.chain_decode(codecs, eh[i].tobytes()), i


def test_few_large_rows_decode_row_by_row(device):
    """Rows of at least batch._LARGE_ROW bytes (at most _FEW_ROWS for the chain) decode
    row by row with the single-chunk decodes (the whole chip per row), both
    for the fused [FixedScaleOffset, Delta, Shuffle] chain and for
    batch.delta_chunks; vs the oracle."""
    n = batch._LARGE_ROW // 2 + 16
    b = 2
    codecs = [FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"), Delta(dtype="<i2"), Shuffle(2)]
    rng = np.random.default_rng(5)
    xh = (1000.0 + rng.uniform(-15, 15, (b, n))).astype("<f4")
    enc = chunks.encode_chunks(codecs, torch.from_numpy(xh).to(device))
    eh = enc.contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    dh = chunks.decode_chunks(codecs, enc).contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    for i in range(b):
        assert dh[i].tobytes() == oracle_chain.chain_decode(codecs, eh[i].tobytes()), i
    d = Delta(dtype="<i4", astype="<i2")
    eh2 = rng.integers(-300, 300, (b, n)).astype("<i2")
    out = batch.delta_chunks(torch.from_numpy(eh2.view(np.uint8)).to(device), d, encode=False).cpu().numpy()
    for i in range(b):
        assert out[i].tobytes() == oracle.delta_decode(eh2[i], "<i4", "<i2").view(np.uint8).tobytes(), i


# ---------------------------------------------------------------------------
# in-process multi-GPU dispatch (numcodecs_amd.multi): devices=[cuda:0,
# cuda:0] runs two independent workers with their own streams and rings on
# the one GPU of the box -- the same partition, threads and gathering as a
# multi-GPU node (unmeasured there)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "fso_delta_shuffle_adler32", "delta_shuffle_crc32c",
                                  "quantize_shuffle_fletcher32"])
@pytest.mark.parametrize("ndev", [2, 3])
def test_multi_device_chunks_vs_oracle(device, name, ndev):
    codecs, dtype = _chains()[name]
    b = 11
    devs = [device] * ndev
    x = _make(dtype, b, 4096 + 64, device, 21)
    xh = x.cpu().numpy()
    enc = chunks.encode_chunks(codecs, x, devices=devs)
    enc_u8 = _rows_u8(enc, b)
    for i in range(b):
        assert enc_u8[i].tobytes() == oracle_chain.chain_encode(codecs, xh[i]), (name, i)
    assert torch.equal(enc.view(torch.uint8).reshape(b, -1), chunks.encode_chunks(codecs, x).view(torch.uint8).reshape(b, -1))
    dec = chunks.decode_chunks(codecs, enc, devices=devs)
    dec_u8 = _rows_u8(dec, b)
    for i in range(b):
        assert dec_u8[i].tobytes() == oracle_chain.chain_decode(codecs, enc_u8[i].tobytes()), (name, i)
    # host-streamed, several workers at once
    host = x.cpu().pin_memory()
    eh = chunks.host_encode_chunks(codecs, host, slice_chunks=2, devices=devs).numpy()
    assert eh.tobytes() == enc_u8.tobytes()
    out = torch.empty_like(host).pin_memory()
    chunks.host_decode_chunks(codecs, torch.from_numpy(eh).pin_memory(), out, slice_chunks=3, devices=devs)
    assert out.view(torch.uint8).reshape(b, -1).numpy().tobytes() == dec_u8.tobytes()


def test_multi_device_decode_raises_first_mismatch(device):
    """A corrupted row in the second worker's range raises the reference's
    RuntimeError after both workers finished."""
    codecs, dtype = _chains()["bitround_shuffle_crc32"]
    x = _make(dtype, 8, 4096, device, 22)
    enc = chunks.encode_chunks(codecs, x, devices=[device, device]).clone()
    enc.view(torch.uint8)[6, 40] ^= 1
    with pytest.raises(RuntimeError, match="crc32 checksum do not match"):
        chunks.decode_chunks(codecs, enc, devices=[device, device])
    host = enc.cpu().pin_memory()
    out = torch.empty((8, 4096), dtype=torch.float32).pin_memory()
    with pytest.raises(RuntimeError, match="crc32 checksum do not match"):
        chunks.host_decode_chunks(codecs, host, out, slice_chunks=2, devices=[device, device])


@pytest.mark.parametrize("es", [4, 8])
def test_multi_device_host_pipeline_vs_oracle(device, es, monkeypatch):
    b, n = 13, 65536 + 16 * es
    g = torch.Generator().manual_seed(23)
    host_in = torch.randint(0, 256, (b, n), generator=g, dtype=torch.uint8).pin_memory()
    host_out = torch.empty_like(host_in).pin_memory()
    runs = []
    real = multi.run_workers
    monkeypatch.setattr(multi, "run_workers", lambda fns: runs.append(len(fns)) or real(fns))
    batch.host_pipeline(host_in, host_out, es, encode=True, slice_chunks=3, devices=[device, device, device])
    assert runs == [3], runs  # three workers, one per devices entry
    hi, ho = host_in.numpy(), host_out.numpy()
    for i in range(b):
        assert ho[i].tobytes() == oracle.shuffle(hi[i], es).tobytes(), i
    back = torch.empty_like(host_in).pin_memory()
    batch.host_pipeline(host_out, back, es, encode=False, slice_chunks=2, devices=[device, device])
    assert torch.equal(back, host_in)


@pytest.mark.parametrize("name", ["bitround_shuffle_crc32", "fso_delta_shuffle_adler32"])
def test_resident_shards_vs_oracle(device, name):
    """Per-device resident shards (a list of device tensors; here both on the
    box's one GPU): each shard encodes / decodes where it lives, results
    left on its device, byte-identical to the oracle chain row by row."""
    codecs, dtype = _chains()[name]
    xs = [_make(dtype, b, 4096 + 32, device, 30 + b) for b in (5, 3)]
    encs = chunks.encode_chunks(codecs, xs)
    assert isinstance(encs, list) and len(encs) == 2
    for x, e in zip(xs, encs):
        assert e.device == x.device
        eu = _rows_u8(e, x.shape[0])
        xh = x.cpu().numpy()
        for i in range(x.shape[0]):
            assert eu[i].tobytes() == oracle_chain.chain_encode(codecs, xh[i]), (name, i)
    decs = chunks.decode_chunks(codecs, encs)
    for x, e, d in zip(xs, encs, decs):
        du = _rows_u8(d, x.shape[0])
        eu = _rows_u8(e, x.shape[0])
        for i in range(x.shape[0]):
            assert du[i].tobytes() == oracle_chain.chain_decode(codecs, eu[i].tobytes()), (name, i)
    bad = [e.clone() for e in encs]
    bad[1].view(torch.uint8)[2, 17] ^= 1
    with pytest.raises(RuntimeError, match="checksum do not match"):
        chunks.decode_chunks(codecs, bad)


def test_one_device_batch_refuses_other_gpus(device):
    """A batch on one GPU with devices naming another is refused (no silent
    xGMI round trip); the same GPU repeated is the in-place partition."""
    codecs, dtype = _chains()["bitround_shuffle_crc32"]
    x = _make(dtype, 4, 4096, device, 40)
    other = torch.device("cuda", device.index + 1)
    with pytest.raises(ValueError, match="allow_peer_copy"):
        chunks.encode_chunks(codecs, x, devices=[device, other])
