"""HIP-graph captured chains (numcodecs_amd.graphs.GraphChain): every row of
a replayed encode/decode must equal the ORACLE's codecs applied one after
another to that chunk (tests/oracle_chain.py), for new inputs written into
the captured buffer, and deferred checksum verification must still raise
the codec's error."""

import pytest
import torch

from numcodecs_amd import (
    CRC32, CRC32C, Adler32, BitRound, Delta, FixedScaleOffset, Fletcher32, Quantize, Shuffle, chunks,
)
from numcodecs_amd.graphs import GraphChain
from tests import oracle_chain

pytestmark = pytest.mark.gpu


def _chains():
    return {
        "bitround_shuffle_crc32": ([BitRound(10), Shuffle(4), CRC32()], torch.float32),
        "fso_delta_shuffle_adler32": ([FixedScaleOffset(offset=1000, scale=1e3, dtype="<f4", astype="<i2"),
                                       Delta(dtype="<i2"), Shuffle(2), Adler32(location="end")], torch.float32),
        "quantize_shuffle_fletcher32": ([Quantize(3, "<f8", "<f4"), Shuffle(4), Fletcher32()], torch.float64),
        "delta_shuffle_crc32c": ([Delta(dtype="<i4"), Shuffle(4), CRC32C()], torch.int32),
    }


def _make(dtype, b, n, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    if dtype == torch.int32:
        return torch.randint(-1000, 1000, (b, n), generator=g, device=device, dtype=torch.int32)
    return (1000 + 10 * torch.rand((b, n), generator=g, device=device)).to(dtype)


@pytest.mark.parametrize("name", list(_chains()))
def test_graph_chain_vs_oracle(device, name):
    codecs, dtype = _chains()[name]
    b = 16
    x0 = _make(dtype, b, 16384, device, 1)
    genc = GraphChain(codecs, x0, "encode")
    for seed in (2, 3):  # replays on new data
        x = _make(dtype, b, 16384, device, seed)
        xh = x.cpu().numpy()
        got = genc(x).contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
        for i in range(b):
            assert got[i].tobytes() == oracle_chain.chain_encode(codecs, xh[i]), (name, seed, i)
    enc = torch.from_numpy(got.copy()).to(device)
    gdec = GraphChain(codecs, enc, "decode")
    dgot = gdec(enc).contiguous().view(torch.uint8).reshape(b, -1).cpu().numpy()
    for i in range(b):
        assert dgot[i].tobytes() == oracle_chain.chain_decode(codecs, got[i].tobytes()), (name, i)


def test_graph_decode_detects_corruption(device):
    codecs, dtype = _chains()["bitround_shuffle_crc32"]
    x = _make(dtype, 8, 4096, device, 4)
    enc = chunks.encode_chunks(codecs, x).clone()
    g = GraphChain(codecs, enc, "decode")
    g(enc)  # clean
    bad = enc.clone()
    bad.view(torch.uint8)[5, 77] ^= 1
    with pytest.raises(RuntimeError, match="crc32"):
        g(bad)


def test_graph_refuses_host_sync(device):
    x = torch.zeros((4, 1024), dtype=torch.int64, device=device)
    with pytest.raises(ValueError):
        GraphChain([Delta(dtype="<i8", astype="<i4")], x, "encode")


def test_raw_stream_handle_matches_torch(device):
    """_ops.stream reads the raw hipStream_t from torch's C++ side; it must be
    the handle torch.cuda.current_stream reports, on the default and on a
    side stream."""
    from numcodecs_amd import _ops

    x = torch.zeros(4, device=device)
    assert _ops.stream(x) == torch.cuda.current_stream(device).cuda_stream
    s = torch.cuda.Stream(device=device)
    with torch.cuda.stream(s):
        assert _ops.stream(x) == s.cuda_stream
