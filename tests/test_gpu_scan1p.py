"""Single-pass integer scans (csrc/mc_scan1p.hip) on the GPU.

Same-width integer Delta decode (np.cumsum in the dtype, delta.py:69-83) and
the fused FixedScaleOffset <- Delta <- Shuffle decode (fixedscaleoffset.py:
99-113 after delta.py:80 after _shuffle.pyx:23-30) now run as ONE launch that
holds 64 KiB partitions in LDS across a decoupled look-back.  Checked here,
byte for byte against the oracle (numpy's wrapping cumsum, the reference's
codecs applied one by one):

* sizes on both sides of every partition boundary, one partition, thousands
  of partitions, the last partition partial;
* the persistent per-stream state: many calls in a row on one state, two
  streams at once, the state left zero after every call;
* both entry points (the _state one with the persistent state, the plain
  one that zeroes its workspace itself, as HIP-graph capture uses);
* the guard path: with a zero spin bound (lab library) every partition whose
  predecessors have not all published derives its prefix from the data.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, _ops, batch
from numcodecs_amd._native import check, lib
from tests.helpers import lab_lib

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(77)
# elements per partition: 64 KiB of i1/i2 deltas, 32 KiB of i4 deltas
PART = {1: 65536, 2: 32768, 4: 8192}
INT_DTYPES = ["|i1", "|u1", "<i2", "<u2", "<i4", "<u4"]


def _sizes(es):
    e = PART[es]
    unit = 16 // es
    return [unit, 4 * unit, e - unit, e, e + unit, 3 * e + 5 * unit, 37 * e + 16 * unit]


def _rand(dt, n):
    dt = np.dtype(dt)
    info = np.iinfo(dt)
    return RNG.integers(info.min, info.max, n, dtype=dt, endpoint=True)


def _cumsum(enc, dt):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return oracle.delta_decode(enc, dt)


@pytest.mark.parametrize("dt", INT_DTYPES)
def test_int_delta_decode_partition_boundaries(device, dt):
    es = np.dtype(dt).itemsize
    for n in _sizes(es):
        enc = _rand(dt, n)
        got = Delta(dt).decode(torch.from_numpy(enc).to(device)).cpu().numpy()
        assert got.tobytes() == _cumsum(enc, dt).tobytes(), (dt, n)


@pytest.mark.parametrize("dt", ["|u1", "<i2", "<u4"])
def test_state_reuse_and_left_zero(device, dt):
    """Twelve decodes in a row on the stream's persistent state, different
    sizes (more and fewer partitions than the previous call); after each the
    state's ticket/retire counters and status words are zero again."""
    es = np.dtype(dt).itemsize
    codec = Delta(dt)
    for rep in range(12):
        n = PART[es] * (1 + (rep * 7) % 9) + (16 // es) * rep
        enc = _rand(dt, n)
        got = codec.decode(torch.from_numpy(enc).to(device)).cpu().numpy()
        assert got.tobytes() == _cumsum(enc, dt).tobytes(), (dt, rep)
        st = _ops._STATES[(device.index, _ops.stream(torch.empty(0, device=device)))]
        words = st.view(torch.int32).cpu().numpy()
        nparts = -(-n * es // (PART[es] * es))
        assert words[0] == 0 and words[1] == 0, rep
        assert not words[4:4 + 2 * nparts].any(), rep


def test_two_streams_at_once(device):
    """Two streams, each with its own state, decoding concurrently."""
    s1, s2 = torch.cuda.Stream(device), torch.cuda.Stream(device)
    n = PART[2] * 40 + 8
    a, b = _rand("<i2", n), _rand("<i2", n)
    da, db = torch.from_numpy(a).to(device), torch.from_numpy(b).to(device)
    torch.cuda.synchronize()
    outs = {}
    for rep in range(4):
        with torch.cuda.stream(s1):
            outs[("a", rep)] = Delta("<i2").decode(da)
        with torch.cuda.stream(s2):
            outs[("b", rep)] = Delta("<i2").decode(db)
    torch.cuda.synchronize()
    ra, rb = _cumsum(a, "<i2").tobytes(), _cumsum(b, "<i2").tobytes()
    for rep in range(4):
        assert outs[("a", rep)].cpu().numpy().tobytes() == ra
        assert outs[("b", rep)].cpu().numpy().tobytes() == rb


@pytest.mark.parametrize("dt", ["|i1", "<u2", "<i4"])
def test_plain_entry_zeroes_its_workspace(device, dt):
    """mc_delta_decode (no persistent state): the single pass runs on the
    workspace's leading bytes, zeroed by the call itself -- a workspace full
    of garbage must not matter."""
    es = np.dtype(dt).itemsize
    n = PART[es] * 5 + 3 * (16 // es)
    enc = _rand(dt, n)
    src = torch.from_numpy(enc).to(device)
    dst = torch.empty_like(src)
    code = _ops.dtype_code(dt)
    ws = torch.full((lib.mc_delta_decode_workspace(n, code, code),), 0xA5, dtype=torch.uint8, device=device)
    for _ in range(2):
        check(lib.mc_delta_decode(src.data_ptr(), dst.data_ptr(), n, code, code, ws.data_ptr(), ws.numel(),
                                  _ops.stream(src)), "mc_delta_decode")
        assert dst.cpu().numpy().tobytes() == _cumsum(enc, dt).tobytes()


@pytest.mark.parametrize("dt", ["|u1", "<i2", "<i4"])
def test_guard_path_prefix_from_data(device, dt):
    """Spin bound 0 (lab): partitions take the data-derived prefix whenever a
    predecessor has not published yet; the bytes must not change, the state
    counters and status words must still be left zero."""
    lab = lab_lib()
    es = np.dtype(dt).itemsize
    n = PART[es] * 23 + 16 // es
    enc = _rand(dt, n)
    src = torch.from_numpy(enc).to(device)
    dst = torch.empty_like(src)
    state = torch.zeros(lib.mc_delta_decode_state_bytes(n, _ops.dtype_code(dt), _ops.dtype_code(dt)),
                        dtype=torch.uint8, device=device)
    for _ in range(2):
        assert lab.mc_lab_delta_dec1p(src.data_ptr(), dst.data_ptr(), n, es, state.data_ptr(), 0,
                                      _ops.stream(src)) == 0
        assert dst.cpu().numpy().tobytes() == _cumsum(enc, dt).tobytes()
        w = state.view(torch.int32).cpu().numpy()
        assert w[0] == 0 and w[1] == 0 and not w[4:].any()


def test_int_delta_decode_256mib_roundtrip(device):
    """BASELINE-size single chunk (256 MiB of i2 = 128 Mi elements, 4096
    partitions): decode(encode(x)) == x, and the encoded chunk's decode
    equals numpy's cumsum."""
    n = 128 << 20
    x = torch.randint(-32768, 32768, (n,), dtype=torch.int16, device=device)
    d = Delta("<i2")
    enc = d.encode(x)
    assert torch.equal(d.decode(enc), x)
    e = enc.cpu().numpy()
    assert d.decode(enc).cpu().numpy().tobytes() == _cumsum(e, "<i2").tobytes()


# ---------------------------------------------------------------------------
# fused FSO <- Delta <- Shuffle decode
# ---------------------------------------------------------------------------
C4_PART = {"<i2": 32768, "<u2": 32768, "<i4": 16384, "<u4": 16384}


def _c4_chain(dt, at):
    scale = 1e3 if np.dtype(at).itemsize == 2 else 1e6
    return [FixedScaleOffset(offset=1000, scale=scale, dtype=dt, astype=at), Delta(dtype=at),
            Shuffle(np.dtype(at).itemsize)]


def _c4_ref(enc_bytes, codecs):
    fso, dl, sh = codecs
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        u = oracle.unshuffle(enc_bytes, sh.elementsize)
        c = oracle.delta_decode(u, dl.dtype)
        return oracle.fso_decode(c, fso.offset, fso.scale, fso.dtype, fso.astype)


@pytest.mark.parametrize("dt", ["<f4", "<f8"])
@pytest.mark.parametrize("at", ["<i2", "<u2", "<i4", "<u4"])
def test_c4_decode_partition_boundaries(device, dt, at):
    e = C4_PART[at]
    codecs = _c4_chain(dt, at)
    pipe = batch.FilterPipeline(codecs)
    for n in (16, e - 16, e, e + 16, 3 * e + 48, 11 * e + 32):
        x = (1000.0 + RNG.uniform(-15, 15, n)).astype(dt)
        enc = pipe.encode(torch.from_numpy(x).to(device))
        got = pipe.decode(enc).cpu().numpy()
        ref = _c4_ref(enc.cpu().numpy(), codecs)
        assert got.tobytes() == ref.tobytes(), (dt, at, n)


@pytest.mark.parametrize("at", ["<i2", "<u4"])
def test_c4_guard_path_and_three_pass_agree(device, at):
    """The single pass with the guard path forced (spin bound 0), the
    product's three-pass scan (lab variant 1) and the default decode give the
    same bytes."""
    lab = lab_lib()
    dt = "<f4"
    codecs = _c4_chain(dt, at)
    n = C4_PART[at] * 17 + 16
    x = (1000.0 + RNG.uniform(-15, 15, n)).astype(dt)
    pipe = batch.FilterPipeline(codecs)
    enc = pipe.encode(torch.from_numpy(x).to(device)).view(torch.uint8).reshape(-1)
    ref = pipe.decode(enc).view(torch.uint8).reshape(-1)
    _, _, sc3, off4 = batch._c4_scalars(*codecs)
    a, d = _ops.dtype_code(at), _ops.dtype_code(dt)
    out = torch.empty_like(ref)
    state = torch.zeros(lib.mc_fso_delta_shuffle_decode_state_bytes(n, a), dtype=torch.uint8, device=device)
    assert lab.mc_lab_c4_dec1p(enc.data_ptr(), out.data_ptr(), n, a, d, sc3, off4, state.data_ptr(), 0,
                               _ops.stream(enc)) == 0
    assert torch.equal(out, ref)
    w = state.view(torch.int32).cpu().numpy()
    assert w[0] == 0 and w[1] == 0 and not w[4:].any()
    ws = _ops.workspace(lab.mc_lab_c4_decode_workspace(n), enc)
    out.zero_()
    check(lab.mc_lab_c4_decode_variant(enc.data_ptr(), out.data_ptr(), n, a, d, sc3, off4, ws.data_ptr(),
                                       ws.numel(), 1, _ops.stream(enc)), "three-pass")
    assert torch.equal(out, ref)
