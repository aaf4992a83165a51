"""Integer Delta and fused C4 decodes at scan-partition boundaries, and the
lab's single-pass scans (tools/lab/lab_scan1p.hip) on the GPU.

Same-width integer Delta decode (np.cumsum in the dtype, delta.py:69-83) and
the fused FixedScaleOffset <- Delta <- Shuffle decode (fixedscaleoffset.py:
99-113 after delta.py:80 after _shuffle.pyx:23-30) run in the product as
three-pass scans.  The single-pass alternative -- ONE launch holding 16-32 KiB
partitions in LDS across a decoupled look-back -- measured slower (DESIGN.md
§3) and lives in the lab library; it is kept byte-exact here because it is
the measured alternative.  Checked byte for byte against the oracle (numpy's
wrapping cumsum, the reference's codecs applied one by one):

* sizes on both sides of every partition boundary, one partition, thousands
  of partitions, the last partition partial (product decode);
* the lab single pass's persistent state: many calls in a row on one state,
  left zero after every call;
* its guard path: with a zero spin bound every partition whose predecessors
  have not all published derives its prefix from the data.
"""

import warnings

import numpy as np
import pytest
import torch

import oracle
from numcodecs_amd import Delta, FixedScaleOffset, Shuffle, _ops, batch
from numcodecs_amd._native import check
from tests.helpers import lab_lib

pytestmark = pytest.mark.gpu

RNG = np.random.default_rng(77)
# elements per single-pass partition: 32 KiB of i1/i2 deltas, 16 KiB of i4
PART = {1: 32768, 2: 16384, 4: 4096}
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


@pytest.mark.parametrize("dt", INT_DTYPES)
def test_lab_single_pass_partition_boundaries(device, dt):
    lab = lab_lib()
    es = np.dtype(dt).itemsize
    for n in _sizes(es):
        enc = _rand(dt, n)
        src = torch.from_numpy(enc).to(device)
        dst = torch.empty_like(src)
        state = torch.zeros(lab.mc_lab_delta_dec1p_state_bytes(n, es), dtype=torch.uint8, device=device)
        assert lab.mc_lab_delta_dec1p(src.data_ptr(), dst.data_ptr(), n, es, state.data_ptr(), 1 << 14, None,
                                      _ops.stream(src)) == 0
        assert dst.cpu().numpy().tobytes() == _cumsum(enc, dt).tobytes(), (dt, n)


@pytest.mark.parametrize("dt", ["|u1", "<i2", "<u4"])
def test_lab_single_pass_state_reuse(device, dt):
    """Twelve single-pass decodes in a row on one state, different sizes
    (more and fewer partitions than the previous call); after each the
    state's ticket/retire counters and status words are zero again."""
    lab = lab_lib()
    es = np.dtype(dt).itemsize
    state = torch.zeros(lab.mc_lab_delta_dec1p_state_bytes(PART[es] * 9 + 256, es), dtype=torch.uint8,
                        device=device)
    for rep in range(12):
        n = PART[es] * (1 + (rep * 7) % 9) + (16 // es) * rep
        assert lab.mc_lab_delta_dec1p_state_bytes(n, es) <= state.numel()
        enc = _rand(dt, n)
        src = torch.from_numpy(enc).to(device)
        dst = torch.empty_like(src)
        assert lab.mc_lab_delta_dec1p(src.data_ptr(), dst.data_ptr(), n, es, state.data_ptr(), 1 << 14, None,
                                      _ops.stream(src)) == 0
        assert dst.cpu().numpy().tobytes() == _cumsum(enc, dt).tobytes(), (dt, rep)
        w = state.view(torch.int32).cpu().numpy()
        assert w[0] == 0 and w[1] == 0 and not w[4:].any(), rep


@pytest.mark.parametrize("dt", ["|u1", "<i2", "<i4"])
def test_guard_path_prefix_from_data(device, dt):
    """Spin bound 0: partitions take the data-derived prefix whenever a
    predecessor has not published yet; the bytes must not change, the state
    counters and status words must still be left zero."""
    lab = lab_lib()
    es = np.dtype(dt).itemsize
    n = PART[es] * 23 + 16 // es
    enc = _rand(dt, n)
    src = torch.from_numpy(enc).to(device)
    dst = torch.empty_like(src)
    state = torch.zeros(lab.mc_lab_delta_dec1p_state_bytes(n, es), dtype=torch.uint8, device=device)
    for _ in range(2):
        assert lab.mc_lab_delta_dec1p(src.data_ptr(), dst.data_ptr(), n, es, state.data_ptr(), 0, None,
                                      _ops.stream(src)) == 0
        assert dst.cpu().numpy().tobytes() == _cumsum(enc, dt).tobytes()
        w = state.view(torch.int32).cpu().numpy()
        assert w[0] == 0 and w[1] == 0 and not w[4:].any()


def test_int_delta_decode_256mib_roundtrip(device):
    """BASELINE-size single chunk (256 MiB of i2 = 128 Mi elements):
    decode(encode(x)) == x, and the encoded chunk's decode equals numpy's
    cumsum."""
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
C4_PART = {"<i2": 16384, "<u2": 16384, "<i4": 8192, "<u4": 8192}


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
def test_c4_lab_single_pass_and_three_pass_agree(device, at):
    """The lab's single pass (default spin bound, and the guard path forced
    with spin bound 0), the three-pass scan through the lab (variant 1) and
    the product decode give the same bytes; the single pass leaves its state
    zero."""
    lab = lab_lib()
    dt = "<f4"
    codecs = _c4_chain(dt, at)
    n = C4_PART[at] * 17 + 16
    x = (1000.0 + RNG.uniform(-15, 15, n)).astype(dt)
    pipe = batch.FilterPipeline(codecs)
    enc = pipe.encode(torch.from_numpy(x).to(device)).view(torch.uint8).reshape(-1)
    ref = pipe.decode(enc).view(torch.uint8).reshape(-1)
    assert ref.cpu().numpy().tobytes() == _c4_ref(enc.cpu().numpy(), codecs).tobytes()
    _, _, sc3, off4 = batch._c4_scalars(*codecs)
    a, d = _ops.dtype_code(at), _ops.dtype_code(dt)
    out = torch.empty_like(ref)
    state = torch.zeros(lab.mc_lab_c4_dec1p_state_bytes(n, a), dtype=torch.uint8, device=device)
    for spins in (1 << 14, 0):
        out.zero_()
        assert lab.mc_lab_c4_dec1p(enc.data_ptr(), out.data_ptr(), n, a, d, sc3, off4, state.data_ptr(), spins,
                                   None, _ops.stream(enc)) == 0
        assert torch.equal(out, ref), spins
        w = state.view(torch.int32).cpu().numpy()
        assert w[0] == 0 and w[1] == 0 and not w[4:].any()
    ws = _ops.workspace(lab.mc_lab_c4_decode_workspace(n), enc)
    out.zero_()
    check(lab.mc_lab_c4_decode_variant(enc.data_ptr(), out.data_ptr(), n, a, d, sc3, off4, ws.data_ptr(),
                                       ws.numel(), 1, _ops.stream(enc)), "three-pass")
    assert torch.equal(out, ref)
