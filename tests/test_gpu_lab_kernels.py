"""The round-4 lab schedules that lost their A/B (tools/lab: lab_shuffle4.hip,
lab_chain.hip, the batched variant entry point) stay byte-identical to the
oracle, so their measurements in profiles/r04 compare correct kernels."""

import numpy as np
import pytest
import torch

import oracle
from tests.helpers import lab_lib

pytestmark = pytest.mark.gpu


def test_lab_shuffle4_encode_kinds(device):
    """Every Shuffle(4) encode schedule of lab_shuffle4.hip (register / quad-
    major / XCD or spread tile orders / LDS-DMA / 16-B quad-lane stores /
    rotated plane order / temporal accesses; kind 7 is the no-transpose
    access pattern and is skipped) against the oracle on 8 MiB."""
    lab = lab_lib()
    st = torch.cuda.current_stream().cuda_stream
    n = 8 << 20
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=device)
    ref = oracle.shuffle(x.cpu().numpy(), 4)
    for kind in [k for k in range(20) if k != 7]:
        y = torch.zeros_like(x)
        assert lab.mc_lab_shuffle4_enc(x.data_ptr(), y.data_ptr(), n, kind, st) == 0, kind
        assert np.array_equal(y.cpu().numpy(), ref), kind


@pytest.mark.parametrize("es", [4, 8])
def test_lab_shuffle_batch_variants(device, es):
    """The batched entry point with explicit layouts (profiles/r04
    probe_batch_variants*.json) against the oracle row by row."""
    lab = lab_lib()
    st = torch.cuda.current_stream().cuda_stream
    rows, m = 6, (1 << 20) + 4096
    x = torch.randint(0, 256, (rows, m), dtype=torch.uint8, device=device)
    xh = x.cpu().numpy()
    for v, cap in [(0, 0), (513, 0), (129, 0), (21, 0), (5, 0), (1, 0), (133, 0), (513, 1024), (81, 1024),
                   (6, 0), (22, 0)]:
        if (v & 7) == 6 and es != 8:
            continue
        y = torch.zeros_like(x)
        assert lab.mc_lab_shuffle_batch_variant(x.data_ptr(), m, y.data_ptr(), m, rows, m, es, 1, v, cap, st) == 0
        yh = y.cpu().numpy()
        for r in range(rows):
            assert np.array_equal(yh[r], oracle.shuffle(xh[r], es)), (es, v, cap, r)


def test_lab_chain_kinds_write_numpy_cumsum(device):
    """The chain schedules that store their results (tools/probe_chain.py)
    write numpy's float32 cumsum of their input, bit for bit."""
    lab = lab_lib()
    st = torch.cuda.current_stream().cuda_stream
    n = 8192
    init = torch.arange(64, device=device, dtype=torch.float32) * 1e-3
    out = torch.empty(4, device=device)
    cyc = torch.zeros(2, dtype=torch.int64, device=device)
    gin = torch.randn(n, device=device)
    want = np.cumsum(gin.cpu().numpy())
    # (14, 24, 25 chain over their LDS init, not gin; 21 / 22 store each group
    # one group late -- round 4 left the last group unstored, fixed in round 5)
    for kind in (13, 15, 16, 17, 18, 20, 21, 22, 23):
        gout = torch.zeros(n, device=device)
        assert lab.mc_lab_chain_g(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, 1, kind, gin.data_ptr(),
                                  gout.data_ptr(), st) == 0
        torch.cuda.synchronize()
        assert np.array_equal(gout.cpu().numpy().view(np.uint32), want.view(np.uint32)), kind


def test_lab_chain64_kinds_write_numpy_cumsum(device):
    """The f64 chain schedules that store (kinds 42-44) write numpy's float64
    cumsum of their input, bit for bit."""
    lab = lab_lib()
    st = torch.cuda.current_stream().cuda_stream
    n = 4096
    init = torch.arange(64, device=device, dtype=torch.float64) * 1e-3
    out = torch.empty(4, device=device, dtype=torch.float64)
    cyc = torch.zeros(2, dtype=torch.int64, device=device)
    gin = torch.randn(n, device=device, dtype=torch.float64)
    want = np.cumsum(gin.cpu().numpy())
    for kind in (42, 43, 44):
        gout = torch.zeros(n, device=device, dtype=torch.float64)
        assert lab.mc_lab_chain64(init.data_ptr(), out.data_ptr(), cyc.data_ptr(), n, 1, kind, gin.data_ptr(),
                                  gout.data_ptr(), st) == 0
        torch.cuda.synchronize()
        assert np.array_equal(gout.cpu().numpy().view(np.uint64), want.view(np.uint64)), kind
