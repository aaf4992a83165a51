"""In-process multi-GPU dispatch, host logic (CPU only): the row partition
(contiguous, covering, in row order -- shard.chunk_range) and
the worker runner's ordering and error rules (numcodecs_amd.multi)."""

import threading

import pytest

from numcodecs_amd import multi


@pytest.mark.parametrize("nrows,ndev", [(8192, 8), (7, 2), (7, 3), (1, 4), (0, 2), (5, 5), (11, 3)])
def test_split_rows_covers_in_order(nrows, ndev):
    parts = multi.split_rows(nrows, ndev)
    rows = [r for _, lo, hi in parts for r in range(lo, hi)]
    assert rows == list(range(nrows))
    assert all(hi > lo for _, lo, hi in parts)
    assert [g for g, _, _ in parts] == sorted(g for g, _, _ in parts)
    sizes = [hi - lo for _, lo, hi in parts]
    assert not sizes or max(sizes) - min(sizes) <= 1
    assert len(parts) == min(nrows, ndev)


def test_run_workers_order_threads_and_first_error():
    seen = set()

    def mk(i):
        def f():
            seen.add(threading.get_ident())
            return i * i
        return f

    assert multi.run_workers([mk(i) for i in range(5)]) == [0, 1, 4, 9, 16]
    done = []

    def ok():
        done.append(1)
        return 1

    def bad(msg):
        def f():
            raise RuntimeError(msg)
        return f

    with pytest.raises(RuntimeError, match="first"):
        multi.run_workers([ok, bad("first"), ok, bad("second")])
    assert len(done) == 2  # every worker ran to the end before the raise


def test_normalize_devices_rejects_cpu():
    with pytest.raises(ValueError):
        multi.normalize_devices(["cpu"])
    with pytest.raises(ValueError):
        multi.normalize_devices([])
    import torch

    assert multi.normalize_devices([0, "cuda:1", torch.device("cuda", 2)]) == [
        torch.device("cuda", 0), torch.device("cuda", 1), torch.device("cuda", 2)]


def test_peer_devices_refused_unless_allowed():
    """A one-device batch naming other GPUs is refused:
    shipping rows over xGMI and back is opt-in; the batch's own GPU repeated
    is the in-place partition."""
    import torch

    home = torch.device("cuda", 0)
    assert multi.check_peer_devices(home, [home, home], False) is False
    with pytest.raises(ValueError, match="allow_peer_copy"):
        multi.check_peer_devices(home, [home, torch.device("cuda", 1)], False)
    assert multi.check_peer_devices(home, [torch.device("cuda", 1)], True) is True


def test_split_rows_partition_matches_shard():
    """Every row in exactly one worker's range, in order (shard.chunk_range)."""
    from numcodecs_amd import shard

    for nrows in (0, 1, 7, 8, 8193):
        for ndev in (1, 2, 3, 8):
            parts = multi.split_rows(nrows, ndev)
            rows = [r for _, lo, hi in parts for r in range(lo, hi)]
            assert rows == list(range(nrows))
            assert all(shard.chunk_range(nrows, g, ndev) == (lo, hi) for g, lo, hi in parts)
