"""HIP-graph captured chunk pipelines (launch-bound inner loops).

A Zarr chain (filters + checksum) over a small batch of chunks is a handful
of short kernels; issued one by one from Python each costs ~10-15 us of host
time, far more than the kernel itself.  :class:`GraphChain` captures the
whole encode or decode of a fixed-shape device batch
(:func:`numcodecs_amd.chunks.encode_chunks` / ``decode_chunks``) into one HIP
graph (``torch.cuda.CUDAGraph``: hipStreamBeginCapture on the capture
stream, every ``libmcodec`` launch lands on that stream) and replays it with
one launch: same bytes, a fraction of the host cost.

Restrictions (all checked at capture time by the eager warm-up run): the
chain must not synchronise the host inside encode/decode, so checksum
verification is deferred -- :meth:`GraphChain.__call__` replays, then checks
the checksums captured in the graph and raises the codec's RuntimeError --
and Delta chains whose astype cannot hold every dtype value (which replay
numpy's first-element assignment on the host, delta.py:63) are refused.
"""

from __future__ import annotations

import numpy as np
import torch

from . import chunks
from .delta import Delta

__all__ = ["GraphChain"]


class GraphChain:
    """Capture ``codecs`` (encode order) applied to a [B, ...] device batch
    shaped like `example`, in `direction` "encode" or "decode".

    >>> g = GraphChain([BitRound(10), Shuffle(4), CRC32()], x_example)   # doctest: +SKIP
    >>> enc = g(x)            # x: same shape/dtype/device as x_example  # doctest: +SKIP
    """

    def __init__(self, codecs, example: torch.Tensor, direction: str = "encode", warmup: int = 2):
        if direction not in ("encode", "decode"):
            raise ValueError("direction must be 'encode' or 'decode'")
        if not (isinstance(example, torch.Tensor) and example.device.type == "cuda" and example.dim() >= 1):
            raise TypeError("example must be a device tensor [B, ...]")
        self.codecs = list(codecs)
        for c in self.codecs:
            if isinstance(c, Delta) and direction == "encode" and not np.can_cast(c.dtype, c.astype, "safe"):
                raise ValueError(f"{c!r}: the first-element check syncs the host and cannot be captured")
        self.direction = direction
        self.input = torch.empty_like(example)
        self.input.copy_(example)
        self._pending = []
        dev = example.device
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # eager warm-up: allocator pools, lazy init
            for _ in range(max(1, warmup)):
                self._pending.clear()
                self._run()
        torch.cuda.current_stream(dev).wait_stream(side)
        self._pending.clear()
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph):
                self.output = self._run()
        except RuntimeError as e:  # e.g. a host round trip inside the chain
            raise ValueError(f"this chain cannot be captured in a HIP graph: {e}") from e
        self._checks = list(self._pending)

    def _run(self):
        if self.direction == "encode":
            return chunks.encode_chunks(self.codecs, self.input)
        return chunks.decode_chunks(self.codecs, self.input, self._pending)

    def __call__(self, x: "torch.Tensor | None" = None) -> torch.Tensor:
        """Replay on `x` (copied into the captured input buffer; pass None to
        replay on whatever was written into :attr:`input`).  Returns the
        captured output buffer, overwritten by the next call."""
        if x is not None:
            if x.shape != self.input.shape or x.dtype != self.input.dtype:
                raise ValueError(f"expected {tuple(self.input.shape)} {self.input.dtype}")
            self.input.copy_(x)
        self.graph.replay()
        for c, sums, stored in self._checks:  # deferred checksum verification
            chunks._raise_first(c, sums, stored)
        return self.output
