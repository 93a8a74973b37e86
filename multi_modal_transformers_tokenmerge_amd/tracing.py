"""roctx ranges around the phases of a training step (tracing row): MMT_ROCTX=1 turns
them on (torch.cuda.nvtx, which ROCm builds of PyTorch route to roctx); off, `phase` is a no-op.
Ranges are host-side markers: they bracket a phase's launches when the step runs eagerly
(bench.py --no-graph) and the capture of the step's graphs otherwise. Collect them with
`rocprofv3 --marker-trace --kernel-trace` (tools/roctx_summary.py joins the two traces)."""
from __future__ import annotations

import contextlib
import os

import torch

ENABLED = os.environ.get("MMT_ROCTX", "0") == "1"


@contextlib.contextmanager
def phase(name: str):
    if not ENABLED:
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
