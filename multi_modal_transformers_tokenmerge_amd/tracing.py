"""roctx ranges around the phases of a training step (tracing row): MMT_ROCTX=1 turns
them on (torch.cuda.nvtx, which ROCm builds of PyTorch route to roctx); off, `phase` is a no-op.
Ranges are host-side markers: they bracket a phase's launches when the step runs eagerly
(bench.py --no-graph) and the capture of the step's graphs otherwise. Collect them with
`rocprofv3 --marker-trace --kernel-trace` (tools/roctx_summary.py joins the two traces)."""
from __future__ import annotations

import contextlib
import os

import torch

MODE = int(os.environ.get("MMT_ROCTX", "0") or 0)  # 1 ranges, 2 ranges + synchronize at each end
ENABLED = MODE > 0


@contextlib.contextmanager
def phase(name: str):
    """MMT_ROCTX=2 also synchronizes the device when a range closes, so an eager step's kernels
    run inside the range that launched them (per-phase GPU time; the side-stream overlap of the
    weight gradients is lost while measuring)."""
    if not ENABLED:
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        if MODE >= 2 and not torch.cuda.is_current_stream_capturing():
            torch.cuda.synchronize()
        torch.cuda.nvtx.range_pop()
