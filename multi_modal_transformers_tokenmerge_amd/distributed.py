"""Data-parallel training over the GPUs of one node (one process per GPU, torch.distributed with
the "nccl" backend = RCCL over xGMI on ROCm).

The reference has no distributed code at all. Design here:
  * samples are independent (sequence LayerNorm, GroupNorm and ToMe are per sample), so the
    global batch is sharded: rank r owns global samples [r*B, (r+1)*B), and every random stream
    is keyed by the GLOBAL sample index (``sample_offset``), so N ranks x B reproduce 1 rank x N*B;
  * the only exchange is the gradient all-reduce over the flat fp32 gradient buffer, issued as a
    few large contiguous buckets (xGMI rings are per-link bound: few, large collectives); the
    1/N average is folded into the AdamW kernel's grad_scale instead of a separate pass;
  * the attention-dropout mask is keyed by (seed, step, layer) only, identical on every rank
    (Flax broadcasts it over the batch).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


def init_from_env(backend: str | None = None) -> DistInfo:
    """Initialise the process group from torchrun's environment (RANK/WORLD_SIZE/LOCAL_RANK/
    MASTER_ADDR/MASTER_PORT). Single process when WORLD_SIZE is unset or 1."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return DistInfo()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:  # MMT_DIST_BACKEND=gloo: CPU-transport rehearsal of the multi-rank path
        backend = os.environ.get("MMT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return DistInfo(rank, ws, local)


class GradAllReducer:
    """All-reduce (SUM) of the flat gradient buffer in ``bucket_bytes`` contiguous slices.
    The average is applied by AdamW's grad_scale = 1 / world_size."""

    def __init__(self, world_size: int, bucket_bytes: int = 64 << 20, group=None):
        self.world_size = world_size
        self.bucket_elems = max(1, bucket_bytes // 4)
        self.group = group

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world_size

    def __call__(self, flat_grad: torch.Tensor):
        if self.world_size <= 1:
            return
        n = flat_grad.numel()
        for s in range(0, n, self.bucket_elems):
            dist.all_reduce(flat_grad[s:s + self.bucket_elems], op=dist.ReduceOp.SUM, group=self.group)
