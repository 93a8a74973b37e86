"""Continuous action head, mirroring the reference's ``action_heads/continuous.py:12-26``
(``ContinuousActionHead``: mean over the readouts, Dense, ``tanh(mean / max_action) * max_action``)
and the L2 objective of ``Octo.compute_l2_loss`` (models/octo/octo.py:167-174) averaged over the
batch as ``continuous_train_step`` does (:252-262). SURVEY §8f row 4.

Device path: the readout mean comes from the backbone's fused rows-mean kernel, the Dense is the
library GEMM (fp32 output), and one kernel (``mmt_action_head`` kind 0) applies the tanh squash,
the loss and its gradient.
"""
from __future__ import annotations

import torch

from .. import _C, _kernels as K
from ..layers import Dense
from ..params import ParamStore


class ContinuousActionHead:
    def __init__(self, store: ParamStore, name: str, embedding_dim: int, action_dim: int,
                 max_action: float):
        self.D, self.A, self.max_action = embedding_dim, action_dim, float(max_action)
        self.dense = Dense(store, f"{name}/Dense_0", embedding_dim, action_dim)

    def forward(self, readout_mean: torch.Tensor) -> torch.Tensor:
        """(B, D) bf16 -> actions (B, 1, A) fp32 (:23-26)."""
        z = self.dense.fwd(readout_mean, out_mode=K.OUT_F32)
        B = z.shape[0]
        pred = torch.empty((B, self.A), dtype=torch.float32, device=z.device)
        _C.call("mmt_action_head", 0, _C.ptr(z), z.stride(0), B, self.A, None, None, 0,
                self.max_action, 1.0, _C.ptr(pred), None, None, _C.stream_ptr())
        return pred.view(B, 1, self.A)

    def loss_forward(self, readout_mean: torch.Tensor, actions: torch.Tensor):
        """mean_b sum_a (pred - actions)^2 (octo.py:171-174, :262). Returns (loss (1,), saved)."""
        z = self.dense.fwd(readout_mean, out_mode=K.OUT_F32)
        B = z.shape[0]
        if tuple(actions.shape) != (B, self.A) or actions.dtype != torch.float32 \
                or not actions.is_contiguous():
            raise ValueError(f"actions must be contiguous fp32 ({B}, {self.A})")
        loss = torch.zeros(1, dtype=torch.float32, device=z.device)
        dz = torch.empty((B, self.A), dtype=torch.bfloat16, device=z.device)
        _C.call("mmt_action_head", 0, _C.ptr(z), z.stride(0), B, self.A, _C.ptr(actions), None, 0,
                self.max_action, 1.0 / B, None, _C.ptr(loss), _C.ptr(dz), _C.stream_ptr())
        return loss, dict(x=readout_mean, dz=dz)

    def loss_backward(self, sv: dict) -> torch.Tensor:
        """Returns d(readout mean) (B, D) bf16."""
        return self.dense.bwd(sv["dz"], sv["x"])
