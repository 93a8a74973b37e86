"""Categorical action head, mirroring the reference's ``action_heads/categorical.py:12-41``
(``assign_bins``: uniform ``linspace`` edges + ``jnp.digitize``; ``CategoricalActionHead``: the
readouts regrouped "batch (action timestep) embeddings -> batch action timestep embeddings",
averaged over timestep, Dense to ``num_bins`` logits) and ``Octo.compute_ce_loss``
(models/octo/octo.py:187-198: ``one_hot(assign_bins(...), num_bins)`` +
``optax.softmax_cross_entropy``) averaged as ``categorical_train_step`` does (:292-302).
SURVEY §8f row 4.

The reference's off-by-one is kept: ``digitize`` returns 1..num_bins for in-range actions and
``one_hot(num_bins, num_bins)`` is all zero, so actions in the top bin (and >= max_action) carry
no loss, and the lowest bin's actions train class 1.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _C, _kernels as K
from ..layers import Dense
from ..params import ParamStore


def assign_bins(input_data: np.ndarray, bounds, num_bins: int, bin_strategy: str = "uniform"):
    """Reference categorical.py:12-22 (host helper, float32 edges like jnp.linspace)."""
    if bin_strategy != "uniform":
        raise NotImplementedError
    bins = np.linspace(bounds[0], bounds[1], num_bins + 1, dtype=np.float32)
    return np.digitize(np.asarray(input_data, dtype=np.float32), bins)


class CategoricalActionHead:
    def __init__(self, store: ParamStore, name: str, embedding_dim: int, action_dim: int,
                 num_bins: int, max_action: float):
        self.D, self.A, self.num_bins, self.max_action = embedding_dim, action_dim, num_bins, float(max_action)
        self.dense = Dense(store, f"{name}/Dense_0", embedding_dim, num_bins)
        self._edges = {}

    def edges(self, device) -> torch.Tensor:
        if device not in self._edges:
            e = np.linspace(-self.max_action, self.max_action, self.num_bins + 1, dtype=np.float32)
            self._edges[device] = torch.from_numpy(e).to(device)
        return self._edges[device]

    def forward(self, group_means: torch.Tensor) -> torch.Tensor:
        """(B, A, D) bf16 per-action readout means -> logits (B, A, num_bins) fp32 (:38-40)."""
        B = group_means.shape[0]
        z = self.dense.fwd(group_means.reshape(B * self.A, self.D), out_mode=K.OUT_F32)
        return z.view(B, self.A, self.num_bins)

    def loss_forward(self, group_means: torch.Tensor, actions: torch.Tensor):
        """mean over (b, a) of softmax_cross_entropy(logits, one_hot(assign_bins(actions)))."""
        B = group_means.shape[0]
        if tuple(actions.shape) != (B, self.A) or actions.dtype != torch.float32 \
                or not actions.is_contiguous():
            raise ValueError(f"actions must be contiguous fp32 ({B}, {self.A})")
        x = group_means.reshape(B * self.A, self.D)
        z = self.dense.fwd(x, out_mode=K.OUT_F32)
        R = B * self.A
        loss = torch.zeros(1, dtype=torch.float32, device=z.device)
        dz = torch.empty((R, self.num_bins), dtype=torch.bfloat16, device=z.device)
        e = self.edges(z.device)
        _C.call("mmt_action_head", 1, _C.ptr(z), z.stride(0), R, self.num_bins, _C.ptr(actions),
                _C.ptr(e), e.numel(), self.max_action, 1.0 / R, None, _C.ptr(loss), _C.ptr(dz),
                _C.stream_ptr())
        return loss, dict(x=x, dz=dz, B=B)

    def loss_backward(self, sv: dict) -> torch.Tensor:
        """Returns d(group means) (B, A, D) bf16."""
        return self.dense.bwd(sv["dz"], sv["x"]).view(sv["B"], self.A, self.D)
