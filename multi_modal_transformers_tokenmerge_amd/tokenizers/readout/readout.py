"""Readout tokens, mirroring the reference's ``multi_modal_transformers/tokenizers/readout/readout.py``
(AddPositionEmbedding :8-33): ``inputs + pos_embedding`` with a learned (1, n, D) embedding,
applied by Octo to zeros of shape (B, n_obs * tokens_per_readout, D) (octo.py:103-108).

In the training step the add is fused into the sequence assembly kernel (mmt_seq_assemble_fwd);
this module is the standalone form of the same operation on the device (mmt_add_position_embedding,
backward: identity for the input, column sums over the batch for the embedding).
"""
from __future__ import annotations

import torch

from ... import _C
from ...module_api import Bindable, init_from_spec, spec
from ...params import ParamStore


class AddPositionEmbedding(Bindable):
    """``AddPositionEmbedding(posemb_init)(inputs)`` (readout.py:8-33; the same module is
    attention.py:71-85) for inputs (B, n, D) fp32 device tensors. The parameter ``pos_embedding``
    has the shape (n, D) of the first call (the reference's (1, n, D) without the broadcast axis)
    or of ``bind(store, name, n, D)``; posemb_init is the config's initializer node (he_normal in
    model_configs/tokenizers/readouts/octo.yaml), a LayerSpec, or a ParamStore initialiser."""

    def __init__(self, posemb_init=None):
        self.posemb_init = spec(posemb_init)
        self.pe = None
        self.num_tokens = self.D = None

    def _declare(self, store: ParamStore, name: str, num_tokens: int, embedding_dim: int):
        self.num_tokens, self.D = int(num_tokens), int(embedding_dim)
        self.pe = store.add(f"{name}/pos_embedding", (self.num_tokens, self.D),
                            init_from_spec(self.posemb_init, (1, self.num_tokens, self.D)))

    def _check(self, inputs: torch.Tensor):
        if inputs.dim() != 3:  # the reference asserts inputs.ndim == 3 (:28-30)
            raise ValueError(f"Number of dimensions should be 3, but it is: {inputs.dim()}")
        if tuple(inputs.shape[1:]) != (self.num_tokens, self.D):
            raise ValueError(f"inputs {tuple(inputs.shape)} do not match the embedding "
                             f"({self.num_tokens}, {self.D})")
        if inputs.dtype != torch.float32 or not inputs.is_cuda or not inputs.is_contiguous():
            raise ValueError("inputs must be a contiguous fp32 device tensor")

    def __call__(self, inputs: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if inputs.dim() != 3:
            raise ValueError(f"Number of dimensions should be 3, but it is: {inputs.dim()}")
        self._ensure(inputs.device, inputs.shape[1], inputs.shape[2])
        self._check(inputs)
        out = torch.empty_like(inputs) if out is None else out
        B = inputs.shape[0]
        _C.call("mmt_add_position_embedding", _C.ptr(inputs), _C.ptr(self.pe.data), _C.ptr(out), B,
                self.num_tokens, self.D, _C.stream_ptr())
        return out

    def backward(self, dout: torch.Tensor) -> torch.Tensor:
        """Accumulates d(pos_embedding) into the flat gradient buffer; returns d(inputs) = dout."""
        B = dout.shape[0]
        d2 = dout.reshape(B, self.num_tokens * self.D)
        _C.call("mmt_colsum", _C.ptr(d2), 0, d2.stride(0), B, self.num_tokens * self.D,
                _C.ptr(self.pe.grad), _C.stream_ptr())
        return dout
