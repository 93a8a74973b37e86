"""Token compression (ToMe), mirroring the reference's
``multi_modal_transformers/tokenizers/token_compression.py`` API on MI355X.

* ``bipartite_soft_matching(metric, r, class_token, distill_token)`` (reference :54-112) runs the
  gfx950 ``tome_match`` kernel and returns a ``merge`` callable, or the ``(do_nothing, do_nothing)``
  tuple for ``r <= 0`` exactly like the reference (:69-70).
* ``merge(x, mode="sum")`` (:90-109) runs the fused gather/scatter kernel (plain sum).
* ``merge_wavg(merge, x, size)`` (:114-129) is ONE fused kernel (weighted sum + division) with an
  autograd backward (a weighted gather kernel).

All indices are int32 device tensors, bit-exact with the canonical oracle (oracle/tome_ref.c).
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch

from .. import _kernels as K


def do_nothing(x, mode=None):
    return x


class _MergeWavgFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, plan, set_start, flags):
        t, r = plan.t, plan.r
        out, size_out, pos_map = K.tome_merge_fwd(x, set_start, t, r, plan.unm_idx, plan.src_idx,
                                                  plan.dst_idx, size_in=size, flags=flags)
        ctx.save_for_backward(size, size_out, pos_map)
        ctx.meta = (set_start, t, r, bool(flags & K.FLAG_PLAIN_SUM))
        ctx.mark_non_differentiable(size_out)
        return out, size_out

    @staticmethod
    def backward(ctx, g_out, _g_size):
        size, size_out, pos_map = ctx.saved_tensors
        set_start, t, r, plain = ctx.meta
        if plain:
            size, size_out = None, None
        g_in = K.tome_merge_bwd(g_out.contiguous(), set_start, t, r, pos_map, size, size_out)
        return g_in, None, None, None, None


class TokenMerge:
    """The ``merge`` closure of the reference (token_compression.py:90-109), holding the matched
    indices (int32, shapes (n, ta-r), (n, r), (n, r))."""

    def __init__(self, unm_idx, src_idx, dst_idx, t: int, r: int, class_token: bool,
                 distill_token: bool):
        self.unm_idx, self.src_idx, self.dst_idx = unm_idx, src_idx, dst_idx
        self.t, self.r = t, r
        self.flags = (K.FLAG_CLASS if class_token else 0) | (K.FLAG_DISTILL if distill_token else 0)

    def __call__(self, x: torch.Tensor, mode: str = "sum") -> torch.Tensor:
        flags = self.flags | K.FLAG_PLAIN_SUM | (0 if mode == "sum" else K.FLAG_NO_SCATTER)
        out, _ = _MergeWavgFn.apply(x.contiguous(), None, self, 0, flags)
        return out

    def merge_wavg(self, x: torch.Tensor, size: torch.Tensor | None = None, set_start: int = 0):
        """Fused merge_wavg over rows [set_start, set_start + t) of x (n, L, D); other rows are
        copied. size: (n, t) fp32 or None. Returns (x (n, L-r, D), size (n, t-r))."""
        if size is not None and size.dim() == 3:
            size = size[..., 0]
        size = None if size is None else size.contiguous().float()
        return _MergeWavgFn.apply(x, size, self, set_start, self.flags)


def bipartite_soft_matching(metric: torch.Tensor, r: int, class_token: bool = False,
                            distill_token: bool = False):
    """Reference token_compression.py:54-112. metric: (n, t, c) device tensor (fp32 or bf16), or
    (n, t, heads, c) in which case the metric is the sum over heads (tome_attention.py:253)."""
    protected = int(class_token) + int(distill_token)
    t = metric.shape[1]
    r = min(r, (t - protected) // 2)
    if r <= 0:
        return do_nothing, do_nothing
    flags = (K.FLAG_CLASS if class_token else 0) | (K.FLAG_DISTILL if distill_token else 0)
    unm, src, dst = K.tome_match(metric, r, flags)
    return TokenMerge(unm, src, dst, t, r, class_token, distill_token)


def merge_wavg(merge: Callable, x: torch.Tensor,
               size: torch.Tensor | None = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference token_compression.py:114-129: x (n, t, D), size (n, t, 1) or None.
    Returns (x_merged (n, t-r, D), size (n, t-r, 1))."""
    if size is None:
        size = torch.ones_like(x[..., 0, None], dtype=torch.float32)
    if not isinstance(merge, TokenMerge):  # the do_nothing closure
        x = merge(x * size, mode="sum")
        size = merge(size, mode="sum")
        return x / size, size
    out, size_out = merge.merge_wavg(x, size)
    return out, size_out[..., None]


class _TopKFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, embeddings, scores, tokenset_idx, tokenset_k):
        out, idx = K.topk_gather(embeddings, scores, tokenset_idx, tokenset_k)
        ctx.save_for_backward(idx)
        ctx.L = embeddings.shape[1]
        ctx.mark_non_differentiable(idx)
        return out, idx

    @staticmethod
    def backward(ctx, g_out, _g_idx):
        (idx,) = ctx.saved_tensors
        return K.topk_scatter_bwd(g_out.contiguous(), idx, ctx.L), None, None, None


def compute_top_k_tokens(embeddings: torch.Tensor, importance_scores: torch.Tensor,
                         tokenset_idx, tokenset_k, return_indices: bool = False):
    """Reference token_compression.py:15-46: per token set (start, num_tokens), the tokens with
    the k largest importance scores (jax.lax.top_k order: descending, ties to the lower index),
    the sets concatenated in order. Accepts the reference's single-sample (L, D) / (L,) call or
    the vmapped batch (B, L, D) / (B, L) (:168). Differentiable w.r.t. the embeddings (the
    indices carry no gradient). One gfx950 kernel (csrc/prune.hip)."""
    single = embeddings.dim() == 2
    x = embeddings[None] if single else embeddings
    sc = importance_scores[None] if single else importance_scores
    out, idx = _TopKFn.apply(x.contiguous(), sc.float().contiguous(), list(tokenset_idx),
                             list(tokenset_k))
    if single:
        out, idx = out[0], idx[0]
    return (out, idx) if return_indices else out
