"""Top-k token pruning (reference tokenizers/token_compression.py:15-46).

CPU: the oracle's lax.top_k semantics (descending, ties -> lower index, NaN largest, -0 < +0,
per-set offsets, concatenation order). GPU: the gfx950 kernel vs the oracle — bit-exact indices
and gathered rows — and the backward scatter / autograd path.
"""
import numpy as np
import pytest
import torch

from oracle import tome as O


def test_oracle_topk_semantics():
    e = np.arange(20, dtype=np.float32).reshape(10, 2)
    s = np.array([0.1, 0.5, 0.5, 0.2, -0.0, 0.0, np.nan, 0.3, 0.3, 0.9], np.float32)
    rows, ids = O.topk_tokens(e, s, [(0, 4), (4, 6)], [3, 4])
    assert ids.tolist() == [1, 2, 3, 6, 9, 7, 8]
    np.testing.assert_array_equal(rows, e[ids])
    _, ids = O.topk_tokens(e, s, [(4, 2)], [1])
    assert ids.tolist() == [5]                      # +0 ranks above -0 in the total order
    _, ids = O.topk_tokens(e, s, [(4, 6), (0, 4)], [0, 2])
    assert ids.tolist() == [1, 2]                   # k = 0 sets contribute nothing


CASES = [(3, 292, 384, [(32, 256), (288, 4)], [64, 2], torch.float32),
         (2, 74, 768, [(0, 16), (16, 25), (45, 25)], [8, 5, 25], torch.bfloat16),
         (4, 1100, 64, [(30, 1030)], [500], torch.float32)]


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,D,sets,ks,dt", CASES)
def test_topk_gather_bit_exact(dev, B, L, D, sets, ks, dt):
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_compression import (
        compute_top_k_tokens)
    g = torch.Generator().manual_seed(L)
    x = torch.randn((B, L, D), generator=g).to(dt)
    sc = torch.randn((B, L), generator=g)
    sc[:, ::7] = sc[:, 3:4]                          # plenty of ties
    sc[0, 5] = float("nan")
    out, idx = compute_top_k_tokens(x.to(dev), sc.to(dev), sets, ks, return_indices=True)
    torch.cuda.synchronize()
    for b in range(B):
        rows, ids = O.topk_tokens(x[b].float().numpy(), sc[b].numpy(), sets, ks)
        np.testing.assert_array_equal(idx[b].cpu().numpy(), ids)
        np.testing.assert_array_equal(out[b].float().cpu().numpy(), rows)
    # single-sample call of the reference signature
    o1 = compute_top_k_tokens(x[1].to(dev), sc[1].to(dev), sets, ks)
    torch.testing.assert_close(o1.cpu(), out[1].cpu(), rtol=0, atol=0)


@pytest.mark.gpu
def test_topk_backward_scatter(dev):
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_compression import (
        compute_top_k_tokens)
    g = torch.Generator().manual_seed(3)
    x = torch.randn((2, 40, 64), generator=g).to(dev).requires_grad_()
    sc = torch.randn((2, 40), generator=g).to(dev)
    out, idx = compute_top_k_tokens(x, sc, [(0, 20), (20, 20)], [5, 7], return_indices=True)
    gout = torch.randn_like(out)
    out.backward(gout)
    ref = torch.zeros_like(x)
    for b in range(2):
        ref[b, idx[b].long()] = gout[b]
    torch.testing.assert_close(x.grad, ref, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gather_rows_bit_exact(dev, dt):
    """mmt_gather_rows (the pruned block's residual rows) == torch advanced indexing."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    g = torch.Generator().manual_seed(9)
    x = torch.randn((3, 292, 384), generator=g).to(dt).to(dev)
    idx = torch.stack([torch.randperm(292, generator=g)[:276] for _ in range(3)]).int().to(dev)
    out = K.gather_rows(x, idx)
    want = x[torch.arange(3, device=dev)[:, None], idx.long()]
    assert torch.equal(out, want)
