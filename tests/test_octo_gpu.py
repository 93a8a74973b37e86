"""GPU end-to-end parity: the HIP training step (forward loss + every parameter gradient) vs the
fp32 CPU oracle (oracle/octo_ref.py) on identical inputs, identical dropout streams and the HIP
run's own position tokens, diffusion (t, eps) and ToMe indices injected into the oracle.

The oracle computes with the bf16-rounded Dense/attention kernels the HIP path actually multiplies
(its bf16 shadow), fp32 everywhere else. Remaining differences come from bf16 activations
(LayerNorm outputs, q/k/v, attention probabilities, MLP hidden, stem GroupNorm output, im2col
pixels) and from relu gates that flip under the resulting forward perturbation. The end-to-end bar
is set from the measured noise floor of that comparison (tools/parity_sweep.py, 12 runs over
seeds x ToMe on/off x dropout on/off, profiles/r01_parity_sweep.txt: loss within 2.7 %, global
gradient cosine >= 0.988, per-tensor >= 0.970 — the same with fp32 or bf16 LayerNorm input
gradients), with margin, and is checked on two seeds:
  loss: relative difference <= 4e-2
  gradients: cosine similarity >= 0.96 per parameter tensor, >= 0.985 on the concatenation
The per-op GPU tests (GEMM, attention, LayerNorm, ToMe, stem, sampler) carry the tight bars.
"""
import pytest

from oracle.parity import check as _check, run_parity

pytestmark = pytest.mark.gpu


def test_octo_tiny_parity(dev):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    cfg = get_config("octo-tiny", num_blocks=2)
    for seed in (0, 1):
        _check(run_parity(cfg, 3, seed=seed))


def test_octo_small_tome_parity(dev):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    cfg = get_config("octo-small-tome16", num_blocks=3, t5=T5Config(num_layers=2))
    for seed in (0, 1):
        _check(run_parity(cfg, 2, seed=seed))


def test_staged_backward_matches_backward(dev):
    """The block-range stages used to overlap the gradient all-reduce (bench.py, N > 1) write
    the gradients of the one-piece backward (up to the order of the fp32 atomics some bias and
    embedding gradients use), and each stage's region is final after it."""
    import torch
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    from oracle.parity import _inputs
    model = Octo(get_config("octo-tiny", num_blocks=4), dev, seed=0)
    state = create_octo_train_state(model, seed=5)
    images, text, actions = _inputs(model, 3)
    img, act = torch.from_numpy(images).to(dev), torch.from_numpy(actions).to(dev)
    model.store.zero_grad()
    _, st = model.compute_diffusion_denoise_loss(None, img, act, True, state.rng, 0)
    model.backward(st)
    ref = model.store.flat_grad.clone()
    S = 3
    regions = model.grad_regions(S)
    assert regions[0][1] == model.store.n and regions[-1][0] == 0
    assert all(regions[i][0] == regions[i + 1][1] for i in range(S - 1))
    model.store.zero_grad()
    _, st = model.compute_diffusion_denoise_loss(None, img, act, True, state.rng, 0)
    for k in range(S):
        model.backward_stage(st, k, S)
        lo, hi = regions[k]
        torch.cuda.synchronize()
        torch.testing.assert_close(model.store.flat_grad[lo:hi], ref[lo:hi], rtol=1e-4, atol=1e-6,
                                   msg=f"stage {k} region")
    torch.testing.assert_close(model.store.flat_grad, ref, rtol=1e-4, atol=1e-6)
