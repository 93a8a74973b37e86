"""Optimizer and train-state pieces on the GPU:
* mmt_adamw (the fused AdamW over the flat buffer, octo.py:228 apply_gradients with optax.adamw
  semantics) vs torch.optim.AdamW in fp32 on the CPU over 3 steps, with the DDP 1/N grad_scale;
  the bf16 shadow is exactly bf16(master);
* diffusion_train_step returns (state, grads) and merges the loss into the running average
  (octo.py:216-239);
* AddPositionEmbedding (tokenizers/readout/readout.py:8-33) forward/backward vs torch fp32.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("grad_scale", [1.0, 0.5])
def test_adamw_matches_torch(dev, grad_scale):
    from multi_modal_transformers_tokenmerge_amd import _C
    n = 100_003
    g = torch.Generator().manual_seed(3)
    p0 = torch.randn(n, generator=g)
    lr, b1, b2, eps, wd = 3e-3, 0.9, 0.999, 1e-8, 1e-2
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)
    p = p0.to(dev)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=dev)
    state = torch.tensor([1234, 0], dtype=torch.int32, device=dev)
    for it in range(3):
        grad = torch.randn(n, generator=g) * (it + 1)
        ref.grad = grad * grad_scale
        opt.step()
        _C.call("mmt_adamw", _C.ptr(p), _C.ptr(grad.to(dev)), _C.ptr(m), _C.ptr(v), _C.ptr(shadow), n,
                _C.ptr(state), lr, b1, b2, eps, wd, grad_scale, _C.stream_ptr())
        _C.call("mmt_step_advance", _C.ptr(state), _C.stream_ptr())
        torch.cuda.synchronize()
        torch.testing.assert_close(p.cpu(), ref.detach(), rtol=2e-6, atol=2e-7)
        st = opt.state[ref]
        torch.testing.assert_close(m.cpu(), st["exp_avg"], rtol=2e-6, atol=1e-7)
        torch.testing.assert_close(v.cpu(), st["exp_avg_sq"], rtol=2e-6, atol=1e-12)
        assert torch.equal(shadow.cpu(), p.cpu().bfloat16())
    assert int(state[1].item()) == 3


def test_diffusion_train_step_returns_grads_and_metrics(dev):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo import octo as O
    from oracle.parity import _inputs
    model = O.Octo(get_config("octo-tiny", num_blocks=2), dev, seed=0)
    state = O.create_octo_train_state(model, seed=7)
    images, _, actions = _inputs(model, 3)
    img, act = torch.from_numpy(images).to(dev), torch.from_numpy(actions).to(dev)
    losses = []
    for _ in range(3):
        state, grads = O.diffusion_train_step(model, state, None, img, act)
        losses.append(float(state.last_loss))
    assert set(grads) == {p.name for p in model.store.params}
    assert all(grads[p.name].data_ptr() == p.grad.data_ptr() for p in model.store.params)
    assert float(sum(g.abs().sum() for g in grads.values())) > 0
    assert state.step == 3
    assert abs(state.metrics.compute() - np.mean(losses)) <= 1e-5 * abs(np.mean(losses))


def test_add_position_embedding(dev):
    from multi_modal_transformers_tokenmerge_amd.params import ParamStore
    from multi_modal_transformers_tokenmerge_amd.tokenizers.readout.readout import AddPositionEmbedding
    store = ParamStore()
    mod = AddPositionEmbedding().bind(store, "AddPositionEmbedding_0", 8, 64)
    store.materialize(dev, 0)
    x = torch.randn((3, 8, 64), device=dev)
    y = mod(x)
    torch.testing.assert_close(y, x + mod.pe.data[None], rtol=0, atol=0)
    dout = torch.randn_like(x)
    store.zero_grad()
    dx = mod.backward(dout)
    torch.cuda.synchronize()
    assert dx is dout
    torch.testing.assert_close(mod.pe.grad, dout.sum(0), rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):
        mod(torch.zeros((8, 64), device=dev))


def test_wgrad_overlap_schedule_same_gradients(dev):
    """The side-stream weight-gradient schedule (layers.wgrad_overlap: dW GEMMs forked onto a
    second stream at each Dense.bwd, joined per block with lag 0 / 1 and at the end of the
    backward) changes only WHEN work runs: every gradient equals the single-stream backward's,
    eager and HIP-graph captured. The dW products (split-K slabs + ordered combine) are
    deterministic and compared bit for bit; bias / LayerNorm / embedding gradients accumulate
    per-workgroup partials with fp32 atomics (arrival order varies run to run), compared to
    rounding."""
    from multi_modal_transformers_tokenmerge_amd.layers import wgrad_overlap
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo import octo as O
    from oracle.parity import _inputs
    cfg = get_config("octo-tiny", num_blocks=3, token_compression_sequence="[Image{4};Readout{0}]")
    model = O.Octo(cfg, dev, seed=0)
    images, _, actions = _inputs(model, 4)
    img, act = torch.from_numpy(images).to(dev), torch.from_numpy(actions).to(dev)
    rng = torch.tensor([11, 3], dtype=torch.int32, device=dev)

    def fwd_bwd():
        model.store.zero_grad()
        _, st = model.compute_diffusion_denoise_loss(None, img, act, True, rng, 0)
        model.backward(st)

    def run(enabled, lag, graph):
        old = (wgrad_overlap.enabled, wgrad_overlap.lag)
        wgrad_overlap.enabled, wgrad_overlap.lag = enabled, lag
        try:
            if graph:
                side = torch.cuda.Stream()
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    fwd_bwd()
                torch.cuda.current_stream().wait_stream(side)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fwd_bwd()
                g.replay()
            else:
                fwd_bwd()
            torch.cuda.synchronize()
            return model.store.flat_grad.clone()
        finally:
            wgrad_overlap.enabled, wgrad_overlap.lag = old

    ref = run(False, 0, False)
    kernels = [p for p in model.store.params if p.name.endswith("/kernel")]
    for enabled, lag, graph in ((True, 0, False), (True, 1, False), (True, 1, True),
                                (False, 0, True), (True, 2, True)):
        got = run(enabled, lag, graph)
        for p in kernels:
            sl = slice(p.offset, p.offset + p.numel)
            assert torch.equal(got[sl], ref[sl]), (p.name, enabled, lag, graph)
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("fp8", [False, True])
def test_ddpstep_build_leaves_training_state_unchanged(dev, fp8):
    """distributed.DDPStep.build() trains for its warm-up steps outside capture and restores the
    state after them: the fp32 master weights, the bf16 / transposed / e4m3 shadows (+ scales),
    the AdamW moments, the RNG / step counter and the running loss metrics are bitwise what they
    were before build() (world size 1, the one-graph step)."""
    from multi_modal_transformers_tokenmerge_amd.distributed import DDPStep
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo import octo as O
    from oracle.parity import _inputs
    model = O.Octo(get_config("octo-tiny", num_blocks=2, fp8=fp8), dev, seed=0)
    state = O.create_octo_train_state(model, seed=7)
    images, _, actions = _inputs(model, 4)
    img, act = torch.from_numpy(images).to(dev), torch.from_numpy(actions).to(dev)
    for _ in range(2):  # non-trivial moments, step counter and metrics before build()
        state, _ = O.diffusion_train_step(model, state, None, img, act)
    torch.cuda.synchronize()
    st = model.store

    def snap():
        t = [st.flat, st.flat_bf16, st.m, st.v, state.rng, st.flat_bf16_t]
        if st.flat_fp8 is not None:
            t += [st.flat_fp8, st.fp8_scale]
        if state.metrics is not None:
            t += [state.metrics.total, state.metrics.count]
        return [x.clone() for x in t]
    before = snap()
    assert (st.flat_fp8 is not None) == fp8
    DDPStep(model, state, None, img, act, None).build()
    torch.cuda.synchronize()
    for a, b in zip(before, snap()):
        assert torch.equal(a, b)
