"""Deterministic mode (ParamStore.set_deterministic / MMT_DETERMINISTIC=1; include/mmt_api.h
mmt_set_deterministic; SURVEY §5 "deterministic-mode reruns", §8e RNG semantics).

* test_reruns_bitwise: the same step twice gives bitwise-identical gradients (every tensor,
  including the bias / LayerNorm / GroupNorm / embedding gradients that are fp32 atomics
  otherwise) and loss; the mode's result equals the atomic one within the fixed-point
  resolution (2^-36 per contribution).
* test_shards_equal_full_batch: two data-parallel shards (global sample offsets 0 and B) against
  the full 2B batch in the mode: the ToMe index triples of every layer are bitwise equal
  (per-sample forward arithmetic does not depend on the batch composition), and the averaged
  shard gradients equal the full-batch gradients up to the summation order of the weight-
  gradient reductions and of the one all-reduce (relative L2 per tensor <= 1e-4).
"""
import pytest
import torch

from oracle.parity import _inputs

pytestmark = pytest.mark.gpu


def _setup(dev, B):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    cfg = get_config("octo-small-tome16", num_blocks=3, t5=T5Config(num_layers=2))
    model = Octo(cfg, dev, seed=0)
    state = create_octo_train_state(model, seed=11)
    images, text, actions = _inputs(model, B, seed=3)
    return model, state, (torch.from_numpy(text).to(dev), torch.from_numpy(images).to(dev),
                          torch.from_numpy(actions).to(dev))


def _step(model, state, inp, sl, offset):
    txt, img, act = inp
    model.store.zero_grad()
    loss, st = model.compute_diffusion_denoise_loss(txt[sl].contiguous(), img[sl].contiguous(),
                                                    act[sl].contiguous(), True, state.rng, offset)
    model.backward(st)
    torch.cuda.synchronize()
    tome = [tuple(a.clone() for a in sv["tome"][6:9]) for sv in st["stack_sv"] if sv["tome"] is not None]
    return float(loss.item()), model.store.flat_grad.clone(), tome


def test_reruns_bitwise(dev):
    model, state, inp = _setup(dev, 6)
    sl = slice(0, 6)
    try:
        model.store.set_deterministic(True)
        l1, g1, _ = _step(model, state, inp, sl, 0)
        l2, g2, _ = _step(model, state, inp, sl, 0)
        assert l1 == l2
        assert torch.equal(g1, g2)
        assert int(model.store.det_fx.abs().sum().item()) == 0  # flushed and cleared
    finally:
        model.store.set_deterministic(False)
    la, ga, _ = _step(model, state, inp, sl, 0)  # fp32 atomics
    assert la == l1  # the forward does not use the atomic sites
    for p in model.store.params:
        a, b = ga[p.offset:p.offset + p.numel], g1[p.offset:p.offset + p.numel]
        assert float((a - b).norm()) <= 1e-5 * float(b.norm()) + 1e-9, p.name


def test_shards_equal_full_batch(dev):
    B = 3
    model, state, inp = _setup(dev, 2 * B)
    try:
        model.store.set_deterministic(True)
        _, full, tf = _step(model, state, inp, slice(0, 2 * B), 0)
        _, g0, t0 = _step(model, state, inp, slice(0, B), 0)
        _, g1, t1 = _step(model, state, inp, slice(B, 2 * B), B)
    finally:
        model.store.set_deterministic(False)
    assert len(tf) == model.cfg.num_blocks
    for layer, (f, a, b) in enumerate(zip(tf, t0, t1)):
        for nm, ff, aa, bb in zip(("unm", "src", "dst"), f, a, b):
            assert torch.equal(ff[:B], aa), (layer, nm)
            assert torch.equal(ff[B:], bb), (layer, nm)
    avg = (g0 + g1) / 2
    for p in model.store.params:
        a, b = avg[p.offset:p.offset + p.numel].double(), full[p.offset:p.offset + p.numel].double()
        if float(b.norm()) == 0:
            continue
        assert float((a - b).norm() / b.norm()) <= 1e-4, p.name


def test_nan_and_large_contributions_stay_visible(dev):
    """in the mode a NaN / Inf contribution or one beyond the shadow's
    per-contribution bound (|v| >= 2^15) goes to the fp32 gradient as a plain atomic
    (csrc/common.h det_fits), so the gradient shows it after the flush instead of a clamped
    finite value — and many large contributions whose sum exceeds the int64 shadow's 2^27 range
    (4096 rows of 2^17: 2^29, which wrapped under the round-5 per-contribution bound of 2^26)
    come out exact instead of wrapped."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from multi_modal_transformers_tokenmerge_amd.params import ParamStore, const
    st = ParamStore()
    p = st.add("w", (64,), const(0.0))
    st.materialize(dev)
    x = torch.ones((512, 64), dtype=torch.float32, device=dev)
    x[3, 5] = float("nan")
    x[7, 9] = float("inf")
    x[11, 13] = 1e9
    with st.deterministic():
        K.colsum(x, p.grad)
        st.det_flush()
        torch.cuda.synchronize()
        g = p.grad.cpu()
    assert torch.isnan(g[5]) and g[9] == float("inf")
    assert abs(float(g[13]) - (1e9 + 511)) <= 1e9 * 1e-6
    rest = [i for i in range(64) if i not in (5, 9, 13)]
    assert torch.equal(g[rest], torch.full((61,), 512.0))
    p.grad.zero_()
    with st.deterministic():
        K.colsum(torch.full((4096, 64), 2.0 ** 17, device=dev), p.grad)
        st.det_flush()
        torch.cuda.synchronize()
        assert torch.equal(p.grad.cpu(), torch.full((64,), 2.0 ** 29))


def test_second_store_cannot_take_the_registration(dev):
    from multi_modal_transformers_tokenmerge_amd.params import ParamStore, const
    a, b = ParamStore(), ParamStore()
    a.add("w", (8,), const(0.0))
    b.add("w", (8,), const(0.0))
    a.materialize(dev)
    b.materialize(dev)
    with a.deterministic():
        with pytest.raises(RuntimeError):
            b.set_deterministic(True)
    with b.deterministic():  # free again after a's block
        assert ParamStore._det_owner() is b
    assert ParamStore._det_owner is None


def test_dropped_store_releases_the_registration(dev):
    """A store dropped without close() (e.g. a model built under MMT_DETERMINISTIC=1 and thrown
    away) must not lock the mode for the rest of the process: the registration refers to it
    weakly, the library's buffers stay alive until the next store takes over, and that store's
    sums are exact again."""
    import gc
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from multi_modal_transformers_tokenmerge_amd.params import ParamStore, const
    a = ParamStore()
    a.add("w", (64,), const(0.0))
    a.materialize(dev)
    a.set_deterministic(True)
    del a
    gc.collect()
    assert ParamStore._det_buffers is not None  # the device buffers outlive the store
    b = ParamStore()
    p = b.add("w", (64,), const(0.0))
    b.materialize(dev)
    b.set_deterministic(True)  # takes the registration over
    try:
        assert ParamStore._det_owner() is b and ParamStore._det_buffers[1] is b.det_fx
        K.colsum(torch.ones((300, 64), device=dev), p.grad)
        b.det_flush()
        torch.cuda.synchronize()
        assert torch.equal(p.grad.cpu(), torch.full((64,), 300.0))
    finally:
        b.close()
    assert ParamStore._det_owner is None and ParamStore._det_buffers is None
