"""Continuous and categorical action heads (reference continuous.py,
categorical.py, octo.py:158-198, 242-320) on the device vs the float64 oracle
(oracle/heads_ref.py), the grouped readout mean vs torch, and both Octo train steps."""
import numpy as np
import pytest
import torch

from multi_modal_transformers_tokenmerge_amd import _C
from oracle import heads_ref as HR

pytestmark = pytest.mark.gpu


def test_action_head_kernels(dev):
    g = torch.Generator().manual_seed(0)
    B, A, NB, m = 37, 8, 256, 5.0
    z = torch.randn((B, A), generator=g) * 6
    y = torch.randn((B, A), generator=g) * 2
    zd, yd = z.to(dev), y.to(dev)
    loss = torch.zeros(1, device=dev)
    dz = torch.empty((B, A), dtype=torch.bfloat16, device=dev)
    pred = torch.empty((B, A), device=dev)
    _C.call("mmt_action_head", 0, _C.ptr(zd), A, B, A, _C.ptr(yd), None, 0, m, 1.0 / B, _C.ptr(pred),
            _C.ptr(loss), _C.ptr(dz), _C.stream_ptr())
    torch.cuda.synchronize()
    p_ref, l_ref, dz_ref = HR.continuous(z.numpy(), y.numpy(), m)
    np.testing.assert_allclose(pred.cpu().numpy(), p_ref[:, 0], rtol=1e-5, atol=1e-5)
    assert float(loss) == pytest.approx(l_ref, rel=1e-5)
    np.testing.assert_allclose(dz.float().cpu().numpy(), dz_ref, rtol=1e-2, atol=1e-6)

    zl = torch.randn((B, A, NB), generator=g) * 3
    ya = (torch.rand((B, A), generator=g) * 12 - 6)
    ya[0, :3] = torch.tensor([-5.0, 5.0, 4.99])
    zld, yad = zl.to(dev), ya.to(dev)
    edges = torch.from_numpy(np.linspace(-m, m, NB + 1, dtype=np.float32)).to(dev)
    loss.zero_()
    dzl = torch.empty((B * A, NB), dtype=torch.bfloat16, device=dev)
    _C.call("mmt_action_head", 1, _C.ptr(zld), NB, B * A, NB, _C.ptr(yad), _C.ptr(edges), NB + 1, m,
            1.0 / (B * A), None, _C.ptr(loss), _C.ptr(dzl), _C.stream_ptr())
    torch.cuda.synchronize()
    l_ref, dz_ref = HR.categorical(zl.numpy(), ya.numpy(), m, NB)
    assert float(loss) == pytest.approx(l_ref, rel=1e-5)
    np.testing.assert_allclose(dzl.float().cpu().numpy().reshape(B, A, NB), dz_ref, rtol=1e-2,
                               atol=1e-7)


def test_rows_group_mean(dev):
    B, L, D, G = 3, 11, 64, 2
    x = torch.randn((B, L, D), device=dev)
    grp = torch.tensor([-1, 0, 0, -1, 1, 1, 1, -1, 0, 1, -1], dtype=torch.int32, device=dev)
    counts = torch.tensor([3, 4], dtype=torch.int32, device=dev)
    out = torch.empty((B, G, D), dtype=torch.bfloat16, device=dev)
    _C.call("mmt_rows_group_mean_fwd", _C.ptr(x), L * D, D, B, L, D, _C.ptr(grp), G, _C.ptr(counts),
            _C.ptr(out), _C.stream_ptr())
    de = torch.randn((B, G, D), device=dev).to(torch.bfloat16)
    dx = torch.empty((B, L, D), device=dev)
    _C.call("mmt_rows_group_mean_bwd", _C.ptr(de), B, L, D, _C.ptr(grp), G, _C.ptr(counts), _C.ptr(dx),
            _C.stream_ptr())
    torch.cuda.synchronize()
    gl = grp.cpu().long()
    for gi in range(G):
        want = x[:, gl == gi].mean(1)
        torch.testing.assert_close(out[:, gi].float(), want, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(dx[:, gl == gi], (de[:, gi].float() / int(counts[gi]))[:, None].expand(
            B, int(counts[gi]), D), rtol=1e-6, atol=1e-6)
    assert not dx[:, gl < 0].any()


@pytest.mark.parametrize("kind", ["continuous", "categorical"])
def test_octo_head_train_steps(dev, kind):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo import octo as O
    cfg = get_config("octo-tiny", num_blocks=2, input_sequence="[Image{16};Readout{8}]",
                     action_heads=("diffusion", kind), num_bins=32)
    model = O.Octo(cfg, device=dev, seed=0)
    state = O.create_octo_train_state(model, seed=3)
    B = 4
    images = torch.randint(0, 256, (B, model.n_images, 64, 64, 3), dtype=torch.uint8, device=dev)
    actions = (torch.rand((B, 8), device=dev) * 2 - 1).contiguous()
    step = O.continuous_train_step if kind == "continuous" else O.categorical_train_step
    head = model.continuous_head if kind == "continuous" else model.categorical_head
    losses = []
    for _ in range(3):
        state, grads = step(model, state, None, images, actions)
        losses.append(float(state.last_loss))
        assert grads[head.dense.w.name].data_ptr() == head.dense.w.grad.data_ptr()
    assert abs(state.metrics.compute() - np.mean(losses)) <= 1e-5 * abs(np.mean(losses))
    assert all(np.isfinite(losses)) and head.dense.w.grad.abs().sum() > 0
    assert model.stack.blocks[0].qkv.w.grad.abs().sum() > 0
    out = (model.predict_continuous_action(None, images, state.rng) if kind == "continuous"
           else model.predict_action_logits(None, images, state.rng))
    torch.cuda.synchronize()
    assert out.shape == ((B, 1, 8) if kind == "continuous" else (B, 8, 32))


def test_octo_denoise_num_blocks_2(dev):
    """OctoDenoise num_blocks = 2 (diffusion.py:62-63: MLPBlock_0 on concatenate([noisy, temb,
    readout]), MLPBlock_1 on its (B, 8) output): the training step at the block-local bar
    (the head's parameters, MLPBlock_1 included, against the emulating oracle's chain), and the
    predict_action loop path from the fused sampler's initial draw: finite, clipped to [-5, 5],
    and equal to the fused sampler's z."""
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from oracle import parity as P
    cfg = get_config("octo-tiny", num_blocks=2, denoise_blocks=2)
    res = P.hip_blockwise(cfg, 3, seed=0)
    names = [n for n in res["grads"] if "OctoDenoise_0/MLPBlock_1/" in n]
    assert len(names) == 4 and all(np.abs(res["grads"][n]).sum() > 0 for n in names)
    P.check_blockwise(P.oracle_blockwise(cfg, res), cfg=cfg, res=res)
    model = res["model"]
    rng = torch.tensor([5, 0], dtype=torch.int32, device=dev)
    e = torch.randn((3, model.D), device=dev).bfloat16()
    act, z = model.head.predict_action_mean(e, rng, return_noise=True)
    torch.cuda.synchronize()
    assert torch.isfinite(act).all() and act.abs().max() <= 5.0
    one = get_config("octo-tiny", num_blocks=2)
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    m1 = Octo(one, dev, seed=0)
    _, z1 = m1.head.predict_action_mean(e, rng, return_noise=True)
    assert torch.equal(z, z1)
