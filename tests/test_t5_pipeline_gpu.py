"""DDPStep's cross-step T5 pipeline (distributed.DDPStep, txt_next): the frozen T5 encoder of the
next step's text runs on a side stream beside this step's backward, and the forward takes the
output computed one step earlier. The pipelined step must train exactly like the plain one
(reference octo.py:216-239 diffusion_train_step: T5 of the step's own text, stop_gradient) when
the text changes every step: after each step the gradients per parameter (TextProjection's dW
reads the T5 output, so an off-by-one batch shows there first) and the loss agree with a
plain DDPStep fed the same batches, and the encoder output held for the next step is bitwise
T5(next text). Covers the one-graph step, the eager step and the staged schedule's pieces."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def _setup(dev):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    cfg = get_config("octo-small-tome16", num_blocks=2, t5=T5Config(num_layers=2))
    model = Octo(cfg, dev, seed=0)
    state = create_octo_train_state(model, seed=11)
    return model, state


def _batches(model, B, n, dev):
    from oracle.parity import _inputs
    out = []
    for i in range(n):
        images, text, actions = _inputs(model, B, seed=40 + i)
        out.append(tuple(torch.from_numpy(x).to(dev) for x in (images, text, actions)))
    return out


@pytest.mark.parametrize("fork", ["ext", "fwd", "bwd"])
@pytest.mark.parametrize("use_graph", [True, False], ids=["graph", "eager"])
def test_pipelined_step_matches_plain(dev, use_graph, fork, monkeypatch):
    """fork: where the next step's encoder runs (DDPStep.t5_fork_at): its own graph beside the
    step's ("ext", the default) or forked inside the step's graph at its start / after the
    forward."""
    from multi_modal_transformers_tokenmerge_amd.distributed import DDPStep
    monkeypatch.setattr(DDPStep, "t5_fork_at", fork)
    B, n = 2, 4
    ma, sa = _setup(dev)
    mb, sb = _setup(dev)
    assert torch.equal(ma.store.flat, mb.store.flat)
    data = _batches(ma, B, n + 1, dev)
    bufs = []
    for m in (ma, mb):  # built on a batch no step trains on: the loader writes batch 0 after build()
        img, txt, act = (x.clone() for x in data[n])
        bufs.append((img, txt, act))
    txt_next = data[1][1].clone()
    pa = DDPStep(ma, sa, bufs[0][1], bufs[0][0], bufs[0][2], None, use_graph=use_graph,
                 txt_next=txt_next).build()
    pb = DDPStep(mb, sb, bufs[1][1], bufs[1][0], bufs[1][2], None, use_graph=use_graph).build()
    assert pa.t5_pf and not pb.t5_pf
    for i in range(n):
        for (img, txt, act) in bufs:  # this step's batch in both steps' input buffers
            img.copy_(data[i][0]); txt.copy_(data[i][1]); act.copy_(data[i][2])
        txt_next.copy_(data[i + 1][1])
        pa()
        pb()
        torch.cuda.synchronize()
        assert abs(float(pa.loss_buf) - float(pb.loss_buf)) <= 1e-4 * abs(float(pb.loss_buf)) + 1e-6
        ga, gb = ma.store.flat_grad, mb.store.flat_grad
        worst = max((_rel(ga[p.offset:p.offset + p.numel], gb[p.offset:p.offset + p.numel]), p.name)
                    for p in mb.store.params if gb[p.offset:p.offset + p.numel].abs().sum() > 0)
        assert worst[0] <= 1e-3, (i, worst)
        # the output held for step i + 1 is the encoder of step i + 1's text, bit for bit
        assert torch.equal(pa.t5_cur, ma.t5(data[i + 1][1]))
    assert _rel(ma.store.flat, mb.store.flat) <= 1e-5
    # reset_text(): the next call encodes its own txt again (here: a batch txt_next never held)
    for (img, txt, act) in bufs:
        img.copy_(data[1][0]); txt.copy_(data[1][1]); act.copy_(data[1][2])
    pa.reset_text()
    pa()
    pb()
    torch.cuda.synchronize()
    assert abs(float(pa.loss_buf) - float(pb.loss_buf)) <= 1e-4 * abs(float(pb.loss_buf)) + 1e-6


@pytest.mark.parametrize("fork", ["ext", "fwd", "bwd"])
def test_staged_pieces_pipeline(dev, fork, monkeypatch):
    """The staged schedule's pieces in _run's order (the "ext" launch, _stage(k) for k < S, the
    "ext" hand-over, _opt), eagerly over a 2-stage backward split; with an in-graph fork the
    encoder forks in stage 0 and is handed over in the last stage (after the text projection's
    dW)."""
    from multi_modal_transformers_tokenmerge_amd.distributed import DDPStep
    monkeypatch.setattr(DDPStep, "t5_fork_at", fork)
    B = 2
    ma, sa = _setup(dev)
    mb, sb = _setup(dev)
    data = _batches(ma, B, 3, dev)
    img, txt, act = (x.clone() for x in data[0])
    txt_next = data[1][1].clone()
    pa = DDPStep(ma, sa, txt, img, act, None, use_graph=False, txt_next=txt_next).build()
    pa.bounds = ma.stage_bounds(2)
    pa.S = len(pa.bounds) - 1
    assert pa.S == 2
    for i in range(2):
        img.copy_(data[i][0]); txt.copy_(data[i][1]); act.copy_(data[i][2])
        txt_next.copy_(data[i + 1][1])
        pa._t5_ext_launch()
        for k in range(pa.S):
            pa._stage(k)
        pa._t5_ext_join()
        ga = ma.store.flat_grad.clone()
        pa._opt()
        mb.store.zero_grad()
        _, st = mb.compute_diffusion_denoise_loss(data[i][1], data[i][0], data[i][2], True, sb.rng,
                                                  sb.sample_offset)
        mb.backward(st)
        gb = mb.store.flat_grad
        sb.apply_gradients()
        torch.cuda.synchronize()
        worst = max((_rel(ga[p.offset:p.offset + p.numel], gb[p.offset:p.offset + p.numel]), p.name)
                    for p in mb.store.params if gb[p.offset:p.offset + p.numel].abs().sum() > 0)
        assert worst[0] <= 1e-3, (i, worst)
        assert torch.equal(pa.t5_cur, ma.t5(data[i + 1][1]))
