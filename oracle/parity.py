"""ORACLE — test infrastructure only (used by tests/, __graft_entry__.smoke(), tools/parity_*.py).

End-to-end parity harness: run one HIP training step (forward loss + every parameter gradient)
and the CPU restatement (oracle/octo_ref.py, bf16 storage points emulated) on identical inputs,
identical dropout streams and the HIP run's own position tokens and diffusion (t, eps).

Top-k pruning (cfg.compression == "prune"): likewise, the rows each pruning layer kept must
equal the literal compute_top_k_tokens restatement on the step's own importance scores, and the
scores must agree with the oracle's (block-local bar) before the rows are injected.

ToMe: the HIP run's index triples are checked IN SITU first — for every merging layer,
canon_match (oracle/tome_ref.c) on the layer's own K projection (the bf16 qkv buffer the step
wrote, summed over heads) must reproduce the indices the step used, bit for bit. Only then are
they injected into the oracle (its own K differs from the HIP one by fp32 summation order, and
a near-tie could otherwise pick a different merge).

Split in three so a dump taken on the GPU box can be compared offline (tools/parity_dump.py):
  hip_step(cfg, B, seed)          -> results dict (numpy)
  oracle_step(cfg, res, ...)      -> (ref loss, {name: grad})   (CPU, rebuilds the parameters)
  compare(res, ref_loss, ref_g)   -> loss / cosine / norm-ratio report

Bars (bf16 path rtol 2e-2 on loss, gradient cosine >= 0.999; ADVICE r1: magnitude
checked as well as direction):
  loss:      |loss - ref| <= 2e-2 |ref|
  gradients: per tensor cosine >= 0.999 and norm ratio |g|/|g_ref| in [0.98, 1.02];
             global cosine over the concatenation >= 0.9995
"""
from __future__ import annotations

import numpy as np
import torch

LOSS_RTOL = 2e-2
COS_MIN = 0.999
COS_ALL_MIN = 0.9995
NORM_RATIO = (0.98, 1.02)


def _inputs(model, B, seed=0):
    cfg = model.cfg
    g = np.random.default_rng(seed)
    H = cfg.image_size[0]
    images = g.integers(0, 256, (B, model.n_images, H, H, 3), dtype=np.uint8)
    text = g.integers(0, cfg.t5.vocab_size, (B, model.n_text), dtype=np.int32) if model.has_text else None
    actions = g.uniform(-1, 1, (B, cfg.action_space_dim)).astype(np.float32)
    return images, text, actions


def insitu_tome_check(model, st):
    """For every merging layer: canonical matching on the step's own K (qkv buffer, summed over
    heads in the kernel's canonical order) must equal the indices the step merged with."""
    from oracle import tome as T
    H = model.cfg.num_heads
    Dh = model.D // H
    checked = 0
    for layer, sv in enumerate(st["stack_sv"]):
        for tm in _tome_list(sv):   # every merged set of the block (several: one match each)
            s0, t, r = tm[:3]
            qkv = sv["qkv"]
            B, L = qkv.shape[:2]
            metric = qkv.view(B, L, 3, H, Dh)[:, s0:s0 + t, 1].float().cpu().numpy()
            cu, cs, cd, _ = T.canon_match(metric, r)
            for name, got, want in zip(("unm", "src", "dst"), tm[6:9], (cu, cs, cd)):
                g = got.cpu().numpy()
                if not np.array_equal(g, want):
                    bad = np.argwhere(g != want)[:4].tolist()
                    raise AssertionError(f"layer {layer} set at {s0}: in-situ ToMe {name} differs "
                                         f"from canon_match at {bad}")
            checked += 1
    return checked


def _tome_list(sv):
    """The block's merges in set order (one tuple per merged set; empty without ToMe)."""
    tms = sv.get("tome_sets") or ([sv["tome"]] if sv.get("tome") is not None else [])
    return sorted(tms, key=lambda tm: tm[0])


def _size_in(sv, f):
    """The block's incoming per-set token sizes: a tensor (one merged set), {set: tensor}
    (several), or None."""
    if sv.get("tome") is not None:
        return None if sv["tome"][4] is None else f(sv["tome"][4])
    tms = _tome_list(sv)
    if not tms:
        return None
    return {tm[9]: f(tm[4]) for tm in tms if tm[4] is not None} or None


def insitu_prune_check(model, st):
    """For every pruning layer: the literal compute_top_k_tokens restatement (oracle/tome.py
    topk_tokens) on the step's own importance scores must equal the rows the step kept."""
    from oracle.tome import topk_tokens
    checked = 0
    for layer, sv in enumerate(st["stack_sv"]):
        if sv.get("prune") is None:
            continue
        sets, ks = st["ctxs"][layer].prune
        idx, scores = (a.cpu().numpy() for a in sv["prune"])
        for b in range(idx.shape[0]):
            _, want = topk_tokens(np.zeros((scores.shape[1], 1), np.float32), scores[b], sets, ks)
            if not np.array_equal(idx[b], want):
                bad = np.argwhere(idx[b] != want)[:4].ravel().tolist()
                raise AssertionError(f"layer {layer} sample {b}: in-situ top-k differs at {bad}")
        checked += 1
    return checked


def _used(sv, f=lambda a: a.cpu()):
    """The compression indices a block used: the ToMe (unm, src, dst) triple, the top-k rows, or
    None."""
    if sv["tome"] is not None:
        return tuple(f(a) for a in sv["tome"][6:9])
    if sv.get("tome_sets"):  # several merged sets: a triple per set, in set order
        return [tuple(f(a) for a in tm[6:9]) for tm in _tome_list(sv)]
    if sv.get("prune") is not None:
        return f(sv["prune"][0])
    return None


def _inject(x):
    if x is None:
        return None
    if isinstance(x, tuple):
        return tuple(torch.from_numpy(np.asarray(a)) for a in x)
    if isinstance(x, list):  # several merged sets
        return [_inject(t) for t in x]
    return torch.from_numpy(np.asarray(x))


TRACE_KEYS = ("x", "y0", "qkv", "o", "x1", "y1", "h")


def hip_trace(st, layers):
    """HIP intermediates under the oracle's trace names (fp32 numpy)."""
    out = {"img": st["img_tok"].float().cpu().numpy()}
    if st.get("txt") is not None:
        out["txt"] = st["txt"].float().cpu().numpy()
    for i, sv in enumerate(st["stack_sv"]):
        keys = TRACE_KEYS if i in layers else ("x",)
        for k in keys:
            out[f"b{i}/{k}"] = sv[k].float().cpu().numpy()
    return out


def hip_step(cfg, B, seed=0, check_tome=True, trace_layers=None):
    """One HIP forward + backward (no optimizer step) on synthetic inputs; returns numpy results
    (trace_layers: also the intermediates of those blocks and every block input)."""
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    dev = torch.device("cuda")
    model = Octo(cfg, dev, seed=seed)
    state = create_octo_train_state(model, seed=1234)
    images, text, actions = _inputs(model, B, seed)
    d_img = torch.from_numpy(images).to(dev)
    d_txt = torch.from_numpy(text).to(dev) if text is not None else None
    d_act = torch.from_numpy(actions).to(dev)
    model.store.zero_grad()
    loss, st = model.compute_diffusion_denoise_loss(d_txt, d_img, d_act, True, state.rng, 0)
    model.backward(st)
    torch.cuda.synchronize()
    n_tome = insitu_tome_check(model, st) if check_tome else 0
    n_prune = insitu_prune_check(model, st) if check_tome else 0
    res = dict(B=B, seed=seed, loss=float(loss.item()),
               rt=st["rt"].cpu().numpy(), ct=st["ct"].cpu().numpy(),
               t=st["head_sv"]["t"].cpu().numpy(), eps=st["head_sv"]["eps"].cpu().numpy(),
               tome=[_used(sv, lambda a: a.cpu().numpy()) for sv in st["stack_sv"]],
               prune_layers_checked=n_prune,
               grads={p.name: p.grad.detach().cpu().numpy().copy() for p in model.store.params},
               tome_layers_checked=n_tome, model=model)
    if trace_layers is not None:
        res["trace"] = hip_trace(st, set(trace_layers))
    return res


def oracle_params(model):
    """The parameters the kernels multiply: bf16 shadows of the Dense / conv kernels, fp32 masters
    of everything else (biases, norms, embeddings, the Fourier kernel)."""
    params = {}
    for p in model.store.params:
        src = p.bf16 if (p.name.endswith("kernel") and "fourier" not in p.name) else p.data
        params[p.name] = src.detach().float().cpu().clone().requires_grad_()
    t5p = ({p.name: p.bf16.float().cpu() for p in model.t5.store.params} if model.has_text else None)
    return params, t5p


def oracle_step(cfg, res, model=None, emulate_bf16=True):
    """CPU restatement on the inputs / injected randomness of `res`. `model` (any device) supplies
    the parameters; built on the CPU from the same seed when None."""
    from oracle.octo_ref import OctoRef, sequence_spec
    if model is None:
        from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
        model = Octo(cfg, "cpu", seed=res["seed"])
    images, text, actions = _inputs(model, res["B"], res["seed"])
    params, t5p = oracle_params(model)
    ref = OctoRef(cfg, params, t5p, emulate_bf16=emulate_bf16)
    tome = [_inject(x) for x in res["tome"]]
    rloss, _ = ref.forward_loss(text, images.astype(np.float32), actions, seed=1234, step=0,
                                positions=(res["rt"], res["ct"]), t=res["t"], eps=res["eps"],
                                tome_indices=tome,
                                sequence=sequence_spec(cfg.input_sequence, cfg.token_compression_sequence))
    rloss.backward()
    grads = {k: (v.grad.detach().numpy().copy() if v.grad is not None else np.zeros(v.shape, np.float32))
             for k, v in params.items()}
    return float(rloss.item()), grads


def compare(res, ref_loss, ref_grads):
    out = dict(loss=res["loss"], ref_loss=ref_loss, cos={}, ratio={}, rel={})
    ga, gb = [], []
    for name, a in res["grads"].items():
        a = torch.from_numpy(np.asarray(a, np.float64)).flatten()
        b = torch.from_numpy(np.asarray(ref_grads[name], np.float64)).flatten()
        ga.append(a)
        gb.append(b)
        na, nb = float(a.norm()), float(b.norm())
        out["cos"][name] = float((a @ b) / (na * nb)) if na > 0 and nb > 0 else (1.0 if na == nb else 0.0)
        out["ratio"][name] = na / nb if nb > 0 else (1.0 if na == 0 else float("inf"))
        out["rel"][name] = float((a - b).norm() / max(nb, 1e-30))
    A, Bv = torch.cat(ga), torch.cat(gb)
    out["cos_all"] = float((A @ Bv) / (A.norm() * Bv.norm()))
    return out


# ------------------------------------------------------------------ block-local (full depth)
def _cos_ratio(a, b):
    a = torch.as_tensor(np.asarray(a, np.float64)).flatten()
    b = torch.as_tensor(np.asarray(b, np.float64)).flatten()
    na, nb = float(a.norm()), float(b.norm())
    cos = float((a @ b) / (na * nb)) if na > 0 and nb > 0 else (1.0 if na == nb else 0.0)
    ratio = na / nb if nb > 0 else (1.0 if na == 0 else float("inf"))
    return cos, ratio, float((a - b).norm() / max(nb, 1e-30))


def hip_blockwise(cfg, B, seed=0):
    """HIP step with the backward run block by block so that every block's input, output,
    output gradient and input gradient can be handed to the oracle (teacher forcing)."""
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    dev = torch.device("cuda")
    model = Octo(cfg, dev, seed=seed)
    state = create_octo_train_state(model, seed=1234)
    images, text, actions = _inputs(model, B, seed)
    d_img = torch.from_numpy(images).to(dev)
    d_txt = torch.from_numpy(text).to(dev) if text is not None else None
    d_act = torch.from_numpy(actions).to(dev)
    model.store.zero_grad()
    loss, st = model.compute_diffusion_denoise_loss(d_txt, d_img, d_act, True, state.rng, 0)
    svs, ctxs = st["stack_sv"], st["ctxs"]
    dxL = model._backward_head(st)
    g = dxL
    nb = cfg.num_blocks
    douts, dins = [None] * nb, [None] * nb
    for i in reversed(range(nb)):
        douts[i] = g.cpu()
        g, _ = model.stack.blocks[i].backward(g, svs[i], ctxs[i])
        dins[i] = g.cpu()
    model._backward_tokens(st, g)
    torch.cuda.synchronize()
    n_tome = insitu_tome_check(model, st)
    n_prune = insitu_prune_check(model, st)
    f = lambda a: None if a is None else a.detach().float().cpu()  # noqa: E731
    return dict(model=model, B=B, seed=seed, loss=float(loss.item()),
                xs=[f(sv["x"]) for sv in svs], xL=f(st["xL"]), dxL=f(dxL), douts=douts, dins=dins,
                size_in=[_size_in(sv, f) for sv in svs],
                tome=[_used(sv) for sv in svs],
                prune_scores=[None if sv.get("prune") is None else f(sv["prune"][1]) for sv in svs],
                prune_layers_checked=n_prune,
                t5_out=f(st.get("t5_out")), rt=st["rt"].cpu().numpy(), ct=st["ct"].cpu().numpy(),
                t=st["head_sv"]["t"].cpu().numpy(), eps=st["head_sv"]["eps"].cpu().numpy(),
                grads={p.name: p.grad.detach().cpu().numpy().copy() for p in model.store.params},
                tome_layers_checked=n_tome)


def _size_arg(size, dt=None):
    """HIP per-set sizes (B, t) -> the oracle's (B, t, 1) (a dict per set with several)."""
    if size is None:
        return None
    if isinstance(size, dict):
        return {k: _size_arg(v, dt) for k, v in size.items()}
    size = size.unsqueeze(-1)
    return size if dt is None else size.to(dt)


def oracle_blockwise(cfg, res):
    """Teacher-forced oracle: each block gets the HIP block input and the HIP gradient arriving at
    its output; the head gets the HIP final sequence; the stem/assembly gets the HIP gradient of
    the assembled sequence (and the HIP T5 output, which test_t5_layerwise checks on its own).
    Returns per-piece activation / input-gradient agreement and per-parameter gradient agreement."""
    from oracle.octo_ref import OctoRef, sequence_spec
    model = res["model"]
    params, t5p = oracle_params(model)
    ref = OctoRef(cfg, params, t5p, emulate_bf16=True)
    seq = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)
    images, text, actions = _inputs(model, res["B"], res["seed"])
    out = dict(act={}, dinp={})
    nb = cfg.num_blocks
    for i in range(nb):
        x_in = res["xs"][i].clone().requires_grad_()
        size = _size_arg(res["size_in"][i])
        trace = {}
        xo, _, _ = ref.block(x_in, i, seq, size, seed=1234, step=0, tome_indices=res["tome"][i],
                             trace=trace)
        if res.get("prune_scores", [None] * nb)[i] is not None:
            out["act"][f"importance{i}"] = _cos_ratio(res["prune_scores"][i], trace[f"b{i}/imp"])
        want = res["xs"][i + 1] if i + 1 < nb else res["xL"]
        out["act"][f"block{i}"] = _cos_ratio(want, xo.detach())
        xo.backward(res["douts"][i])
        out["dinp"][f"block{i}"] = _cos_ratio(res["dins"][i], x_in.grad)
    xL = res["xL"].clone().requires_grad_()
    loss, _ = ref.head_loss(xL, seq, actions, res["t"], res["eps"])
    loss.backward()
    out["ref_loss"], out["loss"] = float(loss.item()), res["loss"]
    out["dinp"]["head"] = _cos_ratio(res["dxL"], xL.grad)
    img = ref.stem(images.astype(np.float32), (res["rt"], res["ct"]))
    txt = ref.text_proj(res["t5_out"]) if res["t5_out"] is not None else None
    x0 = ref.assemble(img, txt, seq, res["B"])
    out["act"]["assembly"] = _cos_ratio(res["xs"][0], x0.detach())
    x0.backward(res["dins"][0])
    out["cos"], out["ratio"] = {}, {}
    ga, gb = [], []
    for name, v in params.items():
        g = v.grad.numpy() if v.grad is not None else np.zeros(v.shape, np.float32)
        c, r, _ = _cos_ratio(res["grads"][name], g)
        out["cos"][name], out["ratio"][name] = c, r
        ga.append(np.asarray(res["grads"][name], np.float64).ravel())
        gb.append(np.asarray(g, np.float64).ravel())
    out["cos_all"] = _cos_ratio(np.concatenate(ga), np.concatenate(gb))[0]
    return out


def blockwise_floor(cfg, res, blocks):
    """CPU only: for the given blocks, the bf16-emulating block (fp32) against the same block in
    float64 without emulation, both fed the HIP block input and output gradient. Per-parameter
    (cos, ratio) of that comparison: how much of a block-local gradient difference the bf16
    storage points alone explain."""
    from oracle.octo_ref import OctoRef, sequence_spec
    model = res["model"]
    seq = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)
    out = {}
    for i in blocks:
        grads = []
        for emu, dt in ((True, torch.float32), (False, torch.float64)):
            params, t5p = oracle_params(model)
            params = {k: v.detach().to(dt).requires_grad_() for k, v in params.items()}
            ref = OctoRef(cfg, params, t5p, dtype=dt, emulate_bf16=emu)
            x_in = res["xs"][i].to(dt).requires_grad_()
            size = _size_arg(res["size_in"][i], dt)
            xo, _, _ = ref.block(x_in, i, seq, size, seed=1234, step=0, tome_indices=res["tome"][i])
            xo.backward(res["douts"][i].to(dt))
            pre = f"StackedEncoder1DBlock_0/Block_{i}/"
            grads.append({k: v.grad.double().numpy() for k, v in params.items()
                          if k.startswith(pre) and v.grad is not None})
        for k in grads[0]:
            out[k] = _cos_ratio(grads[0][k], grads[1][k])[:2]
    return out


# fp8 weight path (configs[4]): e4m3 keeps 3 mantissa bits and one scale per row, so a 1-ulp bf16
# difference upstream (fp32 summation order) can move a row's amax or an element across an e4m3
# rounding boundary (a 6 % step): block outputs agree to ~2e-2 and per-tensor gradient cosines to
# ~0.995 (measured min 0.9948 at 2 blocks, B = 2). Bar: SURVEY §8c's fp8 cosine >= 0.995 on the
# global gradient, >= 0.99 per tensor, block outputs within 3e-2.
FP8_BAR = dict(cos_min=0.99, ratio=(0.95, 1.05), act_rel=3e-2, cos_all_min=0.995)


def check_blockwise(out, cos_min=COS_MIN, ratio=NORM_RATIO, loss_rel=1e-3, act_rel=5e-3,
                    cos_all_min=0.998, cfg=None, res=None):
    """Block-local bar: every tensor's gradient cosine >= 0.999 with its norm ratio in
    [0.98, 1.02], and the concatenation's cosine >= 0.998 (the per-tensor norm
    ratios, each within 0.3 %, do not all lie on one line, which costs the global cosine a
    little: hi-res at B = 2 measures per tensor >= 0.99927, global 0.99891).

    With cfg and res: a block parameter below 0.999 is still accepted when the HIP-vs-oracle
    deviation is no larger than the bf16 floor of that tensor in that block (blockwise_floor:
    the emulating oracle vs float64 on the same block inputs) — the bias gradients of the
    first blocks are column sums over ~550 rows with heavy cancellation, where the bf16 storage
    points alone cost ~2e-3 of cosine (octo-small-prune16 seed 0: floor 0.99829, HIP 0.99874)."""
    assert abs(out["loss"] - out["ref_loss"]) <= loss_rel * abs(out["ref_loss"]), (out["loss"], out["ref_loss"])
    assert out["cos_all"] >= cos_all_min, out["cos_all"]
    bad = {k: v for k, v in out["act"].items() if v[2] > act_rel}
    assert not bad, f"block outputs differ: {bad}"
    bad = {k: v for k, v in out["dinp"].items() if v[0] < cos_min or not ratio[0] <= v[1] <= ratio[1]}
    assert not bad, f"input gradients differ: {bad}"
    bad = {k: (v, out["ratio"][k]) for k, v in out["cos"].items()
           if v < cos_min or not ratio[0] <= out["ratio"][k] <= ratio[1]}
    if bad and cfg is not None and res is not None:
        import re
        blocks = sorted({int(m.group(1)) for k in bad for m in [re.search(r"/Block_(\d+)/", k)] if m})
        fl = blockwise_floor(cfg, res, blocks) if blocks else {}
        out["floor_accepted"] = {k: (v, fl[k]) for k, v in bad.items()
                                 if k in fl and 1 - v[0] <= 1 - fl[k][0]
                                 and ratio[0] <= v[1] <= ratio[1]}
        bad = {k: v for k, v in bad.items() if k not in out["floor_accepted"]}
    assert not bad, f"parameter gradients differ: {dict(list(sorted(bad.items(), key=lambda kv: kv[1][0]))[:8])}"


def report_blockwise(out, n=10) -> str:
    lines = [f"loss {out['loss']:.6f} ref {out['ref_loss']:.6f} cos_all {out['cos_all']:.6f}"]
    worst_act = max(out["act"].items(), key=lambda kv: kv[1][2])
    worst_din = min(out["dinp"].items(), key=lambda kv: kv[1][0])
    lines.append(f"  worst activation rel {worst_act[1][2]:.2e} ({worst_act[0]}); "
                 f"worst input-grad cos {worst_din[1][0]:.6f} ratio {worst_din[1][1]:.4f} ({worst_din[0]})")
    for k, v in sorted(out["cos"].items(), key=lambda kv: kv[1])[:n]:
        lines.append(f"  cos {v:.6f} ratio {out['ratio'][k]:.4f}  {k}")
    return "\n".join(lines)


def bf16_floor(cfg, res, model):
    """CPU only, no HIP: the bf16-emulating restatement against the same restatement in float64,
    on the HIP run's inputs and injected randomness. How far ANY implementation that rounds at
    the build's storage points drifts from exact arithmetic at this depth — the reference point
    of the free-running end-to-end bar (the network amplifies bf16 noise with depth)."""
    (l_emu, g_emu), (l_f64, g_f64) = oracle_pair(cfg, res, model)
    return compare(dict(res, loss=l_emu, grads=g_emu), l_f64, g_f64)


def oracle_pair(cfg, res, model):
    """The bf16-emulating restatement (fp32) and the exact one (float64, no emulation) on the HIP
    run's inputs / injected randomness: [(loss, {name: grad}) emu, (loss, grads) float64]."""
    from oracle.octo_ref import OctoRef, sequence_spec
    images, text, actions = _inputs(model, res["B"], res["seed"])
    tome = [_inject(x) for x in res["tome"]]
    seq = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)
    outs = []
    for emu, dt in ((True, torch.float32), (False, torch.float64)):
        params, t5p = oracle_params(model)
        params = {k: v.detach().to(dt).requires_grad_() for k, v in params.items()}
        t5p = None if t5p is None else {k: v.to(dt) for k, v in t5p.items()}
        ref = OctoRef(cfg, params, t5p, dtype=dt, emulate_bf16=emu)
        loss, _ = ref.forward_loss(text, images.astype(np.float32), actions, seed=1234, step=0,
                                   positions=(res["rt"], res["ct"]), t=res["t"], eps=res["eps"],
                                   tome_indices=tome, sequence=seq)
        loss.backward()
        outs.append((float(loss.item()), {k: (v.grad.double().numpy() if v.grad is not None
                                               else np.zeros(v.shape)) for k, v in params.items()}))
    return outs


def run_parity(cfg, B, seed=0, floor=False):
    res = hip_step(cfg, B, seed)
    ref_loss, ref_grads = oracle_step(cfg, res, model=res["model"])
    out = compare(res, ref_loss, ref_grads)
    out["tome_layers_checked"] = res["tome_layers_checked"]
    out["prune_layers_checked"] = res["prune_layers_checked"]
    if floor:
        out["floor"] = bf16_floor(cfg, res, res["model"])
    return out


def check_against_floor(out, k=2.0, slack_all=1e-3, slack_min=2e-3):
    """Free-running bar: HIP vs the bf16-emulating oracle may deviate at most k times as much as
    the oracle's own bf16 rounding deviates from float64 (plus a small absolute slack), in loss,
    global gradient cosine and the worst per-tensor cosine."""
    f = out["floor"]
    lr = abs(out["loss"] / out["ref_loss"] - 1)
    flr = abs(f["loss"] / f["ref_loss"] - 1)
    assert lr <= k * flr + 2e-3, (lr, flr)
    assert 1 - out["cos_all"] <= k * (1 - f["cos_all"]) + slack_all, (out["cos_all"], f["cos_all"])
    hmin, fmin = min(out["cos"].values()), min(f["cos"].values())
    assert 1 - hmin <= k * (1 - fmin) + slack_min, (hmin, fmin)


def check_against_floor_seeds(outs, k_loss=2.0, k_cos=1.5, slack=2e-3):
    """Free-running bar at full depth, over seeds. There the bf16 storage noise alone (the
    emulating oracle vs float64: the floor) moves the loss by 0.03 % .. 16 % and the global
    gradient cosine down to 0.58 .. 0.90 depending on the seed (sequence-axis LayerNorms over
    12 blocks amplify it; the merge indices are the HIP run's, injected), so one seed's HIP/floor
    ratio is a ratio of two random draws. The bar compares medians over the seeds instead: HIP vs
    the emulating oracle within k_loss x the floor's median loss deviation and k_cos x its median
    cosine deficits (global and worst tensor). Measured (round 4, tools/noise_sources.py,
    octo-small-tome16 seeds 0-5): HIP 0.56x the floor's median loss deviation and 1.20x its
    median global cosine deficit; the deterministic mode gives the same numbers and reruns are
    bitwise equal at B = 2, so fp32 atomic order contributes nothing measurable here — what HIP
    adds beyond the bf16 storage rounding is fp32 summation order (MFMA / reductions) and
    v_exp_f32. Round 3's bar was 4x / 2x (then 3x measured in loss)."""
    import statistics as st

    def med(f):
        return st.median(f(o) for o in outs)
    lr = med(lambda o: abs(o["loss"] / o["ref_loss"] - 1))
    flr = med(lambda o: abs(o["floor"]["loss"] / o["floor"]["ref_loss"] - 1))
    assert lr <= k_loss * flr + slack, (lr, flr)
    ca = med(lambda o: 1 - o["cos_all"])
    fca = med(lambda o: 1 - o["floor"]["cos_all"])
    assert ca <= k_cos * fca + slack, (ca, fca)
    cm = med(lambda o: 1 - min(o["cos"].values()))
    fcm = med(lambda o: 1 - min(o["floor"]["cos"].values()))
    assert cm <= k_cos * fcm + slack, (cm, fcm)
    return dict(loss=(lr, flr), cos_all=(ca, fca), min_cos=(cm, fcm))


def check(res, cos_min=COS_MIN, cos_all_min=COS_ALL_MIN, loss_rel=LOSS_RTOL, ratio=NORM_RATIO):
    assert abs(res["loss"] - res["ref_loss"]) <= loss_rel * abs(res["ref_loss"]), \
        (res["loss"], res["ref_loss"])
    bad = {k: v for k, v in res["cos"].items() if v < cos_min}
    assert not bad, f"low gradient cosine: {dict(list(sorted(bad.items(), key=lambda kv: kv[1]))[:8])}"
    badr = {k: v for k, v in res["ratio"].items() if not ratio[0] <= v <= ratio[1]}
    assert not badr, f"gradient norm ratio out of {ratio}: {dict(list(badr.items())[:8])}"
    assert res["cos_all"] >= cos_all_min, res["cos_all"]


def report(res, n=12) -> str:
    worst = sorted(res["cos"].items(), key=lambda kv: kv[1])[:n]
    lines = [f"loss {res['loss']:.6f} ref {res['ref_loss']:.6f} "
             f"rel {abs(res['loss'] - res['ref_loss']) / abs(res['ref_loss']):.2e} cos_all {res['cos_all']:.6f}"]
    for k, v in worst:
        lines.append(f"  cos {v:.6f} ratio {res['ratio'][k]:.4f} rel {res['rel'][k]:.3e}  {k}")
    rat = sorted(res["ratio"].items(), key=lambda kv: abs(np.log(max(kv[1], 1e-30))))[-4:]
    for k, v in rat:
        lines.append(f"  ratio {v:.4f} cos {res['cos'][k]:.6f}  {k}")
    return "\n".join(lines)
