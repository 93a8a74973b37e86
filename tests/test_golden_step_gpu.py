"""The HIP training step against the committed §8c step fixtures (tests/golden/step_*_golden.npz,
written on the CPU by tests/golden/make_step_golden.py from the oracle alone: its own counter-
stream restatements for the randomness and its own canonical ToMe matching — nothing from a HIP
run). B = 2 at the reference's geometry (ref_octo_base, one block, Dh 256) and at OCTO-small with
ToMe r = 16 over two blocks.

Exact: the patch position tokens and diffusion t (oracle/rng.py restatements of the counter
streams, reference image_tokenizer.py:74-132, diffusion.py:124) and every ToMe index triple the
HIP matching kernel computes from the fixture's stored metric (the restatement's bf16 K of the
merged set; token_compression.py:54-112, bit-exact by the build's canonical arithmetic). The
step's OWN keys differ from the restatement's by fp32 summation order (MFMA vs CPU), which can
swap two near-tied scores, so the fixture's indices are then injected into the HIP step
(inject["tome"]) for the end-to-end comparison; the step's own matching is checked in situ by
the parity tests (oracle/parity.py). eps: Box-Muller in fp32, the device's logf / cosf vs
numpy's, rtol 1e-5.

Within bars, HIP against the EXACT restatement (float64, no storage rounding: "f64"); the floor
is how far the bf16-emulating restatement ("emu": rounding at every point where the build stores
bf16) lies from that same exact result — what bf16 storage alone costs an honest implementation
(round 5: the round-4 test measured HIP against emu, which is itself a bf16 result; on
small_tome16_2blk HIP is the closer of the two to exact on 50 of the 51 gradient tensors, median
error 0.70x the emulation's — profiles/r05_golden_exact.txt):
  * block inputs, final sequence, loss: relative (L2) <= max(2e-2, 2 x floor);
  * every parameter gradient: relative L2 <= max(5e-2, 2 x floor) (SURVEY §8c rtol 5e-2);
  * the global gradient cosine >= 0.999, or within twice the floor's deficit.
The norm ratio |g| / |g_exact| of one fixture is one draw of bf16 noise (on the cancellation-
heavy first-block bias sums both bf16 implementations err by ~7 %, and the projection of that
error on the gradient moves the norm by a few per cent either way), so it is not barred per
fixture: test_gradients_against_exact_over_seeds bars it over 8 seeds, per tensor, without a
floor term: the median ratio within 0.02 of 1, and HIP's median error at
most 1.3x the emulation's.
"""
import ast
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"


def _cos(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    na, nb = np.linalg.norm(a), np.linalg.norm(b)
    return float(a @ b / (na * nb)) if na > 0 and nb > 0 else (1.0 if na == nb else 0.0)


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _view(z, key, full):
    """The stored sample of `key` and the same positions of the full array `full`."""
    if f"{key}:all" in z:
        return z[f"{key}:all"], np.asarray(full, np.float64).ravel()
    idx = z[f"{key}:idx"]
    return z[f"{key}:val"], np.asarray(full, np.float64).ravel()[idx]


@pytest.mark.parametrize("tag", ["ref_octo_base", "small_tome16_2blk"])
def test_step_matches_golden_fixture(dev, tag):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    z = np.load(GOLDEN / f"step_{tag}_golden.npz")  # our own fixture; allow_pickle stays False
    cfg = get_config(str(z["config"]), **ast.literal_eval(str(z["overrides"])))
    model = Octo(cfg, dev, seed=int(z["seed"]))
    state = create_octo_train_state(model, seed=int(z["rng_seed"]))
    img = torch.from_numpy(z["images"]).to(dev)
    txt = torch.from_numpy(z["text"]).to(dev) if "text" in z else None
    act = torch.from_numpy(z["actions"]).to(dev)
    # the HIP matching kernel on the fixture's metric reproduces the fixture's indices exactly
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    inject_tome = None
    if int(z["n_tome"]):
        inject_tome = []
        for li in range(cfg.num_blocks):
            bits = torch.from_numpy(z[f"tome{li}/metric_bf16"].astype(np.int16))
            got = K.tome_match(bits.view(torch.bfloat16).to(dev), cfg.tome_r)
            for nm, g in zip(("unm", "src", "dst"), got):
                np.testing.assert_array_equal(g.cpu().numpy(), z[f"tome{li}/{nm}"], err_msg=f"block {li} {nm}")
            inject_tome.append(got)
    model.store.zero_grad()
    loss, st = model.compute_diffusion_denoise_loss(txt, img, act, True, state.rng, 0,
                                                    inject=dict(tome=inject_tome))
    model.backward(st)
    torch.cuda.synchronize()
    report, bad = [], []
    # exact randomness
    np.testing.assert_array_equal(st["rt"].cpu().numpy(), z["rt"])
    np.testing.assert_array_equal(st["ct"].cpu().numpy(), z["ct"])
    np.testing.assert_array_equal(st["head_sv"]["t"].cpu().numpy().ravel(), z["t"].ravel())
    np.testing.assert_allclose(st["head_sv"]["eps"].cpu().numpy().reshape(z["eps"].shape), z["eps"],
                               rtol=1e-5, atol=1e-6)
    assert sum(sv["tome"] is not None for sv in st["stack_sv"]) == int(z["n_tome"])
    # activations (vs the exact restatement; floor = emu vs exact)
    acts = [(f"x{i}", sv["x"]) for i, sv in enumerate(st["stack_sv"])] + [("xL", st["xL"])]
    for key, t in acts:
        full = t.float().cpu().numpy()
        f64, hip = _view(z, f"f64/{key}", full)
        emu = _view(z, f"emu/{key}", full)[0]
        r, fl = _rel(hip, f64), _rel(emu, f64)
        report.append(f"{key}: rel {r:.2e} (floor {fl:.2e})")
        if r > max(2e-2, 2 * fl):
            bad.append((key, r, fl))
    # loss
    lh, le, lf = float(loss.item()), float(z["emu/loss"]), float(z["f64/loss"])
    rl, fl = abs(lh / lf - 1), abs(le / lf - 1)
    report.append(f"loss {lh:.6f} emu {le:.6f} f64 {lf:.6f}: rel {rl:.2e} (floor {fl:.2e})")
    if rl > max(2e-2, 2 * fl):
        bad.append(("loss", lh, le, lf))
    # gradients
    worst, all_h, all_e, all_f = [], [], [], []
    for p in model.store.params:
        key = f"f64/grad/{p.name}"
        full = p.grad.detach().float().cpu().numpy()
        f64, hip = _view(z, key, full)
        emu = _view(z, f"emu/grad/{p.name}", full)[0]
        nf, ne = float(z[f"{key}:norm"]), float(z[f"emu/grad/{p.name}:norm"])
        nh = float(np.linalg.norm(full.astype(np.float64)))
        if nf == 0 and nh == 0:
            continue
        r, rfl = _rel(hip, f64), _rel(emu, f64)
        ratio, rf = nh / nf, ne / nf
        worst.append((r, p.name, rfl, ratio, rf, _cos(hip, f64)))
        all_h.append(np.asarray(hip, np.float64))
        all_e.append(np.asarray(emu, np.float64))
        all_f.append(np.asarray(f64, np.float64))
        if r > max(5e-2, 2 * rfl):
            bad.append((p.name, r, rfl, ratio, rf))
    worst.sort(reverse=True)
    cg = _cos(np.concatenate(all_h), np.concatenate(all_f))
    cgf = _cos(np.concatenate(all_e), np.concatenate(all_f))
    report.append(f"gradients: global cosine {cg:.6f} (floor {cgf:.6f})")
    for r, name, rfl, ratio, rf, c in worst[:6]:
        report.append(f"  grad rel {r:.3e} (floor {rfl:.3e}) cos {c:.6f} ratio {ratio:.4f} (floor {rf:.4f}) {name}")
    print(f"\n[{tag}] " + "\n".join(report))
    assert cg >= 0.999 or 1 - cg <= 2 * (1 - cgf) + 1e-4, (cg, cgf)
    assert not bad, bad


def test_gradients_against_exact_over_seeds(dev):
    """Per parameter tensor over 8 seeds of the OCTO-small ToMe r = 16 step (2 blocks, B = 2,
    2-layer T5; each seed its own parameters, inputs and randomness; the oracle on the HIP run's
    injected randomness and ToMe indices), HIP and the bf16-emulating restatement both against the
    EXACT float64 restatement (oracle.parity.oracle_pair), as tools/parity_exact.py measures it:
      * the median over seeds of |g_hip| / |g_exact| within 0.02 of 1 — no systematic shrink or
        growth of any tensor, the block-0 bias sums included, with no floor term;
      * the median over seeds of err_hip / err_emu (relative L2 to exact) at most 1.3 — HIP's
        fp32 summation order and v_exp_f32 may add to the bf16 storage error, not multiply it;
      * the global gradient: median norm ratio within 0.01 of 1, median cosine >= 0.99.
    The table it prints is profiles/r06_golden_multiseed.txt."""
    import statistics as stt

    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    from oracle import parity as P
    cfg = get_config("octo-small-tome16", num_blocks=2, t5=T5Config(num_layers=2))
    per, glob = {}, []
    for seed in range(8):
        h = P.hip_step(cfg, 2, seed)
        (_, ge), (_, gf) = P.oracle_pair(cfg, h, h["model"])
        H, F = [], []
        for k in sorted(gf):
            f = np.asarray(gf[k], np.float64).ravel()
            n = np.linalg.norm(f)
            if n == 0:
                continue
            hh = np.asarray(h["grads"][k], np.float64).ravel()
            ee = np.asarray(ge[k], np.float64).ravel()
            eh, em = np.linalg.norm(hh - f) / n, np.linalg.norm(ee - f) / n
            per.setdefault(k, []).append((np.linalg.norm(hh) / n, eh, em, eh / max(em, 1e-30)))
            H.append(hh)
            F.append(f)
        H, F = np.concatenate(H), np.concatenate(F)
        glob.append((np.linalg.norm(H) / np.linalg.norm(F), _cos(H, F)))
        del h
    lines, bad = [], []
    for k, v in sorted(per.items()):
        ratio = stt.median(x[0] for x in v)
        err_ratio = stt.median(x[3] for x in v)
        lines.append(f"  ratio {ratio:.4f} [{min(x[0] for x in v):.4f}, {max(x[0] for x in v):.4f}]"
                     f"  err hip {stt.median(x[1] for x in v):.2e} emu {stt.median(x[2] for x in v):.2e}"
                     f"  hip/emu {err_ratio:.3f}  {k}")
        if abs(ratio - 1) > 0.02 or err_ratio > 1.3:
            bad.append((k, ratio, err_ratio))
    gr, gc = stt.median(x[0] for x in glob), stt.median(x[1] for x in glob)
    print(f"\n8 seeds, octo-small-tome16 2 blocks B = 2 vs float64: global norm ratio median {gr:.4f}, "
          f"cosine median {gc:.5f}; err_hip/err_emu median over tensors "
          f"{stt.median(stt.median(x[3] for x in v) for v in per.values()):.3f}\n" + "\n".join(lines))
    assert abs(gr - 1) <= 0.01 and gc >= 0.99, (gr, gc)
    assert not bad, bad
