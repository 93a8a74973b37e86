"""Generate tests/golden/step_*_golden.npz: the SURVEY §8c step fixtures — one diffusion training
step (forward loss + every parameter gradient) of the CPU restatement (oracle/octo_ref.py), with
its randomness produced by the oracle's own restatements of the counter streams (oracle/rng.py:
dropout keep-masks, patch position tokens, diffusion t and eps) and its ToMe indices chosen by the
canonical matching (oracle/tome_ref.c) on its own keys. Nothing is taken from a HIP run: the
GPU test (tests/test_golden_step_gpu.py) runs the HIP step on the same inputs and must reproduce
the positions, t and the ToMe indices exactly, eps to a few ulp, and the activations, loss and
gradients within the bf16 bars.

Configs (B = 2): the reference's own geometry `ref_octo_base` (reference model_configs/
octo_base.yaml + vanilla_decoder.yaml + gato_resnet.yaml: D 768, 3 heads of 256, one block, 2-step
280^2 images, patch 56, 16 text tokens; reference files attention.py:20-119,
image_tokenizer.py:35-178, diffusion.py:110-143) and OCTO-small with ToMe r = 16 at two blocks
(token_compression.py:54-129 on the merge path).

Stored per fixture: the inputs, rt / ct / t / eps, the ToMe index triples, the loss of the
bf16-emulating restatement (fp32) and of the exact one (float64, no emulation: the bf16 floor),
every block input, the final sequence and every parameter gradient — tensors up to 2048 values
whole, larger ones as 1024 values at seeded positions (+ the full norm), both for the emulating
and the float64 run.

    python tests/golden/make_step_golden.py      (CPU, ~1 min; no GPU, no network)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo  # noqa: E402
from oracle import rng as R  # noqa: E402
from oracle.octo_ref import OctoRef, sequence_spec  # noqa: E402
from oracle.parity import _inputs, oracle_params  # noqa: E402

FIXTURES = {
    "ref_octo_base": dict(config="ref_octo_base", overrides={}, seed=0),
    "small_tome16_2blk": dict(config="octo-small-tome16", overrides=dict(num_blocks=2), seed=0),
}
B = 2
RNG_SEED, RNG_STEP = 1234, 0   # create_octo_train_state(model, seed=1234), first step
WHOLE, SAMPLE = 2048, 1024


def sample_index(name: str, n: int) -> np.ndarray:
    g = np.random.default_rng(abs(hash_name(name)) % (2 ** 32))
    return np.sort(g.choice(n, size=SAMPLE, replace=False)).astype(np.int64)


def hash_name(s: str) -> int:
    h = 1469598103934665603
    for ch in s.encode():
        h = ((h ^ ch) * 1099511628211) % (1 << 63)
    return h


def pack(out: dict, key: str, arr: np.ndarray):
    a = np.asarray(arr, np.float64).ravel()
    out[f"{key}:norm"] = np.float64(np.linalg.norm(a))
    if a.size <= WHOLE:
        out[f"{key}:all"] = a.astype(np.float32)
    else:  # the same positions for the emu and f64 copies of a tensor
        idx = sample_index(key.split("/", 1)[1], a.size)
        out[f"{key}:idx"] = idx
        out[f"{key}:val"] = a[idx].astype(np.float32)


def run(cfg, model, images, text, actions, positions, t, eps, emulate, dtype, tome=None):
    params, t5p = oracle_params(model)
    params = {k: v.detach().to(dtype).requires_grad_() for k, v in params.items()}
    t5p = None if t5p is None else {k: v.to(dtype) for k, v in t5p.items()}
    ref = OctoRef(cfg, params, t5p, dtype=dtype, emulate_bf16=emulate)
    record, trace = [], {}
    loss, ex = ref.forward_loss(text, images.astype(np.float32), actions, seed=RNG_SEED, step=RNG_STEP,
                                positions=positions, t=t, eps=eps, record=record, tome_indices=tome,
                                sequence=sequence_spec(cfg.input_sequence, cfg.token_compression_sequence),
                                trace=trace)
    run.trace = trace
    loss.backward()
    grads = {k: (v.grad.double().numpy() if v.grad is not None else np.zeros(v.shape)) for k, v in params.items()}
    xs = [x.detach().double().numpy() for x in record]
    return float(loss.item()), grads, xs, ex["x_final"].detach().double().numpy(), ex["tome"]


def make(tag, spec):
    cfg = get_config(spec["config"], **spec["overrides"])
    model = Octo(cfg, torch.device("cpu"), seed=spec["seed"])
    images, text, actions = _inputs(model, B, spec["seed"])
    it = model.image_tokenizer
    rt, ct = R.patch_positions(RNG_SEED, RNG_STEP, 0, B, model.n_images, cfg.image_size[0],
                               it.patch_size, it.Q)
    t, eps = R.diffusion_t_eps(RNG_SEED, RNG_STEP, B, cfg.action_space_dim, cfg.diffusion_steps)
    out = dict(config=np.array(spec["config"]), overrides=np.array(repr(spec["overrides"])),
               seed=np.int64(spec["seed"]), B=np.int64(B), rng_seed=np.int64(RNG_SEED),
               rng_step=np.int64(RNG_STEP), images=images, actions=actions, rt=rt, ct=ct, t=t, eps=eps)
    if text is not None:
        out["text"] = text
    runs = {"emu": run(cfg, model, images, text, actions, (rt, ct), t, eps, True, torch.float32)}
    emu_trace = run.trace
    tome = runs["emu"][4]
    # the float64 floor merges with the same indices (a near-tie must not change the merge)
    # (the ToMe configs merge in every block: tome[li] is block li's triple)
    assert not tome or len(tome) == cfg.num_blocks
    inj = [tuple(torch.as_tensor(np.asarray(a)) for a in tr) for tr in tome] if tome else None
    runs["f64"] = run(cfg, model, images, text, actions, (rt, ct), t, eps, False, torch.float64, inj)
    runs_trace = {"emu_trace": emu_trace}
    trace = runs_trace["emu_trace"]
    seq = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)
    D, H = cfg.token_embedding_dim, cfg.num_heads
    for li, (unm, src, dst) in enumerate(tome):
        for nm, a in (("unm", unm), ("src", src), ("dst", dst)):
            out[f"tome{li}/{nm}"] = np.asarray(a, np.int32)
        # the metric the indices were matched on: K (bf16 values) of the merged set, all heads
        si = next(i for i, c in enumerate(seq) if c[3] > 0)
        s0 = sum(c[1] - li * c[3] for c in seq[:si])
        tt = seq[si][1] - li * seq[si][3]
        qkv = trace[f"b{li}/qkv"].float().numpy()
        metric = np.ascontiguousarray(qkv[:, s0:s0 + tt, D:2 * D].reshape(qkv.shape[0], tt, H, D // H))
        bits = metric.view(np.uint32)
        assert (bits & 0xFFFF == 0).all()  # bf16 values stored exactly
        out[f"tome{li}/metric_bf16"] = (bits >> 16).astype(np.uint16)
        out[f"tome{li}/s0"], out[f"tome{li}/t"] = np.int64(s0), np.int64(tt)
    out["n_tome"] = np.int64(len(tome))
    for kind, (loss, grads, xs, xL, _) in runs.items():
        out[f"{kind}/loss"] = np.float64(loss)
        for i, x in enumerate(xs):
            pack(out, f"{kind}/x{i}", x)
        pack(out, f"{kind}/xL", xL)
        for name, g in grads.items():
            pack(out, f"{kind}/grad/{name}", g)
    path = HERE / f"step_{tag}_golden.npz"
    np.savez_compressed(path, **out)
    print(f"{path.name}: loss emu {runs['emu'][0]:.6f} f64 {runs['f64'][0]:.6f}, "
          f"{len(runs['emu'][1])} gradients, {len(runs['emu'][2])} blocks, {len(tome)} ToMe layers, "
          f"{path.stat().st_size / 1e6:.2f} MB")


if __name__ == "__main__":
    torch.manual_seed(0)
    for tag, spec in FIXTURES.items():
        make(tag, spec)
