"""Locate where the HIP step's gradients leave the bf16-emulating oracle.

  python tools/golden_diag.py dump  [tag]   (GPU)  -> gpurun_out/golden_dump_<tag>.npz
  python tools/golden_diag.py compare [tag] (CPU)  reads that dump, reruns the oracle (emu and
                                                   float64) with retained intermediate gradients

The GPU side runs the test_golden_step_gpu.py step (fixture inputs, injected ToMe indices) and
records, in backward order, every Dense input gradient (keyed by the weight's name), the
attention backward's dqkv, each block's input gradient and every parameter gradient. The CPU side
reports, per intermediate, the relative L2 error, the cosine and the projection coefficient
a = <hip, emu> / |emu|^2 (a systematic shrink shows as a < 1 beyond the noise), for the tensor and
for its column sums over the token rows (what a bias gradient sees), next to the same numbers for
the float64 restatement (the bf16 floor).
"""
from __future__ import annotations

import ast
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"
OUT = ROOT / "gpurun_out"


def dump(tag):
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from multi_modal_transformers_tokenmerge_amd import layers as Ly
    from multi_modal_transformers_tokenmerge_amd.attention_blocks import attention as A
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo, create_octo_train_state
    dev = torch.device("cuda:0")
    z = np.load(GOLDEN / f"step_{tag}_golden.npz")
    cfg = get_config(str(z["config"]), **ast.literal_eval(str(z["overrides"])))
    model = Octo(cfg, dev, seed=int(z["seed"]))
    state = create_octo_train_state(model, seed=int(z["rng_seed"]))
    rec = {}

    def keep(key, t):  # bf16 tensors as their bits (half the bytes; the copy-back is capped)
        torch.cuda.synchronize()
        t = t.detach()
        rec[key] = (t.contiguous().view(torch.int16).cpu().numpy() if t.dtype == torch.bfloat16
                    else t.float().cpu().numpy())

    fb = Ly.Dense.bwd

    def dense_bwd(self, dy2d, x2d, *a, **kw):
        out = fb(self, dy2d, x2d, *a, **kw)
        if "StackedEncoder" in self.w.name:  # the blocks only (the patch-56 stem's are 100s of MB)
            if out is not None:
                keep(f"dX/{self.w.name}", out)
            keep(f"dY/{self.w.name}", dy2d)
        return out
    Ly.Dense.bwd = dense_bwd
    fa = K.attn_bwd

    def attn_bwd(*a, **kw):
        out = fa(*a, **kw)
        keep(f"dqkv/{len([k for k in rec if k.startswith('dqkv/')])}", out)
        return out
    K.attn_bwd = attn_bwd
    fblk = A.Encoder1DBlock.backward

    def blk_bwd(self, dx2, sv, ctx, dz2=None, prev=None):
        keep(f"dout/{ctx.layer}", dx2)
        dx, dz = fblk(self, dx2, sv, ctx, dz2=dz2, prev=prev)
        keep(f"din/{ctx.layer}", dx)
        return dx, dz
    A.Encoder1DBlock.backward = blk_bwd
    img = torch.from_numpy(z["images"]).to(dev)
    txt = torch.from_numpy(z["text"]).to(dev) if "text" in z else None
    act = torch.from_numpy(z["actions"]).to(dev)
    inject_tome = None
    if int(z["n_tome"]):
        inject_tome = []
        for li in range(cfg.num_blocks):
            bits = torch.from_numpy(z[f"tome{li}/metric_bf16"].astype(np.int16))
            inject_tome.append(K.tome_match(bits.view(torch.bfloat16).to(dev), cfg.tome_r))
    model.store.zero_grad()
    loss, st = model.compute_diffusion_denoise_loss(txt, img, act, True, state.rng, 0,
                                                    inject=dict(tome=inject_tome))
    model.backward(st)
    torch.cuda.synchronize()
    for li, sv in enumerate(st["stack_sv"]):
        for k in ("qkv", "o", "y0", "y1", "h"):
            if sv.get(k) is not None:
                keep(f"act/b{li}/{k}", sv[k])
    for p in model.store.params:  # small tensors whole, large ones at 4096 seeded positions
        g = p.grad.detach().float().reshape(-1)
        if g.numel() <= 4096:
            rec[f"grad/{p.name}"] = g.cpu().numpy()
        else:
            idx = np.sort(np.random.default_rng(len(p.name)).choice(g.numel(), 4096, replace=False))
            rec[f"grad/{p.name}:idx"] = idx
            rec[f"grad/{p.name}"] = g[torch.from_numpy(idx).to(g.device)].cpu().numpy()
    rec["loss"] = np.float64(loss.item())
    OUT.mkdir(exist_ok=True)
    np.savez_compressed(OUT / f"golden_dump_{tag}.npz", **rec)
    print(f"dumped {len(rec)} arrays, loss {rec['loss']:.6f}")


def _oracle(tag, emulate, dtype):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    from oracle.octo_ref import OctoRef, sequence_spec
    from oracle.parity import oracle_params
    z = np.load(GOLDEN / f"step_{tag}_golden.npz")
    cfg = get_config(str(z["config"]), **ast.literal_eval(str(z["overrides"])))
    model = Octo(cfg, torch.device("cpu"), seed=int(z["seed"]))
    params, t5p = oracle_params(model)
    params = {k: v.detach().to(dtype).requires_grad_() for k, v in params.items()}
    t5p = None if t5p is None else {k: v.to(dtype) for k, v in t5p.items()}
    ref = OctoRef(cfg, params, t5p, dtype=dtype, emulate_bf16=emulate)
    tome = None
    if int(z["n_tome"]):
        tome = [tuple(torch.as_tensor(z[f"tome{li}/{nm}"]) for nm in ("unm", "src", "dst"))
                for li in range(cfg.num_blocks)]
    record, trace = [], {"_retain": True}
    text = z["text"] if "text" in z else None
    loss, ex = ref.forward_loss(text, z["images"].astype(np.float32), z["actions"], seed=int(z["rng_seed"]),
                                step=0, positions=(z["rt"], z["ct"]), t=z["t"], eps=z["eps"],
                                record=record, tome_indices=tome,
                                sequence=sequence_spec(cfg.input_sequence, cfg.token_compression_sequence),
                                trace=trace)
    xf = ex["x_final"]
    xf.retain_grad()
    loss.backward()
    out = {"loss": float(loss.item()), "dxL": xf.grad.double().numpy()}
    for li, x in enumerate(record):
        out[f"din/{li}"] = x.grad.double().numpy()
    for k, v in trace.items():
        if k.startswith("b") and torch.is_tensor(v) and v.grad is not None:
            out[f"g/{k}"] = v.grad.double().numpy()
    for k, v in params.items():
        out[f"grad/{k}"] = (v.grad.double().numpy() if v.grad is not None else np.zeros(v.shape))
    return out


def _stats(h, e):
    h, e = np.asarray(h, np.float64).ravel(), np.asarray(e, np.float64).ravel()
    ne = np.linalg.norm(e)
    if ne == 0:
        return float("nan"), float("nan"), float("nan")
    rel = np.linalg.norm(h - e) / ne
    cos = h @ e / max(np.linalg.norm(h) * ne, 1e-300)
    a = h @ e / ne ** 2
    return rel, cos, a


def _load_dump(tag):
    z = np.load(OUT / f"golden_dump_{tag}.npz")
    out = {}
    for k in z.files:
        a = z[k]
        out[k] = (a.astype(np.uint16).astype(np.uint32) << 16).view(np.float32) if a.dtype == np.int16 else a
    return out


def compare(tag):
    hip = _load_dump(tag)
    emu = _oracle(tag, True, torch.float32)
    f64 = _oracle(tag, False, torch.float64)
    print(f"loss hip {float(hip['loss']):.6f} emu {emu['loss']:.6f} f64 {f64['loss']:.6f}")
    D = None
    pairs = []
    nb = len([k for k in emu if k.startswith("din/")])
    for li in reversed(range(nb)):
        pre = f"StackedEncoder1DBlock_0/Block_{li}"
        pairs += [(f"b{li} dz1 (Dense_0 out)", f"dY/{pre}/MLPBlock_0/Dense_0/kernel", None),
                  (f"b{li} dy1", f"dX/{pre}/MLPBlock_0/Dense_0/kernel", f"g/b{li}/y1"),
                  (f"b{li} do", f"dX/{pre}/SelfAttention_0/out/kernel", f"g/b{li}/o"),
                  (f"b{li} dqkv", f"dqkv/{nb - 1 - li}", f"g/b{li}/qkv"),
                  (f"b{li} dy0", f"dX/{pre}/SelfAttention_0/qkv/kernel", f"g/b{li}/y0"),
                  (f"b{li} dx (block input)", f"din/{li}", f"din/{li}")]
    print(f"{'intermediate':28s} {'rel':>9s} {'cos':>9s} {'a':>8s} | {'colsum rel':>10s} {'a':>8s} "
          f"|| floor: {'rel':>9s} {'a':>8s} | {'colsum rel':>10s} {'a':>8s}")
    for name, hk, ok in pairs:
        if ok is None or hk not in hip or ok not in emu:
            continue
        e, f = emu[ok], f64[ok]
        h = hip[hk].reshape(e.shape)
        D = e.shape[-1]
        r, c, a = _stats(h, e)
        rf, cf, af = _stats(f, e)
        hc, ec, fc = (np.asarray(v, np.float64).reshape(-1, D).sum(0) for v in (h, e, f))
        r2, _, a2 = _stats(hc, ec)
        r2f, _, a2f = _stats(fc, ec)
        print(f"{name:28s} {r:9.3e} {c:9.6f} {a:8.4f} | {r2:10.3e} {a2:8.4f} || {rf:9.3e} {af:8.4f} | "
              f"{r2f:10.3e} {a2f:8.4f}")
        if name.endswith("dqkv"):  # the q / k / v thirds of the bias gradient
            for j, nm in enumerate("qkv"):
                s = slice(j * D // 3, (j + 1) * D // 3)
                r3, _, a3 = _stats(hc[s], ec[s])
                r3f, _, a3f = _stats(fc[s], ec[s])
                print(f"{'   colsum ' + nm:28s} {'':9s} {'':9s} {'':8s} | {r3:10.3e} {a3:8.4f} || "
                      f"{'':9s} {'':8s} | {r3f:10.3e} {a3f:8.4f}  |emu| {np.linalg.norm(ec[s]):.3e}")
    print("\nparameter gradients (worst projection first)")
    rows = []
    for k in emu:
        if not k.startswith("grad/") or k not in hip:
            continue
        e, f = emu[k].ravel(), f64[k].ravel()
        if f"{k}:idx" in hip:
            e, f = e[hip[f"{k}:idx"]], f[hip[f"{k}:idx"]]
        h = hip[k]
        r, c, a = _stats(h, e)
        rf, cf, af = _stats(f, e)
        if np.isnan(a):
            continue
        rows.append((abs(a - 1) - abs(af - 1), k[5:], r, a, rf, af))
    rows.sort(reverse=True)
    for d, k, r, a, rf, af in rows[:16]:
        print(f"  rel {r:.3e} a {a:.4f} | floor rel {rf:.3e} a {af:.4f}  {k}")


if __name__ == "__main__":
    mode = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else "small_tome16_2blk"
    (dump if mode == "dump" else compare)(tag)
