"""HIP and the bf16-emulating oracle, both against the EXACT restatement (oracle/octo_ref.py in
float64, no storage rounding) on the HIP run's own inputs and injected randomness, over seeds
(is there a systematic shrink of HIP's gradients?). Per seed: loss deviation,
global gradient norm ratio and cosine, and per parameter tensor the ratio of HIP's relative error
to the emulation's; per tensor across seeds: the norm ratios |g_hip| / |g_exact| (a systematic
shrink would keep them below 1 on every seed).

    python tools/parity_exact.py [--seeds=8] [--config=octo-small-tome16] [--blocks=2]
"""
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from oracle import parity as P


def flat(g, keys):
    return np.concatenate([np.asarray(g[k], np.float64).ravel() for k in keys])


def main():
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    seeds, name, blocks = 8, "octo-small-tome16", 2
    for a in sys.argv[1:]:
        if a.startswith("--seeds="):
            seeds = int(a.split("=")[1])
        if a.startswith("--config="):
            name = a.split("=")[1]
        if a.startswith("--blocks="):
            blocks = int(a.split("=")[1])
    cfg = get_config(name, num_blocks=blocks, t5=T5Config(num_layers=2))
    per_tensor = {}
    rows = []
    for seed in range(seeds):
        h = P.hip_step(cfg, 2, seed)
        (le, ge), (lf, gf) = P.oracle_pair(cfg, h, h["model"])
        keys = [k for k in sorted(gf) if np.linalg.norm(gf[k]) > 0]
        H, E, F = flat(h["grads"], keys), flat(ge, keys), flat(gf, keys)
        nf = np.linalg.norm(F)
        r = dict(loss_hip=h["loss"] / lf - 1, loss_emu=le / lf - 1,
                 norm_hip=np.linalg.norm(H) / nf, norm_emu=np.linalg.norm(E) / nf,
                 cos_hip=H @ F / (np.linalg.norm(H) * nf), cos_emu=E @ F / (np.linalg.norm(E) * nf))
        q = []
        for k in keys:
            f = np.asarray(gf[k], np.float64).ravel()
            hh = np.asarray(h["grads"][k], np.float64).ravel()
            ee = np.asarray(ge[k], np.float64).ravel()
            n = np.linalg.norm(f)
            eh, ee_ = np.linalg.norm(hh - f) / n, np.linalg.norm(ee - f) / n
            q.append(eh / max(ee_, 1e-30))
            per_tensor.setdefault(k, []).append((np.linalg.norm(hh) / n, np.linalg.norm(ee) / n, eh, ee_))
        r["err_ratio_median"] = st.median(q)
        r["tensors_hip_worse"] = sum(x > 1 for x in q)
        rows.append(r)
        print(f"seed {seed}: loss hip {r['loss_hip']:+.2e} emu {r['loss_emu']:+.2e} | grad norm hip "
              f"{r['norm_hip']:.4f} emu {r['norm_emu']:.4f} | cos hip {r['cos_hip']:.5f} emu {r['cos_emu']:.5f} "
              f"| per-tensor err hip/emu median {r['err_ratio_median']:.2f}, hip worse on "
              f"{r['tensors_hip_worse']}/{len(q)}", flush=True)
    print(f"\n{name}, {blocks} blocks, B = 2, {seeds} seeds, against the float64 restatement:")
    for k in ("loss_hip", "loss_emu", "norm_hip", "norm_emu", "cos_hip", "cos_emu", "err_ratio_median"):
        v = [r[k] for r in rows]
        print(f"  {k:18s} median {st.median(v):+.4f}  min {min(v):+.4f}  max {max(v):+.4f}")
    print("\nper tensor, norm ratio to exact over seeds (hip: median, min, max, seeds below 1 | emu median):")
    for k, v in sorted(per_tensor.items(), key=lambda kv: st.median(x[0] for x in kv[1])):
        hr = [x[0] for x in v]
        if k.endswith("bias") or "LayerNorm" in k:
            print(f"  {st.median(hr):.4f} {min(hr):.4f} {max(hr):.4f} {sum(x < 1 for x in hr)}/{len(hr)} | "
                  f"{st.median(x[1] for x in v):.4f}  {k}")


if __name__ == "__main__":
    main()
