"""Where HIP's excess over the bf16 floor comes from (DESIGN §4 noise table).
Full depth octo-small-tome16 (12 blocks, 12 T5 layers), B = 2, seeds 0..S-1, each HIP run
compared with the bf16-emulating CPU oracle on its own injected randomness / merge indices:
  floor   the emulating oracle vs the same oracle in float64 (bf16 storage rounding alone)
  hip     the default HIP step (fp32 atomics at 19 gradient sites) vs the emulating oracle
  det     the deterministic HIP step (MMT_DETERMINISTIC=1: fixed-point gradient accumulation,
          no order-dependent sums left) vs the emulating oracle
  rerun   two default HIP runs against each other (what atomic ordering alone moves)
Loss: |rel|; gradients: 1 - global cosine over every parameter gradient.
    python tools/noise_sources.py [--seeds=6] [--config=octo-small-tome16]"""
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from oracle import parity as P


def gcos(ga, gb):
    a = np.concatenate([np.asarray(ga[k], np.float64).ravel() for k in sorted(ga)])
    b = np.concatenate([np.asarray(gb[k], np.float64).ravel() for k in sorted(ga)])
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def main():
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    seeds, name = 6, "octo-small-tome16"
    for a in sys.argv[1:]:
        if a.startswith("--seeds="):
            seeds = int(a.split("=")[1])
        if a.startswith("--config="):
            name = a.split("=")[1]
    cfg = get_config(name)
    rows = []
    for seed in range(seeds):
        r = {}
        os.environ.pop("MMT_DETERMINISTIC", None)
        h1 = P.hip_step(cfg, 2, seed)
        h2 = P.hip_step(cfg, 2, seed)
        os.environ["MMT_DETERMINISTIC"] = "1"
        hd = P.hip_step(cfg, 2, seed)
        os.environ.pop("MMT_DETERMINISTIC", None)
        same_idx = all(all(np.array_equal(x, y) for x, y in zip(a, b)) if a is not None else b is None
                       for a, b in zip(h1["tome"], h2["tome"]))
        r["rerun"] = (abs(h1["loss"] / h2["loss"] - 1), 1 - gcos(h1["grads"], h2["grads"]), same_idx)
        for tag, h in (("hip", h1), ("det", hd)):
            ref_loss, ref_grads = P.oracle_step(cfg, h, model=h["model"])
            r[tag] = (abs(h["loss"] / ref_loss - 1), 1 - gcos(h["grads"], ref_grads))
        hd["model"].store.close()  # release the deterministic registration for the next seed
        f = P.bf16_floor(cfg, h1, h1["model"])
        r["floor"] = (abs(f["loss"] / f["ref_loss"] - 1), 1 - f["cos_all"])
        rows.append(r)
        print(f"seed {seed}: " + "  ".join(f"{k} loss {v[0]:.2e} cos-def {v[1]:.2e}"
                                           for k, v in r.items() if k != "rerun")
              + f"  rerun loss {r['rerun'][0]:.2e} cos-def {r['rerun'][1]:.2e} same-merge {r['rerun'][2]}",
              flush=True)
    print(f"\nmedians over {seeds} seeds ({name}, 12 blocks, B = 2):")
    for k in ("floor", "hip", "det", "rerun"):
        ml = st.median(r[k][0] for r in rows)
        mc = st.median(r[k][1] for r in rows)
        fl = st.median(r["floor"][0] for r in rows)
        fc = st.median(r["floor"][1] for r in rows)
        print(f"  {k:6s} loss {ml:.2e} ({ml / fl:.2f}x floor)   1-cos {mc:.2e} ({mc / fc:.2f}x floor)")


if __name__ == "__main__":
    torch.backends.cuda.matmul.allow_tf32 = False
    main()
