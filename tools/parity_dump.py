"""Run the end-to-end parity comparison on the GPU box and (optionally) dump the HIP side so the
oracle can be re-run offline (tools/parity_offline.py) without another GPU call.

    python tools/parity_dump.py CONFIG [--blocks N] [--t5-layers N] [--B 2] [--seed 0]
                                [--dump gpurun_out/x.npz] [--no-oracle]

Gradients of tensors above 65,536 elements are dumped as bf16 bits (the comparison bar is
cosine >= 0.999; bf16 storage of one side moves the cosine by < 1e-5).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def make_cfg(name, blocks=None, t5_layers=None):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
    kw = {}
    if blocks:
        kw["num_blocks"] = blocks
    if t5_layers:
        kw["t5"] = T5Config(num_layers=t5_layers)
    return get_config(name, **kw)


def save(path, cfg_args, res, grads=True):
    d = dict(meta=json.dumps(dict(cfg_args, B=res["B"], seed=res["seed"])), loss=res["loss"],
             rt=res["rt"], ct=res["ct"], t=res["t"], eps=res["eps"])
    for i, tr in enumerate(res["tome"]):
        if isinstance(tr, tuple):
            for k, a in zip(("unm", "src", "dst"), tr):
                d[f"tome_{i}_{k}"] = a
        elif tr is not None:          # top-k pruning rows
            d[f"tome_{i}_topk"] = np.asarray(tr)
    for name, a in res.get("trace", {}).items():
        d["tr/" + name] = a.astype(np.float32)
    for name, g in (res["grads"].items() if grads else ()):
        if g.size > 65536:
            d["g16/" + name] = torch.from_numpy(g).bfloat16().view(torch.int16).numpy()
        else:
            d["g32/" + name] = g
    np.savez(path, **d)


def load(path):
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    res = dict(B=meta["B"], seed=meta["seed"], loss=float(z["loss"]), rt=z["rt"], ct=z["ct"],
               t=z["t"], eps=z["eps"], grads={})
    nb = 0
    for k in z.files:
        if k.startswith("g16/"):
            res["grads"][k[4:]] = torch.from_numpy(z[k]).view(torch.bfloat16).float().numpy()
        elif k.startswith("g32/"):
            res["grads"][k[4:]] = z[k]
        elif k.startswith("tr/"):
            res.setdefault("trace", {})[k[3:]] = z[k]
        elif k.startswith("tome_"):
            nb = max(nb, int(k.split("_")[1]) + 1)
    res["tome"] = []
    for i in range(max(nb, 0)):
        if f"tome_{i}_unm" in z.files:
            res["tome"].append(tuple(z[f"tome_{i}_{k}"] for k in ("unm", "src", "dst")))
        elif f"tome_{i}_topk" in z.files:
            res["tome"].append(z[f"tome_{i}_topk"])
        else:
            res["tome"].append(None)
    return meta, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--blocks", type=int)
    ap.add_argument("--t5-layers", type=int)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dump")
    ap.add_argument("--no-oracle", action="store_true")
    ap.add_argument("--blockwise", action="store_true", help="teacher-forced block-local comparison")
    ap.add_argument("--trace", help="comma-separated blocks whose intermediates are dumped "
                                    "(every block input is dumped too); gradients are not")
    a = ap.parse_args()
    from oracle import parity as P
    cfg = make_cfg(a.config, a.blocks, a.t5_layers)
    t0 = time.time()
    if a.blockwise:
        t0 = time.time()
        res = P.hip_blockwise(cfg, a.B, a.seed)
        out = P.oracle_blockwise(cfg, res)
        print(f"[{a.config} blockwise] {time.time() - t0:.1f}s, in-situ ToMe layers "
              f"{res['tome_layers_checked']}\n" + P.report_blockwise(out), flush=True)
        return
    tl = [int(v) for v in a.trace.split(",")] if a.trace else None
    res = P.hip_step(cfg, a.B, a.seed, trace_layers=tl)
    print(f"[{a.config}] hip step done ({time.time() - t0:.1f}s), in-situ ToMe layers checked: "
          f"{res['tome_layers_checked']}", flush=True)
    if a.dump:
        save(a.dump, dict(config=a.config, blocks=a.blocks, t5_layers=a.t5_layers), res,
             grads=tl is None)
    if not a.no_oracle:
        t0 = time.time()
        rl, rg = P.oracle_step(cfg, res, model=res["model"])
        out = P.compare(res, rl, rg)
        print(f"[{a.config}] oracle {time.time() - t0:.1f}s\n" + P.report(out), flush=True)


if __name__ == "__main__":
    main()
