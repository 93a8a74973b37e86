"""Offline end-to-end comparison: re-run the CPU oracle against a HIP dump taken on the GPU box
by tools/parity_dump.py (parameters are rebuilt on the CPU from the same seed).

    python tools/parity_offline.py DUMP.npz [--fp32]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from tools.parity_dump import load, make_cfg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("--fp32", action="store_true", help="plain fp32 oracle (no bf16 emulation)")
    a = ap.parse_args()
    from oracle import parity as P
    meta, res = load(a.dump)
    cfg = make_cfg(meta["config"], meta.get("blocks"), meta.get("t5_layers"))
    t0 = time.time()
    rl, rg = P.oracle_step(cfg, res, emulate_bf16=not a.fp32)
    out = P.compare(res, rl, rg)
    print(f"oracle {time.time() - t0:.1f}s\n" + P.report(out, 20))


if __name__ == "__main__":
    main()
