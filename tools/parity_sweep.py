"""Diagnostic: free-running end-to-end parity against depth (profiles/r02_parity_depth_sweep.txt).

For octo-small-tome16 at depth d (d blocks, d T5 layers, B = 2) it prints
  * HIP vs the bf16-emulating oracle (the test oracle),
  * HIP vs the plain fp32 oracle,
  * CPU only: the bf16-emulating oracle vs the same restatement in float64 — no HIP involved,
    which separates the model's own amplification of bf16 storage noise from kernel error;
and octo-tiny (2 blocks) over seeds against the bf16-emulating oracle.
"""
import sys

sys.path.insert(0, ".")
from oracle import parity as P  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config  # noqa: E402


def line(tag, out):
    worst = min(out["cos"].items(), key=lambda kv: kv[1])
    return (f"{tag:34s} loss_rel {abs(out['loss'] / out['ref_loss'] - 1):.2e} cos_all {out['cos_all']:.5f} "
            f"min_cos {worst[1]:.5f} ({worst[0].split('/', 1)[-1]})")


def main():
    for d in (1, 2, 3, 4, 6, 8, 12):
        cfg = get_config("octo-small-tome16", num_blocks=d, t5=T5Config(num_layers=d))
        res = P.hip_step(cfg, 2, seed=0)
        m = res["model"]
        for emu in (True, False):
            rl, rg = P.oracle_step(cfg, res, model=m, emulate_bf16=emu)
            print(line(f"depth {d:2d} HIP vs {'bf16-emul' if emu else 'fp32'} oracle", P.compare(res, rl, rg)),
                  flush=True)
        print(line(f"depth {d:2d} CPU bf16-emul vs fp64", P.bf16_floor(cfg, res, m)), flush=True)
    for seed in range(5):
        cfg = get_config("octo-tiny", num_blocks=2)
        res = P.hip_step(cfg, 3, seed=seed)
        rl, rg = P.oracle_step(cfg, res, model=res["model"])
        print(line(f"octo-tiny 2 blocks seed {seed}", P.compare(res, rl, rg)), flush=True)


if __name__ == "__main__":
    main()
