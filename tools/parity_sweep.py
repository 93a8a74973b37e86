"""Diagnostic: end-to-end parity over seeds for ToMe on/off and dropout on/off."""
import sys

sys.path.insert(0, ".")
from oracle.parity import run_parity  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config  # noqa: E402

for name in ("octo-small", "octo-small-tome16"):
    for drop in (0.0, 0.1):
        for seed in range(3):
            cfg = get_config(name, num_blocks=3, t5=T5Config(num_layers=2), dropout_rate=drop,
                             attention_dropout_rate=drop)
            res = run_parity(cfg, 2, seed=seed)
            worst = sorted(res["cos"].items(), key=lambda kv: kv[1])[:2]
            print(f"{name:18s} drop={drop} seed={seed} loss_rel={abs(res['loss'] / res['ref_loss'] - 1):.4f} "
                  f"cos_all={res['cos_all']:.5f} worst={[(k.split('/')[-3:], round(v, 4)) for k, v in worst]}",
                  flush=True)
