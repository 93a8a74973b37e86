"""Print the end-to-end parity report (loss, global and lowest per-tensor gradient cosines)."""
import sys

sys.path.insert(0, ".")
from oracle.parity import run_parity  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config  # noqa: E402
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config  # noqa: E402

for name, kw, B in [("octo-small-tome16", dict(num_blocks=3, t5=T5Config(num_layers=2)), 2),
                    ("octo-tiny", {}, 2)]:
    res = run_parity(get_config(name, **kw), B)
    cos = sorted(res["cos"].items(), key=lambda kv: kv[1])
    print(name, "loss", res["loss"], "ref", res["ref_loss"], "cos_all", res["cos_all"])
    for k, v in cos[:12]:
        print(f"  {v:.5f} {k}")
    print({k: v for k, v in res.items() if k not in ("cos",)})
