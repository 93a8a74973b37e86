import sys, json
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_octo_gpu import run_parity
from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config
for name, kw, B in [("octo-tiny", dict(num_blocks=2), 3), ("octo-small-tome16", dict(num_blocks=3, t5=T5Config(num_layers=2)), 2)]:
    res = run_parity(get_config(name, **kw), B)
    worst = sorted(res["cos"].items(), key=lambda kv: kv[1])[:10]
    print(name, "loss", res["loss"], "ref", res["ref_loss"], "cos_all", res["cos_all"])
    for k, v in worst: print("   ", k, round(v, 5), "rel", round(res["rel"][k], 4))
