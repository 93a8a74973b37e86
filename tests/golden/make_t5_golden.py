"""Generate tests/golden/t5_*_golden.npz: FlaxT5-semantics pins for the T5 encoder (oracle on
CPU with d_kv=8; the HIP path on the GPU with d_kv=64, the kernel's head size).

The reference's text tokenizer is transformers' FlaxT5 encoder (t5_base.py:11-15, random init from
AutoConfig); Flax is not installed, so the installed PyTorch `transformers.T5EncoderModel` (same
architecture and arithmetic) is constructed from a LOCAL tiny T5Config (no download) with seeded
random weights, and its parameters (renamed to this build's layout) and output are stored.

    python tests/golden/make_t5_golden.py
"""
from pathlib import Path

import numpy as np
import torch
from transformers import T5Config, T5EncoderModel

HERE = Path(__file__).parent


def make(name, d_model, d_kv, d_ff, heads, seed):
    OUT = HERE / f"t5_{name}_golden.npz"
    torch.manual_seed(seed)
    cfg = T5Config(vocab_size=96, d_model=d_model, d_kv=d_kv, d_ff=d_ff, num_layers=2, num_heads=heads,
                   relative_attention_num_buckets=32, relative_attention_max_distance=128,
                   feed_forward_proj="relu", dropout_rate=0.0, layer_norm_epsilon=1e-6)
    m = T5EncoderModel(cfg).eval()
    with torch.no_grad():
        for p in m.parameters():          # HF's T5 init for matrices; non-trivial norm weights
            if p.dim() == 1:
                p.copy_(1.0 + 0.2 * torch.randn_like(p))
    ids = torch.from_numpy(np.random.default_rng(0).integers(0, 96, (2, 40))).long()
    with torch.no_grad():
        out = m(input_ids=ids).last_hidden_state.float()
    sd = m.state_dict()
    pre = "T5Tokenizer_0"
    arrs = {"ids": ids.numpy().astype(np.int32), "out": out.numpy(),
            f"{pre}/shared/embedding": sd["shared.weight"].numpy(),
            f"{pre}/relative_attention_bias":
                sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"].numpy(),
            f"{pre}/final_layer_norm": sd["encoder.final_layer_norm.weight"].numpy()}
    for i in range(cfg.num_layers):
        b = f"encoder.block.{i}.layer"
        p = f"{pre}/block/{i}"
        arrs[f"{p}/layer_0/layer_norm"] = sd[f"{b}.0.layer_norm.weight"].numpy()
        arrs[f"{p}/SelfAttention/qkv"] = torch.cat(
            [sd[f"{b}.0.SelfAttention.{n}.weight"] for n in "qkv"], 0).numpy()
        arrs[f"{p}/SelfAttention/o"] = sd[f"{b}.0.SelfAttention.o.weight"].numpy()
        arrs[f"{p}/layer_1/layer_norm"] = sd[f"{b}.1.layer_norm.weight"].numpy()
        arrs[f"{p}/DenseReluDense/wi"] = sd[f"{b}.1.DenseReluDense.wi.weight"].numpy()
        arrs[f"{p}/DenseReluDense/wo"] = sd[f"{b}.1.DenseReluDense.wo.weight"].numpy()
    np.savez_compressed(OUT, **arrs)
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


def main():
    make("small", 32, 8, 64, 4, 0)
    make("dkv64", 64, 64, 128, 2, 1)


if __name__ == "__main__":
    main()
