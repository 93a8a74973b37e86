"""Frozen T5-base text encoder, mirroring the reference's ``tokenizers/text/t5_base.py`` (:8-15):
``T5Tokenizer()(input_ids) -> stop_gradient(FlaxT5EncoderModel(AutoConfig('t5-base')).module(
input_ids).last_hidden_state)``, randomly initialised from the t5-base config (the reference never
loads pretrained weights; AutoConfig.from_pretrained needs the network, so the config is
hard-coded here: d_model 768, d_kv 64, d_ff 3072, 12 layers x 12 heads, 32 relative-attention
buckets with max distance 128, RMS-norm eps 1e-6, ReLU feed-forward, vocab 32128).

Forward only (stop_gradient, :14): bf16 weights in a FrozenStore, every op a libmmt_hip kernel
(embedding gather, T5LayerNorm, MFMA GEMMs with fused residual/relu, attention in bias mode with
scale 1). The relative position bias depends only on frozen weights and the fixed length, so it
is computed once per sequence length and cached on the device.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ... import _kernels as K
from ...params import FrozenStore, const, normal


@dataclass
class T5Config:
    vocab_size: int = 32128
    d_model: int = 768
    d_kv: int = 64
    d_ff: int = 3072
    num_layers: int = 12
    num_heads: int = 12
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    layer_norm_epsilon: float = 1e-6
    initializer_factor: float = 1.0


def relative_position_bucket(relative_position: torch.Tensor, bidirectional=True, num_buckets=32,
                             max_distance=128) -> torch.Tensor:
    """T5 bucketing (FlaxT5Attention._relative_position_bucket)."""
    ret = torch.zeros_like(relative_position)
    n = relative_position
    if bidirectional:
        num_buckets //= 2
        ret = ret + (n > 0).long() * num_buckets
        n = n.abs()
    else:
        n = (-n).clamp_min(0)
    max_exact = num_buckets // 2
    is_small = n < max_exact
    large = max_exact + (torch.log(n.float().clamp_min(1) / max_exact) /
                         math.log(max_distance / max_exact) * (num_buckets - max_exact)).long()
    large = large.clamp_max(num_buckets - 1)
    return ret + torch.where(is_small, n, large)


class T5Tokenizer:
    """Frozen T5 encoder; ``__call__(input_ids (B, T) int32) -> (B, T, d_model) bf16``."""

    def __init__(self, config: T5Config | None = None, name: str = "T5Tokenizer_0"):
        self.cfg = c = config or T5Config()
        self.store = FrozenStore()
        f = c.initializer_factor
        inner = c.num_heads * c.d_kv
        add = self.store.add
        self.shared = add(f"{name}/shared/embedding", (c.vocab_size, c.d_model), normal(f * 1.0))
        self.rel_bias = add(f"{name}/relative_attention_bias", (c.relative_attention_num_buckets,
                                                                 c.num_heads), normal(f * c.d_model ** -0.5))
        self.layers = []
        for i in range(c.num_layers):
            p = f"{name}/block/{i}"
            qs, ks = f * (c.d_model * c.d_kv) ** -0.5, f * c.d_model ** -0.5
            # fused [q; k; v] weight (3*inner, d_model), stored [out][in]
            qkv = add(f"{p}/SelfAttention/qkv", (3 * inner, c.d_model), _stack_init(
                [(inner, qs), (inner, ks), (inner, ks)], c.d_model))
            o = add(f"{p}/SelfAttention/o", (c.d_model, inner), normal(f * inner ** -0.5))
            ln0 = add(f"{p}/layer_0/layer_norm", (c.d_model,), const(f))
            wi = add(f"{p}/DenseReluDense/wi", (c.d_ff, c.d_model), normal(f * c.d_model ** -0.5))
            wo = add(f"{p}/DenseReluDense/wo", (c.d_model, c.d_ff), normal(f * c.d_ff ** -0.5))
            ln1 = add(f"{p}/layer_1/layer_norm", (c.d_model,), const(f))
            self.layers.append((qkv, o, ln0, wi, wo, ln1))
        self.final_ln = add(f"{name}/final_layer_norm", (c.d_model,), const(f))
        self._bias_cache = {}

    def materialize(self, device, seed: int = 1):
        self.store.materialize(device, seed)
        return self

    def position_bias(self, T: int) -> torch.Tensor:
        if T not in self._bias_cache:
            c = self.cfg
            pos = torch.arange(T)
            bucket = relative_position_bucket(pos[None, :] - pos[:, None], True,
                                              c.relative_attention_num_buckets,
                                              c.relative_attention_max_distance)
            table = self.rel_bias.bf16.float()                    # (buckets, H)
            bias = table[bucket.to(table.device)].permute(2, 0, 1).contiguous()  # (H, T, T)
            self._bias_cache[T] = bias
        return self._bias_cache[T]

    def __call__(self, input_ids: torch.Tensor, layer_outputs: list | None = None) -> torch.Tensor:
        """input_ids (B, T) int -> last_hidden_state (B, T, d_model) bf16 (stop_gradient, :14).
        Materialises the (seeded, randomly initialised) weights on the ids' device on the first
        call when ``materialize`` was not called (the reference builds the module from the config
        alone, ``T5Tokenizer()``, :10-12). layer_outputs: if a list, receives the residual stream
        after each layer (parity tests)."""
        if self.store.flat_bf16 is None:
            self.materialize(input_ids.device, 1)
        c = self.cfg
        B, T = input_ids.shape
        ids = input_ids.to(torch.int32).contiguous()
        x = K.embedding_gather(ids.view(-1), self.shared.bf16)     # (B*T, d)
        bias = self.position_bias(T)
        for qkv, o, ln0, wi, wo, ln1 in self.layers:
            n = K.rmsnorm(x, ln0.bf16, c.layer_norm_epsilon)
            q = K.gemm(n, qkv.bf16, trans_b=True).view(B, T, -1)
            a, _ = K.attn_fwd(q, c.num_heads, 1.0, None, None, 1.0, bias=bias)
            x = K.gemm(a.view(B * T, -1), o.bf16, trans_b=True, residual=x)
            n = K.rmsnorm(x, ln1.bf16, c.layer_norm_epsilon)
            h = K.gemm(n, wi.bf16, trans_b=True, act=K.ACT_RELU)
            x = K.gemm(h, wo.bf16, trans_b=True, residual=x)
            if layer_outputs is not None:
                layer_outputs.append(x.view(B, T, c.d_model))
        x = K.rmsnorm(x, self.final_ln.bf16, c.layer_norm_epsilon)
        return x.view(B, T, c.d_model)


def _stack_init(parts, fan_in_dim):
    def init(t, g):
        with torch.no_grad():
            r = 0
            for n, std in parts:
                t[r:r + n].copy_(torch.randn((n, fan_in_dim), generator=g) * std)
                r += n
        return t
    return init
