"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

fp32 PyTorch-CPU restatement of the reference's OCTO diffusion training forward
(multi_modal_transformers/...), written op for op from the reference sources and the Flax layer
semantics they configure. Gradients come from torch autograd on this restatement.

Randomness cannot follow JAX Threefry, so it is injected: dropout keep-masks are regenerated
from oracle/rng.py with the same (seed, step, layer, site, counter) keys the HIP path uses; patch
position tokens, diffusion (t, eps) and — for end-to-end runs — the ToMe index triples are taken
from the run under test (ToMe indices are checked bit-exact separately, per op, against
oracle/tome_ref.c on identical metrics).

Parameter layout = the build's ParamStore names/shapes (Dense kernels stored [out][in]).

Follows:
  token_sequencer.py:94-183 (mask), :255-269 (assembly)       image_tokenizer.py:35-71,158-176,300-307
  attention.py:20-69 (MLPBlock, Encoder1DBlock), :97-100        token_compression.py:54-129 (ToMe)
  octo.py:91-126,139-145 (readouts, loss)                       diffusion.py:17-65,102,110-143
  t5_base.py:8-15 + FlaxT5 encoder semantics (pinned against transformers.T5EncoderModel)
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from . import rng as R

# ------------------------------------------------------------------------------ mask (literal)
def literal_mask(sets) -> np.ndarray:
    """sets: list of (kind, num_tokens, timestep) with kind in {"prefix","text","image","readout"}.
    Square (L, L) bool mask, token_sequencer.py:55-183 rules, rows and columns from `sets`."""
    rows = []
    for qk, qn, qt in sets:
        blocks = []
        for kk, kn, kt in sets:
            same_class = (qk == kk)
            if kt == qt and same_class:          # intra rule
                if qk == "text":
                    b = np.tril(np.ones((qn, kn)))
                else:
                    b = np.ones((qn, kn))
            else:                                 # inter rule
                if qk == "prefix":
                    b = np.zeros((qn, kn))
                elif qk in ("text", "image"):
                    b = np.zeros((qn, kn)) if kk == "readout" else (
                        np.ones((qn, kn)) if kt <= qt else np.zeros((qn, kn)))
                else:  # readout
                    b = np.zeros((qn, kn)) if kk == "readout" else (
                        np.ones((qn, kn)) if kt <= qt else np.zeros((qn, kn)))
            blocks.append(b)
        rows.append(np.hstack(blocks))
    return np.vstack(rows).astype(bool)


# ------------------------------------------------------------------------------- image tokenizer
def image_to_patches(image: np.ndarray, patch_size: int, normalize: bool) -> np.ndarray:
    """image_tokenizer.py:35-71 for one (H, W, C) image (einops rearrange written out)."""
    h, w, c = image.shape
    assert h == w and h % patch_size == 0
    n = h // patch_size
    p = image.reshape(n, patch_size, n, patch_size, c).transpose(0, 2, 1, 3, 4).reshape(
        n * n, patch_size, patch_size, c)
    if normalize:
        p = (2 * (p / 255.0)) - 1.0
    return p


def encode_patch_position_eval(h: int, patch_size: int, num_tokens: int):
    """image_tokenizer.py:74-132, eval branch (train draws are injected)."""
    P = h // patch_size
    idx_vals = np.arange(0, h + patch_size, patch_size)
    pairs = np.stack([idx_vals[:-1], idx_vals[1:]], axis=-1)                # (P, 2)
    row_idx = np.tile(pairs, (P, 1))                                        # p -> pairs[p % P]
    col_idx = np.repeat(pairs, P, axis=0)                                   # p -> pairs[p // P]
    idx = np.concatenate([row_idx, col_idx], axis=-1).astype(np.float32)   # (P*P, 4)
    q = np.floor((idx / np.float32(h)) * np.float32(num_tokens - 1))
    rs, re, cs, ce = q.T
    return ((rs + re) // 2).astype(np.int32), ((cs + ce) // 2).astype(np.int32)


def cosine_beta_schedule(timesteps, s=0.008):
    """diffusion.py:17-27."""
    steps = timesteps + 1
    t = np.linspace(0, timesteps, steps, dtype=np.float32) / np.float32(timesteps)
    ac = np.cos((t + np.float32(s)) / np.float32(1 + s) * np.float32(np.pi) * np.float32(0.5)) ** 2
    ac = ac / ac[0]
    betas = 1 - (ac[1:] / ac[:-1])
    return np.clip(betas, 0, 0.999).astype(np.float32)


def groupnorm(x: torch.Tensor, G: int, scale, bias, eps):
    """flax GroupNorm: stats per (sample, group) over every non-batch axis; fast variance."""
    B = x.shape[0]
    C = x.shape[-1]
    xg = x.reshape(B, -1, G, C // G)
    mu = xg.mean(dim=(1, 3), keepdim=True)
    var = torch.clamp((xg * xg).mean(dim=(1, 3), keepdim=True) - mu * mu, min=0)
    y = (xg - mu) * torch.rsqrt(var + eps)
    return y.reshape(x.shape) * scale + bias


def gelu_tanh(x):
    return 0.5 * x * (1 + torch.tanh(math.sqrt(2 / math.pi) * (x + 0.044715 * x ** 3)))


def seq_layernorm(x, scale, bias, eps):
    """LayerNorm(reduction_axes=[1]): stats over the sequence axis, fast variance."""
    mu = x.mean(dim=1, keepdim=True)
    var = torch.clamp((x * x).mean(dim=1, keepdim=True) - mu * mu, min=0)
    return (x - mu) * (torch.rsqrt(var + eps) * scale) + bias


def dense(p, name, x):
    y = x @ p[f"{name}/kernel"].t()
    b = p.get(f"{name}/bias")
    return y + b if b is not None else y


def quant_rows_e4m3(x: torch.Tensor):
    """Row-wise OCP e4m3 quantisation of the fp8 path (csrc/gemm.hip quant_rows_fp8_kernel):
    scale = amax / 448 (1 for a zero row), q = round_to_nearest_even(x / scale) as e4m3."""
    amax = x.detach().abs().amax(-1, keepdim=True)
    scale = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (x.detach() / scale).to(torch.float8_e4m3fn).float()
    return q, scale


def dense_fp8(p, name, x):
    """The fp8 forward product (e4m3 activations per row x e4m3 weights per output channel,
    fp32 accumulation, scales applied after the sum) with the bf16 product's gradient
    (straight-through: the build's backward runs on the bf16 shadow)."""
    y = dense(p, name, x)
    w = p[f"{name}/kernel"]
    xs = x.reshape(-1, x.shape[-1])
    xq, sx = quant_rows_e4m3(xs)
    wq, sw = quant_rows_e4m3(w.detach())
    y8 = (xq @ wq.t()) * sx * sw.reshape(1, -1)
    b = p.get(f"{name}/bias")
    if b is not None:
        y8 = y8 + b.detach()
    return y + (y8.reshape(y.shape) - y).detach()


# ------------------------------------------------------------------ bf16 storage emulation
class _RoundFwd(torch.autograd.Function):
    """bf16 rounding of a stored activation; the gradient passes through unchanged."""
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """Identity forward; the gradient is rounded to bf16 (a bf16-stored gradient tensor)."""
    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class _RoundBoth(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


def _bf(x):
    return x.to(torch.bfloat16).to(x.dtype)


class FlashAttnBF16(torch.autograd.Function):
    """Softmax attention with the storage points of csrc/attention.hip: probabilities enter the
    P.V product as bf16 (after the dropout keep mask), dS = P*(dP*keep/kp - delta) enters the dQ
    and dK products as bf16, dV = bf16(P*keep)^T dO / kp, delta = rowsum(dO * bf16(O)).
    q, k, v (B, L, H, Dh) bf16-valued fp32; allowed (L, L) bool; keep (L, L) bool or None;
    bias (H, L, L) or None (T5 mode, added after the scale)."""
    @staticmethod
    def forward(ctx, q, k, v, allowed, keep, kp, scale, bias):
        s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
        if bias is not None:
            s = s + bias[None]
        s = s.masked_fill(~allowed[None, None], float("-inf"))
        m = s.amax(-1, keepdim=True)
        p = torch.exp(s - m)
        l = p.sum(-1, keepdim=True)
        pk = p if keep is None else p * keep[None, None]
        o = torch.einsum("bhqk,bkhd->bqhd", _bf(pk), v) / l.permute(0, 2, 1, 3) / kp
        lse = m + torch.log(l)
        ctx.save_for_backward(q, k, v, s, lse, _bf(o))
        ctx.keep, ctx.kp, ctx.scale = keep, kp, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, s, lse, o16 = ctx.saved_tensors
        keep, kp, scale = ctx.keep, ctx.kp, ctx.scale
        P = torch.exp(s - lse)
        dp = torch.einsum("bqhd,bkhd->bhqk", do, v) / kp
        pk = P
        if keep is not None:
            dp = dp * keep[None, None]
            pk = P * keep[None, None]
        delta = (do * o16).sum(-1).permute(0, 2, 1)[..., None]          # (B, H, L, 1)
        ds = _bf(P * (dp - delta))
        dq = torch.einsum("bhqk,bkhd->bqhd", ds, k) * scale
        dk = torch.einsum("bhqk,bqhd->bkhd", ds, q) * scale
        dv = torch.einsum("bhqk,bqhd->bkhd", _bf(pk), do) / kp
        return dq, dk, dv, None, None, None, None, None


# ----------------------------------------------------------------------------------- T5
def t5_bucket(rel, num_buckets=32, max_distance=128):
    ret = (rel > 0).long() * (num_buckets // 2)
    n = rel.abs()
    nb = num_buckets // 2
    max_exact = nb // 2
    large = max_exact + (torch.log(n.float().clamp_min(1) / max_exact) / math.log(max_distance / max_exact)
                         * (nb - max_exact)).long()
    large = large.clamp_max(nb - 1)
    return ret + torch.where(n < max_exact, n, large)


def t5_position_bias(tp, T, prefix="T5Tokenizer_0", num_buckets=32, max_distance=128):
    pos = torch.arange(T)
    bucket = t5_bucket(pos[None, :] - pos[:, None], num_buckets, max_distance)
    return tp[f"{prefix}/relative_attention_bias"][bucket].permute(2, 0, 1)  # (H, T, T)


def t5_rms(x, w, eps, emulate_bf16=False):
    y = x * torch.rsqrt((x * x).mean(-1, keepdim=True) + eps) * w
    return _bf(y) if emulate_bf16 else y


def t5_layer(tp, x, i, bias, H, d_kv, eps=1e-6, prefix="T5Tokenizer_0", emulate_bf16=False):
    """One FlaxT5 encoder layer: pre-RMS-norm self-attention (relative bias, no 1/sqrt(d)) and
    ReLU feed-forward, each added to the residual stream."""
    q16 = _bf if emulate_bf16 else (lambda a: a)
    B, T, _ = x.shape
    inner = H * d_kv
    p = f"{prefix}/block/{i}"
    n = t5_rms(x, tp[f"{p}/layer_0/layer_norm"], eps, emulate_bf16)
    qkv = q16(n @ tp[f"{p}/SelfAttention/qkv"].t())
    q, k, v = qkv.split(inner, dim=-1)
    q, k, v = (a.reshape(B, T, H, d_kv) for a in (q, k, v))
    if emulate_bf16:
        o = FlashAttnBF16.apply(q, k, v, torch.ones((T, T), dtype=torch.bool), None, 1.0, 1.0, bias)
    else:
        s = torch.einsum("bqhd,bkhd->bhqk", q, k) + bias[None]
        o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v)
    o = q16(o).reshape(B, T, inner)
    x = q16(x + o @ tp[f"{p}/SelfAttention/o"].t())
    n = t5_rms(x, tp[f"{p}/layer_1/layer_norm"], eps, emulate_bf16)
    return q16(x + q16(torch.relu(n @ tp[f"{p}/DenseReluDense/wi"].t())) @ tp[f"{p}/DenseReluDense/wo"].t())


def t5_encoder(tp: Dict[str, torch.Tensor], ids: torch.Tensor, num_layers: int, H: int, d_kv: int,
               eps: float = 1e-6, prefix="T5Tokenizer_0", num_buckets=32, max_distance=128,
               emulate_bf16: bool = False):
    """FlaxT5 encoder forward (t5_base.py:11-15): RMS layer norm, relative-position-biased
    attention without 1/sqrt(d) scaling, ReLU FF, pre-norm residuals, final norm.
    emulate_bf16: round at the build's storage points (bf16 residual stream, norm outputs,
    projections, attention probabilities; tokenizers/text/t5_base.py)."""
    B, T = ids.shape
    x = tp[f"{prefix}/shared/embedding"][ids.long()]
    bias = t5_position_bias(tp, T, prefix, num_buckets, max_distance)
    for i in range(num_layers):
        x = t5_layer(tp, x, i, bias, H, d_kv, eps, prefix, emulate_bf16)
    return t5_rms(x, tp[f"{prefix}/final_layer_norm"], eps, emulate_bf16)


# ------------------------------------------------------------------------------ ToMe (torch)
def tome_merge_wavg(x_set, size, unm, src, dst, r):
    """token_compression.py:90-129 on the token set (n, t, D) with given indices (torch,
    differentiable w.r.t. x)."""
    n = x_set.shape[0]
    if size is None:
        size = torch.ones(x_set.shape[:2] + (1,), dtype=x_set.dtype)
    def merge(z):
        a, b = z[:, ::2], z[:, 1::2]
        outs = []
        for bi in range(n):
            dstb = b[bi]
            for i in range(r):
                j = int(dst[bi, i])
                dstb = torch.cat([dstb[:j], (dstb[j] + a[bi, int(src[bi, i])])[None], dstb[j + 1:]])
            outs.append(torch.cat([a[bi, unm[bi].long()], dstb]))
        return torch.stack(outs)
    xm = merge(x_set * size)
    sm = merge(size)
    return xm / sm, sm


# ---------------------------------------------------------------------------- the model
class OctoRef:
    """cfg: the build's OctoConfig; params: {name: fp32 CPU tensor requiring grad};
    t5_params: {name: fp32 CPU tensor} (frozen).

    emulate_bf16=True rounds to bf16 at every point where the build STORES a bf16 tensor, in the
    forward (LayerNorm / GroupNorm outputs, q/k/v, attention probabilities, attention output, MLP
    hidden, stem im2col pixels, token embeddings, head inputs, the whole T5) and in the backward
    (every gradient the build writes as bf16: dz of each dropout/Dense output, dq/dk/dv, dS,
    dy of each LayerNorm-fed Dense, the head's dpred/dcat). What then remains between the two
    is fp32 summation order, which is what the tight end-to-end bar measures. Without it the
    restatement is plain fp32 (the CPU baseline)."""

    def __init__(self, cfg, params: Dict[str, torch.Tensor], t5_params: Optional[Dict] = None,
                 dtype=torch.float32, emulate_bf16: bool = False):
        self.cfg = cfg
        self.dtype = dtype
        self.residual_round = None
        self.p = params
        self.t5p = t5_params
        self.emulate = emulate_bf16

    # storage-point rounding (identity without emulation)
    def rb(self, x):
        return _RoundFwd.apply(x) if self.emulate else x

    def gb(self, x):
        return _RoundGrad.apply(x) if self.emulate else x

    def rbg(self, x):
        return _RoundBoth.apply(x) if self.emulate else x

    def _q(self, x):
        """Optional emulation of a storage rounding of the residual stream (diagnostics only)."""
        if self.residual_round is None:
            return x
        return x + (x.detach().to(self.residual_round).to(x.dtype) - x.detach())

    # -------------------------------------------------------------------------- pieces
    def stem(self, images, positions, trace=None):
        """image_tokenizer.py:235-309: patches -> ResNetV2 stem -> Dense (+ row/col embeddings).
        images (B, I, H, W, 3) in [0, 255]; returns (B, I*NP, D)."""
        cfg, p, dt = self.cfg, self.p, self.dtype
        rb, gb, rbg = self.rb, self.gb, self.rbg
        images = torch.as_tensor(images).to(dt)
        B, I = images.shape[:2]
        P = cfg.patch_size
        NP = (cfg.image_size[0] // P) ** 2
        patches = torch.stack([torch.stack([torch.from_numpy(image_to_patches(
            images[b, i].numpy(), P, True)) for i in range(I)]) for b in range(B)]).to(dt)
        x = rb(patches.reshape(B * I * NP, P, P, 3).permute(0, 3, 1, 2))       # NCHW
        name = "ImageTokenizer_0/ResNetV2Block_0"
        wc = p[f"{name}/Conv_0/kernel"].view(64, 12, 12, 3).permute(0, 3, 1, 2)
        x = gb(F.conv2d(x, wc, None, stride=2)) + p[f"{name}/Conv_0/bias"].view(1, -1, 1, 1)
        x = F.max_pool2d(x, 3, stride=1)                                       # (N, 64, PH, PW)
        PH, PW = x.shape[2], x.shape[3]
        x = x.permute(0, 2, 3, 1).reshape(B, I * NP * PH * PW, 64)            # NHWC rows
        residual = x
        for k in range(2):
            x = groupnorm(x, 32, p[f"{name}/GroupNorm_{k}/scale"], p[f"{name}/GroupNorm_{k}/bias"], 1e-6)
            x = rb(gelu_tanh(x))
            if PH * PW == 1:   # 3x3 SAME conv on a 1x1 map = centre tap
                x = gb(dense(p, f"{name}/Conv_{k + 1}", x))
            else:              # full 3x3 SAME conv (image_tokenizer.py:164-167)
                w3 = p[f"{name}/Conv_{k + 1}/kernel"].view(64, 3, 3, 64).permute(0, 3, 1, 2)
                xn = x.reshape(B * I * NP, PH, PW, 64).permute(0, 3, 1, 2)
                y = F.conv2d(xn, w3, p[f"{name}/Conv_{k + 1}/bias"], padding=1)
                x = gb(y.permute(0, 2, 3, 1).reshape(B, I * NP * PH * PW, 64))
        x = (x + residual).reshape(B, I * NP, PH * PW * 64)                    # flatten (h, w, c)
        img = self.rbg(dense(p, f"{name}/Dense_0", rb(x)))                      # (B, I*NP, D)
        if trace is not None:
            trace["img"] = img.detach().clone()
        rt, ct = (torch.as_tensor(a).long() for a in positions)
        return img + p["ImageTokenizer_0/image_row_position_embedding/embedding"][rt] + \
            p["ImageTokenizer_0/image_col_position_embedding/embedding"][ct]

    def text(self, text_ids, trace=None):
        """t5_base.py:8-15 (frozen) + the build's Dense(768 -> D) when D != 768."""
        cfg, p = self.cfg, self.p
        if self.t5p is None or text_ids is None:
            return None
        t5o = t5_encoder(self.t5p, torch.as_tensor(text_ids), cfg.t5.num_layers,
                         cfg.t5.num_heads, cfg.t5.d_kv, cfg.t5.layer_norm_epsilon,
                         emulate_bf16=self.emulate).detach()
        txt = self.text_proj(t5o)
        if trace is not None:
            trace["t5"], trace["txt"] = t5o.detach().clone(), txt.detach().clone()
        return txt

    def text_proj(self, t5o):
        p = self.p
        return self.rbg(dense(p, "TextProjection_0", t5o)) if "TextProjection_0/kernel" in p else t5o

    def assemble(self, img, txt, sequence, B):
        """token_sequencer.py:255-269 + readout.py:18-33 (zeros + embedding) + the stack's
        learned position embedding (attention.py:97-100)."""
        p = self.p
        NP = (self.cfg.image_size[0] // self.cfg.patch_size) ** 2
        ro = p["AddPositionEmbedding_0/pos_embedding"][None].expand(B, -1, -1)
        parts, ti, ii, ri = [], 0, 0, 0
        for kind, n, ts, _ in sequence:
            if kind in ("prefix", "text"):
                parts.append(txt[:, ti:ti + n]); ti += n
            elif kind == "image":
                parts.append(img[:, ii * NP:(ii + 1) * NP]); ii += 1
            else:
                parts.append(ro[:, ri:ri + n]); ri += n
        x = torch.cat(parts, dim=1)
        return self._q(x + p["StackedEncoder1DBlock_0/posembed_input/pos_embedding"][None])

    def block(self, x, layer, sequence, size, *, seed, step, sample_offset=0, train=True,
              tome_indices=None, trace=None):
        """Encoder1DBlock (attention.py:41-69) with ToMe after the attention residual
        (tome_attention.py:249-256 placement), or top-k pruning of the attention output when
        cfg.compression == "prune". Returns (x_out, size_out, used) with used = the ToMe
        (unm, src, dst) triple, the (B, K) top-k row indices, or None; tome_indices injects
        either instead of recomputing it."""
        def tr(name, v):
            if trace is not None:
                if trace.get("_retain"):  # diagnostics (tools/golden_diag.py): keep the graph node
                    if v.requires_grad:
                        v.retain_grad()
                    trace[f"b{layer}/{name}"] = v
                else:
                    trace[f"b{layer}/{name}"] = v.detach().clone()
            return v
        cfg, p = self.cfg, self.p
        rb, gb, rbg = self.rb, self.gb, self.rbg
        D, H = cfg.token_embedding_dim, cfg.num_heads
        Dh = D // H
        B, L = x.shape[:2]
        kp = 1.0 - cfg.dropout_rate
        kpa = 1.0 - cfg.attention_dropout_rate
        blk = f"StackedEncoder1DBlock_0/Block_{layer}"
        lens = [s[1] for s in sequence]
        tr("x", x)
        cur = [(k, lens[i] - layer * c, ts) for i, (k, _, ts, c) in enumerate(sequence)]
        mask = torch.from_numpy(literal_mask(cur))
        y = tr("y0", rbg(seq_layernorm(x, p[f"{blk}/LayerNorm_0/scale"], p[f"{blk}/LayerNorm_0/bias"],
                                       cfg.layer_norm_eps)))
        bdense = dense_fp8 if getattr(cfg, "fp8", False) else dense
        # the residual-stream products (out-projection, Dense_1) in e4m3 only with fp8_residual
        rdense = dense_fp8 if getattr(cfg, "fp8", False) and getattr(cfg, "fp8_residual", False) else dense
        qkv = tr("qkv", rbg(bdense(p, f"{blk}/SelfAttention_0/qkv", y)))
        q, k, v = qkv.split(D, dim=-1)
        k, v = k.reshape(B, L, H, Dh), v.reshape(B, L, H, Dh)
        keep = (torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 0, L, L, 0, kpa))
                if train else None)
        if self.emulate:
            o = FlashAttnBF16.apply(q.reshape(B, L, H, Dh), k, v, mask, keep,
                                    kpa if train else 1.0, 1.0 / math.sqrt(Dh), None)
            o = tr("o", rbg(o.reshape(B, L, D)))
        else:
            s = torch.einsum("bqhd,bkhd->bhqk", q.reshape(B, L, H, Dh) / math.sqrt(Dh), k)
            s = torch.where(mask[None, None], s, torch.finfo(torch.float32).min)
            a = torch.softmax(s, -1)
            if train:
                a = torch.where(keep[None, None], a / kpa, torch.zeros_like(a))
            o = tr("o", torch.einsum("bhqk,bkhd->bqhd", a, v).reshape(B, L, D))
        used = None
        merged = [i for i, c in enumerate(sequence) if c[3] > 0]
        pruning = bool(merged) and getattr(cfg, "compression", "tome") == "prune"
        if pruning:
            # compressed_attention.py:302-308: importance = mean over keys, then heads, of the
            # post-dropout attention weights; top-k per token set on it (token_compression.py:
            # 15-46) applied to the attention output before the out-projection; the residual
            # takes the block input's rows at the same indices (attention_blocks/attention.py)
            with torch.no_grad():
                sc = torch.einsum("bqhd,bkhd->bhqk", q.reshape(B, L, H, Dh).float(), k.float()) / math.sqrt(Dh)
                sc = sc.masked_fill(~mask[None, None], float("-inf"))
                a = torch.softmax(sc, -1)
                if train:
                    a = torch.where(keep[None, None], a / kpa, torch.zeros_like(a))
                imp = tr("imp", a.mean(-1).mean(1))                              # (B, L)
            if tome_indices is not None:
                idx = torch.as_tensor(np.asarray(tome_indices)).long()
            else:
                from .tome import topk_tokens
                sets, starts = [], 0
                for (_, ln, _) in cur:
                    sets.append((starts, ln))
                    starts += ln
                ks = [lens[i] - (layer + 1) * c[3] for i, c in enumerate(sequence)]
                idx = torch.from_numpy(np.stack([topk_tokens(np.zeros((L, 1), np.float32),
                                                             imp[b].numpy(), sets, ks)[1]
                                                 for b in range(B)])).long()
            used = idx.to(torch.int32)
            bidx = torch.arange(B)[:, None]
            o, x = o[bidx, idx], x[bidx, idx]
        Lo = o.shape[1]
        o = gb(rdense(p, f"{blk}/SelfAttention_0/out", o))
        if train:
            keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 1, B * Lo, D,
                                                      sample_offset * Lo, kp)).view(B, Lo, D)
            o = torch.where(keep, o / kp, torch.zeros_like(o))
        x = self._q(x + o)
        if merged and not pruning:
            # one bipartite match + merge_wavg per compressed set (token_sequencer.py:222-238
            # counts per set), the last set first so the earlier sets' starts stay valid; with
            # several sets `size` / `tome_indices` / `used` are per set ({set: (B, t, 1)} /
            # [triple per set in set order]), with one set a tensor / a triple as before
            multi = len(merged) > 1
            given = (list(tome_indices) if multi else [tome_indices]) if tome_indices is not None \
                else [None] * len(merged)
            sizes = (size or {}) if multi else {merged[0]: size}
            new_sizes, used_l = {}, []
            for si, tri in sorted(zip(merged, given), key=lambda z: -z[0]):
                r = sequence[si][3]
                s0 = sum(ln for _, ln, _ in cur[:si])
                tcur = cur[si][1]
                if tri is not None:
                    unm, src, dst = tri
                else:  # canonical C matching on this restatement's own key metric (sum over heads)
                    from . import tome as T
                    km = k.detach().float()[:, s0:s0 + tcur].contiguous().numpy()
                    unm, src, dst, _ = T.canon_match(km, r)
                    unm, src, dst = (torch.from_numpy(a) for a in (unm, src, dst))
                xs, new_sizes[si] = tome_merge_wavg(x[:, s0:s0 + tcur], sizes.get(si), unm, src, dst, r)
                x = torch.cat([x[:, :s0], xs, x[:, s0 + tcur:]], dim=1)
                used_l.append((si, (unm, src, dst)))
            used_l.sort(key=lambda z: z[0])
            used = [u for _, u in used_l] if multi else used_l[0][1]
            size = new_sizes if multi else new_sizes[merged[0]]
        L2 = x.shape[1]
        tr("x1", x)
        z = tr("y1", rbg(seq_layernorm(x, p[f"{blk}/LayerNorm_1/scale"], p[f"{blk}/LayerNorm_1/bias"],
                                       cfg.layer_norm_eps)))
        h = torch.relu(gb(bdense(p, f"{blk}/MLPBlock_0/Dense_0", z)))
        if train:
            keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 2, B * L2, cfg.mlp_dim,
                                                      sample_offset * L2, kp)).view(B, L2, -1)
            h = torch.where(keep, h / kp, torch.zeros_like(h))
        h = tr("h", rb(h))
        z = gb(rdense(p, f"{blk}/MLPBlock_0/Dense_1", h))
        if train:
            keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 3, B * L2, D,
                                                      sample_offset * L2, kp)).view(B, L2, D)
            z = torch.where(keep, z / kp, torch.zeros_like(z))
        return self._q(x + z), size, used

    def readout_rows(self, sequence):
        """Readout positions in the final (compressed) layout (octo.py:122-124)."""
        nb = self.cfg.num_blocks
        idx, cur_pos = [], 0
        for kind, n, _, c in sequence:
            n = n - nb * c
            if kind == "readout":
                idx.extend(range(cur_pos, cur_pos + n))
            cur_pos += n
        return idx

    def head_loss(self, x, sequence, actions, t, eps):
        """Readout mean (diffusion.py:102) -> denoise_loss (diffusion.py:110-143)."""
        cfg, p, dt = self.cfg, self.p, self.dtype
        rb, gb, rbg = self.rb, self.gb, self.rbg
        B = x.shape[0]
        e = rbg(x[:, self.readout_rows(sequence)].mean(dim=1))
        hp = "diffusion_action_head/OctoDenoise_0"
        betas = cosine_beta_schedule(cfg.diffusion_steps)
        alphas = 1 - betas
        ahat = torch.from_numpy(np.array([np.prod(alphas[:i + 1], dtype=np.float32)
                                          for i in range(cfg.diffusion_steps)], dtype=np.float32)).to(dt)
        tt = torch.as_tensor(t).long().view(B, 1)
        eps_t = torch.as_tensor(eps).to(dt)
        ah = ahat[tt]
        noisy = rb(torch.sqrt(ah) * torch.as_tensor(actions).to(dt) + torch.sqrt(1 - ah) * eps_t)
        w = p[f"{hp}/FourierFeatures_0/fourier_kernel"]                        # (F, 1)
        hh = 2 * math.pi * tt.to(dt) @ w.t()
        feats = rbg(torch.cat([torch.cos(hh), torch.sin(hh)], dim=-1))
        ht = rb(torch.relu(gb(dense(p, f"{hp}/FourierFeatures_0/MLPBlock_0/Dense_0", feats))))
        temb = dense(p, f"{hp}/FourierFeatures_0/MLPBlock_0/Dense_1", ht)
        cat = rbg(torch.cat([noisy, temb, e], dim=-1))
        hd = rb(torch.relu(gb(dense(p, f"{hp}/MLPBlock_0/Dense_0", cat))))
        pred = gb(dense(p, f"{hp}/MLPBlock_0/Dense_1", hd))
        i = 1   # OctoDenoise num_blocks > 1 (diffusion.py:62-63): the next MLPBlocks on pred
        while f"{hp}/MLPBlock_{i}/Dense_0/kernel" in p:
            h = rb(torch.relu(gb(dense(p, f"{hp}/MLPBlock_{i}/Dense_0", rbg(pred)))))
            pred = gb(dense(p, f"{hp}/MLPBlock_{i}/Dense_1", h))
            i += 1
        loss = (0.5 * (pred - eps_t) ** 2).sum(-1).mean()
        return loss, dict(pred=pred, e=e)

    # ---------------------------------------------------------------------- whole step
    def forward_loss(self, text_ids, images, actions, *, seed: int, step: int, positions,
                     t, eps, tome_indices: Optional[List] = None, sequence=None,
                     sample_offset: int = 0, train: bool = True, record: Optional[list] = None,
                     trace: Optional[dict] = None):
        """octo.py:91-126,139-145. Returns (loss, extras). sequence: list of (kind, n, timestep,
        compressed_per_layer). record (list): receives per block the block input x
        (retain_grad); extras["tome"] lists the ToMe index triples used. trace (dict): receives
        detached intermediates by name (b{layer}/{x,y0,qkv,o,x1,y1,h}, txt, img)."""
        images = torch.as_tensor(images)
        B = images.shape[0]
        img = self.stem(images, positions, trace)
        txt = self.text(text_ids, trace)
        x = self.assemble(img, txt, sequence, B)
        size = None
        used_tome = []
        for layer in range(self.cfg.num_blocks):
            if record is not None:
                x.retain_grad()
                record.append(x)
            x, size, used = self.block(x, layer, sequence, size, seed=seed, step=step,
                                       sample_offset=sample_offset, train=train,
                                       tome_indices=None if tome_indices is None else tome_indices[layer],
                                       trace=trace)
            if used is not None:
                used_tome.append(used)
        loss, ex = self.head_loss(x, sequence, actions, t, eps)
        return loss, dict(pred=ex["pred"], e=ex["e"], x_final=x, tome=used_tome)


def sequence_spec(token_sequence_str: str, compression_str: Optional[str]):
    """(kind, n, timestep, compressed_per_layer) list parsed with the reference grammar
    (token_sequencer.py:199-253)."""
    import re
    kinds = {"TaskDescriptionPrefix": "prefix", "Text": "text", "Image": "image", "Readout": "readout"}
    blocks = re.findall(r"\[(.*?)\]", token_sequence_str)
    reps = []
    for rep in re.findall(r"(?<=\])(.*?)(?=\[|$)", token_sequence_str):
        reps.append(1 if rep.strip() == "" else int(re.findall(r"\*(\d+)", rep)[0]))
    cblocks = re.findall(r"\[(.*?)\]", compression_str) if compression_str else [None] * len(blocks)
    out, t = [], 0
    for blk, cblk, rep in zip(blocks, cblocks, reps):
        groups = blk.split(";")
        cgroups = cblk.split(";") if cblk else [None] * len(groups)
        for _ in range(rep):
            for g, cg in zip(groups, cgroups):
                name = re.search(r"^\s*(.*?)\{", g).group(1).strip()
                n = int(re.search(r"\d+", g).group())
                c = int(re.search(r"\d+", cg).group()) if cg else 0
                out.append((kinds[name], n, t, c))
            t += 1
    return out
