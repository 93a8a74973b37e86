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


def t5_encoder(tp: Dict[str, torch.Tensor], ids: torch.Tensor, num_layers: int, H: int, d_kv: int,
               eps: float = 1e-6, prefix="T5Tokenizer_0", num_buckets=32, max_distance=128):
    """FlaxT5 encoder forward (t5_base.py:11-15): RMS layer norm, relative-position-biased
    attention without 1/sqrt(d) scaling, ReLU FF, pre-norm residuals, final norm."""
    def rms(x, w):
        return x * torch.rsqrt((x * x).mean(-1, keepdim=True) + eps) * w
    B, T = ids.shape
    x = tp[f"{prefix}/shared/embedding"][ids.long()]
    pos = torch.arange(T)
    bucket = t5_bucket(pos[None, :] - pos[:, None], num_buckets, max_distance)
    bias = tp[f"{prefix}/relative_attention_bias"][bucket].permute(2, 0, 1)  # (H, T, T)
    inner = H * d_kv
    for i in range(num_layers):
        p = f"{prefix}/block/{i}"
        n = rms(x, tp[f"{p}/layer_0/layer_norm"])
        qkv = n @ tp[f"{p}/SelfAttention/qkv"].t()
        q, k, v = qkv.split(inner, dim=-1)
        q, k, v = (a.view(B, T, H, d_kv) for a in (q, k, v))
        s = torch.einsum("bqhd,bkhd->bhqk", q, k) + bias[None]
        a = torch.softmax(s, -1)
        o = torch.einsum("bhqk,bkhd->bqhd", a, v).reshape(B, T, inner)
        x = x + o @ tp[f"{p}/SelfAttention/o"].t()
        n = rms(x, tp[f"{p}/layer_1/layer_norm"])
        x = x + torch.relu(n @ tp[f"{p}/DenseReluDense/wi"].t()) @ tp[f"{p}/DenseReluDense/wo"].t()
    return rms(x, tp[f"{prefix}/final_layer_norm"])


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
    t5_params: {name: fp32 CPU tensor} (frozen)."""

    def __init__(self, cfg, params: Dict[str, torch.Tensor], t5_params: Optional[Dict] = None,
                 dtype=torch.float32):
        self.cfg = cfg
        self.dtype = dtype
        self.residual_round = None
        self.p = params
        self.t5p = t5_params

    def _q(self, x):
        """Optional emulation of a storage rounding of the residual stream (diagnostics only)."""
        if self.residual_round is None:
            return x
        return x + (x.detach().to(self.residual_round).to(x.dtype) - x.detach())

    def forward_loss(self, text_ids, images, actions, *, seed: int, step: int, positions,
                     t, eps, tome_indices: Optional[List] = None, sequence=None,
                     sample_offset: int = 0, train: bool = True, record: Optional[list] = None):
        """Returns (loss, extras). sequence: list of (kind, n, timestep, compressed_per_layer)."""
        cfg, p = self.cfg, self.p
        D, H = cfg.token_embedding_dim, cfg.num_heads
        Dh = D // H
        dt = self.dtype
        images = torch.as_tensor(images).to(dt)
        B, I = images.shape[:2]
        # ---- image tokenizer (image_tokenizer.py:235-309)
        P = cfg.patch_size
        NP = (cfg.image_size[0] // P) ** 2
        patches = torch.stack([torch.stack([torch.from_numpy(image_to_patches(
            images[b, i].numpy(), P, True)) for i in range(I)]) for b in range(B)]).to(dt)
        x = patches.reshape(B * I * NP, P, P, 3).permute(0, 3, 1, 2)           # NCHW
        name = "ImageTokenizer_0/ResNetV2Block_0"
        wc = p[f"{name}/Conv_0/kernel"].view(64, 12, 12, 3).permute(0, 3, 1, 2)
        x = F.conv2d(x, wc, p[f"{name}/Conv_0/bias"], stride=2)
        x = F.max_pool2d(x, 3, stride=1)                                       # (N, 64, 1, 1)
        x = x.reshape(B, I * NP, 64)
        residual = x
        for k in range(2):
            x = groupnorm(x, 32, p[f"{name}/GroupNorm_{k}/scale"], p[f"{name}/GroupNorm_{k}/bias"], 1e-6)
            x = gelu_tanh(x)
            x = dense(p, f"{name}/Conv_{k + 1}", x)   # 3x3 SAME conv on a 1x1 map = centre tap
        x = x + residual
        img = dense(p, f"{name}/Dense_0", x)                                    # (B, I*NP, D)
        rt, ct = (torch.as_tensor(a).long() for a in positions)
        img = img + p["ImageTokenizer_0/image_row_position_embedding/embedding"][rt] + \
            p["ImageTokenizer_0/image_col_position_embedding/embedding"][ct]
        # ---- text
        txt = None
        if self.t5p is not None and text_ids is not None:
            t5o = t5_encoder(self.t5p, torch.as_tensor(text_ids), cfg.t5.num_layers,
                             cfg.t5.num_heads, cfg.t5.d_kv, cfg.t5.layer_norm_epsilon).detach()
            txt = dense(p, "TextProjection_0", t5o) if "TextProjection_0/kernel" in p else t5o
        # ---- readouts (readout.py:18-33 on zeros)
        ro = p["AddPositionEmbedding_0/pos_embedding"][None].expand(B, -1, -1)
        # ---- assemble (token_sequencer.py:255-269)
        parts, ti, ii, ri = [], 0, 0, 0
        for kind, n, ts, _ in sequence:
            if kind in ("prefix", "text"):
                parts.append(txt[:, ti:ti + n]); ti += n
            elif kind == "image":
                parts.append(img[:, ii * NP:(ii + 1) * NP]); ii += 1
            else:
                parts.append(ro[:, ri:ri + n]); ri += n
        x = torch.cat(parts, dim=1)
        L0 = x.shape[1]
        x = self._q(x + p["StackedEncoder1DBlock_0/posembed_input/pos_embedding"][None])
        # ---- stack
        kp = 1.0 - cfg.dropout_rate
        kpa = 1.0 - cfg.attention_dropout_rate
        lens = [s[1] for s in sequence]
        size = None
        for layer in range(cfg.num_blocks):
            blk = f"StackedEncoder1DBlock_0/Block_{layer}"
            L = x.shape[1]
            if record is not None:
                x.retain_grad()
                record.append(x)
            cur = [(k, lens[i] - layer * c, ts) for i, (k, _, ts, c) in enumerate(sequence)]
            mask = torch.from_numpy(literal_mask(cur))
            y = seq_layernorm(x, p[f"{blk}/LayerNorm_0/scale"], p[f"{blk}/LayerNorm_0/bias"], cfg.layer_norm_eps)
            qkv = dense(p, f"{blk}/SelfAttention_0/qkv", y)
            q, k, v = qkv.split(D, dim=-1)
            q = q.view(B, L, H, Dh) / math.sqrt(Dh)
            k, v = k.view(B, L, H, Dh), v.view(B, L, H, Dh)
            s = torch.einsum("bqhd,bkhd->bhqk", q, k)
            s = torch.where(mask[None, None], s, torch.finfo(torch.float32).min)
            a = torch.softmax(s, -1)
            if train:
                keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 0, L, L, 0, kpa))
                a = torch.where(keep[None, None], a / kpa, torch.zeros_like(a))
            o = torch.einsum("bhqk,bkhd->bqhd", a, v).reshape(B, L, D)
            o = dense(p, f"{blk}/SelfAttention_0/out", o)
            if train:
                keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 1, B * L, D,
                                                          sample_offset * L, kp)).view(B, L, D)
                o = torch.where(keep, o / kp, torch.zeros_like(o))
            x = self._q(x + o)
            # ToMe after the attention residual (tome_attention.py:249-256 placement)
            merged = [i for i, c in enumerate(sequence) if c[3] > 0]
            if merged:
                si = merged[0]
                r = sequence[si][3]
                s0 = sum(ln for _, ln, _ in cur[:si])
                tcur = cur[si][1]
                if tome_indices is not None:
                    unm, src, dst = tome_indices[layer]
                else:  # standalone: canonical C matching on this restatement's own key metric
                    from . import tome as T
                    km = k.detach().float()[:, s0:s0 + tcur].contiguous().numpy()
                    unm, src, dst, _ = T.canon_match(km, r)
                    unm, src, dst = (torch.from_numpy(a) for a in (unm, src, dst))
                xs, size = tome_merge_wavg(x[:, s0:s0 + tcur], size, unm, src, dst, r)
                x = torch.cat([x[:, :s0], xs, x[:, s0 + tcur:]], dim=1)
            L2 = x.shape[1]
            z = seq_layernorm(x, p[f"{blk}/LayerNorm_1/scale"], p[f"{blk}/LayerNorm_1/bias"], cfg.layer_norm_eps)
            h = torch.relu(dense(p, f"{blk}/MLPBlock_0/Dense_0", z))
            if train:
                keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 2, B * L2, cfg.mlp_dim,
                                                          sample_offset * L2, kp)).view(B, L2, -1)
                h = torch.where(keep, h / kp, torch.zeros_like(h))
            z = dense(p, f"{blk}/MLPBlock_0/Dense_1", h)
            if train:
                keep = torch.from_numpy(R.dropout_mask_2d(seed, step, layer, 3, B * L2, D,
                                                          sample_offset * L2, kp)).view(B, L2, D)
                z = torch.where(keep, z / kp, torch.zeros_like(z))
            x = self._q(x + z)
        # ---- readouts (octo.py:122-124) and head (diffusion.py:88-143)
        final = [(k, lens[i] - cfg.num_blocks * c, ts) for i, (k, _, ts, c) in enumerate(sequence)]
        idx, cur_pos = [], 0
        for kind, n, _ in final:
            if kind == "readout":
                idx.extend(range(cur_pos, cur_pos + n))
            cur_pos += n
        e = x[:, idx].mean(dim=1)
        hp = "diffusion_action_head/OctoDenoise_0"
        betas = cosine_beta_schedule(cfg.diffusion_steps)
        alphas = 1 - betas
        ahat = torch.from_numpy(np.array([np.prod(alphas[:i + 1], dtype=np.float32)
                                          for i in range(cfg.diffusion_steps)], dtype=np.float32)).to(dt)
        tt = torch.as_tensor(t).long().view(B, 1)
        eps_t = torch.as_tensor(eps).to(dt)
        ah = ahat[tt]
        noisy = torch.sqrt(ah) * torch.as_tensor(actions).to(dt) + torch.sqrt(1 - ah) * eps_t
        w = p[f"{hp}/FourierFeatures_0/fourier_kernel"]                        # (F, 1)
        hh = 2 * math.pi * tt.to(dt) @ w.t()
        feats = torch.cat([torch.cos(hh), torch.sin(hh)], dim=-1)
        temb = dense(p, f"{hp}/FourierFeatures_0/MLPBlock_0/Dense_1",
                     torch.relu(dense(p, f"{hp}/FourierFeatures_0/MLPBlock_0/Dense_0", feats)))
        cat = torch.cat([noisy, temb, e], dim=-1)
        pred = dense(p, f"{hp}/MLPBlock_0/Dense_1", torch.relu(dense(p, f"{hp}/MLPBlock_0/Dense_0", cat)))
        loss = (0.5 * (pred - eps_t) ** 2).sum(-1).mean()
        return loss, dict(pred=pred, e=e, x_final=x)


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
