"""Transformer blocks, mirroring the reference's
``multi_modal_transformers/attention_blocks/attention.py`` (MLPBlock :20-39, Encoder1DBlock
:41-69, AddPositionEmbedding :71-85, StackedEncoder1DBlock :87-119) with ToMe inserted the way
``tome_attention.py:249-256`` intends (after the attention residual, before the MLP LayerNorm).

Semantics kept from the reference:
  * pre-LN block: y = LN0(x); y = MHA(y); y = Dropout(y); x = x + y; z = LN1(x); MLP; x + z,
    with LayerNorm over the SEQUENCE axis (reduction_axes=[1]);
  * Flax SelfAttention: q/sqrt(Dh), finfo.min masking, fp32 softmax, dropout(0.1) with one (L, L)
    mask broadcast over batch and heads; q/k/v/out DenseGeneral with bias (fused QKV here);
  * MLPBlock: Dense -> relu -> Dropout -> Dense -> Dropout (the YAML key ``norm`` is the Dropout);
  * ToMe metric = sum over heads of the key projection of the image token set, merged with
    merge_wavg and the set's token sizes carried across layers (no proportional attention);
  * top-k pruning (OctoConfig.compression == "prune"): importance = mean over keys, then over
    heads, of the post-dropout attention weights (compressed_attention.py:302-306, written by the
    attention forward as per-query row sums), compute_top_k_tokens per token set
    (token_compression.py:15-46) applied to the attention output BEFORE the out-projection
    (compressed_attention.py:308-326). The reference's CompressedEncoder1DBlock then discards
    the attention output (:349-354); the build adds it to the block input's
    rows at the same indices — the only residual that matches the pruned shape.
Every op is a libmmt_hip kernel (see layers.py); backward is explicit.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import os

import torch

from .. import _kernels as K
from ..layers import (DROP_ATTN, DROP_ATTN_OUT, DROP_MLP_HIDDEN, DROP_MLP_OUT, Dense, wgrad_overlap,
                      SeqLayerNorm)
from ..config_loader import LayerSpec
from ..module_api import Bindable, init_from_spec, merge_param, sget, spec
from ..params import ParamStore, he_normal, normal
from ..tracing import phase
from ..tokenizers.token_sequencer import LayerSets, sets_from_mask


@dataclass
class LayerCtx:
    """Static (capture-time) description of one block's sequence plus the step's RNG state."""
    layer: int
    sets: LayerSets                # token-set table entering the block
    table: K.SetTable
    tome_set: int = -1             # index of the merged token set, -1 = no merge, -2 = several
    r: int = 0                     # tokens merged away in this block (over every merged set)
    # top-k pruning: (((start, num_tokens) per set), (k per set)) or None
    prune: Optional[tuple] = None
    train: bool = True
    rng: Optional[torch.Tensor] = None
    sample_offset: int = 0         # global index of this rank's first sample (RNG counters)
    tome_forced: Optional[tuple] = None  # injected (unm, src, dst) in place of the matching (tests;
    #                                      a list of triples, one per merged set, with several)
    tome_plan: tuple = ()          # ((set index, r), ...): one ToMe match + merge per compressed set

    def tome_sets(self):
        """The merged sets as ((set index, r), ...)."""
        if self.tome_plan:
            return tuple(self.tome_plan)
        return ((self.tome_set, self.r),) if self.r > 0 else ()


_SIDE = {}


_RELU_BITS = os.environ.get("MMT_RELU_BITS", "1") != "0"  # benchmarking knob: bf16 gate instead
# MMT_KEEP_BITS=1: the MLP hidden dropout keeps drawn by their own kernel on the side queue
# (beside attention) and read as bits by the MLP-up GEMM's epilogue instead of drawn there
# (bit-identical outputs). Off by default: the MLP-up GEMM did not get faster (210.4 vs 209.7 us
# average over the step) and the step lost 0.7 % (15.10k vs 15.20k samples/s, 3 interleaved
# rounds) to the 27-66 us draw kernel beside attention — the epilogue's draws were not its cost.
_KEEP_BITS = os.environ.get("MMT_KEEP_BITS", "0") == "1"


def side_stream(device) -> torch.cuda.Stream:
    """Second HIP stream for small independent kernels (attention-dropout bits, ToMe matching)
    that overlap the main stream's GEMMs and attention. Discipline: every side launch follows a
    fork (side waits on main), and main waits on the side before consuming its results, so
    tensors passed between the streams are never reused early (this also holds under HIP-graph
    capture, where the side stream joins the capture through the fork)."""
    key = torch.device(device).index
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


class MLPBlock(Bindable):
    """attention.py:20-39: ``MLPBlock(dense, activation, norm, dense_out)(inputs, train=False)``
    = Dense -> activation -> Dropout (``norm``) -> Dense -> Dropout. The fields are the reference's
    config nodes (flax.linen.Dense features, flax.linen.relu, flax.linen.Dropout rate); the input
    width is taken from the first call (nn.compact), or from ``bind``. On the device: the NT GEMM
    with a fused bias + relu + dropout epilogue, then the GEMM with bias + dropout."""

    fp8 = False
    fp8_residual = False  # Dense_1 (the residual-stream product) in e4m3 too (OctoConfig.fp8_residual)

    def __init__(self, dense=None, activation=None, norm=None, dense_out=None):
        self.dense_spec, self.activation, self.norm, self.dense_out_spec = \
            spec(dense), spec(activation), spec(norm), spec(dense_out)
        act = getattr(self.activation, "target", "flax.linen.relu") if self.activation is not None \
            else "flax.linen.relu"
        if not act.endswith(".relu"):
            raise NotImplementedError(f"MLPBlock activation {act!r}: the fused GEMM epilogue is relu")
        self.rate = float(sget(self.norm, "rate", 0.0))
        self.dense = self.dense_out = None

    @classmethod
    def create(cls, store: ParamStore, name: str, in_f: int, hidden: int, out_f: int,
               dropout_rate: float = 0.1, fp8: bool = False, fp8_residual: bool = False) -> "MLPBlock":
        """The block from its dimensions, declared in ``store`` (the Octo model's path)."""
        m = cls(LayerSpec("flax.linen.Dense", {"features": hidden}),
                LayerSpec("flax.linen.relu", partial=True),
                LayerSpec("flax.linen.Dropout", {"rate": dropout_rate}),
                LayerSpec("flax.linen.Dense", {"features": out_f}))
        m.fp8, m.fp8_residual = fp8, fp8_residual
        return m.bind(store, name, in_f)

    def _declare(self, store, name, in_f):
        hidden = int(sget(self.dense_spec, "features"))
        out_f = int(sget(self.dense_out_spec, "features"))
        self.dense = Dense(store, f"{name}/Dense_0", in_f, hidden, fp8=self.fp8,
                           kernel_init=init_from_spec(sget(self.dense_spec, "kernel_init"), (in_f, hidden)),
                           bias_init=init_from_spec(sget(self.dense_spec, "bias_init"), (hidden,), normal(0.01)))
        self.dense_out = Dense(store, f"{name}/Dense_1", hidden, out_f, fp8=self.fp8 and self.fp8_residual,
                               kernel_init=init_from_spec(sget(self.dense_out_spec, "kernel_init"), (hidden, out_f)),
                               bias_init=init_from_spec(sget(self.dense_out_spec, "bias_init"), (out_f,), normal(0.01)))

    def __call__(self, inputs: torch.Tensor, train: bool = False, *, rng=None, layer: int = 0,
                 sample_offset: int = 0) -> torch.Tensor:
        """inputs (..., in) fp32 / bf16 device tensor -> (..., out) fp32. train=True applies the
        two dropouts with the counter RNG ``rng`` (a (seed, step) int32 device tensor, the
        'dropout' collection of the reference), keyed by (layer, site, row)."""
        self._ensure(inputs.device, int(inputs.shape[-1]))
        lead = inputs.shape[:-1]
        x2 = inputs.reshape(-1, inputs.shape[-1])
        if x2.dtype != torch.bfloat16:
            x2 = K.cast_f32_bf16(x2.float().contiguous(),
                                 torch.empty(x2.shape, dtype=torch.bfloat16, device=x2.device))
        drop = self.rate > 0.0 and train
        if drop and rng is None:
            raise ValueError("MLPBlock(train=True) needs the dropout rng (rng=)")
        kp = 1.0 - self.rate

        def epi(site):
            return dict(rng=rng, drop_layer=layer, drop_site=site, keep_prob=kp,
                        drop_row_offset=sample_offset) if drop else {}
        h = self.dense.fwd(x2.contiguous(), act=K.ACT_RELU, **epi(DROP_MLP_HIDDEN))
        y = self.dense_out.fwd(h, out_mode=K.OUT_F32, **epi(DROP_MLP_OUT))
        return y.view(*lead, y.shape[-1])


class Encoder1DBlock(Bindable):
    """attention.py:41-69 (+ ToMe between the attention residual and LN1 on the Octo path).

    ``Encoder1DBlock(layer_norm, dropout, self_attention, mlp_block, train=None, mask=None)`` with
    the reference's config nodes: flax.linen.LayerNorm (epsilon; reduction over the SEQUENCE
    axis, reduction_axes [1], vanilla_decoder.yaml:5-13), flax.linen.Dropout (rate),
    flax.linen.SelfAttention (num_heads, qkv_features = the input width, dropout_rate,
    kernel_init, bias_init) and an MLPBlock node (or MLPBlock). ``__call__(inputs, mask=None,
    train=None) -> (x, None)`` as the reference (train / mask from the constructor or the call,
    flax merge_param); the dense mask is converted to the token-set table the kernels evaluate
    (token_sequencer.sets_from_mask). Differentiable through torch autograd: the backward runs
    the block's explicit backward kernels and accumulates the parameter gradients in the store's
    flat gradient buffer (the ``grads`` of the reference's value_and_grad)."""

    fp8 = False
    fp8_residual = False  # the out-projection in e4m3 too (OctoConfig.fp8_residual)

    def __init__(self, layer_norm=None, dropout=None, self_attention=None, mlp_block=None,
                 train=None, mask=None):
        self.layer_norm, self.dropout, self.self_attention = spec(layer_norm), spec(dropout), \
            spec(self_attention)
        mlp = spec(mlp_block)
        if mlp is None:
            raise ValueError("Encoder1DBlock needs an mlp_block")
        if not isinstance(mlp, MLPBlock):
            raise TypeError(f"mlp_block must be an MLPBlock node, got {type(mlp).__name__}")
        self.mlp = mlp
        self.train, self.mask = train, mask
        ra = sget(self.layer_norm, "reduction_axes", [1])
        ra = list(ra) if isinstance(ra, (list, tuple)) else [ra]
        if ra != [1]:
            raise NotImplementedError(f"LayerNorm reduction_axes {ra}: the build normalises over the "
                                      "sequence axis, reduction_axes [1] (vanilla_decoder.yaml:10)")
        self.eps = float(sget(self.layer_norm, "epsilon", 1e-6))
        self.rate = float(sget(self.dropout, "rate", 0.0))
        self.H = int(sget(self.self_attention, "num_heads", 1))
        self.attn_rate = float(sget(self.self_attention, "dropout_rate", 0.0))

    @classmethod
    def create(cls, store: ParamStore, name: str, D: int, num_heads: int, mlp_dim: int,
               eps: float = 1e-6, dropout_rate: float = 0.1, attn_dropout_rate: float = 0.1,
               fp8: bool = False, fp8_residual: bool = False) -> "Encoder1DBlock":
        """The block from its dimensions, declared in ``store`` (the Octo model's path)."""
        blk = cls(LayerSpec("flax.linen.LayerNorm", {"epsilon": eps, "reduction_axes": [1],
                                                     "feature_axes": [-1]}),
                  LayerSpec("flax.linen.Dropout", {"rate": dropout_rate}),
                  LayerSpec("flax.linen.SelfAttention", {"num_heads": num_heads, "qkv_features": D,
                                                         "dropout_rate": attn_dropout_rate}),
                  MLPBlock(LayerSpec("flax.linen.Dense", {"features": mlp_dim}),
                           LayerSpec("flax.linen.relu", partial=True),
                           LayerSpec("flax.linen.Dropout", {"rate": dropout_rate}),
                           LayerSpec("flax.linen.Dense", {"features": D})))
        blk.fp8, blk.fp8_residual = fp8, fp8_residual
        return blk.bind(store, name, D)

    def _declare(self, store: ParamStore, name: str, D: int):
        qkv_f = sget(self.self_attention, "qkv_features")
        if qkv_f is not None and int(qkv_f) != D:
            raise ValueError(f"qkv_features {qkv_f} != the input width {D} (the fused QKV projection)")
        if D % self.H:
            raise ValueError("qkv_features must be divisible by num_heads")
        self.D, self.Dh = D, D // self.H
        sa = self.self_attention
        kinit = lambda: init_from_spec(sget(sa, "kernel_init"), (D, D))   # noqa: E731
        binit = init_from_spec(sget(sa, "bias_init"), (D,), normal(0.01))
        self.ln0 = SeqLayerNorm(store, f"{name}/LayerNorm_0", D, self.eps)
        self.qkv = Dense(store, f"{name}/SelfAttention_0/qkv", D, 3 * D, kernel_init=kinit(),
                         bias_init=binit, fp8=self.fp8)
        self.out = Dense(store, f"{name}/SelfAttention_0/out", D, D, kernel_init=kinit(),
                         bias_init=binit, fp8=self.fp8 and self.fp8_residual)
        self.ln1 = SeqLayerNorm(store, f"{name}/LayerNorm_1", D, self.eps)
        self.mlp.fp8, self.mlp.fp8_residual = self.fp8, self.fp8_residual
        self.mlp.bind(store, f"{name}/MLPBlock_0", D)
        if self.mlp.dense_out.out_f != D:
            raise ValueError("mlp_block.dense_out.features must equal the input width (residual)")
        self.M = self.mlp.dense.out_f
        self.scale = self.Dh ** -0.5

    def __call__(self, inputs: torch.Tensor, mask=None, train=None, *, rng=None, layer: int = 0,
                 sample_offset: int = 0):
        """inputs (B, L, D) -> (x, None), x fp32 (B, L, D). ``mask``: the dense reference mask
        (or a token-set table); ``rng``: the 'dropout' collection, a (seed, step) int32 device
        tensor (needed when train and a rate > 0); ``layer`` / ``sample_offset`` key the dropout
        streams like the Octo path (block index, global index of the first sample)."""
        train = bool(merge_param("train", self.train, train))
        mask = merge_param("mask", self.mask, mask)
        if inputs.dim() != 3:
            raise ValueError(f"inputs must be (batch, length, features), got {tuple(inputs.shape)}")
        self._ensure(inputs.device, int(inputs.shape[-1]))
        ctx = LayerCtx(layer=layer, sets=None, table=set_table_of(mask, inputs.shape[1]),
                       train=train, rng=rng, sample_offset=sample_offset)
        if train and (self.rate > 0 or self.attn_rate > 0 or self.mlp.rate > 0) and rng is None:
            raise ValueError("Encoder1DBlock(train=True) needs the dropout rng (rng=)")
        x = inputs.float().contiguous()
        return _EncoderBlockFn.apply(x, self, ctx), None

    # ------------------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, ctx: LayerCtx, size: Optional[torch.Tensor]):
        B, L, D = x.shape
        H, Dh = self.H, self.Dh
        train = ctx.train
        # attention-output dropout: the block's `dropout` node; the two MLP dropouts: the
        # mlp_block's own Dropout (`norm`) rate (reference attention.py:20-39, 60)
        kp = 1.0 - self.rate if train else 1.0
        kpm = 1.0 - self.mlp.rate if train else 1.0
        kpa = 1.0 - self.attn_rate if train else 1.0

        def drop(site, rows_per_sample, keep=None):
            keep = kp if keep is None else keep
            if not train or keep >= 1.0:
                return {}
            return dict(rng=ctx.rng, drop_layer=ctx.layer, drop_site=site, keep_prob=keep,
                        drop_row_offset=ctx.sample_offset * rows_per_sample)

        main = torch.cuda.current_stream()
        side = side_stream(x.device)
        bits = None
        y0, mu0, rs0 = self.ln0.fwd(x)
        qkv = self.qkv.fwd(y0.view(B * L, D)).view(B, L, 3 * D)
        tome_idx = None
        Mh = self.mlp.dense.out_f

        def relu_bits_ok(rows):
            return (train and not self.mlp.dense.fp8 and _RELU_BITS
                    and K.gemm_bits_supported(rows, Mh, D))
        kbits = None
        plan = ctx.tome_sets()
        multi = len(plan) > 1
        if ctx.r > 0:  # ToMe matching needs only K: it runs beside attention + out-projection
            metrics = []
            for si, _ in plan:
                s0, t = ctx.sets.starts[si], ctx.sets.lens[si]
                metrics.append(qkv.view(B, L, 3, H, Dh)[:, s0:s0 + t, 1])  # (B, t, H, Dh): sum_h K
            L2p = L - ctx.r  # the merged length (no pruning in this block)
            if (_KEEP_BITS and train and kpm < 1.0 and ctx.prune is None and Mh % 256 == 0
                    and relu_bits_ok(B * L2p)):
                kbits = torch.empty((-(-B * L2p // 256) * 256, Mh // 32), dtype=torch.int32,
                                    device=x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if ctx.tome_forced is not None:
                    tome_idx = ctx.tome_forced
                elif multi:
                    tome_idx = [K.tome_match(m, r) for m, (_, r) in zip(metrics, plan)]
                else:
                    tome_idx = K.tome_match(metrics[0], ctx.r)
                if kbits is not None:
                    K.gemm_dropout_keep_bits(ctx.rng, ctx.layer, DROP_MLP_HIDDEN, B * L2p, Mh, kpm,
                                             ctx.sample_offset * L2p, out=kbits)
        if train and kpa < 1:
            # the (L, L) attention keep mask (RNG state only), on the main stream: a 7 us launch
            # costs less than the cross-queue wait it took beside the QKV GEMM (~10 us idle)
            bits = K.dropout_bits(ctx.rng, ctx.layer, DROP_ATTN, L, L, kpa)
        wsum = (torch.empty((B, H, L), dtype=torch.float32, device=x.device)
                if ctx.prune is not None else None)
        o, lse = K.attn_fwd(qkv, H, self.scale, ctx.table, bits, kpa, wsum=wsum)
        prune = None
        o_in, x_res, Lo = o, x, L
        if ctx.prune is not None:
            scores = K.prune_importance(wsum)
            o_in, pidx = K.topk_gather(o, scores, *ctx.prune)
            x_res = K.gather_rows(x, pidx)
            Lo = o_in.shape[1]
            prune = (pidx, scores)
        # residual stream stays fp32 (sequence-axis LayerNorm conditioning, csrc/norm.hip)
        x1 = self.out.fwd(o_in.reshape(B * Lo, D), residual=x_res.reshape(B * Lo, D),
                          out_mode=K.OUT_F32, **drop(DROP_ATTN_OUT, Lo))
        x1 = x1.view(B, Lo, D)
        tome = None
        tome_sets = []
        new_size = size
        ln1_done = None
        if ctx.r > 0 and multi:
            # several merged sets: one merge per set, the last set first so the earlier sets'
            # starts stay valid; sizes carried per set ({set index: (B, t) sizes}); LayerNorm_1
            # on the merged sequence after them (unfused)
            main.wait_stream(side)
            sizes = size if isinstance(size, dict) else {}
            new_size = {}
            for (si, r), (unm, src, dst) in sorted(zip(plan, tome_idx), key=lambda z: -z[0][0]):
                s0, t = ctx.sets.starts[si], ctx.sets.lens[si]
                x1, ns, pos = K.tome_merge_fwd(x1, s0, t, r, unm, src, dst, size_in=sizes.get(si))
                new_size[si] = ns
                tome_sets.append((s0, t, r, pos, sizes.get(si), ns, unm, src, dst, si))
        elif ctx.r > 0:
            main.wait_stream(side)
            unm, src, dst = tome_idx
            if x1.dtype == torch.float32 and Lo - ctx.r <= 512:
                # merge + LayerNorm_1 in one pass over the fp32 sequence (bit-identical outputs)
                x1, new_size, pos, y1, mu1, rs1 = K.tome_merge_seqnorm_fwd(
                    x1, s0, t, ctx.r, unm, src, dst, self.ln1.scale.data, self.ln1.bias.data,
                    self.ln1.eps, size_in=size)
                ln1_done = (y1, mu1, rs1)
            else:
                x1, new_size, pos = K.tome_merge_fwd(x1, s0, t, ctx.r, unm, src, dst, size_in=size)
            tome = (s0, t, ctx.r, pos, size, new_size, unm, src, dst, plan[0][0])
            tome_sets = [tome]
        L2 = x1.shape[1]
        y1, mu1, rs1 = ln1_done if ln1_done is not None else self.ln1.fwd(x1)
        # the relu gate of the backward as 1 bit per hidden unit where the launch supports it
        # (the gated dX then reads M*Mh/8 bytes instead of h's 2*M*Mh)
        hbits = (torch.empty((-(-B * L2 // 256) * 256, Mh // 32), dtype=torch.int32, device=x.device)
                 if relu_bits_ok(B * L2) else None)
        if kbits is not None and hbits is not None and L2 == L - ctx.r:
            hdrop = dict(keep_bits=kbits, keep_prob=kpm)   # (joined with the side queue above)
        else:
            hdrop = drop(DROP_MLP_HIDDEN, L2, kpm)
        h = self.mlp.dense.fwd(y1.view(B * L2, D), act=K.ACT_RELU, relu_bits=hbits, **hdrop)
        x2 = self.mlp.dense_out.fwd(h, residual=x1.view(B * L2, D), out_mode=K.OUT_F32,
                                    **drop(DROP_MLP_OUT, L2, kpm))
        saved = dict(x=x, y0=y0, mu0=mu0, rs0=rs0, qkv=qkv, o=o, o_in=o_in, lse=lse, bits=bits,
                     x1=x1, y1=y1, mu1=mu1, rs1=rs1, h=h, hbits=hbits, tome=tome, prune=prune,
                     kp=kp, kpm=kpm, kpa=kpa,
                     # every merge of the block in the order applied (one set: [tome]; several:
                     # the last set first, `tome` then None)
                     tome_sets=tome_sets)
        return x2.view(B, L2, D), saved, new_size

    # ----------------------------------------------------------------------------- backward
    def backward(self, dx2: torch.Tensor, sv: dict, ctx: LayerCtx, dz2=None, prev=None):
        """Returns (dx, dz_prev). dz2: this block's MLP-output dropout backward of dx2, already
        produced by the next block's LayerNorm_0 backward (with this block's Dense_1 bias
        gradient), or None; prev = (block, saved, ctx) of the block before this one, whose
        dropout backward this block's LayerNorm_0 backward then produces (dz_prev)."""
        B, L2, D = dx2.shape
        L = sv["x"].shape[1]
        kp, kpm, kpa, train = sv["kp"], sv["kpm"], sv["kpa"], ctx.train
        dropping, dropping_m = train and kp < 1.0, train and kpm < 1.0
        dx2f = dx2.reshape(B * L2, D)                      # fp32 residual-stream gradient
        rng = ctx.rng if dropping else None
        rng_m = ctx.rng if dropping_m else None
        # MLP out: x2 = x1 + drop3(h W2^T + b2); dropout backward = mask/scale + cast to bf16,
        # fused with the bias gradient (column sum)
        if dz2 is None:
            dz2 = K.dropout_bwd(dx2f, rng_m, ctx.layer, DROP_MLP_OUT, kpm,
                                row_offset=ctx.sample_offset * L2,
                                colsum_out=self.mlp.dense_out.b.grad)
        # dh gated by (h > 0): relu + hidden-dropout backward fused into the dX GEMM epilogue,
        # which also writes per-256-row column sums of dz1 (Dense_0's bias gradient) where the
        # launch supports it
        Mh = self.mlp.dense.out_f
        rows = K.gemm_colsum_rows(B * L2, Mh, D)
        cs = torch.empty((rows, Mh), dtype=torch.float32, device=dz2.device) if rows else None
        gate = dict(gate_bits=sv["hbits"]) if sv.get("hbits") is not None else dict(gate=sv["h"])
        dz1 = self.mlp.dense_out.bwd(dz2, sv["h"], bias_grad_done=True,
                                     gate_scale=(1.0 / kpm) if dropping_m else 1.0, colsum=cs, **gate)
        # dX of the LN-fed Dense in bf16 (the LN backward accumulates in fp32): halves its traffic
        dy1 = self.mlp.dense.bwd(dz1, sv["y1"].view(B * L2, D), dy_colsum=cs)
        Lo = sv["o_in"].shape[1]
        if (sv["tome"] is not None and K.ln_unmerge_ok(Lo, L2)
                and sv["x1"].dtype == torch.float32):
            # LayerNorm_1 backward + unmerge + attention-output dropout backward in one pass (the
            # merged-layout gradient never reaches HBM)
            dx1, dzo = K.ln_unmerge_dropout_bwd(
                dy1.view(B, L2, D), sv["x1"], sv["mu1"], sv["rs1"], self.ln1.scale.data,
                self.ln1.scale.grad, self.ln1.bias.grad, dx2, sv["tome"][:6], rng, ctx.layer,
                DROP_ATTN_OUT, kp, ctx.sample_offset * Lo, bias_grad=self.out.b.grad)
            dzo = dzo.view(B * Lo, D)
        else:
            dx1 = self.ln1.bwd(dy1.view(B, L2, D), sv["x1"], sv["mu1"], sv["rs1"], addend=dx2)
            for tm in reversed(sv.get("tome_sets") or []):  # the merges undone in reverse order
                s0, t, r, pos, size_in, size_out = tm[:6]
                dx1 = K.tome_merge_bwd(dx1, s0, t, r, pos, size_in, size_out)
            dx1f = dx1.reshape(B * Lo, D)
            dzo = K.dropout_bwd(dx1f, rng, ctx.layer, DROP_ATTN_OUT, kp,
                                row_offset=ctx.sample_offset * Lo, colsum_out=self.out.b.grad)
        do = self.out.bwd(dzo, sv["o_in"].reshape(B * Lo, D), bias_grad_done=True)
        if sv["prune"] is not None:  # the top-k indices carry no gradient (lax.top_k indices)
            pidx = sv["prune"][0]
            do = K.topk_scatter_bwd(do.view(B, Lo, D), pidx, L)
            dx1 = K.topk_scatter_bwd(dx1.view(B, Lo, D), pidx, L)
        # the QKV bias gradient (column sums of dqkv) is accumulated inside the attention backward
        dqkv = K.attn_bwd(sv["qkv"], sv["o"], do.view(B, L, D), sv["lse"], self.H, self.scale,
                          ctx.table, sv["bits"], kpa, bias_grad=self.qkv.b.grad)
        dy0 = self.qkv.bwd(dqkv.view(B * L, 3 * D), sv["y0"].view(B * L, D), bias_grad_done=True)
        if prev is not None and sv["x"].dtype == torch.float32 and dy0.dtype == torch.bfloat16:
            pblk, psv, pctx = prev
            pkp = psv["kpm"]  # block i-1's MLP-output dropout
            prng = pctx.rng if (pctx.train and pkp < 1.0) else None
            dx, dzp = K.seqnorm_dropout_bwd(
                dy0.view(B, L, D), sv["x"], sv["mu0"], sv["rs0"], self.ln0.scale.data,
                self.ln0.scale.grad, self.ln0.bias.grad, dx1, prng, pctx.layer, DROP_MLP_OUT, pkp,
                pctx.sample_offset * L, colsum=pblk.mlp.dense_out.b.grad)
            return dx, dzp.view(B * L, D)
        return self.ln0.bwd(dy0.view(B, L, D), sv["x"], sv["mu0"], sv["rs0"], addend=dx1), None


def set_table_of(mask, L: int) -> K.SetTable:
    """The kernels' token-set table for a reference mask (dense array / tensor), a LayerSets, or
    an existing SetTable."""
    if isinstance(mask, K.SetTable):
        sets = mask
    else:
        ls = mask if isinstance(mask, LayerSets) else sets_from_mask(mask)
        sets = K.SetTable(ls.starts, ls.lens, ls.vis, ls.causal)
    if sets.L != L:
        raise ValueError(f"mask covers {sets.L} tokens, inputs have {L}")
    return sets


class _EncoderBlockFn(torch.autograd.Function):
    """One Encoder1DBlock under torch autograd: forward/backward are the block's explicit
    kernel schedules; parameter gradients go to the store's flat gradient buffer."""

    @staticmethod
    def forward(fctx, x, blk, ctx):
        y, sv, _ = blk.forward(x, ctx, None)
        fctx.blk, fctx.ctx, fctx.sv = blk, ctx, sv
        return y

    @staticmethod
    def backward(fctx, dy):
        dx, _ = fctx.blk.backward(dy.float().contiguous(), fctx.sv, fctx.ctx)
        fctx.sv = None
        return dx, None, None


class _StackFn(torch.autograd.Function):
    """posembed_input + the blocks under torch autograd (StackedEncoder1DBlock.__call__)."""

    @staticmethod
    def forward(fctx, x, stack, ctxs):
        y, saved = stack.forward(stack.pos(x), ctxs)
        fctx.stack, fctx.ctxs, fctx.saved = stack, ctxs, saved
        return y

    @staticmethod
    def backward(fctx, dy):
        dx = fctx.stack.backward(dy.float().contiguous(), fctx.saved, fctx.ctxs)
        fctx.stack.pos.backward(dx)      # d(pos_embedding) += column sums over the batch
        fctx.saved = None
        return dx, None, None


class StackedEncoder1DBlock(Bindable):
    """attention.py:87-119: ``StackedEncoder1DBlock(num_blocks, encoder_1d_block)(x, train=False,
    mask=None)`` = x + posembed_input (AddPositionEmbedding, normal(0.02)), then num_blocks
    Encoder1DBlocks built from the ``encoder_1d_block`` node (nn.scan over identical blocks in the
    reference). With ToMe the sequence shrinks per block, so the stack is a Python loop over
    per-block parameter sets (names Block_{i}); the Octo path drives ``forward`` / ``backward``
    with per-layer contexts (token-set tables, ToMe / pruning) directly."""

    def __init__(self, num_blocks: int = 1, encoder_1d_block=None):
        self.num_blocks = int(num_blocks)
        node = encoder_1d_block
        if isinstance(node, Encoder1DBlock):
            raise TypeError("encoder_1d_block must be the block's config node (one block per layer "
                            "is built from it)")
        self.block_node = node
        self.blocks: List[Encoder1DBlock] = []
        self.pos = None

    def _make_block(self) -> Encoder1DBlock:
        node = self.block_node
        if node is None:
            raise ValueError("StackedEncoder1DBlock needs encoder_1d_block")
        if isinstance(node, dict):
            kw = {k: v for k, v in node.items() if k not in ("_target_", "_partial_", "_recursive_")}
            return Encoder1DBlock(**kw)
        return Encoder1DBlock(node.layer_norm, node.dropout, node.self_attention, node.mlp)

    @classmethod
    def create(cls, store: ParamStore, name: str, num_blocks: int, D: int, num_heads: int,
               mlp_dim: int, eps: float = 1e-6, dropout_rate: float = 0.1,
               attn_dropout_rate: float = 0.1, fp8: bool = False,
               fp8_residual: bool = False) -> "StackedEncoder1DBlock":
        """The stack's blocks declared in ``store`` (the Octo model's path; its posembed_input
        is declared by the model, which adds it inside the fused sequence assembly)."""
        st = cls(num_blocks, None)
        st.blocks = [Encoder1DBlock.create(store, f"{name}/Block_{i}", D, num_heads, mlp_dim, eps,
                                           dropout_rate, attn_dropout_rate, fp8, fp8_residual)
                     for i in range(num_blocks)]
        st._store, st._name = store, name
        return st

    def _declare(self, store: ParamStore, name: str, L: int, D: int):
        from ..tokenizers.readout.readout import AddPositionEmbedding
        self.pos = AddPositionEmbedding(normal(0.02)).bind(store, f"{name}/posembed_input", L, D)
        self.blocks = [self._make_block().bind(store, f"{name}/Block_{i}", D)
                       for i in range(self.num_blocks)]

    def __call__(self, x: torch.Tensor, train: bool = False, mask=None, *, rng=None,
                 sample_offset: int = 0) -> torch.Tensor:
        """x (B, L, D) -> (B, L, D) fp32: posembed_input, then the blocks with the same mask
        (train / mask forwarded to every block, attention.py:111-117)."""
        if x.dim() != 3:
            raise ValueError(f"x must be (batch, length, features), got {tuple(x.shape)}")
        B, L, D = x.shape
        self._ensure(x.device, L, D)
        if self.pos is None:
            raise RuntimeError("this stack was built by create() without posembed_input; call "
                               "forward() with per-layer contexts")
        if mask is None:
            raise ValueError('"mask" must be set (merge_param of Encoder1DBlock, attention.py:55)')
        table = set_table_of(mask, L)
        if train and rng is None:
            raise ValueError("StackedEncoder1DBlock(train=True) needs the dropout rng (rng=)")
        ctxs = [LayerCtx(layer=i, sets=None, table=table, train=bool(train), rng=rng,
                         sample_offset=sample_offset) for i in range(self.num_blocks)]
        return _StackFn.apply(x.float().contiguous(), self, ctxs)

    def forward(self, x, ctxs: List[LayerCtx]):
        saved = []
        size = None
        for blk, ctx in zip(self.blocks, ctxs):
            with phase(f"fwd/block{ctx.layer}"):
                x, sv, size = blk.forward(x, ctx, size)
            saved.append(sv)
        return x, saved

    def backward(self, dx, saved, ctxs, lo: int = 0, hi: int | None = None):
        """Backward through blocks hi-1 .. lo (all by default); a staged backward (gradient
        all-reduce overlapped with the remaining blocks) calls it in several ranges."""
        hi = len(self.blocks) if hi is None else hi
        dz = None
        for i in range(hi - 1, lo - 1, -1):
            # block i's LayerNorm_0 backward also does block i-1's MLP-output dropout backward
            prev = (self.blocks[i - 1], saved[i - 1], ctxs[i - 1]) if i - 1 >= lo else None
            with phase(f"bwd/block{i}"):
                dx, dz = self.blocks[i].backward(dx, saved[i], ctxs[i], dz2=dz, prev=prev)
            wgrad_overlap.block_done()
        return dx
