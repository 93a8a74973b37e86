"""OCTO model and diffusion training step, mirroring the reference's
``multi_modal_transformers/models/octo/octo.py`` (Octo :55-198, generate_readouts :91-126,
compute_diffusion_denoise_loss :139-145, diffusion_train_step :204-240, OCTOTrainState :326-332,
create_octo_train_state :334-386).

MI355X design of the step (SURVEY §3.1 call stack):
  tokenizers  : frozen T5 (bf16 GEMM/attention kernels) -> Dense(768->D) [build addition for D!=768];
                image stem kernels; device-drawn patch positions
  sequence    : ONE fused kernel writes the token sequence (text | image + row/col emb | readout
                embedding) + the learned position embedding; the blockwise mask is a token-set
                table evaluated inside the attention kernel, never an (B, H, L, L) tensor
  backbone    : StackedEncoder1DBlock with ToMe, explicit fwd/bwd (attention_blocks/attention.py)
  head        : diffusion denoise loss (action_heads/diffusion.py)
  optimizer   : one fused AdamW launch over the flat parameter buffer; device step counter
Everything after the input upload is stream-ordered device work with no host sync, so the whole
step is captured into a HIP graph and replayed (see OCTOTrainState.graphed_step).
"""
from __future__ import annotations

import os

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from ... import _C, _kernels as K
from ...tracing import phase
from ...action_heads.categorical import CategoricalActionHead
from ...action_heads.continuous import ContinuousActionHead
from ...action_heads.diffusion import DiffusionActionHead
from ...attention_blocks.attention import LayerCtx, StackedEncoder1DBlock
from ...layers import Dense, wgrad_overlap
from ...params import ParamStore, he_normal, normal
from ...tokenizers.images.image_tokenizer import ImageTokenizer
from ...tokenizers.readout.readout import AddPositionEmbedding
from ...tokenizers.text.t5_base import T5Tokenizer
from ...tokenizers.token_sequencer import Image, Readout, Text, TokenSequence
from .config import OctoConfig, get_config

KIND_TEXT, KIND_IMAGE, KIND_READOUT = 0, 1, 2


class Octo:
    """Reference octo.py:55-198. ``Octo(config, device)`` declares, initialises (seeded, Flax
    initialisers) and uploads every parameter. ``config``: a preset / model_configs name, an
    OctoConfig, or a composed reference-schema dict (``config_loader.compose("octo_base")``,
    the DictConfig the reference's Octo(config) takes)."""

    def __init__(self, config: OctoConfig | str = "octo-small", device="cuda", seed: int = 0):
        if isinstance(config, dict):   # a composed reference-schema config (config_loader.compose)
            from ...config_loader import octo_config_from_yaml
            config = octo_config_from_yaml(config)
        self.cfg = cfg = get_config(config) if isinstance(config, str) else config
        self.device = torch.device(device)
        D = cfg.token_embedding_dim
        self.D = D
        self.seq = TokenSequence(cfg.input_sequence, cfg.token_compression_sequence)
        sets0 = self.seq.token_sequence
        self.L0 = sum(ts.num_tokens for ts in sets0)
        self.n_images = sum(isinstance(ts, Image) for ts in sets0)
        self.n_text = sum(ts.num_tokens for ts in sets0 if isinstance(ts, Text))
        self.n_readout = sum(ts.num_tokens for ts in sets0 if isinstance(ts, Readout))
        self.has_text = self.n_text > 0
        if self.has_text and cfg.text_tokens != self.n_text:
            raise ValueError("text_tokens must equal the text set sizes of input_sequence")
        store = self.store = ParamStore()
        # ---- tokenizers
        self.image_tokenizer = ImageTokenizer(cfg.image_size, cfg.patch_size, True,
                                              cfg.position_interval, "patch_encoding", D,
                                              resnet=cfg.stem).bind(store, "ImageTokenizer_0")
        NP = self.image_tokenizer.num_patches
        for ts in sets0:
            if isinstance(ts, Image) and ts.num_tokens != NP:
                raise ValueError(f"Image set of {ts.num_tokens} tokens != {NP} patches")
        self.text_proj = None
        if self.has_text and cfg.t5.d_model != D:
            self.text_proj = Dense(store, "TextProjection_0", cfg.t5.d_model, D)
        # readouts = AddPositionEmbedding(zeros) (octo.py:103-108); the add itself is fused into
        # the sequence assembly kernel, the module owns the parameter
        self.readout_encoder = AddPositionEmbedding().bind(store, "AddPositionEmbedding_0",
                                                           self.n_readout, D)
        self.readout_pe = self.readout_encoder.pe
        # ---- backbone (posembed_input of StackedEncoder1DBlock, attention.py:97-100)
        self.pos_embed = store.add("StackedEncoder1DBlock_0/posembed_input/pos_embedding",
                                   (self.L0, D), normal(0.02))
        self.stack = StackedEncoder1DBlock.create(store, "StackedEncoder1DBlock_0", cfg.num_blocks,
                                                  D, cfg.num_heads, cfg.mlp_dim, cfg.layer_norm_eps,
                                                  cfg.dropout_rate, cfg.attention_dropout_rate,
                                                  fp8=cfg.fp8, fp8_residual=cfg.fp8_residual)
        # ---- head
        self.head = DiffusionActionHead.create(store, "diffusion_action_head", D,
                                               cfg.action_space_dim, cfg.diffusion_steps,
                                               num_blocks=cfg.denoise_blocks)
        self.continuous_head = self.categorical_head = None
        if "continuous" in cfg.action_heads:
            self.continuous_head = ContinuousActionHead(store, "continuous_action_head", D,
                                                        cfg.action_space_dim, cfg.max_action)
        if "categorical" in cfg.action_heads:
            self.categorical_head = CategoricalActionHead(store, "categorical_action_head", D,
                                                          cfg.action_space_dim, cfg.num_bins,
                                                          cfg.max_action)
        store.materialize(self.device, seed)
        # MMT_DETERMINISTIC=1: bitwise-reproducible gradients (ParamStore.set_deterministic)
        if os.environ.get("MMT_DETERMINISTIC", "0") == "1" and torch.device(self.device).type == "cuda":
            store.set_deterministic(True)
        self.t5 = T5Tokenizer(cfg.t5).materialize(self.device, seed + 1) if self.has_text else None
        self._build_tables()

    # ------------------------------------------------------------------ static tables
    def _build_tables(self):
        cfg = self.cfg
        NP = self.image_tokenizer.num_patches
        row_src = []
        ti = ii = ri = 0
        for ts in self.seq.token_sequence:
            for j in range(ts.num_tokens):
                if isinstance(ts, Text):
                    row_src.append((KIND_TEXT << 24) | (ti + j))
                elif isinstance(ts, Image):
                    row_src.append((KIND_IMAGE << 24) | (ii * NP + j))
                else:
                    row_src.append((KIND_READOUT << 24) | (ri + j))
            if isinstance(ts, Text):
                ti += ts.num_tokens
            elif isinstance(ts, Image):
                ii += 1
            else:
                ri += ts.num_tokens
        self.row_src = torch.tensor(row_src, dtype=torch.int32, device=self.device)
        img_rows = np.zeros(ii * NP, np.int32)                 # image token -> sequence row
        for row, v in enumerate(row_src):
            if v >> 24 == KIND_IMAGE:
                img_rows[v & 0xFFFFFF] = row
        self.img_rows = torch.from_numpy(img_rows).to(self.device)
        # per-layer token-set tables (square masks) + ToMe set / r
        self.layer_sets = []
        if cfg.compression not in ("tome", "prune"):
            raise ValueError(f"compression must be 'tome' or 'prune', got {cfg.compression!r}")
        for layer in range(cfg.num_blocks):
            sets = self.seq.set_table(layer)
            merged = [i for i, ts in enumerate(self.seq._parse(layer) if cfg.token_compression_sequence
                                                else self.seq.token_sequence)
                      if ts.tokens_compressed_per_layer > 0]
            if cfg.compression == "prune":
                # top-k per token set, uncompressed sets keep all their tokens (k = n)
                prune = None
                if merged:
                    nxt = self.seq.set_table(layer + 1)
                    if min(nxt.lens) < 0:
                        raise ValueError(f"layer {layer}: pruning empties a token set")
                    prune = (tuple(zip(sets.starts, sets.lens)), tuple(nxt.lens))
                self.layer_sets.append((sets, K.SetTable(sets.starts, sets.lens, sets.vis, sets.causal),
                                        -1, 0, prune, ()))
                continue
            # ToMe per compressed token set (token_sequencer.py:222-238 gives every set its own
            # per-layer count): one bipartite match + merge per set, sizes carried per set
            parsed = self.seq._parse(layer)
            plan = []
            for si in merged:
                r = parsed[si].tokens_compressed_per_layer
                t = sets.lens[si]
                if r > t // 2:
                    raise ValueError(f"layer {layer}: ToMe r={r} exceeds t//2={t // 2} in set {si}")
                plan.append((si, r))
            tome_set = plan[0][0] if len(plan) == 1 else (-2 if plan else -1)
            self.layer_sets.append((sets, K.SetTable(sets.starts, sets.lens, sets.vis, sets.causal),
                                    tome_set, sum(r for _, r in plan), None, tuple(plan)))
        final = self.seq.set_table(cfg.num_blocks) if cfg.token_compression_sequence else self.seq.set_table(0)
        self.L_final = final.L
        rows = [s + j for s, n, m in zip(final.starts, final.lens, final.modalities) if m == "readouts"
                for j in range(n)]
        self.readout_rows = torch.tensor(rows, dtype=torch.int32, device=self.device)
        flag = np.full(self.L_final, -1, np.int32)
        flag[rows] = np.arange(len(rows))
        self.readout_flag = torch.from_numpy(flag).to(self.device)
        # categorical head: readout i belongs to action i // (n / A) ("batch (action timestep)
        # embeddings", categorical.py:32-36)
        A = cfg.action_space_dim
        self.readout_group = self.readout_group_counts = None
        if len(rows) % A == 0:
            per = len(rows) // A
            grp = np.full(self.L_final, -1, np.int32)
            grp[rows] = np.arange(len(rows)) // per
            self.readout_group = torch.from_numpy(grp).to(self.device)
            self.readout_group_counts = torch.full((A,), per, dtype=torch.int32, device=self.device)

    def layer_ctxs(self, train: bool, rng, sample_offset: int) -> List[LayerCtx]:
        return [LayerCtx(layer=i, sets=s, table=t, tome_set=ts, r=r, prune=pr, train=train, rng=rng,
                         sample_offset=sample_offset, tome_plan=plan)
                for i, (s, t, ts, r, pr, plan) in enumerate(self.layer_sets)]

    # ------------------------------------------------------------------ forward / backward
    def generate_readouts(self, text_tokens, images, train=True, rng=None, sample_offset=0,
                          positions=None, tome=None, t5_out=None):
        """Reference :91-126. Returns the final sequence (B, L_final, D) and the saved state.
        t5_out: the frozen T5 encoder's output for text_tokens, computed ahead (DDPStep's
        cross-step T5 pipeline); None runs the encoder here."""
        B = images.shape[0]
        D = self.D
        st: Dict = dict(B=B, train=train, rng=rng, sample_offset=sample_offset)
        txt, T = None, max(self.n_text, 1)
        if self.has_text:
            if t5_out is None:
                with phase("fwd/t5"):
                    t5_out = self.t5(text_tokens)                           # stop_gradient
            st["t5_out"] = t5_out
            if self.text_proj is not None:
                txt = self.text_proj.fwd(t5_out.view(B * self.n_text, -1)).view(B, self.n_text, D)
            else:
                txt = t5_out
        with phase("fwd/stem"):
            img_tok, (rt, ct), isv = self.image_tokenizer.forward(images, train, rng, sample_offset,
                                                                  positions)
        st.update(img_sv=isv, rt=rt, ct=ct, img_tok=img_tok, txt=txt)
        x0 = torch.empty((B, self.L0, D), dtype=torch.float32, device=images.device)  # fp32 residual
        NI = img_tok.shape[1]
        _C.call("mmt_seq_assemble_fwd", B, self.L0, D, _C.ptr(self.row_src), _C.ptr(txt), T,
                _C.ptr(img_tok), NI, _C.ptr(rt), _C.ptr(ct), _C.ptr(self.image_tokenizer.row_emb.data),
                _C.ptr(self.image_tokenizer.col_emb.data), _C.ptr(self.readout_pe.data),
                _C.ptr(self.pos_embed.data), _C.ptr(x0), _C.stream_ptr())
        ctxs = self.layer_ctxs(train, rng, sample_offset)
        if tome is not None:  # injected ToMe index triples (tests: the golden step fixtures)
            for c, idx in zip(ctxs, tome):
                c.tome_forced = idx
        with phase("fwd/blocks"):
            xL, ssv = self.stack.forward(x0, ctxs)
        st.update(ctxs=ctxs, stack_sv=ssv, NI=NI, T=T)
        return xL, st

    def compute_diffusion_denoise_loss(self, text_tokens, images, actions, train=True, rng=None,
                                       sample_offset=0, inject: Optional[dict] = None, t5_out=None):
        """Reference :139-145. Returns (loss (1,) fp32 device tensor, saved state). inject (tests):
        positions (rt, ct), t, eps, tome (per block an (unm, src, dst) triple of int32 device
        tensors or None) replace the step's own draws / matching. t5_out: the frozen encoder's
        output for text_tokens computed ahead (generate_readouts)."""
        inject = inject or {}
        xL, st = self.generate_readouts(text_tokens, images, train, rng, sample_offset,
                                        inject.get("positions"), inject.get("tome"), t5_out)
        B = xL.shape[0]
        cat = self.head.new_cat(B, xL.device)
        _C.call("mmt_rows_mean_fwd", _C.ptr(xL), xL.stride(0), xL.stride(1), B, self.D,
                _C.ptr(self.readout_rows), self.readout_rows.numel(),
                _C.ptr(self.head.readout_slot(cat)), cat.stride(0), _C.stream_ptr())
        with phase("fwd/head"):
            loss, hsv = self.head.loss_forward(cat, actions, rng, sample_offset, inject.get("t"),
                                               inject.get("eps"))
        st.update(head_sv=hsv, xL_shape=tuple(xL.shape), xL=xL)
        return loss, st

    def predict_diffusion_denoise_term(self, text_tokens, images, time, noisy_actions, rng=None,
                                       sample_offset=0, train=True):
        """Reference :130-137: readouts -> readout mean -> OctoDenoise (diffusion.py:88-107)."""
        xL, _ = self.generate_readouts(text_tokens, images, train, rng, sample_offset)
        return self.head.predict_denoise_term_mean(self._readout_mean(xL), time, noisy_actions)

    def predict_diffusion_action(self, text_tokens, images, rng, sample_offset=0, train=True,
                                 z: Optional[torch.Tensor] = None, return_noise=False,
                                 positions=None):
        """Reference :147-154: readouts (the reference's backbone always runs with
        train=True, :120, and its image encoder samples positions by default) -> readout mean ->
        the 32-step DDPM sampler (action_heads/diffusion.py:146-209). Returns (B, 8) fp32."""
        xL, _ = self.generate_readouts(text_tokens, images, train, rng, sample_offset, positions)
        B = xL.shape[0]
        e = torch.empty((B, self.D), dtype=torch.bfloat16, device=xL.device)
        _C.call("mmt_rows_mean_fwd", _C.ptr(xL), xL.stride(0), xL.stride(1), B, self.D,
                _C.ptr(self.readout_rows), self.readout_rows.numel(), _C.ptr(e), e.stride(0),
                _C.stream_ptr())
        return self.head.predict_action_mean(e, rng, sample_offset, z, return_noise)

    # ------------------------------------------------------------------ other action heads
    def _readout_mean(self, xL):
        B = xL.shape[0]
        e = torch.empty((B, self.D), dtype=torch.bfloat16, device=xL.device)
        _C.call("mmt_rows_mean_fwd", _C.ptr(xL), xL.stride(0), xL.stride(1), B, self.D,
                _C.ptr(self.readout_rows), self.readout_rows.numel(), _C.ptr(e), e.stride(0),
                _C.stream_ptr())
        return e

    def _readout_group_means(self, xL):
        if self.readout_group is None:
            raise ValueError("the readout count must be a multiple of action_space_dim "
                             "(categorical.py:32-36)")
        B, A = xL.shape[0], self.cfg.action_space_dim
        g = torch.empty((B, A, self.D), dtype=torch.bfloat16, device=xL.device)
        _C.call("mmt_rows_group_mean_fwd", _C.ptr(xL), xL.stride(0), xL.stride(1), B, self.L_final,
                self.D, _C.ptr(self.readout_group), A, _C.ptr(self.readout_group_counts), _C.ptr(g),
                _C.stream_ptr())
        return g

    def _need(self, head, name):
        if head is None:
            raise ValueError(f"{name} head not built: add it to OctoConfig.action_heads")
        return head

    def predict_continuous_action(self, text_tokens, images, rng=None, sample_offset=0, train=True):
        """Reference :158-165 -> (B, 1, A) fp32."""
        h = self._need(self.continuous_head, "continuous")
        xL, _ = self.generate_readouts(text_tokens, images, train, rng, sample_offset)
        return h.forward(self._readout_mean(xL))

    def compute_l2_loss(self, text_tokens, images, actions, train=True, rng=None, sample_offset=0):
        """Reference :167-174, batch-averaged as continuous_train_step (:262). (loss, saved)."""
        h = self._need(self.continuous_head, "continuous")
        xL, st = self.generate_readouts(text_tokens, images, train, rng, sample_offset)
        loss, hsv = h.loss_forward(self._readout_mean(xL), actions)
        st.update(head_kind="continuous", head_sv=hsv, xL_shape=tuple(xL.shape))
        return loss, st

    def predict_action_logits(self, text_tokens, images, rng=None, sample_offset=0, train=True):
        """Reference :178-185 -> (B, A, num_bins) fp32."""
        h = self._need(self.categorical_head, "categorical")
        xL, _ = self.generate_readouts(text_tokens, images, train, rng, sample_offset)
        return h.forward(self._readout_group_means(xL))

    def compute_ce_loss(self, text_tokens, images, actions, train=True, rng=None, sample_offset=0):
        """Reference :187-198, averaged as categorical_train_step (:302). (loss, saved)."""
        h = self._need(self.categorical_head, "categorical")
        xL, st = self.generate_readouts(text_tokens, images, train, rng, sample_offset)
        loss, hsv = h.loss_forward(self._readout_group_means(xL), actions)
        st.update(head_kind="categorical", head_sv=hsv, xL_shape=tuple(xL.shape))
        return loss, st

    # ------------------------------------------------------------------ staged backward
    def _block_offset(self, j: int) -> int:
        """Flat index of block j's first parameter (store.n for j = num_blocks)."""
        if j >= self.cfg.num_blocks:
            return self.store.n
        return self.store.by_name[f"StackedEncoder1DBlock_0/Block_{j}/LayerNorm_0/scale"].offset

    def stage_bounds(self, stages) -> List[int]:
        """Block boundaries nb = b[0] > b[1] > ... > b[S] = 0 of a backward split into S stages
        (stage i runs blocks [b[i+1], b[i]); stage 0 also the heads, the last stage the tokens).
        `stages`: an int S (blocks split evenly), an explicit list, or "auto[:MB]": gradient
        regions of ~MB megabytes (default 24) from the top, and a last stage of block 0 alone, so
        the region all-reduced after the backward ends (block 0 and everything declared before
        it: the tokenizers, the stem) is the smallest possible."""
        nb = self.cfg.num_blocks
        if isinstance(stages, (list, tuple)):
            return self._check_bounds(list(stages))
        if isinstance(stages, str):
            mb = float(stages.split(":", 1)[1]) if ":" in stages else 24.0
            target = mb * (1 << 20)
            bounds, acc = [nb], 0.0
            for j in range(nb - 1, 0, -1):
                acc += 4.0 * (self._block_offset(j + 1) - self._block_offset(j))
                if acc >= target:
                    bounds.append(j)
                    acc = 0.0
            if nb > 1 and bounds[-1] != 1:
                bounds.append(1)
            bounds.append(0)
            return self._check_bounds(bounds)
        n = max(1, min(int(stages), nb))
        return self._check_bounds([nb * (n - i) // n for i in range(n + 1)])  # nb .. 0

    def _check_bounds(self, b: List[int]) -> List[int]:
        """A stage plan must cover blocks nb .. 0 once: b[0] == nb, b[-1] == 0, strictly
        decreasing — otherwise gradient regions would be missing or overlap, parts of the
        gradient never (or twice) all-reduced, and the ranks would drift apart silently."""
        nb = self.cfg.num_blocks
        if (len(b) < 2 or b[0] != nb or b[-1] != 0 or any(int(x) != x for x in b)
                or any(b[i] <= b[i + 1] for i in range(len(b) - 1))):
            raise ValueError(f"stage bounds {b}: need {nb} = b[0] > b[1] > ... > b[-1] = 0")
        return [int(x) for x in b]

    def _stage_bounds(self, n_stages) -> List[int]:
        return self.stage_bounds(n_stages)

    def grad_regions(self, stages) -> List[tuple]:
        """Flat-gradient index ranges that are final after each backward stage (stage 0: the
        heads and the last blocks, declared last in the store; the last stage: the first blocks
        and everything declared before them). `stages` as in stage_bounds."""
        b = self.stage_bounds(stages)
        n_stages = len(b) - 1
        off = [self._block_offset(j) for j in b]
        regions = []
        for i in range(n_stages):
            hi = self.store.n if i == 0 else off[i]
            lo = 0 if i == n_stages - 1 else off[i + 1]
            regions.append((lo, hi))
        return regions

    def backward_stage(self, st: Dict, stage: int, stages):
        """Stage `stage` of a backward split as stage_bounds(stages) (the heads run in stage 0,
        the stem / embeddings in the last): backward(st) == all stages in order."""
        b = self.stage_bounds(stages)
        n_stages = len(b) - 1
        with wgrad_overlap(self.device):  # dW products beside the critical path; joined here
            if stage == 0:
                with phase("bwd/head"):
                    st["_dx"] = self._backward_head(st)
            with phase(f"bwd/blocks[{b[stage + 1]},{b[stage]})"):
                dx = self.stack.backward(st["_dx"], st["stack_sv"], st["ctxs"], lo=b[stage + 1],
                                         hi=b[stage])
            if stage == n_stages - 1:
                with phase("bwd/tokens+stem"):
                    self._backward_tokens(st, dx)
                st.pop("_dx", None)
            else:
                st["_dx"] = dx
        if self.store.det_fx is not None:  # deterministic mode: this stage's final region
            self.store.det_flush(*self.grad_regions(stages)[stage])

    def backward(self, st: Dict):
        """Reverse schedule of compute_diffusion_denoise_loss / compute_l2_loss / compute_ce_loss;
        writes every parameter gradient into the flat gradient buffer (which must be zeroed
        before the forward)."""
        self.backward_stage(st, 0, 1)

    def _backward_head(self, st: Dict):
        B = st["B"]
        D = self.D
        kind = st.get("head_kind", "diffusion")
        if kind == "categorical":
            dg = self.categorical_head.loss_backward(st["head_sv"])
            dxL = torch.empty(st["xL_shape"], dtype=torch.float32, device=dg.device)
            _C.call("mmt_rows_group_mean_bwd", _C.ptr(dg), B, self.L_final, D,
                    _C.ptr(self.readout_group), self.cfg.action_space_dim,
                    _C.ptr(self.readout_group_counts), _C.ptr(dxL), _C.stream_ptr())
        else:
            head = self.continuous_head if kind == "continuous" else self.head
            de = head.loss_backward(st["head_sv"])
            dxL = torch.empty(st["xL_shape"], dtype=torch.float32, device=de.device)
            _C.call("mmt_rows_mean_bwd", _C.ptr(de), de.stride(0), B, self.L_final, D,
                    _C.ptr(self.readout_flag), self.readout_rows.numel(), _C.ptr(dxL),
                    _C.stream_ptr())
        return dxL

    def _backward_tokens(self, st: Dict, dx0):
        B = st["B"]
        D = self.D
        NI, T = st["NI"], st["T"]
        dimg = torch.empty((B, NI, D), dtype=torch.bfloat16, device=dx0.device)
        dtxt = torch.empty((B, T, D), dtype=torch.bfloat16, device=dx0.device) if self.text_proj else None
        it = self.image_tokenizer
        # token gradients (and the readout embedding's); the image row / column position
        # embedding gradients by token window (mmt_patch_embed_grad)
        _C.call("mmt_seq_assemble_bwd", B, self.L0, D, _C.ptr(self.row_src), _C.ptr(dx0),
                _C.ptr(dtxt), T, _C.ptr(dimg), NI, _C.ptr(st["rt"]), _C.ptr(st["ct"]),
                _C.ptr(self.img_rows), it.Q, None, None, _C.ptr(self.readout_pe.grad),
                _C.stream_ptr())
        if NI:
            _C.call("mmt_patch_embed_grad", B, self.L0, D, self.n_images, self.cfg.image_size[0],
                    self.cfg.patch_size, it.Q, _C.ptr(self.img_rows), _C.ptr(dx0),
                    _C.ptr(st["rt"]), _C.ptr(st["ct"]), _C.ptr(it.row_emb.grad),
                    _C.ptr(it.col_emb.grad), _C.stream_ptr())
        K.colsum(dx0.view(B, self.L0 * D), self.pos_embed.grad.view(-1))
        it.backward(dimg, st["img_sv"])
        if self.text_proj is not None:
            self.text_proj.bwd(dtxt.view(B * T, D), st["t5_out"].view(B * T, -1), need_dx=False)

    def num_params(self) -> int:
        return self.store.num_params()


# ---------------------------------------------------------------------- train state / step
@dataclass
class AdamW:
    """The reference takes an optax tx from its caller (octo.py:341); this is optax.adamw with
    these defaults (decoupled weight decay applied to every parameter, as optax without a mask)."""
    learning_rate: float = 3e-4
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8
    weight_decay: float = 1e-4


class OCTOMetrics:
    """Reference octo.py:322-324 (``clu.metrics.Average.from_output("loss")``): running sum and
    count kept on the device, merged without a host sync (the reference's wandb.log forces one
    every step, :231-233). ``compute()`` is the average (a host read)."""

    def __init__(self, device):
        self.total = torch.zeros(1, dtype=torch.float64, device=device)
        self.count = torch.zeros(1, dtype=torch.float64, device=device)

    def merge(self, loss: torch.Tensor) -> "OCTOMetrics":
        """single_from_model_output(loss=loss) merged in place (Average.merge: sums add)."""
        self.total.add_(loss.detach().reshape(-1)[:1].double())
        self.count.add_(1.0)
        return self

    def compute(self) -> float:
        c = float(self.count.item())
        return float(self.total.item()) / c if c else float("nan")

    def reset(self):
        self.total.zero_()
        self.count.zero_()


@dataclass
class OCTOTrainState:
    """Reference octo.py:326-332: params (flat store), optimizer, rngs (device {seed, step}),
    step, metrics (running loss average, clu.metrics.Average equivalent)."""
    model: Octo
    tx: AdamW
    rng: torch.Tensor
    allreduce: Optional[Callable] = None        # DDP gradient all-reduce (distributed.py)
    sample_offset: int = 0
    metrics: Optional[OCTOMetrics] = None
    last_loss: Optional[torch.Tensor] = None    # loss of the latest step (device)

    @property
    def params(self):
        return self.model.store.state_dict()

    @property
    def step(self) -> int:
        return int(self.rng[1].item())

    def apply_gradients(self):
        with phase("optimizer"):
            self._apply_gradients()

    def _apply_gradients(self):
        s = self.model.store
        tx = self.tx
        _C.call("mmt_adamw", _C.ptr(s.flat), _C.ptr(s.flat_grad), _C.ptr(s.m), _C.ptr(s.v),
                _C.ptr(s.flat_bf16), s.flat.numel(), _C.ptr(self.rng), tx.learning_rate, tx.b1,
                tx.b2, tx.eps, tx.weight_decay, getattr(self.allreduce, "grad_scale", 1.0),
                _C.stream_ptr())
        s.refresh_transposed()
        s.refresh_fp8()
        _C.call("mmt_step_advance", _C.ptr(self.rng), _C.stream_ptr())


def create_octo_train_state(model: Octo, tx: AdamW | None = None, seed: int = 1234,
                            allreduce=None, sample_offset: int = 0) -> OCTOTrainState:
    """Reference octo.py:334-386 (parameters were initialised by Octo(...))."""
    rng = torch.tensor([seed, 0], dtype=torch.int32, device=model.device)
    return OCTOTrainState(model, tx or AdamW(), rng, allreduce, sample_offset,
                          metrics=OCTOMetrics(model.device))


def grads_tree(model: Octo) -> Dict[str, torch.Tensor]:
    """The step's gradients by parameter name (views into the flat fp32 gradient buffer, valid
    until the next step zeroes it) — the ``grads`` the reference's train steps return."""
    return {p.name: p.grad for p in model.store.params}


def _train_step(loss_fn, model: Octo, train_state: OCTOTrainState, text_tokens, images, actions,
                **kw):
    """value_and_grad -> apply_gradients -> metrics merge (octo.py:216-239); returns
    (train_state, grads). The step's loss stays on the device: train_state.last_loss."""
    model.store.zero_grad()
    loss, st = loss_fn(text_tokens, images, actions, True, train_state.rng,
                       train_state.sample_offset, **kw)
    model.backward(st)
    if train_state.allreduce is not None:
        train_state.allreduce(model.store.flat_grad)
    train_state.apply_gradients()
    train_state.last_loss = loss
    if train_state.metrics is not None:
        train_state.metrics.merge(loss)
    return train_state, grads_tree(model)


def continuous_train_step(model: Octo, train_state: OCTOTrainState, text_tokens, images, actions):
    """Reference octo.py:242-280: value_and_grad of mean(compute_l2_loss), apply_gradients,
    metrics merge. Returns (train_state, grads)."""
    return _train_step(model.compute_l2_loss, model, train_state, text_tokens, images, actions)


def categorical_train_step(model: Octo, train_state: OCTOTrainState, text_tokens, images, actions):
    """Reference octo.py:282-320: value_and_grad of mean(compute_ce_loss), apply_gradients,
    metrics merge. Returns (train_state, grads)."""
    return _train_step(model.compute_ce_loss, model, train_state, text_tokens, images, actions)


def diffusion_train_step(model: Octo, train_state: OCTOTrainState, text_tokens, images, actions,
                         inject: Optional[dict] = None):
    """Reference octo.py:204-240: value_and_grad of the denoise loss, apply_gradients, metrics
    merge. Returns (train_state, grads) like the reference; grads are views of the flat gradient
    buffer by parameter name, the loss is train_state.last_loss (device) and the running average
    train_state.metrics."""
    return _train_step(model.compute_diffusion_denoise_loss, model, train_state, text_tokens,
                       images, actions, inject=inject)
