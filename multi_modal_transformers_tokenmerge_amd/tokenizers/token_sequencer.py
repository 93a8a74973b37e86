"""Token sequence grammar and blockwise attention rules, mirroring the reference's
``multi_modal_transformers/tokenizers/token_sequencer.py`` (TokenSet :20-52, Text :55-91,
TaskDescriptionPrefix :94-113, Image :116-148, Readout :151-183, TokenSequence :186-340).

The reference materialises the (H, L, L) boolean mask with Python loops on every apply
(:313-321). Here that dense form exists for API parity and tests only; the hot path consumes the
*token-set table* (:meth:`TokenSequence.set_table`): per set its start/length and the bitmask of
key sets it attends to, which the gfx950 attention kernel evaluates per tile (and skips invisible
tiles). Per-layer ToMe/compression counts follow ``_parse(layer)`` (:222-238); the build's mask is
square per layer (rows AND columns compressed), where the reference pairs compressed rows with
uncompressed columns (:317-318), which cannot be applied to a shrunken sequence.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List

import numpy as np


class TokenSet:
    """A set of tokens and its attention rule (reference :20-52)."""

    modality = None

    def __init__(self, num_tokens: int, timestep: int, tokens_compressed_per_layer: int = 0):
        self.num_tokens = num_tokens
        self.timestep = timestep
        self.tokens_compressed_per_layer = tokens_compressed_per_layer
        self.modality_sequence_idx = None

    # --- set-level rules: return "ones", "zeros" or "causal"
    def intra_kind(self) -> str:
        raise NotImplementedError

    def inter_kind(self, other: "TokenSet") -> str:
        raise NotImplementedError

    def rule_kind(self, other: "TokenSet") -> str:
        if other.timestep == self.timestep and isinstance(other, self.__class__):
            return self.intra_kind()
        return self.inter_kind(other)

    # --- dense forms (reference API)
    def intra_attention_rule(self) -> np.ndarray:
        return _block(self.intra_kind(), self.num_tokens, self.num_tokens)

    def inter_attention_rule(self, tokenset: "TokenSet") -> np.ndarray:
        return _block(self.inter_kind(tokenset), self.num_tokens, tokenset.num_tokens)

    def attention_rule(self, token_sequence: List["TokenSet"]) -> np.ndarray:
        return np.hstack([_block(self.rule_kind(ts), self.num_tokens, ts.num_tokens)
                          for ts in token_sequence])


def _block(kind: str, n: int, m: int) -> np.ndarray:
    if kind == "ones":
        return np.ones((n, m), np.float32)
    if kind == "zeros":
        return np.zeros((n, m), np.float32)
    if kind == "causal":  # nn.make_causal_mask: key index <= query index
        return np.tril(np.ones((n, m), np.float32))
    raise ValueError(kind)


class Text(TokenSet):
    """Reference :55-91: causal within the set, all past non-readout sets."""
    modality = "text"

    def inter_kind(self, other):
        if isinstance(other, Readout):
            return "zeros"
        return "ones" if other.timestep <= self.timestep else "zeros"

    def intra_kind(self):
        return "causal"


class TaskDescriptionPrefix(Text):
    """Reference :94-113: attends only to itself."""

    def inter_kind(self, other):
        return "zeros"

    def intra_kind(self):
        return "ones"


class Image(TokenSet):
    """Reference :116-148: same-timestep images + every non-readout set with t' <= t."""
    modality = "images"

    def inter_kind(self, other):
        if isinstance(other, Readout):
            return "zeros"
        return "ones" if other.timestep <= self.timestep else "zeros"

    def intra_kind(self):
        return "ones"


class Readout(TokenSet):
    """Reference :151-183: own set + every non-readout set with t' <= t."""
    modality = "readouts"

    def inter_kind(self, other):
        if isinstance(other, self.__class__):
            return "zeros"
        return "ones" if other.timestep <= self.timestep else "zeros"

    def intra_kind(self):
        return "ones"


_CLASSES = {"Text": Text, "TaskDescriptionPrefix": TaskDescriptionPrefix, "Image": Image,
            "Readout": Readout}


@dataclass
class TokenEmbeddings:
    """Reference :342-346 (flax.struct.dataclass)."""
    text: object = None
    images: object = None
    readouts: object = None


@dataclass
class LayerSets:
    """Token-set table of one layer as the attention kernel consumes it."""
    starts: List[int]
    lens: List[int]
    vis: List[int]
    causal: List[bool] = field(default_factory=list)
    modalities: List[str] = field(default_factory=list)

    @property
    def L(self) -> int:
        return int(sum(self.lens))


class TokenSequence:
    """Reference :186-340."""

    def __init__(self, token_sequence: str, token_compression_sequence: str | None = None):
        self.token_sequence_str = token_sequence
        self.token_compression_sequence_str = token_compression_sequence
        self.token_sequence = self._parse()
        self.slice_idx = self._generate_embedding_slices()
        self.tokenset_slices = self._generate_embedding_subsets()

    # ------------------------------------------------------------------ grammar (:199-253)
    def _blocks(self):
        blocks = re.findall(r"\[(.*?)\]", self.token_sequence_str)
        repeats = []
        for rep in re.findall(r"(?<=\])(.*?)(?=\[|$)", self.token_sequence_str):
            rep = rep.strip()
            repeats.append(1 if rep == "" else int(re.findall(r"\*(\d+)", rep)[0]))
        return blocks, repeats

    def _parse(self, layer: int | None = 0) -> List[TokenSet]:
        blocks, repeats = self._blocks()
        comp_blocks = (re.findall(r"\[(.*?)\]", self.token_compression_sequence_str)
                       if self.token_compression_sequence_str is not None else None)
        seq: List[TokenSet] = []
        t = 0
        for bi, (block, repeat) in enumerate(zip(blocks, repeats)):
            groups = re.split(r";", block)
            cgroups = re.split(r";", comp_blocks[bi]) if comp_blocks is not None else [None] * len(groups)
            for _ in range(repeat):
                for grp, cgrp in zip(groups, cgroups):
                    name = re.search(r"^\s*(.*?)\{", grp).group(1).strip()
                    n = int(re.search(r"\d+", grp).group())
                    per_layer = 0
                    if cgrp is not None:
                        per_layer = int(re.search(r"\d+", cgrp).group())
                        if layer is None:
                            raise TypeError("layer must be given with a compression sequence")
                        n = n - layer * per_layer
                    if name not in _CLASSES:
                        raise ValueError(f"unknown token set {name!r}")
                    ts = _CLASSES[name](n, t)
                    ts.tokens_compressed_per_layer = per_layer
                    seq.append(ts)
                t += 1
        return seq

    # ------------------------------------------------------------------ slices (:272-304)
    def _generate_embedding_slices(self):
        idx = {"images": 0, "text": 0, "readouts": 0}
        out = []
        for ts in self.token_sequence:
            out.append((idx[ts.modality], ts.num_tokens))
            idx[ts.modality] += ts.num_tokens
        return out

    def _generate_embedding_subsets(self):
        out, cur = [], 0
        for ts in self.token_sequence:
            out.append((cur, ts.num_tokens))
            cur += ts.num_tokens
        return out

    def assemble_embeddings(self, embeddings: TokenEmbeddings, slice_idx=None):
        """Reference :255-269 (concatenate modality slices in sequence order). Host/torch API
        helper; the training path writes each tokenizer's rows in place instead."""
        import torch
        slice_idx = slice_idx or self.slice_idx
        parts = [getattr(embeddings, ts.modality)[:, s:s + n]
                 for (s, n), ts in zip(slice_idx, self.token_sequence)]
        return torch.cat(parts, dim=1)

    # ------------------------------------------------------------------ masks (:306-334)
    def generate_layer_token_sequence(self, layer: int) -> List[TokenSet]:
        return self._parse(layer=layer)

    def generate_attention_mask(self, repeats: int = 1, layer: int | None = None,
                                square: bool = False) -> np.ndarray:
        """Dense (repeats, Lq, Lk) bool mask. square=False is the reference's form (rows from the
        layer's parse, columns from the layer-0 sequence); square=True is what the build uses."""
        rows = self._parse(layer=layer if self.token_compression_sequence_str is not None else 0)
        cols = rows if square else self.token_sequence
        m = np.vstack([ts.attention_rule(cols) for ts in rows]).astype(bool)
        return np.repeat(m[None], repeats, axis=0)

    def get_modality_idx(self, modality: str, layer: int = 0) -> np.ndarray:
        seq = self._parse(layer=layer) if self.token_compression_sequence_str else self.token_sequence
        cur, idx = 0, []
        for ts in seq:
            if ts.modality == modality:
                idx.append(np.arange(cur, cur + ts.num_tokens))
            cur += ts.num_tokens
        return np.concatenate(idx) if idx else np.zeros((0,), np.int64)

    def set_table(self, layer: int = 0) -> LayerSets:
        """Token-set table of ``layer`` (square mask): the form the attention kernel consumes."""
        seq = self._parse(layer=layer) if self.token_compression_sequence_str else self.token_sequence
        starts, lens, vis, causal, mods = [], [], [], [], []
        cur = 0
        for ts in seq:
            starts.append(cur)
            lens.append(ts.num_tokens)
            cur += ts.num_tokens
        for i, q in enumerate(seq):
            bits = 0
            for j, k in enumerate(seq):
                kind = q.rule_kind(k)
                if kind == "causal" and i != j:
                    raise NotImplementedError("causal rule between distinct sets")
                if kind != "zeros":
                    bits |= 1 << j
            vis.append(bits)
            causal.append(q.rule_kind(q) == "causal")
            mods.append(q.modality)
        return LayerSets(starts, lens, vis, causal, mods)

    def num_layers_until_empty(self) -> int:
        return min((ts.num_tokens // ts.tokens_compressed_per_layer
                    for ts in self.token_sequence if ts.tokens_compressed_per_layer), default=10 ** 9)


def sets_from_mask(mask) -> LayerSets:
    """A dense attention mask in the reference's form — ``generate_attention_mask`` repeated over
    the batch (octo.py:66-68, 119): (B, H, L, L), (H, L, L), (B, L, L) or (L, L), bool or 0/1 — as
    the token-set table the attention kernels evaluate (contiguous sets, per query set the key
    sets it sees, causal sets). The mask must be the same for every batch entry and head (Flax
    broadcasts one pattern; the kernels take one table) and must BE a block mask of at most 16
    contiguous sets whose diagonal blocks are all-ones, all-zeros or lower-triangular (causal);
    anything else raises ValueError. Segmentation is greedy over positions in O(L^2): token j
    joins the open set when its row and column agree with the set's outside the set and the
    diagonal block keeps the set's kind; the table is then checked by rebuilding the mask."""
    if hasattr(mask, "detach"):
        mask = mask.detach().cpu().numpy()
    m = np.asarray(mask)
    if m.dtype != bool:
        m = m != 0
    while m.ndim > 2:
        if not (m == m[:1]).all():
            raise ValueError("the attention mask differs across batch / heads: the kernels take one "
                             "token-set pattern per layer")
        m = m[0]
    if m.ndim != 2 or m.shape[0] != m.shape[1]:
        raise ValueError(f"attention mask must be square (.., L, L), got {m.shape}")
    L = m.shape[0]
    starts, lens, kinds = [], [], []
    i = 0
    while i < L:
        j = i + 1
        kind = None  # "full" | "zeros" | "causal" once the set holds two tokens
        while j < L:
            if kind is None:
                blk = (m[i, i], m[i, j], m[j, i], m[j, j])
                k = {(True, True, True, True): "full", (False, False, False, False): "zeros",
                     (True, False, True, True): "causal"}.get(tuple(bool(v) for v in blk))
                if k is None:
                    break
            else:
                k = kind
                row_in, col_in = m[j, i:j + 1], m[i:j, j]
                if k == "full" and not (row_in.all() and col_in.all()):
                    break
                if k == "zeros" and (row_in.any() or col_in.any()):
                    break
                if k == "causal" and not (row_in.all() and not col_in.any()):
                    break
            # outside the set [i, j]: row j / column j must match row i / column i
            if not (np.array_equal(m[j, :i], m[i, :i]) and np.array_equal(m[j, j + 1:], m[i, j + 1:])
                    and np.array_equal(m[:i, j], m[:i, i]) and np.array_equal(m[j + 1:, j], m[j + 1:, i])):
                break
            kind = k
            j += 1
        starts.append(i)
        lens.append(j - i)
        kinds.append(kind or ("full" if m[i, i] else "zeros"))
        i = j
    n = len(starts)
    if n > 16:
        raise ValueError(f"the attention mask needs {n} token sets (the kernels take at most 16)")
    vis, causal = [], []
    for a in range(n):
        bits = 0
        for b in range(n):
            if a == b:
                on = kinds[a] != "zeros"
            else:
                on = bool(m[starts[a], starts[b]])
            bits |= int(on) << b
        vis.append(bits)
        causal.append(kinds[a] == "causal")
    if any(v == 0 for v in vis):
        # a query row that sees no key: Flax fills its logits with finfo.min and returns the
        # uniform average of V there; the kernels give a zero row (lse = -inf). Not a pattern
        # the reference's TokenSequence produces (every set sees itself).
        raise ValueError("the attention mask has fully masked query rows (a token set that sees "
                         "no key): not supported")
    sets = LayerSets(starts, lens, vis, causal, ["?"] * n)
    if not np.array_equal(dense_mask_of(sets), m):
        raise ValueError("the attention mask is not a block mask of contiguous token sets")
    return sets


def dense_mask_of(sets: LayerSets) -> np.ndarray:
    """The (L, L) bool mask a token-set table stands for (inverse of sets_from_mask)."""
    L = sets.L
    sid = np.zeros(L, np.int64)
    for k, (s, n) in enumerate(zip(sets.starts, sets.lens)):
        sid[s:s + n] = k
    vis = np.array(sets.vis, np.int64)
    m = ((vis[sid][:, None] >> sid[None, :]) & 1).astype(bool)
    for k, c in enumerate(sets.causal or []):
        if c:
            s, n = sets.starts[k], sets.lens[k]
            m[s:s + n, s:s + n] &= np.tril(np.ones((n, n), bool))
    return m
