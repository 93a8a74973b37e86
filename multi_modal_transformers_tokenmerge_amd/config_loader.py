"""YAML configuration surface of the reference (Hydra `compose` + `instantiate(_target_)`,
``models/octo/octo.py:75-84``, ``model_configs/octo_base.yaml:12-18``) without Hydra/OmegaConf,
which are not available on the GPU box.

* :func:`compose` reads a root YAML (e.g. ``octo_base``) from a config directory, merges its
  ``defaults:`` list (``- tokenizers/text: t5_base`` loads ``tokenizers/text/t5_base.yaml`` under
  the key path ``tokenizers.text``), applies dotted ``key=value`` overrides and resolves OmegaConf
  ``${a.b.c}`` interpolations (absolute paths from the root, as the reference's YAMLs use them,
  e.g. ``gato_resnet.yaml:17-18``).
* :func:`instantiate` turns a node with a ``_target_`` into the object the build uses for that
  dotted path (:data:`TARGETS`), honouring ``_partial_``. Flax layer targets become
  :class:`LayerSpec` records (the build's kernels implement them; see octo_config_from_yaml).
* :func:`octo_config_from_yaml` maps the reference schema onto :class:`OctoConfig`. Both key
  layouts are accepted: the one the shipped YAMLs define (``attention_blocks.num_blocks``,
  ``attention_blocks.encoder_1d_block``, ``vanilla_decoder.yaml:1-4``) and the one ``octo.py``
  reads (``attention_blocks.stacked_encoder_1d_block.{num_blocks, encoder_1d_block}``,
  ``octo.py:67,80``). New keys: ``token_compression_sequence`` (ToMe),
  ``token_compression_method`` ("tome" | "prune"), ``fp8_matmul``, ``t5_num_layers`` and
  ``text_tokens``.

Errors follow the reference's conventions: a missing key or an unknown ``_target_`` raises
``KeyError`` / ``ValueError`` (Hydra raises on both).
"""
from __future__ import annotations

import copy
import functools
import importlib
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Optional

import yaml

CONFIG_DIR = Path(__file__).resolve().parent / "model_configs"
_INTERP = re.compile(r"\$\{([^}]+)\}")


# ---------------------------------------------------------------------------- compose
def _load(path: Path) -> dict:
    with open(path) as fh:
        d = yaml.safe_load(fh)
    return d or {}


def _set_path(root: dict, dotted: str, value):
    keys = dotted.split(".")
    node = root
    for k in keys[:-1]:
        node = node.setdefault(k, {})
    node[keys[-1]] = value


def _get_path(root: dict, dotted: str):
    node = root
    for k in dotted.split("."):
        if isinstance(node, list):
            node = node[int(k)]
        elif isinstance(node, dict) and k in node:
            node = node[k]
        else:
            raise KeyError(f"interpolation key {dotted!r} not found")
    return node


def _merge(dst: dict, src: dict) -> dict:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _resolve(node, root, depth=0):
    if depth > 32:
        raise ValueError("interpolation cycle")
    if isinstance(node, dict):
        return {k: _resolve(v, root, depth) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root, depth) for v in node]
    if isinstance(node, str):
        m = _INTERP.fullmatch(node.strip())
        if m:  # whole-string interpolation keeps the referenced value's type
            return _resolve(_get_path(root, m.group(1).strip()), root, depth + 1)
        if _INTERP.search(node):
            return _INTERP.sub(lambda mm: str(_resolve(_get_path(root, mm.group(1).strip()), root,
                                                       depth + 1)), node)
    return node


def _parse_scalar(v: str):
    try:
        return yaml.safe_load(v)
    except yaml.YAMLError:
        return v


def compose(config_name: str = "octo_base", config_dir: str | Path | None = None,
            overrides: Optional[List[str]] = None) -> dict:
    """hydra.compose(config_name, overrides) restated: root YAML + its defaults list + overrides,
    interpolations resolved. Returns a plain nested dict."""
    cdir = Path(config_dir) if config_dir else CONFIG_DIR
    root_path = cdir / (config_name if config_name.endswith(".yaml") else config_name + ".yaml")
    if not root_path.exists():
        raise KeyError(f"config {config_name!r} not found in {cdir}")
    root = _load(root_path)
    defaults = root.pop("defaults", []) or []
    cfg: dict = {}
    for item in defaults:
        if isinstance(item, str):        # "- name": another root-level file
            if item == "_self_":
                continue
            _merge(cfg, _load(cdir / f"{item}.yaml"))
            continue
        (group, option), = item.items()
        sub = _load(cdir / group / f"{option}.yaml")
        node: dict = {}
        _set_path(node, group.replace("/", "."), sub)
        _merge(cfg, node)
    _merge(cfg, root)                   # the root's own keys win over its defaults (_self_ last)
    for ov in overrides or []:
        if "=" not in ov:
            raise ValueError(f"override {ov!r} is not key=value")
        k, v = ov.split("=", 1)
        _set_path(cfg, k.strip().lstrip("+"), _parse_scalar(v.strip()))
    return _resolve(cfg, cfg)


# ------------------------------------------------------------------------- instantiate
@dataclass
class LayerSpec:
    """A Flax layer (or initializer / function) named by a ``_target_`` the build implements in
    its kernels: the dotted path plus its keyword arguments."""
    target: str
    kwargs: Dict[str, Any] = field(default_factory=dict)
    partial: bool = False

    def get(self, k, default=None):
        return self.kwargs.get(k, default)


_REF = "multi_modal_transformers."
_BUILD = "multi_modal_transformers_tokenmerge_amd."
# reference dotted path -> build dotted path (same module layout under the build's package)
TARGETS = {
    _REF + "attention_blocks.attention.Encoder1DBlock": _BUILD + "attention_blocks.attention.Encoder1DBlock",
    _REF + "attention_blocks.attention.StackedEncoder1DBlock": _BUILD + "attention_blocks.attention.StackedEncoder1DBlock",
    _REF + "attention_blocks.attention.MLPBlock": _BUILD + "attention_blocks.attention.MLPBlock",
    _REF + "tokenizers.readout.readout.AddPositionEmbedding": _BUILD + "tokenizers.readout.readout.AddPositionEmbedding",
    _REF + "tokenizers.images.image_tokenizer.ImageTokenizer": _BUILD + "tokenizers.images.image_tokenizer.ImageTokenizer",
    _REF + "tokenizers.images.image_tokenizer.ResNetV2Block": _BUILD + "tokenizers.images.image_tokenizer.ResNetV2Block",
    _REF + "tokenizers.text.t5_base.T5Tokenizer": _BUILD + "tokenizers.text.t5_base.T5Tokenizer",
    _REF + "action_heads.diffusion.DiffusionActionHead": _BUILD + "action_heads.diffusion.DiffusionActionHead",
    _REF + "action_heads.continuous.ContinuousActionHead": _BUILD + "action_heads.continuous.ContinuousActionHead",
    _REF + "action_heads.categorical.CategoricalActionHead": _BUILD + "action_heads.categorical.CategoricalActionHead",
    _REF + "models.octo.octo.Octo": _BUILD + "models.octo.octo.Octo",
}
# targets whose semantics live inside the build's fused kernels: instantiated as LayerSpec
SPEC_PREFIXES = ("flax.linen.", "transformers.", "optax.",
                 _REF + "action_heads.diffusion.OctoDenoise", _REF + "action_heads.diffusion.FourierFeatures",
                 _REF + "attention_blocks.attention.MultiHeadAttentionPooling",
                 _REF + "attention_blocks.attention.AddPositionEmbedding")


def resolve_target(target: str):
    """The build class for a reference dotted path, or a LayerSpec factory."""
    if target in TARGETS:
        mod, _, name = TARGETS[target].rpartition(".")
        return getattr(importlib.import_module(mod), name)
    if target.startswith(_BUILD):
        mod, _, name = target.rpartition(".")
        return getattr(importlib.import_module(mod), name)
    if target.startswith(SPEC_PREFIXES):
        return functools.partial(LayerSpec, target)
    raise ValueError(f"unknown _target_ {target!r} (not part of the build's hot path)")


def instantiate(node, *args, _recursive_: bool = True, **kwargs):
    """hydra.utils.instantiate restated for the build: nested ``_target_`` nodes are built first
    (unless _recursive_=False), ``_partial_: true`` returns a functools.partial."""
    if isinstance(node, list):
        return [instantiate(v, _recursive_=_recursive_) for v in node]
    if not isinstance(node, dict):
        return node
    if "_target_" not in node:
        return {k: instantiate(v, _recursive_=_recursive_) if _recursive_ else v for k, v in node.items()}
    target = node["_target_"]
    partial = bool(node.get("_partial_", False))
    kw = {k: v for k, v in node.items() if k not in ("_target_", "_partial_", "_recursive_")}
    if _recursive_:
        kw = {k: instantiate(v) for k, v in kw.items()}
    kw.update(kwargs)
    fn = resolve_target(target)
    if isinstance(fn, functools.partial) and fn.func is LayerSpec:
        return LayerSpec(target, kw, partial)
    if partial:
        return functools.partial(fn, *args, **kw)
    return fn(*args, **kw)


# ------------------------------------------------------------------- schema -> OctoConfig
def _first(d: dict, *paths, default=KeyError):
    for p in paths:
        try:
            return _get_path(d, p)
        except (KeyError, IndexError, TypeError):
            continue
    if default is KeyError:
        raise KeyError(f"none of {paths} in the config")
    return default


def octo_config_from_yaml(cfg: dict, name: str = "yaml"):
    """The reference schema (octo_base.yaml + its component YAMLs, keys read by octo.py:58-87)
    as the build's OctoConfig."""
    from .models.octo.config import OctoConfig
    from .tokenizers.text.t5_base import T5Config
    ab = cfg.get("attention_blocks", {})
    stack = ab.get("stacked_encoder_1d_block", ab)
    blk = stack.get("encoder_1d_block", {})
    sa = blk.get("self_attention", {})
    mlp = blk.get("mlp_block", {})
    D = int(cfg["token_embedding_dim"])
    img = _first(cfg, "tokenizers.images.encoder")
    heads_cfg = cfg.get("action_heads", {})
    diff = heads_cfg.get("diffusion_action_head", {})
    den = diff.get("denoising_model", {})
    action_dim = int(_first(heads_cfg, "action_space_dim", default=0) or
                     _first(den, "mlp_block.dense_out.features", default=8))
    head_names = ["diffusion"]
    for h in heads_cfg.get("heads", []) or []:
        n = str(h.get("name", ""))
        for k in ("continuous", "categorical"):
            if k in n and k not in head_names:
                head_names.append(k)
    kw = dict(
        name=name,
        token_embedding_dim=D,
        num_heads=int(sa.get("num_heads", 8)),
        mlp_dim=int(_first(mlp, "dense.features", default=4 * D)),
        num_blocks=int(stack.get("num_blocks", 1)),
        image_size=tuple(int(v) for v in img.get("image_size", (256, 256, 3))),
        patch_size=int(img.get("patch_size", 16)),
        position_interval=int(img.get("position_interval", 128)),
        input_sequence=str(cfg["input_sequence"]),
        token_compression_sequence=cfg.get("token_compression_sequence"),
        tokens_per_readout=int(cfg.get("tokens_per_readout", 4)),
        num_observation_blocks=int(cfg.get("num_observation_blocks", 1)),
        action_space_dim=action_dim,
        diffusion_steps=int(diff.get("diffusion_steps", 32)),
        denoise_blocks=int(den.get("num_blocks", 1)),
        action_heads=tuple(head_names),
        num_bins=int(heads_cfg.get("num_bins", 256)),
        max_action=float(heads_cfg.get("max_action", 5.0)),
        dropout_rate=float(_first(blk, "dropout.rate", default=0.1)),
        attention_dropout_rate=float(sa.get("dropout_rate", 0.1)),
        layer_norm_eps=float(_first(blk, "layer_norm.epsilon", default=1e-6)),
    )
    qkv = sa.get("qkv_features")
    if qkv is not None and int(qkv) != D:
        raise ValueError(f"qkv_features {qkv} != token_embedding_dim {D} (the build's fused QKV)")
    if "resnet" in img:
        kw["stem"] = dict(features=int(_first(img, "resnet.input_conv.features", default=64)),
                          conv_kernel=tuple(_first(img, "resnet.input_conv.kernel_size", default=(12, 12))),
                          conv_stride=int(_first(img, "resnet.input_conv.strides", default=(2, 2))[0]),
                          pool=tuple(_first(img, "resnet.input_pool.window_shape", default=(3, 3))),
                          num_blocks=int(_first(img, "resnet.num_blocks", default=2)),
                          num_groups=int(_first(img, "resnet.resnet_norm.num_groups", default=32)),
                          gn_eps=float(_first(img, "resnet.resnet_norm.epsilon", default=1e-6)))
    # text: the sequence string fixes the number of text tokens (TaskDescriptionPrefix{n})
    m = re.findall(r"(?:TaskDescriptionPrefix|Text)\{(\d+)\}", kw["input_sequence"])
    kw["text_tokens"] = int(cfg.get("text_tokens", sum(int(v) for v in m)))
    kw["fp8"] = bool(cfg.get("fp8_matmul", False))
    kw["compression"] = str(cfg.get("token_compression_method", "tome"))
    t5_layers = cfg.get("t5_num_layers")
    if t5_layers:
        kw["t5"] = T5Config(num_layers=int(t5_layers))
    return OctoConfig(**kw)


def load_octo_config(config_name: str = "octo_small_tome16", config_dir=None, overrides=None):
    cfg = compose(config_name, config_dir, overrides)
    return octo_config_from_yaml(cfg, name=Path(config_name).stem)
