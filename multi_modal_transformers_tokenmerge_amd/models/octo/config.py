"""OCTO configurations.

The reference pins only ``model_configs/octo_base.yaml`` (D 768, 3 heads, 1 block, 280^2 images,
patch 56) and reads keys its YAMLs do not define. BASELINE names OCTO-tiny/small/base,
which the reference does not define; the sizes below are SURVEY §8.0's (upstream Octo ViT-t/s/b
widths with the reference architecture and quirks).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Optional

from ...tokenizers.text.t5_base import T5Config


@dataclass
class OctoConfig:
    name: str = "octo-small"
    token_embedding_dim: int = 384
    num_heads: int = 6
    mlp_dim: int = 1536
    num_blocks: int = 12
    image_size: tuple = (256, 256, 3)
    patch_size: int = 16
    position_interval: int = 128
    input_sequence: str = "[TaskDescriptionPrefix{32}] [Image{256};Readout{4}]"
    token_compression_sequence: Optional[str] = None
    tokens_per_readout: int = 4
    num_observation_blocks: int = 1
    action_space_dim: int = 8
    diffusion_steps: int = 32
    # OctoDenoise num_blocks (diffusion.py:62-63): MLPBlocks applied in sequence, the first on
    # concatenate([noisy, time_emb, readout]), the others on the previous block's output
    denoise_blocks: int = 1
    # action heads built (octo.py:83-87 config.action_heads.heads); the bench path is diffusion only
    action_heads: tuple = ("diffusion",)
    num_bins: int = 256
    max_action: float = 5.0
    dropout_rate: float = 0.1
    attention_dropout_rate: float = 0.1
    layer_norm_eps: float = 1e-6
    t5: T5Config = field(default_factory=T5Config)
    text_tokens: int = 32
    # ResNetV2Block hyper-parameters (gato_resnet.yaml:41-104); None = the build defaults
    stem: Optional[dict] = None
    # fp8 weight path (BASELINE configs[4]): the encoder blocks' Dense forward products in e4m3 —
    # the QKV projection and MLP Dense_0 (activation-stationary fp8 kernel, 1.8x its bf16 twin);
    # fp8_residual also puts the residual-stream products (out-projection, MLP Dense_1, fp32
    # residual epilogue) in e4m3, measured slower than their bf16 kernels — off
    fp8: bool = False
    fp8_residual: bool = False
    # how token_compression_sequence's per-layer counts are realised: "tome" (bipartite soft
    # matching + merge_wavg, token_compression.py:54-129, per compressed set) or "prune"
    # (per-set top-k on the attention importance, compressed_attention.py:302-308 +
    # token_compression.py:15-46, every set); YAML key token_compression_method
    compression: str = "tome"

    @property
    def tome_r(self) -> int:
        if not self.token_compression_sequence or self.compression != "tome":
            return 0
        import re
        return max(int(x) for x in re.findall(r"\{(\d+)\}", self.token_compression_sequence))


TOME16 = "[TaskDescriptionPrefix{0}] [Image{16};Readout{0}]"

PRESETS = {
    # configs[0]: CPU plumbing case (no text, 64^2, 1 step)
    "octo-tiny": OctoConfig(name="octo-tiny", token_embedding_dim=192, num_heads=3, mlp_dim=768,
                            image_size=(64, 64, 3), input_sequence="[Image{16};Readout{4}]",
                            text_tokens=0),
    # configs[1]: small, ToMe off
    "octo-small": OctoConfig(),
    # configs[2]: small, ToMe r=16 per block (BASELINE metric config)
    "octo-small-tome16": OctoConfig(name="octo-small-tome16", token_compression_sequence=TOME16),
    # configs[3]: base, 2 cameras, 2-step history
    "octo-base-2cam": OctoConfig(
        name="octo-base-2cam", token_embedding_dim=768, num_heads=12, mlp_dim=3072,
        input_sequence="[TaskDescriptionPrefix{32}] [Image{256};Image{256};Readout{4}]*2",
        num_observation_blocks=2),
    # configs[3] with ToMe on every image set: two cameras x two steps, r = 16 per set and block
    # (one bipartite match + merge per set, token_sequencer.py:222-238 per-set counts)
    "octo-base-2cam-tome16": OctoConfig(
        name="octo-base-2cam-tome16", token_embedding_dim=768, num_heads=12, mlp_dim=3072,
        input_sequence="[TaskDescriptionPrefix{32}] [Image{256};Image{256};Readout{4}]*2",
        token_compression_sequence="[TaskDescriptionPrefix{0}] [Image{16};Image{16};Readout{0}]*2",
        num_observation_blocks=2),
    # configs[4]: base hi-res 512^2, ToMe r=32, fp8 weight path
    "octo-base-hires-tome32": OctoConfig(
        name="octo-base-hires-tome32", token_embedding_dim=768, num_heads=12, mlp_dim=3072,
        image_size=(512, 512, 3), input_sequence="[TaskDescriptionPrefix{32}] [Image{1024};Readout{4}]",
        token_compression_sequence="[TaskDescriptionPrefix{0}] [Image{32};Readout{0}]", fp8=True),
    # top-k pruning on the small geometry: 16 image tokens per block
    "octo-small-prune16": OctoConfig(name="octo-small-prune16", token_compression_sequence=TOME16,
                                     compression="prune"),
}


def get_config(name: str, **overrides) -> OctoConfig:
    """A preset by name ("octo-small-tome16"), or a YAML config of the reference schema from
    model_configs/ ("octo_small_tome16", "ref_octo_base", or a path ending in .yaml)."""
    if name not in PRESETS:
        from ...config_loader import CONFIG_DIR, load_octo_config
        from pathlib import Path
        p = Path(name)
        if name.endswith(".yaml") and p.exists():
            return replace(load_octo_config(p.name, p.parent), **overrides)
        if (CONFIG_DIR / f"{name}.yaml").exists():
            return replace(load_octo_config(name), **overrides)
        raise KeyError(f"unknown config {name!r}; known: {sorted(PRESETS)} or "
                       f"model_configs/*.yaml")
    return replace(PRESETS[name], **overrides)
