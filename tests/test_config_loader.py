"""CPU: the YAML configuration surface (config_loader.py) — the reference's Hydra compose +
instantiate(_target_) schema (octo.py:75-84, octo_base.yaml:12-18) restated without Hydra."""
import functools

import pytest

from multi_modal_transformers_tokenmerge_amd import config_loader as C
from multi_modal_transformers_tokenmerge_amd.models.octo.config import PRESETS, get_config


@pytest.mark.parametrize("yaml_name,preset", [
    ("octo_tiny", "octo-tiny"), ("octo_small", "octo-small"),
    ("octo_small_tome16", "octo-small-tome16"), ("octo_base_2cam", "octo-base-2cam"),
    ("octo_base_hires_tome32", "octo-base-hires-tome32")])
def test_yaml_configs_equal_presets(yaml_name, preset):
    from dataclasses import asdict
    a, b = asdict(C.load_octo_config(yaml_name)), asdict(PRESETS[preset])
    diff = {k: (a[k], b[k]) for k in a if k not in ("name", "stem") and a[k] != b[k]}
    assert not diff


def test_compose_defaults_interpolation_overrides():
    cfg = C.compose("octo_small_tome16", overrides=["num_blocks=3", "token_embedding_dim=256",
                                                     "attention_blocks.stacked_encoder_1d_block.encoder_1d_block.dropout.rate=0.2"])
    blk = cfg["attention_blocks"]["stacked_encoder_1d_block"]
    assert blk["num_blocks"] == 3                                   # ${num_blocks} after override
    assert blk["encoder_1d_block"]["mlp_block"]["dense_out"]["features"] == 256
    assert cfg["tokenizers"]["images"]["encoder"]["row_position_embedding"]["num_embeddings"] == 128
    assert cfg["action_heads"]["heads"][0]["module"]["_target_"].endswith("DiffusionActionHead")
    oc = C.octo_config_from_yaml(cfg)
    assert (oc.num_blocks, oc.token_embedding_dim, oc.dropout_rate, oc.tome_r) == (3, 256, 0.2, 16)
    with pytest.raises(KeyError):
        C.compose("no_such_config")
    with pytest.raises(ValueError):
        C.compose("octo_small", overrides=["num_blocks"])


def test_reference_geometry_config():
    c = get_config("ref_octo_base")            # the reference's own octo_base.yaml geometry
    assert (c.token_embedding_dim, c.num_heads, c.mlp_dim, c.num_blocks) == (768, 3, 768, 1)
    assert (c.image_size, c.patch_size, c.text_tokens, c.num_observation_blocks) == ((280, 280, 3), 56, 16, 2)


def test_instantiate_targets():
    node = {"_target_": "multi_modal_transformers.tokenizers.readout.readout.AddPositionEmbedding",
            "posemb_init": {"_target_": "flax.linen.initializers.he_normal"}}
    cls = C.resolve_target(node["_target_"])
    from multi_modal_transformers_tokenmerge_amd.tokenizers.readout.readout import AddPositionEmbedding
    assert cls is AddPositionEmbedding
    spec = C.instantiate({"_target_": "flax.linen.Dense", "features": 8})
    assert isinstance(spec, C.LayerSpec) and spec.get("features") == 8
    act = C.instantiate({"_target_": "flax.linen.relu", "_partial_": True})
    assert act.partial and act.target == "flax.linen.relu"
    p = C.instantiate({"_target_": "multi_modal_transformers.models.octo.octo.Octo", "_partial_": True})
    assert isinstance(p, functools.partial)
    with pytest.raises(ValueError):
        C.instantiate({"_target_": "multi_modal_transformers.models.deprecated.gato.Gato"})
