"""CPU tests of the parameter-tree / checkpoint interchange:
reference-layout Flax tree round trip through the flax msgpack wire format, the layout rules
(scan-stacked blocks, (D, H, Dh) attention kernels, (kh, kw, cin, cout) convolutions), a
hand-built flax.serialization byte string, transformers-T5 import and resume files."""
import msgpack
import numpy as np
import pytest
import torch

from multi_modal_transformers_tokenmerge_amd import checkpoint as C


@pytest.fixture(scope="module")
def models():
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    cfg = get_config("octo-tiny", num_blocks=3)
    return Octo(cfg, device="cpu", seed=0), Octo(cfg, device="cpu", seed=7)


def test_flax_tree_round_trip(models):
    m1, m2 = models
    tree = C.flax_msgpack_loads(C.flax_msgpack_dumps(C.to_flax_params(m1)))
    assert C.load_flax_params(m2, tree) == []
    for p1, p2 in zip(m1.store.params, m2.store.params):
        assert torch.equal(p1.data, p2.data), p1.name
    assert torch.equal(m2.store.flat_bf16, m2.store.flat.to(torch.bfloat16))


def test_flax_tree_layout(models):
    m1, _ = models
    tree = C.to_flax_params(m1)
    D, H = m1.D, m1.cfg.num_heads
    Dh = D // H
    nb = m1.cfg.num_blocks
    att = tree["attention_blocks"]["ScanEncoder1DBlock_0"]["SelfAttention_0"]
    assert att["query"]["kernel"].shape == (nb, D, H, Dh)
    assert att["out"]["kernel"].shape == (nb, H, Dh, D)
    blk = m1.stack.blocks[1]
    x = np.random.default_rng(0).normal(size=(5, D)).astype(np.float32)
    # q = x . Wq (Flax: einsum('...d,dhk->...hk')) equals this build's rows 0:D of qkv (x W^T)
    q_flax = np.einsum("nd,dhk->nhk", x, att["query"]["kernel"][1]).reshape(5, D)
    q_ours = x @ blk.qkv.w.data[:D].numpy().T
    np.testing.assert_allclose(q_flax, q_ours, rtol=1e-5, atol=1e-5)
    v = np.random.default_rng(1).normal(size=(5, H, Dh)).astype(np.float32)
    o_flax = np.einsum("nhk,hkd->nd", v, att["out"]["kernel"][1])
    o_ours = v.reshape(5, D) @ blk.out.w.data.numpy().T
    np.testing.assert_allclose(o_flax, o_ours, rtol=1e-5, atol=1e-5)
    conv = tree["image_encoder"]["embedding_function"]["Conv_0"]["kernel"]
    assert conv.shape == (12, 12, 3, 64)
    patch = np.random.default_rng(2).normal(size=(12, 12, 3)).astype(np.float32)
    w = m1.image_tokenizer.resnet.conv.w.data.numpy()          # (64, 432), (kh, kw, c) order
    np.testing.assert_allclose(np.einsum("hwc,hwco->o", patch, conv), w @ patch.reshape(-1),
                               rtol=1e-5, atol=1e-5)
    c1 = tree["image_encoder"]["embedding_function"]["Conv_1"]["kernel"]
    assert c1.shape == (3, 3, 64, 64) and not c1[0].any() and not c1[2].any()
    assert tree["attention_blocks"]["posembed_input"]["pos_embedding"].shape == (1, m1.L0, D)


def test_flax_msgpack_wire_format():
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    # flax.serialization: ndarray -> ExtType(1, packb((shape, dtype.name, bytes)))
    want = msgpack.packb({"w": msgpack.ExtType(1, msgpack.packb(((2, 3), "float32", a.tobytes()),
                                                                use_bin_type=True))},
                         use_bin_type=True)
    assert C.flax_msgpack_dumps({"w": a}) == want
    back = C.flax_msgpack_loads(want)
    assert back["w"].dtype == np.float32 and np.array_equal(back["w"], a)
    # chunked big-array leaves are reassembled
    old = C.MAX_CHUNK
    try:
        C.MAX_CHUNK = 16
        big = np.arange(40, dtype=np.float32).reshape(5, 8)
        assert np.array_equal(C.flax_msgpack_loads(C.flax_msgpack_dumps({"b": big}))["b"], big)
    finally:
        C.MAX_CHUNK = old


def test_load_accepts_alternative_names_and_reports_missing(models):
    m1, m2 = models
    tree = C.to_flax_params(m1)
    ie = tree["image_encoder"]
    ie["image_row_position_embedding"] = ie.pop("row_embeddings")
    del tree["readout_encoder"]
    with pytest.raises(KeyError):
        C.load_flax_params(m2, tree)
    missing = C.load_flax_params(m2, tree, strict=False)
    assert missing == ["AddPositionEmbedding_0/pos_embedding"]
    assert torch.equal(m2.image_tokenizer.row_emb.data, m1.image_tokenizer.row_emb.data)


def test_hf_t5_import():
    from transformers import T5Config as HFConfig, T5EncoderModel
    from multi_modal_transformers_tokenmerge_amd.tokenizers.text.t5_base import T5Config, T5Tokenizer
    torch.manual_seed(0)
    hf = T5EncoderModel(HFConfig(vocab_size=96, d_model=64, d_kv=64, d_ff=128, num_layers=2,
                                 num_heads=2, feed_forward_proj="relu"))
    t5 = T5Tokenizer(T5Config(vocab_size=96, d_model=64, d_kv=64, d_ff=128, num_layers=2,
                              num_heads=2)).materialize("cpu", seed=0)
    C.hf_t5_to_store(t5, hf.state_dict())
    by = t5.store.by_name
    sd = hf.state_dict()
    assert torch.equal(by["T5Tokenizer_0/block/1/SelfAttention/qkv"].bf16[128:256],
                       sd["encoder.block.1.layer.0.SelfAttention.k.weight"].to(torch.bfloat16))
    assert torch.equal(by["T5Tokenizer_0/shared/embedding"].bf16, sd["shared.weight"].to(torch.bfloat16))


def test_train_state_resume(tmp_path, models):
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import create_octo_train_state
    m1, m2 = models
    s1 = create_octo_train_state(m1, seed=3)
    s1.model.store.m.normal_()
    s1.rng[1] = 17
    s1.sample_offset = 512
    path = tmp_path / "state.pt"
    C.save_train_state(str(path), s1)
    s2 = create_octo_train_state(m2, seed=9)
    C.load_train_state(str(path), s2)
    assert torch.equal(m2.store.flat, m1.store.flat) and torch.equal(m2.store.m, m1.store.m)
    assert s2.step == 17 and s2.sample_offset == 512
