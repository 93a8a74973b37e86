"""CPU tests of the host-side logic and the oracle's known-answer tests (no GPU needed).

KAT-3 / KAT-4 restate the reference's own tests (tokenizers/images/tests/test_image_tokenizer.py
:22-36 raster round trip, :41-53 eval position tokens); KAT-5 is the block mask of SURVEY §8c
derived from token_sequencer.py:94-183.
"""
import numpy as np
import pytest
import torch

from oracle import octo_ref as OR
from oracle import rng as R


# ----------------------------------------------------------------------------- KAT-4 patches
def test_kat4_image_to_patches_raster_round_trip():
    # 16 constant patches of 70x70x3 with values 1..16 assigned in raster order
    patches = np.ones((16, 70, 70, 3), np.float32) * (np.arange(16, dtype=np.float32) + 1)[:, None, None, None]
    image = patches.reshape(4, 4, 70, 70, 3).transpose(0, 2, 1, 3, 4).reshape(280, 280, 3)
    out = OR.image_to_patches(image, 70, normalize=False)
    assert out.shape == (16, 70, 70, 3)
    np.testing.assert_array_equal(out, patches)
    norm = OR.image_to_patches(np.full((32, 32, 3), 255.0, np.float32), 16, normalize=True)
    np.testing.assert_allclose(norm, 1.0)


# ----------------------------------------------------------------------------- KAT-3 positions
def test_kat3_encode_patch_position_reference_case():
    row, col = OR.encode_patch_position_eval(128, 1, 128)
    assert row.shape == (128 * 128,) and col.shape == (128 * 128,)
    assert row[123] == 122                      # test_image_tokenizer.py:53
    # transposed convention (image_tokenizer.py:91-92): row token follows p % P, col p // P
    p = np.arange(128 * 128)
    np.testing.assert_array_equal(col, row[p // 128])
    np.testing.assert_array_equal(row, row[p % 128])


def test_kat3_encode_patch_position_small_geometry():
    row, col = OR.encode_patch_position_eval(256, 16, 128)
    p = np.arange(256)
    np.testing.assert_array_equal(row, 3 + 8 * (p % 16))
    np.testing.assert_array_equal(col, 3 + 8 * (p // 16))


# ----------------------------------------------------------------------------- KAT-5 masks
def _dense_from_table(sets):
    L = sets.L
    m = np.zeros((L, L), bool)
    for i, (si, li) in enumerate(zip(sets.starts, sets.lens)):
        for j, (sj, lj) in enumerate(zip(sets.starts, sets.lens)):
            if sets.vis[i] >> j & 1:
                m[si:si + li, sj:sj + lj] = True
    return m


def test_kat5_small_block_mask():
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_sequencer import TokenSequence
    seq = TokenSequence("[TaskDescriptionPrefix{32}] [Image{256};Readout{4}]")
    sets = seq.set_table(0)
    assert sets.lens == [32, 256, 4]
    vis = [[sets.vis[i] >> j & 1 for j in range(3)] for i in range(3)]
    assert vis == [[1, 0, 0], [1, 1, 0], [1, 1, 1]]
    m = seq.generate_attention_mask(repeats=2)
    assert m.shape == (2, 292, 292)
    assert m[0].sum(1).min() > 0                  # no fully masked row


CASES = [
    ("[TaskDescriptionPrefix{32}] [Image{256};Readout{4}]", None, [0]),
    ("[TaskDescriptionPrefix{32}] [Image{256};Readout{4}]",
     "[TaskDescriptionPrefix{0}] [Image{16};Readout{0}]", [0, 1, 5, 11]),
    ("[TaskDescriptionPrefix{32}] [Image{256};Image{256};Readout{4}]*2", None, [0]),
    ("[Image{16};Readout{4}]", None, [0]),
    ("[TaskDescriptionPrefix{16}] [Image{25};Readout{4}]*2", None, [0]),
]


@pytest.mark.parametrize("seq_str,comp,layers", CASES)
def test_set_table_matches_literal_mask(seq_str, comp, layers):
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_sequencer import TokenSequence
    seq = TokenSequence(seq_str, comp)
    spec = OR.sequence_spec(seq_str, comp)
    for layer in layers:
        sets = seq.set_table(layer)
        lit = OR.literal_mask([(k, n - layer * c, t) for k, n, t, c in spec])
        np.testing.assert_array_equal(_dense_from_table(sets), lit)
        np.testing.assert_array_equal(seq.generate_attention_mask(layer=layer if comp else None,
                                                                  square=True)[0], lit)


def test_modality_idx_and_slices():
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_sequencer import TokenSequence
    seq = TokenSequence("[TaskDescriptionPrefix{32}] [Image{256};Readout{4}]*2")
    np.testing.assert_array_equal(seq.get_modality_idx("readouts"),
                                  np.r_[288:292, 548:552])
    assert seq.slice_idx == [(0, 32), (0, 256), (0, 4), (256, 256), (4, 4)]


# ----------------------------------------------------------------------------- diffusion
def test_cosine_schedule_matches_oracle():
    from multi_modal_transformers_tokenmerge_amd.action_heads.diffusion import (
        alpha_hats_of, cosine_beta_schedule)
    b = cosine_beta_schedule(32)
    np.testing.assert_array_equal(b, OR.cosine_beta_schedule(32))
    ah = alpha_hats_of(b)
    assert ah.shape == (32,) and np.all(np.diff(ah) < 0) and 0 < ah[-1] < ah[0] <= 1
    np.testing.assert_allclose(ah, np.cumprod(1 - b.astype(np.float64)), rtol=1e-6)


# ----------------------------------------------------------------------------- RNG / sharding
def test_dropout_streams_shard_by_global_sample():
    """N ranks x B samples draw exactly the keep-masks of 1 rank x N*B (row offsets are global)."""
    B, L, D, N = 3, 20, 64, 4
    full = R.dropout_mask_2d(1234, 7, 2, 2, N * B * L, D, 0, 0.9)
    for r in range(N):
        part = R.dropout_mask_2d(1234, 7, 2, 2, B * L, D, r * B * L, 0.9)
        np.testing.assert_array_equal(part, full[r * B * L:(r + 1) * B * L])
    assert abs(full.mean() - 0.9) < 0.01


def test_keep_threshold_edges():
    assert R.keep_thresh16(1.0) == 65536 and R.keep_thresh16(0.0) == 0
    assert R.keep_mask(R.stream_key(1, 0, 0, 0), np.arange(1000), 1.0).all()
    assert not R.keep_mask(R.stream_key(1, 0, 0, 0), np.arange(1000), 0.0).any()


# ----------------------------------------------------------------------------- fail loudly
def test_product_ops_refuse_host_tensors():
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_compression import (
        bipartite_soft_matching)
    with pytest.raises((ValueError, ImportError)):
        bipartite_soft_matching(torch.randn(2, 16, 8), 4)
    # r <= 0 is the reference's do-nothing tuple (token_compression.py:69-70), no kernel call
    a, b = bipartite_soft_matching(torch.randn(2, 16, 8), 0)
    x = torch.randn(2, 16, 8)
    assert a(x) is x and b(x) is x


# ----------------------------------------------------------------------------- T5 oracle pin
def test_t5_oracle_matches_transformers_golden():
    """oracle t5_encoder vs transformers.T5EncoderModel (tests/golden/make_t5_golden.py)."""
    from pathlib import Path
    g = np.load(Path(__file__).parent / "golden" / "t5_small_golden.npz")
    tp = {k: torch.from_numpy(g[k]) for k in g.files if k.startswith("T5Tokenizer_0")}
    out = OR.t5_encoder(tp, torch.from_numpy(g["ids"]), num_layers=2, H=4, d_kv=8)
    np.testing.assert_allclose(out.numpy(), g["out"], rtol=1e-4, atol=1e-4 * np.abs(g["out"]).max())


# ----------------------------------------------------------------------------- DDPM sampler
def test_sampler_oracle_quirks_and_coefficients():
    """oracle/sampler_ref.py vs a hand loop of diffusion.py:182-188 with a zero denoiser: the
    update degenerates to x <- clip(c1 x + c3 z) with the SAME z every step (the reference never
    splits its keys, :178), noise included at t = 0; the last beta is clipped to 0.999 (:27)."""
    from multi_modal_transformers_tokenmerge_amd.action_heads.diffusion import DiffusionActionHead
    from multi_modal_transformers_tokenmerge_amd.params import ParamStore
    from oracle import sampler_ref as SR
    head = DiffusionActionHead.create(ParamStore(), "h", 16, 8, 32)
    assert head.betas_np[-1] == pytest.approx(0.999)
    coef = SR.sampler_coefficients(head.betas_np, head.alpha_hats_np)
    np.testing.assert_allclose(head.sampler_coef(torch.device("cpu")).numpy(), coef, rtol=1e-5)
    g = np.random.default_rng(0)
    B, A, T, D, H = 3, 8, 4, 8, 16
    z = g.normal(size=(B, A))
    x = z.copy()
    for t in range(31, -1, -1):
        x = np.clip(coef[t, 0] * x + coef[t, 2] * z, -5, 5)
    got = SR.predict_action(np.zeros((B, D)), z, np.zeros((32, T)), np.zeros((H, A + T + D)),
                            np.zeros(H), np.zeros((A, H)), np.zeros(A), coef)
    np.testing.assert_allclose(got, x, rtol=0, atol=1e-12)
    # a denoiser that predicts eps = x (W1 = I on the action block, W2 = I) stays inside [-5, 5]
    w1 = np.zeros((H, A + T + D)); w1[:A, :A] = np.eye(A)
    w2 = np.zeros((A, H)); w2[:, :A] = np.eye(A)
    out = SR.predict_action(np.zeros((B, D)), z, np.zeros((32, T)), w1, np.zeros(H), w2,
                            np.zeros(A), coef)
    assert np.all(np.abs(out) <= 5.0) and np.isfinite(out).all()


# ----------------------------------------------------------------------------- action heads
def test_assign_bins_reference_off_by_one():
    """categorical.py:12-22 + octo.py:191-192: digitize returns 1..num_bins for in-range actions,
    so one_hot(bin, num_bins) shifts every class up by one and drops the top bin."""
    from multi_modal_transformers_tokenmerge_amd.action_heads.categorical import assign_bins
    from oracle import heads_ref as HR
    a = np.array([-5.0, -4.99, -0.01, 0.0, 4.99, 5.0, 7.0, -9.0], np.float32)
    bins = assign_bins(a, (-5.0, 5.0), 10)
    np.testing.assert_array_equal(bins, [1, 1, 5, 6, 10, 11, 11, 0])
    np.testing.assert_array_equal(HR.digitize_bins(a, 5.0, 10), bins)
    z = np.zeros((1, 8, 10))
    loss, dz = HR.categorical(z, a[None], 5.0, 10)
    # bins >= 10 carry no label: 5 of the 8 actions (bins 1, 1, 5, 6 and 0) contribute log(10)
    assert loss == pytest.approx(5 * np.log(10) / 8)
    assert np.allclose(dz[0, 4:7], 0) and not np.allclose(dz[0, 7], 0)


def test_continuous_head_oracle_gradient():
    from oracle import heads_ref as HR
    g = np.random.default_rng(0)
    z, y = g.normal(size=(3, 8)) * 4, g.normal(size=(3, 8))
    _, loss, dz = HR.continuous(z, y, 5.0)
    eps = 1e-6
    num = np.zeros_like(z)
    for i in np.ndindex(z.shape):
        zp = z.copy(); zp[i] += eps
        num[i] = (HR.continuous(zp, y, 5.0)[1] - loss) / eps
    np.testing.assert_allclose(dz, num, rtol=1e-4, atol=1e-6)


def test_ddp_stage_plan_regions_cover_the_store():
    """distributed.DDPStep's backward split (Octo.stage_bounds / grad_regions) on the CPU-built
    model: "auto[:MB]" gives byte-sized regions from the top and block 0 alone in the last stage;
    for every plan the regions tile [0, n) without overlap, stage 0 holds the heads (the top of
    the store) and the last stage everything below block 1."""
    import torch
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    m = Octo(get_config("octo-small-tome16"), torch.device("cpu"), seed=0)
    nb = m.cfg.num_blocks
    for plan in ("auto", "auto:12", "auto:0.001", 1, 3, nb, [nb, 6, 1, 0]):
        b = m.stage_bounds(plan)
        assert b[0] == nb and b[-1] == 0 and all(x > y for x, y in zip(b, b[1:])), (plan, b)
        regs = m.grad_regions(b)
        assert regs[0][1] == m.store.n and regs[-1][0] == 0
        assert all(regs[i][0] == regs[i + 1][1] for i in range(len(regs) - 1))
        if isinstance(plan, str):
            assert b[-2] == 1  # block 0 alone in the last stage
    b = m.stage_bounds("auto")
    exposed = 4 * (m.grad_regions(b)[-1][1] - m.grad_regions(b)[-1][0])
    even = 4 * (m.grad_regions(3)[-1][1] - m.grad_regions(3)[-1][0])
    assert exposed < even / 3, (exposed, even)
    assert m.stage_bounds("auto:0.001") == list(range(nb, -1, -1))
    for bad in ([nb, 6, 6, 0], [nb - 1, 0], [nb, 3], [nb, 7, 9, 0], [0], [nb, 2.5, 0]):
        with pytest.raises(ValueError):   # regions missing / overlapping: refused
            m.stage_bounds(bad)


def test_step_fixtures_randomness_and_position_kats():
    """The committed step fixtures (tests/golden/step_*_golden.npz) hold the oracle's counter-stream
    restatements (oracle/rng.py): recomputed here they agree exactly (t, positions) / bitwise
    (eps, same numpy); the position restatement also meets SURVEY §8c KAT-3 (eval midpoints of a
    256^2 image, patch 16) and the reference's own test_image_tokenizer.py:41-53 case
    (128^2, patch 1: row[123] == 122, shape (16384,))."""
    import ast
    from pathlib import Path
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    g = Path(__file__).resolve().parent / "golden"
    for f in sorted(g.glob("step_*_golden.npz")):
        z = np.load(f)
        cfg = get_config(str(z["config"]), **ast.literal_eval(str(z["overrides"])))
        B, seed, step = int(z["B"]), int(z["rng_seed"]), int(z["rng_step"])
        n_img = z["images"].shape[1]
        patch = z["images"].shape[2] // int(round(np.sqrt(z["rt"].shape[1] / n_img)))
        rt, ct = R.patch_positions(seed, step, 0, B, n_img, cfg.image_size[0], patch, 128)
        np.testing.assert_array_equal(rt, z["rt"])
        np.testing.assert_array_equal(ct, z["ct"])
        t, eps = R.diffusion_t_eps(seed, step, B, cfg.action_space_dim, cfg.diffusion_steps)
        np.testing.assert_array_equal(t, z["t"])
        np.testing.assert_array_equal(eps, z["eps"])
        assert (0 <= z["t"]).all() and (z["t"] < cfg.diffusion_steps).all()
        from oracle import tome as T
        for li in range(int(z["n_tome"])):  # the stored indices are the canonical match of the metric
            metric = (z[f"tome{li}/metric_bf16"].astype(np.uint32) << 16).view(np.float32)
            unm, src, dst, _ = T.canon_match(metric, cfg.tome_r)
            for nm, a in (("unm", unm), ("src", src), ("dst", dst)):
                np.testing.assert_array_equal(a, z[f"tome{li}/{nm}"])
    rte, cte = R.patch_positions(0, 0, 0, 1, 1, 256, 16, 128, train=False)
    assert (rte[0] == 3 + 8 * (np.arange(256) % 16)).all() and (cte[0] == 3 + 8 * (np.arange(256) // 16)).all()
    r2, _ = R.patch_positions(0, 0, 0, 1, 1, 128, 1, 128, train=False)
    assert r2.shape == (1, 16384) and r2[0, 123] == 122


def test_wgrad_split_sizing():
    """layers.split_k_for: the split-K factor of a weight-gradient launch is sized for `wgs`
    workgroups of the TN kernel's tiles (384 x 192 where n_out % 384 == 0, else 256 x 192) —
    half the chip (128) by default for the step's side-queue launches, the whole chip (256) for a
    standalone launch — capped at 64 and at one 256-token chunk per split."""
    from multi_modal_transformers_tokenmerge_amd.layers import split_k_for, _TN_BM
    if _TN_BM != 384:
        pytest.skip("MMT_TN_BM=256 changes the tile")
    M = 512 * 276
    assert split_k_for(1536, 384, M) == 16           # 8 tiles: 128 // 8
    assert split_k_for(1536, 384, M, wgs=256) == 32  # the bench's full-chip probe
    assert split_k_for(1152, 384, M, wgs=256) == 42  # 6 tiles
    assert split_k_for(384, 384, M, wgs=256) == 128  # 2 tiles: capped at 128
    assert split_k_for(384, 384, 1000) == 3          # 1000 // 256 chunks
    assert split_k_for(4096, 384, M, wgs=256) == 8   # 4096 % 384 != 0: 16 x 2 tiles of 256 x 192


def test_multiset_tome_plan_and_oracle_merge():
    """ToMe on several token sets per layer: the model's per-layer plan takes every set's own
    count from the compression string (token_sequencer.py:222-238), and the oracle merges each
    set with its own matching and carried sizes (the shapes the HIP path must produce)."""
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo.octo import Octo
    from oracle.octo_ref import OctoRef, sequence_spec
    from oracle.parity import _inputs, oracle_params
    cfg = get_config("octo-tiny", num_blocks=2, image_size=(128, 128, 3),
                     input_sequence="[Image{64};Image{64};Readout{4}]*2", num_observation_blocks=2,
                     token_compression_sequence="[Image{8};Image{4};Readout{1}]*2")
    model = Octo(cfg, torch.device("cpu"), seed=0)
    ctxs = model.layer_ctxs(True, None, 0)
    assert [c.tome_sets() for c in ctxs] == [((0, 8), (1, 4), (2, 1), (3, 8), (4, 4), (5, 1))] * 2
    assert [c.r for c in ctxs] == [26, 26] and all(c.tome_set == -2 for c in ctxs)
    assert ctxs[1].sets.lens == [56, 60, 3, 56, 60, 3]
    single = Octo(get_config("octo-small-tome16", num_blocks=2), torch.device("cpu"), seed=0)
    c0 = single.layer_ctxs(True, None, 0)[0]
    assert c0.tome_sets() == ((1, 16),) and c0.tome_set == 1 and c0.r == 16
    # the oracle: per-set canonical matching, sizes carried per set, 264 -> 238 -> 212 tokens
    B = 2
    images, _, actions = _inputs(model, B, 0)
    params, _ = oracle_params(model)
    ref = OctoRef(cfg, params, None, emulate_bf16=True)
    seq = sequence_spec(cfg.input_sequence, cfg.token_compression_sequence)
    rt, ct = R.patch_positions(1234, 0, 0, B, model.n_images, 128, 16, 128)
    t, eps = R.diffusion_t_eps(1234, 0, B, cfg.action_space_dim, cfg.diffusion_steps)
    rec = []
    loss, ex = ref.forward_loss(None, images.astype(np.float32), actions, seed=1234, step=0,
                                positions=(rt, ct), t=t, eps=eps, sequence=seq, record=rec)
    assert [x.shape[1] for x in rec] == [264, 238] and ex["x_final"].shape[1] == 212
    assert all(isinstance(u, list) and len(u) == 6 for u in ex["tome"])
    assert [len(u[0]) for u in ex["tome"][0]] == [2] * 6  # (unm, src, dst) per set
    assert [u[1].shape[1] for u in ex["tome"][0]] == [8, 4, 1, 8, 4, 1]
    loss.backward()
    assert torch.isfinite(loss)
