"""GPU parity: gfx950 ToMe kernels vs the canonical C oracle — bit-exact indices and merges."""
import numpy as np
import pytest
import torch

from oracle import tome as O

pytestmark = pytest.mark.gpu


def _bf16_round(a: np.ndarray) -> np.ndarray:
    return torch.from_numpy(a).bfloat16().float().numpy()


@pytest.fixture(params=[True, False], ids=["mfma", "valu"])
def match_path(request):
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    K.set_tome_match_path(request.param)
    yield request.param
    K.set_tome_match_path(True)


CASES = [(4, 256, 64, 1, 16, 0), (3, 257, 64, 1, 16, 0), (2, 64, 32, 1, 8, 1), (2, 64, 32, 1, 8, 2),
         (2, 64, 32, 1, 8, 3), (2, 31, 6, 1, 7, 0), (5, 292, 64, 6, 16, 0), (2, 512, 64, 1, 32, 0),
         (64, 256, 64, 6, 16, 0),
         # hi-res config (configs[4]): t = 1024 image tokens, heads = 12, r = 32; the maximum t;
         # Dh = 256 (ref-octo_base); a partial last a tile (t = 1000) and a tiny odd t
         (4, 1024, 64, 12, 32, 0), (2, 2048, 64, 1, 64, 0), (2, 26, 256, 3, 5, 0),
         (3, 1000, 64, 2, 100, 3), (2, 3, 8, 1, 1, 0),
         # t = 1024 / 1000 with more than 256 (sample, a tile) pairs: the b-resident score kernel
         # takes two a tiles per workgroup (and a partial last pair at t = 1000)
         (20, 1024, 64, 2, 32, 1), (40, 1000, 64, 1, 50, 2)]


@pytest.mark.parametrize("n,t,c,heads,r,flags", CASES)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_match_bit_exact(dev, match_path, n, t, c, heads, r, flags, dtype):
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    if c % 2 and match_path:
        pass  # odd c falls back to the VALU path inside the library
    g = torch.Generator().manual_seed(n * 1000 + t + c + heads + flags)
    m = torch.randn((n, t, heads, c), generator=g).to(dtype)
    exact = m.float().numpy()
    cu, cs, cd, cn = O.canon_match(exact, r, flags)
    dm = m.to(dev) if heads > 1 else m[:, :, 0].to(dev)
    unm, src, dst, nmax = K.tome_match(dm, r, flags, return_node_max=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(unm.cpu().numpy(), cu)
    np.testing.assert_array_equal(src.cpu().numpy(), cs)
    np.testing.assert_array_equal(dst.cpu().numpy(), cd)
    np.testing.assert_array_equal(nmax.cpu().numpy().view(np.uint32), cn.view(np.uint32))


def test_match_ties_and_zero_rows(dev, match_path):
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    m = np.ones((2, 16, 4), np.float32)
    m[1, 3] = 0.0  # zero row -> NaN scores (no eps in the reference, :72)
    m[1, 8] = 0.0
    cu, cs, cd, _ = O.canon_match(m, 5)
    unm, src, dst = K.tome_match(torch.from_numpy(m).to(dev), 5)
    np.testing.assert_array_equal(src.cpu().numpy(), cs)
    np.testing.assert_array_equal(dst.cpu().numpy(), cd)
    np.testing.assert_array_equal(unm.cpu().numpy(), cu)
    # KAT-1 through the kernel
    unm, src, dst = K.tome_match(torch.ones((1, 8, 4), device=dev), 2)
    assert src.tolist() == [[3, 2]] and dst.tolist() == [[0, 0]] and unm.tolist() == [[1, 0]]


@pytest.mark.parametrize("n,L,set_start,t,D,r,flags", [
    (3, 256, 0, 256, 64, 16, 0), (4, 292, 32, 256, 384, 16, 0), (2, 100, 10, 61, 64, 20, 0),
    (2, 80, 5, 64, 128, 8, 2), (2, 80, 5, 64, 128, 8, 4), (2, 80, 5, 64, 128, 8, 12),
    (8, 1060, 32, 1024, 768, 32, 0)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_merge_fwd_bwd_bit_exact(dev, n, L, set_start, t, D, r, flags, dtype):
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    rng = np.random.default_rng(n + L + t + D + r + flags)
    metric = rng.standard_normal((n, t, 16)).astype(np.float32)
    cu, cs, cd, _ = O.canon_match(metric, r)
    x = rng.standard_normal((n, L, D)).astype(np.float32)
    if dtype == torch.bfloat16:
        x = _bf16_round(x)
    size = rng.integers(1, 6, (n, t)).astype(np.float32)
    xo_ref, so_ref = O.canon_merge_wavg(x[:, set_start:set_start + t], size, cu, cs, cd, r, flags)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    xd = tt(x).to(dtype)
    out, so, pos = K.tome_merge_fwd(xd, set_start, t, r, tt(cu), tt(cs), tt(cd), size_in=tt(size),
                                    flags=flags)
    torch.cuda.synchronize()
    out = out.float().cpu().numpy()
    exp = xo_ref if dtype == torch.float32 else _bf16_round(xo_ref)
    np.testing.assert_array_equal(out[:, set_start:set_start + t - r].view(np.uint32),
                                  exp.view(np.uint32))
    np.testing.assert_array_equal(out[:, :set_start], x[:, :set_start])
    np.testing.assert_array_equal(out[:, set_start + t - r:], x[:, set_start + t:])
    np.testing.assert_array_equal(so.cpu().numpy(), so_ref)
    if flags & 8:
        return  # dropped src tokens have no merged row: pos_map only covers scattered merges
    pos_ref = O.canon_pos_map(cu, cs, cd, t, r, flags)
    np.testing.assert_array_equal(pos.cpu().numpy(), pos_ref)
    # backward
    g = rng.standard_normal((n, L - r, D)).astype(np.float32)
    if dtype == torch.bfloat16:
        g = _bf16_round(g)
    plain = bool(flags & 4)
    gi = K.tome_merge_bwd(tt(g).to(dtype), set_start, t, r, pos, None if plain else tt(size),
                          None if plain else so)
    torch.cuda.synchronize()
    gi = gi.float().cpu().numpy()
    gref = O.canon_merge_bwd(g[:, set_start:set_start + t - r], None if plain else size,
                             np.ones_like(so_ref) if plain else so_ref, pos_ref)
    if dtype == torch.bfloat16:
        gref = _bf16_round(gref)
    np.testing.assert_array_equal(gi[:, set_start:set_start + t].view(np.uint32), gref.view(np.uint32))
    np.testing.assert_array_equal(gi[:, :set_start], g[:, :set_start])
    np.testing.assert_array_equal(gi[:, set_start + t:], g[:, set_start + t - r:])


def test_reference_api_merge_wavg_autograd(dev):
    from multi_modal_transformers_tokenmerge_amd.tokenizers.token_compression import (
        bipartite_soft_matching, merge_wavg, do_nothing)
    rng = np.random.default_rng(3)
    metric = torch.from_numpy(rng.standard_normal((2, 40, 8)).astype(np.float32)).to(dev)
    x = torch.from_numpy(rng.standard_normal((2, 40, 16)).astype(np.float32)).to(dev).requires_grad_()
    merge = bipartite_soft_matching(metric, 6)
    out, size = merge_wavg(merge, x)
    assert out.shape == (2, 34, 16) and size.shape == (2, 34, 1)
    lit_merge, *_ = O.literal_bipartite_soft_matching(metric.cpu().numpy(), 6)
    lo, ls = O.literal_merge_wavg(lit_merge, x.detach().cpu().numpy())
    np.testing.assert_allclose(out.detach().cpu().numpy(), lo, rtol=1e-6, atol=1e-6)
    w = torch.randn_like(out)
    (out * w).sum().backward()
    # torch-CPU autograd reference of the same gather/scatter
    xc = x.detach().cpu().double().requires_grad_()
    unm, src, dst = (a.long().cpu() for a in (merge.unm_idx, merge.src_idx, merge.dst_idx))
    a, b = xc[:, ::2], xc[:, 1::2]
    rows = []
    for bi in range(2):
        dstb = b[bi].clone()
        sz = torch.ones(b.shape[1], dtype=torch.float64)
        for i in range(6):
            dstb[dst[bi, i]] = dstb[dst[bi, i]] + a[bi, src[bi, i]]
            sz[dst[bi, i]] += 1
        rows.append(torch.cat([a[bi, unm[bi]], dstb / sz[:, None]]))
    (torch.stack(rows) * w.cpu().double()).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), xc.grad.numpy(), rtol=1e-5, atol=1e-6)
    # r = 0: reference returns the do_nothing pair
    assert bipartite_soft_matching(metric[:, :1], 3) == (do_nothing, do_nothing)


@pytest.mark.parametrize("n,L,D,s0,t,r,sized", [(3, 292, 384, 32, 256, 16, False),
                                                (2, 276, 384, 32, 240, 16, True),
                                                (2, 40, 64, 4, 33, 16, True)])
def test_merge_seqnorm_fused_bit_exact(dev, n, L, D, s0, t, r, sized):
    """The fused ToMe merge + sequence LayerNorm forward equals the merge kernel followed by
    mmt_seqnorm_fwd bit for bit: merged rows, sizes, position map, y, mean and rstd."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    g = torch.Generator().manual_seed(n * L + t)
    x = (torch.randn((n, L, D), generator=g) * 3 + 1).to(dev)
    metric = torch.randn((n, t, 64), generator=g).bfloat16().to(dev)
    unm, src, dst = K.tome_match(metric, r)
    size = (torch.rand((n, t), generator=g) * 3 + 1).to(dev) if sized else None
    gamma = torch.randn(D, generator=g).to(dev)
    beta = torch.randn(D, generator=g).to(dev)
    a_x, a_s, a_p = K.tome_merge_fwd(x, s0, t, r, unm, src, dst, size_in=size)
    a_y, a_m, a_r = K.seqnorm_fwd(a_x, gamma, beta, 1e-6)
    b_x, b_s, b_p, b_y, b_m, b_r = K.tome_merge_seqnorm_fwd(x, s0, t, r, unm, src, dst, gamma,
                                                            beta, 1e-6, size_in=size)
    for a, b in ((a_x, b_x), (a_s, b_s), (a_p, b_p), (a_y, b_y), (a_m, b_m), (a_r, b_r)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,L,D,s0,t,r,drop", [(3, 292, 384, 32, 256, 16, True),
                                               (2, 276, 384, 32, 240, 16, False),
                                               (2, 40, 64, 4, 33, 16, True)])
def test_ln_unmerge_dropout_bwd_fused(dev, n, L, D, s0, t, r, drop):
    """LayerNorm backward + ToMe unmerge + dropout backward in one launch against the three
    kernels in sequence: the unmerged gradient and the dropout output bit for bit, the LayerNorm
    parameter gradients and the bias column sums to fp32 atomic-order rounding."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    g = torch.Generator().manual_seed(n * L + r)
    metric = torch.randn((n, t, 64), generator=g).bfloat16().to(dev)
    unm, src, dst = K.tome_match(metric, r)
    size = (torch.rand((n, t), generator=g) * 3 + 1).to(dev)
    x = (torch.randn((n, L, D), generator=g) * 2).to(dev)
    gamma, beta = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    x1, size_out, pos, _, mu, rs = K.tome_merge_seqnorm_fwd(x, s0, t, r, unm, src, dst, gamma, beta,
                                                            1e-6, size_in=size)
    L2 = L - r
    dy = torch.randn((n, L2, D), generator=g).bfloat16().to(dev)
    addend = torch.randn((n, L2, D), generator=g).to(dev)
    rng = torch.tensor([5, 9], dtype=torch.int32, device=dev) if drop else None
    grads = [torch.zeros(D, device=dev) for _ in range(6)]
    dx = K.seqnorm_bwd(dy, x1, mu, rs, gamma, grads[0], grads[1], addend=addend)
    a_g = K.tome_merge_bwd(dx, s0, t, r, pos, size, size_out)
    a_z = K.dropout_bwd(a_g.reshape(n * L, D), rng, 3, 1, 0.9, row_offset=7 * L, colsum_out=grads[2])
    b_g, b_z = K.ln_unmerge_dropout_bwd(dy, x1, mu, rs, gamma, grads[3], grads[4], addend,
                                        (s0, t, r, pos, size, size_out), rng, 3, 1, 0.9, 7 * L,
                                        bias_grad=grads[5])
    assert torch.equal(a_g, b_g)
    assert torch.equal(a_z.view(n, L, D), b_z)
    for i in range(3):
        torch.testing.assert_close(grads[i + 3], grads[i], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("L2", [384, 385])
def test_ln_unmerge_gate_boundary(dev, L2):
    """The Python gate of the fused LN-1 backward + unmerge (K.ln_unmerge_ok, used by
    Encoder1DBlock.backward) mirrors the C entry point's limits: at 384 merged rows the fused
    kernel runs and equals the three-kernel path; at 385 the gate says no and the C entry refuses
    (MMTError), so the block takes the three-kernel path instead of failing mid-backward."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from multi_modal_transformers_tokenmerge_amd._C import MMTError
    n, D, r, s0 = 2, 64, 16, 32
    L = L2 + r
    t = L - s0 - 4
    g = torch.Generator().manual_seed(L2)
    metric = torch.randn((n, t, 64), generator=g).bfloat16().to(dev)
    unm, src, dst = K.tome_match(metric, r)
    x = torch.randn((n, L, D), generator=g).to(dev)
    gamma, beta = torch.randn(D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    x1, size_out, pos, _, mu, rs = K.tome_merge_seqnorm_fwd(x, s0, t, r, unm, src, dst, gamma, beta, 1e-6)
    dy = torch.randn((n, L2, D), generator=g).bfloat16().to(dev)
    grads = [torch.zeros(D, device=dev) for _ in range(5)]
    dx = K.seqnorm_bwd(dy, x1, mu, rs, gamma, grads[0], grads[1])
    a_g = K.tome_merge_bwd(dx, s0, t, r, pos, None, size_out)
    a_z = K.dropout_bwd(a_g.reshape(n * L, D), None, 3, 1, 1.0)
    tome = (s0, t, r, pos, None, size_out)
    assert K.ln_unmerge_ok(L, L2) == (L2 <= 384)
    if K.ln_unmerge_ok(L, L2):
        b_g, b_z = K.ln_unmerge_dropout_bwd(dy, x1, mu, rs, gamma, grads[2], grads[3], None, tome,
                                            None, 3, 1, 1.0, 0)
        assert torch.equal(a_g, b_g) and torch.equal(a_z.view(n, L, D), b_z)
    else:
        with pytest.raises(MMTError):
            K.ln_unmerge_dropout_bwd(dy, x1, mu, rs, gamma, grads[2], grads[3], None, tome, None, 3,
                                     1, 1.0, 0)


def test_out_of_range_indices_are_reported_not_faulted(dev):
    """A broken producer of the merge maps (the round-5 fault: an ablated matcher whose maps were
    not a partition of the a half, so the forward left holes in pos_map and the backward read rows
    far outside g_out) must give MMTError from mmt_device_status, never an illegal address. Every
    index-consuming entry point is fed out-of-range and repeated indices; the context stays usable
    (a valid merge afterwards is still bit-exact and the status is clean)."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as K
    from multi_modal_transformers_tokenmerge_amd._C import MMTError
    n, L, s0, t, D, r = 4, 292, 32, 256, 384, 16
    ta = (t + 1) // 2
    K.device_status()  # clean start
    g = torch.Generator().manual_seed(11)
    x = torch.randn((n, L, D), generator=g).to(dev)
    metric = torch.randn((n, t, 64), generator=g).to(dev)
    unm, src, dst = K.tome_match(metric, r)
    gamma, beta = torch.ones(D, device=dev), torch.zeros(D, device=dev)

    def expect(bit_text, fn):
        fn()
        with pytest.raises(MMTError, match=bit_text):
            K.device_status()
        K.device_status()  # cleared by the report

    huge = torch.full_like(unm, 1 << 28)
    expect("out of range", lambda: K.tome_merge_fwd(x, s0, t, r, huge, src, dst))
    expect("out of range", lambda: K.tome_merge_fwd(x, s0, t, r, unm, src - 4 * ta, dst))
    expect("out of range", lambda: K.tome_merge_fwd(x, s0, t, r, unm, src, dst + t))
    expect("out of range", lambda: K.tome_merge_seqnorm_fwd(x, s0, t, r, huge, src, dst, gamma, beta, 1e-6))
    dup = unm.clone()
    dup[:, 1] = dup[:, 0]  # in range, but an a token named twice: pos_map would keep a hole
    expect("partition", lambda: K.tome_merge_fwd(x, s0, t, r, dup, src, dst))
    expect("partition", lambda: K.tome_merge_seqnorm_fwd(x, s0, t, r, dup, src, dst, gamma, beta, 1e-6))
    xo, so, pos = K.tome_merge_fwd(x, s0, t, r, unm, src, dst)
    gout = torch.randn_like(xo)
    bad_pos = pos.clone()
    bad_pos[:, 5] = 1 << 30
    bad_pos[:, 6] = -7
    expect("pos_map", lambda: K.tome_merge_bwd(gout, s0, t, r, bad_pos, None, so))
    x1, so1, pos1, _, mu, rs = K.tome_merge_seqnorm_fwd(x, s0, t, r, unm, src, dst, gamma, beta, 1e-6)
    bad_pos1 = pos1.clone()
    bad_pos1[:, 0] = 1 << 29
    dy = torch.randn((n, L - r, D), generator=g).bfloat16().to(dev)
    dgam, dbet = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    expect("pos_map", lambda: K.ln_unmerge_dropout_bwd(dy, x1, mu, rs, gamma, dgam, dbet, None,
                                                       (s0, t, r, bad_pos1, None, so1), None, 0, 1,
                                                       1.0, 0))
    rows = torch.tensor([[0, 3, L + 100], [1, -1, 2], [0, 0, 0], [5, 6, 7]], dtype=torch.int32, device=dev)
    expect("row index", lambda: K.gather_rows(x, rows))
    expect("row index", lambda: K.topk_scatter_bwd(torch.randn((n, 3, D), device=dev), rows, L))
    # the context survived: a valid merge is still bit-exact against the oracle, status clean
    cu, cs, cd = (a.cpu().numpy() for a in (unm, src, dst))
    xc = x.cpu().numpy()
    ref, _ = O.canon_merge_wavg(xc[:, s0:s0 + t], np.ones((n, t), np.float32), cu, cs, cd, r, 0)
    xo2, _, _ = K.tome_merge_fwd(x, s0, t, r, unm, src, dst)
    K.device_status()
    np.testing.assert_array_equal(xo2[:, s0:s0 + t - r].cpu().numpy().view(np.uint32), ref.view(np.uint32))
