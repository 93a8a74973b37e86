"""GPU numerics of the persistent 256 x BN NT GEMM (gemm_nt256_kernel) for each tile width, with
partial last row tiles, several tiles per workgroup (persistent walk) and every epilogue, against
a torch fp32 reference of the same bf16 operands (same bars as tests/test_gemm_gpu.py)."""
import os

import pytest
import torch

from oracle import rng as R

pytestmark = pytest.mark.gpu

VARIANTS = {256: 5, 192: 6, 128: 7}


def _mk(shape, dev, g):
    return torch.randn(shape, generator=g).to(torch.bfloat16).to(dev)


def _close_bf16(out, ref):
    err = (out.float() - ref).abs()
    tol = (ref.abs() * 2 ** -7) + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item()}"
    assert (out.float() == ref.to(torch.bfloat16).float()).float().mean().item() > 0.97


@pytest.fixture
def variant():
    from multi_modal_transformers_tokenmerge_amd import _C
    yield lambda bn: _C.call("mmt_gemm_set_variant", VARIANTS[bn])
    _C.call("mmt_gemm_set_variant", -1)


# (M, K): partial last tile, one tile, many tiles per workgroup (> 256 tiles), long K
@pytest.mark.parametrize("bn", [256, 192, 128])
@pytest.mark.parametrize("M,K", [(300, 64), (256, 384), (70000, 128), (1000, 1536)])
def test_nt256_plain(dev, variant, bn, M, K):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    variant(bn)
    N = 2 * bn if M < 5000 else bn * 3
    g = torch.Generator().manual_seed(M + K + bn)
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    ref = a.float() @ w.float().t()
    out = Kn.gemm(a, w, False, True, split_k=1)
    _close_bf16(out, ref)
    out32 = Kn.gemm(a, w, False, True, out_mode=Kn.OUT_F32, split_k=1)
    torch.testing.assert_close(out32, ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


@pytest.mark.parametrize("bn", [256, 192, 128])
def test_nt256_epilogues(dev, variant, bn):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    variant(bn)
    g = torch.Generator().manual_seed(bn)
    M, N, K = 1300, 2 * bn * 3, 192
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    rng = torch.tensor([1234, 7], dtype=torch.int32, device=dev)
    keep = torch.from_numpy(R.dropout_mask_2d(1234, 7, 3, 2, M, N, 5 * M, 0.9)).to(dev)
    base = a.float() @ w.float().t()
    # bias + relu + dropout + bf16 residual, bf16 out
    res = _mk((M, N), dev, g)
    out = Kn.gemm(a, w, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=3,
                  drop_site=2, keep_prob=0.9, drop_row_offset=5 * M, residual=res, split_k=1)
    ref = torch.where(keep, torch.relu(base + bias) / 0.9, torch.zeros_like(base)) + res.float()
    _close_bf16(out, ref)
    # dropout + fp32 residual, fp32 out (the residual-stream projections)
    res32 = torch.randn((M, N), generator=g).to(dev)
    out = Kn.gemm(a, w, False, True, bias=bias, rng=rng, drop_layer=3, drop_site=2,
                  keep_prob=0.9, drop_row_offset=5 * M, residual=res32, out_mode=Kn.OUT_F32,
                  split_k=1)
    ref = torch.where(keep, (base + bias) / 0.9, torch.zeros_like(base)) + res32
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    # gate (relu-backward mask) and fp32 accumulate (beta = 1)
    gate = _mk((M, N), dev, g)
    out = Kn.gemm(a, w, False, True, gate=gate, gate_scale=1 / 0.9, split_k=1)
    _close_bf16(out, base * (gate.float() > 0).float() / 0.9)
    c = torch.randn((M, N), generator=g).to(dev)
    c0 = c.clone()
    Kn.gemm(a, w, False, True, out=c, out_mode=Kn.OUT_F32, beta=1.0, split_k=1)
    torch.testing.assert_close(c, c0 + base, rtol=1e-5, atol=1e-3)


def test_nt256_auto_matches_reference_path(dev):
    """Auto choice at a step shape (MLP up-projection, B = 64) vs the 128 x 128 glds kernel."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn, _C
    g = torch.Generator().manual_seed(3)
    M, N, K = 64 * 276, 1536, 384
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    o_new = Kn.gemm(a, w, False, True, bias=bias, act=Kn.ACT_RELU, split_k=1)
    _C.call("mmt_gemm_set_variant", 4)
    try:
        o_old = Kn.gemm(a, w, False, True, bias=bias, act=Kn.ACT_RELU, split_k=1)
    finally:
        _C.call("mmt_gemm_set_variant", -1)
    # identical accumulation order is not guaranteed across kernels: compare within 1 bf16 ulp
    _close_bf16(o_new, torch.relu(a.float() @ w.float().t() + bias))
    assert ((o_new.float() - o_old.float()).abs() <= o_old.float().abs() * 2 ** -7 + 1e-6).all()


@pytest.mark.parametrize("M", [300, 70656])
def test_nt256_colsum_slab(dev, variant, M):
    """gemm(..., colsum=slab) on the gated dX shape (N = 1536, K = 384): the slab rows are the
    column sums of each 256-row panel of the bf16 output exactly as stored (fp32 sums of bf16
    values; summation order differs from torch's), the output itself unchanged."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M)
    N, K = 1536, 384
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    gate = _mk((M, N), dev, g)
    if M < 5000:  # too few tiles for the automatic choice of the 256-wide kernel: force it
        assert Kn.gemm_colsum_rows(M, N, K) == 0
        variant(256)
    rows = Kn.gemm_colsum_rows(M, N, K)
    assert rows == (M + 255) // 256
    slab = torch.full((rows, N), float("nan"), dtype=torch.float32, device=dev)
    out = Kn.gemm(a, w, False, True, gate=gate, gate_scale=1.25, colsum=slab)
    plain = Kn.gemm(a, w, False, True, gate=gate, gate_scale=1.25)
    assert torch.equal(out, plain)
    pad = torch.zeros((rows * 256, N), dtype=torch.float64, device=dev)
    pad[:M] = out.double()
    want = pad.view(rows, 256, N).sum(1)
    torch.testing.assert_close(slab.double(), want, rtol=1e-5, atol=1e-4 * want.abs().max().item())
    # shapes the 256-wide kernel does not take report 0 rows and reject a slab
    assert Kn.gemm_colsum_rows(M, 384, K) == 0 and Kn.gemm_colsum_rows(M, N, K, out_mode=Kn.OUT_F32) == 0
    with pytest.raises(ValueError):
        Kn.gemm(a, w[:384], False, True, colsum=torch.zeros((rows, 384), device=dev))


def _bits_to_mask(bits, M, N):
    """Expand relu_bits / gate_bits (include/mmt_api.h layout) to an (M, N) bool mask."""
    m = torch.arange(M, device=bits.device)
    g = (m // 256) * 64 + ((m // 64) & 3) * 16 + (m & 15)
    f = (m // 16) & 3
    words = bits.view(-1, N // 32, 4)[g, :, f].to(torch.int64) & 0xFFFFFFFF  # (M, N/32)
    wi = torch.arange(N // 32, device=bits.device)
    c = torch.arange(4, device=bits.device)
    e = torch.arange(8, device=bits.device)
    col = ((256 * (wi // 8) + 128 * ((wi // 4) & 1) + 8 * (wi & 3))[:, None, None]
           + 32 * c[None, :, None] + e[None, None, :])
    bit = (8 * c[:, None] + e[None, :])[None, None]                 # (1, 1, 4, 8)
    val = (words[:, :, None, None] >> bit) & 1                       # (M, N/32, 4, 8)
    mask = torch.zeros((M, N), dtype=torch.bool, device=bits.device)
    mask[:, col.reshape(-1)] = val.reshape(M, -1).bool()
    return mask


@pytest.mark.parametrize("M", [11264, 11000])
def test_relu_bits_and_gate_bits(dev, M):
    """MLP hidden layer in 1-bit form: the forward's relu_bits equal (stored h > 0) under the
    documented layout, and the gated input gradient from gate_bits is bit-identical (values and
    epilogue column sums) to the one gated by h itself."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    N, K = 1536, 384
    assert Kn.gemm_bits_supported(M, N, K)
    g = torch.Generator().manual_seed(M)
    y, w1 = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = (torch.randn(N, generator=g) * 0.5).to(dev)
    rng = torch.tensor([11, 3], dtype=torch.int32, device=dev)
    bits = torch.empty((-(-M // 256) * 256, N // 32), dtype=torch.int32, device=dev)
    h = Kn.gemm(y, w1, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=1, drop_site=2,
                keep_prob=0.9, relu_bits=bits)
    h_ref = Kn.gemm(y, w1, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=1,
                    drop_site=2, keep_prob=0.9)
    assert torch.equal(h, h_ref)
    torch.testing.assert_close(_bits_to_mask(bits, M, N), h.float() > 0, rtol=0, atol=0)
    dz2, w2t = _mk((M, K), dev, g), _mk((N, K), dev, g)  # dX of a Dense with W2^T (N, K)
    rows = Kn.gemm_colsum_rows(M, N, K)
    cs_a = torch.empty((rows, N), device=dev)
    cs_b = torch.empty((rows, N), device=dev)
    d_a = Kn.gemm(dz2, w2t, False, True, gate=h, gate_scale=1 / 0.9, colsum=cs_a)
    d_b = Kn.gemm(dz2, w2t, False, True, gate_bits=bits, gate_scale=1 / 0.9, colsum=cs_b)
    assert torch.equal(d_a, d_b)
    assert torch.equal(cs_a, cs_b)
    d_c = Kn.gemm(dz2, w2t, False, True, gate_bits=bits, gate_scale=1 / 0.9)  # no column sums
    assert torch.equal(d_a, d_c)


@pytest.mark.parametrize("M,row_off", [(11264, 0), (11000, 7 * 11000), (149504, 512 * 292)])
def test_keep_bits_match_epilogue_draws(dev, M, row_off):
    """MLP hidden dropout from precomputed keep bits (gemm_dropout_keep_bits + keep_bits=): the
    words equal the oracle's counter-RNG keeps (oracle/rng.py) under the relu_bits layout, and the
    MLP-up output and its relu_bits are bit-identical to the epilogue-draw launch."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    N, K = 1536, 384
    g = torch.Generator().manual_seed(M + 1)
    y, w1 = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = (torch.randn(N, generator=g) * 0.5).to(dev)
    rng = torch.tensor([21, 5], dtype=torch.int32, device=dev)
    kb = Kn.gemm_dropout_keep_bits(rng, 4, 2, M, N, 0.9, row_off)
    if M <= 12000:  # the oracle's mask (numpy) at the small sizes
        keep = torch.from_numpy(R.dropout_mask_2d(21, 5, 4, 2, M, N, row_off, 0.9)).to(dev)
        assert torch.equal(_bits_to_mask(kb, M, N), keep)
    rows = -(-M // 256) * 256
    b1 = torch.empty((rows, N // 32), dtype=torch.int32, device=dev)
    b2 = torch.empty_like(b1)
    h1 = Kn.gemm(y, w1, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=4, drop_site=2,
                 keep_prob=0.9, drop_row_offset=row_off, relu_bits=b1)
    h2 = Kn.gemm(y, w1, False, True, bias=bias, act=Kn.ACT_RELU, keep_bits=kb, keep_prob=0.9,
                 relu_bits=b2)
    assert torch.equal(h1, h2)
    assert torch.equal(b1, b2)
    with pytest.raises(ValueError):  # keep_bits replaces rng, only in a relu_bits launch
        Kn.gemm(y, w1, False, True, keep_bits=kb, keep_prob=0.9)


def test_bits_rejected_off_the_256_path(dev):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    M, N, K = 300, 1536, 384
    assert not Kn.gemm_bits_supported(M, N, K)
    a, w = torch.zeros((M, K), dtype=torch.bfloat16, device=dev), torch.zeros((N, K), dtype=torch.bfloat16, device=dev)
    with pytest.raises(ValueError):
        Kn.gemm(a, w, False, True, relu_bits=torch.empty((512, N // 32), dtype=torch.int32, device=dev))


@pytest.mark.parametrize("M,N,K", [(4133, 1536, 384), (70656, 1536, 384), (9000, 1152, 384),
                                   (5000, 1024, 1536)])
def test_ntws_matches_nt256(dev, M, N, K):
    """The warp-specialised wide NT kernel (gemm_ntws_kernel, the automatic choice for these bf16
    products) against gemm_nt256_kernel forced by variant 5 / 6 (BN 256 / 192): the same MFMA
    order per output element, so every epilogue the step uses must agree bit for bit — outputs,
    relu_bits and the per-256-row column-sum slab."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn, _C
    if N % 256 == 0 and os.environ.get("MMT_NTWS", "1") != "2":
        pytest.skip("the warp-specialised kernel takes N % 256 == 0 only with MMT_NTWS=2")
    g = torch.Generator().manual_seed(M + N + K)
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    rng = torch.tensor([99, 4], dtype=torch.int32, device=dev)
    rows = -(-M // 256)
    ref_variant = 5 if N % 256 == 0 else 6

    def both(**kw):
        bits_ = kw.pop("bits", None)
        cs_ = kw.pop("cs", None)
        outs = []
        for v in (-1, ref_variant):
            _C.call("mmt_gemm_set_variant", v)
            try:
                extra = {}
                if bits_ is not None:
                    extra["relu_bits"] = torch.full_like(bits_, -1)
                if cs_ is not None:
                    extra["colsum"] = torch.full((rows, N), float("nan"), device=dev)
                o = Kn.gemm(a, w, False, True, split_k=1, **kw, **extra)
                outs.append((o, extra))
            finally:
                _C.call("mmt_gemm_set_variant", -1)
        return outs

    (o1, _), (o2, _) = both()
    assert torch.equal(o1, o2)
    _close_bf16(o1, a.float() @ w.float().t())
    (o1, _), (o2, _) = both(bias=bias)
    assert torch.equal(o1, o2)
    if N % 256 == 0 and Kn.gemm_bits_supported(M, N, K):  # relu_bits / gate_bits / colsum
        bits = torch.empty((rows * 256, N // 32), dtype=torch.int32, device=dev)
        (o1, e1), (o2, e2) = both(bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=2, drop_site=2,
                                  keep_prob=0.9, drop_row_offset=3 * M, bits=bits)
        assert torch.equal(o1, o2)
        assert torch.equal(e1["relu_bits"], e2["relu_bits"])  # every word written
        gbits = e1["relu_bits"]
        (o1, e1), (o2, e2) = both(gate_bits=gbits, gate_scale=1 / 0.9, cs=True)
        assert torch.equal(o1, o2)
        assert torch.equal(e1["colsum"], e2["colsum"])
