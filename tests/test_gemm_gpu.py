"""GPU numerics: MFMA bf16 GEMM (all operand layouts, tails, epilogues) vs a torch fp32 reference
of the same bf16 inputs. Tolerance: fp32 accumulation order only (products of bf16 are exact in
fp32) -> rel 1e-5 before the bf16 output rounding; bf16 outputs compared to 1 bf16 ulp."""
import numpy as np
import pytest
import torch

from oracle import rng as R

pytestmark = pytest.mark.gpu


def _mk(shape, dev, g):
    return torch.randn(shape, generator=g).to(torch.bfloat16).to(dev)


def _ref(a, b, ta, tb):
    A = a.float().t() if ta else a.float()
    B = b.float().t() if tb else b.float()
    return A @ B


def _close_bf16(out, ref):
    ref_b = ref.to(torch.bfloat16).float()
    err = (out.float() - ref).abs()
    tol = (ref.abs() * 2 ** -7) + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item()}"
    # most elements round identically
    assert (out.float() == ref_b).float().mean().item() > 0.97


SHAPES = [(128, 128, 64), (256, 384, 384), (300, 200, 136), (18688 // 8, 1152, 384), (64, 8, 776),
          (33, 1536, 72), (1, 8, 8)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_layouts(dev, M, N, K, ta, tb):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K + ta * 2 + tb)
    if (ta and M % 8) or (not tb and N % 8) or (not ta and K % 8) or (tb and K % 8):
        pytest.skip("contiguous dim must be a multiple of 8")
    a = _mk((K, M) if ta else (M, K), dev, g)
    b = _mk((N, K) if tb else (K, N), dev, g)
    out = Kn.gemm(a, b, ta, tb)
    ref = _ref(a, b, ta, tb)
    _close_bf16(out, ref)
    out32 = Kn.gemm(a, b, ta, tb, out_mode=Kn.OUT_F32)
    torch.testing.assert_close(out32, ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


def test_gemm_epilogue_bias_relu_dropout_residual(dev):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(1)
    M, N, K = 300, 256, 192
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    res = _mk((M, N), dev, g)
    rng = torch.tensor([1234, 7], dtype=torch.int32, device=dev)
    out = Kn.gemm(a, w, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=3,
                  drop_site=2, keep_prob=0.9, drop_row_offset=5 * M, residual=res)
    keep = torch.from_numpy(R.dropout_mask_2d(1234, 7, 3, 2, M, N, 5 * M, 0.9)).to(dev)
    ref = torch.relu(a.float() @ w.float().t() + bias)
    ref = torch.where(keep, ref / 0.9, torch.zeros_like(ref)) + res.float()
    _close_bf16(out, ref)
    frac = keep.float().mean().item()
    assert 0.88 < frac < 0.92


def test_gemm_gate_and_beta_and_atomic_splitk(dev):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(2)
    M, N, K = 200, 128, 512
    a, b = _mk((M, K), dev, g), _mk((K, N), dev, g)
    gate = _mk((M, N), dev, g)
    out = Kn.gemm(a, b, False, False, gate=gate, gate_scale=1 / 0.9)
    ref = (a.float() @ b.float()) * (gate.float() > 0).float() / 0.9
    _close_bf16(out, ref)
    c = torch.randn(M, N, generator=g).to(dev)
    c0 = c.clone()
    Kn.gemm(a, b, out=c, out_mode=Kn.OUT_F32, beta=1.0)
    torch.testing.assert_close(c, c0 + a.float() @ b.float(), rtol=1e-5, atol=1e-3)
    # dW-style: A^T . B with split-K atomics over a long reduction
    x, dy = _mk((4096, 96), dev, g), _mk((4096, 160), dev, g)
    dw = torch.zeros(160, 96, device=dev)
    Kn.gemm(dy, x, trans_a=True, out=dw, out_mode=Kn.OUT_F32_ACCUM, split_k=8)
    ref = dy.float().t() @ x.float()
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,N,K", [(1536, 384, 16384), (1152, 384, 9997), (384, 1536, 12288),
                                   (640, 200, 30000), (384, 384, 20480)])
def test_gemm_tn_splitk_weight_gradient(dev, M, N, K):
    """The step's weight-gradient launches (TN, fp32 split-K slabs + combine, C += A^T B): the
    direct-to-LDS TN kernel at full and partial M / N tiles and a partial last K-step."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    from multi_modal_transformers_tokenmerge_amd.layers import split_k_for
    g = torch.Generator().manual_seed(M + N + K)
    dy, x = _mk((K, M), dev, g), _mk((K, N), dev, g)
    dw = torch.randn(M, N, generator=g).to(dev)
    ref = dw + dy.float().t() @ x.float()
    Kn.gemm(dy, x, trans_a=True, out=dw, out_mode=Kn.OUT_F32_ACCUM, split_k=split_k_for(M, N, K))
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


def test_gemm_rejects_bad_shapes(dev):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn, _C
    a = torch.zeros((16, 12), dtype=torch.bfloat16, device=dev)
    b = torch.zeros((12, 16), dtype=torch.bfloat16, device=dev)
    with pytest.raises(_C.MMTError):
        Kn.gemm(a, b)  # K = 12 not a multiple of 8


@pytest.mark.parametrize("split", [2, 3, 5])
def test_gemm_splitk_applies_epilogue(dev, split):
    """Split-K slabs + combine kernel: bias / relu / dropout / residual (bf16 out) and gate."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(10 + split)
    M, N, K = 200, 256, 1024
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    res = torch.randn((M, N), generator=g).to(dev)
    rng = torch.tensor([99, 3], dtype=torch.int32, device=dev)
    out = Kn.gemm(a, w, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=1,
                  drop_site=3, keep_prob=0.8, drop_row_offset=7, residual=res, split_k=split)
    keep = torch.from_numpy(R.dropout_mask_2d(99, 3, 1, 3, M, N, 7, 0.8)).to(dev)
    ref = torch.relu(a.float() @ w.float().t() + bias)
    ref = torch.where(keep, ref / 0.8, torch.zeros_like(ref)) + res
    _close_bf16(out, ref)
    gate = _mk((M, N), dev, g)
    b2 = _mk((K, N), dev, g)
    o2 = Kn.gemm(a, b2, gate=gate, gate_scale=2.0, split_k=split, out_mode=Kn.OUT_F32)
    ref2 = (a.float() @ b2.float()) * (gate.float() > 0).float() * 2.0
    torch.testing.assert_close(o2, ref2, rtol=1e-4, atol=1e-3)


def test_auto_split_small_m(dev):
    """T5-like projection (M = 2048, N = 768): auto split-K path vs the unsplit kernel."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    assert Kn.auto_split_k(2048, 768, 3072) > 1 and Kn.auto_split_k(17664, 1536, 384) == 1
    g = torch.Generator().manual_seed(5)
    a, w = _mk((2048, 3072), dev, g), _mk((768, 3072), dev, g)
    res = _mk((2048, 768), dev, g)
    o_auto = Kn.gemm(a, w, trans_b=True, residual=res)
    o_one = Kn.gemm(a, w, trans_b=True, residual=res, split_k=1)
    ref = a.float() @ w.float().t() + res.float()
    _close_bf16(o_auto, ref)
    _close_bf16(o_one, ref)


def test_t5_relu_product(dev):
    """The frozen T5's FF input relu(x W_i^T) (t5_base.py) on libmmt_hip against fp32 torch."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    M, N, K = 8192, 3072, 768
    g = torch.Generator().manual_seed(5)
    a, b = _mk((M, K), dev, g), _mk((N, K), dev, g)
    ref = torch.relu(a.float() @ b.float().t())
    _close_bf16(Kn.gemm(a, b, False, True, act=Kn.ACT_RELU), ref)


@pytest.mark.parametrize("M,N,K,ep,variant", [
    (8200, 384, 1536, "none", -1), (138496, 384, 1536, "none", -1), (8192, 768, 3072, "res", -1),
    (9000, 3072, 768, "relu", -1), (300, 384, 128, "none", 8), (70, 768, 64, "res", 8),
    (1000, 1152, 192, "relu", 8)])
def test_narrow_nt_kernel(dev, M, N, K, ep, variant):
    """gemm_ntw_kernel (the products formerly on hipBLASLt: N <= 768 over K >= 1152, the T5 relu
    product; variant 8 forces it on any N % 192 == 0, K % 64 == 0 launch): ragged row counts,
    the two-launch plan (full rounds of 256-row tiles + one round of smaller tiles at M = 138,496),
    residual and relu epilogues, against fp32 torch on the same bf16 operands."""
    from multi_modal_transformers_tokenmerge_amd import _C
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M + N + K)
    a, b = _mk((M, K), dev, g), _mk((N, K), dev, g)
    r = _mk((M, N), dev, g) if ep == "res" else None
    act = Kn.ACT_RELU if ep == "relu" else Kn.ACT_NONE
    _C.call("mmt_gemm_set_variant", variant)
    try:
        out = Kn.gemm(a, b, False, True, residual=r, act=act)
        torch.cuda.synchronize()
    finally:
        _C.call("mmt_gemm_set_variant", -1)
    ref = a.float() @ b.float().t() + (r.float() if r is not None else 0.0)
    if ep == "relu":
        ref = ref.clamp_min(0)
    _close_bf16(out, ref)


@pytest.mark.parametrize("M,N,K,alpha", [(141312, 384, 1536, 1.0), (149504, 384, 384, 1.0),
                                         (8200, 384, 384, 0.5), (4100, 768, 128, 1.0),
                                         (5000, 384, 64, 1.0)])
def test_residual_stream_kernel(dev, M, N, K, alpha):
    """The residual-stream products as the step runs them (fp32 C = fp32 residual + dropout(alpha
    A.W^T + bias): the out-projection and MLP Dense_1, reference attention.py:36-37,59-63, on the
    128 x 128 direct-to-LDS kernel) at the B = 512 block-0 shapes, ragged rows and one-K-step
    reductions: the dropout keeps are the shared counter stream's (oracle/rng.py), the sum within
    fp32 accumulation order of a torch reference. (Round 4's warp-specialised kernel for these
    products measured slower and was deleted in round 6.)"""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M + N + K)
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = torch.randn(N, generator=g).to(dev)
    res = torch.randn((M, N), generator=g).to(dev)
    rng = torch.tensor([31, 4], dtype=torch.int32, device=dev)
    kw = dict(bias=bias, rng=rng, drop_layer=2, drop_site=3, keep_prob=0.9, drop_row_offset=3 * M,
              residual=res, alpha=alpha, out_mode=Kn.OUT_F32)
    out = Kn.gemm(a, w, False, True, **kw)
    torch.cuda.synchronize()
    keep = torch.from_numpy(R.dropout_mask_2d(31, 4, 2, 3, M, N, 3 * M, 0.9)).to(dev)
    ref = alpha * (a.float() @ w.float().t()) + bias
    ref = torch.where(keep, ref / 0.9, torch.zeros_like(ref)) + res
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,N,bias", [(149504, 1152, True), (141312, 1536, False), (33001, 192, True),
                                      (40000, 64, False), (700, 1536, True)])
def test_activation_stationary_kernel(dev, M, N, bias):
    """gemm_xs_kernel (csrc/gemm_xs.hip: K = 384 products with a bias-only epilogue, the step's QKV
    projection, reference attention.py:41-69 Dense): the same fp32 sums in the same k order as the
    128 x 128 kernel (variant 4), so bit-identical bf16 outputs — at the B = 512 shapes, ragged
    row panels (rows past M neither read nor stored), one-chunk N and M below the dispatch floor
    (mmt_gemm_xs called directly); and within bf16 rounding of a torch fp32 reference."""
    from multi_modal_transformers_tokenmerge_amd import _C
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M + N)
    K = 384
    a, w = _mk((M, K), dev, g), _mk((N, K), dev, g)
    b = torch.randn(N, generator=g).to(dev) if bias else None
    out = torch.full((M + 3, N), 7.0, dtype=torch.bfloat16, device=dev)  # rows past M: untouched
    _C.call("mmt_gemm_xs", M, N, K, a.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N,
            None if b is None else b.data_ptr(), _C.stream_ptr())
    _C.call("mmt_gemm_set_variant", 4)
    try:
        old = Kn.gemm(a, w, False, True, bias=b)
    finally:
        _C.call("mmt_gemm_set_variant", -1)
    disp = Kn.gemm(a, w, False, True, bias=b)  # mmt_gemm's own dispatch (XS where it applies)
    torch.cuda.synchronize()
    assert torch.equal(out[:M], old) and torch.equal(disp, old)
    assert bool((out[M:] == 7.0).all())
    ref = a.float() @ w.float().t() + (b if b is not None else 0.0)
    _close_bf16(out[:M], ref)


@pytest.mark.parametrize("M,row_off", [(141312, 0), (33001, 7 * 33001)])
def test_activation_stationary_relu_bits(dev, M, row_off):
    """The step's MLP up-projection on gemm_xs_kernel<bf16, RB> (reference attention.py:20-39
    MLPBlock: Dense_0 + bias, relu, dropout; mmt_gemm's own dispatch) against gemm_nt256_kernel
    forced by variant 5: bf16 output AND the relu-bit image (include/mmt_api.h layout, every word
    including the padded rows of the last 256-row panel) bit-identical; the image equals
    (stored h > 0)."""
    from multi_modal_transformers_tokenmerge_amd import _C
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    from tests.test_gemm_nt256_gpu import _bits_to_mask
    N, K = 1536, 384
    g = torch.Generator().manual_seed(M + 5)
    y, w1 = _mk((M, K), dev, g), _mk((N, K), dev, g)
    bias = (torch.randn(N, generator=g) * 0.5).to(dev)
    rng = torch.tensor([13, 6], dtype=torch.int32, device=dev)
    rows = -(-M // 256) * 256
    outs = []
    for v in (-1, 5):
        bits = torch.full((rows, N // 32), -1, dtype=torch.int32, device=dev)
        _C.call("mmt_gemm_set_variant", v)
        try:
            h = Kn.gemm(y, w1, False, True, bias=bias, act=Kn.ACT_RELU, rng=rng, drop_layer=3,
                        drop_site=2, keep_prob=0.9, drop_row_offset=row_off, relu_bits=bits)
        finally:
            _C.call("mmt_gemm_set_variant", -1)
        outs.append((h, bits))
    torch.cuda.synchronize()
    (h1, b1), (h2, b2) = outs
    assert torch.equal(h1, h2)
    assert torch.equal(b1, b2)
    torch.testing.assert_close(_bits_to_mask(b1, M, N), h1.float() > 0, rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K,split", [(1536, 384, 16384, 8), (1152, 384, 9997, 3),
                                         (384, 1536, 12288, 5), (640, 200, 30000, 7),
                                         (384, 384, 20480, 16), (1536, 384, 141312, 32),
                                         (384, 384, 1040, 4), (768, 192, 48, 1)])
def test_tn_kernels_bit_identical(dev, M, N, K, split):
    """The TN weight-gradient kernels: the two-stage kernel on 32x32x16 MFMAs (variant 10), on
    16x16x32 (13, the default) and the four-stage ring of 32-row K-steps (18, the default for
    K chunks of at most 2,048 rows) — at the step's shapes (384-row tiles), partial M tiles
    (256-row tiles), partial N tiles, ragged K, K chunks shorter than the ring and a split with a
    single K-step; 13 and 18 share the per-k32 MFMA order (bit-identical), 10 groups k by 16
    (fp32 rounding apart); all match an fp32 reference."""
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn, _C
    g = torch.Generator().manual_seed(M * 7 + N + K)
    dy, x = _mk((K, M), dev, g), _mk((K, N), dev, g)
    outs = {}
    try:
        for v in (10, 13, 18):
            _C.call("mmt_gemm_set_variant", v)
            dw = torch.zeros(M, N, device=dev)
            Kn.gemm(dy, x, trans_a=True, out=dw, out_mode=Kn.OUT_F32_ACCUM, split_k=split)
            torch.cuda.synchronize()
            outs[v] = dw
    finally:
        _C.call("mmt_gemm_set_variant", -1)
    ref = dy.float().t() @ x.float()
    for v in (10, 13):
        torch.testing.assert_close(outs[v], ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
    assert torch.equal(outs[18], outs[13])
