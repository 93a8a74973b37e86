"""GPU: the fp8 weight path of BASELINE configs[4] (OCP e4m3 forward products, csrc/gemm.hip):
* row quantisation bit-exact vs torch's float8_e4m3fn cast of x / (amax / 448);
* the MX-fp8 GEMM vs an fp32 product of the same dequantised operands (fp8 x fp8 products are
  exact in fp32, only the summation order differs: relative L2 <= 5e-5, measured 1.5e-5), with
  epilogues;
* the fp8 Dense shadow is refreshed from the bf16 shadow by AdamW's step.
The end-to-end bar (cosine >= 0.995) is test_octo_gpu.py::test_blockwise_base_hires_tome32
(the oracle emulates the same quantisation, so it holds far tighter)."""
import pytest
import torch

from oracle.octo_ref import quant_rows_e4m3

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,K", [(37, 768), (300, 3072), (8, 64)])
def test_quant_rows_bit_exact(dev, R, K):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(R + K)
    x = (torch.randn((R, K), generator=g) * torch.logspace(-3, 2, R)[:, None]).bfloat16()
    x[0] = 0  # zero row -> scale 1
    q, s = Kn.quant_rows_fp8(x.to(dev))
    torch.cuda.synchronize()
    rq, rs = quant_rows_e4m3(x.float())
    assert torch.equal(s.cpu(), rs.view(-1))
    assert torch.equal(q.cpu().view(torch.float8_e4m3fn).float(), rq)


@pytest.mark.parametrize("M,N,K,out_mode,epi", [
    (1000, 2304, 768, 0, {}), (517, 768, 3072, 1, {"residual": "f32"}),
    (256, 3072, 768, 0, {"act": 1, "drop": True}), (64, 128, 64, 1, {})])
def test_gemm_fp8(dev, M, N, K, out_mode, epi):
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn((M, K), generator=g).bfloat16()
    w = (torch.randn((N, K), generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, generator=g) * 0.1
    xq, sx = Kn.quant_rows_fp8(x.to(dev))
    wq, sw = Kn.quant_rows_fp8(w.to(dev))
    kw = dict(bias=bias.to(dev))
    res = None
    if epi.get("residual"):
        res = torch.randn((M, N), generator=g)
        kw["residual"] = res.to(dev)
    if epi.get("act"):
        kw["act"] = Kn.ACT_RELU
    if epi.get("drop"):
        kw.update(rng=torch.tensor([3, 4], dtype=torch.int32, device=dev), keep_prob=0.9)
    y = Kn.gemm_fp8(xq, sx, wq, sw, out_mode=out_mode, **kw).float().cpu()
    a = xq.cpu().view(torch.float8_e4m3fn).float()
    b = wq.cpu().view(torch.float8_e4m3fn).float()
    ref = (a @ b.t()) * sx.cpu()[:, None] * sw.cpu()[None, :] + bias
    if epi.get("act"):
        ref = torch.relu(ref)
    if epi.get("drop"):  # compare on the kept entries (the mask is the GEMM epilogue's stream)
        kept = y != 0
        ref = torch.where(kept, ref / 0.9, torch.zeros_like(ref))
    if res is not None:
        ref = ref + res
    tol = 5e-5 if out_mode == 1 else 8e-3   # fp32: summation order; bf16: output rounding
    assert float((y - ref).norm() / ref.norm()) <= tol


def test_fp8_shadow_follows_adamw(dev):
    from multi_modal_transformers_tokenmerge_amd.models.octo.config import get_config
    from multi_modal_transformers_tokenmerge_amd.models.octo import octo as O
    from oracle.parity import _inputs
    cfg = get_config("octo-tiny", num_blocks=1, token_embedding_dim=192, fp8=True)
    model = O.Octo(cfg, dev, seed=0)
    state = O.create_octo_train_state(model, seed=3)
    images, _, actions = _inputs(model, 2)
    O.diffusion_train_step(model, state, None, torch.from_numpy(images).to(dev),
                           torch.from_numpy(actions).to(dev))
    torch.cuda.synchronize()
    p = model.stack.blocks[0].qkv.w
    rq, rs = quant_rows_e4m3(p.bf16.float().cpu())
    assert torch.equal(p.q8.cpu().view(torch.float8_e4m3fn).float(), rq)
    assert torch.equal(p.q8_scale.cpu(), rs.view(-1))


@pytest.mark.parametrize("M,N,epi", [(33920, 3072, {"act": 1, "drop": True}), (33920, 2304, {}),
                                     (4101, 768, {"drop": True})])
def test_fp8_activation_stationary_kernel(dev, M, N, epi):
    """The K = 768 fp8 products on the activation-stationary kernel (csrc/gemm_xs.hip; OCTO-base
    QKV projection and MLP up-projection, configs[4]): the same MX-fp8 MFMAs in the same k order
    and epilogue order as gemm_fp8_nt_kernel (forced with variant 4), so bit-identical bf16
    outputs, dropout draws included; ragged last panel (M % 256 != 0)."""
    from multi_modal_transformers_tokenmerge_amd import _C
    from multi_modal_transformers_tokenmerge_amd import _kernels as Kn
    K = 768
    g = torch.Generator().manual_seed(M + N + 1)
    x = torch.randn((M, K), generator=g).bfloat16()
    w = (torch.randn((N, K), generator=g) / K ** 0.5).bfloat16()
    xq, sx = Kn.quant_rows_fp8(x.to(dev))
    wq, sw = Kn.quant_rows_fp8(w.to(dev))
    kw = dict(bias=(torch.randn(N, generator=g) * 0.1).to(dev))
    if epi.get("act"):
        kw["act"] = Kn.ACT_RELU
    if epi.get("drop"):
        kw.update(rng=torch.tensor([3, 4], dtype=torch.int32, device=dev), keep_prob=0.9,
                  drop_layer=5, drop_site=2, drop_row_offset=17)
    new = Kn.gemm_fp8(xq, sx, wq, sw, **kw)
    _C.call("mmt_gemm_set_variant", 4)
    try:
        old = Kn.gemm_fp8(xq, sx, wq, sw, **kw)
    finally:
        _C.call("mmt_gemm_set_variant", -1)
    torch.cuda.synchronize()
    assert torch.equal(new, old)
