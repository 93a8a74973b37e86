"""Stem and head side kernels vs torch fp32/fp64 references of the same op (same inputs):
GroupNorm+gelu forward/backward (image_tokenizer.py:165-167, gato_resnet.yaml:68-77; both the
register-resident kernels, R*C = NV*1024, and the general one), per-patch max-pool forward/backward
(:159, window 3x3 stride 1 VALID on the conv map) and the FourierFeatures kernel gradient
(diffusion.py:41-48)."""
import math

import numpy as np
import pytest
import torch

from multi_modal_transformers_tokenmerge_amd import _C, _kernels as K

pytestmark = pytest.mark.gpu


def _gelu_tanh(z):
    return 0.5 * z * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (z + 0.044715 * z ** 3)))


def _gn_gelu_ref(x, G, gamma, beta, eps):
    B, R, C = x.shape
    xg = x.view(B, R, G, C // G)
    mu = xg.mean(dim=(1, 3), keepdim=True)
    var = xg.var(dim=(1, 3), unbiased=False, keepdim=True)
    xh = ((xg - mu) / torch.sqrt(var + eps)).view(B, R, C)
    return _gelu_tanh(xh * gamma + beta)


@pytest.mark.parametrize("B,R,C,G", [(5, 256, 64, 32), (3, 64, 64, 32), (2, 100, 64, 32),
                                     (4, 512, 64, 16)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_groupnorm_gelu(dev, B, R, C, G, accumulate):
    g = torch.Generator().manual_seed(R + C)
    x = torch.randn((B, R, C), generator=g) * 2 + 0.5
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn((B, R, C), generator=g)
    prior = torch.randn((B, R, C), generator=g)
    eps = 1e-6
    xd, gd, bd, dyd = x.to(dev), gamma.to(dev), beta.to(dev), dy.to(dev)
    y, mu, rs = K.groupnorm_gelu_fwd(xd.contiguous(), G, gd, bd, eps)
    dgam = torch.zeros(C, device=dev)
    dbet = torch.zeros(C, device=dev)
    dx = prior.to(dev).clone() if accumulate else None
    dx = K.groupnorm_gelu_bwd(dyd, xd, G, gd, bd, mu, rs, dgam, dbet, dx=dx, accumulate=accumulate)
    torch.cuda.synchronize()

    x64 = x.double().requires_grad_()
    g64 = gamma.double().requires_grad_()
    b64 = beta.double().requires_grad_()
    ref = _gn_gelu_ref(x64, G, g64, b64, eps)
    ref.backward(dy.double())
    np.testing.assert_allclose(y.float().cpu().numpy(), ref.detach().numpy(), atol=2e-2, rtol=1e-2)
    want_dx = x64.grad + (prior.double() if accumulate else 0)
    np.testing.assert_allclose(dx.cpu().double().numpy(), want_dx.numpy(), atol=2e-3, rtol=2e-3)
    np.testing.assert_allclose(dgam.cpu().double().numpy(), g64.grad.numpy(), rtol=2e-3, atol=1e-2)
    np.testing.assert_allclose(dbet.cpu().double().numpy(), b64.grad.numpy(), rtol=2e-3, atol=1e-2)


@pytest.mark.parametrize("npatch,win,C", [(37, 9, 64), (8, 4, 16)])
def test_maxpool_patch_fwd_bwd(dev, npatch, win, C):
    g = torch.Generator().manual_seed(npatch)
    conv = torch.randn((npatch * win, C), generator=g)
    conv[:win, :3] = 1.0  # ties: the first maximum wins
    pooled, arg = K.maxpool_patch(conv.to(dev), win)
    dpooled = torch.randn((npatch, C), generator=g)
    G = K.maxpool_patch_bwd(dpooled.to(dev), arg, win)
    torch.cuda.synchronize()
    v = conv.view(npatch, win, C)
    want_arg = torch.argmax((v == v.max(dim=1, keepdim=True).values).int(), dim=1)  # first max
    assert torch.equal(pooled.cpu(), v.max(dim=1).values)
    assert torch.equal(arg.cpu().long(), want_arg)
    want_G = torch.zeros((npatch, win, C))
    want_G.scatter_(1, want_arg.unsqueeze(1), dpooled.unsqueeze(1))
    assert torch.equal(G.cpu().float().view(npatch, win, C), want_G.to(torch.bfloat16).float())


@pytest.mark.parametrize("B,F", [(256, 192), (7, 96)])
def test_fourier_bwd(dev, B, F):
    g = torch.Generator().manual_seed(B)
    dfeats = torch.randn((B, 2 * F), generator=g).to(torch.bfloat16)
    t = torch.randint(0, 32, (B,), generator=g, dtype=torch.int32)
    w = torch.randn(F, generator=g)
    dw = torch.full((F,), 0.25)
    dwd = dw.to(dev)
    dfd, td, wd = dfeats.to(dev), t.to(dev), w.to(dev)  # keep the device copies alive
    _C.call("mmt_fourier_bwd", _C.ptr(dfd), B, F, _C.ptr(td), _C.ptr(wd), _C.ptr(dwd),
            _C.stream_ptr())
    torch.cuda.synchronize()
    tt = 2 * np.pi * t.double().numpy()[:, None]
    h = tt * w.double().numpy()[None, :]
    d = dfeats.double().numpy()
    want = 0.25 + (tt * (np.cos(h) * d[:, F:] - np.sin(h) * d[:, :F])).sum(0)
    np.testing.assert_allclose(dwd.cpu().double().numpy(), want, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("npatch,OH,C", [(3, 23, 64), (4, 5, 16)])
def test_maxpool2d_general(dev, npatch, OH, C):
    """max_pool 3x3 s1 VALID on a larger map (the reference's patch 56: 23x23 -> 21x21) vs torch
    max_pool2d; backward (first-maximum routing, gather over overlapping windows) vs autograd on
    tie-free data, bf16-rounded like the kernel's output."""
    g = torch.Generator().manual_seed(OH)
    x = torch.randn((npatch, OH, OH, C), generator=g)
    y, arg = K.maxpool2d(x.reshape(-1, C).contiguous().to(dev), npatch, OH, OH, 3)
    xt = x.permute(0, 3, 1, 2).clone().requires_grad_()
    ref = torch.nn.functional.max_pool2d(xt, 3, stride=1)
    PH = OH - 2
    torch.testing.assert_close(y.cpu().view(npatch, PH, PH, C), ref.detach().permute(0, 2, 3, 1),
                               rtol=0, atol=0)
    dy = torch.randn((npatch, PH, PH, C), generator=g)
    ref.backward(dy.permute(0, 3, 1, 2))
    G = K.maxpool2d_bwd(dy.reshape(-1, C).contiguous().to(dev), arg, npatch, OH, OH, 3)
    want = xt.grad.permute(0, 2, 3, 1).reshape(-1, C)
    torch.testing.assert_close(G.float().cpu(), want.bfloat16().float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("npatch,H,C", [(2, 21, 64), (3, 4, 16)])
def test_same_conv_im2col_col2im(dev, npatch, H, C):
    """3x3 SAME conv as im2col + GEMM vs torch conv2d(padding=1), and col2im as the adjoint of
    im2col (<im2col(x), c> == <x, col2im(c)>) in fp32."""
    g = torch.Generator().manual_seed(H)
    x = torch.randn((npatch, H, H, C), generator=g).bfloat16()
    w = torch.randn((C, 3, 3, C), generator=g) * 0.05          # (out, ky, kx, in)
    cols = K.im2col_same(x.reshape(-1, C).contiguous().to(dev), npatch, H, H, 3)
    y = cols.float() @ w.reshape(C, 9 * C).t().to(dev)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=1)
    torch.testing.assert_close(y.cpu().view(npatch, H, H, C), ref.permute(0, 2, 3, 1), rtol=1e-4, atol=1e-4)
    c = torch.randn((npatch * H * H, 9 * C), generator=g)
    dx = K.col2im_same(c.to(dev), npatch, H, H, C, 3)
    lhs = float((cols.float().cpu().double() * c.double()).sum())
    rhs = float((x.float().reshape(-1, C).double() * dx.cpu().double()).sum())
    assert abs(lhs - rhs) <= 1e-6 * max(1.0, abs(lhs)), (lhs, rhs)


@pytest.mark.parametrize("B,I,H,P,Q,D", [(64, 1, 256, 16, 128, 384), (5, 2, 256, 16, 128, 768),
                                         (3, 1, 128, 16, 256, 192), (4, 1, 64, 8, 256, 64)])
def test_patch_embed_grad(dev, B, I, H, P, Q, D):
    """Image row / column position-embedding gradients by token window (mmt_patch_embed_grad;
    windows of 8 and 16 tokens and the wide-window fallback at 32) against a float64 index_add
    over the training-mode tokens, and against the LDS-histogram form of mmt_seq_assemble_bwd."""
    rng = torch.tensor([11, 3], dtype=torch.int32, device=dev)
    rt, ct = K.patch_positions(B, I, H, P, Q, True, rng)
    NP = (H // P) ** 2
    NI = I * NP
    L = NI + 7
    g = torch.Generator().manual_seed(B + D)
    img_rows = torch.randperm(L, generator=g)[:NI].to(torch.int32).to(dev)
    dx0 = torch.randn((B, L, D), generator=g).to(dev)
    drow = torch.zeros((Q, D), device=dev)
    dcol = torch.zeros((Q, D), device=dev)
    _C.call("mmt_patch_embed_grad", B, L, D, I, H, P, Q, _C.ptr(img_rows), _C.ptr(dx0), _C.ptr(rt),
            _C.ptr(ct), _C.ptr(drow), _C.ptr(dcol), _C.stream_ptr())
    rows = dx0[:, img_rows.long()].double().reshape(B * NI, D)
    want_r = torch.zeros((Q, D), dtype=torch.float64, device=dev).index_add_(0, rt.reshape(-1).long(), rows)
    want_c = torch.zeros((Q, D), dtype=torch.float64, device=dev).index_add_(0, ct.reshape(-1).long(), rows)
    for got, want in ((drow, want_r), (dcol, want_c)):
        torch.testing.assert_close(got.double(), want, rtol=1e-5, atol=1e-4)
    # the LDS-histogram form (seq_assemble_bwd with tables) agrees
    row_src = torch.zeros(L, dtype=torch.int32)
    row_src[img_rows.cpu().long()] = (1 << 24) | torch.arange(NI, dtype=torch.int32)
    row_src = row_src.to(dev)
    dimg = torch.empty((B, NI, D), dtype=torch.bfloat16, device=dev)
    hr, hc, pe = torch.zeros((Q, D), device=dev), torch.zeros((Q, D), device=dev), torch.zeros((1, D), device=dev)
    _C.call("mmt_seq_assemble_bwd", B, L, D, _C.ptr(row_src), _C.ptr(dx0), None, 0, _C.ptr(dimg),
            NI, _C.ptr(rt), _C.ptr(ct), _C.ptr(img_rows), Q, _C.ptr(hr), _C.ptr(hc), _C.ptr(pe),
            _C.stream_ptr())
    torch.testing.assert_close(hr, drow, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(hc, dcol, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("B,I,H", [(3, 1, 256), (2, 2, 64), (1, 1, 512), (2, 1, 48)])
def test_stem_conv_pool_fused(dev, B, I, H):
    """The fused 12x12 s2 conv + 3x3 pool on uint8 patches against the im2col + GEMM +
    maxpool_patch path on the same bf16 weights: pooled within fp32 summation-order noise, argmax
    equal wherever the top two positions are not a near-tie."""
    g = torch.Generator().manual_seed(B * H + I)
    img = torch.randint(0, 256, (B, I, H, H, 3), generator=g, dtype=torch.uint8).to(dev)
    w = (torch.randn((64, 432), generator=g) * 0.05).bfloat16().to(dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    pooled, arg = K.stem_conv_pool(img, w, bias)
    A = K.patch_im2col(img, 16, 12, 12, 2, True)
    conv = K.gemm(A, w, False, True, out_mode=K.OUT_F32, bias=bias)
    ref_p, ref_a = K.maxpool_patch(conv, 9)
    torch.testing.assert_close(pooled, ref_p, rtol=1e-5, atol=1e-5)
    c = conv.view(-1, 9, 64)
    top2 = c.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-4
    assert bool((arg[clear] == ref_a[clear]).all())
    # exact fp64 reference of the conv on the same bf16 operands
    want = (A.double() @ w.double().t() + bias.double()).view(-1, 9, 64).amax(1)
    torch.testing.assert_close(pooled.double(), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("B,I,H", [(3, 1, 256), (2, 2, 64), (1, 1, 512), (2, 1, 48)])
def test_stem_conv_wgrad_implicit(dev, B, I, H):
    """Weight gradient of the fused stem conv from the pooled gradient and argmax, straight from the
    images, against G^T . im2col in float64 (G = maxpool_patch_bwd, bf16), accumulated into an
    existing gradient."""
    g = torch.Generator().manual_seed(7 * B + H)
    img = torch.randint(0, 256, (B, I, H, H, 3), generator=g, dtype=torch.uint8).to(dev)
    w = (torch.randn((64, 432), generator=g) * 0.05).bfloat16().to(dev)
    bias = (torch.randn(64, generator=g) * 0.1).to(dev)
    _, arg = K.stem_conv_pool(img, w, bias)
    n = arg.shape[0]
    dpooled = torch.randn((n, 64), generator=g).to(dev)
    base = torch.randn((64, 432), generator=g).to(dev)
    wg = base.clone()
    K.stem_conv_wgrad(img, dpooled, arg, wg)
    G = K.maxpool_patch_bwd(dpooled, arg, 9)
    A = K.patch_im2col(img, 16, 12, 12, 2, True)
    want = base.double() + G.double().t() @ A.double()
    torch.testing.assert_close(wg.double(), want, rtol=1e-4, atol=1e-3)
