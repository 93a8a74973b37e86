"""The HBM-bound LayerNorm / ToMe kernels of block 0 at B = 512 (L = 292, r = 16, D = 384), each
graph-timed alone, as GB/s of algorithmic bytes and the fraction of 8 TB/s (the bench.py probe
byte counts). A/B by environment (MMT_SNB512=0 ...).
    python tools/ln_bench.py [--b=512]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = 512
    for a in sys.argv[1:]:
        if a.startswith("--b="):
            B = int(a.split("=")[1])
    L, D, r, H, s0 = 292, 384, 16, 6, 36
    t = 256
    L2 = L - r
    g = torch.Generator(device="cpu").manual_seed(0)

    def rnd(*shape, dt=torch.bfloat16):
        return torch.randn(shape, generator=g).to(dt).to(dev)
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    res = []

    def run(name, fn, byts):
        us = timeit(fn)
        res.append((name, us, byts / us / 1e3))
        print(f"{name:24s} {us:8.1f} us {byts / us / 1e3:7.0f} GB/s  frac {byts / us / 1e3 / 8000:.3f}", flush=True)

    qkv = rnd(B, L, 3 * D)
    metric = qkv.view(B, L, 3, H, D // H)[:, s0:s0 + t, 1]
    run("tome_match", lambda: K.tome_match(metric, r), B * t * H * (D // H) * 2 + B * ((t + 1) // 2) * 4)
    unm, src, dst = K.tome_match(metric, r)
    x1 = rnd(B, L, D, dt=torch.float32)
    gam = torch.ones(D, device=dev)
    bet = torch.zeros(D, device=dev)
    nidx = (t + 1) // 2 + r
    run("tome_merge_seqnorm_fwd", lambda: K.tome_merge_seqnorm_fwd(x1, s0, t, r, unm, src, dst, gam, bet, 1e-6),
        B * L * D * 4 + B * L2 * D * 6 + B * (t - r) * 4 + B * t * 4 + 2 * B * D * 4 + B * nidx * 4)
    xm, so, pos, _, mu1, rs1 = K.tome_merge_seqnorm_fwd(x1, s0, t, r, unm, src, dst, gam, bet, 1e-6)
    dy1 = rnd(B, L2, D)
    dx2 = rnd(B, L2, D, dt=torch.float32)
    ggam, gbet, gb = (torch.zeros(D, device=dev) for _ in range(3))
    run("ln_unmerge_dropout_bwd", lambda: K.ln_unmerge_dropout_bwd(
        dy1, xm, mu1, rs1, gam, ggam, gbet, dx2, (s0, t, r, pos, None, so), rng, 0, 1, 0.9, 0, bias_grad=gb),
        B * L2 * D * 10 + B * L * D * 6 + B * t * 4 + B * (t - r) * 4 + 2 * B * D * 4)
    x = rnd(B, L2, D, dt=torch.float32)
    run("seqnorm_fwd", lambda: K.seqnorm_fwd(x, gam, bet, 1e-6), B * L2 * D * 6 + 2 * B * D * 4)
    _, mu, rs = K.seqnorm_fwd(x, gam, bet, 1e-6)
    dy = rnd(B, L2, D)
    addend = rnd(B, L2, D, dt=torch.float32)
    run("seqnorm_bwd", lambda: K.seqnorm_bwd(dy, x, mu, rs, gam, ggam, gbet, addend=addend),
        B * L2 * D * 14)
    run("seqnorm_dropout_bwd", lambda: K.seqnorm_dropout_bwd(dy, x, mu, rs, gam, ggam, gbet, addend, rng, 0, 3, 0.9, 0,
                                                              colsum=gb),
        B * L2 * D * 16)


if __name__ == "__main__":
    main()
