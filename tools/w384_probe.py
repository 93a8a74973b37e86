"""The narrow-output NT kernel (gemm_ntw_kernel) against hipBLASLt (torch.mm / addmm / relu
epilogue) on the step's narrow-output products: graph-timed, and the result vs an fp32 torch
product of the same bf16 operands (both sides' max |diff| to it over max |ref|). MMT_NTW_MT forces the row-panel height (no two-launch plan), MMT_NTW_BN=384 the 384-wide tile."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = 512
    shapes = [("MLP dX L292", B * 292 - 11008, 384, 1536, "none"), ("MLP dX L212", B * 212, 384, 1536, "none"),
              ("MLP dX L116", B * 116, 384, 1536, "none"), ("QKV dX L292", B * 292, 384, 1152, "none"),
              ("QKV dX L164", B * 164, 384, 1152, "none"), ("T5 FF-out+res", B * 32, 768, 3072, "res"),
              ("T5 FF-in relu", B * 32, 3072, 768, "relu")]
    for name, M, N, Kd, ep in shapes:
        g = torch.Generator(device="cpu").manual_seed(M + N + Kd)
        a = torch.randn((M, Kd), generator=g).bfloat16().to(dev)
        b = torch.randn((N, Kd), generator=g).bfloat16().to(dev)
        r = torch.randn((M, N), generator=g).bfloat16().to(dev) if ep == "res" else None
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        act = K.ACT_RELU if ep == "relu" else K.ACT_NONE
        ours = lambda: K.gemm(a, b, False, True, out=out, residual=r, act=act)  # noqa: E731
        if ep == "relu":
            z = torch.zeros(N, device=dev, dtype=torch.bfloat16)
            lib = lambda: torch._addmm_activation(z, a, b.t())  # noqa: E731
        else:
            lib = ((lambda: torch.addmm(r, a, b.t())) if r is not None  # noqa: E731
                   else (lambda: torch.mm(a, b.t())))  # hipBLASLt, for comparison only
        t_o, t_l = timeit(ours), timeit(lib)
        ref = a.float() @ b.float().t()
        if r is not None:
            ref = ref + r.float()
        if ep == "relu":
            ref = ref.clamp_min(0)
        o, lb = ours().float(), lib().float()
        scale = ref.abs().max().item()
        e_o, e_l = (o - ref).abs().max().item() / scale, (lb - ref).abs().max().item() / scale
        flops = 2.0 * M * N * Kd
        byts = 2.0 * (M * Kd + N * Kd + M * N * (2 if r is not None else 1))
        print(f"{name:14s} {M:6d} x {N:4d} x {Kd:4d}: w384 {t_o:7.1f} us ({flops / t_o / 1e6:6.1f} TF/s, "
              f"{byts / t_o / 1e3:6.0f} GB/s)  hipBLASLt {t_l:7.1f} us   max |err| / max |ref|: {e_o:.2e} vs {e_l:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
