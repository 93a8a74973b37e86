"""Plain NT products of the step: libmmt_hip's kernel vs hipBLASLt (torch.mm / addmm), graph-timed
(tools/gemm_bench.timeit). Decides K.library_gemm_ok's shape rule."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    B = 512
    shapes = [("MLP dX", B * 276, 384, 1536, False), ("QKV dX", B * 292, 384, 1152, False),
              ("out-proj dX", B * 292, 384, 384, False), ("T5 QKV", B * 32, 2304, 768, False),
              ("T5 O + res", B * 32, 768, 768, True), ("T5 FF-out + res", B * 32, 768, 3072, True),
              ("T5 FF-in (plain)", B * 32, 3072, 768, False), ("text proj", B * 32, 384, 768, False)]
    for name, M, N, Kd, res in shapes:
        a = torch.randn((M, Kd), device=dev).bfloat16()
        b = torch.randn((N, Kd), device=dev).bfloat16()
        r = torch.randn((M, N), device=dev).bfloat16() if res else None
        out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        t_ours = timeit(lambda: K.gemm(a, b, False, True, out=out, residual=r))
        t_lib = timeit(lambda: K.library_gemm_nt(a, b, residual=r, out=out))
        print(f"{name:18s} M={M:6d} N={N:5d} K={Kd:5d}: libmmt {t_ours:7.1f} us  hipBLASLt {t_lib:7.1f} us",
              flush=True)
    # relu products (T5 FF-in): our fused epilogue vs hipBLASLt's relu epilogue (zero bias)
    M, N, Kd = B * 32, 3072, 768
    a = torch.randn((M, Kd), device=dev).bfloat16()
    b = torch.randn((N, Kd), device=dev).bfloat16()
    z = torch.zeros(N, device=dev, dtype=torch.bfloat16)
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    t_ours = timeit(lambda: K.gemm(a, b, False, True, out=out, act=K.ACT_RELU))
    t_lib = timeit(lambda: torch._addmm_activation(z, a, b.t()))
    ref = K.gemm(a, b, False, True, act=K.ACT_RELU)
    lib = torch._addmm_activation(z, a, b.t())
    diff = (ref.float() - lib.float()).abs().max().item()
    print(f"T5 FF-in relu      M={M:6d} N={N:5d} K={Kd:5d}: libmmt {t_ours:7.1f} us  hipBLASLt+relu {t_lib:7.1f} us"
          f"  max |diff| {diff:.3g}", flush=True)


if __name__ == "__main__":
    main()
