"""The residual-stream products of the step at B = 512, graph-timed (tools/gemm_bench.timeit):
MLP Dense_1 (141,312 x 384 x 1536) and the attention out-projection (149,504 x 384 x 384) with
bias + dropout + fp32 residual -> fp32 (the step's epilogue, reference attention.py:36-37,59-63),
plus the plain narrow product of the same Dense_1 operands (bf16 out) — the A-stream rate without
the residual epilogue. Prints µs, TF/s and GB/s of algorithmic bytes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from multi_modal_transformers_tokenmerge_amd import _kernels as K
from tools.gemm_bench import timeit


def main():
    dev = torch.device("cuda")
    rng = torch.tensor([7, 1], dtype=torch.int32, device=dev)
    g = torch.Generator(device="cpu").manual_seed(0)
    for name, M, N, Kd in [("dense1", 512 * 276, 384, 1536), ("outproj", 512 * 292, 384, 384)]:
        a = torch.randn((M, Kd), generator=g).bfloat16().to(dev)
        w = (torch.randn((N, Kd), generator=g) * Kd ** -0.5).bfloat16().to(dev)
        bias = torch.randn(N, generator=g).to(dev)
        res = torch.randn((M, N), generator=g).to(dev)
        out = torch.empty((M, N), device=dev)
        fused = lambda: K.gemm(a, w, trans_b=True, bias=bias, out=out, out_mode=K.OUT_F32,  # noqa: E731
                               residual=res, rng=rng, drop_layer=0, drop_site=3, keep_prob=0.9)
        t = timeit(fused)
        byts = 2 * (M * Kd + N * Kd) + 8 * M * N
        print(f"{name} fused+res {M}x{N}x{Kd}: {t:7.1f} us  {2 * M * N * Kd / t / 1e6:6.1f} TF/s  "
              f"{byts / t / 1e3:6.0f} GB/s", flush=True)
        ob = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        plain = lambda: K.gemm(a, w, trans_b=True, out=ob)  # noqa: E731
        t = timeit(plain)
        byts = 2 * (M * Kd + N * Kd) + 2 * M * N
        print(f"{name} plain bf16 {M}x{N}x{Kd}: {t:7.1f} us  {2 * M * N * Kd / t / 1e6:6.1f} TF/s  "
              f"{byts / t / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
